# kernel trace of a short bench run per CAPGEN_FWD_SPLIT value; prints the first kernels of the
# last step's forward (does the encoder overlap the decoder front?)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  rm -rf gpurun_out/fp$v
  CAPGEN_FWD_SPLIT=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fp$v -o run -- \
    python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-host-batches > gpurun_out/fp$v.log 2>&1 || { tail -20 gpurun_out/fp$v.log; exit 1; }
  d=$(dirname "$(find gpurun_out/fp$v -name run_kernel_trace.csv | head -1)")
  echo "== CAPGEN_FWD_SPLIT=$v"; python tools/timeline.py "$d" --steps 5 | head -4
  python tools/timeline.py "$d" --list | awk '/bump_seed/{f=1} f' | head -16 | cut -c1-110
done
