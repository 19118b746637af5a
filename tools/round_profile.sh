#!/bin/bash
# Measurement artifacts of a round (run on the GPU box from the repo root):
#   bash tools/round_profile.sh <tag>        e.g. r01
# writes gpurun_out/<tag>/: bench.json (the bench line, CPU baseline included), the rocprofv3
# kernel-trace + stats of a profiled bench run (kernel_stats.csv, timeline.txt with the
# dominant-GEMM launches' trace average), and the HBM traffic of one step from two separate PMC
# passes (pmc_traffic.json; FETCH_SIZE x2 per the gfx950 correction, WRITE_SIZE as is), and the
# MFMA utilisation per kernel class from a third PMC pass (pmc_mfma.json, tools/pmc_mfma.py).
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r02}
out=gpurun_out/$tag
rm -rf "$out" && mkdir -p "$out"
timeout -k 10 300 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 1; }
cut -c1-400 "$out/bench.json"; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-batches > "$out/trace.log" 2>&1 || { tail -20 "$out/trace.log"; exit 1; }
d=$(dirname "$(find "$out/trace" -name run_kernel_trace.csv | head -1)")
cp "$d/run_kernel_stats.csv" "$out/kernel_stats.csv"
python tools/timeline.py "$d" --steps 10 > "$out/timeline.txt"
python tools/timeline.py "$d" --dominant >> "$out/timeline.txt"
head -8 "$out/timeline.txt"; tail -2 "$out/timeline.txt"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$out/pmc_$c" -o run -- \
    python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-host-batches > "$out/pmc_$c.log" 2>&1 || { tail -20 "$out/pmc_$c.log"; exit 1; }
done
python tools/pmcsum.py "$out/pmc_FETCH_SIZE" "$out/pmc_WRITE_SIZE" "$out/pmc_traffic.json" | head -4
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
  -d "$out/pmc_mfma" -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-host-batches > "$out/pmc_mfma.log" 2>&1 \
  || { tail -20 "$out/pmc_mfma.log"; exit 1; }
python tools/pmc_mfma.py "$out/pmc_mfma" "$out/pmc_mfma.json" | head -6
python tools/class_table.py "$out" > "$out/class_table.txt" && cat "$out/class_table.txt"
