set -o pipefail
mkdir -p gpurun_out/gg
for r in 1 2 3; do for g in 0 1; do
  CAPGEN_GEN_GRAPH=$g timeout -k 10 150 python -u tools/bench_generate.py --reps 5 --warmup 3 > gpurun_out/gg/g${g}_$r.jsonl 2>gpurun_out/gg/err_$g_$r.txt || exit 1
  echo "graph=$g round $r: $(cut -c1-40,100-200 gpurun_out/gg/g${g}_$r.jsonl | tr '\n' ' ')"
done; done
