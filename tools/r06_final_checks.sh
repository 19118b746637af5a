set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06j; mkdir -p $out
bash tools/gpu_check.sh r06j suite || exit 1
timeout -k 10 200 python -u tools/bench_generate.py > $out/generate.jsonl 2> $out/generate.err || exit 1
cat $out/generate.jsonl
timeout -k 10 200 python -u tools/bench_scst.py > $out/scst.json 2> $out/scst.err || exit 1
cat $out/scst.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/dec_beam -o run -- python3 tools/bench_generate.py --reps 3 --modes beam5 > $out/dec_beam.log 2>&1 || exit 1
find $out/dec_beam -name "run_kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/dec_beam_kernel_stats.csv
head -12 $out/dec_beam_kernel_stats.csv | cut -c1-160
