#!/bin/bash
# round-4 check 18: ce_finish with 16-B accesses (CAPGEN_CE_VEC8) -- bit-identity test, kernel time
# under rocprofv3 both ways, bench A/B; then the full -m gpu suite and the decode profile (check 17)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "ce_finish or fused_classifier or c2_full_size" > $O/pytest_ab.log 2>&1 || { tail -40 $O/pytest_ab.log; exit 1; }
tail -1 $O/pytest_ab.log
for v in 1 0; do
CAPGEN_CE_VEC8=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$v -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-batches > $O/prof$v.log 2>&1 || { tail -20 $O/prof$v.log; exit 1; }
f=$(find $O/prof$v -name run_kernel_stats.csv | head -1)
echo "vec8=$v $(grep ce_finish $f | cut -d, -f2-4)"
done
for i in 1 2; do
for v in 1 0; do
CAPGEN_CE_VEC8=$v timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host-batches > $O/b$v.$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/b$v.$i.json'));print('vec8 $v', d['ms_per_step'], d['final_loss'])"
done
done
bash tools/r04_check17.sh
