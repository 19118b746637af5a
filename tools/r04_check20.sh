#!/bin/bash
# round-4 check 20: the fused attention kernels skip the staged rows past L / Lk instead of loading
# them clamped to the last row (CAPGEN_QKV_CLAMP=1 restores the clamped loads): parity subset, isolated
# kernel times under rocprofv3 both ways, then the step A/B (three alternating rounds)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ad
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fused_attention or fused_qkv or attention_bwd_wo or c2_full_size or bf16_train_mode or bit_reproducible" > $O/pytest_ab.log 2>&1 || { tail -40 $O/pytest_ab.log; exit 1; }
tail -1 $O/pytest_ab.log
for c in 0 1; do
CAPGEN_QKV_CLAMP=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$c -o run -- python3 tools/attn_bwd_microbench.py > $O/prof$c.log 2>&1 || { tail -20 $O/prof$c.log; exit 1; }
f=$(find $O/prof$c -name run_kernel_stats.csv | head -1)
python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'qkv_attn' in r['Name']: print('clamp=$c', r['Calls'], round(float(r['AverageNs'])/1e3, 2), r['Name'][:70])
"
done
for i in 1 2 3; do
for c in 0 1; do
CAPGEN_QKV_CLAMP=$c timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host-batches > $O/b$c.$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/b$c.$i.json'));c=d['dominant_kernel']['classes_us_per_step'];print('clamp $c', d['ms_per_step'], c['attn_bwd_wo'], c['qkv_attn'])"
done
done
