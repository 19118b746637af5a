#!/bin/bash
# round-4: fused attention front with 4 / 6 / 12 waves splitting the projection columns
# (CAPGEN_QKV_WAVES): kernel parity vs torch, isolated cost (tools/front_microbench.py), bench A/B
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
for w in 4 6 12; do
CAPGEN_QKV_WAVES=$w timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused_qkv_attention" > $O/pytest_$w.log 2>&1 || { tail -30 $O/pytest_$w.log; exit 1; }
echo "waves $w: $(tail -1 $O/pytest_$w.log)"
CAPGEN_QKV_WAVES=$w timeout -k 10 120 python -u tools/front_microbench.py > $O/micro_$w.json 2> $O/micro.err || { tail -20 $O/micro.err; exit 1; }
cat $O/micro_$w.json
done
for i in 1 2; do
for w in 4 6 12; do
CAPGEN_QKV_WAVES=$w timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-batches > $O/bench_$w.$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_$w.$i.json'));c=d['dominant_kernel']['classes_us_per_step'];print('waves $w', d['ms_per_step'], c.get('qkv_attn'))"
done
done
