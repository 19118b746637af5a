#!/bin/bash
# round-4 check 3: fused attention fronts (training self / cross, decode cross / self): kernels vs torch,
# fused vs separate engines, bench + decode A/B, then the full -m gpu suite
set -o pipefail
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fused_qkv or fused_attention_fronts or c4_bf16 or bf16_decode or grouped_decode or slab_decode" > $O/pytest_fused.log 2>&1 || { tail -30 $O/pytest_fused.log; exit 1; }
tail -2 $O/pytest_fused.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-batches > $O/bench_fused$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_fused$i.json'));print('fused', d['ms_per_step'], d['dominant_kernel']['classes_us_per_step'])"
CAPGEN_FUSED_QKV=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-batches > $O/bench_unfused$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_unfused$i.json'));print('unfused', d['ms_per_step'], d['dominant_kernel']['classes_us_per_step'])"
done
timeout -k 10 300 python -u tools/bench_generate.py > $O/generate.json 2> $O/generate.err || { tail -20 $O/generate.err; exit 1; }
cat $O/generate.json
CAPGEN_FUSED_QKV=0 timeout -k 10 300 python -u tools/bench_generate.py > $O/generate_unfused.json 2> $O/generate.err || { tail -20 $O/generate.err; exit 1; }
cat $O/generate_unfused.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
