#!/bin/bash
# round-4 check 11: the output side of the attention backward fused (qkv_attn_bwd) -- kernel / engine
# parity, bench A/B on CAPGEN_FUSED_ATTN_BWD, then the full suite
set -o pipefail
O=gpurun_out/r04u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "attention_bwd_wo or fused_attention_fronts or c2_full_size or bf16_train_mode or attention_kernels" > $O/pytest_ab.log 2>&1 || { tail -40 $O/pytest_ab.log; exit 1; }
tail -1 $O/pytest_ab.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-batches > $O/fused$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/fused$i.json'));c=d['dominant_kernel']['classes_us_per_step'];print('fused', d['ms_per_step'], c)"
CAPGEN_FUSED_ATTN_BWD=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-batches > $O/sep$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/sep$i.json'));c=d['dominant_kernel']['classes_us_per_step'];print('separate', d['ms_per_step'], c)"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
