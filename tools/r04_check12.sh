#!/bin/bash
# round-4 check 12: fork / join / bucket event fence scope (CAPGEN_EVENT_FENCE 0 / 1 / 2), bench A/B
# with the final loss compared, then the DP / bucketed-update parity tests under the chosen scope
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
for i in 1 2 3; do
for f in 0 1 2; do
CAPGEN_EVENT_FENCE=$f timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host-batches > $O/f$f.$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/f$f.$i.json'));c=d['dominant_kernel']['classes_us_per_step'];print('fence $f', d['ms_per_step'], d['final_loss'], c['gemm dX'], c['ln_bwd'])"
done
done
CAPGEN_EVENT_FENCE=${1:-2} timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c2_full_size or bf16_train_mode or dp or bucket or sharded or streams" > $O/pytest_ab.log 2>&1 || { tail -40 $O/pytest_ab.log; exit 1; }
tail -1 $O/pytest_ab.log
