#!/bin/bash
# round-4: fused attention fronts reading tiled weights -- kernel + engine parity, isolated cost, bench, suite
set -o pipefail
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fused_qkv or fused_attention_fronts or c2_full_size or bf16_train_mode" > $O/pytest_fr.log 2>&1 || { tail -40 $O/pytest_fr.log; exit 1; }
tail -1 $O/pytest_fr.log
timeout -k 10 120 python -u tools/front_microbench.py > $O/micro.json 2> $O/micro.err || { tail -20 $O/micro.err; exit 1; }
cat $O/micro.json
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-batches > $O/bench$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench$i.json'));c=d['dominant_kernel']['classes_us_per_step'];print('tiled', d['ms_per_step'], c)"
CAPGEN_FUSED_QKV=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-batches > $O/bench_sep$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_sep$i.json'));c=d['dominant_kernel']['classes_us_per_step'];print('separate', d['ms_per_step'], c)"
done
timeout -k 10 300 python -u tools/bench_generate.py > $O/gen.json 2> $O/gen.err || { tail -20 $O/gen.err; exit 1; }
cat $O/gen.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
