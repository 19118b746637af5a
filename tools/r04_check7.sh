#!/bin/bash
# round-4 check 7: ce_finish with the loss finalisation merged (last-workgroup ticket), decoder front
# forked after encoder block 0 -- full -m gpu suite, then bench A/B on CAPGEN_FRONT_LATE
set -o pipefail
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-batches > $O/late$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/late$i.json'));print('late', d['ms_per_step'], d['final_loss'], d['dominant_kernel']['classes_us_per_step'])"
CAPGEN_FRONT_LATE=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-batches > $O/early$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/early$i.json'));print('early', d['ms_per_step'], d['final_loss'], d['dominant_kernel']['classes_us_per_step'])"
done
