#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hazard.py -q --timeout 120 --timeout-method thread > gpurun_out/hz3.log 2>&1
tail -1 gpurun_out/hz3.log
bash tools/ab_env.sh CAPGEN_FLUSH_DEFER 0 1 && bash tools/ab_env.sh CAPGEN_FLUSH_DEFER 0 1
