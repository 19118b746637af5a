#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 180 --timeout-method thread \
  tests/test_gpu_parity.py::test_grouped_weight_gradients_match_single_launches_bf16 \
  "tests/test_gpu_parity.py::test_train_step_equals_forward_backward_adam_bf16" > gpurun_out/t2.log 2>&1 || { tail -30 gpurun_out/t2.log; exit 1; }
tail -5 gpurun_out/t2.log
timeout -k 10 200 python -u tools/r03_streams1_graph.py 2>&1 | grep "^{" 
