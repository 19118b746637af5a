#!/bin/bash
# GEMM fragment-order A/B: GEMM parity tests on the new build, then bench old vs new library.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread \
  -k "gemm or splitk or k_groups or weight_gradients" > gpurun_out/frag_tests.log 2>&1 || { tail -30 gpurun_out/frag_tests.log; exit 1; }
tail -1 gpurun_out/frag_tests.log
bash tools/ab_env.sh CAPGEN_LIB_PATH $PWD/image-caption_amd/capgen/libcapgen_old.so $PWD/image-caption_amd/capgen/libcapgen.so
