#!/bin/bash
# per-shape GEMM time, old vs new fragment order (tuned choice + fixed variants, no split-K)
set -o pipefail
mkdir -p gpurun_out
for lib in old new; do
  p=$PWD/image-caption_amd/capgen/libcapgen.so; [ $lib = old ] && p=$PWD/image-caption_amd/capgen/libcapgen_old.so
  CAPGEN_LIB_PATH=$p timeout -k 10 300 python -u tools/gemm_splitk_sweep.py --variants 1,7,8,10,21,23 --splits 1 --out frag_$lib.json > gpurun_out/frag_$lib.log 2>&1 || { tail -20 gpurun_out/frag_$lib.log; exit 1; }
done
python3 - <<'PY'
import json
o=json.load(open('gpurun_out/frag_old.json')); n=json.load(open('gpurun_out/frag_new.json'))
for a,b in zip(o,n):
    ks=[k for k in a if k.startswith('v') or k=='tuned_us']
    print(f"{a['shape']:16s}", " ".join(f"{k}:{a[k]:.1f}->{b.get(k,0):.1f}" for k in ks))
PY
