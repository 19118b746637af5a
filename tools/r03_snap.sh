#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/snap.log
for rep in 1 2 3 4 5 6 7 8 9 10; do
  CAPGEN_LNB_COH=${COH:-0} CHAIN=1 CAPGEN_FWD_GRAPH=0 CAPGEN_STREAMS=2 timeout -k 10 180 python -u tools/enc_snap_probe.py 2>&1 | grep '^{' >> gpurun_out/snap.log || { echo fail; exit 1; }
done
grep -v '"fb": null, "step1": null, "step2": null' gpurun_out/snap.log
