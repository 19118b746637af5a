# gradient determinism probe (tools/grad_det_probe.py) in several fresh processes per setting
set -o pipefail
mkdir -p gpurun_out
for ov in "$@"; do
  for proc in 1 2 3; do
    CAPGEN_OVERLAP_DEC0=$ov timeout -k 10 150 python -u tools/grad_det_probe.py 8 > gpurun_out/det_ov$ov.$proc.log 2>&1
    rc=$?
    echo "ov=$ov proc=$proc rc=$rc"; grep -E "^iter|^probe" gpurun_out/det_ov$ov.$proc.log | tail -6
    [ $rc -eq 0 ] || exit $rc
  done
done
