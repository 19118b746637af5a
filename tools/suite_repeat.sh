# run the -m gpu suite N times (no -x; every failure listed per run): looking for intermittent mismatches
set -o pipefail
mkdir -p gpurun_out
n=${1:-3}
for i in $(seq 1 "$n"); do
  timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/suite_rep$i.log 2>&1
  rc=$?
  echo "run $i rc=$rc $(tail -1 gpurun_out/suite_rep$i.log)"; grep -E "^FAILED" gpurun_out/suite_rep$i.log | head -5
  [ $rc -le 1 ] || exit $rc
done
