# tools/shard_diag.py once per argument, each argument a space-separated list of VAR=VALUE settings
# (e.g. "CAPGEN_EVENT_FENCE=2" "GPU_MAX_HW_QUEUES=16 DIAG_PAD=1"); appends to gpurun_out/shard_modes.txt
out=gpurun_out/shard_modes.txt
for m in "$@"; do
  echo "== $m" >> $out
  env $m timeout -k 10 200 python -u tools/shard_diag.py 8 2 2>&1 | grep -E "^==|^step|rank|chunk" >> $out || exit 1
done
