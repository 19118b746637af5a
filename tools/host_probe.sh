# ms/step and host enqueue ms/step of a 100-step bench per "ENV=.. [--flag]" spec
set -o pipefail
mkdir -p gpurun_out
for spec in "$@"; do
  envs=$(echo "$spec" | tr ' ' '\n' | grep '=' | tr '\n' ' ')
  flags=$(echo "$spec" | tr ' ' '\n' | grep -- '^--' | tr '\n' ' ')
  env $envs timeout -k 10 120 python -u bench.py --steps 100 --no-cpu-baseline --no-host-batches $flags > gpurun_out/hp.json 2> gpurun_out/hp.err \
    || { tail -20 gpurun_out/hp.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/hp.json').read().strip().splitlines()[-1]); print('[$spec]', d['ms_per_step'], 'host', d['host_issue_ms_per_step'])"
done
