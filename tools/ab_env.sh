#!/bin/bash
# A/B timing of runtime switches (environment variables) on the product build, interleaved twice.
# Run on the GPU box:  tools/ab_env.sh "NAME=VALUE ..." "NAME=VALUE ..." ...   ("" = defaults)
# Output: one line per run, "<env> <ms_per_step> <launch_ms...>".
set -o pipefail
ARGS=${ARGS:---steps 100 --warmup 50 --no-cpu-baseline}
for rep in 1 2; do
  for envs in "$@"; do
    out=$(env $envs timeout -k 10 180 python3 bench.py $ARGS 2>/dev/null | tail -1) || { echo "[$envs] FAILED"; exit 1; }
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print('[' + sys.argv[1] + ']', round(d['ms_per_step'],4), [round(x,4) for x in d.get('roofline',{}).get('launch_ms',[])])" "$envs" "$out"
  done
done
