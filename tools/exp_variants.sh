#!/bin/bash
# A/B timing of experiment builds (ntt_amd/libntt_<tag>.so) against the product build, interleaved
# twice to average out box drift.  Run on the GPU box:  tools/exp_variants.sh tag1 tag2 ...
# Output: one line per run, "<tag> <ms_per_step> <launch_ms...>".
set -o pipefail
ARGS=${ARGS:---steps 100 --warmup 50 --no-cpu-baseline}
for rep in 1 2; do
  for tag in base "$@"; do
    if [ "$tag" = base ]; then lib=ntt_amd/libntt.so; else lib=ntt_amd/libntt_$tag.so; fi
    out=$(NTT_LIB_PATH=$lib timeout -k 10 120 python3 bench.py $ARGS 2>/dev/null | tail -1) || { echo "$tag FAILED"; exit 1; }
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1], round(d['ms_per_step'],4), [round(x,4) for x in d.get('roofline',{}).get('launch_ms',[])])" "$tag" "$out"
  done
done
