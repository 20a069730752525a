#!/bin/bash
# Compare library variants on the GPU box: tools/cmp_libs.sh OUTDIR lib1 lib2 ...  (bench.py, 2^24 BN254)
set -o pipefail
O=$1; shift; mkdir -p $O
for rep in 1 2; do
  for L in "$@"; do
    NTT_LIB_PATH=ntt_amd/$L timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 ${BENCH_ARGS} > $O/$L.$rep.json 2> $O/$L.$rep.err || exit 1
    python -c "import json,sys; d=json.load(open('$O/$L.$rep.json')); print('$L', round(d['ms_per_step'],4), [round(x,4) for x in d['roofline']['launch_ms']])"
  done
done
