#!/bin/bash
# Timing-only sensitivity of the 2^24 BN254 forward to each arithmetic category:
# libntt_ab<bits>.so built with NTT_AB_SKIP=<bits> (engines.hpp; results are wrong by design):
# 1 reductions, 2 Shoup products, 4 Montgomery products, 8 carry normalisations, 15 all four.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_ab}
mkdir -p $O
ARGS="--steps 100 --warmup 50 --no-cpu-baseline" timeout -k 10 900 bash tools/exp_variants.sh ab1 ab2 ab4 ab8 ab15 > $O/ab.txt 2> $O/ab.err || { cat $O/ab.txt; tail $O/ab.err; exit 1; }
cat $O/ab.txt
