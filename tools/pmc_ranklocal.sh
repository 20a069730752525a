#!/bin/bash
# HBM traffic (PMC) of the four-step's rank-local launches at G = 2, 4, 8:
# rank 0 of a G-rank plan (ntt_rplan) on ONE GPU, forward rows + columns, no exchange
# (tools/exp_ranklocal.py --no-plain).  One rocprofv3 pass per counter, each under its own time limit.
# Run on the GPU box from the repo root; then, here:
#   python tools/pmc_to_traffic.py $O/w$G f1_L4_n24_w${G}_fs --per 3 --note "..."
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/pmc_rl}
for G in ${WORLDS:-2 4 8}; do
  mkdir -p $O/w$G
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c -d $O/w$G/$d -o run --output-format csv -- \
      python3 tools/exp_ranklocal.py --no-plain --worlds $G --warmup 2 --steps 4 > $O/w$G/$d.log 2>&1 || exit 1
  done
done
echo pmc-ranklocal-done
