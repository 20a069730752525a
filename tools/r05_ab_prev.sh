#!/bin/bash
# Same-box A/B of the current library against ntt_amd/libntt_prev.so (a build of an earlier commit,
# made beside this tree): the headline bench, interleaved three times.  Usage: bash tools/r05_ab_prev.sh TAG
set -o pipefail
O=gpurun_out/${1:-r05_abprev}
mkdir -p $O
P=$PWD/ntt_amd/libntt_prev.so
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-parity > $O/cur_$i.json 2>>$O/err.log || exit 1
  NTT_LIB_PATH=$P timeout -k 10 120 python bench.py --no-cpu-baseline --no-parity > $O/prev_$i.json 2>>$O/err.log || exit 1
done
echo ab-done
