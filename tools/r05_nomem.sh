#!/bin/bash
# Where the 256-bit pass time goes: the product library against the NTT_DEBUG_NOMEM diagnostic build
# (every data / table access folded into an L2-resident window: wrong results by design), same box:
# bench launch times, then one SQ + GRBM PMC pass each (clock = GRBM_GUI_ACTIVE cycles / duration).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05_nomem}
mkdir -p $O
N=$PWD/ntt_amd/libntt_nomem.so
for i in 1 2; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-parity > $O/prod_$i.json 2>>$O/err.log || exit 1
  NTT_LIB_PATH=$N timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-parity > $O/nomem_$i.json 2>>$O/err.log || exit 1
done
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C -d $O/pmc_prod -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --prewarm-s 0 > $O/pmc_prod.log 2>&1 || exit 1
NTT_LIB_PATH=$N timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C -d $O/pmc_nomem -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --prewarm-s 0 > $O/pmc_nomem.log 2>&1 || exit 1
echo nomem-done
