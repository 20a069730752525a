#!/bin/bash
# rocprofv3 PMC passes over the default bench workload (run on the GPU box from the repo root).
# Each counter group is its own rocprofv3 run (--pmc never combined with trace domains).
# Output: gpurun_out/pmc/<group>/... ; summarise with tools/pmc_summary.py.
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
ARGS=${ARGS:---steps 3 --warmup 1 --no-cpu-baseline}
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
}
run sq   SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run lds  SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
echo pmc-done
