#!/bin/bash
# HBM traffic (PMC) of the four-step's local launches: bench.py --four-step at world size 1 (RCCL
# all-to-all included), one rocprofv3 pass per counter group.  Run on the GPU box.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/pmc_fs}
mkdir -p $O
ARGS="--four-step --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py $ARGS > $O/fetch.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 bench.py $ARGS > $O/write.log 2>&1 || exit 1
python3 tools/pmc_summary.py $O $O/pmc_counters.json
