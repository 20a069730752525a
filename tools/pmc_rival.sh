#!/bin/bash
# PMC of the default schedule's passes next to GZKP(B,G)'s (tools/exp_rival_pair.py), 2^24 BN254.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/pmc_rival}
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/sq -o run --output-format csv -- python3 tools/exp_rival_pair.py > $O/sq.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 tools/exp_rival_pair.py > $O/fetch.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 tools/exp_rival_pair.py > $O/write.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 tools/exp_rival_pair.py > $O/stats.log 2>&1 || exit 1
python3 tools/pmc_summary.py $O $O/pmc_counters.json
