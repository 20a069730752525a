#!/bin/bash
# One GPU-box session that refreshes every judged artefact for the current tree (run from the repo
# root on the box via gpurun).  Every GPU step has its own time limit; the first failure ends it.
#   TAG=r01_v10 tools/round_gpu.sh [tests|bench|all]
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-latest}
WHAT=${1:-all}
O=gpurun_out/$TAG
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  echo "[round_gpu] $name" >&2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[round_gpu] $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -30 $O/$name.log >&2; exit $rc; fi
}
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
  step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  step bench 300 python -u bench.py
  # the same command as the bench line above, so the kernel averages can be compared with it
  step rocprof_stats 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py
  step pmc_sq 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/pmc/sq -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
  step pmc_fetch 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc/fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
  step pmc_write 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc/write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
  step traffic 60 python -u tools/pmc_to_traffic.py $O/pmc f1_L4_n24_w1 $O/pmc_summary.json
  step configs 600 python -u tools/bench_configs.py --out $O/configs.jsonl
  # the N > 1 default (partitioned four-step over RCCL), rehearsed at world size 1
  step bench_fourstep_w1 300 python -u bench.py --four-step --steps 20 --warmup 10 --no-cpu-baseline
fi
echo "[round_gpu] done" >&2
