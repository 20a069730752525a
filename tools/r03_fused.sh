#!/bin/bash
# Single-launch (k_fused3) schedule: GPU tests, same-box A/B against the 3-launch schedule, rocprof.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_fused2}
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  echo "[fused] $name" >&2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[fused] $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -30 $O/$name.log >&2; exit $rc; fi
}
step pytest 400 python -u -m pytest tests/test_gpu_single_launch.py -x -v --timeout 200 --timeout-method thread
C=""
for n in 20 18 19 21 22 23 24 20; do C="$C --cfg f1_L4_n$n --cfg f1_L4_n${n}_sl"; done
step ab 400 python -u tools/exp_launches.py $C --out $O/ab.jsonl
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/exp_launches.py --cfg f1_L4_n20 --cfg f1_L4_n20_sl --warmup 30 --steps 50
echo "[fused] done" >&2
