#!/bin/bash
# Round-3 baseline on one box: headline bench, per-launch timings of the SSIP (P, 8-B) path at
# 2^24/2^26 and of C2, rocprof kernel stats + HBM PMC of the P 2^26 transform.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_base}
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  echo "[r03] $name" >&2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[r03] $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -30 $O/$name.log >&2; exit $rc; fi
}
step bench 300 python -u bench.py --no-cpu-baseline
step launches 300 python -u tools/exp_launches.py --cfg f0_L1_n26 --cfg f0_L1_n24 --cfg f1_L4_n20 --cfg f1_L4_n24 --out $O/launches.jsonl
step p26_stats 200 rocprofv3 --kernel-trace --stats -d $O/p26_prof -o run --output-format csv -- python3 tools/exp_launches.py --cfg f0_L1_n26 --warmup 20 --steps 20
step p26_fetch 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/p26_fetch -o run --output-format csv -- python3 tools/exp_launches.py --cfg f0_L1_n26 --warmup 1 --steps 3
step p26_write 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/p26_write -o run --output-format csv -- python3 tools/exp_launches.py --cfg f0_L1_n26 --warmup 1 --steps 3
echo "[r03] done" >&2
