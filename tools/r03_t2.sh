#!/bin/bash
# Full GPU test suite + P-path A/B on the current tree.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_t2}
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  echo "[t2] $name" >&2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[t2] $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -30 $O/$name.log >&2; exit $rc; fi
}
step pytest 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
step launches 300 python -u tools/exp_launches.py --cfg f0_L1_n26 --cfg f0_L1_n24 --cfg f0_L1_n26_ip --cfg f0_L1_n24_ip --cfg f1_L4_n24 --cfg f1_L4_n24_ip --cfg f1_L4_n20 --cfg f0_L1_n26 --out $O/launches.jsonl
echo "[t2] done" >&2
