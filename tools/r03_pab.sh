#!/bin/bash
# P-path (SSIP field, 8-B elements) A/B of the new Shoup / lazy engine: pass-1 table vs two-level
# twiddles, XCD tile order, schedules.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_pab}
mkdir -p $O
run() {  # name env... -- args
  local name=$1; shift
  echo "[pab] $name" >&2
  env "$@" timeout -k 10 120 python -u tools/exp_launches.py --cfg f0_L1_n26 --cfg f0_L1_n24 --cfg f0_L1_n26_ip --warmup 30 --steps 50 > $O/$name.jsonl 2>$O/$name.log || { tail $O/$name.log >&2; exit 1; }
}
for rep in 1 2; do
  run base$rep NTT_XCD_ORDER=2
  run noxcd$rep NTT_XCD_ORDER=0
  run p1full$rep NTT_PASS1_FULL=1
  run s989_$rep NTT_SCHEDULE=9,8,9
  run s998_$rep NTT_SCHEDULE=9,9,8
  run p1full_s989_$rep NTT_PASS1_FULL=1 NTT_SCHEDULE=9,8,9
done
echo "[pab] done" >&2
