#!/bin/bash
# 2^28 BN254 radix schedules (NTT_SCHEDULE, experiments only) against the planner's 7+7+7+7, two
# interleaved repetitions, fresh process each.  Usage: bash tools/r05_sched28.sh TAG
set -o pipefail
O=gpurun_out/${1:-r05_sched28}
mkdir -p $O
for i in 1 2; do
  for s in default 8,8,8,4 4,8,8,8 8,4,8,8 8,8,4,8; do
    if [ $s = default ]; then
      timeout -k 10 120 python3 -u tools/exp_launches.py --cfg f1_L4_n28 --warmup 5 --steps 10 --out $O/s_${s}_$i.jsonl > $O/s_${s}_$i.log 2>&1 || exit 1
    else
      NTT_SCHEDULE=$s timeout -k 10 120 python3 -u tools/exp_launches.py --cfg f1_L4_n28 --warmup 5 --steps 10 --out $O/s_${s}_$i.jsonl > $O/s_${s}_$i.log 2>&1 || exit 1
    fi
  done
done
echo sched-done
