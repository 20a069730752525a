#!/bin/bash
# Round-3 hand-off polling A/B on the product build (relaxed-load polls in every inter-workgroup
# wait): single-launch forms (NTT_FUSED_MODE=0 dataflow, =1 grid barrier) vs three launches at
# 2^18..2^24, and the in-place plans (fused digit reversal) vs the default schedule.
set -o pipefail
O=gpurun_out/${TAG:-r03_sync}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_single_launch.py tests/test_gpu_inplace.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -20 $O/pytest.txt; exit 1; }
NTT_FUSED_MODE=0 timeout -k 10 200 python -u -m pytest tests/test_gpu_single_launch.py -x -q --timeout 120 --timeout-method thread > $O/pytest_mode0.txt 2>&1 || { tail -20 $O/pytest_mode0.txt; exit 1; }
tail -1 $O/pytest.txt; tail -1 $O/pytest_mode0.txt
L="--warmup 30 --steps 50"
for rep in 1 2; do
  for m in 1 0; do
    NTT_FUSED_MODE=$m timeout -k 10 200 python -u tools/exp_launches.py --cfg f1_L4_n18_sl --cfg f1_L4_n20_sl --cfg f1_L4_n22_sl --cfg f1_L4_n24_sl $L 2>/dev/null | sed "s/^/mode$m /" >> $O/ab.txt || exit 1
  done
  timeout -k 10 300 python -u tools/exp_launches.py --cfg f1_L4_n18 --cfg f1_L4_n20 --cfg f1_L4_n22 --cfg f1_L4_n24 --cfg f1_L4_n24_ip --cfg f0_L1_n26 --cfg f0_L1_n26_ip --cfg f1_L4_n28_ip --cfg f1_L4_n28 $L 2>/dev/null | sed "s/^/default /" >> $O/ab.txt || exit 1
done
python3 - "$O/ab.txt" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    tag, js = l.split(" ", 1); d = json.loads(js)
    print(tag, d["cfg"], round(d["ms"], 4), [round(x, 4) for x in d["launch_ms"]])
PY
