#!/bin/bash
# In-place plans with the digit reversal fused into the final pass (k_final_ipn): GPU tests, A/B
# against the separate tile-swap pass (NTT_IPN=0) and the default ping-pong schedule.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_ipn}
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  echo "[ipn] $name" >&2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[ipn] $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -30 $O/$name.log >&2; exit $rc; fi
}
step pytest 600 python -u -m pytest tests/test_gpu_inplace.py tests/test_gpu_dropin_c.py -x -v --timeout 200 --timeout-method thread
for k in 1 0 1 0; do
  NTT_IPN=$k step ab$k 300 python -u tools/exp_launches.py --cfg f1_L4_n24_ip --cfg f1_L4_n24 --cfg f0_L1_n26_ip --cfg f0_L1_n26 --cfg f0_L1_n24_ip --cfg f1_L4_n20_ip --out $O/ab_ipn$k.jsonl
done
NTT_IPN=1 step ab28 300 python -u tools/exp_launches.py --cfg f1_L4_n28_ip --cfg f1_L4_n28 --warmup 3 --steps 5 --out $O/ab28_ipn1.jsonl
NTT_IPN=0 step ab28b 300 python -u tools/exp_launches.py --cfg f1_L4_n28_ip --warmup 3 --steps 5 --out $O/ab28_ipn0.jsonl
echo "[ipn] done" >&2
