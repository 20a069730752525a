#!/bin/bash
# Diagnostic variants of the fused single-launch kernel (NTT_FUSED_DBG bits; wrong outputs allowed).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_fused_dbg4}
mkdir -p $O
for d in 8 64 72 80 68 76 1; do
  echo "[dbg] $d" >&2
  NTT_FUSED_DBG=$d timeout -k 10 120 python -u tools/exp_launches.py --cfg f1_L4_n18_sl --cfg f1_L4_n20_sl --cfg f1_L4_n20 --cfg f1_L4_n24_sl --warmup 20 --steps 30 --out $O/dbg$d.jsonl > $O/dbg$d.log 2>&1 || { tail $O/dbg$d.log >&2; exit 1; }
done
echo "[dbg] done" >&2
