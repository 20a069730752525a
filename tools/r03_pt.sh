#!/bin/bash
# Round-3 GPU step: the checked build's test, then the P path with 16384-element tiles (libntt_pt14.so:
# 16 elements per thread, >= 32 columns per column-pass workgroup) -- parity under NTT_LIB_PATH, then
# an interleaved per-launch A/B against the product build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_pt}
mkdir -p $O
[ -n "$SKIP_DEBUG" ] || timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_debug_build.py \
  > $O/pytest_debug.log 2>&1 || { tail -30 $O/pytest_debug.log; exit 1; }
[ -n "$SKIP_DEBUG" ] || tail -2 $O/pytest_debug.log
[ -n "$SKIP_PARITY" ] || NTT_LIB_PATH=ntt_amd/libntt_pt14.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_ref_pinned.py tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_inplace.py tests/test_gpu_rivals.py \
  > $O/pytest_pt14.log 2>&1 || { tail -30 $O/pytest_pt14.log; exit 1; }
[ -n "$SKIP_PARITY" ] || tail -2 $O/pytest_pt14.log
CFG="--cfg f0_L1_n26 --cfg f0_L1_n24 --cfg f0_L1_n22 --cfg f0_L1_n20 --cfg f0_L1_n26_ip"
for rep in 1 2; do
  for v in base pt14; do
    lib=ntt_amd/libntt.so; [ $v = pt14 ] && lib=ntt_amd/libntt_pt14.so
    NTT_LIB_PATH=$lib timeout -k 10 180 python -u tools/exp_launches.py $CFG --warmup 30 --steps 50 > $O/$v$rep.jsonl 2> $O/$v$rep.log || { tail $O/$v$rep.log; exit 1; }
  done
done
for f in $O/base1.jsonl $O/pt141.jsonl $O/base2.jsonl $O/pt142.jsonl; do echo "== $f"; python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d['cfg'], round(d['ms'],4), d['passes'], [round(x,4) for x in d['launch_ms']])
" $f; done
