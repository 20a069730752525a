#!/bin/bash
# Round-3 GPU step: 4-B element-format twiddle tables for the P engines (EngPI in-place pass 1).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_tabw}
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_inplace.py tests/test_gpu_rivals.py tests/test_gpu_parity.py tests/test_gpu_ref_pinned.py \
  tests/test_gpu_edges.py tests/test_gpu_coset_mont.py tests/test_gpu_dropin_c.py tests/test_gpu_distributed.py \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
  timeout -k 10 180 python -u tools/exp_launches.py --cfg f0_L1_n26_ip --cfg f0_L1_n26 --cfg f0_L1_n24_ip --cfg f0_L1_n24 \
    --warmup 30 --steps 50 > $O/launches$rep.jsonl 2> $O/launches$rep.log || { tail $O/launches$rep.log; exit 1; }
done
cat $O/launches1.jsonl $O/launches2.jsonl
