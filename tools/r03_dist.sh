#!/bin/bash
# Round-3 GPU step: the two-sided piece schedule (FourStep column pieces, ntt_rplan_*_piece).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_dist}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_distributed.py tests/test_gpu_polymul_dist.py tests/test_gpu_mplan_faults.py tests/test_gpu_parity.py \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
