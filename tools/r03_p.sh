#!/bin/bash
# Round-3 GPU step: shim-cache / lazy-table tests, then the P469762049 (SSIP field) 2^26 per-pass
# evidence: per-launch HIP-event times, rocprofv3 kernel-trace stats, FETCH_SIZE and WRITE_SIZE
# passes (each its own rocprofv3 run, never combined with trace domains).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_p}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_shim_cache.py tests/test_gpu_ref_pinned.py tests/test_gpu_inplace.py tests/test_gpu_parity.py tests/test_gpu_edges.py \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
CMD="python3 tools/exp_launches.py --cfg f0_L1_n26 --cfg f0_L1_n26_ip --warmup 20 --steps 30"
timeout -k 10 120 $CMD > $O/launches.jsonl 2> $O/launches.log || { tail $O/launches.log; exit 1; }
cat $O/launches.jsonl
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- $CMD > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc/fetch -o run --output-format csv -- \
  python3 tools/exp_launches.py --cfg f0_L1_n26 --warmup 2 --steps 3 > $O/pmc_fetch.log 2>&1 || { tail $O/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc/write -o run --output-format csv -- \
  python3 tools/exp_launches.py --cfg f0_L1_n26 --warmup 2 --steps 3 > $O/pmc_write.log 2>&1 || { tail $O/pmc_write.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc $O/pmc_counters.json > $O/pmc_summary.txt 2>&1 || true
echo "[r03_p] done"
