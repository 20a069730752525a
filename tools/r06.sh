#!/bin/bash
# Round-6 GPU session steps (run from the repo root on the box via gpurun).  Every GPU step has its own
# time limit; the first failure ends the session.  Usage: TAG=r06_x tools/r06.sh step [step ...]
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r06}
O=gpurun_out/$TAG
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  echo "[r06] $name" >&2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[r06] $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -40 $O/$name.log >&2; exit $rc; fi
}
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
BQ="--steps 3 --warmup 1 --no-cpu-baseline --no-parity --prewarm-s 0"
ARGS="$@"
[ "$ARGS" = final ] && ARGS="tests smoke bench prof pmc configs fs1"
for s in $ARGS; do
  case $s in
    tp) step two_pass_check 300 env NTT_TWO_PASS_24=1 python3 -u tools/exp_two_pass.py ;;
    tp2) step two_pass_check_bls 300 env NTT_TWO_PASS_24=1 python3 -u tools/exp_two_pass.py --fid 2 ;;
    ab24) # 2^24 BN254 forward: 8 + 8 + 8 (default) against 12 + 12 (NTT_TWO_PASS_24=1), with and without the
      # XCD-grouped order of the one-column passes; two interleaved repetitions, fresh process each
      for i in 1 2; do
        step ab_default_$i 200 python3 -u tools/exp_launches.py --cfg f1_L4_n24 --cfg f1_L4_n24_inv --warmup 50 --steps 200 --out $O/ab_default_$i.jsonl
        step ab_tp_$i 200 env NTT_TWO_PASS_24=1 python3 -u tools/exp_launches.py --cfg f1_L4_n24 --cfg f1_L4_n24_inv --warmup 50 --steps 200 --out $O/ab_tp_$i.jsonl
        step ab_tp_noxcd_$i 200 env NTT_TWO_PASS_24=1 NTT_XCD_ORDER=3 python3 -u tools/exp_launches.py --cfg f1_L4_n24 --warmup 50 --steps 200 --out $O/ab_tp_noxcd_$i.jsonl
      done ;;
    pmc24) # the same two schedules under PMC: durations (kernel trace) and GRBM_GUI_ACTIVE cycles from ONE
      # run, then HBM bytes in their own passes
      for v in ${PMC_V:-default tp}; do
        E=""; [ $v = tp ] && E="NTT_TWO_PASS_24=1"
        step pmc_${v}_sq 120 env $E rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $O/pmc_$v/sq -o run --output-format csv -- python3 bench.py $BQ
        step pmc_${v}_fetch 120 env $E rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_$v/fetch -o run --output-format csv -- python3 bench.py $BQ
        step pmc_${v}_write 120 env $E rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_$v/write -o run --output-format csv -- python3 bench.py $BQ
        step pmc_${v}_l2 120 env $E rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $O/pmc_$v/l2 -o run --output-format csv -- python3 bench.py $BQ
      done ;;
    new) step pytest_new 900 $PYT tests/test_gpu_fused_order.py tests/test_gpu_wide_tiles.py tests/test_gpu_single_launch.py tests/test_gpu_watchdog.py ;;
    dist1) step pytest_dist1 600 $PYT tests/test_gpu_distributed.py -k "rccl_world1" ;;
    wt) # timing only: k_fused2b with plain (not write-through) pass-1 stores (libntt_wt.so, results not
      # guaranteed) against the product, per-phase trace and per-call time, interleaved twice
      for i in 1 2; do
        step trace_prod_$i 300 python3 -u tools/exp_fused_trace.py --calls 60 --out $O/trace_prod_$i.jsonl
        step trace_wt_$i 300 env NTT_LIB_PATH=ntt_amd/libntt_wt.so python3 -u tools/exp_fused_trace.py --calls 60 --out $O/trace_wt_$i.jsonl
        step c2_prod_$i 200 python3 -u tools/exp_launches.py --cfg f1_L4_n20 --cfg f1_L4_n20_sl --warmup 50 --steps 200 --out $O/c2_prod_$i.jsonl
        step c2_wt_$i 200 env NTT_LIB_PATH=ntt_amd/libntt_wt.so python3 -u tools/exp_launches.py --cfg f1_L4_n20 --cfg f1_L4_n20_sl --warmup 50 --steps 200 --out $O/c2_wt_$i.jsonl
      done ;;
    rel) # timing only: k_fused2b with plain pass-1 stores and one agent-scope release per workgroup before
      # the barrier (libntt_rel.so) against the product, interleaved twice
      for i in 1 2; do
        step trace_prod_$i 300 python3 -u tools/exp_fused_trace.py --calls 60 --out $O/trace_prod_$i.jsonl
        step trace_rel_$i 300 env NTT_LIB_PATH=ntt_amd/libntt_rel.so python3 -u tools/exp_fused_trace.py --calls 60 --out $O/trace_rel_$i.jsonl
        step c2_prod_$i 200 python3 -u tools/exp_launches.py --cfg f1_L4_n20 --cfg f1_L4_n20_sl --warmup 50 --steps 200 --out $O/c2_prod_$i.jsonl
        step c2_rel_$i 200 env NTT_LIB_PATH=ntt_amd/libntt_rel.so python3 -u tools/exp_launches.py --cfg f1_L4_n20 --cfg f1_L4_n20_sl --warmup 50 --steps 200 --out $O/c2_rel_$i.jsonl
      done
      step rel_parity 300 env NTT_LIB_PATH=ntt_amd/libntt_rel.so python3 -u -c "
import sys, torch; sys.path.insert(0, '.')
from ntt_amd.ntt import NTTPlan
a = NTTPlan(1, 20, 4, single_launch=True); r = NTTPlan(1, 20, 4)
bad = 0
for s in range(20):
    x = a.fill(a.empty(), 'random', seed=s); y = x.clone(); a.forward(x); r.forward(y); bad += int(not torch.equal(x, y))
print('mismatches', bad, 'of 20')" ;;
    trace) step fused_trace 300 python3 -u tools/exp_fused_trace.py --calls 60 --out $O/fused_trace.jsonl ;;
    c2) # the C2 forms, two interleaved repetitions, fresh process each: the library's single-launch
      # ordering on (default) and off (NTT_FUSED_ORDER=0)
      C2="--cfg f1_L4_n20 --cfg f1_L4_n20_sl --cfg f1_L4_n20_ip_sl --cfg f1_L4_n19_sl --cfg f1_L4_n19_ip_sl"
      for i in ${C2_REPS:-1 2}; do
        step c2_order_$i 200 python3 -u tools/exp_launches.py $C2 --warmup 50 --steps 200 --out $O/c2_order_$i.jsonl
        step c2_noorder_$i 200 env NTT_FUSED_ORDER=0 python3 -u tools/exp_launches.py $C2 --warmup 50 --steps 200 --out $O/c2_noorder_$i.jsonl
      done ;;
    tests) step pytest_gpu 1100 $PYT tests -m gpu ;;
    dbg) step pytest_dbg 600 $PYT tests/test_gpu_debug_build.py ;;
    smoke) step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 300 python3 -u bench.py ;;
    benchd) step bench_driver 300 python3 -u bench.py --steps 20 --warmup 5 ;;
    fs1) step bench_fourstep_w1 300 python3 -u bench.py --four-step --steps 20 --warmup 10 --no-cpu-baseline ;;
    prof) step rocprof_stats 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py ;;
    configs) step configs 900 python3 -u tools/bench_configs.py --out $O/configs.jsonl ;;
    pmc_rl) step pmc_ranklocal 900 env O=$O/pmc_rl WORLDS="1 2 4 8" bash tools/pmc_ranklocal.sh ;;
    reh2) step bench_n2_rehearsal 400 env NTT_BENCH_EXCHANGE=host python3 -u bench.py --gpus 2 --steps 20 --warmup 10 ;;
    reh4) step bench_n4_rehearsal 600 env NTT_BENCH_EXCHANGE=host python3 -u bench.py --gpus 4 --steps 10 --warmup 5 ;;
    reh8) step bench_n8_rehearsal 600 env NTT_BENCH_EXCHANGE=host python3 -u bench.py --gpus 8 --steps 10 --warmup 5 ;;
    rl28) step ranklocal_c4 300 python3 -u tools/exp_ranklocal.py --log-n 28 --worlds 8 --warmup 5 --steps 10 --out $O/ranklocal_c4.jsonl ;;
    stress) step stress 1000 python3 -u tools/stress_sync.py --reps ${STRESS_REPS:-400} --out $O/stress.jsonl ;;
    pmc)
      step pmc_sq 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/pmc/sq -o run --output-format csv -- python3 bench.py $BQ
      step pmc_fetch 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc/fetch -o run --output-format csv -- python3 bench.py $BQ
      step pmc_write 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc/write -o run --output-format csv -- python3 bench.py $BQ ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
  esac
done
echo "[r06] done" >&2
