#!/bin/bash
# Round-5 GPU session steps (run from the repo root on the box via gpurun).  Every GPU step has its own
# time limit; the first failure ends the session.  Usage: TAG=r05_x tools/r05.sh step [step ...]
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r05}
O=gpurun_out/$TAG
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  echo "[r05] $name" >&2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[r05] $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -40 $O/$name.log >&2; exit $rc; fi
}
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
C2="--cfg f1_L4_n20 --cfg f1_L4_n20_sl --cfg f1_L4_n20_ip --cfg f1_L4_n20_ip_sl --cfg f2_L4_n20_sl --cfg f2_L4_n20_ip_sl"
ARGS="$@"
[ "$ARGS" = final ] && ARGS="tests smoke bench prof pmc configs fs1"
for s in $ARGS; do
  case $s in
    new) step pytest_new 900 $PYT tests/test_gpu_single_launch.py tests/test_gpu_wide_tiles.py tests/test_gpu_watchdog.py tests/test_gpu_rivals.py ;;
    dist) step pytest_dist 900 $PYT tests/test_gpu_distributed.py tests/test_gpu_polymul_dist.py tests/test_gpu_mplan_faults.py tests/test_gpu_mplan_copy.py ;;
    dbg) step pytest_dbg 600 $PYT tests/test_gpu_debug_build.py ;;
    tests) step pytest_gpu 1100 $PYT tests -m gpu ;;
    smoke) step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 300 python3 -u bench.py ;;
    reh2) step bench_n2_rehearsal 400 env NTT_BENCH_EXCHANGE=host python3 -u bench.py --gpus 2 --steps 20 --warmup 10 ;;
    reh4) step bench_n4_rehearsal 600 env NTT_BENCH_EXCHANGE=host python3 -u bench.py --gpus 4 --steps 10 --warmup 5 ;;
    reh8) step bench_n8_rehearsal 600 env NTT_BENCH_EXCHANGE=host python3 -u bench.py --gpus 8 --steps 10 --warmup 5 ;;
    benchd) step bench_driver 300 python3 -u bench.py --steps 20 --warmup 5 ;;
    fs1) step bench_fourstep_w1 300 python3 -u bench.py --four-step --steps 20 --warmup 10 --no-cpu-baseline ;;
    c2) # the C2 forms, two interleaved repetitions, fresh process each (ms per transform over 200 calls)
      for i in 1 2; do
        step c2_wide_$i 200 python3 -u tools/exp_launches.py $C2 --warmup 50 --steps 200 --out $O/c2_wide_$i.jsonl
        step c2_t10_$i 200 env NTT_WIDE_TILES=0 python3 -u tools/exp_launches.py $C2 --warmup 50 --steps 200 --out $O/c2_t10_$i.jsonl
      done ;;
    prof_c2) step rocprof_c2 200 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 tools/exp_launches.py --cfg f1_L4_n20_sl --cfg f1_L4_n20_ip_sl --cfg f1_L4_n20 --warmup 5 --steps 20 ;;
    prof_coop) step rocprof_coop 200 env NTT_WIDE_TILES=0 rocprofv3 --kernel-trace --stats -d $O/prof_coop -o run --output-format csv -- python3 tools/exp_launches.py --cfg f1_L4_n20_sl --warmup 5 --steps 20 ;;
    rl) step ranklocal_fwd 300 python3 -u tools/exp_ranklocal.py --out $O/ranklocal_fwd.jsonl
        step ranklocal_inv 300 python3 -u tools/exp_ranklocal.py --inverse --out $O/ranklocal_inv.jsonl ;;
    rl28) step ranklocal_c4 300 python3 -u tools/exp_ranklocal.py --log-n 28 --worlds 8 --warmup 5 --steps 10 --out $O/ranklocal_c4.jsonl ;;
    rl_split) for v in 8 9; do step ranklocal_n2_$v 300 env NTT_FS_LOG_N2=$v python3 -u tools/exp_ranklocal.py --out $O/ranklocal_n2_$v.jsonl; done ;;
    rl_ab) # the split rule's A/B on one box: default (16 + 8 since round 5) against 14 + 10, forward and inverse, twice
      for i in 1 2; do
        step rl_default_fwd_$i 300 python3 -u tools/exp_ranklocal.py --out $O/rl_default_fwd_$i.jsonl
        step rl_n2_10_fwd_$i 300 env NTT_FS_LOG_N2=10 python3 -u tools/exp_ranklocal.py --out $O/rl_n2_10_fwd_$i.jsonl
      done
      step rl_default_inv 300 python3 -u tools/exp_ranklocal.py --inverse --out $O/rl_default_inv.jsonl
      step rl_n2_10_inv 300 env NTT_FS_LOG_N2=10 python3 -u tools/exp_ranklocal.py --inverse --out $O/rl_n2_10_inv.jsonl ;;
    rl_sh) # pass-1 Shoup tables of the 2^16 column transforms: default against NTT_SHOUP_OUTER=1, twice
      for i in 1 2; do
        step rl_sh_default_$i 300 python3 -u tools/exp_ranklocal.py --out $O/rl_sh_default_$i.jsonl
        step rl_sh_off_$i 300 env NTT_SHOUP_OUTER=1 python3 -u tools/exp_ranklocal.py --out $O/rl_sh_off_$i.jsonl
      done ;;
    rows_t) step pytest_rows 600 $PYT tests/test_gpu_rows.py tests/test_gpu_distributed.py tests/test_gpu_polymul_dist.py tests/test_gpu_mplan_copy.py tests/test_gpu_debug_build.py ;;
    rows_b) RB="--cfg f1_L4_n3_b15 --cfg f1_L4_n4_b15 --cfg f1_L4_n5_b15 --cfg f1_L4_n6_b15 --cfg f1_L4_n7_b15 --cfg f1_L4_n7_inv_b15 --cfg f2_L4_n7_b15"
      for i in 1 2; do
        step batchs_rows_on_$i 200 python3 -u tools/exp_launches.py $RB --warmup 30 --steps 100 --out $O/batchs_rows_on_$i.jsonl
        step batchs_rows_off_$i 200 env NTT_ROWS=0 python3 -u tools/exp_launches.py $RB --warmup 30 --steps 100 --out $O/batchs_rows_off_$i.jsonl
      done ;;
    rows_ab) # KIND_ROWS (several row transforms per workgroup) against NTT_ROWS=0 (one per workgroup), twice:
      # rank-local four-step launches at G = 1..8 and batched short transforms
      RB="--cfg f1_L4_n8_b15 --cfg f1_L4_n8_inv_b15 --cfg f1_L4_n7_b15 --cfg f1_L4_n9_b14 --cfg f1_L4_n6_b15"
      [ -n "$RB_CFG" ] && RB="$RB_CFG"
      for i in 1 2; do
        step rl_rows_on_$i 300 python3 -u tools/exp_ranklocal.py --out $O/rl_rows_on_$i.jsonl
        step rl_rows_off_$i 300 env NTT_ROWS=0 python3 -u tools/exp_ranklocal.py --out $O/rl_rows_off_$i.jsonl
        step batch_rows_on_$i 200 python3 -u tools/exp_launches.py $RB --warmup 30 --steps 100 --out $O/batch_rows_on_$i.jsonl
        step batch_rows_off_$i 200 env NTT_ROWS=0 python3 -u tools/exp_launches.py $RB --warmup 30 --steps 100 --out $O/batch_rows_off_$i.jsonl
      done
      step rl_rows_on_inv 300 python3 -u tools/exp_ranklocal.py --inverse --out $O/rl_rows_on_inv.jsonl
      step rl_rows_off_inv 300 env NTT_ROWS=0 python3 -u tools/exp_ranklocal.py --inverse --out $O/rl_rows_off_inv.jsonl ;;
    prof_configs) step rocprof_configs 900 rocprofv3 --kernel-trace --stats -d $O/prof_configs -o run --output-format csv -- python3 tools/bench_configs.py --out $O/configs_traced.jsonl ;;
    pmc_rl) step pmc_ranklocal 900 env O=$O/pmc_rl bash tools/pmc_ranklocal.sh ;;
    rivals) step rivals 600 python3 -u tools/bench_rivals.py --out $O/rivals.jsonl ;;
    prof) step rocprof_stats 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py ;;
    configs) step configs 900 python3 -u tools/bench_configs.py --out $O/configs.jsonl ;;
    pmc)
      step pmc_sq 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/pmc/sq -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --prewarm-s 0
      step pmc_fetch 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc/fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --prewarm-s 0
      step pmc_write 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc/write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --prewarm-s 0 ;;
    # the exit-time SIGSEGV of cooperative launches under rocprofv3: the probe
    # dumps /proc/self/maps at Python exit; tools/symbolize_trace.py resolves the trace.  probe_coop is
    # expected to crash at exit: run it LAST in a call.
    probe_plain) step probe_plain 200 rocprofv3 --kernel-trace --stats -d $O/probe_plain -o run --output-format csv -- python3 tools/exit_crash_probe.py $O/maps_plain.txt --coop 0 ;;
    probe_coop) step probe_coop 200 rocprofv3 --kernel-trace --stats -d $O/probe_coop -o run --output-format csv -- python3 tools/exit_crash_probe.py $O/maps_coop.txt --coop 1 ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
  esac
done
echo "[r05] done" >&2
