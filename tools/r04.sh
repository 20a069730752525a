#!/bin/bash
# Round-4 GPU session steps (run from the repo root on the box via gpurun).  Every GPU step has its own
# time limit; the first failure ends the session.  Usage: TAG=r04_x tools/r04.sh step [step ...]
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r04}
O=gpurun_out/$TAG
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  echo "[r04] $name" >&2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[r04] $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -40 $O/$name.log >&2; exit $rc; fi
}
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
ARGS="$@"
[ "$ARGS" = final ] && ARGS="tests smoke bench prof pmc configs fs1 reh2"
for s in $ARGS; do
  case $s in
    new) step pytest_new 400 $PYT tests/test_gpu_mplan_copy.py tests/test_gpu_watchdog.py ;;
    sl) step pytest_sl 600 $PYT tests/test_gpu_single_launch.py tests/test_gpu_inplace.py tests/test_gpu_watchdog.py ;;
    dist) step pytest_dist 600 $PYT tests/test_gpu_distributed.py tests/test_gpu_polymul_dist.py tests/test_gpu_mplan_faults.py tests/test_gpu_mplan_copy.py ;;
    tests) step pytest_gpu 1100 $PYT tests -m gpu ;;
    smoke) step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    reh2) step bench_n2_rehearsal 400 env NTT_BENCH_EXCHANGE=host python3 -u bench.py --gpus 2 --steps 20 --warmup 10 ;;
    reh4) step bench_n4_rehearsal 600 env NTT_BENCH_EXCHANGE=host python3 -u bench.py --gpus 4 --steps 10 --warmup 5 ;;
    reh8) step bench_n8_rehearsal 600 env NTT_BENCH_EXCHANGE=host python3 -u bench.py --gpus 8 --steps 10 --warmup 5 ;;
    bench) step bench 300 python3 -u bench.py ;;
    benchd) step bench_driver 300 python3 -u bench.py --steps 20 --warmup 5 ;;
    fs1) step bench_fourstep_w1 300 python3 -u bench.py --four-step --steps 20 --warmup 10 --no-cpu-baseline ;;
    profd) step rocprof_driver 300 rocprofv3 --kernel-trace --stats -d $O/profd -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    prof_plain) step rocprof_plain 200 rocprofv3 --kernel-trace --stats -d $O/prof_plain -o run --output-format csv -- python3 tools/exp_launches.py --cfg f1_L4_n20 --warmup 5 --steps 10 ;;
    prof_ip) step rocprof_ip 200 rocprofv3 --kernel-trace --stats -d $O/prof_ip -o run --output-format csv -- python3 tools/exp_launches.py --cfg f1_L4_n20_ip --warmup 5 --steps 10 ;;
    prof_sl) step rocprof_sl 200 rocprofv3 --kernel-trace --stats -d $O/prof_sl -o run --output-format csv -- python3 tools/exp_launches.py --cfg f1_L4_n20_sl --warmup 5 --steps 10 ;;
    prof) step rocprof_stats 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py ;;
    pmc)
      step pmc_sq 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/pmc/sq -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --prewarm-s 0
      step pmc_fetch 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc/fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --prewarm-s 0
      step pmc_write 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc/write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --prewarm-s 0
      step traffic 60 python -u tools/pmc_to_traffic.py $O/pmc f1_L4_n24_w1 $O/pmc_summary.json ;;
    pmcp)  # the PMC passes, the summary written into this box's profiles/ so a later bench step reports traffic
      step pmc_sq 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/pmc/sq -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --prewarm-s 0
      step pmc_fetch 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc/fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --prewarm-s 0
      step pmc_write 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc/write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --prewarm-s 0
      step traffic 60 bash -c "python -u tools/pmc_to_traffic.py $O/pmc f1_L4_n24_w1 profiles/pmc_summary.json && cp profiles/pmc_summary.json $O/pmc_summary.json" ;;
    limb30)
      step limb30_prep 60 python tools/mb_limb30_check.py prep $O/limb30
      step limb30_run 300 tools/mb_limb30 $O/limb30/consts.bin $O/limb30/xs.bin $O/limb30/rs.bin
      step limb30_verify 120 python tools/mb_limb30_check.py verify $O/limb30 ;;
    c2)  # BASELINE C2 (2^20 BN254) forms: 3 launches, single launch (barriers / dataflow), in place, in place as one kernel
      L="--warmup 50 --steps 200"
      C="--cfg f1_L4_n20 --cfg f1_L4_n20_sl --cfg f1_L4_n20_ip --cfg f1_L4_n20_ip_sl --cfg f1_L4_n19_ip_sl --cfg f1_L4_n18_ip_sl --cfg f1_L4_n18_sl"
      for rep in 1 2; do
        step c2_ab_m1_$rep 200 python -u tools/exp_launches.py $C $L
        cat $O/c2_ab_m1_$rep.log | grep '^{' | sed "s/^/mode1 /" >> $O/c2_ab.txt
        step c2_ab_m0_$rep 200 env NTT_FUSED_MODE=0 python -u tools/exp_launches.py --cfg f1_L4_n20_sl $L
        cat $O/c2_ab_m0_$rep.log | grep '^{' | sed "s/^/mode0 /" >> $O/c2_ab.txt
      done
      step c2_prof 300 rocprofv3 --kernel-trace --stats -d $O/c2prof -o run --output-format csv -- python3 tools/exp_launches.py $C --warmup 20 --steps 100 ;;
    coop)  # the grid-barrier single launches as a cooperative launch (default) and as a plain launch
      L="--warmup 50 --steps 200"
      C="--cfg f1_L4_n20 --cfg f1_L4_n20_sl --cfg f1_L4_n20_ip --cfg f1_L4_n20_ip_sl --cfg f1_L4_n18_sl --cfg f1_L4_n18_ip_sl"
      for rep in 1 2; do
        step coop1_$rep 200 python -u tools/exp_launches.py $C $L
        grep '^{' $O/coop1_$rep.log | sed "s/^/coop /" >> $O/coop_ab.txt
        step coop0_$rep 200 env NTT_FUSED_COOP=0 python -u tools/exp_launches.py $C $L
        grep '^{' $O/coop0_$rep.log | sed "s/^/plain /" >> $O/coop_ab.txt
      done
      step coop0_sl 300 env NTT_FUSED_COOP=0 $PYT tests/test_gpu_single_launch.py ;;
    coop2)  # 2^18 / 2^19: three launches against the plain-launch single launch, same box
      L="--warmup 50 --steps 200"
      C="--cfg f1_L4_n18 --cfg f1_L4_n18_sl --cfg f1_L4_n18_ip --cfg f1_L4_n18_ip_sl --cfg f1_L4_n19 --cfg f1_L4_n19_sl --cfg f1_L4_n19_ip --cfg f1_L4_n19_ip_sl --cfg f2_L4_n20 --cfg f2_L4_n20_sl"
      for rep in 1 2; do
        step coop2p_$rep 200 env NTT_FUSED_COOP=0 python -u tools/exp_launches.py $C $L
        grep '^{' $O/coop2p_$rep.log | sed "s/^/plain /" >> $O/coop2_ab.txt
        step coop2c_$rep 200 python -u tools/exp_launches.py $C $L
        grep '^{' $O/coop2c_$rep.log | sed "s/^/coop /" >> $O/coop2_ab.txt
      done ;;
    t12)  # 4096-element tiles (NTT_TILE_LOG_256=12, one 1024-thread workgroup per CU): 2^20 in two passes
      L="--warmup 50 --steps 200"
      C="--cfg f1_L4_n20 --cfg f2_L4_n20 --cfg f1_L4_n20_inv --cfg f1_L4_n18 --cfg f1_L4_n19 --cfg f1_L4_n21 --cfg f1_L4_n22 --cfg f1_L4_n24"
      for rep in 1 2; do
        step t12b_$rep 300 python -u tools/exp_launches.py $C $L
        grep '^{' $O/t12b_$rep.log | sed "s/^/base /" >> $O/t12_ab.txt
        step t12v_$rep 300 env NTT_LIB_PATH=ntt_amd/libntt_t12.so python -u tools/exp_launches.py $C $L
        grep '^{' $O/t12v_$rep.log | sed "s/^/t12 /" >> $O/t12_ab.txt
      done
      step t12_parity 600 env NTT_LIB_PATH=ntt_amd/libntt_t12.so $PYT tests/test_gpu_parity.py ;;
    t12batch)
      for rep in 1 2; do
        step t12batch_b$rep 300 python -u tools/exp_batch.py --log-n 20 --batches 1,2,4,8
        step t12batch_v$rep 300 env NTT_LIB_PATH=ntt_amd/libntt_t12.so python -u tools/exp_batch.py --log-n 20 --batches 1,2,4,8
      done ;;
    wide)  # 2^20 4-limb plans: one vector's transforms on the 4096-element-tile plan (default) vs off
      L="--warmup 50 --steps 200"
      C="--cfg f1_L4_n20 --cfg f1_L4_n20_inv --cfg f2_L4_n20 --cfg f2_L4_n20_inv"
      step wide_tests 600 $PYT tests/test_gpu_wide_tiles.py tests/test_gpu_single_launch.py tests/test_gpu_parity.py
      for rep in 1 2; do
        step wide1_$rep 200 python -u tools/exp_launches.py $C $L
        grep '^{' $O/wide1_$rep.log | sed "s/^/wide /" >> $O/wide_ab.txt
        step wide0_$rep 200 env NTT_WIDE_TILES=0 python -u tools/exp_launches.py $C $L
        grep '^{' $O/wide0_$rep.log | sed "s/^/off /" >> $O/wide_ab.txt
      done ;;
    naive)  # the reference's `naive` rival: parity, then its time against the default and the other rivals
      step naive_tests 600 $PYT tests/test_gpu_rivals.py
      step naive_bench 300 python -u tools/bench_rivals.py --out $O/rivals.jsonl ;;
    pack)  # pack29 with v_alignbit (no scratch copy) + 32-B reads of the 48-B layout, against the previous build
      L="--warmup 50 --steps 100"
      C="--cfg f2_L6_n24 --cfg f2_L6_n24_inv --cfg f2_L4_n24 --cfg f1_L4_n24 --cfg f1_L4_n20 --cfg f2_L6_n20"
      for rep in 1 2; do
        step packn_$rep 300 python -u tools/exp_launches.py $C $L
        grep '^{' $O/packn_$rep.log | sed "s/^/new /" >> $O/pack_ab.txt
        step packo_$rep 300 env NTT_LIB_PATH=ntt_amd/libntt_old.so python -u tools/exp_launches.py $C $L
        grep '^{' $O/packo_$rep.log | sed "s/^/old /" >> $O/pack_ab.txt
      done ;;
    abmmc) step ab_mmc 600 tools/exp_variants.sh mmc ;;
    ptrace)  # C4 over 8 virtual ranks: kernel + copy traces of the piece schedules
      for c in 1,1 4,4 4,1 1,4; do
        t=$(echo $c | tr , x)
        step ptrace_$t 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/ptrace_$t -o run --output-format csv -- python3 tools/exp_pieces.py --cfg 8,28,$c --reps 3 --forward-only
      done ;;
    ptrace_seq)  # the same configs in ONE process, in bench_configs.py's order (1x1, 4x1, 4x4)
      step ptrace_seq 400 rocprofv3 --kernel-trace --stats -d $O/ptrace_seq -o run --output-format csv -- python3 tools/exp_pieces.py --cfg 8,28,1,1 --cfg 8,28,4,1 --cfg 8,28,4,4 --reps 3 --forward-only ;;
    ptrace_q)  # 4 x 4 with 0..3 extra streams created first: which hardware queue the side stream gets
      for k in 0 1 2 3; do
        step ptrace_q$k 300 rocprofv3 --kernel-trace -d $O/ptrace_q$k -o run --output-format csv -- python3 tools/exp_pieces.py --cfg 8,28,4,4 --reps 3 --forward-only --extra-streams $k
      done ;;
    ctrace) step configs_trace 600 rocprofv3 --kernel-trace -d $O/ctrace -o run --output-format csv -- python3 tools/bench_configs.py --out $O/configs_traced.jsonl ;;
    c5d) step c5dist_1 200 python3 -u tools/exp_c5dist.py --pieces 1 && step c5dist_4 200 python3 -u tools/exp_c5dist.py --pieces 4 ;;
    c5b)  # the same with every exchange unit as one multi-tensor copy, and C4 forwards both ways
      X="python3 -u tools/exp_c5dist.py --no-profile"
      step c5b_1 200 $X --batched --pieces 1 && step c5b_4 200 $X --batched --pieces 4 &&
      step c4_1 200 $X --log-n 28 --ops forward --steps 5 --pieces 1 &&
      step c4_1b 200 $X --log-n 28 --ops forward --steps 5 --pieces 1 --batched &&
      step c4_4 200 $X --log-n 28 --ops forward --steps 5 --pieces 4 &&
      step c4_4b 200 $X --log-n 28 --ops forward --steps 5 --pieces 4 --batched ;;
    c5dt) step c5dist_trace 300 rocprofv3 --kernel-trace --stats -d $O/c5dt -o run --output-format csv -- python3 tools/exp_c5dist.py --pieces 1 --steps 10 ;;
    configs) step configs 600 python -u tools/bench_configs.py --out $O/configs.jsonl ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
  esac
done
echo "[r04] done" >&2
