#!/bin/bash
# GPU-box validation run: parity tests, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; after a crash / fault / timeout the
# script stops (no further GPU work in the same call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }

STEPS="${STEPS:-tests bench prof}"
for s in $STEPS; do
  case $s in
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$? ;;
    tests)
      # PYTEST_K: a -k expression (may contain spaces); PYTEST_ARGS: extra words
      if [ -n "${PYTEST_K:-}" ]; then
        timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 400 -p no:cacheprovider -k "$PYTEST_K" ${PYTEST_ARGS:-} > $OUT/gpu_tests.log 2>&1; rc=$?
      else
        timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 400 -p no:cacheprovider ${PYTEST_ARGS:-} > $OUT/gpu_tests.log 2>&1; rc=$?
      fi
      if [ $rc -ge 2 ] && [ $rc -le 5 ]; then rc=0; fi ;;  # pytest usage/collection codes are not GPU faults
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench${SFX:-}.json 2> $OUT/bench${SFX:-}.err; rc=$? ;;
    prof)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof${SFX:-} -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile --no-knn ${BENCH_ARGS:-} > $GRAFT_REPO_ROOT/$OUT/prof_bench${SFX:-}.json 2> $GRAFT_REPO_ROOT/$OUT/prof${SFX:-}.err); rc=$? ;;
    online)
      # the configs[4]-shaped mapper loop (graph-replayed steady state by default)
      timeout -k 10 600 python tools/bench_online.py ${ONLINE_ARGS:-} > $OUT/online${SFX:-}.json 2> $OUT/online${SFX:-}.err; rc=$? ;;
    online0)
      # ... the same run with every iteration eager (A/B)
      WGSR_ONLINE_GRAPH=0 timeout -k 10 600 python tools/bench_online.py ${ONLINE_ARGS:-} > $OUT/online0${SFX:-}.json 2> $OUT/online0${SFX:-}.err; rc=$? ;;
    onlineprof)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/onlineprof${SFX:-} -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/bench_online.py --keyframes 4 --init-iters 100 --iters 150 --refine-iters 100 ${ONLINE_ARGS:-} > $GRAFT_REPO_ROOT/$OUT/onlineprof${SFX:-}.json 2> $GRAFT_REPO_ROOT/$OUT/onlineprof${SFX:-}.err); rc=$? ;;
    f1)
      timeout -k 10 300 python tools/bench_f1.py > $OUT/bench_f1.json 2> $OUT/bench_f1.err; rc=$? ;;
    f2)
      timeout -k 10 300 python tools/bench_f2.py > $OUT/bench_f2.json 2> $OUT/bench_f2.err; rc=$? ;;
    f2prof)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/f2prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/bench_f2.py > $GRAFT_REPO_ROOT/$OUT/f2prof.json 2> $GRAFT_REPO_ROOT/$OUT/f2prof.err); rc=$? ;;
    f3)
      timeout -k 10 300 python tools/bench_f3.py > $OUT/bench_f3.json 2> $OUT/bench_f3.err; rc=$? ;;
    f3prof)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/f3prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/bench_f3.py > $GRAFT_REPO_ROOT/$OUT/f3prof.json 2> $GRAFT_REPO_ROOT/$OUT/f3prof.err); rc=$? ;;
    trace)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $GRAFT_REPO_ROOT/$OUT/trace${SFX:-} -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-profile --no-knn ${BENCH_ARGS:-} > /dev/null 2> $GRAFT_REPO_ROOT/$OUT/trace${SFX:-}.err); rc=$? ;;
    listpmc)
      (cd /tmp && timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/$OUT/pmc_list.txt 2>&1); rc=$? ;;
    f1prof)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/f1prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/bench_f1.py --iters 20 > $GRAFT_REPO_ROOT/$OUT/f1prof.json 2> $GRAFT_REPO_ROOT/$OUT/f1prof.err); rc=$? ;;
    pmc_fetch)
      (cd /tmp && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/pmc_fetch${SFX:-} -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-knn ${BENCH_ARGS:-} > /dev/null 2> $GRAFT_REPO_ROOT/$OUT/pmc_fetch${SFX:-}.err); rc=$? ;;
    pmc_write)
      (cd /tmp && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/pmc_write${SFX:-} -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-knn ${BENCH_ARGS:-} > /dev/null 2> $GRAFT_REPO_ROOT/$OUT/pmc_write${SFX:-}.err); rc=$? ;;
    pmc_sq)
      (cd /tmp && timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/pmc_sq${SFX:-} -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-knn ${BENCH_ARGS:-} > /dev/null 2> $GRAFT_REPO_ROOT/$OUT/pmc_sq${SFX:-}.err); rc=$? ;;
    pmc_sq2)
      # VALU pipe occupancy (SQ_ACTIVE_INST_VALU, quad-cycles incl. multi-cycle ops) and the SQ clock (SQ_BUSY_CYCLES per SE)
      (cd /tmp && timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VALU_TRANS_F32 SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/pmc_sq2${SFX:-} -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-knn ${BENCH_ARGS:-} > /dev/null 2> $GRAFT_REPO_ROOT/$OUT/pmc_sq2${SFX:-}.err); rc=$? ;;
    pmc_ta)
      # the vector memory path: TA (address) / TD (data) busy and stalls, TCP (L1) tag accesses and L2 waits
      (cd /tmp && timeout -k 10 600 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/pmc_ta${SFX:-} -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-knn ${BENCH_ARGS:-} > /dev/null 2> $GRAFT_REPO_ROOT/$OUT/pmc_ta${SFX:-}.err); rc=$? ;;
    ab)
      # AB_LIBS="name ...": bench each lib/variants/<name>.so ("base" = lib/libwgsr.so), twice, interleaved
      rc=0
      # an entry may carry one env setting: name:VAR=value (e.g. base:WGSR_SORT=onesweep)
      for rep in $(seq 1 ${REPS:-2}); do for v in ${AB_LIBS}; do
        lname=${v%%:*}; envset=""; tag=$lname
        if [ "$v" != "$lname" ]; then envset=${v#*:}; tag=${lname}_${envset//=/_}; fi
        if [ "$lname" = base ]; then lib=wildgs-slam-blackwell_amd/lib/libwgsr.so; else lib=wildgs-slam-blackwell_amd/lib/variants/$lname.so; fi
        env WGSR_LIB=$lib $envset timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/ab_${tag}${SFX:-}_$rep.json 2> $OUT/ab_${tag}${SFX:-}_$rep.err; rc=$?
        if [ $rc -ne 0 ]; then break 2; fi
      done; done ;;
    knnab)
      # distCUDA2 timings per AB_LIBS entry (tools/bench_knn.py), then a kernel profile of the base lib
      rc=0
      for v in ${AB_LIBS}; do
        if [ "$v" = base ]; then lib=wildgs-slam-blackwell_amd/lib/libwgsr.so; else lib=wildgs-slam-blackwell_amd/lib/variants/$v.so; fi
        WGSR_LIB=$lib timeout -k 10 300 python tools/bench_knn.py > $OUT/knn_$v.json 2> $OUT/knn_$v.err; rc=$?
        if [ $rc -ne 0 ]; then break; fi
      done
      if [ $rc -eq 0 ]; then
        (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/knnprof -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/bench_knn.py > /dev/null 2> $GRAFT_REPO_ROOT/$OUT/knnprof.err); rc=$?
      fi ;;
    knnpmc)
      (cd /tmp && timeout -k 10 300 rocprofv3 --pmc ${PMC_COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES} --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/knnpmc -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/bench_knn.py > /dev/null 2> $GRAFT_REPO_ROOT/$OUT/knnpmc.err); rc=$? ;;
    pmc_custom)
      # PMC_COUNTERS="A B C" PMC_NAME=name: one extra counter pass (SQ block: at most 8 counters)
      (cd /tmp && timeout -k 10 600 rocprofv3 --pmc ${PMC_COUNTERS} --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/pmc_${PMC_NAME:-custom} -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-knn > /dev/null 2> $GRAFT_REPO_ROOT/$OUT/pmc_${PMC_NAME:-custom}.err); rc=$? ;;
    pmcab)
      # one PMC_COUNTERS pass per AB_LIBS entry (bench.py, 3 steps) -> pmc_ab_<name>/
      rc=0
      for v in ${AB_LIBS}; do
        if [ "$v" = base ]; then lib=wildgs-slam-blackwell_amd/lib/libwgsr.so; else lib=wildgs-slam-blackwell_amd/lib/variants/$v.so; fi
        (cd /tmp && WGSR_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 rocprofv3 --pmc ${PMC_COUNTERS} --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/pmc_ab_$v -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-knn ${BENCH_ARGS:-} > /dev/null 2> $GRAFT_REPO_ROOT/$OUT/pmc_ab_$v.err); rc=$?
        if [ $rc -ne 0 ]; then break; fi
      done ;;
    profenv)
      # ENV_AB="base NAME=VALUE ...": rocprofv3 kernel stats of bench.py per setting (tools/prof_env.sh)
      bash tools/prof_env.sh; rc=$? ;;
    dp2)
      # N = 2 rehearsal of the multi-GPU bench path on the box's one GPU: two
      # ranks share cuda:0 over gloo (device tensors staged through host memory)
      WGSR_BENCH_BACKEND=gloo WGSR_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 \
        --no-profile ${BENCH_ARGS:-} > $OUT/bench_dp2.json 2> $OUT/bench_dp2.err; rc=$? ;;
    *) echo "unknown step $s"; rc=0 ;;
  esac
  echo "$s rc=$rc" | tee -a $OUT/steps.log
  if fatal $rc; then echo "stopping after fatal rc=$rc in $s"; exit $rc; fi
done
exit 0
