#!/bin/bash
# Profile session of one round: every GPU step under its own time limit; stop
# at the first crash / timeout.  Outputs under gpurun_out/$ROUND/ (the
# summaries are copied to profiles/$ROUND/ afterwards; trace csvs dropped).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
# (round 5 profiled with KORALI_AMD_PLAIN_LAUNCH=1 because
#  rocprofv3 faulted at exit after a cooperative launch; PLAIN=1 restores that)
# round 6: the product's cooperative launches (one HIP+HSA pair under the profiler, korali_amd/__init__.py)
[ -n "$PLAIN" ] && export KORALI_AMD_PLAIN_LAUNCH=1
R=$PWD
O=$R/gpurun_out/${ROUND:-r6}
mkdir -p $O
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a "$O/steps.log"
  (cd /tmp && timeout -k 10 "$secs" "$@") > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$O/steps.log"
  tail -3 "$O/$name.log"
  # keep what is copied back small (<64 MiB): stats only, no per-dispatch traces
  [ "$name" = timeline ] && python $R/tools/timeline_c2.py $O/tl_c2 4 > $O/timeline_c2.txt 2>&1
  find $O -name "*kernel_trace.csv" -delete
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "FATAL step $name rc=$rc"; exit $rc; fi
  return 0
}
# per-kernel KB per dispatch from a FETCH_SIZE and a WRITE_SIZE pass, then
# the per-dispatch counter files are dropped
pmcsum() {
  python $R/tools/pmc_summary.py $O/$1 $O/$2 > $O/$3 && find $O/$1 $O/$2 -name "*counter_collection.csv" -delete
  head -12 $O/$3
}
for s in ${STEPS:-tests}; do
  case $s in
    tests) step tests 1000 python -u -m pytest $R/tests -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider --rootdir $R ;;
    avail) step avail 60 rocprofv3 --list-avail ;;
    bench) step bench 300 python $R/bench.py --steps 200 --warmup 10 ;;
    quick) step quick 200 python $R/bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-c1 ;;
    c3) step c3 400 python $R/bench.py --workload c3 --steps 40 --warmup 3 ;;
    c4) step c4 400 python $R/bench.py --workload c4 --steps 20 --warmup 3 ;;
    cpu) step cpu 200 bash -c "$R/tools/host_tridiag_phases 128 400; $R/tools/host_tridiag_phases 512 12; $R/tools/chase_bench 128 300; $R/tools/chase_bench 512 20"
         cat $O/cpu.log ;;
    timeline) step timeline 300 rocprofv3 --kernel-trace -d $O/tl_c2 -o run --output-format csv -- python $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-c1 ;;
    prof) step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c1 ;;
    profc3) step profc3 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python $R/bench.py --workload c3 --steps 20 --warmup 2 --no-cpu-baseline ;;
    profc4) step profc4 300 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python $R/bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline ;;
    profc4dev) step profc4dev 300 env KORALI_AMD_TRIDIAG=mw2 rocprofv3 --kernel-trace --stats -d $O/prof_c4dev -o run --output-format csv -- python $R/bench.py --workload c4 --steps 6 --warmup 2 --no-cpu-baseline ;;
    pmcf) step pmcf 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run --output-format csv -- python $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-c1 ;;
    pmcw) step pmcw 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run --output-format csv -- python $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-c1
          pmcsum pmc_fetch pmc_write c2_pmc_traffic.csv ;;
    pmcm) step pmcm 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_mfma -o run --output-format csv -- python $R/bench.py --steps 20 --warmup 2 --cov mfma --no-cpu-baseline
          python $R/tools/pmc_mfma_summary.py $O/pmc_mfma > $O/c2_mfma_counters.csv && find $O/pmc_mfma -name "*counter_collection.csv" -delete; cat $O/c2_mfma_counters.csv ;;
    pmcf3) step pmcf3 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch_c3 -o run --output-format csv -- python $R/bench.py --workload c3 --steps 12 --warmup 1 --no-cpu-baseline ;;
    pmcw3) step pmcw3 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write_c3 -o run --output-format csv -- python $R/bench.py --workload c3 --steps 12 --warmup 1 --no-cpu-baseline
           pmcsum pmc_fetch_c3 pmc_write_c3 c3_pmc_traffic.csv ;;
    pmcf4) step pmcf4 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch_c4 -o run --output-format csv -- python $R/bench.py --workload c4 --steps 4 --warmup 1 --no-cpu-baseline ;;
    pmcw4) step pmcw4 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write_c4 -o run --output-format csv -- python $R/bench.py --workload c4 --steps 4 --warmup 1 --no-cpu-baseline
           pmcsum pmc_fetch_c4 pmc_write_c4 c4_pmc_traffic.csv ;;
    trace2) step trace2 200 env KORALI_AMD_TRACE_EIGEN=1 python $R/tools/trace_c2.py ;;
    trace4) step trace4 300 env KORALI_AMD_TRACE_EIGEN=1 python $R/tools/trace_c4.py ;;
    dist) step dist 700 python -u -m pytest $R/tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --rootdir $R ;;
    engvr) step engvr 500 python -u -m pytest $R/tests/test_gpu_engine.py -x -v -k vracer --timeout 300 --timeout-method thread -p no:cacheprovider --rootdir $R ;;
    vrtests) step vrtests 400 python -u -m pytest $R/tests/test_gpu_vracer.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider --rootdir $R ;;
    c5) step c5 300 python $R/bench.py --workload c5 --steps 10 --warmup 2 ;;
    # (graph-replayed updates crash inside rocprofv3's graph interception with
    #  /opt/rocm's HIP, profiles/r6/c5_profiler_graph_segv.txt: the profiled
    #  C5 runs launch the update kernels one by one, KORALI_AMD_VR_GRAPH=0)
    profc5) step profc5 300 env KORALI_AMD_VR_GRAPH=0 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python $R/bench.py --workload c5 --steps 2 --warmup 0 --no-cpu-baseline ;;
    pmcf5) step pmcf5 300 env KORALI_AMD_VR_GRAPH=0 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch_c5 -o run --output-format csv -- python $R/bench.py --workload c5 --steps 2 --warmup 0 --no-cpu-baseline ;;
    pmcw5) step pmcw5 300 env KORALI_AMD_VR_GRAPH=0 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write_c5 -o run --output-format csv -- python $R/bench.py --workload c5 --steps 2 --warmup 0 --no-cpu-baseline
           pmcsum pmc_fetch_c5 pmc_write_c5 c5_pmc_traffic.csv ;;
    pmcm4) step pmcm4 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_mfma_c4 -o run --output-format csv -- python $R/bench.py --workload c4 --steps 5 --warmup 1 --cov mfma --no-cpu-baseline
           python $R/tools/pmc_mfma_summary.py $O/pmc_mfma_c4 > $O/c4_mfma_counters.csv && find $O/pmc_mfma_c4 -name "*counter_collection.csv" -delete; cat $O/c4_mfma_counters.csv ;;
  esac
done
echo "session done"
