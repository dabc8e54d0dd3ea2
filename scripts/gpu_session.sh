#!/bin/bash
# One gpurun session: each GPU step under its own time limit; stop at the
# first crash/timeout (exit >= 124), keep going on ordinary test failures.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${SESSION:-s}
mkdir -p "$OUT"
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "FATAL step $name rc=$rc"; exit $rc; fi
  return 0
}
for s in ${STEPS:-smoke tests bench prof}; do
  case $s in
    rs) step rs 600 env KORALI_AMD_DEBUG_OCC=1 python -u -m pytest tests/test_gpu_cmaes.py -x -v --timeout 300 --timeout-method thread -k "resampl or overflow or interleaved or mirrored or discrete" ;;
    diag) K="test_mirrored_sampling_matches_oracle_bit_exact"; step diag_sq0 300 env KORALI_AMD_SQ_DPP=0 python -u -m pytest tests/test_gpu_cmaes.py -x -q --timeout 250 --timeout-method thread -k "$K" ; step diag_row0 300 env KORALI_AMD_ROWCHAINS=0 python -u -m pytest tests/test_gpu_cmaes.py -x -q --timeout 250 --timeout-method thread -k "$K" ; step diag_both0 300 env KORALI_AMD_ROWCHAINS=0 KORALI_AMD_SQ_DPP=0 python -u -m pytest tests/test_gpu_cmaes.py -x -q --timeout 250 --timeout-method thread -k "$K" ;;
    trsc) step trsc_t 600 python -u -m pytest tests/test_gpu_cmaes.py -x -v --timeout 300 --timeout-method thread -k scalar_operand && step trsc_b0 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline && step trsc_b8 300 env KORALI_AMD_TRANSFORM_SC=8 python bench.py --steps 200 --warmup 10 --no-cpu-baseline && step trsc_c4 300 env KORALI_AMD_TRANSFORM_SC=8 python -u -m pytest tests/test_gpu_baseline_shapes.py -x -v -s --timeout 250 --timeout-method thread -k c4_shape_two && step trsc_c4b 300 env KORALI_AMD_TRANSFORM_SC=8 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline ;;
    dist) step dist 900 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 600 --timeout-method thread ;;
    dppc) step dppc 120 ./tools/check_dpp_chains && step tri 900 python -u -m pytest tests/test_gpu_cmaes.py -v --timeout 300 --timeout-method thread -k tridiagonalisation_kernels ;;
    occsys) step occ_sys 300 env KORALI_AMD_HIP_RUNTIME=system KORALI_AMD_DEBUG_OCC=1 python -u -m pytest tests -m gpu -x -v -s --timeout 250 --timeout-method thread -k c4_shape_two && step occ_one 300 env KORALI_AMD_DEBUG_OCC=1 python -u -m pytest tests -m gpu -x -v -s --timeout 250 --timeout-method thread -k c4_shape_two ;;
    c4ab) step c4_sc0 300 env KORALI_AMD_TRANSFORM_SC=0 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline && step c4_sc8 300 env KORALI_AMD_TRANSFORM_SC=8 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline ;;
    prof2) step prof2 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof2" -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline ;;
    prof4) step prof4 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof4" -o run --output-format csv -- python bench.py --workload c4 --steps 6 --warmup 2 --no-cpu-baseline ;;
    pmc2) step pmc2f 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc2_fetch" -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline && step pmc2w 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc2_write" -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline ;;
    pmc4) step pmc4f 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc4_fetch" -o run --output-format csv -- python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline && step pmc4w 300 env KORALI_AMD_PLAIN_LAUNCH=1 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc4_write" -o run --output-format csv -- python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline ;;
    mfma) step mfma2 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/mfma2" -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline --cov mfma && step mfma4 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/mfma4" -o run --output-format csv -- python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline ;;
    trace2dpp) step trace2_dpp0 200 env KORALI_AMD_SQ_DPP=0 KORALI_AMD_TRACE_EIGEN=1 python tools/trace_c2.py ;;
    c4p) step prof4p 400 env KORALI_AMD_PLAIN_LAUNCH=1 rocprofv3 --kernel-trace --stats -d "$OUT/prof4" -o run --output-format csv -- python bench.py --workload c4 --steps 6 --warmup 2 --no-cpu-baseline && step pmc4fp 300 env KORALI_AMD_PLAIN_LAUNCH=1 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc4_fetch" -o run --output-format csv -- python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline && step pmc4wp 300 env KORALI_AMD_PLAIN_LAUNCH=1 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc4_write" -o run --output-format csv -- python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline && step mfma4p 300 env KORALI_AMD_PLAIN_LAUNCH=1 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/mfma4" -o run --output-format csv -- python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline ;;
    c4eng) step c4eng 600 env KORALI_AMD_C4_ENGINE=1 python bench.py --workload c4 --steps 8 --warmup 2 --no-cpu-baseline ;;
    nmab) step nm_sym0 300 env KORALI_AMD_NM_SYM=0 python tools/nm_probe.py 8192 && step nm_sym1 300 env KORALI_AMD_NM_SYM=1 python tools/nm_probe.py 8192 ;;
    pmc5g) step pmc5gf 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex "k_vr_gemm" -d "$OUT/pmc5_fetch" -o run --output-format csv -- python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline && step pmc5gw 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --kernel-include-regex "k_vr_gemm" -d "$OUT/pmc5_write" -o run --output-format csv -- python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline ;;
    ub) step ub 120 ./tools/ubench_chains ;;
    c3t) step c3t 600 python -u -m pytest tests/test_gpu_baseline_shapes.py -x -v --timeout 150 --timeout-method thread -k "tmcmc" ;;
    vr) step vr 600 python -u -m pytest tests/test_gpu_vracer.py tests/test_gpu_engine.py -x -q --timeout 150 --timeout-method thread -k "vracer or VRACER" ;;
    pmc3) step pmc3f 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc3_fetch" -o run --output-format csv -- python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline && step pmc3w 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc3_write" -o run --output-format csv -- python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline && python tools/pmc_summary.py "$OUT/pmc3_fetch" "$OUT/pmc3_write" > "$OUT/c3_pmc_traffic.csv" && rm -rf "$OUT/pmc3_fetch" "$OUT/pmc3_write" ;;
    prof3) step prof3 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof3" -o run --output-format csv -- python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline ;;
    prof5) step prof5 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof5" -o run --output-format csv -- python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline && rm -f "$OUT"/prof5/run_kernel_trace.csv ;;
    pmc5s) step pmc5gf 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex "k_vr_gemm" -d "$OUT/pmc5_fetch" -o run --output-format csv -- python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline && step pmc5gw 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --kernel-include-regex "k_vr_gemm" -d "$OUT/pmc5_write" -o run --output-format csv -- python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline && python tools/pmc_c5.py "$OUT/pmc5_fetch" "$OUT/pmc5_write" > "$OUT/c5_pmc_traffic.csv" && python tools/pmc_summary.py "$OUT/pmc5_fetch" "$OUT/pmc5_write" > "$OUT/c5_pmc_all_dispatches.csv" && du -sh "$OUT"/pmc5_* && rm -rf "$OUT/pmc5_fetch" "$OUT/pmc5_write" ;;
    rowab) step bench_row0 300 env KORALI_AMD_ROWCHAINS=0 python bench.py --steps 300 --warmup 10 --no-cpu-baseline && step bench_row1 300 python bench.py --steps 300 --warmup 10 --no-cpu-baseline ;;
    sqab) step bench_sq0 300 python bench.py --steps 300 --warmup 10 --no-cpu-baseline && step bench_sq1 300 env KORALI_AMD_SQ_DPP=1 python bench.py --steps 300 --warmup 10 --no-cpu-baseline ;;
    ccm) step ccm 600 python -u -m pytest tests/test_gpu_ccmaes.py -x -v --timeout 300 --timeout-method thread ;;
    mtt) step mtt 900 python -u -m pytest tests/test_gpu_cmaes.py -x -v --timeout 300 --timeout-method thread -k "chunked or seeded_run" ;;
    mtab) for q in 1 4 8 16; do step mt_c2_p$q 300 env KORALI_AMD_MT_CHUNK_PARTS=$q python bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-c1 || exit 1; done && for q in 1 8; do step mt_c4_p$q 300 env KORALI_AMD_MT_CHUNK_PARTS=$q python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline || exit 1; done ;;
    vrt) step vrt 600 python -u -m pytest tests/test_gpu_vracer.py -x -v --timeout 300 --timeout-method thread ;;
    c5g) for g in 0 16 64; do step c5_g$g 300 env KORALI_AMD_VR_GRAPH=$g python bench.py --workload c5 --steps 60 --warmup 5 --no-cpu-baseline || exit 1; done ;;
    c5di) for v in 0 1; do step c5_di$v 300 env KORALI_AMD_VR_DRAW_IN=$v python bench.py --workload c5 --steps 60 --warmup 5 --no-cpu-baseline || exit 1; done ;;
    metat) for v in 512; do step vrt_m$v 600 env KORALI_AMD_VR_META_TPB=$v python -u -m pytest tests/test_gpu_vracer.py -x -q --timeout 300 --timeout-method thread || exit 1; done ;;
    metab) for v in 256 512; do step c5_m$v 300 env KORALI_AMD_VR_META_TPB=$v python bench.py --workload c5 --steps 60 --warmup 5 --no-cpu-baseline || exit 1; done ;;
    c5da) for v in 1 0; do step c5_da$v 300 env KORALI_AMD_VR_DRAW_AHEAD=$v python bench.py --workload c5 --steps 60 --warmup 5 --no-cpu-baseline || exit 1; done ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    occ2) step occ_pair 300 env KORALI_AMD_DEBUG_OCC=1 python -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_cxx_api.py::test_reference_idioms_run_cmaes_direct tests/test_gpu_baseline_shapes.py::test_c4_shape_two_generations_bit_exact ; step occ_coll 300 env KORALI_AMD_DEBUG_OCC=1 python -u -m pytest tests -m gpu -x -v -s --timeout 250 --timeout-method thread -k c4_shape_two ;;
    testsdbg) step testsdbg 1100 env KORALI_AMD_DEBUG_OCC=1 python -u -m pytest tests -x -v -s -m gpu --timeout 300 --timeout-method thread ;;
    tests) step tests 1100 python -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread ;;
    trace2) step trace2 200 env KORALI_AMD_TRACE_EIGEN=1 python tools/trace_c2.py ;;
    trace4) step trace4 300 env KORALI_AMD_TRACE_EIGEN=1 python tools/trace_c4.py ;;
    eng) step eng 900 python -m pytest tests/test_gpu_engine.py -q --maxfail=20 ;;
    tm) step tm 900 python -u -m pytest tests/test_gpu_tmcmc.py -x -v --timeout 150 --timeout-method thread ;;
    c3) step c3 600 python bench.py --workload c3 --steps ${C3_STEPS:-40} --warmup 3 ;;
    bench) step bench 600 python bench.py --steps ${BENCH_STEPS:-200} --warmup 10 ;;
    benchx) step benchx 600 python bench.py --steps ${BENCH_STEPS:-200} --warmup 10 --cov exact --no-cpu-baseline ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof" -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c1 ;;
    profc3) step profc3 600 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof_c3" -o run --output-format csv -- python bench.py --workload c3 --steps 20 --warmup 2 --no-cpu-baseline ;;
    profc4) step profc4 600 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof_c4" -o run --output-format csv -- python bench.py --workload c4 --steps 10 --warmup 2 ;;
    pmcf) step pmcf 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline ;;
    c4) step c4 600 python tools/probe_c4.py ${C4_ARGS:-512 65536 3} ;;
    shard) step shard 900 python -m pytest tests/test_gpu_shard.py -q -x ;;
    cm) step cm 900 python -u -m pytest tests/test_gpu_cmaes.py tests/test_gpu_baseline_shapes.py -x -v --timeout 150 --timeout-method thread ;;
    benchc4) step benchc4 600 python bench.py --workload c4 --steps ${C4_STEPS:-20} --warmup 3 ;;
    pmc5) step pmc5f 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc5_fetch" -o run --output-format csv -- python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline && step pmc5w 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc5_write" -o run --output-format csv -- python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline ;;
    bench5) step bench5 600 python bench.py --workload c5 ;;
    bench3) step bench3 600 python bench.py --workload c3 ;;
    bench4) step bench4 600 python bench.py --workload c4 ;;
    mtb) step mtb 300 python -u -m pytest tests/test_gpu_mtmcmc.py -x -v --timeout 120 --timeout-method thread ;;
    dprobe) step dprobe 120 python tools/discrete_probe.py ;;
    tmt) step tmt 600 python -u -m pytest tests/test_gpu_mtmcmc.py tests/test_gpu_tmcmc.py tests/test_gpu_baseline_shapes.py -x -v --timeout 300 --timeout-method thread ;;
    occc) step occ_coll 300 env KORALI_AMD_DEBUG_OCC=1 python -u -m pytest tests -m gpu -x -v -s --timeout 250 --timeout-method thread -k c4_shape_two ;;
    occt) step occ_torch 120 python tools/occ_probe.py exact torch ;;
    occ) step occ_exact 120 python tools/occ_probe.py exact && step occ_mfma 120 python tools/occ_probe.py mfma ;;
    benchab) step bench_old 300 env KORALI_AMD_ADAPTC2=1 python bench.py --steps 200 --warmup 10 --no-cpu-baseline && step bench_new 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline ;;
    profq) step profq 300 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof" -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline ;;
    c4t) step c4t 300 env KORALI_AMD_DEBUG_OCC=1 python -u -m pytest tests/test_gpu_baseline_shapes.py -x -v -s --timeout 250 --timeout-method thread -k c4_shape_two ;;
    benchq) step benchq 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline ;;
    benchteam) step bench_t16 300 env KORALI_AMD_APPLY_TEAM=16 python bench.py --steps 200 --warmup 10 --no-cpu-baseline && step bench_t64 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline ;;
    pmcw) step pmcw 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline ;;
    pmc2s) step pmcf 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-c1 && step pmcw 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-c1 && python tools/pmc_summary.py "$OUT/pmc_fetch" "$OUT/pmc_write" > "$OUT/c2_pmc_traffic.csv" && rm -rf "$OUT/pmc_fetch" "$OUT/pmc_write" ;;
    pmc4s) step pmc4f 300 env KORALI_AMD_PLAIN_LAUNCH=1 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc4_fetch" -o run --output-format csv -- python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline && step pmc4w 300 env KORALI_AMD_PLAIN_LAUNCH=1 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc4_write" -o run --output-format csv -- python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline && python tools/pmc_summary.py "$OUT/pmc4_fetch" "$OUT/pmc4_write" > "$OUT/c4_pmc_traffic.csv" && rm -rf "$OUT/pmc4_fetch" "$OUT/pmc4_write" ;;
    givab) for i in 1 2; do step giv_bf$i 300 python bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-c1 && step giv_br$i 300 env KORALI_AMD_LIB_VARIANT=branchy python bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-c1; done ;;
    laneab) step lane_c2 300 python bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-c1 && step row_c2 300 env KORALI_AMD_ADAPTC_LANE_MIN=100000 python bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-c1 && step lane_c4 300 python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline && step row_c4 300 env KORALI_AMD_ADAPTC_LANE_MIN=100000 python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline ;;
    lwab) for lw in 15 16 17; do step lw$lw 300 env KORALI_AMD_MT_CHUNK_LOG2=$lw python bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-c1 && step plw$lw 300 env KORALI_AMD_MT_CHUNK_LOG2=$lw rocprofv3 --kernel-trace --stats -d "$OUT/plw$lw" -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c1 && rm -f "$OUT/plw$lw/run_kernel_trace.csv"; done ;;
    c5ab) step c5s0 300 env KORALI_AMD_VR_STAGED=0 python bench.py --workload c5 --no-cpu-baseline --steps 60 && step c5s1 300 env KORALI_AMD_VR_STAGED=1 python bench.py --workload c5 --no-cpu-baseline --steps 60 ;;
  esac
done
echo "session done"
