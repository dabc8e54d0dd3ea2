#!/bin/bash
# k_adaptC_lane change: C4-sized parity, then the C4 A/B against the
# previous build (KORALI_AMD_LIB_VARIANT=cur).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_gpu_cmaes.py::test_seeded_run_matches_oracle_bit_exact" tests/test_gpu_shard.py::test_sharded_population_matches_unsharded \
  tests/test_gpu_baseline_shapes.py > gpurun_out/ab/lane_tests.log 2>&1 || { tail -30 gpurun_out/ab/lane_tests.log; exit 1; }
tail -2 gpurun_out/ab/lane_tests.log
AB_ARGS="--workload c4 --steps 20 --warmup 3" bash scripts/ab_env.sh - KORALI_AMD_LIB_VARIANT=cur - KORALI_AMD_LIB_VARIANT=cur
