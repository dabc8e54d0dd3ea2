#!/bin/bash
# Quad-chain exact rank-mu kernel: CMA-ES parity suite, C2 A/B against the
# row chains (KORALI_AMD_ADAPTC_QUAD=0), kernel times under rocprofv3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_cmaes.py tests/test_gpu_shard.py tests/test_gpu_baseline_shapes.py > gpurun_out/ab/quad_tests.log 2>&1 || { tail -30 gpurun_out/ab/quad_tests.log; exit 1; }
tail -2 gpurun_out/ab/quad_tests.log
bash scripts/ab_env.sh - KORALI_AMD_ADAPTC_QUAD=0 - KORALI_AMD_ADAPTC_QUAD=0 || exit 1
rm -rf gpurun_out/ab/prof_new
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof_new -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c1 > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
for r in csv.DictReader(open(glob.glob("gpurun_out/ab/prof_new/**/*kernel_stats.csv", recursive=True)[0])):
    if any(k in r["Name"] for k in ("adaptC", "k_apply", "unpack")):
        print(r["Name"][:44].ljust(44), r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), round(float(r["MinNs"]) / 1e3, 2))
PY
