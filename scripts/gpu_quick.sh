#!/bin/bash
# quick GPU check: eigen/CMA-ES parity tests, then the C2 bench (exact) and the tridiag trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_cmaes.py tests/test_gpu_engine.py tests/test_cxx_api.py tests/test_gpu_tmcmc.py -x -q --timeout 300 --timeout-method thread > gpurun_out/q_tests.log 2>&1
rc=$?; tail -4 gpurun_out/q_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --cov ${COV:-exact} --no-cpu-baseline > gpurun_out/q_bench.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/q_bench.log').read().strip().splitlines()[-1]);print(round(d['value'],1), d.get('engine_generations_per_sec'), {k:round(v,3) for k,v in d['stage_ms'].items()})"
KORALI_AMD_TRACE_EIGEN=1 timeout -k 10 100 python tools/trace_c2.py 2>&1 | grep "one-workgroup" | tail -1
