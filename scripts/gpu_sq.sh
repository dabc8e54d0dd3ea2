#!/bin/bash
# tridiagonalisation kernels check: variant parity tests, seeded parity, the C2 bench, phase traces, C4 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_cmaes.py -x -v --timeout 150 --timeout-method thread \
  -k "tridiagonalisation_kernels or seeded_run or teacher_forced or multi_workgroup" > gpurun_out/sq_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/sq_tests.log | tail -40
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/sq_bench.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/sq_bench.log').read().strip().splitlines()[-1]);print(round(d['value'],1), d.get('engine_generations_per_sec'), {k:round(v,3) for k,v in d['stage_ms'].items()})"
KORALI_AMD_TRACE_EIGEN=1 timeout -k 10 100 python tools/trace_c2.py 2>&1 | grep "sq tridiag" | tail -1
timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sq_c4.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/sq_c4.log').read().strip().splitlines()[-1]);print(round(d['value'],2), {k:round(v,3) for k,v in d.get('stage_ms',{}).items()})"
KORALI_AMD_TRACE_EIGEN=1 timeout -k 10 200 python tools/trace_c4.py 2>&1 | grep "mw2 tridiag" | tail -1
