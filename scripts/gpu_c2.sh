#!/bin/bash
# C2 check: CMA-ES parity tests (all), the C2 bench and the C4 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_cmaes.py tests/test_gpu_engine.py tests/test_gpu_baseline_shapes.py tests/test_gpu_shard.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c2_tests.log 2>&1
rc=$?; tail -5 gpurun_out/c2_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/c2_bench.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/c2_bench.log').read().strip().splitlines()[-1]);print(round(d['value'],1), d.get('engine_generations_per_sec'), {k:round(v,3) for k,v in d['stage_ms'].items()})"
timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c4_bench.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/c4_bench.log').read().strip().splitlines()[-1]);print(round(d['value'],2), {k:round(v,3) for k,v in d.get('stage_ms_rank0',{}).items()})"
