#!/bin/bash
# rank-mu MFMA kernel check: MFMA-mode and shard parity tests, C2 (mfma) and C4 bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rk
timeout -k 10 500 python -u -m pytest tests/test_gpu_cmaes.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > gpurun_out/rk/tests.log 2>&1
rc=$?; tail -4 gpurun_out/rk/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --cov mfma --no-cpu-baseline > gpurun_out/rk/c2.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/rk/c2.log').read().strip().splitlines()[-1]);print(round(d['value'],1), d['rankmu_mfma_roofline'])"
timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/rk/c4.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/rk/c4.log').read().strip().splitlines()[-1]);print(round(d['value'],2), d['rankmu_mfma_roofline'], d['stage_ms_rank0'])"
