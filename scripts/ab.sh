#!/bin/bash
# Quick eigensolver iteration on a GPU box: CMA-ES parity, C2 bench, phase trace.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_cmaes.py tests/test_gpu_shard.py -x -q --timeout 200 \
  --timeout-method thread 2>&1 | tail -3
timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab_a.log 2>&1
KORALI_AMD_TRACE_EIGEN=1 timeout -k 10 100 python tools/trace_c2.py 2>&1 | grep "korali_amd"
python -c "import json;d=json.loads(open('gpurun_out/ab_a.log').read().strip().splitlines()[-1]);print(round(d['value'],1),{k:round(v,3) for k,v in d['stage_ms'].items()})"
