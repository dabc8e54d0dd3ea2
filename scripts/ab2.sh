#!/bin/bash
# Determinism stress (3 concurrent processes) + CMA-ES / shard parity + C2 bench + eigen trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  (timeout -k 10 200 python -u tools/flake_tmcmc.py 15 > gpurun_out/fl_a$i.log 2>&1 &
   timeout -k 10 200 python -u tools/flake_tmcmc.py 15 > gpurun_out/fl_b$i.log 2>&1 &
   timeout -k 10 200 python -u tools/flake_tmcmc.py 15 > gpurun_out/fl_c$i.log 2>&1 & wait)
done
grep -h "FLAKE_CHECK" gpurun_out/fl_*.log | sort | uniq -c
timeout -k 10 600 python -u -m pytest tests/test_gpu_cmaes.py tests/test_gpu_shard.py tests/test_gpu_tmcmc.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/ab2_tests.log 2>&1; rc=$?
tail -3 gpurun_out/ab2_tests.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab_a.log 2>&1 || exit $?
KORALI_AMD_TRACE_EIGEN=1 timeout -k 10 100 python tools/trace_c2.py 2>&1 | grep "korali_amd" || true
python -c "import json;d=json.loads(open('gpurun_out/ab_a.log').read().strip().splitlines()[-1]);print(round(d['value'],1),{k:round(v,3) for k,v in d['stage_ms'].items()})"
