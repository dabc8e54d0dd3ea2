#!/bin/bash
# device annealing search check: TMCMC parity tests (incl. C3 full run), search probe, C3 bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/nm
timeout -k 10 600 python -u -m pytest tests/test_gpu_tmcmc.py tests/test_gpu_baseline_shapes.py -k "tmcmc or c3" -x -q --timeout 300 --timeout-method thread > gpurun_out/nm/tests.log 2>&1
rc=$?; tail -4 gpurun_out/nm/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/nm_probe.py 1024 8192 > gpurun_out/nm/probe.log 2>&1 || exit $?
grep "TOTAL\|per round" gpurun_out/nm/probe.log
timeout -k 10 300 python bench.py --workload c3 --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/nm/c3.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/nm/c3.log').read().strip().splitlines()[-1]);print(round(d['value'],1), d['annealing_search'], {k:round(v,3) for k,v in d['stage_ms'].items()})"
