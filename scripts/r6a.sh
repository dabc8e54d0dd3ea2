#!/bin/bash
# round 6, session A: host tridiagonalisation on the box's core (timing per
# ISA), C2 bench host vs device tridiagonalisation, then the GPU suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6a; mkdir -p $O
timeout -k 5 120 python tools/time_host_tridiag.py > $O/ht.log 2>&1; cat $O/ht.log
timeout -k 10 240 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-c1 > $O/b_host.log 2>&1 || { tail -20 $O/b_host.log; exit 1; }
python -c "import json;d=json.loads(open('$O/b_host.log').read().strip().splitlines()[-1]);print('host', round(d['value'],1), d.get('engine_generations_per_sec'), {k:round(v,3) for k,v in d['stage_ms'].items()})"
KORALI_AMD_TRIDIAG=sq timeout -k 10 240 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-c1 > $O/b_dev.log 2>&1 || { tail -20 $O/b_dev.log; exit 1; }
python -c "import json;d=json.loads(open('$O/b_dev.log').read().strip().splitlines()[-1]);print('device', round(d['value'],1), d.get('engine_generations_per_sec'), {k:round(v,3) for k,v in d['stage_ms'].items()})"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; exit $rc
