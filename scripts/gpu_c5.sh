#!/bin/bash
# VRACER (C5): GPU parity tests, bench line, kernel stats (trace files dropped: only the summaries come back)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5
timeout -k 10 400 python -u -m pytest tests/test_gpu_vracer.py -q -x --timeout 200 --timeout-method thread > gpurun_out/c5/tests.log 2>&1 || { tail -30 gpurun_out/c5/tests.log; exit 1; }
tail -2 gpurun_out/c5/tests.log
timeout -k 10 300 python -u bench.py --workload c5 --steps ${C5_STEPS:-10} --warmup 2 ${C5_ARGS:-} > gpurun_out/c5/bench.log 2>&1 || { tail -20 gpurun_out/c5/bench.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/c5/bench.log').read().strip().splitlines()[-1]);print(round(d['value'],1), d['policy_updates_per_sec'], {k:round(v,4) for k,v in d['stage_ms'].items()})"
if [ -n "${C5_PROF:-1}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/c5prof -o run --output-format csv -- python bench.py --workload c5 --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/c5/prof.log 2>&1 || exit 1
  find /tmp/c5prof -name "*kernel_stats*" -exec cp {} gpurun_out/c5/ \;
  python -c "
import csv
r=list(csv.DictReader(open('gpurun_out/c5/run_kernel_stats.csv')))
for x in r[:12]: print(x['Name'][:50].ljust(50), x['Calls'], round(float(x['AverageNs'])/1e3,2), round(float(x['Percentage']),1))"
fi
