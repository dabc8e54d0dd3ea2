#!/bin/bash
# mt19937 producer at C2: single-workgroup ring producer vs the chunked
# multi-workgroup producer (GF(2) jump-ahead) at several chunk sizes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/mt
for v in default 15 16 17; do
  if [ $v = default ]; then envs=""; else envs="KORALI_AMD_MT_PARALLEL_MIN=0 KORALI_AMD_MT_CHUNK_LOG2=$v"; fi
  env $envs timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/mt/b_$v.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/mt/b_$v.log').read().strip().splitlines()[-1]);print('$v', round(d['value'],1), round(d['stage_ms']['eigen'],3))"
done
