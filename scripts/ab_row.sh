#!/bin/bash
# Row-chain kernel check: CMA-ES parity suite, the C2 bench line, then the
# kernel times under rocprofv3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_cmaes.py tests/test_gpu_shard.py tests/test_gpu_baseline_shapes.py > gpurun_out/ab/row_tests.log 2>&1 || { tail -30 gpurun_out/ab/row_tests.log; exit 1; }
tail -2 gpurun_out/ab/row_tests.log
bash scripts/ab_env.sh - - ${AB_EXTRA} || exit 1
rm -rf gpurun_out/ab/prof_new
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof_new -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c1 > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
for r in csv.DictReader(open(glob.glob("gpurun_out/ab/prof_new/**/*kernel_stats.csv", recursive=True)[0])):
    if any(k in r["Name"] for k in ("adaptC", "k_apply", "unpack", "transform", "mean3", "paths")):
        print(r["Name"][:44].ljust(44), r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), round(float(r["MinNs"]) / 1e3, 2))
PY
# the engine's exchange timing on two ranks sharing the one GPU (Host transport)
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 2 --workload c4 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/ab/c4_2rank.log 2>&1 || { tail -20 gpurun_out/ab/c4_2rank.log; exit 1; }
grep '^{' gpurun_out/ab/c4_2rank.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['config']['workload'][-40:], d.get('exchange_ms_per_generation'))"
