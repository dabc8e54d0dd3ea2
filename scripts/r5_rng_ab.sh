#!/bin/bash
# RNG changes: correctness (CMA-ES + sharding tests), then C2 A/B over the
# chunk size of the parallel mt19937 producer, then kernel stats.
set -o pipefail
OUT=${1:-gpurun_out/r5j}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { echo "=== $1" >> "$OUT/steps.log"; shift; "$@"; rc=$?; echo "rc=$rc" >> "$OUT/steps.log"; return $rc; }
run tests timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cmaes.py tests/test_gpu_shard.py > "$OUT/tests.log" 2>&1 || exit 1
for lw in 15 17 19; do
  run "bench lw=$lw" env KORALI_AMD_MT_CHUNK_LOG2=$lw timeout -k 10 200 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline > "$OUT/bench_lw$lw.json" 2> "$OUT/bench_lw$lw.err" || exit 1
done
run prof2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof2" -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/prof2.log" 2>&1 || exit 1
run c4probe timeout -k 10 120 python -u tools/probe_c4.py 512 65536 3 exact > "$OUT/probe_c4.log" 2>&1
run efixed timeout -k 10 200 python -u tools/probe_engine_fixed.py > "$OUT/engine_fixed.json" 2> "$OUT/engine_fixed.err"
