#!/bin/bash
# C5 PMC passes over every update kernel (FETCH_SIZE, then WRITE_SIZE, each
# its own rocprofv3 run), summarised on the box; the raw directories are
# removed so that gpurun_out stays small.  Usage: scripts/pmc_c5_update.sh <out dir>
set -o pipefail
OUT=${1:-gpurun_out/r5f}
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  KORALI_AMD_SEGV_MAPS=1 timeout -s KILL 600 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc5_$c" -o run --output-format csv -- \
    python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc5_$c.log" 2>&1
  rc=$?
  echo "pmc $c rc=$rc" >> "$OUT/steps.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 tools/pmc_c5_update.py "$OUT/pmc5_FETCH_SIZE" "$OUT/pmc5_WRITE_SIZE" > "$OUT/c5_pmc_update_traffic.csv" &&
  rm -rf "$OUT/pmc5_FETCH_SIZE" "$OUT/pmc5_WRITE_SIZE"
