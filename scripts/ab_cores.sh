#!/bin/bash
# Helper-core choice A/B on C4 (idle-first vs topology order), with the
# chosen cores printed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; head -3 /proc/stat | cut -c1-60; grep -c '^cpu[0-9]' /proc/stat
KORALI_AMD_HOST_TRIDIAG_VERBOSE=1 timeout -k 10 100 python bench.py --workload c4 --steps 5 --warmup 1 --no-cpu-baseline 2>&1 | grep "host tridiag" | head -4
AB_ARGS="--workload c4 --steps 20 --warmup 3" bash scripts/ab_env.sh - KORALI_AMD_HOST_TRIDIAG_BUSY_MS=0 KORALI_AMD_HOST_TRIDIAG_PIN_CALLER=1 - KORALI_AMD_HOST_TRIDIAG_BUSY_MS=0 KORALI_AMD_HOST_TRIDIAG_PIN_CALLER=1
