#!/bin/bash
# A/B of environment switches on the C2 bench line: each argument is one
# setting ("-" = defaults, or VAR=VALUE[,VAR=VALUE]); prints generations/s and
# the per-stage device times of each.  Every run under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for cfg in "$@"; do
  envs=()
  [ "$cfg" != "-" ] && IFS=, read -ra envs <<< "$cfg"
  thr0=$(grep -E "nr_throttled|throttled_usec" /sys/fs/cgroup/cpu.stat 2>/dev/null | tr '\n' ' ')
  timeout -k 10 200 env "${envs[@]}" python bench.py ${AB_ARGS:---steps 200 --warmup 10 --no-c1} --no-cpu-baseline \
    > gpurun_out/ab/run.log 2>&1 || { echo "FAILED $cfg"; tail -5 gpurun_out/ab/run.log; exit 1; }
  python3 - "$cfg" <<'PY'
import json, sys
d = [json.loads(l) for l in open("gpurun_out/ab/run.log") if l.startswith("{")][-1]
st = {k: round(v * 1e3, 1) for k, v in (d.get("stage_ms") or d.get("stage_ms_rank0") or {}).items()}
print(f"{sys.argv[1]:40s} {d['value']:8.1f} gen/s  {st}", flush=True)
PY
  echo "   cgroup before: $thr0 after: $(grep -E "nr_throttled|throttled_usec" /sys/fs/cgroup/cpu.stat 2>/dev/null | tr '\n' ' ')"
done
