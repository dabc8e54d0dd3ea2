#!/bin/bash
# C2 engine-path A/B (korali.Engine rates beside the C-ABI loop).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for cfg in "$@"; do
  envs=()
  [ "$cfg" != "-" ] && IFS=, read -ra envs <<< "$cfg"
  timeout -k 10 250 env "${envs[@]}" python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-c1 > gpurun_out/ab/eng.log 2>&1 || { echo "FAILED $cfg"; tail -5 gpurun_out/ab/eng.log; exit 1; }
  python3 - "$cfg" <<'PY'
import json, sys
d = [json.loads(l) for l in open("gpurun_out/ab/eng.log") if l.startswith("{")][-1]
e = {k[7:]: round(v, 1) for k, v in d.items() if k.startswith("engine")}
print(f"{sys.argv[1]:36s} capi {d['value']:7.1f}  {e}", flush=True)
PY
done
