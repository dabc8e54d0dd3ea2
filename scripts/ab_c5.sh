#!/bin/bash
# C5 update A/B: graph length and metadata-kernel width.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for cfg in - KORALI_AMD_VR_GRAPH=128 KORALI_AMD_VR_GRAPH=256 KORALI_AMD_VR_META_TPB=256 -; do
  envs=()
  [ "$cfg" != "-" ] && IFS=, read -ra envs <<< "$cfg"
  timeout -k 10 200 env "${envs[@]}" python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab/c5.log 2>&1 || { echo "FAILED $cfg"; tail -5 gpurun_out/ab/c5.log; exit 1; }
  python3 - "$cfg" <<'PY'
import json, sys
d = [json.loads(l) for l in open("gpurun_out/ab/c5.log") if l.startswith("{")][-1]
print(f"{sys.argv[1]:32s} {d['value']:9.1f} exp/s  update {d['stage_ms']['update']*1e3:.1f} us", flush=True)
PY
done
