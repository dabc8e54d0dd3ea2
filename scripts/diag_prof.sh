#!/bin/bash
# Which part of a run makes rocprofv3's process teardown segfault: a bare
# torch run, the CMA-ES path with the device Givens chase (no cooperative
# launch), then with the host chase (cooperative streamed apply).  Stops at
# the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/diag
mkdir -p $O
run() {
  local name=$1; shift
  (cd /tmp && timeout -k 10 120 "$@") > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -v "^W20\|^E20" $O/$name.log | tail -3
  [ $rc -ne 0 ] && exit $rc
  return 0
}
export PYTHONPATH=$PWD
export KORALI_AMD_APPLY_PLAIN=1
run hostplain rocprofv3 --kernel-trace --stats -d $O/hp -o run --output-format csv -- python $PWD/tools/prof_probe.py
unset KORALI_AMD_APPLY_PLAIN
run tmcmc rocprofv3 --kernel-trace --stats -d $O/tm -o run --output-format csv -- python $PWD/tools/prof_probe_tmcmc.py
run hostchase rocprofv3 --kernel-trace --stats -d $O/h -o run --output-format csv -- python $PWD/tools/prof_probe.py
echo "all passed"
