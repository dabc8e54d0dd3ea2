#!/bin/bash
# One PMC pass (counters in $CTRS) over a short bench run ($WL workload),
# summarised per kernel matching $KPAT by tools/pmc_kernel.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp KORALI_AMD_PLAIN_LAUNCH=1
O=$PWD/gpurun_out/pmcp
mkdir -p $O
(cd /tmp && timeout -k 10 200 rocprofv3 --pmc $CTRS --kernel-trace -d $O/run -o run --output-format csv -- python $OLDPWD/bench.py --workload ${WL:-c4} --steps ${STEPS:-2} --warmup 0 --no-cpu-baseline) > $O/log 2>&1
rc=$?
echo "rc=$rc"
[ $rc -ne 0 ] && { grep -v "^W20" $O/log | tail -5; exit $rc; }
python tools/pmc_kernel.py $O/run "${KPAT:-k_transform}"
find $O -name "*kernel_trace.csv" -delete
