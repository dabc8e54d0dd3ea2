set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/s1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s1/smoke.log 2>&1 &&
timeout -k 10 200 python tools/trace_c2.py > gpurun_out/s1/trace_c2.log 2>&1 &&
timeout -k 10 200 python tools/trace_c4.py > gpurun_out/s1/trace_c4.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --cov exact --no-cpu-baseline > gpurun_out/s1/benchx.log 2>&1 &&
timeout -k 10 300 python tools/probe_c4.py 512 65536 3 > gpurun_out/s1/c4.log 2>&1
