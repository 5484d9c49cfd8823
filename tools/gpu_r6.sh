#!/bin/bash
# Round-6 GPU call: the GPU tests, smoke, the headline bench (both trust-region rules, CPU baseline), c2 and c4
# lines, then the PMC traffic passes and the kernel-trace stats of the headline rule (tools/gpu_pmc.sh).  Every GPU
# step under its own time limit; a crash or timeout (anything but pytest's "tests failed" rc 1) ends the script.
# usage: tools/gpu_r6.sh TAG [PMC=0]
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r6}
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
tail -n 2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c3_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --config c2 > gpurun_out/bench_c2_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --config c4 --no-cpu > gpurun_out/bench_c4_$TAG.log 2>&1
if [ "${PMC:-1}" = 1 ]; then bash tools/gpu_pmc.sh $TAG; fi
echo done
