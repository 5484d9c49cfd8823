#!/bin/bash
# Round-4 GPU call b: the user-model subproblem tests + the dist_scvx_3d sweep, C4/C5 bench lines, then the PMC
# passes and kernel-trace stats of the C3 bench (tools/gpu_pmc.sh).  A crash / timeout ends the script.
# usage: tools/gpu_r4b.sh TAG
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4b}
timeout -k 10 400 python -u -m pytest tests/test_rtc_subproblem_gpu.py tests/test_compat_gpu.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 240 python -u bench.py --config c4 --no-cpu > gpurun_out/bench_c4_$TAG.log 2>&1
timeout -k 10 240 python -u bench.py --config c5 --no-cpu > gpurun_out/bench_c5_$TAG.log 2>&1
bash tools/gpu_pmc.sh $TAG
echo done
