#!/bin/bash
# Round-4 GPU call c: region trace of the QP kernel (one agent, cycles per IPM iteration) at N = 1024 and the
# user-model QP test.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4c}
TRACE=1 REPS=2 timeout -k 10 120 python -u tools/gpurun_quick.py 1024 > gpurun_out/trace_$TAG.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_rtc_subproblem_gpu.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
echo done
