#!/bin/bash
# Round-4 GPU call k (in-tree build: factor micro-optimisations, per-template SCP waves, ABI 4): QP / SCP / Nash
# tests, C3 bench x2 (no CPU leg) against r4i's 751 it/s, the cold region trace.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4k}
timeout -k 10 800 python -u -m pytest tests/test_qp_gpu.py tests/test_warm_start_gpu.py tests/test_jacobi_update_gpu.py tests/test_timed_region_gpu.py tests/test_coupled_gpu.py tests/test_virtual_control_gpu.py tests/test_c4_late_gpu.py tests/test_compat_gpu.py tests/test_scp_gpu.py tests/test_nash_gpu.py tests/test_compat_scp_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
for r in 1 2; do timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/bench_c3_${TAG}_$r.log 2>&1; done
TRACE=1 REPS=2 timeout -k 10 120 python -u tools/gpurun_quick.py 1024 > gpurun_out/trace_$TAG.log 2>&1
echo done
