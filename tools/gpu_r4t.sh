#!/bin/bash
# Round-4 GPU call t: the QP dispatch order (scvx_qp_solve_batched_ordered; JacobiSCvx dispatch_order="lpt"):
# its GPU tests + the QP / coupled / warm-start / RTC suites on the in-tree build, then C4 / C3 / C5 bench lines
# with --dispatch-order none vs lpt (alternating, two runs each for C4).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4t}
timeout -k 10 700 python -u -m pytest tests/test_dispatch_order_gpu.py tests/test_qp_gpu.py tests/test_coupled_gpu.py tests/test_warm_start_gpu.py tests/test_rtc_subproblem_gpu.py tests/test_jacobi_update_gpu.py tests/test_timed_region_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
for r in 1 2; do
  timeout -k 10 240 python -u bench.py --config c4 --no-cpu --dispatch-order none > gpurun_out/ab_${TAG}_c4_none_$r.log 2>&1
  timeout -k 10 240 python -u bench.py --config c4 --no-cpu --dispatch-order lpt > gpurun_out/ab_${TAG}_c4_lpt_$r.log 2>&1
done
timeout -k 10 240 python -u bench.py --no-cpu --dispatch-order none > gpurun_out/ab_${TAG}_c3_none.log 2>&1
timeout -k 10 240 python -u bench.py --no-cpu --dispatch-order lpt > gpurun_out/ab_${TAG}_c3_lpt.log 2>&1
timeout -k 10 240 python -u bench.py --config c5 --no-cpu --dispatch-order none > gpurun_out/ab_${TAG}_c5_none.log 2>&1
timeout -k 10 240 python -u bench.py --config c5 --no-cpu --dispatch-order lpt > gpurun_out/ab_${TAG}_c5_lpt.log 2>&1
echo done
