#!/bin/bash
# Round-4 GPU call w: A/B of dbg/p2l (n <= 8: every lane forms Rh's lower triangle in phase 2 and factors it
# there, overlapping the serial LDL' with the phase's element-parallel work; bit-identical arithmetic) against
# the in-tree library: QP GPU tests with p2l, C3 bench x2 each alternating, C4 line of both.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
V=dbg/p2l/libscvx_hip.so; TAG=${1:-r4w}
SCVX_HIP_LIB=$V timeout -k 10 700 python -u -m pytest tests/test_qp_gpu.py tests/test_warm_start_gpu.py tests/test_timed_region_gpu.py tests/test_coupled_gpu.py tests/test_virtual_control_gpu.py tests/test_dispatch_order_gpu.py tests/test_rtc_subproblem_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/ab_pytest_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/ab_${TAG}_c3_base_$r.log 2>&1
  SCVX_HIP_LIB=$V timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/ab_${TAG}_c3_var_$r.log 2>&1
done
timeout -k 10 240 python -u bench.py --config c4 --no-cpu > gpurun_out/ab_${TAG}_c4_base.log 2>&1
SCVX_HIP_LIB=$V timeout -k 10 240 python -u bench.py --config c4 --no-cpu > gpurun_out/ab_${TAG}_c4_var.log 2>&1
echo done
