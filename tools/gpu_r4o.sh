#!/bin/bash
# Round-4 GPU call o: A/B of dbg/dt (dense global packet in the LDS layout, n = 12 descriptor table in the
# workspace, per-stage opaque lane in the factor) against the in-tree library: QP GPU tests with dt, C5 / C3 / C4
# bench lines of both, the C5 factor phase trace of dbg/dtp (dt + -DQP_PHASE_TRACE).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
V=dbg/dt/libscvx_hip.so; TAG=${1:-r4o}
SCVX_HIP_LIB=$V timeout -k 10 700 python -u -m pytest tests/test_qp_gpu.py tests/test_warm_start_gpu.py tests/test_jacobi_update_gpu.py tests/test_timed_region_gpu.py tests/test_coupled_gpu.py tests/test_virtual_control_gpu.py tests/test_compat_gpu.py tests/test_rtc_subproblem_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/ab_pytest_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
SCVX_HIP_LIB=$V timeout -k 10 240 python -u bench.py --config c5 --no-cpu > gpurun_out/ab_${TAG}_c5_var.log 2>&1
SCVX_HIP_LIB=dbg/dtp/libscvx_hip.so timeout -k 10 180 python -u tools/trace_coupled.py c5 > gpurun_out/ab_${TAG}_trace_c5_var.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/ab_${TAG}_c3_base_$r.log 2>&1
  SCVX_HIP_LIB=$V timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/ab_${TAG}_c3_var_$r.log 2>&1
done
SCVX_HIP_LIB=$V timeout -k 10 240 python -u bench.py --config c4 --no-cpu > gpurun_out/ab_${TAG}_c4_var.log 2>&1
SCVX_HIP_LIB=$V timeout -k 10 700 python -u -m pytest tests/test_c4_late_gpu.py tests/test_nash_gpu.py tests/test_scp_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/ab_pytest2_$TAG.log 2>&1 || { rc=$?; echo "pytest2 rc $rc"; [ $rc -eq 1 ] || exit $rc; }
echo done
