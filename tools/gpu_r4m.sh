#!/bin/bash
# Round-4 GPU call m: A/B of dbg/f4 (phase 3: cofactor inverse of Rh for NU = 3, Rh^-1 applied in the solve
# passes) against the in-tree library: QP tests with f4, C3 bench x2 each, cold traces; C4 / C5 lines with f4.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
V=dbg/f4/libscvx_hip.so; TAG=${1:-r4m}
SCVX_HIP_LIB=$V timeout -k 10 700 python -u -m pytest tests/test_qp_gpu.py tests/test_warm_start_gpu.py tests/test_jacobi_update_gpu.py tests/test_timed_region_gpu.py tests/test_coupled_gpu.py tests/test_virtual_control_gpu.py tests/test_c4_late_gpu.py tests/test_compat_gpu.py tests/test_rtc_subproblem_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/ab_pytest_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/ab_${TAG}_base_$r.log 2>&1
  SCVX_HIP_LIB=$V timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/ab_${TAG}_var_$r.log 2>&1
done
SCVX_HIP_LIB=$V TRACE=1 REPS=2 timeout -k 10 120 python -u tools/gpurun_quick.py 1024 > gpurun_out/ab_${TAG}_trace_var.log 2>&1
SCVX_HIP_LIB=$V timeout -k 10 240 python -u bench.py --config c4 --no-cpu --warm-status 1 > gpurun_out/ab_${TAG}_c4_var.log 2>&1
SCVX_HIP_LIB=$V timeout -k 10 240 python -u bench.py --config c5 --no-cpu > gpurun_out/ab_${TAG}_c5_var.log 2>&1
echo done
