#!/bin/bash
# Round-4 GPU call g: n = 12 QP classes -- A: factor descriptors per stage + prefetch depth 1 (dbg/spillA),
# B: A + row slacks / duals in workspace columns (four waves per CU; dbg/spillB).  Tests with B, C5 region
# traces and bench lines for base / A / B, C3 for B (its classes are untouched).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4g}
A=dbg/spillA/libscvx_hip.so; B=dbg/spillB/libscvx_hip.so
SCVX_HIP_LIB=$B timeout -k 10 500 python -u -m pytest tests/test_virtual_control_gpu.py tests/test_coupled_gpu.py tests/test_qp_gpu.py tests/test_warm_start_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/ab_pytest_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
for v in A B; do
  eval L=\$$v
  SCVX_HIP_LIB=$L timeout -k 10 200 python -u tools/trace_coupled.py c5 4 > gpurun_out/trace_c5_${v}_$TAG.log 2>&1
  SCVX_HIP_LIB=$L timeout -k 10 240 python -u bench.py --config c5 --no-cpu > gpurun_out/ab_${TAG}_c5_$v.log 2>&1
done
SCVX_HIP_LIB=$B timeout -k 10 240 python -u bench.py --config c3 --no-cpu > gpurun_out/ab_${TAG}_c3_B.log 2>&1
echo done
