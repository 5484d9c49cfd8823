#!/bin/bash
# Round-4 GPU call p: C5 A/B of the in-tree library (dense packet + descriptor table) against dbg/unr (the n = 12
# translation unit built with -mllvm -pragma-unroll-threshold=500000: the 49-row loops fully unrolled, no
# dynamically indexed row arrays in scratch) and dbg/unrgj (unr + reciprocal pivots in the virtual-control
# Gauss-Jordan); QP / VC GPU tests with unrgj.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4p}
SCVX_HIP_LIB=dbg/unrgj/libscvx_hip.so timeout -k 10 600 python -u -m pytest tests/test_qp_gpu.py tests/test_virtual_control_gpu.py tests/test_coupled_gpu.py tests/test_warm_start_gpu.py tests/test_rtc_subproblem_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/ab_pytest_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
for r in 1 2; do
  timeout -k 10 240 python -u bench.py --config c5 --no-cpu > gpurun_out/ab_${TAG}_c5_base_$r.log 2>&1
  SCVX_HIP_LIB=dbg/unr/libscvx_hip.so timeout -k 10 240 python -u bench.py --config c5 --no-cpu > gpurun_out/ab_${TAG}_c5_unr_$r.log 2>&1
  SCVX_HIP_LIB=dbg/unrgj/libscvx_hip.so timeout -k 10 240 python -u bench.py --config c5 --no-cpu > gpurun_out/ab_${TAG}_c5_unrgj_$r.log 2>&1
done
timeout -k 10 240 python -u bench.py --config c4 --no-cpu > gpurun_out/ab_${TAG}_c4_base.log 2>&1
echo done
