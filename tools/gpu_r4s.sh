#!/bin/bash
# Round-4 GPU call s: C5 A/B of the in-tree library against dbg/cpg (n = 12 classes read the predictor products
# ds_a dl_a from their workspace columns at each use instead of holding 49 + 24 doubles from the corrector's
# Newton rhs to its update); QP / VC GPU tests with cpg.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
V=dbg/cpg/libscvx_hip.so; TAG=${1:-r4s}
SCVX_HIP_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_qp_gpu.py tests/test_virtual_control_gpu.py tests/test_coupled_gpu.py tests/test_warm_start_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/ab_pytest_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
for r in 1 2; do
  timeout -k 10 240 python -u bench.py --config c5 --no-cpu > gpurun_out/ab_${TAG}_c5_base_$r.log 2>&1
  SCVX_HIP_LIB=$V timeout -k 10 240 python -u bench.py --config c5 --no-cpu > gpurun_out/ab_${TAG}_c5_var_$r.log 2>&1
done
echo done
