#!/bin/bash
# Round-4 GPU call e: A/B of dbg/spill (streamed soft rows / disc columns in the large QP classes) against the
# in-tree library: VC + coupled tests with the variant, C5 / C4 / C3 bench lines both, C5 region traces both.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
V=dbg/spill/libscvx_hip.so; TAG=${1:-r4e}
SCVX_HIP_LIB=$V timeout -k 10 500 python -u -m pytest tests/test_virtual_control_gpu.py tests/test_coupled_gpu.py tests/test_c4_late_gpu.py tests/test_qp_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/ab_pytest_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 200 python -u tools/trace_coupled.py c5 4 > gpurun_out/trace_c5_base_$TAG.log 2>&1
SCVX_HIP_LIB=$V timeout -k 10 200 python -u tools/trace_coupled.py c5 4 > gpurun_out/trace_c5_var_$TAG.log 2>&1
for c in c5 c3; do
  timeout -k 10 240 python -u bench.py --config $c --no-cpu > gpurun_out/ab_${TAG}_${c}_base.log 2>&1
  SCVX_HIP_LIB=$V timeout -k 10 240 python -u bench.py --config $c --no-cpu > gpurun_out/ab_${TAG}_${c}_var.log 2>&1
done
echo done
