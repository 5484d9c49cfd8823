#!/bin/bash
# Round-4 GPU call q: A/B of dbg/gm (SCP / game kernel: the regularisation a breakdown forced stays in the end game)
# against the in-tree library: nash (incl. the batched game kernel's status counts) and scp bench lines of both,
# the SCP / Nash GPU tests with gm.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
V=dbg/gm/libscvx_hip.so; TAG=${1:-r4q}
SCVX_HIP_LIB=$V timeout -k 10 700 python -u -m pytest tests/test_nash_gpu.py tests/test_scp_gpu.py tests/test_compat_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/ab_pytest_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
for c in nash scp; do
  timeout -k 10 240 python -u bench.py --config $c --no-cpu > gpurun_out/ab_${TAG}_${c}_base.log 2>&1
  SCVX_HIP_LIB=$V timeout -k 10 240 python -u bench.py --config $c --no-cpu > gpurun_out/ab_${TAG}_${c}_var.log 2>&1
done
echo done
