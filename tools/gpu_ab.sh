#!/bin/bash
# A/B on one box: the in-tree library against SCVX_HIP_LIB=$1 -- QP/warm/timed-region GPU tests with the
# variant, then the C3 bench (no CPU leg) and the in-kernel region trace of both, alternating.
# usage: tools/gpu_ab.sh VARIANT_SO TAG
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$1; TAG=${2:-ab}
SCVX_HIP_LIB=$V timeout -k 10 500 python -u -m pytest tests/test_qp_gpu.py tests/test_warm_start_gpu.py tests/test_jacobi_update_gpu.py tests/test_timed_region_gpu.py tests/test_coupled_gpu.py tests/test_virtual_control_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/ab_pytest_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/ab_${TAG}_base_$r.log 2>&1
  SCVX_HIP_LIB=$V timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/ab_${TAG}_var_$r.log 2>&1
done
TRACE=1 REPS=2 timeout -k 10 120 python -u tools/gpurun_quick.py 1024 > gpurun_out/ab_${TAG}_trace_base.log 2>&1
SCVX_HIP_LIB=$V TRACE=1 REPS=2 timeout -k 10 120 python -u tools/gpurun_quick.py 1024 > gpurun_out/ab_${TAG}_trace_var.log 2>&1
for f in gpurun_out/ab_${TAG}_base_*.log gpurun_out/ab_${TAG}_var_*.log; do python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f', round(d['value'],1), round(d['ms_per_step_median'],4), round(d['stage_ms_median']['qp'],4), d['ipm_iters_per_agent'], d['ipm_iters_max_per_step'][:8], d['status_counts'])"; done
echo done
