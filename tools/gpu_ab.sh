#!/bin/bash
# One GPU call for an A/B of a library variant (tools/build_variant.sh -> variants/NAME/libscvx_hip.so) against the
# in-tree library: the QP GPU tests with the variant, then each bench config of both libraries alternating REPS
# times, and (TRACE=1) the in-kernel region trace of both.  Every GPU step has its own time limit; a crash or a
# timeout (anything but pytest's "tests failed" rc 1) ends the script.
# usage: [CONFIGS="c3 c4 c5"] [REPS=2] [TRACE=1] [TESTS="tests/test_qp_gpu.py ..."] tools/gpu_ab.sh VARIANT_SO TAG
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$1; TAG=${2:-ab}
CONFIGS=${CONFIGS:-c3}; REPS=${REPS:-2}
TESTS=${TESTS:-"tests/test_qp_gpu.py tests/test_warm_start_gpu.py tests/test_jacobi_update_gpu.py tests/test_timed_region_gpu.py tests/test_coupled_gpu.py tests/test_virtual_control_gpu.py tests/test_highs_qp_gpu.py"}
if [ "$TESTS" != none ]; then
  SCVX_HIP_LIB=$V timeout -k 10 600 python -u -m pytest $TESTS -v -s --timeout 300 --timeout-method thread > gpurun_out/ab_pytest_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
fi
for c in $CONFIGS; do
  for r in $(seq 1 $REPS); do
    timeout -k 10 240 python -u bench.py --config $c --no-cpu > gpurun_out/ab_${TAG}_${c}_base_$r.log 2>&1
    SCVX_HIP_LIB=$V timeout -k 10 240 python -u bench.py --config $c --no-cpu > gpurun_out/ab_${TAG}_${c}_var_$r.log 2>&1
  done
done
if [ "${TRACE:-0}" = 1 ]; then
  TRACE=1 REPS=2 timeout -k 10 120 python -u tools/gpurun_quick.py 1024 > gpurun_out/ab_${TAG}_trace_base.log 2>&1
  SCVX_HIP_LIB=$V TRACE=1 REPS=2 timeout -k 10 120 python -u tools/gpurun_quick.py 1024 > gpurun_out/ab_${TAG}_trace_var.log 2>&1
fi
for f in gpurun_out/ab_${TAG}_*_base_*.log gpurun_out/ab_${TAG}_*_var_*.log; do python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f', round(d['value'],2), round(d['ms_per_step_median'],4), round(d['stage_ms_median']['qp'],4), d['ipm_iters_per_agent'], d['ipm_iters_max_per_step'][:8], d['status_counts'])"; done
echo done
