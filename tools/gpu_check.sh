#!/bin/bash
# One GPU call on the in-tree library: the GPU tests TESTS (default: every -m gpu test), then the bench configs
# CONFIGS (no CPU leg unless CPU=1), each GPU step under its own time limit; a crash or a timeout (anything but
# pytest's "tests failed" rc 1) ends the script.
# usage: [TESTS="tests/test_qp_gpu.py ..."|none] [CONFIGS="c3 c4"] [CPU=1] tools/gpu_check.sh TAG
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-chk}
TESTS=${TESTS:-"tests -m gpu"}
CONFIGS=${CONFIGS:-c3}
if [ "$TESTS" != none ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
  tail -n 3 gpurun_out/pytest_$TAG.log
fi
[ "$CONFIGS" = none ] && CONFIGS=""
for c in $CONFIGS; do
  if [ "${CPU:-0}" = 1 ] && [ $c = c3 ]; then X=""; else X="--no-cpu"; fi
  timeout -k 10 300 python -u bench.py --config $c $X > gpurun_out/bench_${c}_$TAG.log 2>&1
  python -c "
import json; l=[x for x in open('gpurun_out/bench_${c}_$TAG.log') if x.startswith('{')][-1]; d=json.loads(l); print('$c', round(d['value'],2), round(d['ms_per_step_median'],4), d.get('ipm_iters_per_agent'), d.get('ipm_iters_max_per_step', [])[:10], d.get('status_counts'), d.get('status_counts_per_step'))"
done
echo done
