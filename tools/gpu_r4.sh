#!/bin/bash
# Round-4 GPU call: parity tests, smoke, C3 bench (with the like-for-like CPU baseline), C4 drift diagnostics.
# Each GPU step time-limited; a crash / timeout (anything but pytest's "tests failed" rc 1) ends the script.
# usage: tools/gpu_r4.sh TAG [pytest-args...]
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4}
shift || true
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 240 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
timeout -k 10 200 python -u tools/c4_drift.py 25 12,18 > gpurun_out/c4_drift_$TAG.log 2>&1
echo done
