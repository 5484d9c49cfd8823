#!/bin/bash
# One GPU call: parity tests, smoke, bench, rocprof kernel stats. Each GPU step time-limited; stop on first failure.
# usage: tools/gpu_full.sh TAG [pytest-args...]
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r2}
shift || true
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread "$@" > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/bench_prof_$TAG.log 2>&1
echo done
