#!/bin/bash
# One GPU call: parity tests, smoke, bench, rocprof kernel stats. Each GPU step time-limited; stop on first failure.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r1}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/bench_prof_$TAG.log 2>&1
echo done
