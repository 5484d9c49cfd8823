#!/bin/bash
# One GPU call: parity tests, smoke, bench (c3 with both trust-region rules + c2 + c4 + c5), rocprof kernel stats.
# Each GPU step time-limited;
# a crash / timeout (anything but pytest's "tests failed" rc 1) ends the script.
# usage: tools/gpu_full.sh TAG [pytest-args...]
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r2}
shift || true
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --config c2 > gpurun_out/bench_c2_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --config c4 --no-cpu > gpurun_out/bench_c4_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --no-cpu > gpurun_out/bench_c5_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --no-cpu --rules one --steps 10 --warmup 3 > gpurun_out/bench_prof_$TAG.log 2>&1
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
echo done
