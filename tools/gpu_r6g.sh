#!/bin/bash
# Round-6 A/B of the bench bookkeeping (one stacked copy per step) and the one-launch warm flags: timed-region and
# warm-start tests, then the default bench and C2.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r6g}
timeout -k 10 400 python -u -m pytest tests/test_timed_region_gpu.py tests/test_warm_start_gpu.py tests/test_dispatch_order_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c3_$T.log 2>&1
timeout -k 10 300 python -u bench.py --config c2 > gpurun_out/bench_c2_$T.log 2>&1
echo done
