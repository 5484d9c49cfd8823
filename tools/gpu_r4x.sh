#!/bin/bash
# Round-4 GPU call x: sanity of the rebuilt in-tree library (same sources as round4_r4u): smoke, the QP /
# dispatch-order / timed-region tests, the C3 bench line with its CPU baseline.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4x}
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_qp_gpu.py tests/test_dispatch_order_gpu.py tests/test_timed_region_gpu.py tests/test_virtual_control_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
timeout -k 10 240 python -u bench.py > gpurun_out/bench_c3_$TAG.log 2>&1
echo done
