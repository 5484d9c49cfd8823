#!/bin/bash
# Round-4 GPU call l: A/B of dbg/varD (n = 12 factor: repetition descriptors rebuilt per stage, prefetch depth
# kept at 2) against the in-tree library on C5: VC/coupled tests with D, region traces and bench lines.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
D=dbg/varD/libscvx_hip.so; TAG=${1:-r4l}
SCVX_HIP_LIB=$D timeout -k 10 500 python -u -m pytest tests/test_virtual_control_gpu.py tests/test_coupled_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/ab_pytest_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 200 python -u tools/trace_coupled.py c5 4 > gpurun_out/trace_c5_base_$TAG.log 2>&1
SCVX_HIP_LIB=$D timeout -k 10 200 python -u tools/trace_coupled.py c5 4 > gpurun_out/trace_c5_D_$TAG.log 2>&1
timeout -k 10 240 python -u bench.py --config c5 --no-cpu > gpurun_out/ab_${TAG}_c5_base.log 2>&1
SCVX_HIP_LIB=$D timeout -k 10 240 python -u bench.py --config c5 --no-cpu > gpurun_out/ab_${TAG}_c5_D.log 2>&1
SCVX_HIP_LIB=dbg/ptr/libscvx_hip.so TRACE=1 REPS=2 timeout -k 10 120 python -u tools/gpurun_quick.py 1024 > gpurun_out/trace_ptr_$TAG.log 2>&1
timeout -k 10 240 python -u bench.py --config c4 --no-cpu --warm-status 1 > gpurun_out/bench_c4_ws1_$TAG.log 2>&1
echo done
