#!/bin/bash
# Round-4 GPU call y: region + factor-phase traces (-DQP_PHASE_TRACE build of the final sources, dbg/ptrace) of a
# warm-started C5 step and a cold C3 solve, for the next round's starting point.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4y}
SCVX_HIP_LIB=dbg/ptrace/libscvx_hip.so timeout -k 10 180 python -u tools/trace_coupled.py c5 > gpurun_out/trace_c5_$TAG.log 2>&1
SCVX_HIP_LIB=dbg/ptrace/libscvx_hip.so TRACE=1 REPS=2 timeout -k 10 120 python -u tools/gpurun_quick.py 1024 > gpurun_out/trace_c3_$TAG.log 2>&1
echo done
