#!/bin/bash
# Round-6 diagnostics: the stage-system printf build on the stiff fixtures, the corrected FP64 MFMA micro-benchmark.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r6e}
SCVX_HIP_LIB=variants/stfdebug/libscvx_hip.so timeout -k 10 300 python -u -m pytest tests/test_stiff_facets_gpu.py -v -s --timeout 200 --timeout-method thread > gpurun_out/stfdebug_$T.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 120 tools/ubench/mfma_stage > gpurun_out/mfma_stage_$T.log 2>&1
echo done
