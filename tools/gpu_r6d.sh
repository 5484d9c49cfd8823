#!/bin/bash
# Round-6 diagnostics call: GPU tests + benches (c3, c2, c4, c5), the stage-system printf build on the C4 HiGHS
# fixtures, the per-region byte trace (bulk and tail agent), the FP64 MFMA micro-benchmark, and the quadrotor FOH
# occupancy A/B.  Every GPU step under its own time limit; a crash or timeout ends the script.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r6d}
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
tail -n 2 gpurun_out/pytest_gpu_$T.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c3_$T.log 2>&1
timeout -k 10 300 python -u bench.py --config c4 --no-cpu > gpurun_out/bench_c4_$T.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --no-cpu > gpurun_out/bench_c5_$T.log 2>&1
SCVX_HIP_LIB=variants/focc2/libscvx_hip.so timeout -k 10 300 python -u bench.py --config c5 --no-cpu > gpurun_out/bench_c5_focc2_$T.log 2>&1
SCVX_HIP_LIB=variants/stfdebug/libscvx_hip.so timeout -k 10 300 python -u -m pytest tests/test_highs_qp_gpu.py tests/test_stiff_facets_gpu.py -v -s --timeout 200 --timeout-method thread > gpurun_out/stfdebug_$T.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
SCVX_HIP_LIB=variants/bytetrace/libscvx_hip.so WHO=bulk timeout -k 10 200 python -u tools/qp_bytes_trace.py 10 gpurun_out/bytes_bulk_$T.json > gpurun_out/bytes_bulk_$T.log 2>&1
SCVX_HIP_LIB=variants/bytetrace/libscvx_hip.so WHO=tail timeout -k 10 200 python -u tools/qp_bytes_trace.py 10 gpurun_out/bytes_tail_$T.json > gpurun_out/bytes_tail_$T.log 2>&1
timeout -k 10 120 tools/ubench/mfma_stage > gpurun_out/mfma_stage_$T.log 2>&1
timeout -k 10 200 python -u tools/qp_div_accuracy.py > gpurun_out/qpdiv_intree_$T.log 2>&1
SCVX_HIP_LIB=variants/exactdiv/libscvx_hip.so timeout -k 10 200 python -u tools/qp_div_accuracy.py > gpurun_out/qpdiv_exact_$T.log 2>&1
echo done
