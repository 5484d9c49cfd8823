#!/bin/bash
# Round-4 GPU call h: (1) the SCP kernel with the end-game step fraction and its iteration trace (dbg/scpt):
# the dumped failing best response, the batched game statuses; (2) dbg/varC (n = 12 row state in workspace
# columns + the original factor + the SCP end game): SCP / Nash / VC / coupled tests, c5, scp, nash, c3 lines.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4h}
T=dbg/scpt/libscvx_hip.so; C=dbg/varC/libscvx_hip.so
SCVX_HIP_LIB=$T timeout -k 10 120 python -u tools/nash_fail_replay.py 1e-9 > gpurun_out/nash_replay9_$TAG.log 2>&1
SCVX_HIP_LIB=$T timeout -k 10 120 python -u tools/nash_fail_replay.py 1e-8 > gpurun_out/nash_replay8_$TAG.log 2>&1
SCVX_HIP_LIB=$T timeout -k 10 300 python -u tools/nash_batch_diag.py > gpurun_out/nash_diag_$TAG.log 2>&1
SCVX_HIP_LIB=$C timeout -k 10 700 python -u -m pytest tests/test_scp_gpu.py tests/test_nash_gpu.py tests/test_compat_scp_gpu.py tests/test_virtual_control_gpu.py tests/test_coupled_gpu.py tests/test_rtc_subproblem_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/ab_pytest_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
for c in c5 scp nash c3; do
  SCVX_HIP_LIB=$C timeout -k 10 240 python -u bench.py --config $c --no-cpu > gpurun_out/ab_${TAG}_${c}_C.log 2>&1
done
timeout -k 10 240 python -u bench.py --config scp --no-cpu > gpurun_out/ab_${TAG}_scp_base.log 2>&1
timeout -k 10 240 python -u bench.py --config nash --no-cpu > gpurun_out/ab_${TAG}_nash_base.log 2>&1
echo done
