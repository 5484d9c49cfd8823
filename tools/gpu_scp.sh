#!/bin/bash
# One GPU call for the SCP kernel (SCProblem / AgentSolver / SCVXSolver / Nash paths): its parity tests,
# then the scp and nash benches.  Each GPU step time-limited; anything but pytest's rc 1 ends the script.
# usage: tools/gpu_scp.sh TAG
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-scp}
timeout -k 10 400 python -u -m pytest tests/test_scp_gpu.py tests/test_compat_scp_gpu.py tests/test_nash_gpu.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_scp_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; tail -30 gpurun_out/pytest_scp_$TAG.log; [ $rc -eq 1 ] || exit $rc; }
tail -2 gpurun_out/pytest_scp_$TAG.log
timeout -k 10 300 python -u bench.py --config scp --no-cpu > gpurun_out/bench_scp_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --config nash --no-cpu > gpurun_out/bench_nash_$TAG.log 2>&1
grep -ho '"ms_per[a-z_]*": [0-9.]*' gpurun_out/bench_scp_$TAG.log gpurun_out/bench_nash_$TAG.log
echo done
