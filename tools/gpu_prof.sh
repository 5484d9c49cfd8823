#!/bin/bash
# rocprofv3 kernel stats (csv) + PMC HBM passes + in-kernel cycle breakdown of one agent.
set -e
export TMPDIR=/tmp
TAG=${1:-r1}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/bench_prof_$TAG.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$TAG -o run -- python3 -u bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/pmc_fetch_$TAG.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$TAG -o run -- python3 -u bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/pmc_write_$TAG.log 2>&1
TRACE=1 timeout -k 10 120 python3 -u tools/gpurun_quick.py 1024 > gpurun_out/trace_$TAG.log 2>&1
echo done
