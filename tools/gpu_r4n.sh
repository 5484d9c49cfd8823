#!/bin/bash
# Round-4 GPU call n (in-tree library at HEAD): full GPU suite, smoke, the C3 bench with its CPU baseline,
# c4 / c5 / scp / nash lines, PMC passes + kernel stats (tools/gpu_pmc.sh).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4n}
timeout -k 10 800 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 240 python -u bench.py > gpurun_out/bench_c3_$TAG.log 2>&1
for c in c4 c5 scp nash; do
  timeout -k 10 240 python -u bench.py --config $c --no-cpu > gpurun_out/bench_${c}_$TAG.log 2>&1
done
bash tools/gpu_pmc.sh $TAG
echo done
