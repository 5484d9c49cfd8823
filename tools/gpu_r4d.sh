#!/bin/bash
# Round-4 GPU call d: the late-step C4 test + the full GPU suite (the twin now mirrors the kernel's pivot clamp).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4d}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { rc=$?; echo "pytest rc $rc"; [ $rc -eq 1 ] || exit $rc; }
echo done
