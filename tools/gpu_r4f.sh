#!/bin/bash
# Round-4 GPU call f: the batched game kernel's status by agent kind at tolerances 1e-9 / 1e-8 (ECOS's default,
# the solver agent_best_response.py:100 calls) and iteration caps; dumps one instance (gpurun_out/nash_fail.npz).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4f}
timeout -k 10 300 python -u tools/nash_batch_diag.py > gpurun_out/nash_diag_$TAG.log 2>&1
echo done
