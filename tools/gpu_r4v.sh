#!/bin/bash
# Round-4 GPU call v: C3 dispatch-order placement experiment (tools/dispatch_ab.py), 60 steps alternating orders.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4v}
timeout -k 10 300 python -u tools/dispatch_ab.py 60 > gpurun_out/dispatch_ab_$TAG.log 2>&1
echo done
