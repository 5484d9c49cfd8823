#!/bin/bash
# Round-6 A/B: the QP kernels built with -mllvm -amdgpu-sched-strategy=max-ilp (variants/maxilp) against the in-tree
# build, C3 / C2 / C4 / C5 on one box, alternating.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r6o}
for v in base maxilp; do
  L=""; [ $v = maxilp ] && L=variants/maxilp/libscvx_hip.so
  SCVX_HIP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/ab_${T}_c3_$v.log 2>&1
  SCVX_HIP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu --config c2 > gpurun_out/ab_${T}_c2_$v.log 2>&1
  SCVX_HIP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu --config c4 > gpurun_out/ab_${T}_c4_$v.log 2>&1
  SCVX_HIP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu --config c5 > gpurun_out/ab_${T}_c5_$v.log 2>&1
done
SCVX_HIP_LIB=variants/maxilp/libscvx_hip.so timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/ab_${T}_c3_maxilp2.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/ab_${T}_c3_base2.log 2>&1
echo done
