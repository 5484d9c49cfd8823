#!/bin/bash
# Per-CU contention counters of the QP kernel at N=768 (3 waves per CU) and N=1024 (4 waves per CU):
# instruction cache, issue waits, TA busy, L1 (TCP) -> L2 requests and their latency.
# usage: tools/pmc_icache.sh  (writes gpurun_out/pmc_cu_*)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 768 1024; do
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD --output-format csv -d gpurun_out/pmc_cu_sq_$n -o run -- python3 -u tools/gpurun_quick.py $n > gpurun_out/pmc_cu_sq_$n.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_cu_ta_$n -o run -- python3 -u tools/gpurun_quick.py $n > gpurun_out/pmc_cu_ta_$n.log 2>&1
done
echo ok
