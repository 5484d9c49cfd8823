#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, each under its own kill timeout) over a short C3 bench
# (bench.py --no-cpu --steps 3 --warmup 1), then the kernel-trace stats of the default bench command.
# usage: tools/gpu_pmc.sh TAG
set -e
export TMPDIR=/tmp
TAG=${1:-r2}
mkdir -p gpurun_out
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_${TAG}_$name -o run -- python3 -u bench.py --no-cpu --rules one --steps 3 --warmup 1 > gpurun_out/pmc_${TAG}_$name.log 2>&1
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run sq2 SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
run sq3 SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SMEM
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --no-cpu --rules one > gpurun_out/bench_prof_$TAG.log 2>&1
echo done
