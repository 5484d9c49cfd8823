#!/bin/bash
# A/B of the C3 bench: default library vs SCVX_HIP_LIB=$1, alternating, each time-limited
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/ab_base_$r.log 2>&1
  SCVX_HIP_LIB=$1 timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/ab_var_$r.log 2>&1
done
for f in gpurun_out/ab_*.log; do python -c "
import json,sys; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f', round(d['value'],1), round(d['ms_per_step_median'],4), round(d['stage_ms_median']['qp'],4), d['ipm_iters_max_per_step'][:6])"; done
