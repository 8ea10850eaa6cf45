#!/bin/bash
# GPU box: DR-sweep env kernel, session-start library vs current (and current with permutes)
set -o pipefail
mkdir -p gpurun_out/dr
export TMPDIR=/tmp
for cfg in "libexo_amd_old.so 2" "libexo_amd.so 2" "libexo_amd.so 0"; do
  set -- $cfg
  EXO_AMD_LIB=$1 EXO_RP_GATHER=$2 timeout -k 10 200 python3 bench.py --workload dr_sweep --mode env --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/dr/env_$1_$2.log 2>&1 || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/dr/env_$1_$2.log').read().strip().splitlines()[-1]); print('$1 $2', round(d['value']), round(d['ms_per_step'],4), d['roofline']['avg_kernel_ms'], d['roofline'].get('training_loop_variant'))" | tee -a gpurun_out/dr/summary.txt
done
