#!/bin/bash
# GPU box: phase stamps of exo_step_rp (diagnostic library) for both RHS pull forms.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in 0 1; do
  EXO_RP_GATHER=$g timeout -k 10 120 python3 profiles/stamps_rp.py > gpurun_out/rp_stamps_$g.json 2>&1 || exit $?
done
