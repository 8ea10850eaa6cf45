#!/bin/bash
# GPU box: every bench.py variant once (short), one JSON line each
set -o pipefail
mkdir -p gpurun_out/variants
for v in "--workload wide" "--workload dr_sweep" "--physics multibody" "--precision fp32" "--precision fp16" "--eager" "--mode env"; do
  tag=$(echo $v | tr -d ' -')
  timeout -k 10 300 python bench.py $v --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/variants/$tag.json 2> gpurun_out/variants/$tag.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/variants/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value']), round(d['ms_per_step'], 4), d.get('weights_finite'))"
done | tee gpurun_out/variants/summary.txt
