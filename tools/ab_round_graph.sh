#!/bin/bash
# A/B of the reference-schedule rollout: per-step graph replays (0), the
# branch-overlapped round graph (1), the serial round graph (2), and the episode
# scores by torch where + add_ (FS=0) or inside the mask advance (FS=1); 3 alternations.
set -o pipefail
O=gpurun_out/${1:-ab_rg}
mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_ref_schedule_gpu.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || exit 1
for i in $(seq 1 ${2:-3}); do
  for v in 0:0 0:1 2:1 1:1; do
    rg=${v%:*}; fs=${v#*:}
    EXO_REF_ROUND_GRAPH=$rg EXO_REF_FUSED_SCORE=$fs timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-td7-variants > $O/b_${rg}_${fs}_$i.log 2>&1 || exit 1
    python - $O/b_${rg}_${fs}_$i.log "$rg FS=$fs" >> $O/ab.txt <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
r = d["reference_schedule"]
print(f"ROUND_GRAPH={sys.argv[2]} {r['env_steps_per_sec']/1e6:.3f} M env-steps/s {r['ms_per_round']:.2f} ms/round "
      f"{r['rollout_ms_per_round']:.2f} rollout ms {r['burst_ms_per_round']:.2f} burst ms; default loop {d['value']/1e6:.3f} M")
PY
  done
done
cat $O/ab.txt
