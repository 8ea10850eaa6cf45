# r05: the priority update + sample right after the insert's rank launch
# (EXO_EARLY_LAP): tests, then a same-box A/B
set -e
mkdir -p gpurun_out/r05el
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05el/tests.log 2>&1
A="--steps 1000 --warmup 100 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $A > gpurun_out/r05el/on_$i.log 2>&1
  EXO_EARLY_LAP=0 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05el/off_$i.log 2>&1
done
