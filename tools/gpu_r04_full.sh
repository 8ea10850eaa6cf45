# round-4 full GPU check: every GPU test, then smoke()
set -o pipefail
O=gpurun_out/r04full
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
