# every GPU test (no -x: the whole list of failures), then smoke()
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest -q -rf --timeout 400 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
