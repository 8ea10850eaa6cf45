# diagnostic: target prefetch capture segfault (see tools/seg_bisect.py)
set -o pipefail
O=gpurun_out/r04g3
mkdir -p $O
export PYTHONUNBUFFERED=1
EXO_PREFETCH_FORK=2 timeout -k 10 120 python3 tools/seg_bisect.py 128 512 1 > $O/fork_fside.log 2>&1 && \
EXO_PREFETCH_FORK=3 timeout -k 10 120 python3 tools/seg_bisect.py 128 512 1 > $O/fork_swapped.log 2>&1
