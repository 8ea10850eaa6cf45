#!/bin/bash
# Runs tools/graph_stream_pool_repro against torch's bundled HIP runtime (the
# one the product loads) -- usage: tools/graph_pool_repro.sh keep|destroy [trials] [seed]
set -o pipefail
TL=$(python3 -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
mkdir -p /tmp/torchhip && ln -sf "$TL/libamdhip64.so" /tmp/torchhip/libamdhip64.so.7
LD_LIBRARY_PATH=/tmp/torchhip:$TL exec "$(dirname "$0")/graph_stream_pool_repro" "$@"
