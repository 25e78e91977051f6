#!/usr/bin/env bash
# nn_tile_kernel's launch duration in a C1 trace for timing-diagnostic builds (ICP4R_DIAG_TILE: 1 = later
# passes return at entry, 2 = later passes store no results; both give wrong registrations).
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for v in base dtile1 dtile2; do
    ICP4R_LIBRARY=_var/ab/$v/libicp4r.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/td_$v -o run --output-format csv -- \
        python3 tools/experiments/c1_loop.py 2048 30 fixed > gpurun_out/td_$v.log 2>&1
    echo "== $v"
    python3 tools/experiments/trace_gaps.py gpurun_out/td_$v | grep -E "nn_tile|update|span"
done
