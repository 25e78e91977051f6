#!/usr/bin/env bash
# nn_tile_kernel's launch duration (kernel trace) against its workgroups' span (phase stamps) for C1 at
# each query run length: does the time outside the workgroups grow with the workgroup count?
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for run in 64 32 16 8; do
    ICP4R_TILE_RUN=$run timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/trr_$run -o run --output-format csv -- \
        python3 tools/experiments/c1_loop.py 2048 30 > gpurun_out/trr_$run.log 2>&1
    echo "== tile_run $run"
    python3 tools/experiments/trace_gaps.py gpurun_out/trr_$run | grep -E "nn_tile|span"
    ICP4R_TILE_RUN=$run timeout -k 10 120 python3 tools/experiments/tile_ticks.py 2048 | tail -1
done
