#!/usr/bin/env bash
# Kernel trace of one single-pair config's registrations (run on the GPU box):
#   tools/experiments/trace_config.sh <C1|C2|C5> [name]    -> gpurun_out/tc_<name>/
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
CFG=$1; NAME=${2:-$1}
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace -d "gpurun_out/tc_$NAME" -o run --output-format csv -- \
    python3 bench.py --plan-from-env --no-c3 --no-cpu --check 0 --configs "$CFG" > "gpurun_out/tc_$NAME.log" 2>&1
echo "trace_config: $NAME done"
