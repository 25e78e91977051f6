#!/usr/bin/env bash
# Kernel statistics and HBM traffic of the benchmark workload, for profiles/<tag>/ (run on the GPU box).
#   tools/profile_round.sh <tag>
# rocprofv3 --kernel-trace --stats, then separate --pmc passes for FETCH_SIZE and WRITE_SIZE (counters
# are never combined with tracing domains other than the kernel trace), then tools/pmc_traffic.py.
set -eu
TAG=${1:-round1}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
# kernel-level profiles of the single-stream configuration (bench.py prices its kernels on the same)
export ICP4R_GROUPS=1
mkdir -p gpurun_out
ARGS="--steps 5 --warmup 1 --no-cpu --check 0 --no-upload --no-c5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- \
    python3 bench.py $ARGS > gpurun_out/prof_stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/prof_fetch -o run --output-format csv -- \
    python3 bench.py $ARGS > gpurun_out/prof_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/prof_write -o run --output-format csv -- \
    python3 bench.py $ARGS > gpurun_out/prof_write.log 2>&1
python3 tools/pmc_traffic.py --stats gpurun_out/prof_stats --fetch gpurun_out/prof_fetch \
    --write gpurun_out/prof_write --tag "$TAG" > gpurun_out/pmc_summary.json
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
cp "profiles/$TAG/kernel_stats.csv" gpurun_out/kernel_stats.csv
echo "profile_round: done"
