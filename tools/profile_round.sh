#!/usr/bin/env bash
# Kernel statistics and HBM traffic of every benchmark config, for profiles/<tag>/ (run on the GPU box).
#   tools/profile_round.sh <tag> [configs]        configs: any of C3,C1,C2,C5 (default all)
# Per config: rocprofv3 --kernel-trace --stats, then separate --pmc passes for FETCH_SIZE and
# WRITE_SIZE (counters are never combined with tracing domains other than the kernel trace), then
# tools/pmc_traffic.py, which stamps profiles/pmc_traffic.json with the library's sha256.
# C3 is profiled on one pair group (bench.py prices its kernels on the same configuration).
set -eu
TAG=${1:-round3}
CONFIGS=${2:-C3,C1,C2,C5}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out "profiles/$TAG"
run() {  # run <config> <dir-suffix> <rocprof args...>
    local cfg=$1 d=$2
    shift 2
    local args
    if [ "$cfg" = C3 ]; then
        args="--steps 3 --warmup 1 --no-cpu --check 0 --no-upload --configs="
    else
        args="--no-c3 --no-cpu --check 0 --configs $cfg"
    fi
    ICP4R_GROUPS=1 timeout -k 10 300 rocprofv3 "$@" -d "gpurun_out/prof_${cfg}_$d" -o run --output-format csv -- \
        python3 bench.py --plan-from-env $args > "gpurun_out/prof_${cfg}_$d.log" 2>&1
}
for cfg in ${CONFIGS//,/ }; do
    run "$cfg" stats --kernel-trace --stats
    run "$cfg" fetch --pmc FETCH_SIZE --kernel-trace
    run "$cfg" write --pmc WRITE_SIZE --kernel-trace
    python3 tools/pmc_traffic.py --config "$cfg" --stats "gpurun_out/prof_${cfg}_stats" \
        --fetch "gpurun_out/prof_${cfg}_fetch" --write "gpurun_out/prof_${cfg}_write" --tag "$TAG" \
        > "gpurun_out/pmc_${cfg}.json"
    echo "profile_round: $cfg done"
done
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
cp profiles/"$TAG"/kernel_stats_*.csv gpurun_out/
echo "profile_round: done"
