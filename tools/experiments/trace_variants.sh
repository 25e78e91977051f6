#!/usr/bin/env bash
# Kernel traces of the C3 step under several runtime settings (run on the GPU box):
#   tools/experiments/trace_variants.sh "<name>:<ENV=V ...>" ...      ("<name>:" = defaults)
# Each: rocprofv3 --kernel-trace over bench.py (2 timed steps, no CPU / upload / single-pair legs);
# the traces land in gpurun_out/tv_<name>/ for tools/experiments/overlap.py / trace_groups.py.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
    name=${spec%%:*}
    envs=${spec#*:}
    env $envs timeout -k 10 240 rocprofv3 --kernel-trace -d "gpurun_out/tv_$name" -o run --output-format csv -- \
        python3 bench.py --plan-from-env --steps 2 --warmup 1 --no-cpu --check 0 --no-upload --configs= > "gpurun_out/tv_$name.log" 2>&1
    echo "trace_variants: $name done"
done
