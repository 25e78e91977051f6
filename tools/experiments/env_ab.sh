#!/usr/bin/env bash
# A/B of runtime switches on one box: tools/experiments/env_ab.sh <rounds> "<ENV=V ...>" "<ENV=V ...>" ...
# Alternates bench.py (C3, no CPU / upload / C5 legs) over the settings and prints value, search /
# update launch averages and batch time per setting ("-" = defaults).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 "$R"); do
    for setting in "$@"; do
        envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
        out=$(env "${envs[@]}" timeout -k 10 120 python3 bench.py --plan-from-env --no-cpu --no-upload --configs= --check 2 --steps 20 \
              2> gpurun_out/env_ab_err.log | grep '^{')
        rc=$?
        if [ $rc -ne 0 ]; then echo "env_ab: bench failed on '$setting' (rc=$rc)"; tail -5 gpurun_out/env_ab_err.log; exit 2; fi
        python3 tools/experiments/benchline.py "$setting" "$out"
    done
done
