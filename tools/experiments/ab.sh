#!/usr/bin/env bash
# A/B of library builds on one box (boxes differ by up to ~6 %, so only same-session pairs compare).
#   tools/experiments/ab.sh <rounds> <lib_a.so> <lib_b.so> [more libs...]
# Alternates `bench.py` (C3, no CPU baseline / upload / C5 legs) over the libraries, `rounds` times,
# and prints per library: value, search / update launch averages (ICP4R_LIBRARY selects the build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 "$R"); do
    for lib in "$@"; do
        out=$(ICP4R_LIBRARY="$lib" timeout -k 10 120 python3 bench.py --plan-from-env --no-cpu --no-upload --configs= --check 2 --steps 20 \
              2> gpurun_out/ab_err.log | grep '^{')
        rc=$?
        if [ $rc -ne 0 ]; then echo "ab: bench failed on $lib (rc=$rc)"; tail -5 gpurun_out/ab_err.log; exit 2; fi
        echo "$out" >> gpurun_out/ab.jsonl
        python3 tools/experiments/benchline.py "$lib" "$out"
    done
done
