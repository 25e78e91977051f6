#!/usr/bin/env bash
# C3 A/B of one plan option on the GPU box: bench.py lines for each value, interleaved, repeated.
#   tools/experiments/plan_ab.sh <option> "<v1> <v2> ..." [rounds=2] [steps=20]
# Writes gpurun_out/plan_ab_<option>.jsonl (one bench line per run, tagged with the value).
set -eu
OPT=$1; VALS=$2; ROUNDS=${3:-2}; STEPS=${4:-20}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
out=gpurun_out/plan_ab_${OPT}.jsonl
: > "$out"
for r in $(seq "$ROUNDS"); do
    for v in $VALS; do
        line=$(timeout -k 10 240 python3 bench.py --steps "$STEPS" --warmup 3 --no-cpu --check 0 --no-upload --configs= \
               --plan "$OPT=$v" 2>/dev/null | tail -1)
        echo "{\"$OPT\": $v, \"round\": $r, \"line\": $line}" >> "$out"
        echo "$OPT=$v round $r: $(echo "$line" | python3 -c 'import sys,json; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
    done
done
