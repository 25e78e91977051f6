#!/usr/bin/env bash
# SQ instruction / wait counters of the benchmark's kernels (separate --pmc passes, kernel trace only).
#   tools/experiments/sq_counters.sh <outdir>
set -eu
OUT=${1:-gpurun_out/sq}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
# kernel-level profiles of the single-stream configuration (bench.py prices its kernels on the same)
export ICP4R_GROUPS=1
ARGS="--steps 1 --warmup 0 --no-cpu --check 0 --no-upload --no-c5"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    --kernel-trace -d "$OUT/p1" -o run --output-format csv -- python3 bench.py --plan-from-env $ARGS > "$OUT.p1.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    --kernel-trace -d "$OUT/p2" -o run --output-format csv -- python3 bench.py --plan-from-env $ARGS > "$OUT.p2.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA \
    --kernel-trace -d "$OUT/p3" -o run --output-format csv -- python3 bench.py --plan-from-env $ARGS > "$OUT.p3.log" 2>&1
echo "sq_counters: done"
