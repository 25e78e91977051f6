set -u
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sums_tail or c3_full or fused or sigma or golden" || exit 3
timeout -k 10 900 tools/experiments/env_ab.sh 3 "ICP4R_SUMS_TAIL=0" "ICP4R_SUMS_TAIL=1" || exit 3
