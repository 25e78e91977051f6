set -u
timeout -k 10 900 tools/experiments/env_ab.sh 2 "-" "ICP4R_GROUPS=3" "ICP4R_GROUPS=4" "ICP4R_GROUPS=3 ICP4R_SEARCH_CU_DIV=2" "ICP4R_PART=2048" "ICP4R_PART=512" > gpurun_out/groups_ab.log 2>&1 || exit 3
