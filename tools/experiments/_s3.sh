set -u
for r in 1 2; do
timeout -k 10 400 tools/experiments/env_ab.sh 1 "ICP4R_SUMS_TAIL=0" "ICP4R_SUMS_TAIL=1" "ICP4R_SUMS_TAIL=1 ICP4R_LIBRARY=_var/ab/sp1/libicp4r.so" "ICP4R_SUMS_TAIL=1 ICP4R_LIBRARY=_var/ab/sp3/libicp4r.so" >> gpurun_out/sums3_ab.log 2>&1 || exit 5
done
