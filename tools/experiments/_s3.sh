set -u
ICP4R_SUMS_TAIL=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "c3_full or fused or golden or sums or sigma" > gpurun_out/gt.log 2>&1 || { tail -20 gpurun_out/gt.log; exit 3; }
tail -2 gpurun_out/gt.log
ICP4R_SUMS_TAIL=1 ICP4R_LIBRARY=_var/ab/sp2/libicp4r.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sums or fused" > gpurun_out/gt2.log 2>&1 || { tail -20 gpurun_out/gt2.log; exit 3; }
tail -2 gpurun_out/gt2.log
for r in 1 2 3; do
timeout -k 10 300 tools/experiments/env_ab.sh 1 "ICP4R_SUMS_TAIL=0" "ICP4R_SUMS_TAIL=1" "ICP4R_SUMS_TAIL=1 ICP4R_LIBRARY=_var/ab/sp2/libicp4r.so" >> gpurun_out/sums2_ab.log 2>&1 || exit 5
done
