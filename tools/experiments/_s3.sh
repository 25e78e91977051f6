set -u
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1 || { tail -20 gpurun_out/gt.log; exit 3; }
tail -2 gpurun_out/gt.log
timeout -k 10 900 tools/experiments/ab.sh 3 icp-4dradar_amd/icp4r/_lib/libicp4r.so _var/ab/prev/libicp4r.so > gpurun_out/idx_ab.log 2>&1 || exit 4
ICP4R_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_idx -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --check 0 --no-upload --configs= > gpurun_out/prof_idx.log 2>&1 || exit 5
