set -u
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lds or c3_full or fused or golden or part or batch" > gpurun_out/gt.log 2>&1 || { tail -20 gpurun_out/gt.log; exit 3; }
tail -2 gpurun_out/gt.log
timeout -k 10 900 tools/experiments/ab.sh 3 icp-4dradar_amd/icp4r/_lib/libicp4r.so _var/ab/pf0/libicp4r.so > gpurun_out/pf_ab.log 2>&1 || exit 4
