set -u
L=icp-4dradar_amd/icp4r/_lib/libicp4r.so
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
for v in "$L 0" "$L -1"; do set -- $v
  echo "== narrow $1 L1=$2"; ICP4R_LIBRARY=$1 EIGEN_L1=$2 ICP4R_WIDE_UPDATE=0 timeout -k 10 200 python tools/experiments/phase_ticks.py || exit 3
done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sigma or random_pairs or c3_full or c5_full or fused or nn_modes or batch_equals or golden" || exit 3
timeout -k 10 900 tools/experiments/ab.sh 2 _var/ab/old/libicp4r.so $L
