set -u
timeout -k 10 900 bash tools/profile_round.sh round4 > gpurun_out/profile_round.log 2>&1 || { tail -5 gpurun_out/profile_round.log; exit 3; }
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench_err.log || exit 4
