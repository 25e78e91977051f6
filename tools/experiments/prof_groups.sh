set -eu
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu --check 0 --no-upload --no-c5"
for G in 2 4; do
export ICP4R_GROUPS=$G
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pg$G/stats -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pg$G.stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pg$G/fetch -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pg$G.fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pg$G/write -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pg$G.write.log 2>&1
done
echo done
