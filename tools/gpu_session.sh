#!/usr/bin/env bash
# One GPU session on the box: every GPU step has its own time limit; the session stops at the first
# crash/abort/timeout (exit codes other than 0 = ok and 1 = test failures).  Logs -> gpurun_out/.
# usage: tools/gpu_session.sh "step-name:timeout:command" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
    name="${spec%%:*}"; rest="${spec#*:}"; to="${rest%%:*}"; cmd="${rest#*:}"
    echo "=== [$name] (timeout ${to}s) $cmd" | tee -a gpurun_out/session.log
    start=$(date +%s)
    timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/${name}.log" 2>&1
    rc=$?
    echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
    tail -n 25 "gpurun_out/${name}.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "=== stopping: step $name ended with rc=$rc" | tee -a gpurun_out/session.log
        exit $rc
    fi
done
