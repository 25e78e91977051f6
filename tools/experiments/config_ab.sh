#!/usr/bin/env bash
# A/B of runtime switches on the single-pair configs (same box): tools/experiments/config_ab.sh <rounds> <configs> "<ENV=V ...>" ...
#   e.g. tools/experiments/config_ab.sh 2 C5 - ICP4R_FUSE_SEED=0      ("-" = defaults)
# Prints per setting and config: registration device time, wall time, bit-exactness vs the oracle.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
R=$1; CFG=$2; shift 2
for r in $(seq 1 "$R"); do
  for setting in "$@"; do
    envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
    env "${envs[@]}" timeout -k 10 150 python3 bench.py --plan-from-env --no-c3 --no-cpu --check 1 --configs "$CFG" > gpurun_out/config_ab.json 2> gpurun_out/config_ab_err.log || { echo "bench failed: $setting"; tail -20 gpurun_out/config_ab_err.log; exit 2; }
    python3 - "$setting" <<'PY'
import json, sys
r = json.loads([l for l in open("gpurun_out/config_ab.json") if l.startswith("{")][-1])
for c in ("c1", "c2", "c5"):
    d = r.get(c)
    if not d:
        continue
    print(f"{sys.argv[1]:34s} {c}: device {d.get('registration_device_ms'):.4f} ms  wall {d.get('registration_wall_ms_incl_pcie'):.4f} ms  "
          f"exact {d.get('bit_exact_vs_oracle')}  iters {d.get('iterations')}  solo {d.get('plan', {}).get('solo')}", flush=True)
PY
  done
done
