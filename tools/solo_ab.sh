#!/usr/bin/env bash
# C1/C2 registration device time: the solo plan (default), the solo plan with the sources ordered by
# the target's tree (ICP4R_SRC_ORDER=1) and the multi-launch plan (ICP4R_SOLO=0), same box, 2 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for s in "ICP4R_SOLO=1" "ICP4R_SOLO=1 ICP4R_SRC_ORDER=1" "ICP4R_SOLO=0"; do
    env $s timeout -k 10 120 python3 bench.py --no-c3 --no-cpu --check 1 --configs C1,C2 > gpurun_out/solo_ab.json 2> gpurun_out/solo_ab_err.log || { echo "bench failed: $s"; tail -20 gpurun_out/solo_ab_err.log; exit 2; }
    python3 - "$s" <<'PY'
import json, sys
r = json.loads([l for l in open("gpurun_out/solo_ab.json") if l.startswith("{")][-1])
for c in ("c1", "c2"):
    d = r.get(c) or {}
    print(f"{sys.argv[1]:34s} {c}: device {d.get('registration_device_ms'):.4f} ms  wall {d.get('registration_wall_ms_incl_pcie'):.4f} ms  "
          f"exact {d.get('bit_exact_vs_oracle')}  iters {d.get('iterations')}  solo {d.get('plan', {}).get('solo')}", flush=True)
PY
  done
done
