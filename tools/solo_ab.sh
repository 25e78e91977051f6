#!/usr/bin/env bash
# C1/C2 registration time with the solo plan on / off (same box), 2 rounds
set -u
cd "${GRAFT_REPO_ROOT:-.}"
for r in 1 2; do
  for s in 1 0; do
    ICP4R_SOLO=$s timeout -k 10 120 python3 bench.py --no-c3 --no-cpu --check 0 --configs C1,C2 > gpurun_out/solo_$s.json 2> gpurun_out/solo_err_$s.log || { echo "bench failed solo=$s"; tail -20 gpurun_out/solo_err_$s.log; exit 2; }
    python3 - "$s" <<'PY'
import json,sys
s=sys.argv[1]
r=json.loads([l for l in open(f"gpurun_out/solo_{s}.json") if l.startswith("{")][-1])
for c in ("c1","c2"):
    d=r.get(c) or {}
    print(f"solo={s} {c}: device {d.get('registration_device_ms')} ms wall {d.get('registration_wall_ms_incl_pcie')} exact {d.get('bit_exact_vs_oracle')} iters {d.get('iterations')} plan {d.get('plan')}")
PY
  done
done
