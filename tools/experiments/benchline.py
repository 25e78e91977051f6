"""Summary of one bench.py JSON line for the A/B scripts (ab.sh, env_ab.sh):
    python3 tools/experiments/benchline.py <label> '<json line>'
The search and the update are found by kernel name in `roofline` / `nn_kernel` / `update_kernel`
(`roofline` holds whichever has the larger share of the step's device time)."""
import json
import sys


def kernels(r: dict) -> dict:
    out = {}
    for key in ("roofline", "nn_kernel", "update_kernel"):
        v = r.get(key)
        if isinstance(v, dict) and v.get("kernel"):
            out[v["kernel"]] = v
    return out


def main():
    label, r = sys.argv[1], json.loads(sys.argv[2])
    k = kernels(r)
    s = k.get("nn_lds_kernel", {}).get("avg_launch_ms", 0.0) * 1e3
    u = k.get("fold_update_kernel", {})
    print(f"{label:40s} value {r['value']:9.0f}  search {s:6.1f} us  update {u.get('avg_launch_ms', 0.0) * 1e3:6.1f} us  "
          f"batch {r['batch_device_ms']:6.3f} ms  hit {u.get('cache_hit_rate') or 0:.4f}  parity {r['parity_ok']}",
          flush=True)


if __name__ == "__main__":
    main()
