#!/usr/bin/env python3
"""Per-kernel register / scratch / LDS table from hipcc's -Rpass-analysis=kernel-resource-usage remarks.

  tools/resource_usage.py [kernel.hip] [-I dir ...]     (default: icp-4dradar_amd/csrc/icp4r_kernels.hip)

Compiles the file for gfx950 with the library's flags (nothing is written) and prints one line per
kernel: VGPRs, SGPRs, scratch bytes per lane, LDS bytes per block.  Used to check that a refactor
leaves a kernel's register allocation unchanged (diff two runs).
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def usage(path, incs):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
           "-fno-slp-vectorize", "-fPIC", "-I" + os.path.join(ROOT, "include")]
    cmd += ["-I" + d for d in incs] + ["-c", "-o", "/dev/null", path, "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+(.*?)\s+\[-Rpass", line)
        if not m:
            continue
        txt = m.group(1)
        if txt.startswith("Function Name:"):
            cur = {"name": txt.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in txt:
            k, v = txt.split(":", 1)
            cur[k.strip()] = v.strip()
    return rows


def main():
    args = sys.argv[1:]
    path = args[0] if args and not args[0].startswith("-I") else os.path.join(ROOT, "icp-4dradar_amd/csrc/icp4r_kernels.hip")
    incs = [a[2:] for a in args if a.startswith("-I")] or [os.path.dirname(path)]
    demangle = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in usage(path, incs)), capture_output=True,
                              text=True)
    rows = usage(path, incs)
    names = demangle.stdout.splitlines() if demangle.returncode == 0 else [r["name"] for r in rows]
    for r, n in zip(rows, names):
        n = re.sub(r"\(.*\)$", "", n)
        print(f"{n:60s} VGPR {r.get('VGPRs', '?'):>4} SGPR {r.get('TotalSGPRs', '?'):>4} "
              f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>4} LDS {r.get('LDS Size [bytes/block]', '?'):>6}")


if __name__ == "__main__":
    main()
