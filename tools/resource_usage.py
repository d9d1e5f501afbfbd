#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of the libp2v device code, from the
compiler's kernel-resource-usage remarks (no GPU needed).

usage: tools/resource_usage.py [-D...]...   (extra hipcc flags, e.g. -DP2V_MUL_PRODUCT=0)
"""
import concurrent.futures as cf
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "plonky2-verifier_amd")
FILES = ["kernels", "vanish", "vanish_poseidon", "json_pack"]


def usage(name, extra):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-result",
           "--cuda-device-only", "-c", "-o", os.devnull, f"csrc/{name}.hip", "-Rpass-analysis=kernel-resource-usage"] + extra
    out = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"kernel": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\S+) \[-Rpass", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    return rows


def main():
    extra = sys.argv[1:]
    with cf.ThreadPoolExecutor(len(FILES)) as ex:
        res = list(ex.map(lambda f: usage(f, extra), FILES))
    print(f"{'kernel':28s} {'VGPRs':>6s} {'SGPRs':>6s} {'scratch':>8s} {'waves/SIMD':>10s} {'LDS':>7s}")
    for rows in res:
        for r in rows:
            print(f"{r['kernel']:28s} {r.get('VGPRs', '?'):>6s} {r.get('TotalSGPRs', '?'):>6s} "
                  f"{r.get('ScratchSize', '?'):>8s} {r.get('Occupancy', '?'):>10s} {r.get('LDS Size', '?'):>7s}")


if __name__ == "__main__":
    main()
