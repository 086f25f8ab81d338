"""Per-kernel register / scratch / occupancy report of every libecgpu
translation unit (hipcc -Rpass-analysis=kernel-resource-usage, device code
only).  Dev tool: flags kernels that use scratch memory or run below
2 waves/SIMD.  Usage: python tools/kernel_resources.py [--all]"""
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "0g-ec-gpu_amd")
UNITS = [("msm_inst.hip", f"-DECG_INST={i}") for i in range(4)] + [
    ("ecfft.hip", f"-DECG_INST={i}") for i in range(4)] + [(f, "") for f in ("ntt.hip", "prep.hip", "dfft.hip")]


def scan(unit):
    src, flag = unit
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--offload-device-only",
           "-c", "-Rpass-analysis=kernel-resource-usage", os.path.join("csrc", src), "-o", os.devnull]
    if flag:
        cmd.insert(1, flag)
    out = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True).stderr
    info, cur = {}, None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            info[cur] = {}
            continue
        m = re.search(r"(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
        if m and cur:
            info[cur][m.group(1).split()[0]] = int(m.group(2))
    return f"{src} {flag}".strip(), info


def main():
    show_all = "--all" in sys.argv
    with ThreadPoolExecutor(4) as ex:
        for name, info in ex.map(scan, UNITS):
            print(f"{name}: {len(info)} kernels")
            for k, v in info.items():
                bad = v.get("ScratchSize", 0) > 0 or v.get("Occupancy", 9) < 2
                if bad or show_all:
                    print(f"  {'!' if bad else ' '} {k[:100]:100s} {v}")


if __name__ == "__main__":
    main()
