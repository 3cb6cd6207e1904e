#!/usr/bin/env python3
"""Per-kernel register / LDS / scratch usage of ebd_kernels.hip for given -D flags.

  python tools/kstat.py [-DEBD_EXP_...] [--filter fresh]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    flags = [a for a in sys.argv[1:] if a.startswith("-D")]
    filt = None
    if "--filter" in sys.argv:
        filt = sys.argv[sys.argv.index("--filter") + 1]
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-I" + os.path.join(ROOT, "ebpf-discovery_amd/csrc"), "-I" + os.path.join(ROOT, "include"),
                        "--cuda-device-only", "-S", "-o", out, *flags,
                        os.path.join(ROOT, "ebpf-discovery_amd/csrc/ebd_kernels.hip")], check=True,
                       stderr=subprocess.DEVNULL)
        s = open(out).read()
    for m in re.finditer(r"\.name:\s+(\S+)\n(.*?)\.vgpr_spill_count:\s+(\d+)", s, re.S):
        name, blk = m.group(1), m.group(2)
        if filt and filt not in name:
            continue
        g = {k: (re.search(r"\." + k + r":\s+(\d+)", blk) or [None, "?"])[1]
             for k in ("vgpr_count", "sgpr_count", "sgpr_spill_count", "private_segment_fixed_size",
                       "group_segment_fixed_size")}
        print(f"{name:60s} vgpr {g['vgpr_count']:>4} sgpr {g['sgpr_count']:>4} sspill {g['sgpr_spill_count']:>3} "
              f"vspill {m.group(3):>3} scratch {g['private_segment_fixed_size']:>4} lds {g['group_segment_fixed_size']}")


if __name__ == "__main__":
    main()
