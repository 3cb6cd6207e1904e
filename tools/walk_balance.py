#!/usr/bin/env python3
"""When each k_walk wave ends (a clock-stamp build, tools/stamp_walk.py): one config-4 batch
through tools/perf_walk.py's harness, then every wave's start and end on the 100 MHz wall
clock and its events, from the build's device array.  Prints the distribution of wave and
workgroup end times, to tell imbalance across workgroups from the walk's own speed.

  EBD_LIB=ebpf-discovery_amd/build/variants/libebd_amd_wstamp.so python tools/walk_balance.py --events 80000000
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402

import perf_walk  # noqa: E402


def main():
    sys.argv += ["--reps", "1"] if "--reps" not in sys.argv else []
    perf_walk.main()
    import ebd
    lib = C.CDLL(ebd.LIB_PATH)
    n = 8 * 16384
    buf = (C.c_ulonglong * n)()
    assert lib.ebd_stamp_read(buf, n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8).astype(np.float64)
    a = a[a[:, 1] > 0]
    t0 = a[:, 0].min()
    start, end, evs = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0, a[:, 2]  # microseconds
    q = np.percentile(end, [0, 10, 50, 90, 99, 100])
    print(f"waves {len(a)}: start max {start.max():.0f} us; end p0/p10/p50/p90/p99/max " + " / ".join(f"{x:.0f}" for x in q) + " us")
    wg = end[: len(end) // 4 * 4].reshape(-1, 4).max(axis=1)
    we = evs[: len(evs) // 4 * 4].reshape(-1, 4).sum(axis=1)
    print(f"workgroups {len(wg)}: end p10/p50/p90/max " + " / ".join(f"{x:.0f}" for x in np.percentile(wg, [10, 50, 90, 100]))
          + f" us; events per workgroup mean {we.mean():.0f}, min {we.min():.0f}, max {we.max():.0f}; corr(end, events) "
          f"{np.corrcoef(wg, we)[0, 1]:.2f}")
    by, ss, rc, blk, it = (a[: len(a) // 4 * 4, k].reshape(-1, 4) for k in (3, 4, 5, 6, 7))
    order = np.argsort(wg)
    print("per workgroup: end us, events, MB walked, sessions, and of its slowest wave: refill and walk Mcycles, iterations")
    mid = len(order) // 2
    for name, sel in (("slowest", order[-8:]), ("median", order[mid - 2: mid + 2]), ("fastest", order[:4])):
        print(name)
        for i in sel:
            print(f"  {i}: {wg[i]:.0f}, {we[i]:.0f}, {by[i].sum() / 1e6:.2f}, {ss[i].sum():.0f}, {rc[i].max() / 1e6:.1f}, "
                  f"{blk[i].max() / 1e6:.1f}, {it[i].max():.0f}")

if __name__ == "__main__":
    main()
