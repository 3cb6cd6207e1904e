#!/usr/bin/env python3
"""When each k_fresh workgroup ends (a clock-stamp build, tools/stamp_fresh.py): one batch of
config-3 events, then every wave's start and end on the 100 MHz wall clock.  Prints the
distribution of workgroup end times and the slowest workgroups, to tell imbalance across
workgroups (or CUs) from the kernel's own speed.

  EBD_LIB=ebpf-discovery_amd/build/variants/libebd_amd_fstamp.so python tools/fresh_balance.py --events 100000000
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ebpf-discovery_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ebd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=100_000_000)
    ap.add_argument("--config", type=int, default=3)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    E, cfg = args.events, args.config
    ctx = ebd.Context(max_events=E, service_capacity=1 << max(20, int(np.ceil(np.log2(E * 0.8)))),
                      string_arena=max(256 << 20, E * 48), timing=True)
    E, size = ebd.trace_size_device(ctx, cfg, cfg, 0, E, align=16, with_events=True)
    ev = torch.empty(E * 36, dtype=torch.uint8, device=dev)
    ln = torch.empty(E, dtype=torch.int32, device=dev)
    of = torch.empty(E, dtype=torch.int64, device=dev)
    pay = torch.empty(size + 64, dtype=torch.uint8, device=dev)
    ebd.generate_device(ctx, cfg, cfg, 0, E, ev, ln, of, pay, pay.numel(), align=16)
    for k in range(2):
        ctx.clear()
        ctx.reset_kernel_times()
        ctx.set_seq_base((k + 1) * E)
        ctx.submit_device(ev, ln, of, pay, E)
        ctx.sync()
    kt = ctx.kernel_times()
    lib = C.CDLL(ebd.LIB_PATH)
    n = 4 * 16 * 4096
    buf = (C.c_ulonglong * n)()
    assert lib.ebd_stamp_read(buf, n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 16, 4).astype(np.float64)
    a = a[a[:, 0, 1] > 0]
    t0 = a[:, :, 0].min()
    end = (a[:, :, 1].max(axis=1) - t0) / 100.0
    start = (a[:, :, 0].min(axis=1) - t0) / 100.0
    scan_end = (np.where(a[:, :, 3] > 0, a[:, :, 1], 0).max(axis=1) - t0) / 100.0
    evs = a[:, :, 2].sum(axis=1)
    print(f"k_fresh {kt['k_fresh'][1] / kt['k_fresh'][0]:.2f} ms per launch; workgroups {len(a)}; start max {start.max():.0f} us")
    print("workgroup end p0/p10/p50/p90/p99/max " + " / ".join(f"{x:.0f}" for x in np.percentile(end, [0, 10, 50, 90, 99, 100]))
          + " us; scan end p50/max " + " / ".join(f"{x:.0f}" for x in np.percentile(scan_end, [50, 100])) + " us")
    order = np.argsort(end)
    print("slowest (workgroup: end us, events):", ", ".join(f"{i}: {end[i]:.0f}, {evs[i]:.0f}" for i in order[-12:]))
    print("fastest:", ", ".join(f"{i}: {end[i]:.0f}, {evs[i]:.0f}" for i in order[:6]))
    xcd = np.arange(len(a)) % 8
    print("mean end by XCD (block % 8):", " ".join(f"{end[xcd == x].mean():.0f}" for x in range(8)))
    loc = (np.arange(len(a)) // 8) % 32
    print("mean end by in-XCD index (block / 8) % 32:", " ".join(f"{end[loc == x].mean():.0f}" for x in range(32)))


if __name__ == "__main__":
    main()
