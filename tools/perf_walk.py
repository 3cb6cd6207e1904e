#!/usr/bin/env python3
"""Config-4 session-path harness: one device-resident batch of fragmented keep-alive events,
submitted as one poll cycle; prints kernel times and the context stats (a profiling build,
EBD_EXP_WALK_PROF, puts k_walk's clock-cycle split into stats fields it does not otherwise use).

  python tools/perf_walk.py --events 20000000
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ebpf-discovery_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import ebd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=20_000_000)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--lru", type=int, default=0, help="LRU capacity (0: EBD_MAX_SESSIONS); below the trace's 4096 "
                    "live connections the batch takes the exact LRU walker")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    E = args.events
    ctx = ebd.Context(max_events=E, service_capacity=1 << max(20, int(np.ceil(np.log2(E / 3.2 * 0.8)))),
                      string_arena=max(256 << 20, E * 16), timing=True, lru_capacity=args.lru)
    ev, ln, of, pay, gidx, n, size = bench.generate_shard(ctx, 4, 4, E, 1, 0, dev)
    import time
    for k in range(args.reps):
        ctx.clear()
        ctx.reset_kernel_times()
        ctx.set_seq_base(k * n)
        torch.cuda.synchronize()
        t = time.perf_counter()
        ctx.submit_device(ev, ln, of, pay, n)
        ctx.sync()
        dt = time.perf_counter() - t
    kt = ctx.kernel_times()
    st = ctx.stats()
    print(json.dumps({"lib": os.path.basename(ebd.LIB_PATH), "events": n, "payload": size, "batch_ms": dt * 1e3,
                      "events_per_s": n / dt, "kernel_ms": {k: v[1] / v[0] for k, v in kt.items() if v[0]},
                      "kernel_total_ms": {k: v[1] for k, v in kt.items() if v[0]},
                      "launches": {k: v[0] for k, v in kt.items() if v[0]}, "stats": st}))


if __name__ == "__main__":
    main()
