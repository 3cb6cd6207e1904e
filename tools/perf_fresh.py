#!/usr/bin/env python3
"""Small perf harness for profiling runs: one device-resident batch, a few submits.

  python tools/perf_fresh.py --events 20000000 --reps 3
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ebpf-discovery_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ebd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=20_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--cold", action="store_true", help="ebd_clear before every submit (services created each time)")
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
    torch.cuda.synchronize()
    ctx.submit_device(ev, ln, of, pay, E)  # cold: creates the services
    ctx.sync()
    ctx.reset_kernel_times()
    t = time.perf_counter()
    for k in range(args.reps):
        if args.cold:
            ctx.clear()
        ctx.set_seq_base((k + 1) * E)
        ctx.submit_device(ev, ln, of, pay, E)
    ctx.sync()
    dt = (time.perf_counter() - t) / args.reps
    kt = ctx.kernel_times()
    res = ctx.results()
    alg = int(res["consumed"].astype(np.uint64).sum()) + 40 * int((res["status"] != 0).sum())
    fr = kt["k_fresh"][1] / max(kt["k_fresh"][0], 1)
    print(json.dumps({"lib": os.path.basename(ebd.LIB_PATH), "cold": args.cold, "events": E, "step_ms": dt * 1e3, "events_per_s": E / dt,
                      "k_fresh_ms": fr, "k_fresh_alg_gbps": alg / fr / 1e6,
                      "session_events": ctx.stats()["session_events"],
                      "kernel_ms": {k: v[1] / v[0] for k, v in kt.items() if v[0]},
                      "errors": ctx.stats()["error_names"]}))


if __name__ == "__main__":
    main()
