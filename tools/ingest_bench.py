#!/usr/bin/env python3
"""End-to-end rate of the ingest pipeline: host-resident batches of
captured events -> H2D on the copy stream (ebd_stage_batch) -> the parse path
(ebd_submit_staged) -> per-event results back to host memory (ebd_fetch_results_async),
batch k+1's upload overlapping batch k's kernels.

The batches are config-3 traces (distinct slices, so services keep being created), generated
on the GPU (bit-identical to the host generator) and copied once into host memory before the
timed loop; the loop then streams them from the host as a BPF consumer would.

  python tools/ingest_bench.py --events 20000000 --batches 2 --steps 6 [--pageable]

Prints one JSON line: events/s including H2D and the results D2H, the H2D bytes/s, and the
device-resident step time of the same batches for comparison.
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


def host_batch(ctx, cfg, seed, first, E, pinned, dev):
    n, size = ebd.trace_size_device(ctx, cfg, seed, first, E, align=1, with_events=True)
    ev = torch.empty(n * 36, dtype=torch.uint8, device=dev)
    ln = torch.empty(n, dtype=torch.int32, device=dev)
    of = torch.empty(n, dtype=torch.int64, device=dev)
    pay = torch.empty(size + 64, dtype=torch.uint8, device=dev)
    ebd.generate_device(ctx, cfg, seed, first, E, ev, ln, of, pay, pay.numel(), align=1)
    torch.cuda.synchronize()
    if pinned:
        h = (ctx.pinned_empty(n, ebd.EVENT_DTYPE), ctx.pinned_empty(n, np.uint32), ctx.pinned_empty(n, np.uint64),
             ctx.pinned_empty(size + 16, np.uint8))
    else:
        h = (np.zeros(n, ebd.EVENT_DTYPE), np.zeros(n, np.uint32), np.zeros(n, np.uint64), np.zeros(size + 16, np.uint8))
    h[0].view(np.uint8)[:] = ev.cpu().numpy()
    h[1][:] = ln.cpu().numpy().view(np.uint32)
    h[2][:] = of.cpu().numpy().view(np.uint64)
    h[3][:size + 16] = pay[:size + 16].cpu().numpy()
    return h + (size,)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=20_000_000)
    ap.add_argument("--batches", type=int, default=2, help="distinct host batches, streamed round robin")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--pageable", action="store_true", help="plain (pageable) host arrays instead of pinned ones")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    E = a.events
    ctx = ebd.Context(max_events=E, service_capacity=1 << max(20, int(np.ceil(np.log2(E * a.steps * 0.8)))),
                      string_arena=max(256 << 20, E * a.steps * 48), timing=True)
    t = time.perf_counter()
    batches = [host_batch(ctx, a.config, a.config, k * E, E, not a.pageable, dev) for k in range(a.batches)]
    prep = time.perf_counter() - t
    res = [ctx.pinned_empty(E, ebd.RESULT_DTYPE) for _ in range(2)]
    n_ev = [len(b[0]) for b in batches]
    h2d = [b[0].nbytes + b[1].nbytes + b[2].nbytes + b[4] for b in batches]

    def run(steps):
        tickets = [None] * (steps + 1)
        b0 = batches[0]
        tickets[0] = ctx.stage(b0[0], b0[1], b0[2], b0[3][:b0[4] + 16])
        for k in range(steps):
            if k + 1 < steps:
                bn = batches[(k + 1) % len(batches)]
                tickets[k + 1] = ctx.stage(bn[0], bn[1], bn[2], bn[3][:bn[4] + 16])
            ctx.submit_staged(tickets[k])
            ctx.results_async(res[k % 2])
        ctx.sync()

    run(2)  # warm-up: allocations, first service creation
    ctx.clear()
    ctx.reset_kernel_times()
    t = time.perf_counter()
    run(a.steps)
    el = time.perf_counter() - t
    kt = ctx.kernel_times()
    events = sum(n_ev[k % len(batches)] for k in range(a.steps))
    bytes_h2d = sum(h2d[k % len(batches)] for k in range(a.steps))
    bytes_d2h = events * ebd.RESULT_DTYPE.itemsize
    gpu_ms = sum(v[1] for v in kt.values())
    st = ctx.stats()
    print(json.dumps({
        "metric": "HTTP events parsed/s end to end (host batches: H2D + parse + results D2H)",
        "value": events / el, "unit": "events/s", "source_memory": "pageable" if a.pageable else "pinned",
        "events_per_batch": n_ev, "steps": a.steps, "elapsed_s": el, "h2d_gbps": bytes_h2d / el / 1e9,
        "d2h_gbps": bytes_d2h / el / 1e9, "h2d_bytes_per_event": bytes_h2d / events,
        "kernel_ms_per_step": gpu_ms / a.steps, "device_resident_equiv_events_per_s": events / (gpu_ms / 1e3),
        "prep_s": prep, "services": st["services"], "errors": st["error_names"],
        "config": a.config}), flush=True)


if __name__ == "__main__":
    main()
