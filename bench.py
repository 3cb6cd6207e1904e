#!/usr/bin/env python3
"""Benchmark: HTTP events parsed per second, device-resident, on the MI355X path.

A step = one poll cycle of the hot path (Discovery::fetchAndHandleEvents -> per-buffer
HttpRequestParser::parse -> Aggregator::newRequest) over one batch of captured events
already resident in HBM.  Default workload: SURVEY.md 8(d) config 3 — 100 M mixed
32-1024 B GET/POST requests (mean ~252 B), Zipf endpoints, client-IP headers, ~1 %
invalid bytes, generated in HBM from Philox (identical to the host generator).

  python bench.py                      # N=1, config 3, 5 timed steps
  torchrun --nproc-per-node N bench.py --gpus N   # weak scaling, one shard per GPU

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ebpf-discovery_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ebd  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
WORKLOADS = {
    1: "config1: 'GET / HTTP/1.1\\r\\nHost: 127.0.0.1\\r\\n\\r\\n' x N (plumbing)",
    2: "config2: fixed 64-B GET, single endpoint 10.0.0.1:8080/index.html",
    3: "config3: mixed 32-1024 B GET/POST (mean ~252 B), Zipf(1.1) URLs x 1e5 and hosts x 1e3, 64 pids, "
       "30% client-IP headers, ~1% invalid",
}
DEFAULT_EVENTS = {1: 1_000_000, 2: 10_000_000, 3: 100_000_000}


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--events", type=int, default=0, help="events per GPU (default: the config's size)")
    ap.add_argument("--seed", type=int, default=0, help="trace seed (default: the config number)")
    ap.add_argument("--service-capacity", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline budget (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", choices=("cold", "warm"), default="cold",
                    help="cold: every step is one report interval, the service table cleared before the batch "
                         "(every service of the batch is created inside the timed step); warm: the table keeps "
                         "the services of earlier steps (all hits after the first batch)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_fetch_config3.json"),
                    help="rocprofv3 FETCH_SIZE summary giving HBM traffic per k_fresh launch")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def stream_read_peak(dev):
    """Measured HBM read bandwidth of a plain 4 GiB reduction (for context, not the roofline)."""
    x = torch.ones(1 << 30, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    best = 0.0
    for _ in range(5):
        t = time.perf_counter()
        x.sum()
        torch.cuda.synchronize()
        best = max(best, x.numel() * 4 / (time.perf_counter() - t) / 1e9)
    del x
    torch.cuda.empty_cache()
    return best


def cpu_baseline(config, seed, budget_s):
    """The oracle (C restatement of the reference path, 1 thread) on a bounded sample of
    the same workload, regenerated on the host."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O

    o = O.Oracle()
    chunk = 250_000 if config == 3 else 1_000_000
    done, spent, first = 0, 0.0, 0
    while spent < budget_s:
        ev, lens, offs, payload = ebd.generate_host(config, seed, first, chunk)
        t = time.perf_counter()
        o.process(ev, lens, offs, payload)
        spent += time.perf_counter() - t
        done += chunk
        first += chunk
    return dict(value=done / spent, unit="events/s", cores=1, kind="port",
                sample=f"first {done} events of the same config-{config} trace (seed {seed}) regenerated on the host, "
                       f"oracle/ C restatement (Discovery+HttpRequestParser+Aggregator semantics), 1 thread, "
                       f"{spent:.1f} s")


def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cfg = args.config
    seed = args.seed or cfg
    E = args.events or DEFAULT_EVENTS[cfg]
    first = rank * E  # shard = a contiguous range of connections (one event per connection here)

    svc_cap = args.service_capacity or (1 << max(20, int(np.ceil(np.log2(max(E, 1) * 0.8)))))
    ctx = ebd.Context(max_events=E, device=local, service_capacity=svc_cap, string_arena=max(256 << 20, E * 48),
                      timing=True)
    # the batch, generated straight into HBM
    t0 = time.perf_counter()
    size = ebd.trace_size_device(ctx, cfg, seed, first, E, align=16)
    ev_t = torch.empty(E * 36, dtype=torch.uint8, device=dev)
    len_t = torch.empty(E, dtype=torch.int32, device=dev)
    off_t = torch.empty(E, dtype=torch.int64, device=dev)
    pay_t = torch.empty(size + 64, dtype=torch.uint8, device=dev)
    ebd.generate_device(ctx, cfg, seed, first, E, ev_t, len_t, off_t, pay_t, pay_t.numel(), align=16)
    torch.cuda.synchronize()
    log(f"[rank {rank}] generated {E} events, {size / 1e9:.2f} GB payload in {time.perf_counter() - t0:.1f} s")

    def step(k, cold):
        if cold:
            ctx.clear()  # Aggregator::clear after the previous interval's report (Aggregator.cpp:136-153)
        ctx.set_seq_base(k * world * E + first)  # global trace order of this shard's events
        ctx.submit_device(ev_t, len_t, off_t, pay_t, E)

    def timed_steps(k0, cold):
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(k0, k0 + args.steps):
            step(k, cold)
        ctx.sync()
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        el = time.perf_counter() - t
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
            el = float(tt.item())
        return el

    cold = args.mode == "cold"
    for k in range(args.warmup):
        step(k, cold)
    ctx.sync()
    ctx.reset_kernel_times()
    elapsed = timed_steps(args.warmup, cold)
    kt = ctx.kernel_times()
    st = ctx.stats()
    # the other mode, reported beside (same batch, same number of steps)
    other_mode = "warm" if cold else "cold"
    ctx.reset_kernel_times()
    other_elapsed = timed_steps(args.warmup + args.steps, not cold)
    other_kt = ctx.kernel_times()

    # algorithmic bytes of one batch: sum(consumed + 40) per data event
    res = ctx.results()
    data_events = int((res["status"] != ebd.STATUS_NONE).sum())
    alg_bytes = int(res["consumed"].astype(np.uint64).sum()) + 40 * data_events
    fresh_launches, fresh_ms = kt["k_fresh"]
    fresh_avg_ms = fresh_ms / max(fresh_launches, 1)
    achieved = alg_bytes / (fresh_avg_ms / 1e3) / 1e9
    traffic = None
    if os.path.exists(args.pmc):
        try:
            with open(args.pmc) as f:
                pm = json.load(f)
            if pm.get("events") == E and pm.get("config") == cfg and pm.get("build_id") == ebd.build_id():
                traffic = pm["hbm_bytes_per_launch"]
            else:
                log(f"[bench] {args.pmc} is for build {pm.get('build_id')} / {pm.get('events')} events: traffic null")
        except (OSError, ValueError, KeyError):
            traffic = None

    # the final per-(pid, endpoint) merge across GPUs, once, after the timed steps: owner-
    # partitioned all_to_all over RCCL (ebd.shard); seq numbers are already global
    merge_ms = None
    if world > 1:
        from ebd import shard
        tm = time.perf_counter()
        merged = shard.exchange_merge(shard.ServiceTable.from_context(ctx), device=dev)
        n_services = merged.rec.size if merged is not None else None
        merge_ms = (time.perf_counter() - tm) * 1e3
    else:
        n_services = st["services"]

    if rank != 0:
        torch.distributed.destroy_process_group()
        return
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, seed, args.cpu_seconds)
    peak_read = stream_read_peak(dev)
    total_events = E * world * args.steps
    out = {
        "metric": "HTTP events parsed/s (device-resident)",
        "value": total_events / elapsed,
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: Philox-seeded trace generated in HBM (bit-identical to the host generator)",
        "config": {"workload": WORKLOADS[cfg], "config": cfg, "events_per_gpu": E, "seed": seed,
                   "payload_bytes_per_gpu": size, "parallelism": f"{world} shard(s) by connection id, RCCL merge"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "k_fresh", "kernel_avg_ms": fresh_avg_ms, "alg_bytes_per_launch": alg_bytes},
        "cpu_baseline": cpu,
        "step_gbps_alg": alg_bytes * world * args.steps / elapsed / 1e9,
        "kernel_ms": {k: (v[1] / v[0] if v[0] else 0.0) for k, v in kt.items()},
        "measured_stream_read_gbps": peak_read,
        "services": n_services,
        "errors": st["error_names"],
        "merge_ms": merge_ms,
        "mode": args.mode,
        other_mode: {"value": total_events / other_elapsed, "ms_per_step": other_elapsed / args.steps * 1e3,
                     "kernel_ms": {k: (v[1] / v[0] if v[0] else 0.0) for k, v in other_kt.items()}},
        "build_id": ebd.build_id(),
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
