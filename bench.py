#!/usr/bin/env python3
"""Benchmark: HTTP events parsed per second, device-resident, on the MI355X path.

A step = one poll cycle of the hot path (Discovery::fetchAndHandleEvents -> per-buffer
HttpRequestParser::parse -> Aggregator::newRequest) over one batch of captured events
already resident in HBM.  Workloads, generated in HBM from Philox
(bit-identical to the host generator):
  N = 1: config 3 - 100 M mixed 32-1024 B GET/POST requests, Zipf endpoints, client-IP
         headers, ~1 % invalid bytes;
  N > 1: config 5 - the config-3 distribution (seed 5), N x 125 M requests sharded by
         hash(pid, fd, sessionID) across the GPUs (8 GPUs: the 1 B-request trace), one shard
         per GPU, then the owner-partitioned service merge over RCCL (timed as merge_ms).

  python bench.py                          # N=1, config 3
  python bench.py --gpus 8                 # spawns 8 ranks (one process per GPU)
  torchrun --nproc-per-node 8 bench.py --gpus 8
  python bench.py --gpus 2 --dry-run-cpu   # the multi-rank flow on CPU (gloo, no GPU)

Step modes: cold (default) = every step is one report interval: the service table is
cleared (Aggregator::clear) before the batch, so every service of the batch is created
inside the timed step; warm = the table keeps the services of earlier steps.  The other
mode is measured and reported beside.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ebpf-discovery_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
WORKLOADS = {
    1: "config1: 'GET / HTTP/1.1\\r\\nHost: 127.0.0.1\\r\\n\\r\\n' x N (plumbing)",
    2: "config2: fixed 64-B GET, single endpoint 10.0.0.1:8080/index.html",
    3: "config3: mixed 32-1024 B GET/POST (mean ~252 B), Zipf(1.1) URLs x 1e5 and hosts x 1e3, 64 pids, "
       "30% client-IP headers, ~1% invalid",
    4: "config4: 100 M requests (config-3 content, seed 4) each cut into 2-4 recv() events, 1-8 keep-alive requests "
       "per connection then DATA_END, 4096 connections interleaved (~322 M events, multi-buffer reassembly)",
    5: "config5: N x 125 M mixed-length requests (config-3 distribution, seed 5; 8 GPUs = the 1 B-request trace) "
       "sharded by hash(pid, fd, sessionID) across N GPUs, owner-partitioned RCCL service merge",
}
DEFAULT_EVENTS = {1: 1_000_000, 2: 10_000_000, 3: 100_000_000, 4: 322_000_000, 5: 125_000_000}
# config 4 is submitted as several poll cycles per step (sessions carried between them): one
# 322 M-event cycle would need a 322 M-event context (session set, session strings)
SUB_BATCH = {4: 81_000_000}
GEN_CHUNK = 1 << 28  # candidate events per device generation call


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=0, help="default: 3 at one GPU, 5 at several")
    ap.add_argument("--events", type=int, default=0, help="events per GPU (default: the config's size)")
    ap.add_argument("--seed", type=int, default=0, help="trace seed (default: the config number)")
    ap.add_argument("--service-capacity", type=int, default=0)
    ap.add_argument("--sub-batch", type=int, default=0,
                    help="events per poll cycle (default: the whole batch; config 4: 81 M); a step submits them all")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget per thread count (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-config4", action="store_true",
                    help="N = 1 default run: skip the config-4 measurement reported beside the headline")
    ap.add_argument("--config4-steps", type=int, default=3, help="timed config-4 steps (N = 1 default run)")
    ap.add_argument("--mode", choices=("cold", "warm"), default="cold",
                    help="cold: every step is one report interval, the service table cleared before the batch "
                         "(every service of the batch is created inside the timed step); warm: the table keeps "
                         "the services of earlier steps (all hits after the first batch)")
    ap.add_argument("--pmc4", default=os.path.join(ROOT, "profiles", "pmc_fetch_config4.json"),
                    help="rocprofv3 FETCH/WRITE_SIZE summary of the config-4 kernels (tools/profile_config4.sh), "
                         "matched by build id: the config-4 roofline's traffic")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_fetch_config3.json"),
                    help="rocprofv3 FETCH/WRITE_SIZE summary giving HBM traffic per k_fresh launch (matched by build id)")
    ap.add_argument("--dry-run-cpu", action="store_true",
                    help="no GPU: spawn the ranks over gloo, shard a small config-5 trace, replay each shard with the "
                         "oracle (in place of a GPU context) and run the owner-partitioned merge")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def spawn_ranks(n):
    """One process per GPU, started before anything touches a GPU; exits with the worst code."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return max((abs(c) for c in rcs), default=0)


def copy_peak(dev):
    """Measured HBM read+write rate of a 2 x 2 GiB device copy (HIP-event timed): context for
    the 8 TB/s spec peak the roofline uses."""
    import torch
    x = torch.ones(1 << 29, dtype=torch.float32, device=dev)
    y = torch.empty_like(x)
    y.copy_(x)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        y.copy_(x)
    b.record()
    b.synchronize()
    gbps = 10 * 2 * x.numel() * 4 / (a.elapsed_time(b) / 1e3) / 1e9
    del x, y
    torch.cuda.empty_cache()
    return gbps


def cpu_baseline(config, seed, budget_s, threads=True):
    """The oracle (C restatement of the reference path) on a bounded sample of the same
    workload regenerated on the host, 1 thread (the reference's single consumer thread,
    ServiceDetectionTask.cpp:43) and, with threads, all host threads (connection-sharded)."""
    import oracle_py as O
    import ebd
    o = O.Oracle()
    chunk = 250_000 if config in (3, 4, 5) else 1_000_000
    done, spent, first = 0, 0.0, 0
    gen = 3 if config == 5 else config
    if config == 4:  # generated from position 0 only: one sample, replayed in order in chunks
        ev, lens, offs, payload = O.config4_sample(seed, budget_s)
        for a in range(0, len(ev), chunk):
            if spent >= budget_s:
                break
            t = time.perf_counter()
            o.process(ev[a:a + chunk], lens[a:a + chunk], offs[a:a + chunk], payload)
            spent += time.perf_counter() - t
            done += len(ev[a:a + chunk])
        del ev, lens, offs, payload
    while spent < budget_s and config != 4:
        ev, lens, offs, payload = ebd.generate_host(gen, seed, first, chunk)
        t = time.perf_counter()
        o.process(ev, lens, offs, payload)
        spent += time.perf_counter() - t
        done += chunk
        first += chunk
    one = done / spent
    out = dict(value=one, unit="events/s", cores=1, kind="port",
               sample=f"first {done} events of the same config-{config} trace (seed {seed}) regenerated on the host, "
                      f"oracle/ C restatement (Discovery+HttpRequestParser+Aggregator semantics), 1 thread, "
                      f"{spent:.1f} s")
    mt = O.parallel_throughput(gen, seed, budget_s) if threads else None
    if mt:
        out["all_threads"] = mt
    return out


def dry_run_cpu(args):
    """The multi-rank flow without a GPU (gloo): each rank generates its config-5 shard on
    the host, replays it with the oracle (stand-in for its GPU context), keys its services
    with the product's endpoint key and runs the owner-partitioned exchange + merge."""
    import torch.distributed as dist
    import ebd
    import oracle_py as O
    from ebd import shard
    world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    dist.init_process_group("gloo")
    E = args.events or 20_000
    ev, lens, offs, payload, gidx = ebd.generate_host(5, 5, 0, E * world, shard=(world, rank), with_gidx=True)
    t = time.perf_counter()
    o = O.Oracle()
    o.process(ev, lens, offs, payload)
    rows = [(p, ep, dom, sch, i, e, int(gidx[f])) for (p, ep, dom, sch, i, e, f) in o.services_first()]
    table = shard.ServiceTable.from_rows(rows, [ebd.host_endpoint_key(r[0], r[1]) for r in rows])
    el = time.perf_counter() - t
    tm = time.perf_counter()
    mine = shard.exchange_merge(table, device="cpu")
    merge_ms = (time.perf_counter() - tm) * 1e3
    counts = [None] * world
    dist.all_gather_object(counts, (len(ev), mine.rec.size, el))
    dist.destroy_process_group()
    if rank == 0:
        n_ev = sum(c[0] for c in counts)
        print(json.dumps({"metric": "HTTP events parsed/s (CPU dry run: oracle stand-in, no GPU)", "dry_run": True,
                          "value": n_ev / max(c[2] for c in counts), "unit": "events/s", "n_gpus": world,
                          "steps": 1, "warmup": 0, "higher_is_better": True, "scaling": "weak",
                          "events_per_rank": [c[0] for c in counts], "services_merged": sum(c[1] for c in counts),
                          "merge_ms": merge_ms, "config": {"workload": WORKLOADS[5], "config": 5}}), flush=True)


def generate_shard(ctx, cfg, seed, E, world, rank, dev):
    """This rank's batch in HBM: config 5 = the events of candidates [0, world * E) whose
    connection hashes to this rank (generated in chunks); otherwise candidates [0, E).
    Returns (events, len, off, payload, gidx, n)."""
    import torch
    import ebd
    shard_ = (world, rank) if cfg == 5 else (1, 0)
    cand = E * world if cfg == 5 else E
    plan, n_tot, b_tot = [], 0, 0
    step = cand if cfg == 4 else GEN_CHUNK  # config 4's positions interleave connections: one call
    for c0 in range(0, cand, step):
        cn = min(step, cand - c0)
        k, b = ebd.trace_size_device(ctx, cfg, seed, c0, cn, align=16, shard=shard_, with_events=True)
        plan.append((c0, cn, k, b, n_tot, b_tot))
        n_tot += k
        b_tot += b
    ev_t = torch.empty(n_tot * 36, dtype=torch.uint8, device=dev)
    len_t = torch.empty(n_tot, dtype=torch.int32, device=dev)
    off_t = torch.empty(n_tot, dtype=torch.int64, device=dev)
    gidx_t = torch.empty(n_tot, dtype=torch.int64, device=dev)
    pay_t = torch.empty(b_tot + 64, dtype=torch.uint8, device=dev)
    for c0, cn, k, b, n0, b0 in plan:
        if k == 0:
            continue
        ebd.generate_device(ctx, cfg, seed, c0, cn, ev_t[n0 * 36:], len_t[n0:], off_t[n0:], pay_t[b0:], b + 64,
                            align=16, shard=shard_, gidx=gidx_t[n0:])
        if b0:
            off_t[n0:n0 + k] += b0
    torch.cuda.synchronize()
    return ev_t, len_t, off_t, pay_t, gidx_t, n_tot, b_tot


def run_config(args, cfg, E, steps, warmup, world, rank, dev, key, mode):
    """One workload on this rank: generate its batch in HBM, `warmup` untimed steps, `steps`
    timed steps (barrier + synchronize on both sides, max over ranks), the other step mode
    beside, and one untimed step that tallies the algorithmic bytes.  Returns the measurement
    (rank 0; other ranks return None at N > 1)."""
    import torch
    import ebd
    local = dev.index
    seed = args.seed or cfg
    cap = int(E * 1.15) if cfg == 5 else E
    sub = args.sub_batch or SUB_BATCH.get(cfg, 0) or cap
    reqs = cap / 3.2 if cfg == 4 else cap  # requests, not events, create services
    # the service table at half a slot per request: config 3's 30 M services of 100 M requests fill
    # 2^26 slots to 45 %, and the cold clear streams 4.3 GB instead of the 8.6 GB of 2^27 slots
    svc_cap = args.service_capacity or (1 << max(20, int(np.ceil(np.log2(max(reqs, 1) * 0.5)))))
    ctx = ebd.Context(max_events=min(cap, sub), device=local, service_capacity=svc_cap,
                      string_arena=max(256 << 20, int(reqs) * 48), timing=True, hash_key=(int(key[0]), int(key[1])))
    t0 = time.perf_counter()
    ev_t, len_t, off_t, pay_t, gidx_t, n, size = generate_shard(ctx, cfg, seed, E, world, rank, dev)
    log(f"[rank {rank}] generated {n} events, {size / 1e9:.2f} GB payload in {time.perf_counter() - t0:.1f} s")
    G = E * world if cfg == 5 else E  # trace positions per step (candidates)

    cuts = list(range(0, n, sub)) + [n]
    if world > 1:
        from ebd import shard

        def map_first(f):  # local first_seq (k * G + local index) -> trace position (k * G + gidx)
            k = torch.div(f, G, rounding_mode="floor")
            return k * G + gidx_t[f - k * G]
    merges = []  # per cold step at N > 1: (ms, exchange stats)

    def step(k, cold, each=None, merge=False):
        if cold:
            ctx.clear()  # Aggregator::clear after the previous interval's report (Aggregator.cpp:136-153)
        # global trace order: step k's event i is at k * G + its position in the trace
        ctx.set_seq_base(k * G if cfg == 5 else k * world * G + rank * G)
        for a, z in zip(cuts[:-1], cuts[1:]):  # poll cycles of the batch, sessions carried between them
            ctx.submit_device(ev_t[a * 36:], len_t[a:], off_t[a:], pay_t, z - a)
            if each is not None:
                ctx.sync()
                each(a, z)
        if merge:
            # the interval's report needs the merged table (Discovery.cpp:60-71): each GPU's
            # services go to their owners and merge there, inside the step
            tm = time.perf_counter()
            x = shard.device_exchange_merge(ctx, dev, map_first=map_first)
            merges.append(((time.perf_counter() - tm) * 1e3, x))

    def timed_steps(k0, cold):
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(k0, k0 + steps):
            step(k, cold, merge=world > 1 and cold)
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

    cold = mode == "cold"
    for k in range(warmup):
        step(k, cold, merge=world > 1 and cold)
    ctx.sync()
    ctx.reset_kernel_times()
    merges.clear()
    elapsed = timed_steps(warmup, cold)
    kt = ctx.kernel_times()
    st = ctx.stats()
    step_merges = list(merges)
    # the other mode, reported beside (same batch, same number of steps)
    other_mode = "warm" if cold else "cold"
    ctx.reset_kernel_times()
    k_other = warmup + steps
    other_elapsed = timed_steps(k_other, not cold)
    other_kt = ctx.kernel_times()

    # algorithmic bytes of one batch: consumed + 40 B per data event (36-B
    # DiscoveryEvent + 4-B length), 36 B per close-only event; one more step, untimed, reads the
    # results of every poll cycle
    acc = {"consumed": 0, "data": 0, "close": 0}
    flags_all = ev_t[:n * 36].view(-1, 36)[:, 32].cpu().numpy()

    def tally(a, z):
        r = ctx.results()
        acc["consumed"] += int(r["consumed"].astype(np.uint64).sum())
        f = flags_all[a:z]
        acc["data"] += int(((f & ebd.FLAG_NEW_DATA) != 0).sum())
        acc["close"] += int(((f & ebd.FLAG_NEW_DATA) == 0).sum())

    step(k_other + steps, cold, each=tally)
    ctx.sync()
    alg_bytes = acc["consumed"] + 40 * acc["data"] + 36 * acc["close"]
    # the roofline's kernel: k_fresh (configs 1-3, 5), or for config 4 the kernel with the most
    # time per step (the session walk), timed over all its launches in one step
    per_step = {k: v[1] / steps for k, v in kt.items() if v[0]}
    top = max(per_step, key=per_step.get) if cfg == 4 else "k_fresh"
    fresh_launches, fresh_ms = kt[top]
    fresh_avg_ms = per_step[top] if cfg == 4 else fresh_ms / max(fresh_launches, 1)
    achieved = alg_bytes / (fresh_avg_ms / 1e3) / 1e9
    traffic = None
    pmc_path = args.pmc4 if cfg == 4 else args.pmc
    if world == 1 and os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pm = json.load(f)
            if pm.get("events") == n and pm.get("config") == cfg and pm.get("build_id") == ebd.build_id():
                # config 4: the top kernel's bytes per step (its launches of the step's poll cycles)
                traffic = pm["kernels"][top]["hbm_bytes_per_step"] if cfg == 4 else pm["hbm_bytes_per_launch"]
            else:
                log(f"[bench] config {cfg}: {pmc_path} is for build {pm.get('build_id')}, config {pm.get('config')}, "
                    f"{pm.get('events')} events; this run is build {ebd.build_id()}, {n} events: traffic null")
        except (OSError, ValueError, KeyError):
            traffic = None

    # the per-(pid, endpoint) merge across GPUs: owner-partitioned all_to_all over RCCL and a
    # device merge on each owner (ebd.shard).  Cold mode: inside every timed step (one report
    # interval per step), so `value` includes it.  Warm mode: once, after the timed steps.
    merge = None
    n_all = n
    if world > 1:
        if step_merges:
            merge_ms = max(m for m, _ in step_merges)
            x = step_merges[-1][1]
            where = "inside every timed step (cold: one report interval per step), included in value"
        else:
            torch.distributed.barrier()
            torch.cuda.synchronize()
            tm = time.perf_counter()
            x = shard.device_exchange_merge(ctx, dev, map_first=map_first)
            ctx.sync()
            torch.distributed.barrier()
            merge_ms = (time.perf_counter() - tm) * 1e3
            where = "once after the timed steps (warm: the table of all steps), not in value"
        owned = ctx.stats()["services"]
        tot = torch.tensor([n, owned, x["sent"], x["record_bytes"], x["string_bytes"], x["need_bytes"],
                            x["string_bytes_one_round"]], dtype=torch.int64, device=dev)
        torch.distributed.all_reduce(tot)
        mt = torch.tensor([merge_ms], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(mt, op=torch.distributed.ReduceOp.MAX)
        n_all = int(tot[0])
        merge = {"merge_ms": float(mt.item()), "where": where, "services_merged": int(tot[1]),
                 "records_exchanged": int(tot[2]), "record_bytes_per_interval": int(tot[3]),
                 "string_bytes_per_interval": int(tot[4]), "need_flag_bytes_per_interval": int(tot[5]),
                 "string_bytes_if_one_round": int(tot[6]), "record_size": shard.REC.itemsize,
                 "protocol": "two rounds: records, need flags back, endpoint bytes only for keys new to the owner",
                 "split_ms_rank0": {"export": x["export_ms"], "exchange": x["exchange_ms"], "device_merge": x["merge_ms"]},
                 "host_reads_per_interval": x["host_reads"]}
        if rank != 0:
            return None

    total_events = n_all * steps
    res = {
        "value": total_events / elapsed, "ms_per_step": elapsed / steps * 1e3, "n": n, "n_all": n_all, "size": size,
        "poll_cycles": len(cuts) - 1, "seed": seed, "alg_bytes": alg_bytes, "elapsed": elapsed, "top": top,
        "achieved": achieved, "kernel_avg_ms": fresh_avg_ms, "traffic": traffic, "merge": merge,
        "kernel_ms": {k: (v[1] / v[0] if v[0] else 0.0) for k, v in kt.items() if v[0]},
        "kernel_ms_per_step": per_step, "services": st["services"], "errors": st["error_names"],
        "other_mode": other_mode,
        "other": {"value": total_events / other_elapsed, "ms_per_step": other_elapsed / steps * 1e3,
                  "kernel_ms": {k: (v[1] / v[0] if v[0] else 0.0) for k, v in other_kt.items() if v[0]}},
    }
    ctx.close()
    del ev_t, len_t, off_t, pay_t, gidx_t
    torch.cuda.empty_cache()
    return res


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    if args.dry_run_cpu:
        return dry_run_cpu(args)
    import torch
    import ebd
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    cfg = args.config or (5 if world > 1 else 3)
    E = args.events or DEFAULT_EVENTS[cfg]
    # every rank keys services with the same secret (the merge matches keys across GPUs)
    key = np.frombuffer(os.urandom(16), np.uint64).copy()
    if world > 1:
        kt_ = torch.tensor(key.view(np.int64), device=dev)
        torch.distributed.broadcast(kt_, 0)
        key = kt_.cpu().numpy().view(np.uint64)
    m = run_config(args, cfg, E, args.steps, args.warmup, world, rank, dev, key, args.mode)
    if m is None:  # a rank other than 0 at N > 1
        torch.distributed.destroy_process_group()
        return
    n, n_all, size, elapsed, alg_bytes, top = m["n"], m["n_all"], m["size"], m["elapsed"], m["alg_bytes"], m["top"]
    seed = m["seed"]
    # config 4 (multi-buffer reassembly) beside the headline at one GPU: its own
    # step time, the session walk's roofline and the 1-thread CPU baseline, driver-timed with the rest
    c4 = None
    if world == 1 and not args.config and not args.events and not args.no_config4:
        t4 = time.perf_counter()
        m4 = run_config(args, 4, DEFAULT_EVENTS[4], args.config4_steps, 1, 1, 0, dev, key, "cold")
        c4 = {"workload": WORKLOADS[4], "config": 4, "events_per_step": m4["n"], "seed": m4["seed"],
              "poll_cycles_per_step": m4["poll_cycles"], "steps": args.config4_steps, "warmup": 1, "mode": "cold",
              "value": m4["value"], "unit": "events/s", "ms_per_step": m4["ms_per_step"],
              "roofline": {"bound": "hbm", "kernel": m4["top"], "kernel_ms_per_step": m4["kernel_avg_ms"],
                           "achieved": m4["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": m4["achieved"] / HBM_PEAK_GBS, "alg_bytes_per_step": m4["alg_bytes"],
                           "traffic": m4["traffic"],
                           "step_frac": m4["alg_bytes"] / (m4["ms_per_step"] / 1e3) / 1e9 / HBM_PEAK_GBS},
              "kernel_ms_per_step": m4["kernel_ms_per_step"], "errors": m4["errors"],
              "warm": m4["other"]}
        if not args.no_cpu_baseline:
            cb = cpu_baseline(4, m4["seed"], args.cpu_seconds / 2, threads=False)
            c4["cpu_baseline"] = cb
        c4["wall_s"] = time.perf_counter() - t4
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, seed, args.cpu_seconds)
    traffic, merge = m["traffic"], m["merge"]
    local = dev.index
    peak_copy = copy_peak(dev)
    # the measured read-stream peak: the faster of two read-only shapes
    rb = ebd.read_bandwidth(local, 4 << 30, 10)
    read_peak = max(rb.values())
    total_events = n_all * args.steps
    out = {
        "metric": "HTTP events parsed/s (device-resident)",
        "value": m["value"],
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
        "config": {"workload": WORKLOADS[cfg], "config": cfg, "events_per_gpu": n, "seed": seed,
                   "payload_bytes_per_gpu": size, "step_mode": args.mode, "poll_cycles_per_step": m["poll_cycles"],
                   "parallelism": (f"{world} shards by hash(pid, fd, sessionID), RCCL owner merge" if world > 1
                                   else "1 GPU")},
        "roofline": {"bound": "hbm", "achieved": m["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": m["achieved"] / HBM_PEAK_GBS, "traffic": traffic,
                     "measured_read_peak": read_peak, "frac_of_measured_read_peak": m["achieved"] / read_peak,
                     "measured_read_shapes_gbps": rb,
                     "kernel": top, "kernel_avg_ms": m["kernel_avg_ms"], "alg_bytes_per_launch": alg_bytes,
                     "alg_bytes_def": "sum(consumed) + 40 B per data event (36-B DiscoveryEvent + 4-B length) + 36 B per "
                                      "close-only event" + (" (kernel time: all its launches in one step of %d poll "
                                                             "cycles)" % m["poll_cycles"] if cfg == 4 else "")},
        "step_roofline_frac": alg_bytes * args.steps / elapsed / 1e9 / HBM_PEAK_GBS,
        "cpu_baseline": cpu,
        "step_gbps_alg": alg_bytes * world * args.steps / elapsed / 1e9,
        "kernel_ms": m["kernel_ms"],
        "measured_copy_gbps": peak_copy,
        "services": m["services"],
        "errors": m["errors"],
        "merge": merge,
        "mode": args.mode,
        m["other_mode"]: m["other"],
        "config4": c4,
        "build_id": ebd.build_id(),
    }
    print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
