#!/usr/bin/env python3
"""Debug harness for the network-map merge (tests/test_gpu_netcounters.py's config-5 case):
which received records have no service, a bad kind or a zero time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ebpf-discovery_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ebd  # noqa: E402
from ebd import shard  # noqa: E402

T0, MIN = 10**12, 60 * 10**9
dev = torch.device("cuda:0")
world, N = 2, 200_000
segs = [[] for _ in range(world)]
for r in range(world):
    ctx = ebd.Context(max_events=N, service_capacity=1 << 19, hash_key=ebd.TEST_HASH_KEY, network_counters=True,
                      net_capacity=1 << 20)
    ctx.set_clock(T0 + r * MIN)
    k, size = ebd.trace_size_device(ctx, 5, 5, 0, N, align=16, shard=(world, r), with_events=True)
    ev = torch.empty(k * 36, dtype=torch.uint8, device=dev)
    ln = torch.empty(k, dtype=torch.int32, device=dev)
    of = torch.empty(k, dtype=torch.int64, device=dev)
    gi = torch.empty(k, dtype=torch.int64, device=dev)
    pay = torch.zeros(size + 64, dtype=torch.uint8, device=dev)
    ebd.generate_device(ctx, 5, 5, 0, N, ev, ln, of, pay, pay.numel(), align=16, shard=(world, r), gidx=gi)
    ctx.submit_device(ev, ln, of, pay, k)
    ctx.sync()
    recs, strs, counts, scounts = ctx.export_services_device(world, dev)
    if "--map" in sys.argv:
        shard.map_wire_first(recs, lambda f: gi[f])
    raw = ctx.networks_device(dev)
    host_nets = raw.cpu().numpy().view(ebd.SERVICE_NET_DTYPE)
    own_keys = set((int(a), int(b)) for a, b in zip(ctx.services_raw()[0]["key_lo"], ctx.services_raw()[0]["key_hi"]))
    miss = sum((int(a), int(b)) not in own_keys for a, b in zip(host_nets["key_lo"], host_nets["key_hi"]))
    print("rank", r, "events", k, "services", sum(counts), "nets", host_nets.size, "nets without own service", miss,
          "kinds", np.unique(host_nets["kind"]).tolist(), "zero times", int((host_nets["time_ns"] == 0).sum()),
          "ctx.networks_raw", ctx.networks_raw().size, flush=True)
    nets, ncounts = shard.group_by_owner(raw, shard.NET_REC_BYTES, world)
    ro = np.concatenate([[0], np.cumsum(counts.astype(np.int64))]) * ebd.WIRE_DTYPE.itemsize
    so = np.concatenate([[0], np.cumsum(scounts.astype(np.int64))])
    no = np.concatenate([[0], np.cumsum(ncounts)]) * shard.NET_REC_BYTES
    for w in range(world):
        segs[w].append((recs[ro[w]:ro[w + 1]], strs[so[w]:so[w + 1]], nets[no[w]:no[w + 1]]))
    ctx.close()
for w, parts in enumerate(segs):
    m = ebd.Context(max_events=1024, max_payload=64, hash_key=ebd.TEST_HASH_KEY, network_counters=True,
                    net_capacity=1 << 20)
    m.merge_services_device(torch.cat([r for r, _, _ in parts]),
                            torch.cat([s for _, s, _ in parts] + [torch.zeros(shard.STR_SLACK, dtype=torch.uint8,
                                                                              device=dev)]))
    print("owner", w, "after services", m.stats()["error_names"], flush=True)
    allnets = torch.cat([n for _, _, n in parts])
    hn = allnets.cpu().numpy().view(ebd.SERVICE_NET_DTYPE)
    keys = set((int(a), int(b)) for a, b in zip(m.services_raw()[0]["key_lo"], m.services_raw()[0]["key_hi"]))
    miss = [(int(a), int(b)) for a, b in zip(hn["key_lo"], hn["key_hi"]) if (int(a), int(b)) not in keys]
    own = [int(a) % world for a in hn["key_lo"]]
    print("owner", w, "nets", hn.size, "missing services", len(miss), "wrong owner", sum(o != w for o in own),
          "kinds", np.unique(hn["kind"]).tolist(), "zero times", int((hn["time_ns"] == 0).sum()), flush=True)
    m.merge_networks_device(allnets)
    print("owner", w, "after nets", m.stats()["error_names"], flush=True)
    m.close()
