"""Config 5 and config 2 at full size through the HIP path.

Config 5 is the config-3 distribution (seed 5) sharded by hash(pid, fd, sessionID)
(Types.h:72-86: the session key; ebd_gen.h conn_shard).  On one GPU every shard runs in its
own context, as one GPU of the node would: the shard is generated in HBM by the device
generator (with each event's trace position), parsed and aggregated, then its services are
grouped by owner on the device (ebd_export_services_device) and every owner's segments are
merged on the device (ebd_merge_services_device) — the exchange that bench.py --gpus N runs
over RCCL.  The owners' tables together must equal the oracle over the unsharded trace
(Aggregator.cpp:155-168: counters add, the first request of a key fixes domain and scheme)."""
import os
import sys

import numpy as np
import pytest

import ebd
import oracle_py as O
import traces as T

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _device_shard(ctx, cfg, seed, first, n, world, rank, dev):
    import torch
    k, size = ebd.trace_size_device(ctx, cfg, seed, first, n, align=16, shard=(world, rank), with_events=True)
    ev = torch.empty(max(k, 1) * 36, dtype=torch.uint8, device=dev)
    ln = torch.empty(max(k, 1), dtype=torch.int32, device=dev)
    of = torch.empty(max(k, 1), dtype=torch.int64, device=dev)
    gi = torch.empty(max(k, 1), dtype=torch.int64, device=dev)
    pay = torch.zeros(size + 64, dtype=torch.uint8, device=dev)
    ebd.generate_device(ctx, cfg, seed, first, n, ev, ln, of, pay, pay.numel(), align=16, shard=(world, rank), gidx=gi)
    torch.cuda.synchronize()
    return k, ev, ln, of, pay, gi


def _merge_owner_segments(segs, dev):
    """Device merge of every owner's segments, concatenated as the all-to-all delivers them
    (wire records need no rebasing), with the merge's 8 readable bytes of slack."""
    import torch
    from ebd import shard
    rows = []
    for parts in segs:
        recs = torch.cat([r for r, _ in parts])
        strs = torch.cat([s for _, s in parts] + [torch.zeros(shard.STR_SLACK, dtype=torch.uint8, device=dev)])
        m = ebd.Context(max_events=1024, max_payload=64, hash_key=ebd.TEST_HASH_KEY)
        m.merge_services_device(recs, strs)
        st = m.stats()
        assert st["errors"] == 0, st
        rows += m.services()
        m.close()
    rows.sort(key=lambda t: (t[0], t[1]))
    return rows


@pytest.mark.parametrize("world", [2, 8])
def test_config5_shards_device_merge_equals_oracle(world):
    """1 M candidate requests of config 5 in `world` connection shards, each parsed on the GPU in
    its own context; export by owner and device merge give exactly the oracle's services over
    the whole unsharded trace."""
    import torch
    from ebd import shard
    dev = torch.device("cuda:0")
    N = 1_000_000
    segs = [[] for _ in range(world)]
    total = 0
    for r in range(world):
        ctx = ebd.Context(max_events=N // world + N // 10, service_capacity=1 << 21, hash_key=ebd.TEST_HASH_KEY)
        k, ev, ln, of, pay, gi = _device_shard(ctx, 5, 5, 0, N, world, r, dev)
        total += k
        ctx.submit_device(ev, ln, of, pay, k)
        ctx.sync()
        st = ctx.stats()
        assert st["errors"] == 0, st
        assert st["session_events"] == 0  # one buffer per connection: the fast path only
        recs, strs, counts, scounts = ctx.export_services_device(world, dev)
        shard.map_wire_first(recs, lambda f: gi[f])  # first arrival: shard order -> trace position
        if recs.numel():
            owner = shard.owner_np(recs.view(torch.int64).view(-1, 5)[:, 0].cpu().numpy().view(np.uint64), world)
            assert np.all(np.diff(owner.astype(np.int64)) >= 0)
        ro = np.concatenate([[0], np.cumsum(counts.astype(np.int64))]) * ebd.WIRE_DTYPE.itemsize
        so = np.concatenate([[0], np.cumsum(scounts.astype(np.int64))])
        for w in range(world):
            segs[w].append((recs[ro[w]:ro[w + 1]], strs[so[w]:so[w + 1]]))
        ctx.close()
    assert total == N  # the shards partition the trace
    got = _merge_owner_segments(segs, dev)
    ev, lens, offs, payload = ebd.generate_host(5, 5, 0, N, align=16)
    o = O.Oracle()
    o.process(ev, lens, offs, payload)
    assert got == o.services()


def test_config5_full_shard_properties():
    """One config-5 shard at its full size: shard 0 of 8 over 1 B candidate requests
    (~125 M events, bench.py's per-GPU batch), generated in HBM.  Random slices of its
    per-event results equal the oracle's on the host-regenerated shard events, the service
    counters add up to the per-event client classes, every FINISHED request is counted, and a
    second submission gives identical results."""
    import torch
    sys.path.insert(0, ROOT)
    import bench
    dev = torch.device("cuda:0")
    world, E = 8, 125_000_000
    cap = int(E * 1.15)
    ctx = ebd.Context(max_events=cap, service_capacity=1 << 27, string_arena=cap * 48, hash_key=ebd.TEST_HASH_KEY)
    ev, ln, of, pay, gi, n, size = bench.generate_shard(ctx, 5, 5, E, world, 0, dev)
    assert 0.98 * E < n < 1.02 * E
    ctx.submit_device(ev, ln, of, pay, n)
    ctx.sync()
    res = ctx.results()
    st = ctx.stats()
    assert st["errors"] == 0, st
    fin = res["status"] == ebd.STATUS_FINISHED
    assert st["requests"] == int(fin.sum())
    cls = (res["info"] >> 4) & 3
    raw, _ = ctx.services_raw()
    assert len(raw) == st["services"]
    assert int(raw["internal"].astype(np.int64).sum()) == int((cls == ebd.CLASS_INTERNAL).sum())
    assert int(raw["external"].astype(np.int64).sum()) == int((cls == ebd.CLASS_EXTERNAL).sum())
    gidx = gi[:n].cpu().numpy().view(np.uint64)
    assert np.all(np.diff(gidx.astype(np.int64)) > 0)
    off_all = of[:n].cpu().numpy().view(np.uint64)
    rng = np.random.default_rng(11)
    for c0 in rng.integers(0, world * E - 200_000, size=6):
        c0 = int(c0)
        hev, hl, ho, hp, hg = ebd.generate_host(5, 5, c0, 160_000, shard=(world, 0), with_gidx=True)
        a = int(np.searchsorted(gidx, hg[0]))
        z = a + len(hg)
        assert np.array_equal(gidx[a:z], hg)
        o = O.Oracle()
        out, blob = o.process(hev, hl, ho, hp)
        want = T.oracle_view(out, blob)
        lo = int(off_all[a])
        hi = int(off_all[z - 1]) + 8300
        got = T.gpu_view(res[a:z], off_all[a:z] - lo, pay[lo:hi].cpu().numpy(), None, None)
        bad = [k for k in range(len(want)) if got[k] != want[k]]
        assert not bad, (c0, [(k, got[k], want[k]) for k in bad[:3]])
    ctx.submit_device(ev, ln, of, pay, n)
    ctx.sync()
    assert np.array_equal(ctx.results().view(np.uint8), res.view(np.uint8))


def test_config2_full_size_properties():
    """Config 2 at its full size (10 M fixed 64-B GETs, one endpoint, generated in HBM):
    every request finishes with 64 bytes consumed, one service whose counters equal the
    oracle's over the same 10 M events."""
    import torch
    dev = torch.device("cuda:0")
    E = 10_000_000
    ctx = ebd.Context(max_events=E)
    n, size = ebd.trace_size_device(ctx, 2, 2, 0, E, align=16, with_events=True)
    ev = torch.empty(n * 36, dtype=torch.uint8, device=dev)
    ln = torch.empty(n, dtype=torch.int32, device=dev)
    of = torch.empty(n, dtype=torch.int64, device=dev)
    pay = torch.empty(size + 64, dtype=torch.uint8, device=dev)
    ebd.generate_device(ctx, 2, 2, 0, E, ev, ln, of, pay, pay.numel(), align=16)
    torch.cuda.synchronize()
    ctx.submit_device(ev, ln, of, pay, n)
    ctx.sync()
    res = ctx.results()
    st = ctx.stats()
    assert st["errors"] == 0, st
    assert np.all(res["status"] == ebd.STATUS_FINISHED) and np.all(res["consumed"] == 64)
    got = ctx.services()
    hev, hl, ho, hp = ebd.generate_host(2, 2, 0, E)
    o = O.Oracle()
    o.process(hev, hl, ho, hp)
    want = o.services()
    assert len(got) == 1 and got == want
    assert got[0][4] + got[0][5] == E
