"""GPU parity: the HIP path through the C ABI against the oracle on the same inputs.

Bit-exact comparison of per-event parse outcomes (status, consumed bytes, host, url,
client-IP front token, client class, scheme) and of the service table
(pid, endpoint, domain, scheme, internal, external)."""
import socket

import numpy as np
import pytest

import ebd
import oracle_py as O
import traces as T

pytestmark = pytest.mark.gpu


def b(s):
    return s.encode("latin-1")


def run_gpu(ev, lens, offs, payload, batches=1, lru=0, v4=(), v6=(), max_events=None, lru_window=0):
    n = len(ev)
    ctx = ebd.Context(max_events=max_events or max(n, 1), max_payload=payload.size, lru_capacity=lru)
    if lru_window:
        ctx.set_lru_window(lru_window)
    if v4 or v6:
        ctx.set_interfaces(v4, v6)
    views = []
    bounds = np.linspace(0, n, batches + 1).astype(int)
    for a, z in zip(bounds[:-1], bounds[1:]):
        ctx.submit(ev[a:z], lens[a:z], offs[a:z], payload)
        res = ctx.results()
        sreq, sstr = ctx.session_requests()
        views += T.gpu_view(res, offs[a:z], payload, sreq, sstr)
    st = ctx.stats()
    svcs = ctx.services()
    return views, svcs, st, ctx


def run_oracle(ev, lens, offs, payload, lru=8192, v4=(), v6=()):
    o = O.Oracle(lru_capacity=lru, v4_ifaces=list(v4), v6_ifaces=list(v6))
    out, blob = o.process(ev, lens, offs, payload)
    return T.oracle_view(out, blob), o.services(), o.stats()


def assert_parity(ev, lens, offs, payload, batches=1, v4=(), v6=()):
    gv, gs, gst, _ = run_gpu(ev, lens, offs, payload, batches=batches, v4=v4, v6=v6)
    ov, os_, ost = run_oracle(ev, lens, offs, payload, v4=v4, v6=v6)
    assert gst["errors"] == 0, gst
    bad = [i for i in range(len(ov)) if gv[i] != ov[i]]
    assert not bad, [(i, gv[i], ov[i]) for i in bad[:5]]
    assert gs == os_
    assert gst["kernel_deletes"] == ost["kernel_deletes"]
    assert gst["live_sessions"] == ost["lru_size"]
    return gv, gs


def test_config1_probe(vectors):
    for case in vectors["config1"]:
        n = case["n"]
        lens, offs, payload = T.pack([b(case["payload"])] * n)
        ev = T.events([dict(sid=i + 1, flags=2 | 8 | 32) for i in range(n)])
        gv, gs, st, _ = run_gpu(ev, lens, offs, payload)
        exp = [(s["pid"], b(s["endpoint"]), b(s["domain"]), b(s["scheme"]), s["internal"], s["external"])
               for s in case["services"]]
        assert gs == exp
        assert st["live_sessions"] == case["saved_sessions"]


def test_reference_parser_vectors_as_sessions(vectors):
    cases = vectors["parser_valid"] + vectors["parser_invalid"]
    chunk_lists = [[b(c) for c in case["chunks"]] for case in cases]
    ev, lens, offs, payload = T.session_trace(chunk_lists)
    gv, gs = assert_parity(ev, lens, offs, payload)
    # per case: total consumed bytes as the reference test expects
    k = 0
    for case, chunks in zip(cases, chunk_lists):
        assert sum(gv[k + j][1] for j in range(len(chunks))) == case["total"], case
        k += len(chunks)


def test_reference_parser_vectors_interleaved_and_closed(vectors):
    cases = vectors["parser_valid"] + vectors["parser_invalid"] + vectors["probe_parser"]
    chunk_lists = [T.probe_chunks(case) for case in cases]
    ev, lens, offs, payload = T.session_trace(chunk_lists, interleave=True, close=True)
    assert_parity(ev, lens, offs, payload)


def test_request_length_cap_on_gpu(vectors):
    """HttpRequestParser.cpp:88-91: before each byte, length > 8192 makes the parser INVALID
    without consuming it, so an 8193-byte request finishes and an 8194-byte one is INVALID
    after 8193 bytes.  The probes run through the session path (k_walk), in one batch and
    split across batches (the request's bytes carried between polls)."""
    probes = [c for c in vectors["probe_parser"] if "lengths" in c]
    assert len(probes) == 2
    chunk_lists = [T.probe_chunks(c) for c in probes]
    expect = [(c["state"], c["total"]) for c in probes]
    for lengths in ([4096, 4097], [1, 8192], [8000, 150, 43], [8192, 2], [4000, 4000, 195], [8192, 808],
                    [3000, 3000, 3000], [8192, 1, 1]):
        chunk_lists.append(T.length_request_chunks(lengths))
        total = sum(lengths)
        expect.append(("FINISHED" if total <= 8193 else "INVALID", min(total, 8193)))
    ev, lens, offs, payload = T.session_trace(chunk_lists)
    for batches in (1, 2, 5):
        gv, _ = assert_parity(ev, lens, offs, payload, batches=batches)
        k = 0
        for chunks, (state, total) in zip(chunk_lists, expect):
            views = gv[k:k + len(chunks)]
            k += len(chunks)
            assert sum(v[1] for v in views) == total, (chunks and len(chunks), total)
            last = [v for v in views if v[0] in (ebd.STATUS_FINISHED, ebd.STATUS_INVALID)]
            assert last and last[-1][0] == (ebd.STATUS_FINISHED if state == "FINISHED" else ebd.STATUS_INVALID)


def test_aggregator_vectors_real_checker(vectors):
    rows, bufs = [], []
    for k, r in enumerate(vectors["aggregator"]["requests"]):
        src = b""
        if r["real_src"]:
            src = socket.inet_pton(socket.AF_INET6, r["real_src"]) if ":" in r["real_src"] else socket.inet_pton(
                socket.AF_INET, r["real_src"])
        rows.append(dict(pid=r["pid"], sid=k + 1, flags=(r["flags"] or 0) | ebd.FLAG_NEW_DATA, src=src))
        bufs.append(b("GET %s HTTP/1.1\r\nHost: %s\r\n\r\n" % (r["url"], r["host"])))
    lens, offs, payload = T.pack(bufs)
    ev = T.events(rows)
    _, gs, _, _ = run_gpu(ev, lens, offs, payload)
    exp = sorted((e["pid"], b(e["endpoint"]), b(e["domain"]), b(e["scheme"]), e["internal"], e["external"])
                 for e in vectors["aggregator"]["expected"])
    assert gs == exp
    assert_parity(ev, lens, offs, payload)


def test_checker_vectors_through_the_path(vectors):
    # every IpAddressCheckerTest address as an X-Forwarded-For client (internal expected)
    addrs = vectors["v4_reserved_internal"] + [t for t, _ in vectors["v6_cases"]] + ["8.8.8.8", "2001:4860::1"]
    bufs = [b("GET /c HTTP/1.1\r\nHost: h\r\nX-Forwarded-For: %s\r\n\r\n" % a) for a in addrs]
    lens, offs, payload = T.pack(bufs)
    ev = T.events([dict(sid=k + 1, flags=2 | 8 | 32) for k in range(len(bufs))])
    v6i = [(socket.inet_pton(socket.AF_INET6, a), socket.inet_pton(socket.AF_INET6, m))
           for a, m in vectors["v6_iface"]["v6_ifaces"]]
    assert_parity(ev, lens, offs, payload, v6=v6i)


@pytest.mark.parametrize("align", [1, 16])
def test_config3_sample_single_and_multi_batch(align):
    ev, lens, offs, payload = ebd.generate_host(3, 3, 0, 60000, align=align)
    assert_parity(ev, lens, offs, payload)
    assert_parity(ev, lens, offs, payload, batches=7)


def test_config2_sample():
    ev, lens, offs, payload = ebd.generate_host(2, 2, 0, 50000)
    gv, gs = assert_parity(ev, lens, offs, payload)
    assert len(gs) == 1 and gs[0][1] == b"10.0.0.1:8080/index.html"


def test_fragmented_keepalive_sessions():
    ev, lens, offs, payload = T.fragmented_trace(3000, seed=4, window=256)
    assert_parity(ev, lens, offs, payload)
    # the same trace across several batches: sessions carried between polls
    assert_parity(ev, lens, offs, payload, batches=9)


def test_missing_buffers_and_data_end_only():
    req = b"GET /a HTTP/1.1\r\nHost: h\r\n\r\n"
    bufs = [req[:10], None, req[10:], None, req, req[:5]]
    rows = [dict(sid=1, seq=1, flags=42), dict(sid=1, seq=2, flags=42), dict(sid=1, seq=3, flags=42),
            dict(sid=1, seq=3, flags=64), dict(sid=2, flags=42 | 64), dict(sid=3, flags=42 | 64)]
    lens, offs, payload = T.pack(bufs)
    assert_parity(T.events(rows), lens, offs, payload)


def test_device_generator_matches_host():
    import torch
    n = 20000
    hev, hl, ho, hp = ebd.generate_host(3, 3, 123, n, align=16)
    ctx = ebd.Context(max_events=n)
    dev = torch.device("cuda:0")
    size = ebd.trace_size(3, 3, 123, n, align=16)
    e = torch.empty(n * 36, dtype=torch.uint8, device=dev)
    l_ = torch.empty(n, dtype=torch.int32, device=dev)
    o_ = torch.empty(n, dtype=torch.int64, device=dev)
    p_ = torch.zeros(size + 64, dtype=torch.uint8, device=dev)
    ebd.generate_device(ctx, 3, 3, 123, n, e, l_, o_, p_, p_.numel(), align=16)
    torch.cuda.synchronize()
    assert np.array_equal(e.cpu().numpy().view(ebd.EVENT_DTYPE), hev)
    assert np.array_equal(l_.cpu().numpy().view(np.uint32), hl)
    assert np.array_equal(o_.cpu().numpy().view(np.uint64), ho)
    pd = p_.cpu().numpy()
    for i in range(0, n, 97):
        a = int(ho[i])
        assert pd[a:a + int(hl[i])].tobytes() == hp[a:a + int(hl[i])].tobytes()
    # the device batch path over the HBM-resident trace equals the host path
    ctx.submit_device(e, l_, o_, p_, n)
    ctx.sync()
    g1 = ctx.services()
    ctx2 = ebd.Context(max_events=n, max_payload=hp.size)
    ctx2.submit(hev, hl, ho, hp)
    assert g1 == ctx2.services()


def test_large_config3_against_oracle():
    ev, lens, offs, payload = ebd.generate_host(3, 3, 0, 1_000_000, align=16)
    gv, gs, st, _ = run_gpu(ev, lens, offs, payload, batches=2)
    ov, os_, _ = run_oracle(ev, lens, offs, payload)
    assert st["errors"] == 0 and st["hash_collisions"] == 0
    assert gs == os_
    assert gv == ov


def test_sharded_contexts_merge_to_whole_trace():
    """Multi-GPU flow on one GPU: connection shards in separate contexts (as separate GPUs
    would run them), first arrival mapped to trace positions, merged by ebd.shard: equals
    the oracle over the whole trace.  Covers the 128-bit key export (ebd_service.key_lo/hi)."""
    from ebd import shard
    for ev, lens, offs, payload in (ebd.generate_host(3, 21, 0, 30000), T.fragmented_trace(400, seed=23, window=64)):
        tables = []
        for idx in shard.shard_indices(ev, 3):
            ctx = ebd.Context(max_events=max(len(idx), 1), max_payload=payload.size, hash_key=ebd.TEST_HASH_KEY)
            ctx.submit(ev[idx], lens[idx], offs[idx], payload)
            assert ctx.stats()["errors"] == 0
            tables.append(shard.ServiceTable.from_context(ctx, global_index=idx))
        got = shard.merge_tables(tables).packed().rows()
        _, want, _ = run_oracle(ev, lens, offs, payload)
        assert got == want


def _owner_segments(recs, strs, counts, scounts):
    ro = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
    so = np.concatenate([[0], np.cumsum(scounts.astype(np.int64))])
    n = ebd.WIRE_DTYPE.itemsize
    return [(recs[ro[w] * n:ro[w + 1] * n], strs[so[w]:so[w + 1]]) for w in range(len(counts))]


def test_device_export_by_owner_and_merge_equals_whole_trace():
    """The cross-GPU merge's device half on one GPU: each connection shard runs in its own
    context (as one GPU would), groups its services by owner on the device
    (ebd_export_services_device), first arrival mapped to trace positions; each owner's
    segments from every shard are merged on the device (ebd_merge_services_device).  The
    owners' tables together equal the oracle over the whole trace."""
    import torch
    from ebd import shard
    dev = torch.device("cuda:0")
    W = 3
    for ev, lens, offs, payload in (ebd.generate_host(3, 21, 0, 30000), T.fragmented_trace(400, seed=23, window=64)):
        segs = [[] for _ in range(W)]
        for idx in shard.shard_indices(ev, W):
            ctx = ebd.Context(max_events=max(len(idx), 1), max_payload=payload.size, hash_key=ebd.TEST_HASH_KEY)
            ctx.submit(ev[idx], lens[idx], offs[idx], payload)
            recs, strs, counts, scounts = ctx.export_services_device(W, dev)
            gpos = torch.tensor(idx.astype(np.int64), device=dev)
            shard.map_wire_first(recs, lambda f: gpos[f])  # first arrival: shard order -> trace position
            if recs.numel():
                owner = shard.owner_np(recs.view(torch.int64).view(-1, 5)[:, 0].cpu().numpy().view(np.uint64), W)
                assert np.all(np.diff(owner.astype(np.int64)) >= 0)  # grouped by owner
            for w, seg in enumerate(_owner_segments(recs, strs, counts, scounts)):
                segs[w].append(seg)
        rows = []
        for w in range(W):
            recs = torch.cat([r for r, _ in segs[w]])  # concatenated as the all-to-all delivers them
            strs = torch.cat([s for _, s in segs[w]] + [torch.zeros(shard.STR_SLACK, dtype=torch.uint8, device=dev)])
            m = ebd.Context(max_events=1024, max_payload=64, hash_key=ebd.TEST_HASH_KEY)
            m.merge_services_device(recs, strs)
            assert m.stats()["errors"] == 0
            rows += m.services()
        rows.sort(key=lambda t: (t[0], t[1]))
        _, want, _ = run_oracle(ev, lens, offs, payload)
        assert rows == want


def test_device_two_round_merge_ships_bytes_once_per_new_key():
    """The two-round merge's device half on one GPU (what device_exchange_merge runs across
    GPUs): W shard contexts export by owner; each owner merges its own records' keys first,
    then the others' (ebd_merge_service_keys_device); the need flags go back to the sources,
    which pack just those records' bytes (ebd_wire_compact_device); the owner copies them in
    (ebd_merge_service_bytes_device).  The owners' tables equal the oracle over the whole trace,
    and fewer endpoint bytes move than the one-round export holds."""
    import torch
    from ebd import shard
    dev = torch.device("cuda:0")
    W = 3
    ev, lens, offs, payload = ebd.generate_host(3, 21, 0, 30000)
    src = []  # per shard: (ctx, recs, strs, counts, device sizes)
    RB = shard.REC.itemsize
    for idx in shard.shard_indices(ev, W):
        ctx = ebd.Context(max_events=max(len(idx), 1), max_payload=payload.size, hash_key=ebd.TEST_HASH_KEY)
        ctx.submit(ev[idx], lens[idx], offs[idx], payload)
        # the export whose counts stay on the device, checked against the host-counted one
        h_recs, h_strs, h_counts, h_scounts = ctx.export_services_device(W, dev)
        recs_all, strs_all, sz = ctx.export_services_device_sized(W, dev)
        counts, scounts = sz.cpu().numpy()
        assert counts.tolist() == h_counts.tolist() and scounts.tolist() == h_scounts.tolist()
        recs, strs = recs_all[:int(counts.sum()) * RB], strs_all[:int(scounts.sum())]
        for w, ((ra, sa), (rb_, sb)) in enumerate(zip(_owner_segments(recs, strs, counts, scounts),
                                                      _owner_segments(h_recs, h_strs, h_counts, h_scounts))):
            # same records per owner (order inside a segment is free), each with the same bytes
            def rows(r, st):
                recs_np = r.cpu().numpy().view(shard.REC)
                nb = shard.wire_bytes(recs_np["endpoint_len"]).astype(np.int64)
                so = np.concatenate([[0], np.cumsum(nb)])
                b = st.cpu().numpy()
                return sorted((bytes(recs_np[k].tobytes()), bytes(b[so[k]:so[k + 1]])) for k in range(recs_np.size))
            assert rows(ra, sa) == rows(rb_, sb)
        gpos = torch.tensor(idx.astype(np.int64), device=dev)
        shard.map_wire_first(recs, lambda f: gpos[f])
        src.append((ctx, recs, strs, counts, sz))

    def seg(s, w):  # source s's records for owner w
        c = src[s][3].astype(np.int64)
        a = int(c[:w].sum())
        return src[s][1][a * RB:(a + int(c[w])) * RB]

    owners, need_for = [], [[None] * W for _ in range(W)]
    for w in range(W):
        m = ebd.Context(max_events=1024, max_payload=64, hash_key=ebd.TEST_HASH_KEY)
        parts = [seg(s, w) for s in range(W)]
        pcounts = torch.tensor([p.numel() // RB for p in parts], dtype=torch.int64, device=dev)
        dsts = [torch.empty(p.numel() // RB, dtype=torch.int64, device=dev) for p in parts]
        for s in [w] + [s for s in range(W) if s != w]:  # the owner's own records first
            m.merge_service_keys_device(parts[s], dsts[s])
        for s in range(W):
            need_for[s][w] = (dsts[s] >= 0).to(torch.uint8)
            if s != w:  # a key the owner had is never asked of another shard
                own_keys = set(map(tuple, parts[w].view(torch.int64).view(-1, 5)[:, :2].cpu().numpy().tolist()))
                keys = parts[s].view(torch.int64).view(-1, 5)[:, :2].cpu().numpy().tolist()
                asked = need_for[s][w].cpu().numpy()
                assert not any(a and tuple(k) in own_keys for a, k in zip(asked, keys))
        owners.append((m, parts, dsts, pcounts))
    sent = 0
    got = [[] for _ in range(W)]
    bcs = []
    for s in range(W):
        ctx, recs, strs, counts, sz = src[s]
        need = torch.cat([need_for[s][w] for w in range(W)])
        packed = ctx.wire_compact_device(recs, strs, need)  # with the size read
        packed2 = ctx.wire_compact_device(recs, strs, need, sized=False)  # without it
        bc = ctx.wire_segment_bytes_device(recs, sz[0], need=need).cpu().numpy()  # per owner, by the kernel
        assert int(bc.sum()) == packed.numel() and torch.equal(packed2[:packed.numel()], packed)
        bcs.append(bc)
        sent += packed.numel()
        a = 0
        for w in range(W):
            got[w].append(packed[a:a + int(bc[w])])
            a += int(bc[w])
    for w, (m, parts, dsts, pcounts) in enumerate(owners):  # the owner's per-source counts, by the kernel
        rbc = m.wire_segment_bytes_device(torch.cat(parts), pcounts, dst=torch.cat(dsts)).cpu().numpy()
        assert rbc.tolist() == [int(bcs[s][w]) for s in range(W)]
    rows = []
    for w, (m, parts, dsts, _) in enumerate(owners):
        strs = torch.cat(got[w] + [torch.zeros(shard.STR_SLACK, dtype=torch.uint8, device=dev)])
        m.merge_service_bytes_device(torch.cat(parts), torch.cat(dsts), strs)
        assert m.stats()["errors"] == 0
        rows += m.services()
    rows.sort(key=lambda t: (t[0], t[1]))
    _, want, _ = run_oracle(ev, lens, offs, payload)
    assert rows == want
    assert 0 < sent < sum(src[s][2].numel() for s in range(W))


def test_device_exchange_merge_over_rccl_world1():
    """shard.device_exchange_merge end to end through RCCL (a world-1 nccl group): export,
    all_to_all_single on GPU tensors, device merge; the table is unchanged."""
    import os
    import torch
    import torch.distributed as dist
    from ebd import shard
    ev, lens, offs, payload = ebd.generate_host(3, 31, 0, 20000)
    ctx = ebd.Context(max_events=len(ev), max_payload=payload.size)
    ctx.submit(ev, lens, offs, payload)
    before = ctx.services()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        x = shard.device_exchange_merge(ctx, torch.device("cuda", 0), map_first=lambda f: f)
    finally:
        dist.destroy_process_group()
    assert x["sent"] == x["received"] == len(before)
    assert x["record_bytes"] == 40 * len(before)
    assert x["host_reads"] == 2  # the sizes, then the bytes round's counts (two rounds)
    assert ctx.services() == before
    os.environ["MASTER_PORT"] = "29518"
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        x = shard.device_exchange_merge(ctx, torch.device("cuda", 0), map_first=lambda f: f, two_round=False)
    finally:
        dist.destroy_process_group()
    assert x["host_reads"] == 1  # one round: the sizes only
    assert ctx.services() == before


def test_device_sharded_generator_matches_host():
    """Config 5 on the device (bench.py's per-rank shard, chunked): the events of a
    connection shard, with their trace positions, equal the host generator's."""
    import torch
    dev = torch.device("cuda:0")
    ctx = ebd.Context(max_events=16)
    for world, rank in ((4, 1), (3, 2), (1, 0)):
        hev, hl, ho, hp, hg = ebd.generate_host(5, 5, 1000, 30000, align=16, shard=(world, rank), with_gidx=True)
        k, size = ebd.trace_size_device(ctx, 5, 5, 1000, 30000, align=16, shard=(world, rank), with_events=True)
        assert k == len(hev) and size <= hp.size
        e = torch.empty(k * 36, dtype=torch.uint8, device=dev)
        l_ = torch.empty(k, dtype=torch.int32, device=dev)
        o_ = torch.empty(k, dtype=torch.int64, device=dev)
        g_ = torch.empty(k, dtype=torch.int64, device=dev)
        p_ = torch.zeros(size + 64, dtype=torch.uint8, device=dev)
        ebd.generate_device(ctx, 5, 5, 1000, 30000, e, l_, o_, p_, p_.numel(), align=16, shard=(world, rank), gidx=g_)
        torch.cuda.synchronize()
        assert np.array_equal(e.cpu().numpy().view(ebd.EVENT_DTYPE), hev)
        assert np.array_equal(l_.cpu().numpy().view(np.uint32), hl)
        assert np.array_equal(o_.cpu().numpy().view(np.uint64), ho)
        assert np.array_equal(g_.cpu().numpy().view(np.uint64), hg)
        pd = p_.cpu().numpy()
        for i in range(0, k, 37):
            a = int(ho[i])
            assert pd[a:a + int(hl[i])].tobytes() == hp[a:a + int(hl[i])].tobytes()


@pytest.mark.parametrize("cap,n_conn,window,batches,lru_window", [(64, 600, 256, 1, 0), (64, 600, 256, 4, 0),
                                                                  (8192, 11000, 11000, 1, 0), (8192, 11000, 11000, 3, 0),
                                                                  (64, 600, 256, 1, 97), (64, 600, 256, 2, 301)])
def test_lru_eviction_exact(cap, n_conn, window, batches, lru_window):
    """More live sessions than the LRU holds (LRUCache.h:50-89; Discovery.cpp:39): the full
    cache evicts its least recently used session on insert, whose later buffers then parse
    as new sessions.  The exact LRU (walk-and-derive rounds, k_lru_*) must reproduce the
    oracle's LRU event for event, within a batch and across batches (recency carried with the
    sessions), and must settle by itself: no batch may fall back to the one-lane replay.  A
    small derivation window makes one batch span many windows, so resumed walks (states
    restored from the per-event snapshot) run on the device."""
    ev, lens, offs, payload = T.fragmented_trace(n_conn, seed=31, window=window)
    gv, gs, gst, _ = run_gpu(ev, lens, offs, payload, batches=batches, lru=cap, lru_window=lru_window)
    ov, os_, ost = run_oracle(ev, lens, offs, payload, lru=cap)
    assert ost["lru_evictions"] > 0
    assert gst["errors"] == 0, gst
    assert gst["lru_exact_batches"] >= 1
    assert gst["lru_sequential"] == 0 and gst["lru_rounds"] > 0, gst
    if lru_window:
        assert gst["lru_rounds"] > len(ev) // batches // lru_window, gst  # several windows per batch
    bad = [i for i in range(len(ov)) if gv[i] != ov[i]]
    assert not bad, [(i, gv[i], ov[i]) for i in bad[:5]]
    assert gs == os_
    assert gst["kernel_deletes"] == ost["kernel_deletes"]
    assert gst["live_sessions"] == ost["lru_size"]
    assert gst["lru_evictions"] == ost["lru_evictions"]


def test_lru_evictions_counted_once_across_merges():
    """ebd_get_stats().lru_evictions after an evicting batch stays put through the calls that
    run k_verify again (ebd_merge_service_keys_device, ebd_aggregate_requests): the batch's
    evictions enter the run total once."""
    import torch
    ev, lens, offs, payload = T.fragmented_trace(600, seed=31, window=256)
    _, _, gst, ctx = run_gpu(ev, lens, offs, payload, lru=64)
    ost = run_oracle(ev, lens, offs, payload, lru=64)[2]
    assert gst["lru_evictions"] == ost["lru_evictions"] > 0
    recs, strs, counts, scounts = ctx.export_services_device(1, "cuda")
    dst = torch.empty(int(counts[0]), dtype=torch.int64, device="cuda")
    other = ebd.Context(max_events=16, hash_key=ctx.hash_key)
    other.merge_service_keys_device(recs, dst)
    assert other.stats()["lru_evictions"] == 0
    ctx.merge_service_keys_device(recs, dst)
    assert ctx.stats()["lru_evictions"] == gst["lru_evictions"]
    ctx.aggregate_requests([(7, b"h", b"/x", None, 2, False, b"\x0a\0\0\x01")])
    assert ctx.stats()["lru_evictions"] == gst["lru_evictions"]
    ctx.aggregate_requests([(7, b"h", b"/y", None, 2, False, b"\x0a\0\0\x01")])
    assert ctx.stats()["lru_evictions"] == gst["lru_evictions"]


def test_lru_bound_keeps_parallel_walker_when_no_eviction():
    """A window of live sessions below the capacity: the bound admits the parallel walker
    (no exact batch) even though the batch holds far more sessions than the capacity."""
    ev, lens, offs, payload = T.fragmented_trace(3000, seed=4, window=200)
    gv, gs, gst, _ = run_gpu(ev, lens, offs, payload, lru=512)
    ov, os_, ost = run_oracle(ev, lens, offs, payload, lru=512)
    assert ost["lru_evictions"] == 0 and gst["lru_exact_batches"] == 0
    assert gv == ov and gs == os_


def test_clear_and_resubmit_creates_each_service_once():
    """Aggregator::clear then the same keys again (every report interval): the table is
    emptied by one kernel and refilled by the next, on other XCDs.  Each (pid, endpoint) must
    be created exactly once per interval: equal to a fresh oracle, no duplicate keys."""
    ev, lens, offs, payload = ebd.generate_host(3, 41, 0, 700_000)
    o = O.Oracle()
    o.process(ev, lens, offs, payload)
    want = o.services()
    ctx = ebd.Context(max_events=len(ev), max_payload=payload.size, service_capacity=1 << 21)
    for k in range(4):
        if k:
            ctx.clear()
        ctx.set_seq_base(0)
        ctx.submit(ev, lens, offs, payload)
        got = ctx.services()
        keys = [(g[0], g[1]) for g in got]
        assert len(keys) == len(set(keys)), (k, len(keys) - len(set(keys)))
        assert got == want, k
        assert ctx.stats()["errors"] == 0


def cip_heavy_trace(n, frac, seed):
    """n single-buffer GETs, a fraction `frac` with an X-Forwarded-For header (v4 and v6
    clients, internal and external), one connection each."""
    rng = np.random.default_rng(seed)
    has = rng.random(n) < frac
    a = rng.integers(0, 256, size=(n, 4))
    bufs = []
    for k in range(n):
        hdr = ""
        if has[k]:
            ip = (f"{a[k, 0]}.{a[k, 1]}.{a[k, 2]}.{a[k, 3]}" if a[k, 3] % 4 else
                  f"[2001:db8:{a[k, 0]:x}::{a[k, 1]:x}]:{8000 + a[k, 2]}")
            hdr = f"X-Forwarded-For: {ip}, 10.0.0.1\r\n"
        bufs.append(f"GET /p{k % 997} HTTP/1.1\r\nHost: h{k % 53}:80\r\n{hdr}\r\n".encode())
    lens, offs, payload = T.pack(bufs)
    ev = T.events([dict(pid=3000 + k % 7, sid=k + 1, flags=ebd.FLAG_IPV4 | ebd.FLAG_UNENCRYPTED | ebd.FLAG_NEW_DATA,
                        src=bytes([11, a[k, 1], a[k, 2], 9])) for k in range(n)])
    return ev, lens, offs, payload


def test_client_ip_queue_drains_every_request():
    """k_agg_fast parses client-IP requests 256 at a time from an LDS queue; a block's last
    step must drain everything left, even more than one full wave's worth (60 % client-IP
    requests and >= 2 steps per block put > 256 in the queue at the last step)."""
    ev, lens, offs, payload = cip_heavy_trace(700_000, 0.6, 5)
    gv, gs = assert_parity(ev, lens, offs, payload)
    gv2, gs2, _, _ = run_gpu(ev, lens, offs, payload)
    assert gv2 == gv and gs2 == gs  # deterministic


def test_full_scale_config3_properties():
    """BASELINE config 3 at its full size (100 M events, generated in HBM): per-event results
    of random slices equal the oracle's (config 3 has one event per connection, so a slice
    replays on its own), the service counters add up to the per-event client classes, every
    FINISHED request is counted, and a second submission gives identical results."""
    import torch
    dev = torch.device("cuda:0")
    E = 100_000_000
    ctx = ebd.Context(max_events=E, service_capacity=1 << 26, string_arena=E * 48)
    n, size = ebd.trace_size_device(ctx, 3, 3, 0, E, align=16, with_events=True)
    ev = torch.empty(n * 36, dtype=torch.uint8, device=dev)
    ln = torch.empty(n, dtype=torch.int32, device=dev)
    of = torch.empty(n, dtype=torch.int64, device=dev)
    pay = torch.empty(size + 64, dtype=torch.uint8, device=dev)
    ebd.generate_device(ctx, 3, 3, 0, E, ev, ln, of, pay, pay.numel(), align=16)
    torch.cuda.synchronize()
    ctx.submit_device(ev, ln, of, pay, n)
    ctx.sync()
    res = ctx.results()
    st = ctx.stats()
    assert st["errors"] == 0, st
    cls = (res["info"] >> 4) & 3
    fin = res["status"] == ebd.STATUS_FINISHED
    assert st["requests"] == int(fin.sum())
    raw, _ = ctx.services_raw()
    assert int(raw["internal"].astype(np.int64).sum()) == int((cls == ebd.CLASS_INTERNAL).sum())
    assert int(raw["external"].astype(np.int64).sum()) == int((cls == ebd.CLASS_EXTERNAL).sum())
    assert len(raw) == st["services"]
    # random slices against the oracle
    rng = np.random.default_rng(7)
    off_all = of.cpu().numpy()
    pay_h = None
    for first in rng.integers(0, E - 20_000, size=8):
        first = int(first)
        hev, hl, ho, hp = ebd.generate_host(3, 3, first, 20_000)
        o = O.Oracle()
        out, blob = o.process(hev, hl, ho, hp)
        want = T.oracle_view(out, blob)
        lo = int(off_all[first])
        hi = int(off_all[first + 19_999]) + 8300
        pay_h = pay[lo:hi].cpu().numpy()
        got = T.gpu_view(res[first:first + 20_000], off_all[first:first + 20_000] - lo, pay_h, None, None)
        bad = [k for k in range(len(want)) if got[k] != want[k]]
        assert not bad, (first, [(k, got[k], want[k]) for k in bad[:3]])
    # deterministic: the same batch again (warm table) gives the same per-event results
    ctx.submit_device(ev, ln, of, pay, n)
    ctx.sync()
    res2 = ctx.results()
    assert np.array_equal(res2.view(np.uint8), res.view(np.uint8))


def _device_trace(ctx, cfg, seed, n, dev, align=1):
    import torch
    k, size = ebd.trace_size_device(ctx, cfg, seed, 0, n, align=align, with_events=True)
    ev = torch.empty(k * 36, dtype=torch.uint8, device=dev)
    ln = torch.empty(k, dtype=torch.int32, device=dev)
    of = torch.empty(k, dtype=torch.int64, device=dev)
    pay = torch.empty(size + 64, dtype=torch.uint8, device=dev)
    ebd.generate_device(ctx, cfg, seed, 0, n, ev, ln, of, pay, pay.numel(), align=align)
    torch.cuda.synchronize()
    return k, size, ev, ln, of, pay


def test_config4_device_generator_matches_host():
    import torch
    dev = torch.device("cuda:0")
    ctx = ebd.Context(max_events=16)
    n = 300_000
    k, size, ev, ln, of, pay = _device_trace(ctx, 4, 4, n, dev)
    hev, hl, ho, hp = ebd.generate_host(4, 4, 0, n)
    assert k == len(hev) and size + 16 == hp.size
    assert np.array_equal(ev.cpu().numpy(), hev.view(np.uint8).reshape(-1))
    assert np.array_equal(ln.cpu().numpy().view(np.uint32), hl)
    assert np.array_equal(of.cpu().numpy().view(np.uint64), ho)
    assert np.array_equal(pay[:size].cpu().numpy(), hp[:size])


@pytest.mark.parametrize("batches", [1, 4])
def test_config4_fragmented_keepalive_parity_1m(batches):
    """Config 4 at 1.2 M events (device-generated): every request arrives in 2-4 pieces, so
    nearly every event takes the session path, with sessions carried across batches."""
    import torch
    dev = torch.device("cuda:0")
    n = 1_200_000
    ctx = ebd.Context(max_events=n)
    k, size, ev, ln, of, pay = _device_trace(ctx, 4, 4, n, dev)
    hev = ev.cpu().numpy().view(ebd.EVENT_DTYPE)
    hl = ln.cpu().numpy().view(np.uint32)
    ho = of.cpu().numpy().view(np.uint64)
    hp = pay.cpu().numpy()
    views = []
    bounds = np.linspace(0, k, batches + 1).astype(int)
    for a, z in zip(bounds[:-1], bounds[1:]):
        ctx.submit_device(ev[a * 36:], ln[a:], of[a:], pay, int(z - a))
        ctx.sync()
        sreq, sstr = ctx.session_requests()
        views += T.gpu_view(ctx.results(), ho[a:z], hp, sreq, sstr)
    st = ctx.stats()
    assert st["errors"] == 0, st
    ov, os_, ost = run_oracle(hev, hl, ho, hp)
    bad = [i for i in range(k) if views[i] != ov[i]]
    assert not bad, [(i, views[i], ov[i]) for i in bad[:5]]
    assert ctx.services() == os_
    assert st["kernel_deletes"] == ost["kernel_deletes"] and st["live_sessions"] == ost["lru_size"]
    assert st["lru_evictions"] == 0 and st["session_events"] > 0.9 * k
