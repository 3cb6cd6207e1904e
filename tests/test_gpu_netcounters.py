"""GPU: network counters (EBD_CFG_NETWORK_COUNTERS; Aggregator.cpp:89-106, 136-153,
182-209) and the service report (Discovery.cpp:60-71, Json.h:32-71) through the C ABI,
against the oracle on the same inputs.

Compared bit-exactly: every service with its three map sizes, every live map entry
(service, map, prefix, time last seen), and the report text object by object (the reference
prints its unordered_map's order, so objects are compared as a sorted list)."""
import json
import os

import numpy as np
import pytest

import ebd
import oracle_py as O
import traces as T

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MIN = 60 * 10**9
T0 = 10**12  # a steady-clock origin (0 means "read the clock" to ebd_set_clock)


def gpu_nets(ctx):
    """sorted [(pid, endpoint, kind, prefix hex (6 bytes), time)] like Oracle.nets()."""
    recs, blob = ctx.services_raw()
    s = blob.tobytes()
    by_key = {(int(r["key_lo"]), int(r["key_hi"])): (int(r["pid"]), s[int(r["endpoint_off"]):int(r["endpoint_off"])
                                                                       + int(r["endpoint_len"])]) for r in recs}
    out = []
    for e in ctx.networks_raw():
        pid, ep = by_key[(int(e["key_lo"]), int(e["key_hi"]))]
        out.append((pid, ep, int(e["kind"]), bytes(e["prefix"]).hex(), int(e["time_ns"])))
    return sorted(out)


def json_objects(text):
    """The report's service objects as text, split at the top level of the array."""
    if not text:
        return []
    assert text.startswith(b'{"service":[') and text.endswith(b"]}\n")
    body = text[len(b'{"service":['):-3]
    objs, depth, start, in_str, esc = [], 0, 0, False, False
    for k, ch in enumerate(body):
        c = chr(ch)
        if in_str:
            esc, in_str = (False, in_str) if esc else (c == "\\", c != '"')
            continue
        if c == '"':
            in_str = True
        elif c == "{":
            depth += 1
        elif c == "}":
            depth -= 1
            if depth == 0:
                objs.append(body[start:k + 1])
                start = k + 2  # past the ','
    json.loads(text)  # well-formed
    return sorted(objs)


def http(host, url, cip):
    return (f"GET {url} HTTP/1.1\r\nHost: {host}\r\nX-Forwarded-For: {cip}\r\n\r\n").encode()


def test_reference_network_counter_scenario_on_gpu(vectors):
    """AggregatorTest.cpp:174-285 as HTTP requests: 10 requests at one time point, cleaning
    at +59 min keeps every map, clear() keeps both services with zeroed counters; cleaning at
    +60 min erases the maps and clear() drops the services."""
    nc = vectors["agg_netcounters"]
    rows, bufs = [], []
    for k, r in enumerate(nc["requests"]):
        rows.append(dict(pid=r["pid"], sid=k + 1, flags=r["flags"] | ebd.FLAG_NEW_DATA))
        bufs.append(http(r["host"], r["url"], r["client_ip"]))
    lens, offs, payload = T.pack(bufs)
    ev = T.events(rows)
    ctx = ebd.Context(max_events=len(ev), max_payload=payload.size, network_counters=True, net_capacity=1 << 12)
    ctx.set_clock(T0)
    ctx.submit(ev, lens, offs, payload)
    want = [(e["pid"], e["endpoint"].encode(), e["domain"].encode(), e["scheme"].encode(), e["internal"],
             e["external"], 2, 3, 2) for e in nc["expected"]]
    assert ctx.services(with_nets=True) == want
    nets = gpu_nets(ctx)
    for pid in (100, 200):
        got = {k: sorted(p for (pp, _, kk, p, t) in nets if pp == pid and kk == k) for k in (1, 2, 3)}
        assert got[1] == sorted(x.ljust(12, "0") for x in nc["nets_v4_16"])
        assert got[2] == sorted(x.ljust(12, "0") for x in nc["nets_v4_24"])
        assert got[3] == sorted(nc["nets_v6"])
    assert all(t == T0 for (_, _, _, _, t) in nets)
    o = O.Oracle(network_counters=True)
    o.set_time(T0)
    o.process(ev, lens, offs, payload)
    assert json_objects(ctx.report_json()) == json_objects(o.services_json())
    ctx.network_counters_cleaning(T0 + 59 * MIN)
    ctx.clear()
    got = ctx.services(with_nets=True)
    assert [g[:4] for g in got] == [w[:4] for w in want]
    assert all(g[4:] == (0, 0, 2, 3, 2) for g in got)
    ctx.network_counters_cleaning(T0 + 60 * MIN)
    assert all(g[6:] == (0, 0, 0) for g in ctx.services(with_nets=True))
    ctx.clear()
    assert ctx.services(with_nets=True) == []
    assert ctx.report_json() == b""
    assert ctx.stats()["errors"] == 0


def run_pair(trace_batches, clocks, cleanings=(), clears=(), v4=(), v6=()):
    """Submits each batch at its clock on the GPU and the oracle; after batch k, runs the
    cleaning at cleanings[k] (if any) and the clear (if k in clears); compares everything
    after every batch."""
    n_max = max(len(b[0]) for b in trace_batches)
    pay_max = max(b[3].size for b in trace_batches)
    ctx = ebd.Context(max_events=n_max, max_payload=pay_max, network_counters=True, net_capacity=1 << 20)
    o = O.Oracle(network_counters=True, v4_ifaces=list(v4), v6_ifaces=list(v6))
    if v4 or v6:
        ctx.set_interfaces(v4, v6)
    cleanings = dict(cleanings)
    for k, ((ev, lens, offs, payload), now) in enumerate(zip(trace_batches, clocks)):
        ctx.set_clock(now)
        o.set_time(now)
        ctx.submit(ev, lens, offs, payload)
        o.process(ev, lens, offs, payload)
        if k in cleanings:
            ctx.network_counters_cleaning(cleanings[k])
            o.network_counters_cleaning(cleanings[k])
        if k in clears:
            ctx.clear()
            o.clear()
        assert ctx.stats()["errors"] == 0, ctx.stats()
        assert ctx.services(with_nets=True) == o.services_nets(), k
        assert gpu_nets(ctx) == o.nets(), k
        assert json_objects(ctx.report_json()) == json_objects(o.services_json()), k
    return ctx, o


def test_config3_network_counters_batches_cleaning_clear():
    """Config-3 requests (client-IP headers, v4/v6 sources, ~1 % invalid) in three batches
    30 min apart: maps last seen in batch 1 expire at the cleaning after batch 3, the clear
    after batch 2 keeps exactly the services with a non-empty map."""
    n = 60_000
    batches = []
    for k in range(3):
        batches.append(ebd.generate_host(3, 3, k * n // 2, n))  # overlapping slices: services recur
    clocks = [T0, T0 + 30 * MIN, T0 + 60 * MIN]
    ctx, o = run_pair(batches, clocks, cleanings={2: T0 + 60 * MIN}, clears={1})
    assert sum(r[8] for r in o.services_nets()) > 0 and sum(r[6] for r in o.services_nets()) > 0


def test_session_path_network_counters():
    """Requests finished by the session path (fragmented keep-alive connections) feed the
    maps too (emit_session_request)."""
    ev, lens, offs, payload = T.fragmented_trace(1500, seed=4, window=256)
    half = len(ev) // 2
    batches = [(ev[:half], lens[:half], offs[:half], payload), (ev[half:], lens[half:], offs[half:], payload)]
    run_pair(batches, [T0, T0 + MIN], cleanings={1: T0 + 61 * MIN})


def test_network_counters_with_interfaces():
    """Internal clients (interface subnets) never enter the maps."""
    ev, lens, offs, payload = ebd.generate_host(3, 7, 0, 40_000)
    v4 = [(bytes([10, 0, 0, 0]), bytes([255, 0, 0, 0])), (bytes([172, 0, 0, 0]), bytes([255, 0, 0, 0]))]
    v6 = [(bytes([0x20, 0x01] + [0] * 14), bytes([0xff, 0xff] + [0] * 14))]
    run_pair([(ev, lens, offs, payload)], [T0], v4=v4, v6=v6)


def test_report_json_config3_matches_oracle_without_network_counters():
    ev, lens, offs, payload = ebd.generate_host(3, 11, 0, 50_000)
    ctx = ebd.Context(max_events=len(ev), max_payload=payload.size)
    ctx.submit(ev, lens, offs, payload)
    o = O.Oracle()
    o.process(ev, lens, offs, payload)
    text = ctx.report_json()
    assert json_objects(text) == json_objects(o.services_json())
    assert len(json_objects(text)) == len(o.services())


def test_v6_dictionary_does_not_fill_across_cleanings_and_clears():
    """The IPv6 /48 prefix dictionary only holds prefixes of live map entries:
    far more distinct external v6 prefixes than net_capacity, cycled through batches an hour
    apart with cleanings (which rebuild the half-full tables) and clears, never fill it, and
    every batch's maps equal the oracle's."""
    cap = 1 << 10
    ctx = ebd.Context(max_events=600, max_payload=1 << 16, network_counters=True, net_capacity=cap)
    o = O.Oracle(network_counters=True)
    for k in range(12):
        bufs, rows = [], []
        for j in range(300):  # 300 fresh /48 prefixes per batch, 12 x 300 > 1024 in all
            bufs.append(http("h", f"/p{j % 3}", f"2001:db8:{k:x}{j:03x}::1"))
            rows.append(dict(pid=100, sid=k * 1000 + j + 1, flags=ebd.FLAG_IPV6 | ebd.FLAG_UNENCRYPTED | ebd.FLAG_NEW_DATA))
        lens, offs, payload = T.pack(bufs)
        ev = T.events(rows)
        now = T0 + k * 61 * MIN
        ctx.set_clock(now)
        o.set_time(now)
        ctx.submit(ev, lens, offs, payload)
        o.process(ev, lens, offs, payload)
        assert ctx.stats()["errors"] == 0, (k, ctx.stats())
        assert gpu_nets(ctx) == o.nets(), k
        assert ctx.services(with_nets=True) == o.services_nets(), k
        ctx.network_counters_cleaning(now + 60 * MIN)  # this batch's prefixes expire
        o.network_counters_cleaning(now + 60 * MIN)
        if k % 4 == 3:
            ctx.clear()
            o.clear()
        assert gpu_nets(ctx) == o.nets(), k


@pytest.mark.parametrize("world", [2, 4])
def test_config5_network_maps_merge_across_shards(world):
    """Config 5 with network counters: each connection shard on its own context with its
    own clock (shard r at T0 + r min), services and network-map entries exported by owner,
    merged into owner contexts (ebd_merge_services_device, then ebd_merge_networks_device).
    The owners' services with their map sizes equal the oracle's over the whole trace, and
    every map entry is the union of the shards' entries with the latest last-seen time."""
    import torch
    from ebd import shard
    dev = torch.device("cuda:0")
    N = 200_000
    ev_all, lens_all, offs_all, pay_all = ebd.generate_host(5, 5, 0, N, align=16)
    segs = [[] for _ in range(world)]
    want_nets = {}
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
        assert ctx.stats()["errors"] == 0
        recs, strs, counts, scounts = ctx.export_services_device(world, dev)
        shard.map_wire_first(recs, lambda f: gi[f])
        nets, ncounts = shard.group_by_owner(ctx.networks_device(dev), shard.NET_REC_BYTES, world)
        ro = np.concatenate([[0], np.cumsum(counts.astype(np.int64))]) * ebd.WIRE_DTYPE.itemsize
        so = np.concatenate([[0], np.cumsum(scounts.astype(np.int64))])
        no = np.concatenate([[0], np.cumsum(ncounts)]) * shard.NET_REC_BYTES
        for w in range(world):
            segs[w].append((recs[ro[w]:ro[w + 1]], strs[so[w]:so[w + 1]], nets[no[w]:no[w + 1]]))
        # the shard's own entries, from the oracle over the shard at the shard's clock
        idx = gi.cpu().numpy()
        lens_s, offs_s, pay_s = T.pack([pay_all[offs_all[i]:offs_all[i] + lens_all[i]].tobytes() for i in idx])
        o_r = O.Oracle(network_counters=True)
        o_r.set_time(T0 + r * MIN)
        o_r.process(ev_all[idx], lens_s, offs_s, pay_s)
        for (pid, ep, kind, pfx, t) in o_r.nets():
            want_nets[(pid, ep, kind, pfx)] = max(t, want_nets.get((pid, ep, kind, pfx), 0))
        ctx.close()
    got_svc, got_nets = [], []
    for parts in segs:
        m = ebd.Context(max_events=1024, max_payload=64, hash_key=ebd.TEST_HASH_KEY, network_counters=True,
                        net_capacity=1 << 20)
        m.merge_services_device(torch.cat([r for r, _, _ in parts]),
                                torch.cat([s for _, s, _ in parts] + [torch.zeros(shard.STR_SLACK, dtype=torch.uint8,
                                                                                  device=dev)]))
        assert m.stats()["errors"] == 0, ("services", m.stats())
        m.merge_networks_device(torch.cat([n for _, _, n in parts]))
        assert m.stats()["errors"] == 0, m.stats()
        got_svc += m.services(with_nets=True)
        got_nets += gpu_nets(m)
        m.close()
    o = O.Oracle(network_counters=True)
    o.set_time(T0)
    o.process(ev_all, lens_all, offs_all, pay_all)
    assert sorted(got_svc) == o.services_nets()
    assert sorted(got_nets) == sorted((pid, ep, kind, pfx, t) for (pid, ep, kind, pfx), t in want_nets.items())
    assert len(got_nets) == len(o.nets())


@pytest.mark.parametrize("trace", ["config3", "fragmented"])
def test_per_event_clock_matches_per_request_time(trace):
    """ebd_set_event_clock: every request takes the clock reading of the event that finishes
    it, as the reference reads getCurrentTime per request (Aggregator.cpp:162,165); the
    oracle is fed one event at a time at that event's time.  The readings span 1.7 hours,
    so the cleaning at +1.5 h erases exactly the entries last seen in the first half hour."""
    import torch
    if trace == "config3":
        ev, lens, offs, payload = ebd.generate_host(3, 3, 0, 4000)
    else:
        ev, lens, offs, payload = T.fragmented_trace(300, seed=12)
    n = len(ev)
    times = (T0 + np.arange(n, dtype=np.int64) * (6000 * 10**9 // n)).astype(np.int64)
    ctx = ebd.Context(max_events=n, max_payload=payload.size, network_counters=True, net_capacity=1 << 16)
    ctx.set_clock(T0)
    ctx.set_event_clock(torch.from_numpy(times).to("cuda:0"))
    ctx.submit(ev, lens, offs, payload)
    ctx.sync()
    o = O.Oracle(network_counters=True)
    for i in range(n):
        o.set_time(int(times[i]))
        o.process(ev[i:i + 1], lens[i:i + 1], offs[i:i + 1], payload)
    assert ctx.stats()["errors"] == 0
    assert ctx.services(with_nets=True) == o.services_nets()
    assert gpu_nets(ctx) == o.nets()
    assert len({t for (_, _, _, _, t) in o.nets()}) > 100  # the readings differ per request
    ctx.network_counters_cleaning(T0 + 90 * MIN)
    o.network_counters_cleaning(T0 + 90 * MIN)
    assert ctx.services(with_nets=True) == o.services_nets()
    assert gpu_nets(ctx) == o.nets()
    assert json_objects(ctx.report_json()) == json_objects(o.services_json())
