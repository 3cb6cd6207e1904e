"""Config 4 at the size it is benched at (bench.py --config 4): 100 M requests
(config-3 content, seed 4) cut into 2-4 recv() events each, 1-8 keep-alive requests per
connection then DATA_END, 4096 connections interleaved: ~322 M events submitted as four poll
cycles of 81 M events, sessions carried from cycle to cycle (Discovery.cpp:123-159,
HttpRequestParser.cpp:85-106).  The oracle cannot replay 322 M events in a test, so the full run
is checked through properties, and windows of it against the oracle:

  * every cycle: the requests counted equal its FINISHED results, and no error is raised;
  * the service counters add up to the per-request client classes over all cycles, and the
    service count matches the table;
  * the LRU never evicts (at most 4096 connections are open at a time);
  * random windows of positions: the connections that start and end inside a window are
    replayed by the oracle on their own (connections are independent while nothing is
    evicted) and every one of their events equals the GPU's result, across cycle boundaries;
  * a second run on a fresh context gives identical per-event results and services.
"""
import hashlib

import numpy as np
import pytest

import ebd
import oracle_py as O
import traces as T

pytestmark = pytest.mark.gpu

CYCLE = 81_000_000
EVENTS = 322_000_000


def _generate(dev):
    import torch
    ctx = ebd.Context(max_events=16)
    n, size = ebd.trace_size_device(ctx, 4, 4, 0, EVENTS, align=16, with_events=True)
    ev = torch.empty(n * 36, dtype=torch.uint8, device=dev)
    ln = torch.empty(n, dtype=torch.int32, device=dev)
    of = torch.empty(n, dtype=torch.int64, device=dev)
    pay = torch.empty(size + 64, dtype=torch.uint8, device=dev)
    ebd.generate_device(ctx, 4, 4, 0, EVENTS, ev, ln, of, pay, pay.numel(), align=16)
    torch.cuda.synchronize()
    ctx.close()
    return n, ev, ln, of, pay


def _run(n, ev, ln, of, pay, keep=None):
    """The four poll cycles on a fresh context.  keep(cycle, a, z, res, sreq, sstr) sees each
    cycle's outputs; returns (per-cycle result digests, services, stats, per-cycle checks)."""
    reqs = n / 3.2
    ctx = ebd.Context(max_events=CYCLE, service_capacity=1 << 26, string_arena=int(reqs * 48),
                      hash_key=ebd.TEST_HASH_KEY)
    digests, fin_total, cls_int, cls_ext = [], 0, 0, 0
    prev_req = 0
    cuts = list(range(0, n, CYCLE)) + [n]
    for c, (a, z) in enumerate(zip(cuts[:-1], cuts[1:])):
        ctx.submit_device(ev[a * 36:], ln[a:], of[a:], pay, z - a)
        ctx.sync()
        res = ctx.results()
        st = ctx.stats()
        assert st["errors"] == 0, (c, st)
        fin = res["status"] == ebd.STATUS_FINISHED
        cls = (res["info"] >> 4) & 3
        assert st["requests"] - prev_req == int(fin.sum()), c
        prev_req = st["requests"]
        fin_total += int(fin.sum())
        cls_int += int((fin & (cls == ebd.CLASS_INTERNAL)).sum())
        cls_ext += int((fin & (cls == ebd.CLASS_EXTERNAL)).sum())
        # a session request's index into the cycle's request list is handed out by an atomic
        # (its order is not part of the result): digest everything else
        det = res.copy()
        sess = (det["info"] & ebd.INFO_SESSION) != 0
        for f in ("url_off", "url_len"):
            det[f][sess] = 0
        digests.append(hashlib.sha256(det.tobytes()).hexdigest())
        if keep is not None:
            sreq, sstr = ctx.session_requests()
            keep(c, a, z, res, sreq, sstr)
    st = ctx.stats()
    raw, _ = ctx.services_raw()
    assert len(raw) == st["services"]
    assert int(raw["internal"].astype(np.int64).sum()) == cls_int
    assert int(raw["external"].astype(np.int64).sum()) == cls_ext
    assert st["requests"] == fin_total
    # the table as a digest (some 30 M services): records sorted by key, every field but the
    # arena offsets (the key is a PRF of pid + endpoint under the fixed test key)
    r = np.sort(raw, order=["key_lo", "key_hi"])
    fields = [r[f].astype(np.uint64) for f in ("key_lo", "key_hi", "pid", "internal", "external", "https", "first_seq",
                                                 "endpoint_len", "domain_off", "domain_len", "host_len")]
    svcs = hashlib.sha256(np.stack(fields).tobytes()).hexdigest()
    ctx.close()
    return digests, svcs, st


def _complete_connections(hev):
    """Positions (in window order) of the events of connections that start and end inside the
    window: the first data event (bufferSeq 1) and the DATA_END event both lie in it."""
    sid = hev["sessionID"]
    starts = set(sid[(hev["bufferSeq"] == 1) & ((hev["flags"] & ebd.FLAG_NEW_DATA) != 0)].tolist())
    ends = set(sid[(hev["flags"] & ebd.FLAG_DATA_END) != 0].tolist())
    keep = np.fromiter((s in starts and s in ends for s in sid.tolist()), bool, count=len(sid))
    return np.flatnonzero(keep)


@pytest.mark.timeout(900)
def test_full_scale_config4_properties():
    import torch
    dev = torch.device("cuda:0")
    n, ev, ln, of, pay = _generate(dev)
    assert n > 300_000_000
    rng = np.random.default_rng(11)
    W = 200_000
    # windows that straddle each cycle boundary, and two inside cycles
    firsts = [CYCLE - W // 2, 2 * CYCLE - W // 3, 3 * CYCLE - W // 4] + [int(x) for x in rng.integers(0, n - W, size=2)]
    windows = []
    for a in firsts:
        hev = ev[a * 36:(a + W) * 36].cpu().numpy().view(ebd.EVENT_DTYPE)
        ow = of[a:a + W].cpu().numpy().view(np.uint64)
        lw = ln[a:a + W].cpu().numpy().view(np.uint32)
        pos = _complete_connections(hev)
        assert len(pos) > W // 4
        lo, hi = int(ow[0]), int(ow[-1]) + 8300
        windows.append(dict(a=a, pos=pos + a, hev=hev[pos], lens=lw[pos], offs=ow[pos] - np.uint64(lo),
                            pay=pay[lo:hi].cpu().numpy(), views={}))

    def keep(c, a, z, res, sreq, sstr):
        for w in windows:
            k = np.flatnonzero((w["pos"] >= a) & (w["pos"] < z))
            if len(k) == 0:
                continue
            got = T.gpu_view(res[w["pos"][k] - a], w["offs"][k], w["pay"], sreq, sstr)
            w["views"].update(zip(w["pos"][k].tolist(), got))

    d1, s1, st1 = _run(n, ev, ln, of, pay, keep)
    assert st1["lru_evictions"] == 0 and 0 < st1["live_sessions"] <= 4096  # the trace ends mid-connection
    assert st1["session_events"] > 0.9 * n
    for w in windows:
        o = O.Oracle()
        out, blob = o.process(w["hev"], w["lens"], w["offs"], w["pay"])
        want = T.oracle_view(out, blob)
        got = [w["views"][p] for p in w["pos"].tolist()]
        bad = [k for k in range(len(want)) if got[k] != want[k]]
        assert not bad, (w["a"], [(int(w["pos"][k]), got[k], want[k]) for k in bad[:3]])
    d2, s2, st2 = _run(n, ev, ln, of, pay)
    assert d1 == d2
    assert s1 == s2
    assert st2["requests"] == st1["requests"] and st2["kernel_deletes"] == st1["kernel_deletes"]
    assert st2["live_sessions"] == st1["live_sessions"]
