"""Config 4: config-3 requests cut into 2-4 recv() events, 1-8 keep-alive
requests per connection, DATA_END, at most 4096 connections open at once (ebd_gen.h
conn4_*).  CPU checks of the generator's shape, and of the oracle over it."""
import numpy as np

import ebd
import oracle_py as O


def test_config4_shape_and_prefix():
    ev, lens, offs, payload = ebd.generate_host(4, 4, 0, 60_000)
    ev2, lens2, offs2, payload2 = ebd.generate_host(4, 4, 0, 30_000)
    assert np.array_equal(ev[:30_000], ev2) and np.array_equal(lens[:30_000], lens2)  # a prefix of the longer trace
    for i in range(30_000):
        if lens2[i] != ebd.NO_BUFFER:
            a, b = int(offs[i]), int(offs2[i])
            assert payload[a:a + lens[i]].tobytes() == payload2[b:b + lens2[i]].tobytes()
    data = (ev["flags"] & ebd.FLAG_NEW_DATA) != 0
    end = (ev["flags"] & ebd.FLAG_DATA_END) != 0
    assert np.all(data ^ end)
    assert np.all(lens[end] == ebd.NO_BUFFER) and np.all(lens[data] <= 8192)
    # per connection: bufferSeq 1, 2, ... over its data events, DATA_END last, requests whole
    sid = ev["sessionID"]
    order = np.argsort(sid, kind="stable")
    bounds = np.flatnonzero(np.diff(sid[order])) + 1
    conns = np.split(order, bounds)
    assert len(conns) > 3000
    for k in conns[:400]:
        d = k[data[k]]
        assert list(ev["bufferSeq"][d]) == list(range(1, len(d) + 1))
        if end[k].any():
            assert end[k[-1]] and end[k].sum() == 1
        stream = b"".join(payload[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes() for i in d)
        starts = [j for j in range(len(stream)) if stream.startswith((b"GET /", b"POST /"), j)]
        assert starts and starts[0] == 0
        first = payload[int(offs[d[0]]):int(offs[d[0]]) + int(lens[d[0]])].tobytes()
        assert len(first) >= 16 and first.startswith((b"GET /", b"POST /"))
    # consecutive events of a connection are kSlots4 = 4096 positions apart (one per round)
    for k in conns[:200]:
        assert np.all(np.diff(k) == 4096)


def test_config4_oracle_sessions_stay_below_lru():
    ev, lens, offs, payload = ebd.generate_host(4, 4, 0, 120_000)
    o = O.Oracle()
    out, _ = o.process(ev, lens, offs, payload)
    st = o.stats()
    assert st["lru_evictions"] == 0 and st["lru_size"] <= 4096
    assert (out["status"] == 2).sum() > 30_000  # requests finished, mostly through saved sessions
    assert (out["kind"] == 2).sum() > (out["kind"] == 1).sum()
