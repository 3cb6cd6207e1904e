"""GPU: the ingest pipeline (ebd_stage_batch / ebd_submit_staged / ebd_fetch_results_async,
SURVEY.md 8(f) row 1) gives the same per-event results and the same services as one
blocking ebd_submit_batch per batch, with pinned and with pageable sources, including
sessions carried from batch to batch (Discovery.cpp:73-198 across poll cycles)."""
import numpy as np
import pytest

import ebd
import oracle_py as O
import traces as T

pytestmark = pytest.mark.gpu


def comparable(res):
    """(status, consumed, info, spans) per event; a session-path request's index into its
    batch's request array depends on the order of the atomics, so it is left out."""
    out = []
    for r in res:
        t = (int(r["status"]), int(r["consumed"]), int(r["info"]))
        if not (r["info"] & ebd.INFO_SESSION):
            t += tuple(int(r[f]) for f in ("url_off", "url_len", "host_off", "host_len", "cip_off", "cip_len"))
        out.append(t)
    return out


def split(trace, k):
    ev, lens, offs, payload = trace
    b = np.linspace(0, len(ev), k + 1).astype(int)
    return [(ev[x:y], lens[x:y], offs[x:y], payload) for x, y in zip(b[:-1], b[1:])]


@pytest.mark.parametrize("pinned", [True, False])
def test_pipeline_equals_blocking_submits(pinned):
    trace = T.fragmented_trace(1200, seed=31, window=300)  # sessions span batch boundaries
    parts = split(trace, 6)
    n_max = max(len(p[0]) for p in parts)
    seq = ebd.Context(max_events=n_max, max_payload=trace[3].size)
    want = []
    for p in parts:
        seq.submit(*p)
        want.append(comparable(seq.results()))
    pipe = ebd.Context(max_events=n_max, max_payload=trace[3].size)
    if pinned:  # the producer writes batches into pinned memory (ebd_host_alloc)
        staged = []
        for ev, ln, of, pay in parts:
            h = (pipe.pinned_empty(len(ev), ebd.EVENT_DTYPE), pipe.pinned_empty(len(ln), np.uint32),
                 pipe.pinned_empty(len(of), np.uint64), pipe.pinned_empty(pay.size, np.uint8))
            h[0][:], h[1][:], h[2][:], h[3][:] = ev, ln, of, pay
            staged.append(h)
        parts = staged
    outs = [pipe.pinned_empty(n_max, ebd.RESULT_DTYPE) for _ in parts]
    tickets = [pipe.stage(*parts[0])]
    for k in range(len(parts)):
        if k + 1 < len(parts):
            tickets.append(pipe.stage(*parts[k + 1]))
        pipe.submit_staged(tickets[k])
        pipe.results_async(outs[k])
    pipe.sync()
    for k, p in enumerate(parts):
        assert comparable(outs[k][:len(p[0])]) == want[k], k
    assert pipe.services() == seq.services()
    st, sq = pipe.stats(), seq.stats()
    assert st["errors"] == 0
    for f in ("requests", "session_events", "kernel_deletes", "live_sessions", "services"):
        assert st[f] == sq[f], f
    # and both equal the oracle over the whole trace
    o = O.Oracle()
    o.process(*trace)
    assert pipe.services() == o.services()


def test_stage_limit_and_bad_ticket():
    ev, lens, offs, payload = ebd.generate_host(3, 3, 0, 1000)
    ctx = ebd.Context(max_events=1000, max_payload=payload.size)
    t1 = ctx.stage(ev, lens, offs, payload)
    t2 = ctx.stage(ev, lens, offs, payload)
    with pytest.raises(ebd.EbdError):
        ctx.stage(ev, lens, offs, payload)  # two staged, none submitted: -EBUSY
    with pytest.raises(ebd.EbdError):
        ctx.submit_staged(t2 + 100)
    ctx.submit_staged(t1)
    ctx.submit_staged(t2)
    ctx.sync()
    o = O.Oracle()
    o.process(ev, lens, offs, payload)
    o.process(ev, lens, offs, payload)
    assert ctx.services() == o.services()


def test_device_submit_returns_before_aggregation_finishes():
    """ebd_submit_batch_device queues the aggregation and returns; ebd_sync completes it and
    the results equal the blocking host submit's."""
    import torch
    ev, lens, offs, payload = ebd.generate_host(3, 5, 0, 200_000)
    dev = torch.device("cuda:0")
    ctx = ebd.Context(max_events=len(ev))
    t = [torch.from_numpy(np.ascontiguousarray(x).view(np.uint8)).to(dev) for x in (ev, lens, offs, payload)]
    for k in range(3):
        ctx.set_seq_base(k * len(ev))
        ctx.submit_device(t[0], t[1], t[2], t[3], len(ev))
    ctx.sync()
    ref = ebd.Context(max_events=len(ev), max_payload=payload.size)
    for k in range(3):
        ref.set_seq_base(k * len(ev))
        ref.submit(ev, lens, offs, payload)
    assert ctx.services() == ref.services()
    assert comparable(ctx.results()) == comparable(ref.results())


def test_tickets_submitted_out_of_order():
    """Stage A, stage B, submit B, then stage C: the slot A still holds is skipped and C goes
    into the free one; submitting A and C afterwards gives every batch's services."""
    parts = [ebd.generate_host(3, 3, k * 1000, 1000) for k in range(3)]
    ctx = ebd.Context(max_events=1000, max_payload=max(p[3].size for p in parts))
    ta = ctx.stage(*parts[0])
    tb = ctx.stage(*parts[1])
    ctx.submit_staged(tb)
    tc = ctx.stage(*parts[2])
    ctx.submit_staged(ta)
    ctx.submit_staged(tc)
    ctx.sync()
    o = O.Oracle()
    for k in (1, 0, 2):
        o.process(*parts[k])
    assert ctx.stats()["errors"] == 0
    got = [(g[0], g[1], g[4], g[5]) for g in ctx.services()]
    want = [(w[0], w[1], w[4], w[5]) for w in o.services()]  # counters; first arrival is batch order
    assert got == want
