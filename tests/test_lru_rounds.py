"""The exact LRU in rounds (ebd_kernels.hip k_lru_*, ebd_api.hip run_lru_rounds), restated in
Python and checked against a plain sequential LRU (LRUCache.h:50-89 as Discovery.cpp:92-198
drives it) on random session traces.  The GPU path itself is checked against the oracle by
test_gpu_parity.py::test_lru_eviction_exact; this pins the algorithm: the size scan, the
marker merge, the victim flags and the convergence of the rounds to the sequential result.

Session model (what the walker's parse decides, reduced to the LRU): an event of a saved
session touches it (find) and keeps it (ACCESS) or drops it (ERASE: INVALID); an event of an
unsaved session inserts it (saveSession after an UNFINISHED fresh parse) or does nothing;
a close (DATA_END) erases a saved session; an event without a buffer does nothing.
"""
from collections import OrderedDict

import numpy as np
import pytest

NONE, INSERT, ERASE, ACCESS = 0, 1, 2, 3


def make_trace(rng, n_sessions, n_events, n_carried):
    """Events (session, has_buffer, op if saved, op if not saved, close) in time order, and the
    carried sessions least recently used first."""
    ev = []
    for _ in range(n_events):
        s = int(rng.integers(0, n_sessions))
        buf = rng.random() < 0.95
        ex_op = ERASE if rng.random() < 0.05 else ACCESS
        new_op = INSERT if rng.random() < 0.6 else NONE
        close = rng.random() < 0.08
        ev.append((s, buf, ex_op, new_op, close))
    carried = [int(x) for x in rng.permutation(n_sessions)[:n_carried]]
    return ev, carried


def sequential(ev, carried, cap):
    """Discovery's loop with a real LRU: per-event operation, evictions, sessions left."""
    lru = OrderedDict((s, True) for s in carried)  # first = least recently used
    ops, evicted = [], 0
    for (s, buf, ex_op, new_op, close) in ev:
        op = NONE
        if buf:
            if s in lru:
                lru.move_to_end(s)  # find touches
                op = ex_op
                if op == ERASE:
                    del lru[s]
            elif new_op == INSERT and not close:
                if len(lru) >= cap:
                    lru.popitem(last=False)
                    evicted += 1
                lru[s] = True
                op = INSERT
        if close and s in lru:
            del lru[s]
            op = ERASE
        ops.append(op)
    return ops, evicted, list(lru)


def walk(ev, carried, flags, tail, cflag):
    """The dry walk in a world of evictions: flags[t] = the event's session was evicted before
    it; tail[s] / cflag[s]: evicted after its last event.  Per-event operations, and the
    sessions saved at the end."""
    live = {s: True for s in carried}
    ops = []
    for t, (s, buf, ex_op, new_op, close) in enumerate(ev):
        if flags[t]:
            live.pop(s, None)
        op = NONE
        if buf:
            if s in live:
                op = ex_op
                if op == ERASE:
                    del live[s]
            elif new_op == INSERT and not close:
                live[s] = True
                op = INSERT
        if close and s in live:
            del live[s]
            op = ERASE
        ops.append(op)
    left = [s for s in live if not tail.get(s) and not cflag.get(s)]
    return ops, left


def derive(ev, carried, ops, cap, tend=None):
    """k_lru_static / scan / compact / greedy / victims: the evictions the operations imply
    (those before tend, when given), as flags."""
    n = len(ev)
    # marker ends: the session's next find (an event with a buffer, or a close), whatever it
    # did in this world (a find of an evicted session misses and does nothing)
    nxt, last = [None] * n, {}
    for t in range(n - 1, -1, -1):
        s, buf, _, _, close = ev[t]
        nxt[t] = last.get(s)
        if buf or close:
            last[s] = t
    first_op = {s: last.get(s) for s in carried}
    # the size scan: min(cap, L + 1) per insert, L - 1 per erase (composed maps)
    fns = [(cap, 1) if o == INSERT else (1 << 60, -1) if o == ERASE else (1 << 60, 0) for o in ops]
    L = len(carried)
    evictions = []
    for t, (a, b) in enumerate(fns):
        if ops[t] == INSERT and L >= cap:
            evictions.append(t)
        L = min(a, L + b)
    # markers, carried ones (least recently used first) before the batch's
    markers = [(-1, first_op[s], s) for s in carried]
    markers += [(t, nxt[t], ev[t][0]) for t in range(n) if ops[t] in (INSERT, ACCESS)]
    flags, tail, cflag = [False] * n, {}, {}
    q = 0
    for t in evictions:
        if tend is not None and t >= tend:
            break
        while q < len(markers) and not (markers[q][1] is None or markers[q][1] > t):
            q += 1
        assert q < len(markers) and markers[q][0] < t
        pos, end, s = markers[q]
        q += 1
        if end is not None:
            flags[end] = True
        elif pos < 0:
            cflag[s] = True
        else:
            tail[s] = True
    return flags, tail, cflag, len(evictions)


def rounds(ev, carried, cap, max_rounds=500):
    flags, tail, cflag = [False] * len(ev), {}, {}
    for r in range(1, max_rounds + 1):
        ops, left = walk(ev, carried, flags, tail, cflag)
        nf, nt, nc, nev = derive(ev, carried, ops, cap)
        if nf == flags and nt == tail and nc == cflag:
            return ops, nev, left, r
        flags, tail, cflag = nf, nt, nc
    raise AssertionError("rounds did not settle")


def rounds_windowed(ev, carried, cap, window, max_rounds=20000):
    """run_lru_rounds' schedule: events before the frontier are settled; a round derives the
    evictions before front + window and moves the frontier to the first changed flag (or past
    the window when nothing changed)."""
    n = len(ev)
    flags, tail, cflag = [False] * n, {}, {}
    front = 0
    for r in range(1, max_rounds + 1):
        ops, left = walk(ev, carried, flags, tail, cflag)
        wend = front + window
        nf, nt, nc, nev = derive(ev, carried, ops, cap, tend=wend)
        changed = nf != flags or nt != tail or nc != cflag
        if not changed and wend >= n:
            return ops, nev, left, r
        if not changed:
            front = wend
        else:
            first = next((t for t in range(n) if nf[t] != flags[t]), None)
            if first is not None:
                assert first >= front  # settled events never change
                front = min(first, wend)
        flags, tail, cflag = nf, nt, nc
    raise AssertionError("rounds did not settle")


@pytest.mark.parametrize("seed,cap,sessions,window", [(1, 8, 40, 50), (2, 16, 100, 300), (3, 64, 500, 1000), (7, 5, 30, 7)])
def test_windowed_rounds_equal_sequential_lru(seed, cap, sessions, window):
    rng = np.random.default_rng(seed)
    ev, car = make_trace(rng, sessions, 3000, min(cap, 5))
    want_ops, want_ev, want_left = sequential(ev, car, cap)
    ops, nev, left, r = rounds_windowed(ev, car, cap, window)
    assert ops == want_ops
    assert nev == want_ev
    assert sorted(left) == sorted(want_left)


@pytest.mark.parametrize("seed,cap,sessions,carried", [(1, 8, 40, 0), (2, 16, 100, 10), (3, 64, 500, 64), (4, 5, 30, 5),
                                                        (5, 128, 3000, 100), (6, 2, 10, 2)])
def test_rounds_equal_sequential_lru(seed, cap, sessions, carried):
    rng = np.random.default_rng(seed)
    ev, car = make_trace(rng, sessions, 4000, carried)
    want_ops, want_ev, want_left = sequential(ev, car, cap)
    ops, nev, left, r = rounds(ev, car, cap)
    assert ops == want_ops
    assert nev == want_ev
    assert sorted(left) == sorted(want_left)
    assert want_ev > 0 or cap >= sessions


def test_rounds_settle_quickly_on_a_keepalive_trace():
    """Many live sessions and steady inserts (config 4 over a small LRU, as in the GPU test):
    the rounds settle in far fewer rounds than there are evictions."""
    rng = np.random.default_rng(9)
    ev, car = make_trace(rng, 2000, 20000, 50)
    want_ops, want_ev, _ = sequential(ev, car, 100)
    ops, nev, _, r = rounds(ev, car, 100)
    assert ops == want_ops and nev == want_ev
    assert want_ev > 1000 and r < 50


def merge_queue(ends, times):
    """derive()'s merge: each eviction time takes the first untaken marker alive then."""
    vict, q = [], 0
    for t in times:
        while q < len(ends) and not ends[q] > t:
            q += 1
        if q == len(ends):
            return vict, False
        vict.append(q)
        q += 1
    return vict, True


def merge_thresholds(ends, times, block=64):
    """k_lru_thresh + k_lru_take: c_m = evictions before the marker's end; per block of markers
    the thresholds X_k = min{x : x + #{k' < k : x < X_k'} >= c_k} (searched in [c_k - k, c_k]);
    the blocks chained by A += #{k : A < X_k}, marker k taken by eviction A + rank.  X_k as the
    kernel finds it: the (c_k - ms)-th positive integer missing from the sorted positive
    thresholds S so far, r + #{j : S_j - j < r} (1-based j), or 0 when c_k <= ms; the binary
    search over [c_k - k, c_k] is the definition it is checked against."""
    import bisect
    nj = len(times)
    X = []
    for b0 in range(0, len(ends), block):
        xs, S = [], []
        for k, e in enumerate(ends[b0:b0 + block]):
            c = bisect.bisect_left(times, e)
            lo, hi = max(0, c - k), c
            while lo < hi:
                mid = (lo + hi) // 2
                if mid + sum(1 for x in xs if x > mid) >= c:
                    hi = mid
                else:
                    lo = mid + 1
            want = lo if c > 0 else 0
            r = c - len(S)
            x = r + sum(1 for j, sj in enumerate(S, 1) if sj - j < r) if r > 0 else 0
            assert x == want
            if x:
                bisect.insort(S, x)
            xs.append(x)
        X += xs
    vict, A = [None] * nj, 0
    for b0 in range(0, len(ends), block):
        taken = [b0 + k for k, x in enumerate(X[b0:b0 + block]) if A < x]
        for r, m in enumerate(taken):
            vict[A + r] = m
        A += len(taken)
    return vict[:A], A == nj


@pytest.mark.parametrize("seed", range(12))
def test_threshold_merge_equals_the_queue_merge(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 700))
    ends = [int(x) for x in rng.integers(0, 2000, n)]
    if seed % 3 == 0:
        ends = [e if rng.random() < 0.5 else 1 << 30 for e in ends]  # never found again
    times = sorted(int(x) for x in rng.choice(2000, int(rng.integers(0, 400)), replace=False))
    want, ok = merge_queue(ends, times)
    got, ok2 = merge_thresholds(ends, times, block=int(rng.choice([1, 3, 64])))
    assert ok == ok2
    if ok:
        assert got == want
