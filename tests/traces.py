"""Trace builders for the parity tests (test tooling, not product code).

A trace is (events, lens, offs, payload) in the packed layout of
include/ebpf_discovery_amd.h: DiscoveryEvent records (Types.h:201-205), buffer
lengths, offsets into one payload arena.
"""
import random

import numpy as np

import ebd

EV = ebd.EVENT_DTYPE


def pack(bufs, align=1):
    lens = np.zeros(len(bufs), np.uint32)
    offs = np.zeros(len(bufs), np.uint64)
    parts, at = [], 0
    for k, bf in enumerate(bufs):
        if bf is None:
            lens[k] = ebd.NO_BUFFER
            offs[k] = 0
            continue
        pad = (-at) % align
        if pad:
            parts.append(b"\0" * pad)
            at += pad
        lens[k] = len(bf)
        offs[k] = at
        parts.append(bf)
        at += len(bf)
    parts.append(b"\0" * 16)
    return lens, offs, np.frombuffer(b"".join(parts), np.uint8).copy()


def events(rows):
    """rows: dicts with pid, fd, sid, seq, flags, src (bytes)."""
    ev = np.zeros(len(rows), EV)
    for k, r in enumerate(rows):
        ev[k]["pid"] = r.get("pid", 1000)
        ev[k]["fd"] = r.get("fd", 5)
        ev[k]["sessionID"] = r["sid"]
        ev[k]["bufferSeq"] = r.get("seq", 1)
        ev[k]["flags"] = r["flags"]
        ev[k]["sourceIP"] = np.frombuffer(r.get("src", b"\x7f\0\0\1").ljust(16, b"\0"), np.uint8)
    return ev


def session_trace(chunk_lists, flags=ebd.FLAG_IPV4 | ebd.FLAG_UNENCRYPTED, close=False, interleave=False):
    """One session per chunk list; each chunk is one recv() event of that session."""
    rows, bufs = [], []
    streams = [[(s, k, c) for k, c in enumerate(chunks)] for s, chunks in enumerate(chunk_lists)]
    order = []
    if interleave:
        while any(streams):
            for st in streams:
                if st:
                    order.append(st.pop(0))
    else:
        for st in streams:
            order.extend(st)
    for s, k, c in order:
        rows.append(dict(sid=s + 1, seq=k + 1, flags=flags | ebd.FLAG_NEW_DATA))
        bufs.append(c)
    if close:
        for s in range(len(chunk_lists)):
            rows.append(dict(sid=s + 1, seq=len(chunk_lists[s]), flags=ebd.FLAG_DATA_END, src=b""))
            bufs.append(None)
    lens, offs, payload = pack(bufs)
    return events(rows), lens, offs, payload


def fragmented_trace(n_conn, seed=4, window=512, max_req=8, kmin=2, kmax=4):
    """Config-4 shape: config-3 requests, each cut at uniform points into
    k in [kmin, kmax] consecutive recv() events (first piece >= 16 B), 1..max_req keep-alive
    requests per connection then a DATA_END event; `window` connections interleaved."""
    rng = random.Random(seed)
    total_req = n_conn * max_req
    ev3, l3, o3, p3 = ebd.generate_host(3, seed, 0, total_req)
    pay = p3.tobytes()
    reqi = 0
    conns = []
    for c in range(n_conn):
        nreq = rng.randint(1, max_req)
        flags = (ebd.FLAG_IPV6 if rng.random() < 0.2 else ebd.FLAG_IPV4) | (
            ebd.FLAG_SSL if rng.random() < 0.15 else ebd.FLAG_UNENCRYPTED)
        src = bytes(rng.getrandbits(8) for _ in range(16))
        pid = 2000 + c % 64
        evs = []
        for _ in range(nreq):
            buf = pay[int(o3[reqi]):int(o3[reqi]) + int(l3[reqi])]
            reqi += 1
            k = rng.randint(kmin, kmax)
            hdr = buf.find(b"\r\n\r\n") + 4  # a POST body stays in the last fragment
            hdr = hdr if hdr >= 4 else len(buf)
            cuts = sorted(rng.sample(range(16, hdr), min(k - 1, max(hdr - 16, 0)))) if hdr > 17 else []
            pieces, at = [], 0
            for cu in cuts:
                pieces.append(buf[at:cu])
                at = cu
            pieces.append(buf[at:])
            for pc in pieces:
                evs.append(("data", pc))
        evs.append(("end", None))
        conns.append(dict(pid=pid, fd=5 + c % 100, sid=c + 1, flags=flags, src=src, evs=evs))
    rows, bufs = [], []
    for g in range(0, n_conn, window):
        group = [dict(cn, i=0, seq=0) for cn in conns[g:g + window]]
        active = list(range(len(group)))
        while active:
            nxt = []
            for a in active:
                cn = group[a]
                kind, pc = cn["evs"][cn["i"]]
                cn["i"] += 1
                if kind == "data":
                    cn["seq"] += 1
                    rows.append(dict(pid=cn["pid"], fd=cn["fd"], sid=cn["sid"], seq=cn["seq"],
                                     flags=cn["flags"] | ebd.FLAG_NEW_DATA, src=cn["src"]))
                    bufs.append(pc)
                else:
                    rows.append(dict(pid=cn["pid"], fd=cn["fd"], sid=cn["sid"], seq=cn["seq"],
                                     flags=ebd.FLAG_DATA_END, src=b""))
                    bufs.append(None)
                if cn["i"] < len(cn["evs"]):
                    nxt.append(a)
            active = nxt
    lens, offs, payload = pack(bufs)
    return events(rows), lens, offs, payload


def probe_chunks(case):
    """Chunks of a parser probe vector: the literal chunks, or for the length-cap probes
    ("lengths") a GET request of sum(lengths) bytes cut at those lengths."""
    if "lengths" in case:
        return length_request_chunks(case["lengths"])
    return [c.encode("latin-1") for c in case["chunks"]]


def length_request_chunks(lengths):
    """A GET request of exactly sum(lengths) bytes (a long URL), cut into recv() pieces of
    the given lengths (each <= 8192, the saved-buffer limit)."""
    total = sum(lengths)
    req = b"GET /" + b"a" * (total - 5 - 13) + b" HTTP/1.1\r\n\r\n"
    assert len(req) == total
    out, at = [], 0
    for n in lengths:
        out.append(req[at:at + n])
        at += n
    return out


def oracle_view(out, blob):
    """Per-event comparable tuples from the oracle."""
    res = []
    for r in out:
        t = (int(r["status"]), int(r["consumed"]))
        if r["status"] == 2:
            cip = blob[r["cip_off"]:r["cip_off"] + r["cip_len"]] if r["has_cip"] else None
            t += (blob[r["host_off"]:r["host_off"] + r["host_len"]], blob[r["url_off"]:r["url_off"] + r["url_len"]],
                  cip, int(r["cls"]), bool(r["is_https"]))
        res.append(t)
    return res


def gpu_view(res, offs, payload, sreq, sstr):
    pay = payload.tobytes() if hasattr(payload, "tobytes") else payload
    out = []
    for i, r in enumerate(res):
        t = (int(r["status"]), int(r["consumed"]))
        if r["status"] == 2:
            info = int(r["info"])
            if info & ebd.INFO_SESSION:
                idx = int(r["url_off"]) | (int(r["url_len"]) << 16)
                q = sreq[idx]
                so, hl, ul = int(q["str_off"]), int(q["host_len"]), int(q["url_len"])
                host, url = sstr[so:so + hl], sstr[so + hl:so + hl + ul]
                cip = sstr[so + int(q["cip_off"]):so + int(q["cip_off"]) + int(q["cip_len"])] if info & ebd.INFO_CIP else None
            else:
                o = int(offs[i])
                host = pay[o + int(r["host_off"]):o + int(r["host_off"]) + int(r["host_len"])]
                url = pay[o + int(r["url_off"]):o + int(r["url_off"]) + int(r["url_len"])]
                cip = pay[o + int(r["cip_off"]):o + int(r["cip_off"]) + int(r["cip_len"])] if info & ebd.INFO_CIP else None
            t += (host, url, cip, (info >> 4) & 3, bool(info & ebd.INFO_HTTPS))
        out.append(t)
    return out
