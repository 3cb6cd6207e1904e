"""Pins the CPU oracle (oracle/) against the reference's own test vectors
(tests/golden/reference_vectors.json), the survey's probes of the compiled
reference, and this host's glibc for inet_pton / inet_ntop.  CPU only."""
import random
import socket

import numpy as np
import pytest

import oracle_py as O

UNENC, SSL = 8, 16


def b(s):
    return s.encode("latin-1")


def run_chunks(chunks, flags):
    p = O.Parser()
    total = sum(p.parse(b(c) if isinstance(c, str) else c, flags) for c in chunks)
    return p, total


def test_parser_valid_vectors(vectors):
    # HttpRequestParserTest.cpp:154-171 TestValidRequest
    for case in vectors["parser_valid"]:
        p, total = run_chunks(case["chunks"], SSL if case["is_https"] else UNENC)
        finished = p.state in ("FINISHED", "INVALID")
        assert finished == case["finished"], case
        assert p.state != "INVALID", case
        assert total == case["total"], case
        r = p.result()
        assert r["method"] == b(case["method"])
        assert r["url"] == b(case["url"])
        assert r["protocol"] == b(case["protocol"])
        assert r["host"] == b(case["host"])
        assert r["client_ip"] == [b(x) for x in case["client_ip"]]
        assert r["is_https"] == case["is_https"]


def test_parser_invalid_vectors(vectors):
    # HttpRequestParserTest.cpp:180-191 testInvalidRequest
    for case in vectors["parser_invalid"]:
        p, total = run_chunks(case["chunks"], UNENC)
        assert p.state == "INVALID", case
        assert total == case["total"], case


def test_client_ip_split_vectors(vectors):
    # HttpRequestParserTest.cpp:75-150
    for case in vectors["client_ip_split"] + vectors["probe_split"]:
        assert O.parse_client_ip(b(case["value"])) == [b(x) for x in case["expected"]], case


def _probe_chunks(case):
    if "lengths" in case:
        total = sum(case["lengths"])
        req = b"GET /" + b"a" * (total - 5 - 13) + b" HTTP/1.1\r\n\r\n"
        assert len(req) == total
        out, at = [], 0
        for n in case["lengths"]:
            out.append(req[at:at + n])
            at += n
        return out
    return [b(c) for c in case["chunks"]]


def test_parser_probe_vectors(vectors):
    for case in vectors["probe_parser"]:
        p, total = run_chunks(_probe_chunks(case), UNENC)
        assert p.state == case["state"], case
        if "total" in case:
            assert total == case["total"], case
        r = p.result()
        if "host" in case:
            assert r["host"] == b(case["host"]), case
        if "client_ip" in case:
            assert r["client_ip"] == [b(x) for x in case["client_ip"]], case


def test_sticky_client_ip_key():
    # HttpRequest::clear (HttpRequestParser.cpp:73-80) does not clear clientIPKey
    p = O.Parser()
    p.parse(b"GET / HTTP/1.1\r\nX-Forwarded-For: 1.2.3.4\r\n\r\n", UNENC)
    assert p.result()["client_ip"] == [b"1.2.3.4"]
    p.reset()
    p.parse(b"GET / HTTP/1.1\r\nTrue-Client-IP: 5.6.7.8\r\nx-forwarded-for: 9.9.9.9\r\n\r\n", UNENC)
    r = p.result()
    assert r["client_ip_key"] == b"x-forwarded-for"
    assert r["client_ip"] == [b"9.9.9.9"]


def test_pton4_probe_and_glibc(vectors):
    for case in vectors["probe_pton4"]:
        exp = bytes(case["expected"]) if case["expected"] is not None else None
        assert O.pton4(b(case["text"])) == exp


def _glibc_pton(af, text):
    try:
        return socket.inet_pton(af, text)
    except (OSError, ValueError):
        return None


PTON_EDGE = ["1.2.3.4", "0.0.0.0", "255.255.255.255", "256.0.0.0", "01.2.3.4", "1.02.3.4", "1.2.3", "1.2.3.4.5",
             "1..2.3", ".1.2.3", "1.2.3.", "", " 1.2.3.4", "1.2.3.4 ", "0.0.0.00", "00.0.0.0", "1.2.3.4:80",
             "::", "::1", "1::", "1:2:3:4:5:6:7:8", "1:2:3:4:5:6:7:8:9", "1:2:3:4:5:6:7::", "::2:3:4:5:6:7:8",
             ":1:2", "1:2:", ":::", "1::2::3", "12345::", "fffff::", "::ffff:1.2.3.4", "::1.2.3.4",
             "1:2:3:4:5:6:1.2.3.4", "1:2:3:4:5:6:7:1.2.3.4", "::ffff:01.2.3.4", "0064:ff9b::", "2001:DB8::1",
             "[::1]", "::ffff", "1:2:3:4:5:6:7:8:", ":", "a", "::ffff:1.2.3", "fe80::1%eth0", "1:2::3:4:5:6:7:8"]


def test_pton_matches_glibc():
    rng = random.Random(7)
    alphabet = "0123456789abcdefABCDEF:.[]x "
    cases = list(PTON_EDGE)
    for _ in range(20000):
        cases.append("".join(rng.choice(alphabet) for _ in range(rng.randint(0, 20))))
    for _ in range(2000):
        a = bytes(rng.getrandbits(8) for _ in range(16))
        if rng.random() < 0.3:
            a = bytes(10) + b"\xff\xff" + a[12:]
        cases.append(socket.inet_ntop(socket.AF_INET6, a))
        cases.append(socket.inet_ntop(socket.AF_INET, a[:4]))
    for t in cases:
        tb = t.encode()
        assert O.pton4(tb) == _glibc_pton(socket.AF_INET, t), t
        assert O.pton6(tb) == _glibc_pton(socket.AF_INET6, t), t


def test_ntop_vectors_and_glibc(vectors):
    for case in vectors["ntop"]:
        if "v4" in case:
            assert O.ntop4(bytes(case["v4"])) == b(case["text"])
        else:
            assert O.ntop6(bytes(case["v6"])) == b(case["text"])
    rng = random.Random(3)
    for _ in range(5000):
        a = bytearray(rng.getrandbits(8) for _ in range(16))
        for k in range(8):  # zero runs
            if rng.random() < 0.4:
                a[2 * k] = a[2 * k + 1] = 0
        if rng.random() < 0.2:
            a[:10] = bytes(10)
            a[10:12] = b"\xff\xff" if rng.random() < 0.5 else b"\x00\x00"
        a = bytes(a)
        assert O.ntop6(a) == socket.inet_ntop(socket.AF_INET6, a).encode()
        assert O.ntop4(a[:4]) == socket.inet_ntop(socket.AF_INET, a[:4]).encode()
        # the source-address path (Aggregator.cpp:57-61) round-trips: ntop -> pton is the identity
        assert O.pton6(O.ntop6(a)) == a
        assert O.pton4(O.ntop4(a[:4])) == a[:4]


def _a4(t):
    return socket.inet_pton(socket.AF_INET, t)


def _a6(t):
    return socket.inet_pton(socket.AF_INET6, t)


def test_checker_vectors(vectors):
    o = O.Oracle()
    for t in vectors["v4_reserved_internal"]:
        assert o.is_v4_external(_a4(t)) is False, t
    for t, exp in vectors["v6_cases"]:
        assert o.is_v6_external(_a6(t)) is exp, t
    o4 = O.Oracle(v4_ifaces=[(_a4(a), _a4(m)) for a, m in vectors["v4_iface"]["v4_ifaces"]])
    for t, exp in vectors["v4_iface"]["cases"]:
        assert o4.is_v4_external(_a4(t)) is exp
    o6 = O.Oracle(v6_ifaces=[(_a6(a), _a6(m)) for a, m in vectors["v6_iface"]["v6_ifaces"]])
    for t, exp in vectors["v6_iface"]["cases"]:
        assert o6.is_v6_external(_a6(t)) is exp, t
    assert o.is_v4_external(_a4("8.8.8.8")) is True
    assert o.is_v4_external(_a4("200.100.1.1")) is True


def test_aggregator_vectors_with_mock(vectors):
    # AggregatorTest.cpp:69-172 with the IpAddressCheckerMock verdict queue
    agg = vectors["aggregator"]
    o = O.Oracle()
    o.set_mock([1 if r["mock"] else 0 for r in agg["requests"] if r["mock"] is not None])
    for r in agg["requests"]:
        o.new_request(r["pid"], b(r["host"]), b(r["url"]), None, r["flags"] or 0)
    exp = sorted((e["pid"], b(e["endpoint"]), b(e["domain"]), b(e["scheme"]), e["internal"], e["external"])
                 for e in agg["expected"])
    assert o.services() == exp
    o.clear()
    assert o.services() == []


def test_aggregator_vectors_with_real_checker(vectors):
    agg = vectors["aggregator"]
    o = O.Oracle()
    for r in agg["requests"]:
        src = None
        if r["real_src"]:
            src = _a6(r["real_src"]) if ":" in r["real_src"] else _a4(r["real_src"]) + bytes(12)
        o.new_request(r["pid"], b(r["host"]), b(r["url"]), None, r["flags"] or 0, src)
    exp = sorted((e["pid"], b(e["endpoint"]), b(e["domain"]), b(e["scheme"]), e["internal"], e["external"])
                 for e in agg["expected"])
    assert o.services() == exp


def test_lru_vectors(vectors):
    for script in vectors["lru"]:
        lru = O.LRU(script["capacity"])
        names = {}
        for op in script["ops"]:
            if op[0] == "insert":
                names.setdefault(op[2], len(names))
                lru.insert(op[1], names[op[2]])
            elif op[0] == "update":
                names.setdefault(op[2], len(names))
                assert lru.update(op[1], names[op[2]])
            elif op[0] == "erase":
                assert lru.erase(op[1])
            else:
                got = lru.find(op[1])
                assert got == (names[op[2]] if op[2] is not None else None), (script["name"], op)


def make_events(n, pid=1000, fd=5, sid=None, seq=None, flags=2 | 8 | 32, src=b"\x7f\x00\x00\x01"):
    ev = np.zeros(n, O.EVENT_DTYPE)
    ev["pid"] = pid
    ev["fd"] = fd
    ev["sessionID"] = np.arange(1, n + 1) if sid is None else sid
    ev["bufferSeq"] = 1 if seq is None else seq
    ev["flags"] = flags
    s = np.frombuffer(src.ljust(16, b"\0"), np.uint8)
    ev["sourceIP"][:] = s
    return ev


def pack(payloads):
    lens = np.array([len(p) for p in payloads], np.uint32)
    offs = np.zeros(len(payloads), np.uint64)
    if len(payloads) > 1:
        offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    return lens, offs, np.frombuffer(b"".join(payloads), np.uint8) if payloads else np.zeros(0, np.uint8)


def test_config1_probe(vectors):
    for case in vectors["config1"]:
        o = O.Oracle()
        n = case["n"]
        lens, offs, payload = pack([b(case["payload"])] * n)
        o.process(make_events(n), lens, offs, payload)
        exp = [(s["pid"], b(s["endpoint"]), b(s["domain"]), b(s["scheme"]), s["internal"], s["external"])
               for s in case["services"]]
        assert o.services() == exp
        assert o.stats()["lru_size"] == case["saved_sessions"]


def test_sessions_fragmented_and_first_arrival():
    o = O.Oracle()
    req = b"GET /a HTTP/1.1\r\nHost: h:80\r\nX-Forwarded-For: 8.8.8.8:5\r\n\r\n"
    parts = [req[:10], req[10:30], req[30:]]
    ev = make_events(4, sid=[7, 7, 7, 9], seq=[1, 2, 3, 1])
    ev["flags"][3] = 4 | 16 | 32  # second session, IPv6 + SSL, source ::1 (internal)
    ev["sourceIP"][3] = np.frombuffer(bytes(15) + b"\x01", np.uint8)
    lens, offs, payload = pack(parts + [b"GET /a HTTP/1.1\r\nHost: h:80\r\n\r\n"])
    out, blob = o.process(ev, lens, offs, payload)
    assert list(out["kind"]) == [1, 2, 2, 1]
    assert list(out["status"]) == [1, 1, 2, 2]
    assert list(out["consumed"]) == [10, 20, len(req) - 30, 31]
    assert out["cls"][2] == O_EXT and out["cls"][3] == O_INT
    # first arrival: scheme from the first request that created the key
    assert o.services() == [(1000, b"h:80/a", b"h", b"http", 1, 1)]
    assert o.stats()["lru_size"] == 1  # finished existing session is kept (Discovery.cpp:138)


O_INT, O_EXT = 1, 2


def test_invalid_existing_session_deletes_kernel_session():
    o = O.Oracle()
    ev = make_events(2, sid=[3, 3], seq=[1, 2])
    lens, offs, payload = pack([b"GET /x HTTP/1.1\r\n", b"\x01bad"])
    out, _ = o.process(ev, lens, offs, payload)
    assert list(out["status"]) == [1, 3]
    st = o.stats()
    assert st["kernel_deletes"] == 1 and st["lru_size"] == 0


def test_lru_eviction_changes_results():
    # SURVEY 8(a) a9 [probe]: an evicted mid-request session's continuation parses as new -> INVALID
    o = O.Oracle(lru_capacity=2)
    ev = make_events(4, sid=[1, 2, 3, 1], seq=[1, 1, 1, 2])
    lens, offs, payload = pack([b"GET / HTTP/1.1\r\n", b"GET / HTTP/1.1\r\n", b"GET / HTTP/1.1\r\n",
                                b"Host: h\r\n\r\n"])
    out, _ = o.process(ev, lens, offs, payload)
    assert list(out["kind"]) == [1, 1, 1, 1]
    assert out["status"][3] == 3
    assert o.stats()["lru_evictions"] == 1


def test_data_end_closes_session():
    o = O.Oracle()
    ev = make_events(3, sid=[5, 5, 5], seq=[1, 1, 2])
    ev["flags"][1] = 64  # DATA_END only
    lens, offs, payload = pack([b"GET / HTTP/1.1\r\n", b"", b"Host: h\r\n\r\n"])
    out, _ = o.process(ev, lens, offs, payload)
    assert list(out["kind"]) == [1, 0, 1]
    assert out["status"][2] == 3  # parsed as a new session after the close
