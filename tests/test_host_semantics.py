"""The product's parse semantics (ebd_spec.h / ebd_fresh.h — the code the GPU kernels
run) executed on the CPU through libebd_amd.so's host hooks, against the oracle and the
reference vectors.  CPU only."""
import random
import socket

import numpy as np
import pytest

import ebd
import oracle_py as O

UNENC, SSL = ebd.FLAG_UNENCRYPTED, ebd.FLAG_SSL
NEW4 = ebd.FLAG_IPV4 | UNENC | ebd.FLAG_NEW_DATA
ST = {"FINISHED": ebd.STATUS_FINISHED, "INVALID": ebd.STATUS_INVALID}
GP_STATE = {10: "FINISHED", 11: "INVALID"}


def b(s):
    return s.encode("latin-1")


def test_dfa_layout():
    i = ebd.dfa_info()
    # HV(client) states are the last two ids, right after the terminal states
    assert i["url_id"] < i["g2"] < i["g3"] < i["g4"]
    assert i["hvc0"] == i["g4"] + 3 and i["nstates"] == i["g4"] + 5 <= 200  # kLdsRows
    assert (i["fin0"], i["fin1"], i["inv"]) == (i["g4"], i["g4"] + 1, i["g4"] + 2)


def oracle_single(buf, flags=NEW4, src=b"\x7f\0\0\1", pid=77, v4=(), v6=()):
    o = O.Oracle(v4_ifaces=list(v4), v6_ifaces=list(v6))
    ev = np.zeros(1, O.EVENT_DTYPE)
    ev["pid"], ev["fd"], ev["sessionID"], ev["bufferSeq"], ev["flags"] = pid, 3, 1, 1, flags
    ev["sourceIP"][0] = np.frombuffer(src.ljust(16, b"\0"), np.uint8)
    out, blob = o.process(ev, np.array([len(buf)], np.uint32), np.zeros(1, np.uint64),
                          np.frombuffer(buf, np.uint8) if buf else np.zeros(1, np.uint8))
    return out[0], blob, o.services()


def scan_shifted(shift):
    """The structural fast path (k_fresh) with the buffer at byte `shift` of its tile."""
    def f(buf, pid=0, flags=NEW4, src16=bytes(16), v4=(), v6=()):
        return ebd.host_scan(buf, pid, flags, src16, v4, v6, shift=shift)
    return f


# the DFA fast path (k_fresh) and the structural scan (k_fresh_scan) at three tile alignments
FAST_PATHS = {"dfa": ebd.host_fresh, "scan0": scan_shifted(0), "scan7": scan_shifted(7), "scan15": scan_shifted(15)}


def check_fresh_against_oracle(buf, flags=NEW4, src=b"\x7f\0\0\1", pid=77, v4=(), v6=(), fn=ebd.host_fresh):
    r, key = fn(buf, pid, flags, src.ljust(16, b"\0"), v4, v6)
    o, blob, svcs = oracle_single(buf, flags, src, pid, v4, v6)
    if o["status"] == O_STATUS_UNF:
        assert r["status"] == ebd.STATUS_UNFINISHED, buf
        assert r["consumed"] == len(buf)
        return
    assert r["status"] == {2: ebd.STATUS_FINISHED, 3: ebd.STATUS_INVALID}[int(o["status"])], buf
    assert r["consumed"] == o["consumed"], buf
    if r["status"] != ebd.STATUS_FINISHED:
        return
    host = blob[o["host_off"]:o["host_off"] + o["host_len"]]
    url = blob[o["url_off"]:o["url_off"] + o["url_len"]]
    assert buf[r["host_off"]:r["host_off"] + r["host_len"]] == host, buf
    assert buf[r["url_off"]:r["url_off"] + r["url_len"]] == url, buf
    assert bool(r["info"] & ebd.INFO_CIP) == bool(o["has_cip"]), buf
    if o["has_cip"]:
        cip = blob[o["cip_off"]:o["cip_off"] + o["cip_len"]]
        assert buf[r["cip_off"]:r["cip_off"] + r["cip_len"]] == cip, buf
    assert (r["info"] >> 4) & 3 == o["cls"], buf
    assert bool(r["info"] & ebd.INFO_HTTPS) == bool(o["is_https"])


O_STATUS_UNF = 1


@pytest.mark.parametrize("path", sorted(FAST_PATHS))
def test_fresh_reference_vectors(vectors, path):
    fn = FAST_PATHS[path]
    for case in vectors["parser_valid"] + vectors["parser_invalid"]:
        if len(case["chunks"]) == 1:
            check_fresh_against_oracle(b(case["chunks"][0]), flags=NEW4 | (SSL if case.get("is_https") else 0), fn=fn)
    for case in vectors["probe_parser"]:
        if "chunks" in case and len(case["chunks"]) == 1:
            check_fresh_against_oracle(b(case["chunks"][0]), fn=fn)


QUIRKS = [
    b"GET / HTTP/1.1\r\nX-Forwarded-For: , 1.2.3.4\r\n\r\n",
    b"GET / HTTP/1.1\r\nX-Forwarded-For: 1.2.3.4 , 5.6.7.8\r\n\r\n",
    b"GET / HTTP/1.1\r\nX-Forwarded-For: [::1]:80\r\n\r\n",
    b"GET / HTTP/1.1\r\nX-Forwarded-For: [ ::1 ]\r\n\r\n",
    b"GET / HTTP/1.1\r\nX-Forwarded-For: [::1\r\n\r\n",
    b"GET / HTTP/1.1\r\nX-Forwarded-For: ::ffff:1.2.3.4\r\n\r\n",
    b"GET / HTTP/1.1\r\nX-Forwarded-For: 01.2.3.4\r\n\r\n",
    b"GET / HTTP/1.1\r\nX-Forwarded-For: 1.2.3.4:5:6\r\n\r\n",
    b"GET / HTTP/1.1\r\nX-Forwarded-For: ,,,\r\n\r\n",
    b"GET / HTTP/1.1\r\nX-Forwarded-For: \"1.2.3.4\r\n\r\n",
    b"GET / HTTP/1.1\r\nTrue-Client-IP: 8.8.8.8\r\nX-Forwarded-For: 10.0.0.1\r\n\r\n",
    b"GET / HTTP/1.1\r\nx-http-client-ip: 2001:db8::1\r\nHost: [fe80::1]:80\r\n\r\n",
    b"GET / HTTP/1.1\r\nrproxy_remote_address: 9.9.9.9\r\n\r\n",
    b"GET / HTTP/1.1\r\nRPROXY_REMOTE_ADDRESS_EXTRA: 9.9.9.9\r\n\r\n",
    b"GET / HTTP/1.1\r\nx-forwarded-forx: 9.9.9.9\r\n\r\n",
    b"GET / HTTP/1.1\r\nHost: [::1\r\n\r\n",
    b"GET / HTTP/1.1\r\nHost: a:b:c\r\n\r\n",
    b"GET / HTTP/1.1\r\nHost : a\r\n\r\n",
    b"GET / HTTP/1.1\r\n Host: a\r\n\r\n",
    b"GET / HTTP/1.1\r\nHost:a\r\n\r\n",
    b"GET /a?b=c&d=%20#x HTTP/1.0\r\n\r\n",
    b"POST /x HTTP/1.1\r\nContent-Length: 3\r\n\r\nabc",
    b"GET / HTTP/1.1\r\nFoo\r\n",
    b"GET / HTTP/1.1\r\nFoo\r\nHost: x\r\n\r\n",
    b"GET / HTTP/1.1\r\n\r\nGET /b HTTP/1.1\r\n\r\n",
    b"GET / HTTP/1.1\r\nA: b\r\r\n",
    b"GET / HTTP/1.1\r\nA: \x80\r\n\r\n",
    b"GET / HTTP/1.1\r\nA:\t b\r\n\r\n",
    b"GET / HTTP/1.12\r\n\r\n",
    b"GET / HTTP/1.\r\n\r\n",
    b"GE",
    b"POS",
    b"",
    b"GET",
    b"GET /",
    b"GET / HTTP/1.1\r\nHost: h\r\nX-Client-IP: 1.1.1.1",
]


@pytest.mark.parametrize("path", sorted(FAST_PATHS))
def test_fresh_quirks(path):
    fn = FAST_PATHS[path]
    for buf in QUIRKS:
        check_fresh_against_oracle(buf, fn=fn)
        check_fresh_against_oracle(buf, flags=ebd.FLAG_IPV6 | SSL | ebd.FLAG_NEW_DATA, src=bytes(15) + b"\x01", fn=fn)


@pytest.mark.parametrize("path", sorted(FAST_PATHS))
def test_fresh_generated_config3_sample(path):
    fn = FAST_PATHS[path]
    ev, lens, offs, payload = ebd.generate_host(3, 3, 0, 4000)
    o = O.Oracle()
    out, blob = o.process(ev, lens, offs, payload)
    pay = payload.tobytes()
    for i in range(len(ev)):
        buf = pay[int(offs[i]):int(offs[i]) + int(lens[i])]
        r, _ = fn(buf, int(ev["pid"][i]), int(ev["flags"][i]), ev["sourceIP"][i].tobytes())
        assert r["consumed"] == out["consumed"][i], i
        assert r["status"] == {1: 1, 2: 2, 3: 3}[int(out["status"][i])], i
        if r["status"] == ebd.STATUS_FINISHED:
            oh = blob[out["host_off"][i]:out["host_off"][i] + out["host_len"][i]]
            ou = blob[out["url_off"][i]:out["url_off"][i] + out["url_len"][i]]
            assert buf[r["host_off"]:r["host_off"] + r["host_len"]] == oh
            assert buf[r["url_off"]:r["url_off"] + r["url_len"]] == ou
            assert (r["info"] >> 4) & 3 == out["cls"][i], (i, buf)


def test_fresh_key_is_streaming_key_of_endpoint():
    """The fast path's block-form key equals the session path's streaming key of
    host + url, for every alignment of the buffer (the key is split invariant)."""
    ev, lens, offs, payload = ebd.generate_host(3, 5, 0, 1500)
    pay = payload.tobytes()
    for i in range(len(ev)):
        buf = pay[int(offs[i]):int(offs[i]) + int(lens[i])]
        pid = int(ev["pid"][i])
        for shift in (0, 3, 13):
            padded = bytearray(b"\0" * (shift + len(buf) + 32))
            padded[shift:shift + len(buf)] = buf
            arr = np.frombuffer(bytes(padded), np.uint8)
            r, key = ebd.host_fresh(bytes(arr[shift:shift + len(buf)]), pid, int(ev["flags"][i]),
                                    ev["sourceIP"][i].tobytes())
            if r["status"] != ebd.STATUS_FINISHED:
                continue
            ep = buf[r["host_off"]:r["host_off"] + r["host_len"]] + buf[r["url_off"]:r["url_off"] + r["url_len"]]
            assert key == ebd.host_endpoint_key(pid, ep), (i, shift)
    # every host/url split of one endpoint gives one key
    ep = b"svc-1.example.internal:8080/api/v1/items?id=123456789"
    k0 = ebd.host_endpoint_key(7, ep)
    for cut in range(len(ep) + 1):
        req = b"GET " + ep[cut:] + b" HTTP/1.1\r\nHost: " + ep[:cut] + b"\r\n\r\n"
        if not ep[cut:].startswith(b"/"):
            continue
        r, key = ebd.host_fresh(req, 7)
        if r["status"] == ebd.STATUS_FINISHED and r["host_len"] == cut:
            assert key == k0, cut
    assert ebd.host_endpoint_key(7, ep) != ebd.host_endpoint_key(8, ep)
    assert ebd.host_endpoint_key(7, b"") != ebd.host_endpoint_key(7, b"\0")


M64 = (1 << 64) - 1


def _rotl(x, r):
    return ((x << r) | (x >> (64 - r))) & M64


def _sipround(v):
    v0, v1, v2, v3 = v
    v0 = (v0 + v1) & M64; v1 = _rotl(v1, 13); v1 ^= v0; v0 = _rotl(v0, 32)
    v2 = (v2 + v3) & M64; v3 = _rotl(v3, 16); v3 ^= v2
    v0 = (v0 + v3) & M64; v3 = _rotl(v3, 21); v3 ^= v0
    v2 = (v2 + v1) & M64; v1 = _rotl(v1, 17); v1 ^= v2; v2 = _rotl(v2, 32)
    return [v0, v1, v2, v3]


def _siphash(k0, k1, words, c, d, out128):
    """SipHash-c-d (Aumasson & Bernstein 2012) over 64-bit message words; the 128-bit output
    variant when out128 (v1 ^= 0xee at init, v2 ^= 0xee, then v1 ^= 0xdd for the 2nd half)."""
    v = [k0 ^ 0x736F6D6570736575, k1 ^ 0x646F72616E646F6D, k0 ^ 0x6C7967656E657261, k1 ^ 0x7465646279746573]
    if out128:
        v[1] ^= 0xEE
    for m in words:
        v[3] ^= m
        for _ in range(c):
            v = _sipround(v)
        v[0] ^= m
    v[2] ^= 0xEE if out128 else 0xFF
    for _ in range(d):
        v = _sipround(v)
    lo = v[0] ^ v[1] ^ v[2] ^ v[3]
    if not out128:
        return lo
    v[1] ^= 0xDD
    for _ in range(d):
        v = _sipround(v)
    return lo, v[0] ^ v[1] ^ v[2] ^ v[3]


def test_siphash_rounds_pinned_by_published_vector():
    """The round function above is pinned by the SipHash paper's test vector (SipHash-2-4,
    key 00..0f, message 00..0e -> a129ca6149be45e5)."""
    msg = bytes(range(15))
    words = [int.from_bytes(msg[0:8], "little"), int.from_bytes(msg[8:15], "little") | (15 << 56)]
    k0, k1 = int.from_bytes(bytes(range(8)), "little"), int.from_bytes(bytes(range(8, 16)), "little")
    assert _siphash(k0, k1, words, 2, 4, False) == 0xA129CA6149BE45E5


def test_service_key_is_siphash13_128_of_pid_and_endpoint():
    """ebd_spec.h KeyHasher = SipHash-1-3-128 over [pid, E as zero-padded LE words, 0xe5<<56|len],
    with the low bit of each half forced to 1 (0 marks an empty table slot)."""
    rng = random.Random(5)
    for t in range(300):
        hk = (rng.getrandbits(64), rng.getrandbits(64)) if t % 3 else ebd.TEST_HASH_KEY
        pid = rng.getrandbits(32)
        ep = bytes(rng.randrange(0x21, 0x7F) for _ in range(rng.randrange(0, 90)))
        words = [pid] + [int.from_bytes(ep[o:o + 8], "little") for o in range(0, len(ep), 8)]
        words.append((0xE5 << 56) | len(ep))
        lo, hi = _siphash(hk[0], hk[1], words, 1, 3, True)
        assert ebd.host_endpoint_key(pid, ep, hash_key=hk) == (lo | 1, hi | 1)


def test_unkeyed_hash_collision_pair_is_separated():
    """two (pid, endpoint) pairs that collided under the round-1 unkeyed wymix
    hash.  Under the keyed PRF they get different keys (under any key we try)."""
    a = (1234, b"/3;9mw7wYuiP611jT,M,4AWTVmL_U37J/api/v1/users")
    b = (99999, b"/[~pQ5)Faj9%d2.%rIb]]?-iOPR2'u%9/api/v1/users")
    rng = random.Random(9)
    for hk in [ebd.TEST_HASH_KEY] + [(rng.getrandbits(64), rng.getrandbits(64)) for _ in range(20)]:
        assert ebd.host_endpoint_key(*a, hash_key=hk) != ebd.host_endpoint_key(*b, hash_key=hk)
    # keys depend on the secret
    assert ebd.host_endpoint_key(*a, hash_key=(1, 2)) != ebd.host_endpoint_key(*a, hash_key=(1, 3))


def test_fresh_random_mutations():
    rng = random.Random(11)
    base = [b"GET /p/q?x=1 HTTP/1.1\r\nHost: svc.example.com:80\r\nX-Forwarded-For: 8.8.8.8:9, 10.0.0.1\r\n"
            b"User-Agent: a b/c\r\nAccept: */*\r\n\r\n",
            b"POST /up HTTP/1.0\r\nhost: [2001:db8::1]:443\r\ntrue-client-ip: [fd00::5]\r\n\r\nBODY"]
    alphabet = b"GETPOSH/ :\r\n,.[]-_xX0123456789\x01\x80\t"
    for _ in range(3000):
        s = bytearray(rng.choice(base))
        for _ in range(rng.randint(1, 3)):
            op = rng.random()
            k = rng.randrange(len(s))
            if op < 0.4:
                s[k] = rng.choice(alphabet)
            elif op < 0.7:
                del s[k]
            else:
                s.insert(k, rng.choice(alphabet))
        check_fresh_against_oracle(bytes(s))


def test_generic_parser_chunked_vectors(vectors):
    for case in vectors["parser_valid"] + vectors["parser_invalid"]:
        chunks = [b(c) for c in case["chunks"]]
        cons, st, data = ebd.host_gp_parse(chunks, SSL if case.get("is_https") else UNENC)
        p = O.Parser()
        ocons = [p.parse(c, SSL if case.get("is_https") else UNENC) for c in chunks]
        assert cons == ocons, case
        assert sum(cons) == case["total"]
        r = p.result()
        name = {10: "FINISHED", 11: "INVALID"}.get(st["state"])
        assert (name or "other") == (p.state if p.state in ("FINISHED", "INVALID") else "other")
        if p.state == "INVALID":
            continue
        assert data[st["url_start"]:st["url_start"] + st["url_len"]] == r["url"], case
        assert data[st["host_start"]:st["host_start"] + st["host_len"]] == r["host"], case
        if r["client_ip"]:
            raw = data[st["cip_start"]:st["cip_start"] + st["cip_len"]]
            assert O.parse_client_ip(raw)[0] == r["client_ip"][0], case
        method = b"GET"[:st["mlen"]] if st["mcand"] == ord("G") else (b"POST"[:st["mlen"]] if st["mlen"] else b"")
        assert method == r["method"], case


def test_generic_parser_length_cap():
    for total, state in ((8193, 10), (8194, 11)):
        req = b"GET /" + b"a" * (total - 18) + b" HTTP/1.1\r\n\r\n"
        cons, st, _ = ebd.host_gp_parse([req[:8192], req[8192:]])
        assert st["state"] == state and sum(cons) == 8193


def test_generic_parser_sticky_key():
    first = b"GET / HTTP/1.1\r\nX-Forwarded-For: 1.2.3.4\r\n\r\n"
    second = b"GET / HTTP/1.1\r\nTrue-Client-IP: 5.6.7.8\r\nx-forwarded-for: 9.9.9.9\r\n\r\n"
    cons, st, data = ebd.host_gp_parse([first, second], reset_between=True)
    assert st["state"] == 10
    base = len(first)  # after reset() stream positions restart at the second request
    raw = data[base + st["cip_start"]:base + st["cip_start"] + st["cip_len"]]
    assert raw == b"9.9.9.9"


def test_pton_matches_oracle_and_glibc():
    rng = random.Random(5)
    alphabet = "0123456789abcdefABCDEF:.[] "
    cases = ["1.2.3.4", "01.2.3.4", "::", "::1", "::ffff:1.2.3.4", "1:2:3:4:5:6:7:8", "1::2::3", ":1", "1:", "",
             "2001:db8::1", "::ffff:01.2.3.4", "1.2.3.4.5", "255.255.255.255", "256.1.1.1"]
    cases += ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, 18))) for _ in range(20000)]
    for t in cases:
        tb = t.encode()
        assert ebd.host_pton(tb, False) == O.pton4(tb), t
        assert ebd.host_pton(tb, True) == O.pton6(tb), t


def test_classification_matches_oracle(vectors):
    o = O.Oracle()
    for t in vectors["v4_reserved_internal"] + ["8.8.8.8", "200.1.2.3"]:
        a = socket.inet_pton(socket.AF_INET, t)
        assert ebd.host_classify_source(a + bytes(12), ebd.FLAG_IPV4) == (2 if o.is_v4_external(a) else 1)
    for t, exp in vectors["v6_cases"]:
        a = socket.inet_pton(socket.AF_INET6, t)
        assert ebd.host_classify_source(a, ebd.FLAG_IPV6) == (2 if exp else 1), t
    v6i = [(socket.inet_pton(socket.AF_INET6, a), socket.inet_pton(socket.AF_INET6, m))
           for a, m in vectors["v6_iface"]["v6_ifaces"]]
    for t, exp in vectors["v6_iface"]["cases"]:
        a = socket.inet_pton(socket.AF_INET6, t)
        assert ebd.host_classify_source(a, ebd.FLAG_IPV6, v6=v6i) == (2 if exp else 1), t
    v4i = [(socket.inet_pton(socket.AF_INET, a), socket.inet_pton(socket.AF_INET, m))
           for a, m in vectors["v4_iface"]["v4_ifaces"]]
    for t, exp in vectors["v4_iface"]["cases"]:
        a = socket.inet_pton(socket.AF_INET, t)
        assert ebd.host_classify_source(a + bytes(12), ebd.FLAG_IPV4, v4=v4i) == (2 if exp else 1)
    assert ebd.host_classify_source(bytes(16), 0) == 0
    assert ebd.host_classify_token(b"1.2.3.4:80") == 2
    assert ebd.host_classify_token(b"[fd00::1]:80") == 1
    assert ebd.host_classify_token(b"01.2.3.4") == 0


def test_generator_is_deterministic_and_shaped():
    a = ebd.generate_host(3, 3, 1000, 2000)
    b_ = ebd.generate_host(3, 3, 1000, 2000)
    for x, y in zip(a, b_):
        assert np.array_equal(x, y)
    # a shard regenerates identically inside a bigger range
    c = ebd.generate_host(3, 3, 0, 3000)
    assert np.array_equal(c[0][1000:], a[0])
    assert np.array_equal(c[1][1000:], a[1])
    ev, lens, offs, payload = ebd.generate_host(3, 3, 0, 20000)
    assert 32 <= lens.min() and lens.max() <= 1100
    assert 230 <= lens.mean() <= 285, lens.mean()
    assert 0.05 < (ev["flags"] & ebd.FLAG_SSL).astype(bool).mean() < 0.25
    ev2, l2, o2, p2 = ebd.generate_host(2, 2, 0, 100)
    assert (l2 == 64).all()
    assert p2[:64].tobytes() == b"GET /index.html HTTP/1.1\r\nHost: 10.0.0.1:8080\r\nAccept: */*xx\r\n\r\n"
    ev1, l1, o1, p1 = ebd.generate_host(1, 0, 0, 10)
    assert (l1 == 35).all() and (ev1["pid"] == 1000).all()
    _, l16, o16, _ = ebd.generate_host(3, 3, 0, 100, align=16)
    assert (o16 % 16 == 0).all()


def test_word_skip_states_are_printable_self_loops():
    """k_fresh skips a 4-byte word without table reads when its start state is di.vl0 or
    di.vl1 and every byte is in [0x20, 0x7e]: exact only if those states step to themselves
    on each such byte (the generic header-value states, HEADER_VALUE of a non-Host,
    non-client key, HttpRequestParser.cpp:321-352 with V-class = printable ASCII)."""
    info = ebd.dfa_info()
    T = ebd.dfa_next()
    vls = [v for v in (info["vl0"], info["vl1"]) if v != 0xFFFFFFFF]
    assert len(vls) == 2 and all(v not in (info["fin0"], info["fin1"], info["inv"]) for v in vls)
    for v in vls:
        assert np.all(T[v, 0x20:0x7F] == v)
        assert T[v, ord("\r")] != v  # CR ends the value


# ---------------------------------------------------------------------------------
# The session path's DFA walker (dfa_parse) against the generic parser gp_step: the same
# chunks, the same consumed counts and outcome, the same spans and sticky key.
# ---------------------------------------------------------------------------------
def _walkers_agree(chunks, flags=UNENC, reset_between=False):
    cg, sg, data = ebd.host_gp_parse(chunks, flags, reset_between)
    cd, sd, _ = ebd.host_gp_parse(chunks, flags, reset_between, walker="dfa")
    assert cd == cg, (chunks, cd, cg)
    fin = {10: 10, 11: 11}
    assert fin.get(sd["state"], -1) == fin.get(sg["state"], -1), (chunks, sd, sg)
    assert sd["cipkey"] == sg["cipkey"], (chunks, sd, sg)
    if sg["state"] == 10:
        keys = ["url_start", "url_len", "host_start", "host_len", "mcand"]
        if sg["f"] & 2:
            keys += ["cip_start", "cip_len"]
        assert {k: sd[k] for k in keys} == {k: sg[k] for k in keys}, (chunks, sd, sg)
        assert sd["f"] & (1 | 2 | 8) == sg["f"] & (1 | 2 | 8), (chunks, sd, sg)


def test_dfa_walker_equals_generic_parser_on_vectors(vectors):
    for case in vectors["parser_valid"] + vectors["parser_invalid"]:
        chunks = [b(c) for c in case["chunks"]]
        _walkers_agree(chunks, SSL if case.get("is_https") else UNENC)
        whole = b"".join(chunks)
        for cut in range(0, len(whole) + 1, 3):
            _walkers_agree([whole[:cut], whole[cut:]])


def test_dfa_walker_length_cap_and_sticky_key():
    for total in (8193, 8194):
        req = b"GET /" + b"a" * (total - 18) + b" HTTP/1.1\r\n\r\n"
        _walkers_agree([req[:8192], req[8192:]])
        _walkers_agree([req[:100], req[100:5000], req[5000:]])
    first = b"GET / HTTP/1.1\r\nX-Forwarded-For: 1.2.3.4\r\n\r\n"
    second = b"GET / HTTP/1.1\r\nTrue-Client-IP: 5.6.7.8\r\nx-forwarded-for: 9.9.9.9\r\n\r\n"
    _walkers_agree([first, second], reset_between=True)
    cons, st, data = ebd.host_gp_parse([first, second], reset_between=True, walker="dfa")
    base = len(first)
    assert data[base + st["cip_start"]:base + st["cip_start"] + st["cip_len"]] == b"9.9.9.9"


def test_dfa_walker_random_sessions():
    """Keep-alive sessions of mutated requests cut at random points: every prefix of the
    chunk list through both walkers (reset after each finished request, as a kept session)."""
    rng = random.Random(11)
    keys = ["X-Forwarded-For", "true-client-ip", "X-Client-IP", "x-http-client-ip", "Rproxy_Remote_Address",
            "rproxy_remote_addressXYZ", "X-Forwarded-Fo", "Host", "User-Agent"]
    alphabet = b"GETPOS /:\r\n ,.[]abcXx-_0123456789\x01\x7f"
    for it in range(600):
        reqs = []
        for _ in range(rng.randint(1, 4)):
            hdrs = [b"Host: h%d.example:80" % rng.randint(0, 9)] if rng.random() < 0.8 else []
            for _ in range(rng.randint(0, 3)):
                k = rng.choice(keys).encode()
                if rng.random() < 0.2:
                    k = k.replace(b"-", b" - ", 1)
                hdrs.append(k + b":" + b" " * rng.randint(0, 2) + rng.choice(
                    [b"1.2.3.4", b"[2001:db8::1]:80", b"10.0.0.1, 8.8.8.8", b"x", b"fd00::1"]))
            rng.shuffle(hdrs)
            r = bytearray((b"POST " if rng.random() < 0.2 else b"GET ") + b"/p%d?q=1 HTTP/1.%d\r\n" % (
                rng.randint(0, 99), rng.randint(0, 1)) + b"".join(h + b"\r\n" for h in hdrs) + b"\r\n")
            if rng.random() < 0.3:
                for _ in range(rng.randint(1, 2)):
                    k = rng.randrange(len(r))
                    r[k] = rng.choice(alphabet)
            reqs.append(bytes(r))
        stream = b"".join(reqs)
        cuts = sorted(rng.sample(range(1, len(stream)), min(len(stream) - 1, rng.randint(1, 6))))
        chunks = [stream[a:b] for a, b in zip([0] + cuts, cuts + [len(stream)])]
        for k in range(1, len(chunks) + 1):
            _walkers_agree(chunks[:k], SSL if it & 1 else UNENC, reset_between=True)
