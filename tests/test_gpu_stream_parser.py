"""httpparser::HttpRequestParser one stream at a time on the GPU (ebd_parse_streams, the
ebd.StreamParser / ebdamd::HttpRequestParser facade) against HttpRequestParserTest.cpp's own
vectors and against the oracle's Parser (oracle.c, the restatement of HttpRequestParser.cpp)
on random chunkings, mutations and reset sequences: consumed bytes per call, isFinished /
isInvalidState, and every HttpRequest field (method, url, protocol, host, clientIPKey, the whole
clientIp vector, isHttps)."""
import random

import numpy as np
import pytest

import ebd
import oracle_py as O

pytestmark = pytest.mark.gpu

UNENC, SSL = 8, 16


def b(s):
    return s.encode("latin-1") if isinstance(s, str) else s


@pytest.fixture(scope="module")
def ctx():
    c = ebd.Context(max_events=16)
    yield c
    c.close()


def run_chunks(ctx, chunks, flags):
    p = ebd.StreamParser(ctx)
    total = sum(p.parse(b(c), flags) for c in chunks)
    return p, total


def test_reference_valid_vectors(ctx, vectors):
    # HttpRequestParserTest.cpp:152-171 TestValidRequest over :193-286
    for case in vectors["parser_valid"]:
        p, total = run_chunks(ctx, case["chunks"], SSL if case["is_https"] else UNENC)
        assert p.is_finished() == case["finished"], case
        assert not p.is_invalid(), case
        assert total == case["total"], case
        r = p.result
        assert r["method"] == b(case["method"]), case
        assert r["url"] == b(case["url"]), case
        assert r["protocol"] == b(case["protocol"]), case
        assert r["host"] == b(case["host"]), case
        assert r["client_ip"] == [b(x) for x in case["client_ip"]], case
        assert r["is_https"] == case["is_https"], case


def test_reference_invalid_vectors(ctx, vectors):
    # HttpRequestParserTest.cpp:178-191 testInvalidRequest over :288-300
    for case in vectors["parser_invalid"]:
        p, total = run_chunks(ctx, case["chunks"], UNENC)
        assert p.is_finished() and p.is_invalid(), case
        assert total == case["total"], case


def test_reference_client_ip_splits(ctx, vectors):
    # HttpRequestParserTest.cpp:75-150 (parseClientIPValue) through a whole request: the value
    # as the only client-IP header's value
    for case in vectors["client_ip_split"] + vectors["probe_split"]:
        v = b(case["value"])
        req = b"GET / HTTP/1.1\r\nX-Forwarded-For: " + v + b"\r\n\r\n"
        p, _ = run_chunks(ctx, [req], UNENC)
        o = O.Parser()
        o.parse(req, UNENC)
        assert p.result["client_ip"] == o.result()["client_ip"], case
        if o.state == "FINISHED":
            assert p.result["client_ip"] == [b(x) for x in case["expected"]], case


def _same(p, o, ctx_note):
    assert p.is_finished() == (o.state in ("FINISHED", "INVALID")), ctx_note
    assert p.is_invalid() == (o.state == "INVALID"), ctx_note
    r, q = p.result, o.result()
    for k in ("method", "url", "protocol", "host", "client_ip", "is_https"):
        assert r[k] == q[k], (k, r[k], q[k], ctx_note)
    assert r["client_ip_key"].encode() == q["client_ip_key"], ctx_note


def _requests(rng):
    keys = [b"X-Forwarded-For", b"x-client-ip", b"True-Client-IP", b"X-HTTP-Client-IP", b"rproxy_remote_address",
            b"Rproxy_Remote_AddressXYZ", b"X-Forwarded-Forr"]
    vals = [b"1.2.3.4", b"1.2.3.4:80, 5.6.7.8", b"[2001:db8::1]:443", b",10.0.0.1", b"a,,b, c ,", b"[fe80::1]",
            b"01.2.3.4", b" 7.7.7.7 :9 ", b"2001:db8::7"]
    for _ in range(400):
        lines = [rng.choice([b"GET", b"POST"]) + b" /" + bytes(rng.choice(b"abc/%?=") for _ in range(rng.randrange(12))) +
                 b" HTTP/1." + rng.choice([b"0", b"1"])]
        if rng.random() < 0.8:
            lines.append(rng.choice([b"Host", b"HOST", b"Ho st"]) + b": " + rng.choice([b"ex.com", b"[::1]:80", b"h:8"]))
        for _ in range(rng.randrange(4)):
            lines.append(rng.choice(keys) + b":" + b" " * rng.randrange(3) + rng.choice(vals))
        if rng.random() < 0.5:
            lines.append(b"User-Agent: x" * rng.randrange(1, 4))
        req = b"\r\n".join(lines) + b"\r\n\r\n"
        if rng.random() < 0.15:  # one byte mutated: invalid somewhere, or not
            k = rng.randrange(len(req))
            req = req[:k] + bytes([rng.choice(b"\x01 :\r\n,[]a\x80")]) + req[k + 1:]
        yield req


def test_random_requests_chunked_against_oracle(ctx):
    rng = random.Random(55)
    for req in _requests(rng):
        flags = rng.choice([UNENC, SSL])
        cuts = sorted(rng.sample(range(1, len(req)), min(len(req) - 1, rng.randrange(0, 5))))
        chunks = [req[a:z] for a, z in zip([0] + cuts, cuts + [len(req)])] + [b"tail"]
        p, o = ebd.StreamParser(ctx), O.Parser()
        for c in chunks:
            assert p.parse(c, flags) == o.parse(c, flags), (req, chunks)
            _same(p, o, (req, chunks))


def test_reset_keeps_the_client_ip_key(ctx):
    # P:374-379: reset() clears the request but not result.clientIPKey, so the next request's
    # client address comes from the first key's headers only
    p, o = ebd.StreamParser(ctx), O.Parser()
    seq = [b"GET / HTTP/1.1\r\nX-Forwarded-For: 1.2.3.4\r\n\r\n", None,
           b"GET /b HTTP/1.1\r\nX-Client-IP: 5.6.7.8\r\nX-Forwarded-For: 9.9.9.9, 8.8.8.8\r\n\r\n", None,
           b"GET /c HTTP/1.1\r\nX-Client-IP: 5.6.7.8\r\n\r\n"]
    for s in seq:
        if s is None:
            p.reset()
            o.reset()
            continue
        assert p.parse(s, UNENC) == o.parse(s, UNENC)
        _same(p, o, s)
    assert p.result["client_ip_key"] == "x-forwarded-for"


def test_length_cap_and_parse_after_the_end(ctx):
    # P:88-91: a byte is refused once more than 8192 were parsed; P:94-103: a parse() on an
    # ended parser takes one byte
    long_url = b"GET /" + b"a" * 8200
    p, o = ebd.StreamParser(ctx), O.Parser()
    for c in (long_url[:5000], long_url[5000:]):
        assert p.parse(c, UNENC) == o.parse(c, UNENC)
        _same(p, o, "cap")
    assert p.is_invalid()
    p, o = ebd.StreamParser(ctx), O.Parser()
    done = b"GET / HTTP/1.1\r\n\r\nGET / HTTP/1.1\r\n\r\n"
    assert p.parse(done, UNENC) == o.parse(done, UNENC) == 18
    assert p.parse(b"more", UNENC) == o.parse(b"more", UNENC)
    _same(p, o, "after end")


def test_many_streams_in_one_call(ctx):
    # the batch form: n parsers, one chunk each, in one ebd_parse_streams call
    rng = random.Random(7)
    reqs = list(_requests(rng))[:200]
    calls = np.zeros(len(reqs), ebd.PARSE_CALL_DTYPE)
    data = b"".join(reqs)
    at = 0
    for k, r in enumerate(reqs):
        assert ebd.lib().ebd_parser_init(ebd._p(calls["state"][k])) == 0
        calls[k]["data_off"], calls[k]["data_len"], calls[k]["flags"] = at, len(r), UNENC
        at += len(r)
    buf = np.frombuffer(data, np.uint8)
    assert ebd.lib().ebd_parse_streams(ctx.h, ebd._p(calls), len(reqs), ebd._p(buf), len(data)) == 0
    for k, r in enumerate(reqs):
        o = O.Parser()
        assert int(calls[k]["consumed"]) == o.parse(r, UNENC), r
        want = {"UNFINISHED": 0, "FINISHED": 1, "INVALID": 2}.get(o.state, 0)
        assert int(calls[k]["status"]) == want, r


def test_corrupted_state_is_rejected(ctx):
    """A state with a token count past the list is refused before the kernel runs."""
    calls = np.zeros(2, ebd.PARSE_CALL_DTYPE)
    for k in range(2):
        assert ebd.lib().ebd_parser_init(ebd._p(calls["state"][k])) == 0
        calls[k]["data_off"], calls[k]["data_len"] = 0, 4
    calls["state"][1].view(np.uint8)[48:52] = np.frombuffer(np.uint32(40).tobytes(), np.uint8)
    buf = np.frombuffer(b"GET ", np.uint8)
    assert ebd.lib().ebd_parse_streams(ctx.h, ebd._p(calls), 2, ebd._p(buf), 4) == -22
    assert int(calls[0]["consumed"]) == 0  # nothing ran
