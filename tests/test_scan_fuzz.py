"""The structural fast path (k_fresh, ebd_scan.h) against the oracle on mutated requests.
CPU only: the host twin runs the same __host__ __device__ code as the kernel, with the buffer
at every alignment inside its tile and "\\r\\n" filler around it."""
import random

import pytest

import ebd
from test_host_semantics import NEW4, check_fresh_against_oracle, scan_shifted

# bytes that sit on a span edge of the state machine (HttpRequestParser.cpp:47-65, 162-364)
EDGE = b" :\r\n\t\x01\x7f\x80\xff[],.-_/?#%\"<>\\^`{|}~@!$&'()*+;=AZaz09Hh"

BASES = [
    b"GET /a/b?c=1 HTTP/1.1\r\nHost: svc1.example.com:8080\r\nUser-Agent: Mozilla/5.0 (X11)\r\nAccept: */*\r\n\r\n",
    b"POST /x HTTP/1.0\r\nHost: 10.1.2.7:8001\r\nX-Forwarded-For: 8.8.8.8, 10.0.0.1\r\nContent-Length: 3\r\n\r\nabc",
    b"GET /i HTTP/1.1\r\nTrue-Client-IP: [fd00::1]:443\r\nHost: [fd00::7]:8443\r\nA: b\r\n\r\n",
    b"GET / HTTP/1.1\r\nrproxy_remote_address: 1.2.3.4\r\nX-Client-IP: 5.6.7.8\r\nHost: h\r\n\r\n",
    b"GET /q HTTP/1.1\r\nX-HTTP-Client-IP: 2001:db8::5\r\nhost: H\r\nx-forwarded-for: 1.1.1.1\r\n\r\n",
]


def mutate(rng, buf):
    b = bytearray(buf)
    for _ in range(rng.randint(1, 3)):
        op = rng.random()
        k = rng.randrange(len(b) + 1)
        c = EDGE[rng.randrange(len(EDGE))]
        if op < 0.4 and k < len(b):
            b[k] = c
        elif op < 0.7:
            b.insert(k, c)
        elif op < 0.85 and k < len(b):
            del b[k]
        else:
            b = b[:k]
    return bytes(b)


@pytest.mark.parametrize("shift", [0, 5, 15])
def test_scan_mutations_against_oracle(shift):
    rng = random.Random(1234 + shift)
    fn = scan_shifted(shift)
    for it in range(1500):
        buf = mutate(rng, BASES[it % len(BASES)])
        flags = NEW4 if it & 1 else ebd.FLAG_IPV6 | ebd.FLAG_SSL | ebd.FLAG_NEW_DATA
        src = b"\x0a\0\0\1" if it & 2 else bytes(15) + b"\x01"
        check_fresh_against_oracle(buf, flags=flags, src=src, fn=fn)


def test_scan_header_shapes_against_oracle():
    """Keys of every length around the client-IP keys', case variants, spaces in keys (the
    generic-parser branch), duplicate and empty Host values, empty keys, partial keys + CR."""
    keys = [b"host", b"HoSt", b"hos", b"hostt", b"x-client-ip", b"X-Client-Ip", b"x-client-iq", b"true-client-ip",
            b"x-forwarded-for", b"X-FORWARDED-FOR", b"x-http-client-ip", b"rproxy_remote_address",
            b"RPROXY_REMOTE_ADDRESSxyz", b"rproxy_remote_addres", b"h ost", b" host", b"host ", b"", b"a" * 40,
            b"x_client_ip", b"user-agent"]
    vals = [b"1.2.3.4", b" 1.2.3.4", b"[::1]:80", b"a b", b"", b"h:1", b"x\x01", b"1.2.3.4 , 5.6.7.8"]
    fn0, fn9 = scan_shifted(0), scan_shifted(9)
    slow = 0
    for k in keys:
        for v in vals:
            for tail in (b"\r\n\r\n", b"\r\nHost: z\r\n\r\n", b"\r\n", b"\r\nFoo\r\n"):
                buf = b"GET /p HTTP/1.1\r\n" + k + b":" + v + tail
                check_fresh_against_oracle(buf, fn=fn0)
                check_fresh_against_oracle(buf, fn=fn9)
                slow += ebd.host_scan(buf, want_slow=True)[2] == 1
    assert slow > 0  # the generic-parser branch ran


def test_scan_key_equals_dfa_key():
    """Both fast paths key a FINISHED request alike (keyed SipHash of pid + host + url)."""
    ev, lens, offs, payload = ebd.generate_host(3, 9, 0, 1500)
    pay = payload.tobytes()
    for i in range(len(ev)):
        buf = pay[int(offs[i]):int(offs[i]) + int(lens[i])]
        a = ebd.host_fresh(buf, int(ev["pid"][i]), int(ev["flags"][i]), ev["sourceIP"][i].tobytes())
        for sh in (0, 11):
            b_ = ebd.host_scan(buf, int(ev["pid"][i]), int(ev["flags"][i]), ev["sourceIP"][i].tobytes(), shift=sh)
            assert a[0].tobytes() == b_[0].tobytes(), i
            assert a[1] == b_[1], i


def test_scan_fast_path_takes_config3():
    """scan_fast (the straight-line form) decides nearly every config-3 buffer; the rest go
    to scan_event.  Both agree with the oracle (test_host_semantics runs every path)."""
    ev, lens, offs, payload = ebd.generate_host(3, 3, 0, 3000)
    pay = payload.tobytes()
    paths = [0, 0, 0]
    for i in range(len(ev)):
        buf = pay[int(offs[i]):int(offs[i]) + int(lens[i])]
        paths[ebd.host_scan(buf, int(ev["pid"][i]), int(ev["flags"][i]), ev["sourceIP"][i].tobytes(),
                            want_slow=True)[2]] += 1
    assert paths[0] >= 0.97 * len(ev), paths
