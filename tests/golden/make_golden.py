#!/usr/bin/env python3
"""Writes tests/golden/reference_vectors.json.

The vectors are DATA transcribed from the reference's own unit tests (inputs and
expected outputs only) plus the survey's probe observations of the compiled
reference (marked [probe]).  Line numbers refer to the
dynatrace-oss/eBPF-Discovery checkout the survey used.

  python tests/golden/make_golden.py     # rewrites reference_vectors.json
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

FLAG_IPV4, FLAG_IPV6, FLAG_UNENC, FLAG_SSL, FLAG_NEW, FLAG_END = 2, 4, 8, 16, 32, 64


def chunk(s, n):
    """chunkString, libhttpparser/test/HttpRequestParserTest.cpp:26-34"""
    return [s[i:i + n] for i in range(0, len(s), n)]


def valid(chunks, method, url, protocol, host, ips, https=False, finished=True, total=None):
    if total is None:
        total = sum(len(c) for c in chunks)
    return dict(chunks=chunks, method=method, url=url, protocol=protocol, host=host,
                client_ip=ips, is_https=https, finished=finished, total=total)


BODY_REQ = ("POST /example/ HTTP/1.1\r\nHost: example.com\r\nUser-Agent: curl/7.81.0\r\nAccept: */*\r\n"
            "X-Forwarded-For: 192.168.0.1:8080, 10.0.0.1, [2001:0db8:85a3::8a2e:0370:7334]\r\n\r\n"
            "{\"name\":\"example\"}\r\n")

# HttpRequestParserTest.cpp:193-282 (INSTANTIATE ... HttpRequestDataParsingTest)
PARSER_VALID = [
    valid(["GET /example HTTP/1.1\r\nHost: example.com\r\n\r\n"], "GET", "/example", "HTTP/1.1", "example.com", []),
    valid(["GET /example HTTP/1.1\r\nHOST: example.com\r\n\r\n"], "GET", "/example", "HTTP/1.1", "example.com", []),
    valid(["POST /example HTTP/1.1\r\nHost: example.com\r\n\r\n"], "POST", "/example", "HTTP/1.1", "example.com", []),
    valid(["POST /example HTTP/1.1\r\nHOST: example.com\r\n\r\n"], "POST", "/example", "HTTP/1.1", "example.com", []),
    valid(["GET /example HTTP/1.0\r\nHost: example.com\r\n\r\n"], "GET", "/example", "HTTP/1.0", "example.com", []),
    valid(["POST /example HTTP/1.0\r\nHost: example.com\r\n\r\n"], "POST", "/example", "HTTP/1.0", "example.com", []),
    valid(["GET /example HTTP/1.1\r\nHost: example.com\r\n\r"], "GET", "/example", "HTTP/1.1", "example.com", [],
          False, False),
    valid(["GET /Hello%20World/index.html HTTP/1.1\r\nHost:  example.com\r\nx-forwarded-for:  127.0.0.1\r\n\r\n"],
          "GET", "/Hello%20World/index.html", "HTTP/1.1", "example.com", ["127.0.0.1"]),
    valid(["GET / HTTP/1.1\r\n\r\n"], "GET", "/", "HTTP/1.1", "", []),
    valid(chunk("GET /example HTTP/1.1\r\nHost: example.com\r\n\r\n", 8), "GET", "/example", "HTTP/1.1",
          "example.com", []),
    valid(chunk("GET /example HTTP/1.1\r\nHost: example.com\r\nX-Forwarded-For: 0.0.0.0\r\n\r\n", 1), "GET",
          "/example", "HTTP/1.1", "example.com", ["0.0.0.0"]),
    valid([BODY_REQ], "POST", "/example/", "HTTP/1.1", "example.com",
          ["192.168.0.1", "10.0.0.1", "2001:0db8:85a3::8a2e:0370:7334"], False, True, 163),
    valid([BODY_REQ], "POST", "/example/", "HTTP/1.1", "example.com",
          ["192.168.0.1", "10.0.0.1", "2001:0db8:85a3::8a2e:0370:7334"], True, True, 163),
    valid(chunk("GET /example/ HTTP/1.1\r\nHost: example.com\r\nX-Forwarded-For: 10.0.0.1\r\nUser-Agent: "
                "curl/7.81.0\r\nAccept: */*\r\nx-forwarded-for: 127.0.0.1,[2001:0db8:85a3::8a2e:0370:7335]:1234\r\n\r\n", 2),
          "GET", "/example/", "HTTP/1.1", "example.com", ["10.0.0.1", "127.0.0.1", "2001:0db8:85a3::8a2e:0370:7335"]),
    valid(["GET /example HTTP/1.1\r\nHost: example.com\r\nReferer: https://example.com/\r\n\r\n"], "GET", "/example",
          "HTTP/1.1", "example.com", []),
    valid(["GET /example HTTP/1.1\r\nHost: example.com\r\nSec-CH-UA: \"Chromium\";v=\"124\"\r\n\r\n"], "GET",
          "/example", "HTTP/1.1", "example.com", []),
    valid(chunk("GET / HTTP/1.1\r\n", 1), "GET", "/", "HTTP/1.1", "", [], False, False),
    valid(["GET /"], "GET", "/", "", "", [], False, False),
    valid(["", ""], "", "", "", "", [], False, False),
]

# HttpRequestParserTest.cpp:284-300 (INSTANTIATE ... HttpRequestParserTestInvalid)
PARSER_INVALID = [
    dict(chunks=["get /example HTTP/1.1\r\nHost: example.com\r\n\r\n"], total=1),
    dict(chunks=["post /example HTTP/1.1\r\nHost: example.com\r\n\r\n"], total=1),
    dict(chunks=["POST  HTTP/1.1\r\nHost: example.com\r\n\r\n"], total=6),
    dict(chunks=["GET / HTTP/1.1\r\nHost: \r\n\r\n"], total=23),
    dict(chunks=["GET  / HTTP/1.1\r\nHost: example.com\r\n\r\n"], total=5),
    dict(chunks=["GET /  HTTP/1.1\r\nHost: example.com\r\n\r\n"], total=7),
    dict(chunks=["GET / HTTP/1.1 \r\nHost: example.com\r\n\r\n"], total=15),
    dict(chunks=["GET / HTTP/1.1\nHost: example.con\n\n"], total=15),
    dict(chunks=["GET /example", "HTTP/1.1\r\nHost: example.com\r\n\r\n"], total=21),
    dict(chunks=["\r\nGET / HTTP/1.1\r\nHost: example.com\r\n\r\n"], total=1),
    dict(chunks=["\nGET / HTTP/1.1\r\nHost: example.com\r\n\r\n"], total=1),
    dict(chunks=["GET / HTTP/0.0\r\nHost: example.com\r\n\r\n"], total=12),
    dict(chunks=["GET http://example.com HTTP/1.1\r\nHost: example.com\r\n\r\n"], total=5),
]

# HttpRequestParserTest.cpp:75-150 (testParseXForwardedFor)
CLIENT_IP_SPLIT = [
    ("fe80:0000:0000:0000:0000:0000:0000:0005", ["fe80:0000:0000:0000:0000:0000:0000:0005"]),
    ("203.0.113.195, 70.41.3.18, 150.172.238.178", ["203.0.113.195", "70.41.3.18", "150.172.238.178"]),
    ("203.0.113.195", ["203.0.113.195"]),
    ("2001:db8:85a3:8d3:1319:8a2e:370:7348", ["2001:db8:85a3:8d3:1319:8a2e:370:7348"]),
    ("203.0.113.195:41237, 198.51.100.100:38523", ["203.0.113.195", "198.51.100.100"]),
    ("[2001:db8::1a2b:3c4d]:41237, 198.51.100.100:26321", ["2001:db8::1a2b:3c4d", "198.51.100.100"]),
    ("[2001:db8::aa:bb]", ["2001:db8::aa:bb"]),
    ("203.0.113.195, 2001:db8:85a3:8d3:1319:8a2e:370:7348", ["203.0.113.195", "2001:db8:85a3:8d3:1319:8a2e:370:7348"]),
    ("203.0.113.195,2001:db8:85a3:8d3:1319:8a2e:370:7348,198.51.100.178",
     ["203.0.113.195", "2001:db8:85a3:8d3:1319:8a2e:370:7348", "198.51.100.178"]),
    ("[2001:db8::1]:30943", ["2001:db8::1"]),
]

# libservice/test/AggregatorTest.cpp:69-172 (ServiceAggregatorTest.aggregate).
# Each request: pid, host, url, flags (None = no flags -> meta.flags 0, isHttps false),
# mock = the IpAddressCheckerMock verdict armed for that call (None = checker not called).
# real_src = a source address that the real IpAddressCheckerImpl classifies the same way
# as the mock verdict (used where the path under test has no mock injection point).
AGG_REQUESTS = [
    dict(pid=100, host="host", url="/url", flags=FLAG_IPV4, mock=True, real_src="8.8.8.8"),
    dict(pid=100, host="host", url="/url", flags=None, mock=None, real_src=None),
    dict(pid=100, host="host", url="/url2", flags=FLAG_IPV4, mock=False, real_src="10.0.0.1"),
    dict(pid=200, host="host", url="/url2", flags=FLAG_IPV4, mock=True, real_src="8.8.8.8"),
    dict(pid=200, host="host", url="/url2", flags=FLAG_IPV4, mock=False, real_src="10.0.0.1"),
    dict(pid=200, host="host", url="/url2", flags=FLAG_IPV4, mock=True, real_src="8.8.4.4"),
    dict(pid=400, host="google.com", url="/url123", flags=FLAG_IPV4 | FLAG_UNENC, mock=True, real_src="8.8.8.8"),
    dict(pid=500, host="8.8.8.8", url="/url123", flags=FLAG_IPV4 | FLAG_UNENC, mock=True, real_src="1.1.1.1"),
    dict(pid=600, host="dynatrace.com", url="/url123", flags=FLAG_IPV4 | FLAG_SSL, mock=True, real_src="8.8.8.8"),
    dict(pid=700, host="[::1]", url="/url123", flags=FLAG_IPV6 | FLAG_UNENC, mock=False, real_src="fd00::1"),
    dict(pid=800, host="[2001:0db8:85a3:0001:0000:0000:0000:0000]", url="/url123", flags=FLAG_IPV6 | FLAG_SSL,
         mock=True, real_src="2001:4860:4860::8888"),
    dict(pid=900, host="[2001:0db8:85a3:0001::]", url="/url123", flags=FLAG_IPV6 | FLAG_SSL, mock=True,
         real_src="2606:4700::1111"),
]
AGG_EXPECTED = [
    dict(pid=100, endpoint="host/url", domain="host", scheme="http", internal=0, external=1),
    dict(pid=100, endpoint="host/url2", domain="host", scheme="http", internal=1, external=0),
    dict(pid=200, endpoint="host/url2", domain="host", scheme="http", internal=1, external=2),
    dict(pid=400, endpoint="google.com/url123", domain="google.com", scheme="http", internal=0, external=1),
    dict(pid=500, endpoint="8.8.8.8/url123", domain="8.8.8.8", scheme="http", internal=0, external=1),
    dict(pid=600, endpoint="dynatrace.com/url123", domain="dynatrace.com", scheme="https", internal=0, external=1),
    dict(pid=700, endpoint="[::1]/url123", domain="[::1]", scheme="http", internal=1, external=0),
    dict(pid=800, endpoint="[2001:0db8:85a3:0001:0000:0000:0000:0000]/url123",
         domain="[2001:0db8:85a3:0001:0000:0000:0000:0000]", scheme="https", internal=0, external=1),
    dict(pid=900, endpoint="[2001:0db8:85a3:0001::]/url123", domain="[2001:0db8:85a3:0001::]", scheme="https",
         internal=0, external=1),
]

# libservice/test/IpAddressCheckerTest.cpp:38-251 — (address, expected isV4AddressExternal)
V4_RESERVED_INTERNAL = [
    "0.0.0.0", "0.255.255.255", "0.54.189.245", "0.128.0.1",
    "10.0.0.0", "10.255.255.255", "10.54.189.245", "10.128.0.1",
    "100.64.0.0", "100.127.255.255", "100.64.128.0", "100.66.0.1",
    "127.0.0.0", "127.255.255.255", "127.0.0.1", "127.128.0.1",
    "169.254.0.0", "169.254.255.255", "169.254.128.0", "169.254.192.1",
    "172.16.0.0", "172.31.255.255", "172.20.0.0", "172.24.0.1",
    "192.0.0.0", "192.0.0.255", "192.0.0.128", "192.0.0.1",
    "192.0.2.0", "192.0.2.255", "192.0.2.128", "192.0.2.1",
    "192.88.99.0", "192.88.99.255", "192.88.99.128", "192.88.99.1",
    "192.168.0.0", "192.168.255.255", "192.168.128.0", "192.168.192.1",
    "198.18.0.0", "198.19.255.255", "198.18.128.0", "198.18.192.1",
    "198.51.100.0", "198.51.100.255", "198.51.100.128", "198.51.100.1",
    "203.0.113.0", "203.0.113.255", "203.0.113.128", "203.0.113.1",
    "224.0.0.0", "239.255.255.255", "225.128.0.0", "230.0.0.1",
    "233.252.0.0", "233.252.0.255", "233.252.0.128", "233.252.0.1",
    "240.0.0.0", "255.255.255.254", "241.128.0.0", "248.0.0.1",
    "255.255.255.255",
]
# IpAddressCheckerTest.cpp:253-263 LocalIfceIpSrc: interface 115.89.3.7 with mask s_addr 0x0000ffff
V4_IFACE_CASE = dict(v4_ifaces=[["115.89.3.7", "255.255.0.0"]], cases=[["115.89.3.7", False]])
# IpAddressCheckerTest.cpp:272-328 — (address, expected isV6AddressExternal)
V6_CASES = [
    ["::FFFF:192.168.0.5", False], ["2001:0db8:85a3:0000:0000:8a2e:0370:7334", True],
    ["::ffff:0:0:0", False], ["0000:0000:0000:0000:fffe:ffff:ffff:ffff", True],
    ["0000:0000:0000:0000:ffff:0001:ffff:ffff", True],
    ["64:ff9b::", False], ["0064:ff9a:ffff:ffff:ffff:ffff:ffff:ffff", True],
    ["0064:ff9b:0000:0000:0000:0001:0000:0000", True],
    ["fc00::1", False], ["fdff:ffff:ffff:ffff:ffff:ffff:ffff:ffff", False],
    ["fbff:ffff:ffff:ffff:ffff:ffff:ffff:ffff", True], ["fe00::", True],
    ["fec0::", False], ["feff:ffff:ffff:ffff:ffff:ffff:ffff:ffff", False], ["ff00::", True],
    ["fe80::", False], ["febf:ffff:ffff:ffff:ffff:ffff:ffff:ffff", False],
    ["fe7f:ffff:ffff:ffff:ffff:ffff:ffff:ffff", True],
    ["::1", False], ["::", True], ["::2", True],
]
# IpAddressCheckerTest.cpp:331-345 Ipv6NetworkSubnet
V6_IFACE_CASE = dict(v6_ifaces=[["2001:db8:85a3::8a2e:370:7336", "ffff:ffff:ffff:ffff::"]],
                     cases=[["2001:0db8:85a3:0000:0000:0000:0000:0000", False],
                            ["2001:0db8:85a3:0001:0000:0000:0000:0000", True],
                            ["2001:0db8:85a3:2::", True],
                            ["2001:0db8:85a2:ffff:ffff:ffff:ffff:ffff", True]])
# libservice/test/IpAddressTest.cpp:28-63 (inet_ntop formatting)
NTOP = [
    dict(v4=[192, 168, 0, 1], text="192.168.0.1"),
    dict(v6=[0x20, 0x01, 0x0d, 0xb8, 0x85, 0xa3, 0x08, 0xd3, 0x13, 0x19, 0x83, 0x01, 0x23, 0x45, 0x67, 0x89],
         text="2001:db8:85a3:8d3:1319:8301:2345:6789"),
    dict(v6=[0] * 16, text="::"),
]
# libebpfdiscovery/test/LRUCacheTest.cpp:26-95 — op scripts over a capacity-3 cache
LRU_SCRIPTS = [
    dict(name="testInsertAndFind", capacity=3,
         ops=[["insert", 1, "one"], ["insert", 2, "two"], ["insert", 3, "three"],
              ["find", 1, "one"], ["find", 2, "two"], ["find", 3, "three"]]),
    dict(name="testErase", capacity=3,
         ops=[["insert", 1, "one"], ["insert", 2, "two"], ["insert", 3, "three"], ["erase", 2],
              ["find", 1, "one"], ["find", 2, None], ["find", 3, "three"]]),
    dict(name="testInsertExistingKey", capacity=3,
         ops=[["insert", 1, "one"], ["insert", 2, "two"], ["insert", 3, "three"], ["insert", 2, "two_updated"],
              ["find", 1, "one"], ["find", 2, "two_updated"], ["find", 3, "three"]]),
    dict(name="testUpdate", capacity=3,
         ops=[["insert", 1, "one"], ["insert", 2, "two"], ["insert", 3, "three"], ["update", 2, "two_updated"],
              ["find", 1, "one"], ["find", 2, "two_updated"], ["find", 3, "three"]]),
    dict(name="testInsertBeyondCapacity", capacity=3,
         ops=[["insert", 1, "one"], ["insert", 2, "two"], ["insert", 3, "three"], ["insert", 4, "four"],
              ["insert", 5, "five"], ["find", 1, None], ["find", 2, None], ["find", 3, "three"],
              ["find", 4, "four"], ["find", 5, "five"]]),
]

# Survey probes of the compiled reference (marked [probe]).
PROBE_PARSER = [
    dict(note="GETT is invalid at byte 4", chunks=["GETT / HTTP/1.1\r\n\r\n"], state="INVALID", total=4),
    dict(note="partial key then CR finishes", chunks=["GET / HTTP/1.1\r\nFoo\r\n"], state="FINISHED", total=21),
    dict(note="first host byte may be any V-class byte", chunks=["GET / HTTP/1.1\r\nHost: /weird\r\n\r\n"],
         state="FINISHED", host="/weird"),
    dict(note="spaces inside the key are skipped", chunks=["GET / HTTP/1.1\r\nHo st : h\r\n\r\n"],
         state="FINISHED", host="h"),
    dict(note="duplicate Host is invalid", chunks=["GET / HTTP/1.1\r\nHost: a\r\nHost: b\r\n\r\n"],
         state="INVALID", total=30),
    dict(note="trailing space in host is invalid", chunks=["GET / HTTP/1.1\r\nHost: a \r\n\r\n"],
         state="INVALID", total=24),
    dict(note="URL with CR is invalid", chunks=["GET /a\rb HTTP/1.1\r\n\r\n"], state="INVALID", total=7),
    dict(note="byte >= 0x80 is invalid in the url", chunks=["GET /aÿ HTTP/1.1\r\n\r\n"], state="INVALID", total=7),
    dict(note="truncated rproxy key is a client key",
         chunks=["GET / HTTP/1.1\r\nrproxy_remote_addressXYZ: 1.2.3.4\r\n\r\n"], state="FINISHED",
         client_ip=["1.2.3.4"]),
    dict(note="8193-byte request is accepted", lengths=[8192, 1], state="FINISHED", total=8193),
    dict(note="8194-byte request is invalid after 8193 bytes", lengths=[8192, 2], state="INVALID", total=8193),
]
# ", 1.2.3.4" is a survey probe; the other three are boost::split token_compress_on semantics
# (boost 1.83, absent here) that no reference test pins: parity unpinned, kept as restatement checks.
PROBE_SPLIT = [(", 1.2.3.4", ["", "1.2.3.4"]), ("", [""]), ("a,,b", ["a", "b"]), ("a,", ["a", ""])]
# "01.2.3.4" is a survey probe; the rest are glibc inet_pton semantics (also checked against this host's glibc).
PROBE_PTON4 = [("01.2.3.4", None), ("1.2.3.4", [1, 2, 3, 4]), ("256.1.1.1", None), ("", None)]
# Config 1 ([probe]): 1000 events of one literal, pid 1000, fd 5,
# sessionID 1..1000, bufferSeq 1, flags IPV4|UNENCRYPTED|NEW_DATA, source 127.0.0.1.
CONFIG1 = [
    dict(payload="GET / HTTP/1.1\r\nHost: 127.0.0.1\r\n\r\n", n=1000,
         services=[dict(pid=1000, endpoint="127.0.0.1/", domain="127.0.0.1", scheme="http", internal=1000,
                        external=0)], saved_sessions=0),
    dict(payload="GET / HTTP/1.1\r\nHost: 127.0.0.1", n=1000, services=[], saved_sessions=1000),
]

# libebpfdiscovery/test/JsonTest.cpp:62-173 — services (Service.h fields; nets = sizes of the
# externalIPv4_16 / _24 / IPv6 maps) and the exact text boost::json::ext::print writes.
# scheme "" is a default-constructed Service's (JsonTest builds them without one).
def _svc(pid, ep, dom, sch, i, e, nets=(0, 0, 0)):
    return dict(pid=pid, endpoint=ep, domain=dom, scheme=sch, internal=i, external=e, nets=list(nets))


JSON_CASES = [
    dict(name="servicesToJson", services=[
        _svc(1, "/endpoint/1", "", "", 1, 2), _svc(2, "/endpoint/1", "", "", 1, 2), _svc(3, "/endpoint/2", "", "", 1, 2),
        _svc(4, "google.com/endpoint/3", "google.com", "http", 1, 2),
        _svc(5, "dynatrace.com/endpoint/4", "dynatrace.com", "https", 1, 2)],
        expected='{"service":['
                 '{"pid":1,"endpoint":"/endpoint/1","internalClientsNumber":1,"externalClientsNumber":2},'
                 '{"pid":2,"endpoint":"/endpoint/1","internalClientsNumber":1,"externalClientsNumber":2},'
                 '{"pid":3,"endpoint":"/endpoint/2","internalClientsNumber":1,"externalClientsNumber":2},'
                 '{"pid":4,"endpoint":"google.com/endpoint/3","domain":"google.com","scheme":"http",'
                 '"internalClientsNumber":1,"externalClientsNumber":2},'
                 '{"pid":5,"endpoint":"dynatrace.com/endpoint/4","domain":"dynatrace.com","scheme":"https",'
                 '"internalClientsNumber":1,"externalClientsNumber":2}]}'),
    dict(name="servicesToJsonNetworkCounters", services=[
        _svc(1, "/endpoint/1", "", "", 1, 3, (2, 3, 0)), _svc(2, "/endpoint/1", "", "", 1, 3, (2, 3, 0)),
        _svc(3, "/endpoint/2", "", "", 1, 3, (2, 3, 0)),
        _svc(4, "google.com/endpoint/3", "google.com", "http", 1, 2, (0, 0, 2)),
        _svc(5, "dynatrace.com/endpoint/4", "dynatrace.com", "https", 1, 2, (0, 0, 2))],
        expected='{"service":[{"pid":1,"endpoint":"/endpoint/1","internalClientsNumber":1,"externalClientsNumber":3,'
                 '"externalIPv4_16ClientNets":2,"externalIPv4_24ClientNets":3},{"pid":2,"endpoint":"/endpoint/1",'
                 '"internalClientsNumber":1,"externalClientsNumber":3,"externalIPv4_16ClientNets":2,'
                 '"externalIPv4_24ClientNets":3},{"pid":3,"endpoint":"/endpoint/2","internalClientsNumber":1,'
                 '"externalClientsNumber":3,"externalIPv4_16ClientNets":2,"externalIPv4_24ClientNets":3},'
                 '{"pid":4,"endpoint":"google.com/endpoint/3","domain":"google.com","scheme":"http",'
                 '"internalClientsNumber":1,"externalClientsNumber":2,"externalIPv6ClientsNets":2},'
                 '{"pid":5,"endpoint":"dynatrace.com/endpoint/4","domain":"dynatrace.com","scheme":"https",'
                 '"internalClientsNumber":1,"externalClientsNumber":2,"externalIPv6ClientsNets":2}]}'),
]

# libservice/test/AggregatorTest.cpp:174-285 aggregateNetworkCounters: every request at time
# point 0 with the checker mocked to "external"; the expected maps (keys as in_addr s_addr
# values on little-endian x86, i.e. the address bytes in order) and sizes after cleaning at
# 59 min (kept) and 60 min (erased), each followed by clear().
_NC_REQ = [("172.143.4.5", FLAG_IPV4), ("172.143.6.89", FLAG_IPV4), ("172.199.45.55", FLAG_IPV4),
           ("1234:2345:3456:4567:5678:6789:7890:8901", FLAG_IPV6), ("2001:4860:4860:0000:0000:0000:0000:8888", FLAG_IPV6)]
AGG_NETCOUNTERS = dict(
    requests=[dict(pid=pid, host="host", url="/url", client_ip=ip, flags=fl | extra, time_ns=0)
              for pid, extra in ((100, FLAG_UNENC), (200, FLAG_SSL)) for ip, fl in _NC_REQ],
    expected=[dict(pid=100, endpoint="host/url", domain="host", scheme="http", internal=0, external=5),
              dict(pid=200, endpoint="host/url", domain="host", scheme="https", internal=0, external=5)],
    nets_v4_16=["ac8f", "acc7"], nets_v4_24=["ac8f04", "ac8f06", "acc72d"],
    nets_v6=["200148604860", "123423453456"],
    after_59min=dict(services=2, external=0, sizes=[2, 3, 2]),
    after_60min=dict(services=0),
)


def main():
    out = dict(
        source="dynatrace-oss/eBPF-Discovery unit tests (transcribed data) + SURVEY.md probes",
        parser_valid=PARSER_VALID, parser_invalid=PARSER_INVALID,
        client_ip_split=[dict(value=v, expected=e) for v, e in CLIENT_IP_SPLIT],
        aggregator=dict(requests=AGG_REQUESTS, expected=AGG_EXPECTED),
        v4_reserved_internal=V4_RESERVED_INTERNAL, v4_iface=V4_IFACE_CASE, v6_cases=V6_CASES,
        v6_iface=V6_IFACE_CASE, ntop=NTOP, lru=LRU_SCRIPTS,
        probe_parser=PROBE_PARSER, probe_split=[dict(value=v, expected=e) for v, e in PROBE_SPLIT],
        probe_pton4=[dict(text=t, expected=e) for t, e in PROBE_PTON4], config1=CONFIG1,
        json_services=JSON_CASES, agg_netcounters=AGG_NETCOUNTERS,
    )
    with open(os.path.join(HERE, "reference_vectors.json"), "w") as f:
        json.dump(out, f, indent=1, ensure_ascii=True)
        f.write("\n")


if __name__ == "__main__":
    main()
