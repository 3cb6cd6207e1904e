"""The service report (Discovery::outputServicesToStdout, Discovery.cpp:60-71 with
Json.h:32-71) and the network counters (Aggregator.cpp:89-106, 136-153, 182-209) on CPU:
the product's JSON formatter against the reference's JsonTest vectors, and the oracle's
network maps against AggregatorTest's aggregateNetworkCounters scenario.  No GPU needed."""
import json
import os

import numpy as np

import ebd
import oracle_py as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VEC = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_vectors.json")))
MIN = 60 * 10**9


def records(services):
    """SERVICE_DTYPE records + string blob for [{pid, endpoint, domain, scheme, ...}] (the
    domain must be a substring of the endpoint, as every service's is)."""
    recs = np.zeros(len(services), ebd.SERVICE_DTYPE)
    blob = b""
    for r, s in zip(recs, services):
        ep = s["endpoint"].encode()
        dom = s["domain"].encode()
        r["pid"], r["internal"], r["external"] = s["pid"], s["internal"], s["external"]
        r["https"] = {"": 2, "http": 0, "https": 1}[s["scheme"]]
        r["endpoint_off"], r["endpoint_len"] = len(blob), len(ep)
        r["domain_off"], r["domain_len"] = (ep.index(dom) if dom else 0), len(dom)
        r["nets_v4_16"], r["nets_v4_24"], r["nets_v6"] = s.get("nets", (0, 0, 0))
        blob += ep
    return recs, blob


def test_json_formatter_matches_reference_vectors():
    for case in VEC["json_services"]:
        recs, blob = records(case["services"])
        # JsonTest compares print()'s text; outputServicesToStdout adds std::endl
        assert ebd.format_services_json(recs, blob) == case["expected"].encode() + b"\n", case["name"]


def test_json_formatter_edges():
    assert ebd.format_services_json(np.zeros(0, ebd.SERVICE_DTYPE), b"") == b""  # nothing printed (Discovery.cpp:62-64)
    recs, blob = records([dict(pid=7, endpoint='"\\x/a', domain='"\\x', scheme="http", internal=0, external=0)])
    assert ebd.format_services_json(recs, blob) == (
        b'{"service":[{"pid":7,"endpoint":"\\"\\\\x/a","domain":"\\"\\\\x","scheme":"http",'
        b'"internalClientsNumber":0,"externalClientsNumber":0}]}\n')


def netcounter_oracle(mock):
    o = O.Oracle(network_counters=True)
    nc = VEC["agg_netcounters"]
    if mock:  # IpAddressCheckerMock answering "external" to every call (AggregatorTest.cpp:181-183)
        o.set_mock([1] * len(nc["requests"]))
    for r in nc["requests"]:
        o.set_time(r["time_ns"])
        o.new_request(r["pid"], r["host"].encode(), r["url"].encode(), r["client_ip"].encode(), r["flags"])
    return o, nc


def test_oracle_network_counters_reference_scenario():
    for mock in (True, False):  # the real checker finds every client of the scenario external too
        o, nc = netcounter_oracle(mock)
        want = [(e["pid"], e["endpoint"].encode(), e["domain"].encode(), e["scheme"].encode(), e["internal"],
                 e["external"], 2, 3, 2) for e in nc["expected"]]
        assert o.services_nets() == want
        nets = o.nets()
        for pid in (100, 200):
            got = {k: sorted(p for (pp, _, kk, p, _) in nets if pp == pid and kk == k) for k in (1, 2, 3)}
            assert got[1] == sorted(x.ljust(12, "0") for x in nc["nets_v4_16"])
            assert got[2] == sorted(x.ljust(12, "0") for x in nc["nets_v4_24"])
            assert got[3] == sorted(nc["nets_v6"])
        # 59 minutes: nothing expires; clear() keeps both (maps non-empty) with zeroed counters
        o.network_counters_cleaning(59 * MIN)
        o.clear()
        rows = o.services_nets()
        assert len(rows) == nc["after_59min"]["services"]
        assert all(r[4] == 0 and r[5] == 0 and list(r[6:]) == nc["after_59min"]["sizes"] for r in rows)
        # 60 minutes: every entry is erased (>= 1 h), and clear() drops both services
        o.network_counters_cleaning(60 * MIN)
        o.clear()
        assert o.services_nets() == []
        assert o.services_json() == b""


def test_oracle_json_agrees_with_product_formatter():
    o, nc = netcounter_oracle(mock=False)
    rows = o.services_nets()
    svcs = [dict(pid=r[0], endpoint=r[1].decode(), domain=r[2].decode(), scheme=r[3].decode(), internal=r[4],
                 external=r[5], nets=r[6:9]) for r in rows]
    recs, blob = records(svcs)  # services_nets is sorted by (pid, endpoint), as is creation order here
    assert o.services_json() == ebd.format_services_json(recs, blob)
    assert o.services_json().startswith(b'{"service":[{"pid":100,"endpoint":"host/url","domain":"host","scheme":"http",'
                                        b'"internalClientsNumber":0,"externalClientsNumber":5,'
                                        b'"externalIPv4_16ClientNets":2,"externalIPv4_24ClientNets":3,'
                                        b'"externalIPv6ClientsNets":2}')


def test_oracle_network_counters_off_is_plain_clear():
    o = O.Oracle()
    o.new_request(1, b"h", b"/u", b"8.8.8.8", ebd.FLAG_IPV4)
    assert o.services_nets() == [(1, b"h/u", b"h", b"http", 0, 1, 0, 0, 0)]
    o.clear()
    assert o.services_nets() == []


def test_oracle_clear_keeps_first_arrival_and_recount():
    """A kept service keeps its domain/scheme; later requests count from zero again; a
    service erased by clear is created afresh by its next request (new first arrival)."""
    o = O.Oracle(network_counters=True)
    o.set_time(10)
    o.new_request(1, b"a:80", b"/x", b"8.8.8.8", ebd.FLAG_IPV4)                       # external: kept
    o.new_request(2, b"b:80", b"/y", b"10.0.0.1", ebd.FLAG_IPV4)                      # internal: erased
    o.clear()
    o.new_request(1, b"a:80", b"/x", b"10.0.0.2", ebd.FLAG_IPV4 | ebd.FLAG_SSL)
    o.new_request(2, b"b:8", b"0/y", b"10.0.0.3", ebd.FLAG_IPV4 | ebd.FLAG_SSL)
    assert o.services_nets() == [(1, b"a:80/x", b"a", b"http", 1, 0, 1, 1, 0),
                                 (2, b"b:80/y", b"b", b"https", 1, 0, 0, 0, 0)]
