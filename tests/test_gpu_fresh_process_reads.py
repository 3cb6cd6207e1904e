"""Reads into caller-owned (pageable) memory right after the first kernels of a fresh process.

The stale parser state of round 5 came from an async device-to-host copy
into pageable memory followed by hipStreamSynchronize: the host read the caller's buffer before
the runtime's staged copy had landed, and only in fresh processes (the first launch of a kernel
also loads its code object, which widens the window).  Every C-ABI read into caller memory now
drains the stream and then copies with a blocking hipMemcpy (ebd_api.hip read_out).  This test
runs the pattern once in a fresh interpreter: a config-3 sample batch, its results and session
requests into new numpy arrays, a chain of ebd_parse_streams calls, each checked against the
oracle."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

SCRIPT = r"""
import sys
import numpy as np
import ebd
import oracle_py as O
import traces as T

ev, lens, offs, payload = ebd.generate_host(3, 11, 0, 3000)
ctx = ebd.Context(max_events=len(ev), max_payload=payload.size, lru_capacity=0)
ctx.submit(ev, lens, offs, payload)
res = ctx.results()                  # first read of the process, straight after the first batch
sreq, sstr = ctx.session_requests()
gv = T.gpu_view(res, offs, payload, sreq, sstr)
o = O.Oracle(lru_capacity=8192)
out, blob = o.process(ev, lens, offs, payload)
ov = T.oracle_view(out, blob)
bad = [i for i in range(len(ov)) if gv[i] != ov[i]]
assert not bad, bad[:5]
assert ctx.services() == o.services()

req = b"GET /a/b HTTP/1.1\r\nHost: example.com\r\nX-Forwarded-For: 1.2.3.4\r\n\r\n"
p = ebd.StreamParser(ctx)
total = sum(p.parse(req[k:k + 1], 8) for k in range(len(req)))  # one byte per call, each from the last state
assert p.is_finished() and not p.is_invalid() and total == len(req), (total, len(req))
assert p.result["host"] == b"example.com" and p.result["url"] == b"/a/b", p.result
assert p.result["client_ip"] == [b"1.2.3.4"], p.result
print("ok")
"""


def test_first_reads_of_a_fresh_process_follow_the_batch():
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(ROOT, "ebpf-discovery_amd"), HERE, env.get("PYTHONPATH", "")])
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "ok" in r.stdout
