#!/usr/bin/env python3
"""Debug helper: clear + resubmit of one batch; checks that every interval gives the same
services (no (pid, endpoint) under two keys) and the same per-event results."""
import collections
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ebpf-discovery_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import ebd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_500_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
t = time.time()
ev, lens, offs, payload = ebd.generate_host(3, 41, 0, n)
print("gen", time.time() - t, flush=True)
ctx = ebd.Context(max_events=len(ev), max_payload=payload.size, service_capacity=1 << 21)
ref_res = None
for k in range(reps):
    if k:
        ctx.clear()
    ctx.set_seq_base(0)
    ctx.submit(ev, lens, offs, payload)
    res = ctx.results()
    if ref_res is None:
        ref_res = res.copy()
    else:
        diff = np.flatnonzero(res.view(np.uint8).reshape(-1, 16).any(axis=1) != ref_res.view(np.uint8).reshape(-1, 16).any(axis=1))
        neq = np.flatnonzero((res.view(np.uint8).reshape(-1, 16) != ref_res.view(np.uint8).reshape(-1, 16)).any(axis=1))
        print("results differing from interval 0:", len(neq), neq[:10].tolist(), flush=True)
        for i in neq[:5]:
            print("  ", int(i), res[i], ref_res[i], flush=True)
    raw, blob = ctx.services_raw()
    s = blob.tobytes()
    eps = collections.defaultdict(list)
    for r in raw:
        o, L = int(r["endpoint_off"]), int(r["endpoint_len"])
        eps[(int(r["pid"]), s[o:o + L])].append((hex(int(r["key_lo"])), int(r["internal"]), int(r["external"]),
                                                 int(r["first_seq"]), int(r["host_len"])))
    dup = {k2: v for k2, v in eps.items() if len(v) > 1}
    print("interval", k, "services", len(raw), "distinct (pid, endpoint)", len(eps), "dups", len(dup),
          ctx.stats()["error_names"], flush=True)
    for k2, v in list(dup.items())[:6]:
        print("   dup", k2, v, flush=True)
