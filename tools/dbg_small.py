#!/usr/bin/env python3
"""Debug helper: a few config-1/3 events through the fast path; prints per-event results and stats."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ebpf-discovery_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import ebd  # noqa: E402

for cfg, n in ((1, 8), (3, 8)):
    ev, lens, offs, payload = ebd.generate_host(cfg, cfg, 0, n)
    ctx = ebd.Context(max_events=n, max_payload=payload.size)
    ctx.submit(ev, lens, offs, payload)
    print(cfg, [tuple(int(x) for x in r) for r in ctx.results()], ctx.stats(), flush=True)
    print(ctx.services()[:3], flush=True)
