#!/usr/bin/env python3
"""Debug helper: the reference parser vectors as sessions through one context; prints the
raw error word (debug builds raise high bits for impossible records / addresses)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ebpf-discovery_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import ebd  # noqa: E402
import traces as T  # noqa: E402

vec = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_vectors.json")))
cases = vec["parser_valid"] + vec["parser_invalid"]
if len(sys.argv) > 2:
    cases = cases[int(sys.argv[1]):int(sys.argv[2])]
chunk_lists = [[c.encode("latin-1") for c in case["chunks"]] for case in cases]
ev, lens, offs, payload = T.session_trace(chunk_lists)
ctx = ebd.Context(max_events=len(ev), max_payload=payload.size)
ctx.submit(ev, lens, offs, payload)
st = ctx.stats()
print(json.dumps({"n": len(ev), "payload": int(payload.size), "errors": hex(st["errors"]), "names": st["error_names"]}))
