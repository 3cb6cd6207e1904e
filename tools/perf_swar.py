#!/usr/bin/env python3
"""The byte-parallel fast-path scan prototype (tools/swar_probe.hip) beside k_fresh: one
device-resident config-3 batch through the library (k_fresh's results), then the probe over the
same buffers. Every event the probe takes must equal k_fresh's result (status FINISHED,
consumed, URL, Host, POST / HTTPS / client-IP bits); prints the share it takes and both times.

  python tools/perf_swar.py --events 20000000 --reps 5
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ebpf-discovery_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ebd  # noqa: E402

SWAR_DTYPE = np.dtype([("consumed", "<u2"), ("status", "u1"), ("info", "u1"), ("url_off", "<u2"), ("url_len", "<u2"),
                       ("host_off", "<u2"), ("host_len", "<u2"), ("cip_off", "<u2"), ("pad", "<u2")])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=20_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--blocks", type=int, default=256 * 8)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    E, cfg = args.events, args.config
    ctx = ebd.Context(max_events=E, service_capacity=1 << max(20, int(np.ceil(np.log2(E * 0.8)))),
                      string_arena=max(256 << 20, E * 48), timing=True)
    E, size = ebd.trace_size_device(ctx, cfg, cfg, 0, E, align=16, with_events=True)
    ev = torch.empty(E * 36, dtype=torch.uint8, device=dev)
    ln = torch.empty(E, dtype=torch.int32, device=dev)
    of = torch.empty(E, dtype=torch.int64, device=dev)
    pay = torch.empty(size + 64, dtype=torch.uint8, device=dev)
    ebd.generate_device(ctx, cfg, cfg, 0, E, ev, ln, of, pay, pay.numel(), align=16)
    torch.cuda.synchronize()
    ctx.submit_device(ev, ln, of, pay, E)
    ctx.sync()
    ctx.reset_kernel_times()
    for k in range(args.reps):
        ctx.clear()
        ctx.set_seq_base((k + 1) * E)
        ctx.submit_device(ev, ln, of, pay, E)
    ctx.sync()
    kt = ctx.kernel_times()
    fresh_ms = kt["k_fresh"][1] / max(kt["k_fresh"][0], 1)
    res = ctx.results()

    lib = C.CDLL(os.path.join(ROOT, "tools", "libswar_probe.so"))
    lib.swar_scan.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_ulonglong, C.c_uint32, C.c_void_p, C.c_int,
                              C.POINTER(C.c_float)]
    out = torch.zeros(E * 16, dtype=torch.uint8, device=dev)
    times = []
    for _ in range(args.reps + 1):
        ms = C.c_float()
        rc = lib.swar_scan(ev.data_ptr(), ln.data_ptr(), of.data_ptr(), pay.data_ptr(), size, E, out.data_ptr(), args.blocks,
                           C.byref(ms))
        assert rc == 0, rc
        times.append(ms.value)
    sw = out.cpu().numpy().view(SWAR_DTYPE)
    took = sw["status"] == 1
    fin = res["status"] == ebd.STATUS_FINISHED if hasattr(ebd, "STATUS_FINISHED") else res["status"] == 1
    bits = 0x01 | 0x02 | 0x08
    same = (took & fin & (sw["consumed"] == res["consumed"]) & (sw["url_off"] == res["url_off"]) & (sw["url_len"] == res["url_len"])
            & (sw["host_off"] == res["host_off"]) & (sw["host_len"] == res["host_len"]) & ((sw["info"] & bits) == (res["info"] & bits)))
    bad = took & ~same
    alg = int(res["consumed"].astype(np.uint64).sum()) + 40 * int((res["status"] != 0).sum())
    swar_ms = float(np.median(times[1:]))
    print(json.dumps({"events": E, "k_fresh_ms": fresh_ms, "swar_ms": swar_ms, "swar_alg_gbps": alg / swar_ms / 1e6,
                      "k_fresh_alg_gbps": alg / fresh_ms / 1e6, "taken": int(took.sum()), "fresh_finished": int(fin.sum()),
                      "missed": int((fin & ~took).sum()), "mismatched": int(bad.sum()),
                      "mismatch_examples": [int(x) for x in np.nonzero(bad)[0][:8]]}))


if __name__ == "__main__":
    main()
