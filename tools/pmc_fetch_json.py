#!/usr/bin/env python3
"""HBM bytes per k_fresh launch from rocprofv3 counter passes, as bench.py reads them.

  python tools/pmc_fetch_json.py --fetch <dir> [--write <dir>] --events N --config C --out profiles/x.json

FETCH_SIZE and WRITE_SIZE are rocprofv3's derived counters in KiB.  How many bytes a FETCH_SIZE
KiB stands for depends on the load shape (profiles/r04_fetch_calibration.json: streams of known
bytes, tools/ubench_stream under one --pmc FETCH_SIZE pass): x1.99 for 16 B per lane over
consecutive addresses and x2.09 for LDS-DMA tiles (the guide's x2 rule, MI355X_MICROARCH.md HBM /
rocprofv3), x1.25 for k_fresh's shape (a quad's 64-byte windows on the 64-byte grid, no work),
x1.19 for the same with the DFA-like work, x1.03 for buffer-relative 64-byte windows.  The
default scale is therefore 1.25 (round 3 used 1, from a round-1 scan-only build).
"""
import argparse
import collections
import csv
import glob
import json
import re


def per_launch(d, counter, kernel):
    # the kernel's own name, not a longer one that starts with it (k_walk, not k_walk_heads)
    own = re.compile(r"(^|::|\s)" + re.escape(kernel) + r"\(")
    vals = collections.defaultdict(float)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if own.search(r["Kernel_Name"]) and r["Counter_Name"] == counter:
                vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} under {d}")
    return sum(vals.values()) / len(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write")
    ap.add_argument("--events", type=int, required=True)
    ap.add_argument("--config", type=int, required=True)
    ap.add_argument("--kernel", default="k_fresh", help="kernel(s), comma-separated; the first is the summary's")
    ap.add_argument("--launches-per-step", type=float, default=0,
                    help="launches of each kernel per bench step (config 4: one per poll cycle): adds per-step bytes")
    ap.add_argument("--out", required=True)
    ap.add_argument("--fetch-scale", type=float, default=1.25)
    ap.add_argument("--build-id", required=True, help="ebd.build_id() of the library the passes measured")
    a = ap.parse_args()
    kernels = a.kernel.split(",")
    per = {}
    for k in kernels:
        fkib, nf = per_launch(a.fetch, "FETCH_SIZE", k)
        e = {"dispatches": nf, "fetch_size_kib_per_launch": fkib, "hbm_read_bytes_per_launch": fkib * 1024 * a.fetch_scale}
        total = e["hbm_read_bytes_per_launch"]
        if a.write:
            wkib, _ = per_launch(a.write, "WRITE_SIZE", k)
            e["write_size_kib_per_launch"] = wkib
            e["hbm_write_bytes_per_launch"] = wkib * 1024
            total += wkib * 1024
        e["hbm_bytes_per_launch"] = total
        if a.launches_per_step:
            e["hbm_bytes_per_step"] = total * a.launches_per_step
        per[k] = e
    out = {"kernel": kernels[0], "events": a.events, "config": a.config, "build_id": a.build_id,
           "fetch_scale": a.fetch_scale, **per[kernels[0]]}
    if len(kernels) > 1 or a.launches_per_step:
        out["kernels"] = per
        out["launches_per_step"] = a.launches_per_step
    out["note"] = ("FETCH_SIZE x 1024 x fetch_scale + WRITE_SIZE x 1024, averaged over the launches; fetch_scale is "
                   "measured on a stream of k_fresh's load shape with known bytes (profiles/r04_fetch_calibration.json: "
                   "x1.25; x2 for plain 16-B-per-lane streams, the guide's rule)")
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
