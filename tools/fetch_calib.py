#!/usr/bin/env python3
"""FETCH_SIZE calibration on streams of known bytes (tools/ubench_stream under
`rocprofv3 --pmc FETCH_SIZE`): per kernel shape, the bytes it reads (the payload arena plus
12 B of offset and length per event) against FETCH_SIZE x 1024.  The scale a shape needs is
known / reported; MI355X_MICROARCH.md's rule is x2 for wide coalesced streaming reads.

  python tools/fetch_calib.py <ubench log> <counter_collection.csv> <out.json>
"""
import collections
import csv
import json
import re
import sys


def main():
    log, counters, out = sys.argv[1:4]
    head = next(l for l in open(log) if l.startswith("events "))
    m = re.match(r"events (\d+), payload ([\d.]+) GB .* arena ([\d.]+) GB", head)
    n, arena = int(m.group(1)), float(m.group(3)) * 1e9
    known = arena + 12 * n
    per = collections.OrderedDict()
    for r in csv.DictReader(open(counters)):
        if r["Counter_Name"] != "FETCH_SIZE":
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if not name.startswith("k_"):
            continue
        per.setdefault(name, []).append(float(r["Counter_Value"]) * 1024)
    shapes = {k: {"fetch_bytes": sum(v) / len(v), "scale": known / (sum(v) / len(v))} for k, v in per.items()}
    json.dump({"events": n, "known_bytes": known, "shapes": shapes,
               "note": "scale = bytes read / (FETCH_SIZE x 1024); k_quad64a<0> is k_fresh's window shape"},
              open(out, "w"), indent=1)
    for k, v in shapes.items():
        print("%-18s FETCH %.3f GB  scale %.2f" % (k, v["fetch_bytes"] / 1e9, v["scale"]))


if __name__ == "__main__":
    main()
