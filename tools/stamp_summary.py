#!/usr/bin/env python3
"""Averages the STAMP lines of a stamp build's run (tools/stamp_patch.py):
  python tools/stamp_summary.py gpurun_out/stamp.log
"""
import sys

import numpy as np


def main():
    scan, fin = [], []
    for line in open(sys.argv[1]):
        f = line.split()
        if len(f) < 3 or f[0] != "STAMP":
            continue
        v = [int(x) for x in f[2:]]
        (scan if f[1] == "scan" else fin).append(v)
    if scan:
        a = np.array(scan, dtype=np.float64)[:, 2:]
        m = a.mean(axis=0)
        names = ["iters", "valid", "wait", "issue", "scan", "push", "resolve"]
        tot = m[2:].sum()
        print("scan waves: %d lines" % len(a))
        for n, x in zip(names, m):
            extra = "  %5.1f%%" % (100 * x / tot) if n not in ("iters", "valid") else ""
            print("  %-8s %14.0f%s" % (n, x, extra))
        print("  cycles/iter %.0f  (wait %.0f issue %.0f scan %.0f push %.0f resolve %.0f)" % (
            tot / m[0], m[2] / m[0], m[3] / m[0], m[4] / m[0], m[5] / m[0], m[6] / m[0]))
    if fin:
        a = np.array(fin, dtype=np.float64)[:, 2:]
        m = a.mean(axis=0)
        tot = m[1:].sum()
        print("finalize waves: %d lines" % len(a))
        for n, x in zip(["batches", "poll", "load", "finalize"], m):
            extra = "  %5.1f%%" % (100 * x / tot) if n != "batches" else ""
            print("  %-8s %14.0f%s" % (n, x, extra))
        print("  cycles/batch: poll %.0f load %.0f finalize %.0f" % (m[1] / m[0], m[2] / m[0], m[3] / m[0]))


if __name__ == "__main__":
    main()
