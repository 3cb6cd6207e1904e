"""Averages the WSTAMP lines of a k_walk clock-stamp build (tools/stamp_walk.py)."""
import sys

import numpy as np

rows = [l.split() for l in open(sys.argv[1]) if l.startswith("WSTAMP")]
a = np.array([[int(x) for x in r[3:]] for r in rows], dtype=float)
it, act, ref, refl, evs, blk, rc, tot = a.T
print(f"waves {len(a)}; per wave: iterations {it.mean():.0f}, active lanes per iteration {(act / it).mean():.1f}, "
      f"refills {ref.mean():.0f} of {(refl / ref).mean():.1f} lanes, events {evs.mean():.0f}")
print(f"cycles per wave: walk {blk.mean():.0f}, refill {rc.mean():.0f}, total {tot.mean():.0f}; "
      f"per iteration {(blk / it).mean():.0f}, per refill {(rc / ref).mean():.0f}")

ref = [l.split() for l in open(sys.argv[1]) if l.startswith("WREF")]
if ref:
    b = np.array([[int(x) for x in r[3:]] for r in ref], dtype=float)
    ce, cp, cl, ss, nr = b.T
    print(f"refill cycles per wave: ending events {ce.mean():.0f}, pipeline stage {cp.mean():.0f}, starting events {cl.mean():.0f}; "
          f"sessions started per wave {ss.mean():.0f}, before their prefetch finished {nr.mean():.0f}")
