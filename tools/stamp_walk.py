#!/usr/bin/env python3
"""Writes a copy of ebd_kernels.hip with per-wave clock stamps in k_walk<false> (a profiling
build, never the product source):

  python tools/stamp_walk.py ebpf-discovery_amd/build/stampsrc/ebd_kernels_walk.hip
  make -C ebpf-discovery_amd variant V=wstamp KSRC=build/stampsrc/ebd_kernels_walk.hip

Each wave of workgroups 0..7 prints one line at its end:
  WSTAMP <wg> <wave> iters active_lanes refills lanes_refilled events_started cyc_block cyc_refill cyc_total
(iters: loop iterations with a lane parsing; active_lanes: their summed popcount).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "ebpf-discovery_amd", "csrc", "ebd_kernels.hip")


def sub(s, old, new, count=1):
    assert s.count(old) == count, (old, s.count(old))
    return s.replace(old, new)


def main():
    out = sys.argv[1]
    s = open(SRC).read()
    s = sub(s, """	uint32_t st_ev = 0, st_by = 0; // DRY with dw.stat: this lane's events and bytes walked
	for (;;) {
		const unsigned long long busy = __ballot(in_ev), wait = __ballot(!in_ev && (ended || h < nh));
		if (busy == 0 && wait == 0)
			break;
		if (busy == 0 || __popcll(wait) >= kWalkRefill) {""", """	uint32_t st_ev = 0, st_by = 0; // DRY with dw.stat: this lane's events and bytes walked
	unsigned long long W_it = 0, W_act = 0, W_ref = 0, W_refl = 0, W_evs = 0, W_blk = 0, W_rc = 0;
	const unsigned long long W_t0 = clock64();
	for (;;) {
		const unsigned long long busy = __ballot(in_ev), wait = __ballot(!in_ev && (ended || h < nh));
		if (busy == 0 && wait == 0)
			break;
		if (busy == 0 || __popcll(wait) >= kWalkRefill) {
			const unsigned long long R0 = clock64();
			W_ref++;
			W_refl += (unsigned long long)__popcll(wait);""")
    s = sub(s, """						if (DRY) {
							st_ev++;
							st_by += ne;
						}""", """						if (DRY) {
							st_ev++;
							st_by += ne;
						}
						W_evs++;""")
    s = sub(s, """					have = false;
					h = DRY ? h + stride : nx_h;
				}
			}
		}
		// the window loaded last iteration""", """					have = false;
					h = DRY ? h + stride : nx_h;
				}
			}
			W_rc += clock64() - R0;
		}
		const unsigned long long B0 = clock64();
		const unsigned long long busy2 = __ballot(in_ev);
		if (busy2) {
			W_it++;
			W_act += (unsigned long long)__popcll(busy2);
		}
		// the window loaded last iteration""")
    s = sub(s, """	if (!DRY) { // the loop ends for the whole wave at once
		for (int o = 32; o > 0; o >>= 1)
			inserts += __shfl_xor(inserts, o, 64);""", """	if (!DRY) {
		for (int o = 32; o > 0; o >>= 1)
			W_evs += __shfl_xor(W_evs, o, 64);
		if ((threadIdx.x & 63) == 0 && blockIdx.x < 8)
			printf("WSTAMP %u %u %llu %llu %llu %llu %llu %llu %llu %llu\\n", blockIdx.x, threadIdx.x >> 6, W_it, W_act, W_ref, W_refl, W_evs,
					W_blk, W_rc, clock64() - W_t0);
	}
	if (!DRY) { // the loop ends for the whole wave at once
		for (int o = 32; o > 0; o >>= 1)
			inserts += __shfl_xor(inserts, o, 64);""")
    # the block step's time: from B0 to the loop's end
    s = sub(s, """			wi++;
			if (4u * wi >= nb || w.tpos != kNone) {
				in_ev = false;
				ended = true;
			}
		}
	}""", """			wi++;
			if (4u * wi >= nb || w.tpos != kNone) {
				in_ev = false;
				ended = true;
			}
		}
		W_blk += clock64() - B0;
	}""")
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    open(out, "w").write(s)


if __name__ == "__main__":
    main()
