#!/usr/bin/env python3
"""Writes a copy of ebd_kernels.hip with per-wave clock stamps in the batch walk k_walk (a
profiling build, never the product source):

  python tools/stamp_walk.py ebpf-discovery_amd/build/stampsrc/ebd_kernels_walk.hip
  make -C ebpf-discovery_amd variant V=wstamp KSRC=build/stampsrc/ebd_kernels_walk.hip

Each wave of workgroups 0..7 prints one line at its end:
  WSTAMP <wg> <wave> iters active_lanes refills lanes_refilled events_started cyc_block cyc_refill cyc_total
(iters: loop iterations with a lane parsing; active_lanes: their summed popcount).  A second line splits the refill:
  WREF <wg> <wave> cyc_end cyc_pipeline cyc_loop session_starts not_ready_starts
(cyc_end: ending the events; cyc_pipeline: the next session's prefetch stage; cyc_loop: starting
the next events; not_ready: a session started before its prefetch pipeline had finished).
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
	unsigned long long W_ce = 0, W_cp = 0, W_cl = 0, W_ss = 0, W_nr = 0, W_by = 0;
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
    # the refill split: events ended | next session's pipeline stage | the loop starting events
    s = sub(s, """			if (have && nx_h < nh && nx_st < kNxStages) { // the next session's pipeline: one stage per refill""",
            """			const unsigned long long R1 = clock64();
			W_ce += R1 - R0;
			if (have && nx_h < nh && nx_st < 4) { // the next session's pipeline: one stage per refill""")
    s = sub(s, """			while (!in_ev && h < nh) { // the next event that needs a parse, finishing the others""",
            """			const unsigned long long R2 = clock64();
			W_cp += R2 - R1;
			while (!in_ev && h < nh) { // the next event that needs a parse, finishing the others""")
    s = sub(s, """					const bool ready = nx_h == h && nx_st == kNxStages;""", """					const bool ready = nx_h == h && nx_st == kNxStages;
					W_ss++;
					W_nr += ready ? 0 : 1;""")
    s = sub(s, """			W_rc += clock64() - R0;""", """			W_cl += clock64() - R2;
			W_rc += clock64() - R0;""")
    s = sub(s, """					W_blk, W_rc, clock64() - W_t0);""", """					W_blk, W_rc, clock64() - W_t0);
		for (int o = 32; o > 0; o >>= 1) {
			W_ss += __shfl_xor(W_ss, o, 64);
			W_nr += __shfl_xor(W_nr, o, 64);
		}
		if ((threadIdx.x & 63) == 0 && blockIdx.x < 8)
			printf("WREF %u %u %llu %llu %llu %llu %llu\\n", blockIdx.x, threadIdx.x >> 6, W_ce, W_cp, W_cl, W_ss, W_nr);""")
    # every wave's start and end on the 100 MHz wall clock and its events, kept in device memory
    # (printf from every wave slowed the waves still walking); tools/walk_balance.py reads them
    s = sub(s, """	const unsigned long long W_t0 = clock64();""", """	const unsigned long long W_t0 = clock64(), W_w0 = wall_clock64();""")
    s = sub(s, """		for (int o = 32; o > 0; o >>= 1)
			W_evs += __shfl_xor(W_evs, o, 64);""", """		const unsigned long long W_w1 = wall_clock64();
		for (int o = 32; o > 0; o >>= 1)
			W_evs += __shfl_xor(W_evs, o, 64);
		unsigned long long W_byw = W_by, W_ssw = W_ss;
		for (int o = 32; o > 0; o >>= 1) {
			W_byw += __shfl_xor(W_byw, o, 64);
			W_ssw += __shfl_xor(W_ssw, o, 64);
		}
		if ((threadIdx.x & 63) == 0 && blockIdx.x * 4u + (threadIdx.x >> 6) < 16384u) {
			unsigned long long* q = g_wend + 8u * (blockIdx.x * 4u + (threadIdx.x >> 6));
			q[0] = W_w0;
			q[1] = W_w1;
			q[2] = W_evs;
			q[3] = W_byw;
			q[4] = W_ssw;
			q[5] = W_rc;
			q[6] = W_blk;
			q[7] = W_it;
		}""")
    s = sub(s, """						W_evs++;""", """						W_evs++;
						W_by += ne;""")
    s = sub(s, """template <bool DRY>
__device__ __forceinline__ void walk_sessions(""", """__device__ unsigned long long g_wend[8 * 16384];
template <bool DRY>
__device__ __forceinline__ void walk_sessions(""")
    s += """
extern "C" int ebd_stamp_read(unsigned long long* out, int n) {
	return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(ebd::g_wend), (size_t)n * 8u, 0, hipMemcpyDeviceToHost);
}
"""
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    open(out, "w").write(s)


if __name__ == "__main__":
    main()
