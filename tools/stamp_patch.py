#!/usr/bin/env python3
"""Writes a copy of ebd_kernels.hip with per-wave clock stamps in k_fresh (a profiling build,
never the product source):

  python tools/stamp_patch.py build/stampsrc/ebd_kernels.hip
  make -C ebpf-discovery_amd variant V=stamp KSRC=build/stampsrc/ebd_kernels.hip

Each wave of workgroups 0..7 prints one line at its end, the clock64() cycles it spent in
each phase:
  STAMP scan <wg> <wave> iters valid wait issue scan push resolve
  STAMP fin  <wg> <wave> batches poll load finalize
tools/stamp_summary.py averages them.
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
    # finalize waves
    s = sub(s, """		uint32_t uh = 0, un = 0; // wave-uniform: ring head and entries
		for (;;) {
			uint32_t c = 0;""", """		uint32_t uh = 0, un = 0; // wave-uniform: ring head and entries
		unsigned long long S_b = 0, S_poll = 0, S_load = 0, S_fin = 0;
		for (;;) {
			unsigned long long P0 = clock64();
			uint32_t c = 0;""")
    s = sub(s, """			if (!__any(st == 1))
				break;
			uint32_t q[R_WORDS];""", """			unsigned long long P1 = clock64();
			S_poll += P1 - P0;
			if (!__any(st == 1))
				break;
			S_b++;
			uint32_t q[R_WORDS];""")
    s = sub(s, """				lds_store_rel(&sh.freed[slot], pos + 1); // the slot may be written again
			}
			bool unf = false;""", """				lds_store_rel(&sh.freed[slot], pos + 1); // the slot may be written again
			}
			unsigned long long P2 = clock64();
			S_load += P2 - P1;
			bool unf = false;""")
    s = sub(s, """					unf = finalize_rec(d, T, q, fs);
			}""", """					unf = finalize_rec(d, T, q, fs);
			}
			S_fin += clock64() - P2;""")
    s = sub(s, """				d.ev_slot[at + lane] = ust[(uh + lane) & 127u];
		}
		return;""", """				d.ev_slot[at + lane] = ust[(uh + lane) & 127u];
		}
		if (lane == 0 && blockIdx.x < 8)
			printf("STAMP fin %u %u %llu %llu %llu %llu\\n", blockIdx.x, wave, S_b, S_poll, S_load, S_fin);
		return;""")
    # scan waves
    s = sub(s, """	while (__any(e0.kind != EK_NONE)) {
		// is the window in flight the one e0 needs?""", """	unsigned long long S_it = 0, S_val = 0, S_wait = 0, S_issue = 0, S_scan = 0, S_push = 0, S_res = 0;
	while (__any(e0.kind != EK_NONE)) {
		unsigned long long Q0 = clock64();
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		unsigned long long Q1 = clock64();
		S_wait += Q1 - Q0;
		S_it++;
		// is the window in flight the one e0 needs?""")
    s = sub(s, """		transpose_quad(X, r);
		bool done = false;""", """		unsigned long long Q2 = clock64();
		S_issue += Q2 - Q1;
		S_val += __any(valid) ? 1 : 0;
		transpose_quad(X, r);
		bool done = false;""")
    s = sub(s, """		uint32_t tw = 0;
		if (done) { // the last chunk""", """		unsigned long long Q3 = clock64();
		S_scan += Q3 - Q2;
		uint32_t tw = 0;
		if (done) { // the last chunk""")
    s = sub(s, """		push(done, tw);
		if (done) {
			e0 = e1;
			e1 = lane_ev(d, lane_load(d, grab(), re));
			resolve();
		}
	}
	if (lane == 0)
		atomicAdd(&sh.scan_done, 1u);""", """		push(done, tw);
		unsigned long long Q4 = clock64();
		S_push += Q4 - Q3;
		if (done) {
			e0 = e1;
			e1 = lane_ev(d, lane_load(d, grab(), re));
			resolve();
		}
		S_res += clock64() - Q4;
	}
	if (lane == 0)
		atomicAdd(&sh.scan_done, 1u);
	// after the finalize waves were released: the print's cost is outside every stamp
	if (lane == 0 && blockIdx.x < 8)
		printf("STAMP scan %u %u %llu %llu %llu %llu %llu %llu %llu\\n", blockIdx.x, wave, S_it, S_val, S_wait, S_issue, S_scan, S_push, S_res);""")
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    open(out, "w").write(s)


if __name__ == "__main__":
    main()
