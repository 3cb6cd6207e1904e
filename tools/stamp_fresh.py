#!/usr/bin/env python3
"""Writes a copy of ebd_kernels.hip in which every k_fresh wave records its start and end on
the 100 MHz wall clock in a device array (a profiling build, never the product source):

  python tools/stamp_fresh.py ebpf-discovery_amd/build/stampsrc/ebd_kernels_fresh.hip
  make -C ebpf-discovery_amd variant V=fstamp KSRC=build/stampsrc/ebd_kernels_fresh.hip
  EBD_LIB=ebpf-discovery_amd/build/variants/libebd_amd_fstamp.so python tools/fresh_balance.py

Record of wave w of workgroup g at g_fend[4 * (g * 16 + w)]: start, end, events taken (scan
waves), 1 for a scan wave.
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
    s = sub(s, """__global__ __launch_bounds__(kFreshThreads)
#if EBD_FRESH_WGS > 1""", """__device__ unsigned long long g_fend[4 * 16 * 4096];
__device__ __forceinline__ void fstamp(unsigned long long t0, uint32_t evs, uint32_t scan) {
	const uint32_t wv = blockIdx.x * 16u + (threadIdx.x >> 6);
	const unsigned long long t1 = wall_clock64();
	if ((threadIdx.x & 63) == 0 && wv < 16u * 4096u) {
		unsigned long long* q = g_fend + 4u * wv;
		q[0] = t0;
		q[1] = t1;
		q[2] = evs;
		q[3] = scan;
	}
}
__global__ __launch_bounds__(kFreshThreads)
#if EBD_FRESH_WGS > 1""")
    s = sub(s, """	FreshShared& sh = lds.sh;
	const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 3;""", """	FreshShared& sh = lds.sh;
	const unsigned long long F_t0 = wall_clock64();
	uint32_t F_ev = 0;
	const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 3;""")
    s = sub(s, """			if (lane < un)
				d.ev_slot[at + lane] = ust[(uh + lane) & 127u];
		}
		return;""", """			if (lane < un)
				d.ev_slot[at + lane] = ust[(uh + lane) & 127u];
		}
		fstamp(F_t0, 0, 0);
		return;""")
    s = sub(s, """	auto grab = [&]() -> uint32_t { return atomicAdd(&sh.next_ev, 1u); };""",
            """	auto grab = [&]() -> uint32_t { F_ev++; return atomicAdd(&sh.next_ev, 1u); };""")
    s = sub(s, """	if (lane == 0)
		atomicAdd(&sh.scan_done, 1u);
}""", """	if (lane == 0)
		atomicAdd(&sh.scan_done, 1u);
	for (int o = 32; o > 0; o >>= 1)
		F_ev += __shfl_xor(F_ev, o, 64);
	fstamp(F_t0, F_ev, 1);
}""")
    s += """
extern "C" int ebd_stamp_read(unsigned long long* out, int n) {
	return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(ebd::g_fend), (size_t)n * 8u, 0, hipMemcpyDeviceToHost);
}
"""
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    open(out, "w").write(s)


if __name__ == "__main__":
    main()
