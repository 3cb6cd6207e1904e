// ubench_stream.hip — the payload-stream shapes a k_fresh workgroup can use, each measured alone
// with a trivial consumer (XOR of every word), on config-3-like events: lengths 32..1024 (mean
// ~256), packed at 16-B alignment, one 1024-thread workgroup per CU owning a contiguous event
// range, as k_fresh.  Shapes:
//   read     every lane global_load_dwordx4 of consecutive 16 B (1 KiB per wave instruction),
//            8 loads in flight per lane: the read-only stream peak
//   quad64   k_fresh r03: a lane per event; the 4 lanes of a quad load 64-B event-relative
//            windows (one member's window per instruction, 16 windows per instruction), DPP
//            4x4 transpose, the next window in flight while the current one is consumed
//   quad64a  quad64 with the windows aligned to 64 B (whole half lines; an event's first and
//            last window are shared with its neighbours)
//   oct128   a lane per event; 8 lanes load 128-B line-aligned windows (one member's line per
//            instruction: every instruction = 8 whole lines), 8x8 transpose, next line in flight
//   oct128e  oct128 with event-relative windows (128 B from the event's 16-B aligned start:
//            each spans two lines)
//   +W       the same with the DFA's cost shape: 16 dependent LDS table steps per 16-B piece
//   dma<L,D> L loader waves copy the workgroup's span into an LDS ring of 16-KiB slots by
//            global_load_lds_dwordx4 (1 KiB per wave instruction), D slots in flight per
//            loader; the other waves read each ready slot once (ds_read_b128) and free it
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_stream tools/ubench_stream.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                                  \
	do {                                                                                       \
		hipError_t e_ = (x);                                                                   \
		if (e_ != hipSuccess) {                                                                \
			fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
			exit(1);                                                                           \
		}                                                                                      \
	} while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4u ld16(const uint8_t* a) { return *(const __attribute__((address_space(1))) v4u*)a; }
__device__ __forceinline__ uint32_t fold(v4u v) { return v.x ^ v.y ^ v.z ^ v.w; }

constexpr int kThreads = 1024;

__device__ __forceinline__ void wg_range(uint32_t n, uint32_t& rb, uint32_t& re) {
	const uint32_t per = (uint32_t)(((unsigned long long)n + gridDim.x - 1) / gridDim.x);
	rb = min(n, blockIdx.x * per);
	re = min(n, rb + per);
}

// ---- read: contiguous 1 KiB per wave instruction, 8 in flight per lane ----
__global__ __launch_bounds__(kThreads) void k_read(const uint8_t* pay, const uint64_t* off, const uint32_t* len, uint32_t n,
		uint32_t* out) {
	uint32_t rb, re;
	wg_range(n, rb, re);
	uint32_t acc = 0;
	if (rb < re) {
		const uint64_t lo = off[rb], hi = (off[re - 1] + len[re - 1] + 15) & ~15ull;
		constexpr uint64_t kStep = kThreads * 16ull;
		for (uint64_t b = lo + threadIdx.x * 16ull; b < hi; b += 8 * kStep) {
			v4u v[8];
#pragma unroll
			for (int k = 0; k < 8; k++)
				v[k] = ld16(pay + min(b + k * kStep, hi - 16));
#pragma unroll
			for (int k = 0; k < 8; k++)
				acc ^= fold(v[k]);
		}
	}
	out[blockIdx.x * kThreads + threadIdx.x] = acc;
}

// ---- quad64 (the r03 k_fresh stream) ----
template <int P>
__device__ __forceinline__ uint32_t qperm(uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, P, 0xf, 0xf, true); }
template <int K>
__device__ __forceinline__ uint32_t qbcast(uint32_t v) { return qperm<K | (K << 2) | (K << 4) | (K << 6)>(v); }
template <int K>
__device__ __forceinline__ unsigned long long qbcast64(unsigned long long v) {
	return (unsigned long long)qbcast<K>((uint32_t)v) | ((unsigned long long)qbcast<K>((uint32_t)(v >> 32)) << 32);
}
constexpr int kQX2 = 2 | (3 << 2) | (0 << 4) | (1 << 6);
constexpr int kQX1 = 1 | (0 << 2) | (3 << 4) | (2 << 6);

__device__ __forceinline__ void transpose_quad(v4u (&X)[4], uint32_t r) {
	const bool lo2 = r < 2, lo1 = (r & 1) == 0;
#pragma unroll
	for (int k = 0; k < 2; k++)
#pragma unroll
		for (int d = 0; d < 4; d++) {
			const uint32_t recv = qperm<kQX2>(lo2 ? X[k + 2][d] : X[k][d]);
			X[k + 2][d] = lo2 ? recv : X[k + 2][d];
			X[k][d] = lo2 ? X[k][d] : recv;
		}
#pragma unroll
	for (int k = 0; k < 4; k += 2)
#pragma unroll
		for (int d = 0; d < 4; d++) {
			const uint32_t recv = qperm<kQX1>(lo1 ? X[k + 1][d] : X[k][d]);
			X[k + 1][d] = lo1 ? recv : X[k + 1][d];
			X[k][d] = lo1 ? X[k][d] : recv;
		}
}

// The DFA's cost shape (WORK = 1): 16 dependent table steps per 16-B piece from a 128-column,
// 196-row byte-major table in LDS (k_fresh's LdsTable layout), plus the running maximum.
constexpr uint32_t kTabStride = 196, kTabBytes = 128 * kTabStride;
__device__ __forceinline__ void load_tab(uint8_t* T) {
	for (uint32_t k = threadIdx.x; k < kTabBytes; k += blockDim.x)
		T[k] = (uint8_t)((k * 2654435761u) >> 24) % 190u;
	__syncthreads();
}
template <int WORK>
__device__ __forceinline__ void consume(const uint8_t* T, const v4u& v, uint32_t& s, uint32_t& acc) {
	if (WORK) {
#pragma unroll
		for (int q = 0; q < 4; q++)
#pragma unroll
			for (int k = 0; k < 4; k++) {
				s = T[min(__builtin_amdgcn_ubfe(v[q], 8 * k, 8), 127u) * kTabStride + s];
				acc = max(acc, s);
			}
	} else {
		acc ^= fold(v);
	}
}

struct Ev {
	uint32_t idx, L;
	const uint8_t* p;
};
__device__ __forceinline__ Ev get_ev(const uint8_t* pay, const uint64_t* off, const uint32_t* len, uint32_t i, uint32_t re) {
	Ev e;
	e.idx = i;
	if (i < re) {
		e.L = len[i];
		e.p = pay + off[i];
	} else {
		e.L = 0;
		e.p = pay;
	}
	return e;
}

template <int WORK>
__global__ __launch_bounds__(kThreads) void k_quad64(const uint8_t* pay, const uint64_t* off, const uint32_t* len, uint32_t n,
		uint32_t* out) {
	__shared__ uint32_t next;
	__shared__ uint8_t T[WORK ? kTabBytes : 4];
	if (WORK)
		load_tab(T);
	uint32_t s = 1;
	uint32_t rb, re;
	wg_range(n, rb, re);
	if (threadIdx.x == 0)
		next = rb + 2 * kThreads;
	__syncthreads();
	const uint32_t r = threadIdx.x & 3;
	Ev e0 = get_ev(pay, off, len, rb + threadIdx.x, re), e1 = get_ev(pay, off, len, rb + kThreads + threadIdx.x, re);
	uint32_t w0 = 0, acc = 0, tidx = e0.idx, tw = 0;
	v4u W[4];
	auto issue = [&](const uint8_t* p, uint32_t L, uint32_t w) {
		const uint32_t last = L ? (L - 1) >> 4 : 0;
		const unsigned long long a = (unsigned long long)(uintptr_t)p;
		const uint32_t pc = (w << 2) | (last << 16);
		unsigned long long ak[4];
		uint32_t pk[4];
		ak[0] = qbcast64<0>(a), pk[0] = qbcast<0>(pc);
		ak[1] = qbcast64<1>(a), pk[1] = qbcast<1>(pc);
		ak[2] = qbcast64<2>(a), pk[2] = qbcast<2>(pc);
		ak[3] = qbcast64<3>(a), pk[3] = qbcast<3>(pc);
#pragma unroll
		for (int k = 0; k < 4; k++) {
			const uint32_t c = min((pk[k] & 0xffffu) + r, pk[k] >> 16);
			W[k] = ld16((const uint8_t*)(uintptr_t)(ak[k] + 16ull * c));
		}
	};
	issue(e0.p, e0.L, 0);
	while (__any(e0.idx < re)) {
		const bool valid = e0.idx < re && tidx == e0.idx && tw == w0;
		v4u X[4] = {W[0], W[1], W[2], W[3]};
		const uint32_t nwin = (e0.L + 63) >> 6;
		{ // the next window's address is chosen per lane; the quad-cooperative loads run uniformly
			const bool same = !valid || w0 + 1 < nwin;
			const uint32_t nw = !valid ? w0 : same ? w0 + 1 : 0;
			const Ev& ne = same ? e0 : e1;
			issue(ne.p, ne.L, nw);
			tidx = ne.idx;
			tw = nw;
		}
		transpose_quad(X, r);
		if (valid) {
#pragma unroll
			for (int k = 0; k < 4; k++)
				consume<WORK>(T, X[k], s, acc);
			w0++;
			if (w0 >= nwin) {
				e0 = e1;
				e1 = get_ev(pay, off, len, atomicAdd(&next, 1u), re);
				w0 = 0;
			}
		}
	}
	out[blockIdx.x * kThreads + threadIdx.x] = acc + s;
}

// ---- oct128: line-aligned 128-B windows, 8 lanes per instruction group ----
template <int D>
__device__ __forceinline__ void xstage(v4u (&X)[8], uint32_t r) {
	const bool lo = (r & D) == 0;
#pragma unroll
	for (int k = 0; k < 8; k++) {
		if (k & D)
			continue;
#pragma unroll
		for (int d = 0; d < 4; d++) {
			const uint32_t send = lo ? X[k + D][d] : X[k][d];
			const uint32_t recv = (uint32_t)__shfl_xor((int)send, D);
			X[k + D][d] = lo ? recv : X[k + D][d];
			X[k][d] = lo ? X[k][d] : recv;
		}
	}
}

template <int WORK, int LINE>
__global__ __launch_bounds__(kThreads) void k_oct128(const uint8_t* pay, const uint64_t* off, const uint32_t* len, uint32_t n,
		uint32_t* out) {
	__shared__ uint32_t next;
	__shared__ uint8_t T[WORK ? kTabBytes : 4];
	if (WORK)
		load_tab(T);
	uint32_t s = 1;
	uint32_t rb, re;
	wg_range(n, rb, re);
	if (threadIdx.x == 0)
		next = rb + 2 * kThreads;
	__syncthreads();
	const uint32_t lane = threadIdx.x & 63, r = lane & 7, ob = lane & ~7u;
	// a lane's event as line-aligned 128-B windows: first line a0, nl lines
	struct LEv {
		uint32_t idx, nl;
		unsigned long long a0;
	};
	auto lev = [&](uint32_t i) {
		LEv e;
		e.idx = i;
		if (i < re) {
			const unsigned long long a = (unsigned long long)(uintptr_t)(pay + off[i]);
			const unsigned long long am = LINE ? 127ull : 15ull;
			e.a0 = a & ~am;
			e.nl = (uint32_t)(((a & am) + len[i] + 127ull) >> 7);
		} else {
			e.a0 = (unsigned long long)(uintptr_t)pay;
			e.nl = 0;
		}
		return e;
	};
	LEv e0 = lev(rb + threadIdx.x), e1 = lev(rb + kThreads + threadIdx.x);
	uint32_t w0 = 0, acc = 0, tidx = e0.idx, tw = 0;
	v4u W[8];
	auto issue = [&](unsigned long long a0, uint32_t nl, uint32_t w) {
		const unsigned long long la = a0 + 128ull * min(w, nl ? nl - 1 : 0u);
#pragma unroll
		for (int k = 0; k < 8; k++) {
			const unsigned long long ak = (unsigned long long)__shfl((long long)la, (int)(ob + k));
			W[k] = ld16((const uint8_t*)(uintptr_t)(ak + 16ull * r));
		}
	};
	issue(e0.a0, e0.nl, 0);
	while (__any(e0.idx < re)) {
		const bool valid = e0.idx < re && tidx == e0.idx && tw == w0;
		v4u X[8];
#pragma unroll
		for (int k = 0; k < 8; k++)
			X[k] = W[k];
		{
			const bool same = !valid || w0 + 1 < e0.nl;
			const uint32_t nw = !valid ? w0 : same ? w0 + 1 : 0;
			const LEv& ne = same ? e0 : e1;
			issue(ne.a0, ne.nl, nw);
			tidx = ne.idx;
			tw = nw;
		}
		xstage<4>(X, r);
		xstage<2>(X, r);
		xstage<1>(X, r);
		if (valid) {
#pragma unroll
			for (int k = 0; k < 8; k++)
				consume<WORK>(T, X[k], s, acc);
			if (++w0 >= e0.nl) {
				e0 = e1;
				e1 = lev(atomicAdd(&next, 1u));
				w0 = 0;
			}
		}
	}
	out[blockIdx.x * kThreads + threadIdx.x] = acc + s;
}

// quad64a: quad64 with 64-B windows aligned to 64 B (each a whole half line)
template <int WORK>
__global__ __launch_bounds__(kThreads) void k_quad64a(const uint8_t* pay, const uint64_t* off, const uint32_t* len, uint32_t n,
		uint32_t* out) {
	__shared__ uint32_t next;
	__shared__ uint8_t T[WORK ? kTabBytes : 4];
	if (WORK)
		load_tab(T);
	uint32_t s = 1;
	uint32_t rb, re;
	wg_range(n, rb, re);
	if (threadIdx.x == 0)
		next = rb + 2 * kThreads;
	__syncthreads();
	const uint32_t r = threadIdx.x & 3;
	struct QEv {
		uint32_t idx, nw;
		unsigned long long a0;
	};
	auto qev = [&](uint32_t i) {
		QEv e;
		e.idx = i;
		if (i < re) {
			const unsigned long long a = (unsigned long long)(uintptr_t)(pay + off[i]);
			e.a0 = a & ~63ull;
			e.nw = (uint32_t)(((a & 63ull) + len[i] + 63ull) >> 6);
		} else {
			e.a0 = (unsigned long long)(uintptr_t)pay;
			e.nw = 0;
		}
		return e;
	};
	QEv e0 = qev(rb + threadIdx.x), e1 = qev(rb + kThreads + threadIdx.x);
	uint32_t w0 = 0, acc = 0, tidx = e0.idx, tw = 0;
	v4u W[4];
	auto issue = [&](unsigned long long a0, uint32_t nw, uint32_t w) {
		const unsigned long long a = a0 + 64ull * min(w, nw ? nw - 1 : 0u);
		unsigned long long ak[4];
		ak[0] = qbcast64<0>(a), ak[1] = qbcast64<1>(a), ak[2] = qbcast64<2>(a), ak[3] = qbcast64<3>(a);
#pragma unroll
		for (int k = 0; k < 4; k++)
			W[k] = ld16((const uint8_t*)(uintptr_t)(ak[k] + 16ull * r));
	};
	issue(e0.a0, e0.nw, 0);
	while (__any(e0.idx < re)) {
		const bool valid = e0.idx < re && tidx == e0.idx && tw == w0;
		v4u X[4] = {W[0], W[1], W[2], W[3]};
		{
			const bool same = !valid || w0 + 1 < e0.nw;
			const uint32_t nw = !valid ? w0 : same ? w0 + 1 : 0;
			const QEv& ne = same ? e0 : e1;
			issue(ne.a0, ne.nw, nw);
			tidx = ne.idx;
			tw = nw;
		}
		transpose_quad(X, r);
		if (valid) {
#pragma unroll
			for (int k = 0; k < 4; k++)
				consume<WORK>(T, X[k], s, acc);
			if (++w0 >= e0.nw) {
				e0 = e1;
				e1 = qev(atomicAdd(&next, 1u));
				w0 = 0;
			}
		}
	}
	out[blockIdx.x * kThreads + threadIdx.x] = acc + s;
}

// ---- dma: LDS-DMA ring ----
constexpr uint32_t kSlot = 16384, kSlots = 8;
constexpr uint32_t kSpinMax = 1u << 24;
__device__ __forceinline__ uint32_t lds_acq(const uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void lds_rel(uint32_t* p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP); }
// slot word: (tile + kSlots) << 1 | ready
__device__ __forceinline__ uint32_t sw(uint32_t t, uint32_t ready) { return ((t + kSlots) << 1) | ready; }

template <int N>
__device__ __forceinline__ void wait_vm() {
	static_assert(N >= 0 && N < 64, "vmcnt");
	asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int L, int D>
__global__ __launch_bounds__(kThreads) void k_dma(const uint8_t* pay, const uint64_t* off, const uint32_t* len, uint32_t n,
		uint32_t* out, uint32_t* err) {
	__shared__ __attribute__((aligned(16))) uint8_t ring[kSlots][kSlot];
	__shared__ uint32_t sst[kSlots], take;
	uint32_t rb, re;
	wg_range(n, rb, re);
	const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
	if (threadIdx.x < kSlots)
		sst[threadIdx.x] = sw(threadIdx.x - kSlots, 0); // "tile slot - kSlots was freed"
	if (threadIdx.x == 0)
		take = 0;
	__syncthreads();
	uint64_t lo = 0, hi = 0;
	if (rb < re) {
		lo = off[rb] & ~15ull;
		hi = (off[re - 1] + len[re - 1] + 15) & ~15ull;
	}
	const uint32_t ntiles = (uint32_t)((hi - lo + kSlot - 1) / kSlot);
	uint32_t acc = 0;
	if (wave < (uint32_t)L) {
		// loader: tiles wave, wave + L, ...; D of its own in flight
		uint32_t issued = 0, marked = 0;
		uint32_t tl[D];
		for (uint32_t t = wave; t < ntiles; t += L) {
			const uint32_t s = t % kSlots;
			uint32_t spins = 0;
			while (lds_acq(&sst[s]) != sw(t - kSlots, 0)) {
				if (++spins > kSpinMax) {
					atomicOr(err, 1u);
					goto done;
				}
				__builtin_amdgcn_s_sleep(1);
			}
			const uint64_t base = lo + (uint64_t)t * kSlot;
#pragma unroll
			for (uint32_t k = 0; k < kSlot / 1024; k++) {
				const uint64_t o = base + k * 1024u + lane * 16u;
				__builtin_amdgcn_global_load_lds((const void*)(pay + min(o, hi - 16)),
						(__attribute__((address_space(3))) void*)(&ring[s][k * 1024u]), 16, 0, 0);
			}
			tl[issued % D] = t;
			issued++;
			if (issued - marked == (uint32_t)D) { // the oldest of D in flight is in LDS
				wait_vm<(D - 1) * (kSlot / 1024)>();
				const uint32_t tt = tl[marked % D];
				lds_rel(&sst[tt % kSlots], sw(tt, 1));
				marked++;
			}
		}
		wait_vm<0>();
		while (marked < issued) {
			const uint32_t tt = tl[marked % D];
			lds_rel(&sst[tt % kSlots], sw(tt, 1));
			marked++;
		}
	} else {
		for (;;) {
			uint32_t t = 0;
			if (lane == 0)
				t = atomicAdd(&take, 1u);
			t = __builtin_amdgcn_readfirstlane(t);
			if (t >= ntiles)
				break;
			const uint32_t s = t % kSlots;
			uint32_t spins = 0;
			while (lds_acq(&sst[s]) != sw(t, 1)) {
				if (++spins > kSpinMax) {
					atomicOr(err, 2u);
					goto done;
				}
				__builtin_amdgcn_s_sleep(1);
			}
#pragma unroll
			for (uint32_t k = 0; k < kSlot / 1024; k++)
				acc ^= fold(*(const v4u*)&ring[s][k * 1024u + lane * 16u]);
			lds_rel(&sst[s], sw(t, 0));
		}
	}
done:
	out[blockIdx.x * kThreads + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
	const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 20000000u;
	const int reps = argc > 2 ? atoi(argv[2]) : 5;
	std::mt19937_64 rng(3);
	std::lognormal_distribution<double> ln(5.3, 0.75);
	std::vector<uint32_t> len(n);
	std::vector<uint64_t> off(n);
	uint64_t at = 0, sum = 0;
	for (uint32_t i = 0; i < n; i++) {
		const double x = ln(rng);
		const uint32_t L = (uint32_t)std::min(1024.0, std::max(32.0, x));
		len[i] = L;
		off[i] = at;
		at = (at + L + 15) & ~15ull;
		sum += L;
	}
	const uint64_t bytes = at + 256;
	printf("events %u, payload %.3f GB (mean %.1f B), arena %.3f GB\n", n, sum / 1e9, (double)sum / n, bytes / 1e9);
	uint8_t* dp;
	uint64_t* doff;
	uint32_t *dlen, *dout, *derr;
	CK(hipMalloc(&dp, bytes));
	CK(hipMemset(dp, 0x41, bytes));
	CK(hipMalloc(&doff, n * 8ull));
	CK(hipMalloc(&dlen, n * 4ull));
	CK(hipMemcpy(doff, off.data(), n * 8ull, hipMemcpyHostToDevice));
	CK(hipMemcpy(dlen, len.data(), n * 4ull, hipMemcpyHostToDevice));
	int cus = 0;
	CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
	CK(hipMalloc(&dout, (size_t)cus * kThreads * 4));
	CK(hipMalloc(&derr, 4));
	CK(hipMemset(derr, 0, 4));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	auto run = [&](const char* name, auto launch) {
		std::vector<float> ms;
		for (int r = 0; r < reps + 1; r++) {
			CK(hipEventRecord(e0));
			launch();
			CK(hipEventRecord(e1));
			CK(hipEventSynchronize(e1));
			float t;
			CK(hipEventElapsedTime(&t, e0, e1));
			if (r)
				ms.push_back(t);
		}
		std::sort(ms.begin(), ms.end());
		uint32_t err = 0;
		CK(hipMemcpy(&err, derr, 4, hipMemcpyDeviceToHost));
		printf("%-10s best %.3f ms  median %.3f ms  %.2f TB/s (payload) %.2f TB/s (arena)%s\n", name, ms[0], ms[ms.size() / 2],
				sum / (ms[0] * 1e9), at / (ms[0] * 1e9), err ? "  SPIN-TIMEOUT" : "");
		fflush(stdout);
	};
	const dim3 g(cus), b(kThreads);
	run("read", [&] { hipLaunchKernelGGL(k_read, g, b, 0, 0, dp, doff, dlen, n, dout); });
	run("quad64", [&] { hipLaunchKernelGGL((k_quad64<0>), g, b, 0, 0, dp, doff, dlen, n, dout); });
	run("quad64a", [&] { hipLaunchKernelGGL((k_quad64a<0>), g, b, 0, 0, dp, doff, dlen, n, dout); });
	run("oct128", [&] { hipLaunchKernelGGL((k_oct128<0, 1>), g, b, 0, 0, dp, doff, dlen, n, dout); });
	run("oct128e", [&] { hipLaunchKernelGGL((k_oct128<0, 0>), g, b, 0, 0, dp, doff, dlen, n, dout); });
	run("quad64+W", [&] { hipLaunchKernelGGL((k_quad64<1>), g, b, 0, 0, dp, doff, dlen, n, dout); });
	run("quad64a+W", [&] { hipLaunchKernelGGL((k_quad64a<1>), g, b, 0, 0, dp, doff, dlen, n, dout); });
	run("oct128+W", [&] { hipLaunchKernelGGL((k_oct128<1, 1>), g, b, 0, 0, dp, doff, dlen, n, dout); });
	run("oct128e+W", [&] { hipLaunchKernelGGL((k_oct128<1, 0>), g, b, 0, 0, dp, doff, dlen, n, dout); });
	run("dma1x3", [&] { hipLaunchKernelGGL((k_dma<1, 3>), g, b, 0, 0, dp, doff, dlen, n, dout, derr); });
	run("dma2x2", [&] { hipLaunchKernelGGL((k_dma<2, 2>), g, b, 0, 0, dp, doff, dlen, n, dout, derr); });
	run("dma2x3", [&] { hipLaunchKernelGGL((k_dma<2, 3>), g, b, 0, 0, dp, doff, dlen, n, dout, derr); });
	run("dma4x1", [&] { hipLaunchKernelGGL((k_dma<4, 1>), g, b, 0, 0, dp, doff, dlen, n, dout, derr); });
	run("dma4x2", [&] { hipLaunchKernelGGL((k_dma<4, 2>), g, b, 0, 0, dp, doff, dlen, n, dout, derr); });
	CK(hipDeviceSynchronize());
	return 0;
}
