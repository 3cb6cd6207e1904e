// ubench_lockstep.hip — the payload stream of a k_fresh built from length-sorted lockstep groups,
// against the lane-refill stream (quad64a) it would replace.  Config-3-like events (lengths
// 32..1024, mean ~256, packed at 16-B alignment), one 1024-thread workgroup per CU owning a
// contiguous event range.  The range is cut into blocks of 1024 events, each block's events
// ordered by their count of 64-B grid windows (the host sorts here; the kernel would sort in
// LDS), and a wave takes 64 consecutive entries of that order at a time: its lanes then walk
// events of nearly one length window by window in lockstep, with no per-lane event hand-off.
//   lock64     that stream with a trivial consumer (XOR)
//   lock64+W   16 dependent LDS table steps per 16-B piece (the DFA's cost shape)
//   lock64+Wh  the table steps on every second 16-B piece only (a chunk skip taking half)
//   quad64a+W  the lane-refill stream with the same work (tools/ubench_stream.hip's)
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_lockstep tools/ubench_lockstep.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
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
constexpr uint32_t kBlock = 1024;

__device__ __forceinline__ void wg_range(uint32_t n, uint32_t& rb, uint32_t& re) {
	const uint32_t per = (uint32_t)(((unsigned long long)n + gridDim.x - 1) / gridDim.x);
	rb = min(n, blockIdx.x * per);
	re = min(n, rb + per);
}

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

struct QEv {
	uint32_t nw;
	unsigned long long a0;
};
__device__ __forceinline__ QEv qev(const uint8_t* pay, const uint64_t* off, const uint32_t* len, bool ok, uint32_t i) {
	QEv e;
	if (ok) {
		const unsigned long long a = (unsigned long long)(uintptr_t)(pay + off[i]);
		e.a0 = a & ~63ull;
		e.nw = (uint32_t)(((a & 63ull) + len[i] + 63ull) >> 6);
	} else {
		e.a0 = (unsigned long long)(uintptr_t)pay;
		e.nw = 0;
	}
	return e;
}

// WORK: 0 none, 1 every piece, 2 every second piece
template <int WORK>
__global__ __launch_bounds__(kThreads) void k_lock(const uint8_t* pay, const uint64_t* off, const uint32_t* len, const uint32_t* order,
		uint32_t n, uint32_t* out) {
	__shared__ uint32_t next;
	__shared__ uint8_t T[WORK ? kTabBytes : 4];
	if (WORK)
		load_tab(T);
	uint32_t rb, re;
	wg_range(n, rb, re);
	if (threadIdx.x == 0)
		next = 0;
	__syncthreads();
	const uint32_t lane = threadIdx.x & 63, r = lane & 3;
	const uint32_t ngroups = (re - rb + 63) / 64;
	uint32_t s = 1, acc = 0;
	auto pop = [&]() {
		uint32_t g = 0;
		if (lane == 0)
			g = atomicAdd(&next, 1u);
		return __builtin_amdgcn_readfirstlane(g);
	};
	auto group_ev = [&](uint32_t g) {
		const uint32_t k = rb + 64 * g + lane;
		const bool ok = g < ngroups && k < re;
		return qev(pay, off, len, ok, ok ? order[k] : 0u);
	};
	v4u W[4];
	auto issue = [&](unsigned long long a0, uint32_t nw, uint32_t w) {
		const unsigned long long a = a0 + 64ull * min(w, nw ? nw - 1 : 0u);
		unsigned long long ak[4];
		ak[0] = qbcast64<0>(a), ak[1] = qbcast64<1>(a), ak[2] = qbcast64<2>(a), ak[3] = qbcast64<3>(a);
#pragma unroll
		for (int k = 0; k < 4; k++)
			W[k] = ld16((const uint8_t*)(uintptr_t)(ak[k] + 16ull * r));
	};
	uint32_t g = pop();
	QEv e = group_ev(g);
	uint32_t g1 = pop();
	QEv e1 = group_ev(g1);
	issue(e.a0, e.nw, 0);
	while (g < ngroups) {
		// lanes walk their events window by window together; the group ends with its longest
		uint32_t w = 0;
		for (;;) {
			v4u X[4] = {W[0], W[1], W[2], W[3]};
			const bool more = __any(w + 1 < e.nw);
			if (more)
				issue(e.a0, e.nw, w + 1);
			else
				issue(e1.a0, e1.nw, 0); // the next group's first window, in flight across the switch
			transpose_quad(X, r);
			if (w < e.nw) {
#pragma unroll
				for (int k = 0; k < 4; k++) {
					if (WORK == 2 && (k & 1))
						acc ^= fold(X[k]);
					else
						consume<WORK>(T, X[k], s, acc);
				}
			}
			w++;
			if (!more)
				break;
		}
		g = g1;
		e = e1;
		g1 = pop();
		e1 = group_ev(g1);
	}
	out[blockIdx.x * kThreads + threadIdx.x] = acc + s;
}

// quad64a+W: the lane-refill stream (tools/ubench_stream.hip)
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
	struct REv {
		uint32_t idx, nw;
		unsigned long long a0;
	};
	auto rev = [&](uint32_t i) {
		REv e;
		e.idx = i;
		const QEv q = qev(pay, off, len, i < re, i);
		e.nw = q.nw;
		e.a0 = q.a0;
		return e;
	};
	REv e0 = rev(rb + threadIdx.x), e1 = rev(rb + kThreads + threadIdx.x);
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
			const REv& ne = same ? e0 : e1;
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
				e1 = rev(atomicAdd(&next, 1u));
				w0 = 0;
			}
		}
	}
	out[blockIdx.x * kThreads + threadIdx.x] = acc + s;
}

int main(int argc, char** argv) {
	const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 20000000u;
	const int reps = argc > 2 ? atoi(argv[2]) : 5;
	std::mt19937_64 rng(3);
	std::lognormal_distribution<double> ln(5.3, 0.75);
	std::vector<uint32_t> len(n), nwin(n), order(n);
	std::vector<uint64_t> off(n);
	uint64_t at = 0, sum = 0;
	for (uint32_t i = 0; i < n; i++) {
		const double x = ln(rng);
		const uint32_t L = (uint32_t)std::min(1024.0, std::max(32.0, x));
		len[i] = L;
		off[i] = at;
		nwin[i] = (uint32_t)(((at & 63) + L + 63) >> 6);
		at = (at + L + 15) & ~15ull;
		sum += L;
	}
	int cus = 0;
	CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
	// each workgroup's range in blocks of kBlock events, each block by window count (longest first)
	const uint32_t per = (uint32_t)(((unsigned long long)n + cus - 1) / cus);
	std::iota(order.begin(), order.end(), 0u);
	uint64_t lock_windows = 0, windows = 0;
	for (uint32_t b = 0; b < (uint32_t)cus; b++) {
		const uint32_t rb = std::min(n, b * per), re = std::min(n, rb + per);
		for (uint32_t k = rb; k < re; k += kBlock) {
			const uint32_t ke = std::min(re, k + kBlock);
			std::stable_sort(order.begin() + k, order.begin() + ke, [&](uint32_t x, uint32_t y) { return nwin[x] > nwin[y]; });
		}
		for (uint32_t k = rb; k < re; k += 64) {
			uint32_t mx = 0;
			for (uint32_t j = k; j < std::min(re, k + 64); j++) {
				mx = std::max(mx, nwin[order[j]]);
				windows += nwin[order[j]];
			}
			lock_windows += 64ull * mx;
		}
	}
	const uint64_t bytes = at + 256;
	printf("events %u, payload %.3f GB (mean %.1f B), arena %.3f GB; lockstep lane use %.3f\n", n, sum / 1e9, (double)sum / n,
			bytes / 1e9, (double)windows / lock_windows);
	uint8_t* dp;
	uint64_t* doff;
	uint32_t *dlen, *dout, *dord;
	CK(hipMalloc(&dp, bytes));
	CK(hipMemset(dp, 0x41, bytes));
	CK(hipMalloc(&doff, n * 8ull));
	CK(hipMalloc(&dlen, n * 4ull));
	CK(hipMalloc(&dord, n * 4ull));
	CK(hipMemcpy(doff, off.data(), n * 8ull, hipMemcpyHostToDevice));
	CK(hipMemcpy(dlen, len.data(), n * 4ull, hipMemcpyHostToDevice));
	CK(hipMemcpy(dord, order.data(), n * 4ull, hipMemcpyHostToDevice));
	CK(hipMalloc(&dout, (size_t)cus * kThreads * 4));
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
		printf("%-10s best %.3f ms  median %.3f ms  %.2f TB/s (payload) %.2f TB/s (arena)\n", name, ms[0], ms[ms.size() / 2],
				sum / (ms[0] * 1e9), at / (ms[0] * 1e9));
		fflush(stdout);
	};
	const dim3 g(cus), b(kThreads);
	run("lock64", [&] { hipLaunchKernelGGL((k_lock<0>), g, b, 0, 0, dp, doff, dlen, dord, n, dout); });
	run("lock64+W", [&] { hipLaunchKernelGGL((k_lock<1>), g, b, 0, 0, dp, doff, dlen, dord, n, dout); });
	run("lock64+Wh", [&] { hipLaunchKernelGGL((k_lock<2>), g, b, 0, 0, dp, doff, dlen, dord, n, dout); });
	run("quad64a", [&] { hipLaunchKernelGGL((k_quad64a<0>), g, b, 0, 0, dp, doff, dlen, n, dout); });
	run("quad64a+W", [&] { hipLaunchKernelGGL((k_quad64a<1>), g, b, 0, 0, dp, doff, dlen, n, dout); });
	CK(hipDeviceSynchronize());
	return 0;
}
