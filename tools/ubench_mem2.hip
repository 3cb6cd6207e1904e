// ubench_mem2.hip — memory pattern of a lane-per-event scan, with and without the DFA's
// dependent LDS chain, on variable-length events scattered inside 4096-event tiles (as the
// tile length sort scatters them).  Variants:
//   lane16   lane reads its own buffer: 16-B loads, 8 per 128-B window, next window in flight
//   perm64   4 lanes {l, l+16, l+32, l+48} read 64 contiguous bytes of one event per
//            instruction (4 instructions = one 64-B window for each of the 4 events), then a
//            4x4 block transpose by v_permlane32_swap / v_permlane16_swap hands every lane
//            its own window; DEPTH windows in flight
// WORK=1 adds 16 dependent ds_read_u8 table steps per chunk (the DFA's cost shape).
//   hipcc --offload-arch=gfx950 -O3 -o ubench_mem2 tools/ubench_mem2.hip && ./ubench_mem2
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4u ld16(uintptr_t a) { return *(const __attribute__((address_space(1))) v4u*)a; }

constexpr int kLds = 132 * 1024;

template <int WORK>
__device__ __forceinline__ void consume(const uint8_t* T, const v4u& w, uint32_t& s, uint32_t& acc) {
	if (WORK) {
#pragma unroll
		for (int k = 0; k < 16; k++) {
			const uint32_t b = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
			s = T[s * 260u + b];
			acc = max(acc, s);
		}
	} else {
		acc ^= w.x ^ w.y ^ w.z ^ w.w;
	}
}

// events: off[i] (16-B aligned), len[i]; order[i] = the event lane slot i scans
template <int WORK>
__global__ __launch_bounds__(1024) void k_lane16(const uint8_t* buf, const unsigned long long* off, const uint32_t* len,
		const uint32_t* order, uint32_t n, const uint8_t* gtab, uint32_t* out) {
	extern __shared__ uint8_t T[];
	for (uint32_t k = threadIdx.x * 4; k < 194 * 260; k += 1024 * 4)
		*(uint32_t*)(T + k) = *(const uint32_t*)(gtab + k);
	__syncthreads();
	uint32_t acc = 0, s = 1;
	for (uint32_t base = blockIdx.x * 1024; base < n; base += gridDim.x * 1024) {
		const uint32_t e = order[min(base + threadIdx.x, n - 1)];
		const uintptr_t q = (uintptr_t)(buf + off[e]) & ~(uintptr_t)127;
		const uint32_t nch = (uint32_t)(((uintptr_t)(buf + off[e]) & 127) + len[e] + 15) >> 4;
		const uint32_t last = nch - 1;
		uint32_t maxch = nch;
		for (int o = 32; o; o >>= 1)
			maxch = max(maxch, (uint32_t)__shfl_xor((int)maxch, o));
		v4u A[8], B[8];
		auto ldw = [&](v4u(&w)[8], uint32_t j) {
#pragma unroll
			for (int k = 0; k < 8; k++)
				w[k] = ld16(q + 16 * (uintptr_t)min(8 * j + k, last));
		};
		ldw(A, 0);
		for (uint32_t j = 0; 8 * j < maxch; j += 2) {
			ldw(B, j + 1);
#pragma unroll
			for (int k = 0; k < 8; k++)
				consume<WORK>(T, A[k], s, acc);
			if (8 * (j + 1) >= maxch)
				break;
			ldw(A, j + 2);
#pragma unroll
			for (int k = 0; k < 8; k++)
				consume<WORK>(T, B[k], s, acc);
		}
	}
	out[blockIdx.x * blockDim.x + threadIdx.x] = acc + s;
}

// 4x4 transpose of 16-B blocks among lanes {l, l+16, l+32, l+48}: lane member j holds
// X[k] = piece j of event k; afterwards it holds piece k of event j.
__device__ __forceinline__ void transpose4(v4u (&X)[4]) {
#pragma unroll
	for (int k = 0; k < 2; k++)
#pragma unroll
		for (int d = 0; d < 4; d++) {
			auto r = __builtin_amdgcn_permlane32_swap(X[k][d], X[k + 2][d], false, false);
			X[k][d] = r[0];
			X[k + 2][d] = r[1];
		}
#pragma unroll
	for (int k = 0; k < 4; k += 2)
#pragma unroll
		for (int d = 0; d < 4; d++) {
			auto r = __builtin_amdgcn_permlane16_swap(X[k][d], X[k + 1][d], false, false);
			X[k][d] = r[0];
			X[k + 1][d] = r[1];
		}
}

template <int WORK, int DEPTH>
__global__ __launch_bounds__(1024) void k_perm64(const uint8_t* buf, const unsigned long long* off, const uint32_t* len,
		const uint32_t* order, uint32_t n, const uint8_t* gtab, uint32_t* out) {
	extern __shared__ uint8_t T[];
	for (uint32_t k = threadIdx.x * 4; k < 194 * 260; k += 1024 * 4)
		*(uint32_t*)(T + k) = *(const uint32_t*)(gtab + k);
	__syncthreads();
	const uint32_t lane = threadIdx.x & 63, j = lane >> 4;
	uint32_t acc = 0, s = 1;
	for (uint32_t base = blockIdx.x * 1024; base < n; base += gridDim.x * 1024) {
		const uint32_t wbase = base + (threadIdx.x & ~63u);
		// the group's 4 events (members k = 0..3 are lanes (lane & 15) + 16 k)
		uintptr_t gq[4];
		uint32_t glast[4];
		uint32_t nch = 0;
#pragma unroll
		for (int k = 0; k < 4; k++) {
			const uint32_t e = order[min(wbase + (lane & 15) + 16 * k, n - 1)];
			const uintptr_t p = (uintptr_t)(buf + off[e]);
			gq[k] = p & ~(uintptr_t)15;
			const uint32_t c = (uint32_t)((p & 15) + len[e] + 15) >> 4;
			glast[k] = c - 1;
			if ((uint32_t)k == j)
				nch = c;
		}
		uint32_t maxch = nch;
		for (int o = 32; o; o >>= 1)
			maxch = max(maxch, (uint32_t)__shfl_xor((int)maxch, o));
		const uint32_t nwin = (maxch + 3) / 4;
		v4u W[DEPTH][4];
		auto ldw = [&](v4u(&w)[4], uint32_t win) {
#pragma unroll
			for (int k = 0; k < 4; k++)
				w[k] = ld16(gq[k] + 16 * (uintptr_t)min(4 * win + j, glast[k]));
		};
#pragma unroll
		for (int d = 0; d < DEPTH; d++)
			ldw(W[d], d);
		for (uint32_t win = 0; win < nwin; win += DEPTH) {
#pragma unroll
			for (int d = 0; d < DEPTH; d++) {
				if (win + d < nwin) {
					v4u X[4] = {W[d][0], W[d][1], W[d][2], W[d][3]};
					ldw(W[d], win + d + DEPTH);
					transpose4(X);
#pragma unroll
					for (int c = 0; c < 4; c++)
						consume<WORK>(T, X[c], s, acc);
				}
			}
		}
	}
	out[blockIdx.x * blockDim.x + threadIdx.x] = acc + s;
}

// quad_perm DPP helper: value of `v` from quad lane pattern
template <int P>
__device__ __forceinline__ uint32_t qperm(uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, P, 0xf, 0xf, true); }
constexpr int kQX2 = (2) | (3 << 2) | (0 << 4) | (1 << 6); // lane r takes r ^ 2
constexpr int kQX1 = (1) | (0 << 2) | (3 << 4) | (2 << 6); // lane r takes r ^ 1

// 4x4 transpose of 16-B blocks among the 4 lanes of a quad: lane r holds X[k] = piece r of
// event k; afterwards piece k of event r.
__device__ __forceinline__ void transpose_quad(v4u (&X)[4], uint32_t r) {
	const bool lo2 = r < 2, lo1 = (r & 1) == 0;
#pragma unroll
	for (int k = 0; k < 2; k++)
#pragma unroll
		for (int d = 0; d < 4; d++) {
			const uint32_t send = lo2 ? X[k + 2][d] : X[k][d];
			const uint32_t recv = qperm<kQX2>(send);
			X[k + 2][d] = lo2 ? recv : X[k + 2][d];
			X[k][d] = lo2 ? X[k][d] : recv;
		}
#pragma unroll
	for (int k = 0; k < 4; k += 2)
#pragma unroll
		for (int d = 0; d < 4; d++) {
			const uint32_t send = lo1 ? X[k + 1][d] : X[k][d];
			const uint32_t recv = qperm<kQX1>(send);
			X[k + 1][d] = lo1 ? recv : X[k + 1][d];
			X[k][d] = lo1 ? X[k][d] : recv;
		}
}

template <int WORK, int DEPTH, int SORTED>
__global__ __launch_bounds__(1024) void k_quad64(const uint8_t* buf, const unsigned long long* off, const uint32_t* len,
		const uint32_t* order, uint32_t n, const uint8_t* gtab, uint32_t* out) {
	extern __shared__ uint8_t T[];
	for (uint32_t k = threadIdx.x * 4; k < 194 * 260; k += 1024 * 4)
		*(uint32_t*)(T + k) = *(const uint32_t*)(gtab + k);
	__syncthreads();
	const uint32_t lane = threadIdx.x & 63, r = lane & 3;
	uint32_t acc = 0, s = 1;
	for (uint32_t base = blockIdx.x * 1024; base < n; base += gridDim.x * 1024) {
		const uint32_t qbase = base + (threadIdx.x & ~3u);
		uintptr_t gq[4];
		uint32_t glast[4];
		uint32_t nch = 0;
#pragma unroll
		for (int k = 0; k < 4; k++) {
			const uint32_t i = min(qbase + k, n - 1);
			const uint32_t e = SORTED ? order[i] : i;
			const uintptr_t p = (uintptr_t)(buf + off[e]);
			gq[k] = p & ~(uintptr_t)15;
			const uint32_t c = (uint32_t)((p & 15) + len[e] + 15) >> 4;
			glast[k] = c - 1;
			if ((uint32_t)k == r)
				nch = c;
		}
		uint32_t maxch = nch;
		for (int o = 32; o; o >>= 1)
			maxch = max(maxch, (uint32_t)__shfl_xor((int)maxch, o));
		const uint32_t nwin = (maxch + 3) / 4;
		v4u W[DEPTH][4];
		auto ldw = [&](v4u(&w)[4], uint32_t win) {
#pragma unroll
			for (int k = 0; k < 4; k++)
				w[k] = ld16(gq[k] + 16 * (uintptr_t)min(4 * win + r, glast[k]));
		};
#pragma unroll
		for (int d = 0; d < DEPTH; d++)
			ldw(W[d], d);
		for (uint32_t win = 0; win < nwin; win += DEPTH) {
#pragma unroll
			for (int d = 0; d < DEPTH; d++) {
				if (win + d < nwin) {
					v4u X[4] = {W[d][0], W[d][1], W[d][2], W[d][3]};
					ldw(W[d], win + d + DEPTH);
					transpose_quad(X, r);
#pragma unroll
					for (int c = 0; c < 4; c++)
						consume<WORK>(T, X[c], s, acc);
				}
			}
		}
	}
	out[blockIdx.x * blockDim.x + threadIdx.x] = acc + s;
}

// Continuous pipeline: the window loads run D windows ahead of consumption, across group
// boundaries (a wave takes groups gw, gw + nW, ...; a group = 64 consecutive slots of order[]).
struct QMeta {
	uintptr_t q[4];
	uint32_t last[4];
	uint32_t nwin; // wave-uniform: windows of the group's longest buffer
};
template <int SORTED>
__device__ __forceinline__ QMeta qmeta(const uint8_t* buf, const unsigned long long* off, const uint32_t* len,
		const uint32_t* order, uint32_t n, uint32_t g, uint32_t lane) {
	QMeta m;
	uint32_t own = 0;
#pragma unroll
	for (int k = 0; k < 4; k++) {
		// SORTED: off / len already permuted into slot order on the host (no dependent loads)
		const uint32_t i = min(g * 64 + (lane & ~3u) + k, n - 1);
		const uintptr_t p = (uintptr_t)(buf + off[i]);
		m.q[k] = p & ~(uintptr_t)15;
		const uint32_t c = (uint32_t)((p & 15) + len[i] + 15) >> 4;
		m.last[k] = c - 1;
		own = (uint32_t)k == (lane & 3) ? c : own;
	}
	uint32_t mx = own;
	for (int o = 32; o; o >>= 1)
		mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
	m.nwin = __builtin_amdgcn_readfirstlane((mx + 3) / 4);
	return m;
}

template <int WORK, int D, int SORTED>
__global__ __launch_bounds__(1024) void k_quad64c(const uint8_t* buf, const unsigned long long* off, const uint32_t* len,
		const uint32_t* order, uint32_t n, const uint8_t* gtab, uint32_t* out) {
	extern __shared__ uint8_t T[];
	for (uint32_t k = threadIdx.x * 4; k < 194 * 260; k += 1024 * 4)
		*(uint32_t*)(T + k) = *(const uint32_t*)(gtab + k);
	__syncthreads();
	const uint32_t lane = threadIdx.x & 63, r = lane & 3;
	const uint32_t nW = gridDim.x * (blockDim.x / 64), gw = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
	const uint32_t ngroups = (n + 63) / 64;
	uint32_t acc = 0, s = 1;
	// prefetch side
	uint32_t pg = gw, pw = 0;
	QMeta pm = qmeta<SORTED>(buf, off, len, order, n, min(pg, ngroups - 1), lane);
	QMeta pn = qmeta<SORTED>(buf, off, len, order, n, min(pg + nW, ngroups - 1), lane);
	unsigned long long qv = pm.nwin; // queue of group window counts, 8 bits each (uniform)
	uint32_t qn = 1;
	auto issue = [&](v4u(&w)[4]) {
#pragma unroll
		for (int k = 0; k < 4; k++)
			w[k] = ld16(pm.q[k] + 16 * (uintptr_t)min(4 * pw + r, pm.last[k]));
		if (++pw == pm.nwin) {
			pw = 0;
			pg += nW;
			pm = pn;
			qv |= (unsigned long long)pm.nwin << (8 * qn); // windows of the group the prefetch enters
			qn++;
			pn = qmeta<SORTED>(buf, off, len, order, n, min(pg + nW, ngroups - 1), lane);
		}
	};
	v4u W[D][4];
#pragma unroll
	for (int d = 0; d < D; d++)
		issue(W[d]);
	// consume side
	uint32_t cg = gw, cw = 0, cn = (uint32_t)(qv & 255);
	qv >>= 8;
	qn--;
	while (cg < ngroups) {
#pragma unroll
		for (int d = 0; d < D; d++) {
			v4u X[4] = {W[d][0], W[d][1], W[d][2], W[d][3]};
			issue(W[d]);
			transpose_quad(X, r);
#pragma unroll
			for (int c = 0; c < 4; c++)
				consume<WORK>(T, X[c], s, acc);
			if (++cw == cn) {
				cw = 0;
				cg += nW;
				if (cg >= ngroups)
					break;
				cn = (uint32_t)(qv & 255);
				qv >>= 8;
				qn--;
				s = 1;
			}
		}
	}
	out[blockIdx.x * blockDim.x + threadIdx.x] = acc + s;
}

int main(int argc, char** argv) {
	hipDeviceProp_t prop;
	(void)hipGetDeviceProperties(&prop, 0);
	const int cus = prop.multiProcessorCount;
	const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 20000000;
	// lengths: lognormal-ish clamp [32, 1024], mean ~256 (like config 3)
	std::mt19937_64 rng(7);
	std::lognormal_distribution<double> ln(5.3, 0.55);
	std::vector<uint32_t> len(n), order(n);
	std::vector<unsigned long long> off(n);
	unsigned long long o = 0, total = 0;
	for (uint32_t i = 0; i < n; i++) {
		double v = ln(rng);
		uint32_t L = (uint32_t)std::min(1024.0, std::max(32.0, v));
		if (getenv("UB_FIXED"))
			L = (uint32_t)atoi(getenv("UB_FIXED"));
		len[i] = L;
		off[i] = o;
		o += (L + 15) & ~15u;
		total += L;
	}
	// within each 4096-event tile, sort by length (longest first), like k_fresh's binning
	for (uint32_t t = 0; t < n; t += 4096) {
		const uint32_t e = std::min(n, t + 4096);
		for (uint32_t i = t; i < e; i++)
			order[i] = i;
		if (getenv("UB_SHUFFLE"))
			std::shuffle(order.begin() + t, order.begin() + e, rng);
		std::stable_sort(order.begin() + t, order.begin() + e, [&](uint32_t a, uint32_t b) { return len[a] / 16 > len[b] / 16; });
	}
	std::vector<uint8_t> tab(194 * 260);
	uint32_t x = 12345;
	for (int st = 0; st < 194; st++)
		for (int b = 0; b < 260; b++) {
			x = x * 1664525u + 1013904223u;
			tab[st * 260 + b] = ((x >> 8) & 7) ? (uint8_t)st : (uint8_t)((x >> 24) % 194);
		}
	uint8_t *buf, *dtab;
	unsigned long long* doff;
	uint32_t *dlen, *dorder, *dout;
	if (hipMalloc(&buf, o + 4096) || hipMalloc(&doff, n * 8ull) || hipMalloc(&dlen, n * 4ull) || hipMalloc(&dorder, n * 4ull) ||
			hipMalloc(&dout, (size_t)cus * 16 * 1024 * 4) || hipMalloc(&dtab, tab.size()))
		return 1;
	(void)hipMemset(buf, 0x61, o + 4096);
	(void)hipMemcpy(doff, off.data(), n * 8ull, hipMemcpyHostToDevice);
	(void)hipMemcpy(dlen, len.data(), n * 4ull, hipMemcpyHostToDevice);
	(void)hipMemcpy(dorder, order.data(), n * 4ull, hipMemcpyHostToDevice);
	(void)hipMemcpy(dtab, tab.data(), tab.size(), hipMemcpyHostToDevice);
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	auto time = [&](const char* name, auto launch) {
		launch();
		(void)hipEventRecord(a);
		launch();
		(void)hipEventRecord(b);
		(void)hipEventSynchronize(b);
		float ms = 0;
		(void)hipEventElapsedTime(&ms, a, b);
		printf("n=%u %-16s %8.3f ms  %7.0f GB/s useful (%.2f GB)\n", n, name, ms, total / (ms * 1e-3) / 1e9, total / 1e9);
	};
	const dim3 g(cus * 2), blk(1024);
	const int lds = getenv("UB_LDS") ? atoi(getenv("UB_LDS")) * 1024 : kLds;
	printf("dynamic LDS per workgroup: %d KB\n", lds / 1024);
#define RUN(NAME, K) time(NAME, [&] { hipLaunchKernelGGL(K, g, blk, lds, 0, buf, doff, dlen, dorder, n, dtab, dout); })
	// slot-ordered copies of off / len for the continuous-pipeline kernels
	std::vector<unsigned long long> soff(n);
	std::vector<uint32_t> slen(n);
	for (uint32_t i = 0; i < n; i++) {
		soff[i] = off[order[i]];
		slen[i] = len[order[i]];
	}
	unsigned long long* dsoff;
	uint32_t* dslen;
	if (hipMalloc(&dsoff, n * 8ull) || hipMalloc(&dslen, n * 4ull))
		return 1;
	(void)hipMemcpy(dsoff, soff.data(), n * 8ull, hipMemcpyHostToDevice);
	(void)hipMemcpy(dslen, slen.data(), n * 4ull, hipMemcpyHostToDevice);
#define RUNS(NAME, K) time(NAME, [&] { hipLaunchKernelGGL(K, g, blk, lds, 0, buf, dsoff, dslen, dorder, n, dtab, dout); })
#define RUNU(NAME, K) time(NAME, [&] { hipLaunchKernelGGL(K, g, blk, lds, 0, buf, doff, dlen, dorder, n, dtab, dout); })
	RUN("lane16/mem", (k_lane16<0>));
	RUN("perm64x1/mem", (k_perm64<0, 1>));
	RUN("perm64x2/mem", (k_perm64<0, 2>));
	RUN("perm64x3/mem", (k_perm64<0, 3>));
	RUN("quad64x1/mem", (k_quad64<0, 1, 1>));
	RUN("quad64x2/mem", (k_quad64<0, 2, 1>));
	RUN("quad64x2/mem/unsorted", (k_quad64<0, 2, 0>));
	RUNS("quad64c2/mem", (k_quad64c<0, 2, 1>));
	RUNS("quad64c3/mem", (k_quad64c<0, 3, 1>));
	RUNU("quad64c3/mem/unsorted", (k_quad64c<0, 3, 0>));
	RUN("lane16/work", (k_lane16<1>));
	RUN("perm64x1/work", (k_perm64<1, 1>));
	RUN("perm64x2/work", (k_perm64<1, 2>));
	RUN("perm64x3/work", (k_perm64<1, 3>));
	RUN("quad64x1/work", (k_quad64<1, 1, 1>));
	RUN("quad64x2/work", (k_quad64<1, 2, 1>));
	RUN("quad64x2/work/unsorted", (k_quad64<1, 2, 0>));
	RUNS("quad64c2/work", (k_quad64c<1, 2, 1>));
	RUNS("quad64c3/work", (k_quad64c<1, 3, 1>));
	RUNU("quad64c3/work/unsorted", (k_quad64c<1, 3, 0>));
	return 0;
}
