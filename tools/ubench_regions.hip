// ubench_regions.hip — does a service-table pass gain from taking the table one region at a time?
// k_agg_fast's per-request work, reduced to its memory shape: a 32-B probe read of a 64-B slot in a
// 2^26-slot (4.3 GB) table, a CAS claim of an empty slot, a counter atomicAdd and a conditional
// atomicMax.  N requests draw D distinct keys (each key ~N/D times, in random order).
//   direct:  one launch over the requests in index order (what k_agg_fast does);
//   regions: requests bucketed by the slot index's top bits (R regions of 2^26 / R slots, probing
//            wraps inside the region), then one launch per region, so that the region's slots
//            (4.3 GB / R) stay in the 256 MiB Infinity Cache while they are hit.
// Reported per mode: ms (bucketing separately), with the table zeroed before each timed pass.
//   hipcc --offload-arch=gfx950 -O3 -o ubench_regions tools/ubench_regions.hip && ./ubench_regions [R...]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define CK(x)                                                                                         \
	do {                                                                                              \
		hipError_t e_ = (x);                                                                          \
		if (e_ != hipSuccess) {                                                                       \
			std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
			std::exit(1);                                                                             \
		}                                                                                             \
	} while (0)

struct Slot {
	unsigned long long tag, hi, nfirst;
	unsigned int internal_clients, external_clients;
	unsigned long long pad[4];
};
static_assert(sizeof(Slot) == 64, "64-B slot");

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
	x ^= x >> 30;
	x *= 0xbf58476d1ce4e5b9ull;
	x ^= x >> 27;
	x *= 0x94d049bb133111ebull;
	x ^= x >> 31;
	return x | 1ull;
}
__device__ __forceinline__ unsigned long long req_key(unsigned long long i, unsigned long long D) {
	return mix((mix(i + 7) % D) + 1);
}

__device__ __forceinline__ void insert(Slot* slots, uint32_t mask, uint32_t rmask, unsigned long long key, unsigned long long first) {
	uint32_t idx = (uint32_t)(key >> 11) & mask;
	for (uint32_t p = 0; p <= rmask; p++) {
		Slot* s = slots + idx;
		const ulonglong2 th = *(const ulonglong2*)&s->tag;
		unsigned long long t = th.x;
		if (t == 0) {
			t = atomicCAS(&s->tag, 0ull, key);
			if (t == 0) {
				atomicExch(&s->hi, key ^ 0x5555ull);
				t = key;
			}
		}
		if (t == key) {
			atomicAdd(&s->internal_clients, 1u);
			if (~first > s->nfirst)
				atomicMax(&s->nfirst, ~first);
			return;
		}
		idx = (idx & ~rmask) | ((idx + 1) & rmask);
	}
}

__global__ __launch_bounds__(256) void k_direct(Slot* slots, uint32_t mask, unsigned long long n, unsigned long long D) {
	for (unsigned long long i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (unsigned long long)gridDim.x * 256)
		insert(slots, mask, mask, req_key(i, D), i);
}

// region of a request = top bits of its first slot index
__global__ __launch_bounds__(256) void k_count(uint32_t mask, uint32_t rshift, unsigned long long n, unsigned long long D,
		unsigned long long* cnt) {
	__shared__ unsigned int h[256];
	h[threadIdx.x] = 0;
	__syncthreads();
	for (unsigned long long i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (unsigned long long)gridDim.x * 256)
		atomicAdd(&h[(((uint32_t)(req_key(i, D) >> 11) & mask) >> rshift) & 255u], 1u);
	__syncthreads();
	if (h[threadIdx.x])
		atomicAdd(&cnt[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

// scatter (key, i) pairs into the region lists: per block-tile one global atomic per region
__global__ __launch_bounds__(256) void k_scatter(uint32_t mask, uint32_t rshift, unsigned long long n, unsigned long long D,
		unsigned long long* cur, ulonglong2* out) {
	__shared__ unsigned int h[256];
	__shared__ unsigned long long base[256];
	for (unsigned long long t0 = blockIdx.x * 4096ull; t0 < n; t0 += (unsigned long long)gridDim.x * 4096) {
		h[threadIdx.x] = 0;
		__syncthreads();
		unsigned long long k[16];
		uint32_t rg[16], rk[16];
#pragma unroll
		for (int j = 0; j < 16; j++) {
			const unsigned long long i = t0 + j * 256 + threadIdx.x;
			k[j] = i < n ? req_key(i, D) : 0;
			rg[j] = (((uint32_t)(k[j] >> 11) & mask) >> rshift) & 255u;
			rk[j] = i < n ? atomicAdd(&h[rg[j]], 1u) : 0;
		}
		__syncthreads();
		if (h[threadIdx.x])
			base[threadIdx.x] = atomicAdd(&cur[threadIdx.x], (unsigned long long)h[threadIdx.x]);
		__syncthreads();
#pragma unroll
		for (int j = 0; j < 16; j++) {
			const unsigned long long i = t0 + j * 256 + threadIdx.x;
			if (i < n)
				out[base[rg[j]] + rk[j]] = make_ulonglong2(k[j], i);
		}
		__syncthreads();
	}
}

__global__ __launch_bounds__(256) void k_region(Slot* slots, uint32_t mask, uint32_t rmask, const ulonglong2* in, unsigned long long b,
		unsigned long long e) {
	for (unsigned long long j = b + blockIdx.x * 256ull + threadIdx.x; j < e; j += (unsigned long long)gridDim.x * 256) {
		const ulonglong2 q = in[j];
		insert(slots, mask, rmask, q.x, q.y);
	}
}

// ---- owned: every 2048-slot range of the table is one workgroup's, in LDS ----
constexpr uint32_t kRangeLg = 11, kRange = 1u << kRangeLg;
struct LSlot {
	unsigned long long tag, hi, nfirst;
	unsigned int cnt, pad;
};

// pass B: the entries of one pass-A bucket tile [b, e) into their ranges (bucket's 256 sub-ranges)
__global__ __launch_bounds__(256) void k_scatter_b(const ulonglong2* in, const unsigned long long* tiles, uint32_t mask,
		unsigned long long* rcur, ulonglong2* out) {
	__shared__ unsigned int h[256];
	__shared__ unsigned long long base[256];
	const unsigned long long t = tiles[blockIdx.x], b = t >> 24, e = b + (t & 0xffffffu);
	h[threadIdx.x] = 0;
	__syncthreads();
	ulonglong2 q[16];
	uint32_t rg[16], rk[16];
	uint32_t top;
#pragma unroll
	for (int j = 0; j < 16; j++) {
		const unsigned long long i = b + j * 256 + threadIdx.x;
		q[j] = i < e ? in[i] : make_ulonglong2(0, 0);
		const uint32_t r = ((uint32_t)(q[j].x >> 11) & mask) >> kRangeLg;
		rg[j] = r & 255u;
		rk[j] = i < e ? atomicAdd(&h[rg[j]], 1u) : 0;
	}
	__syncthreads();
	top = (((uint32_t)(in[b].x >> 11) & mask) >> kRangeLg) >> 8; // every entry of the tile is in b's bucket
	if (h[threadIdx.x])
		base[threadIdx.x] = atomicAdd(&rcur[((unsigned long long)top << 8) | threadIdx.x], (unsigned long long)h[threadIdx.x]);
	__syncthreads();
#pragma unroll
	for (int j = 0; j < 16; j++) {
		const unsigned long long i = b + j * 256 + threadIdx.x;
		if (i < e)
			out[base[rg[j]] + rk[j]] = q[j];
	}
}

// one workgroup per range: its slots into LDS, its requests against them with LDS atomics, back out
__global__ __launch_bounds__(256) void k_own(Slot* slots, uint32_t mask, const ulonglong2* in, const unsigned long long* roff) {
	__shared__ LSlot ls[kRange];
	const uint32_t r = blockIdx.x;
	Slot* g = slots + ((size_t)r << kRangeLg);
	for (uint32_t k = threadIdx.x; k < kRange; k += 256) {
		const ulonglong2 th = *(const ulonglong2*)&g[k].tag;
		ls[k].tag = th.x;
		ls[k].hi = th.y;
		ls[k].nfirst = g[k].nfirst;
		ls[k].cnt = g[k].internal_clients;
	}
	__syncthreads();
	const unsigned long long b = roff[r], e = roff[r + 1];
	for (unsigned long long j = b + threadIdx.x; j < e; j += 256) {
		const ulonglong2 q = in[j];
		const unsigned long long key = q.x, first = q.y;
		uint32_t idx = (uint32_t)(key >> 11) & (kRange - 1);
		for (uint32_t p = 0; p < kRange; p++) {
			unsigned long long t = ls[idx].tag;
			if (t == 0) {
				t = atomicCAS(&ls[idx].tag, 0ull, key);
				if (t == 0) {
					ls[idx].hi = key ^ 0x5555ull;
					t = key;
				}
			}
			if (t == key) {
				atomicAdd(&ls[idx].cnt, 1u);
				atomicMax(&ls[idx].nfirst, ~first);
				break;
			}
			idx = (idx + 1) & (kRange - 1);
		}
	}
	__syncthreads();
	for (uint32_t k = threadIdx.x; k < kRange; k += 256) {
		if (!ls[k].tag)
			continue;
		*(ulonglong2*)&g[k].tag = make_ulonglong2(ls[k].tag, ls[k].hi);
		g[k].nfirst = ls[k].nfirst;
		g[k].internal_clients = ls[k].cnt;
	}
}

int main(int argc, char** argv) {
	const uint32_t lg = 26, slots_n = 1u << lg, mask = slots_n - 1;
	const unsigned long long n = 100000000ull, D = 30000000ull;
	int cus = 256;
	Slot* slots;
	CK(hipMalloc(&slots, (size_t)slots_n * sizeof(Slot)));
	ulonglong2* lists;
	CK(hipMalloc(&lists, n * sizeof(ulonglong2)));
	unsigned long long* cnt;
	CK(hipMalloc(&cnt, 2 * 256 * sizeof(unsigned long long)));
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	auto t = [&](auto fn) {
		CK(hipEventRecord(a));
		fn();
		CK(hipEventRecord(b));
		CK(hipEventSynchronize(b));
		float ms;
		CK(hipEventElapsedTime(&ms, a, b));
		return ms;
	};
	for (int rep = 0; rep < 2; rep++) {
		CK(hipMemset(slots, 0, (size_t)slots_n * sizeof(Slot)));
		const float md = t([&] { k_direct<<<cus * 8, 256>>>(slots, mask, n, D); });
		std::printf("{\"mode\": \"direct\", \"ms\": %.3f}\n", md);
	}
	std::vector<int> Rs;
	for (int k = 1; k < argc; k++)
		Rs.push_back(std::atoi(argv[k]));
	if (Rs.empty())
		Rs = {8, 16, 32, 64};
	for (int R : Rs) {
		uint32_t rl = 0;
		while ((1 << rl) < R)
			rl++;
		const uint32_t rshift = lg - rl, rmask = (1u << rshift) - 1;
		for (int rep = 0; rep < 2; rep++) {
			CK(hipMemset(slots, 0, (size_t)slots_n * sizeof(Slot)));
			CK(hipMemset(cnt, 0, 2 * 256 * sizeof(unsigned long long)));
			const float mc = t([&] { k_count<<<cus * 4, 256>>>(mask, rshift, n, D, cnt); });
			std::vector<unsigned long long> h(256), off(257, 0);
			CK(hipMemcpy(h.data(), cnt, 256 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
			for (int r = 0; r < 256; r++)
				off[r + 1] = off[r] + h[r];
			CK(hipMemcpy(cnt + 256, off.data(), 256 * sizeof(unsigned long long), hipMemcpyHostToDevice));
			const float ms = t([&] { k_scatter<<<cus * 4, 256>>>(mask, rshift, n, D, cnt + 256, lists); });
			const float mr = t([&] {
				for (int r = 0; r < R; r++)
					k_region<<<cus * 8, 256>>>(slots, mask, rmask, lists, off[r], off[r + 1]);
			});
			std::printf("{\"mode\": \"regions\", \"R\": %d, \"region_mb\": %.1f, \"count_ms\": %.3f, \"scatter_ms\": %.3f, \"regions_ms\": %.3f}\n", R,
					(double)slots_n / R * 64 / 1e6, mc, ms, mr);
		}
	}
	// owned mode: pass A (128 buckets by the range's top 7 bits), pass B (256 ranges per bucket),
	// one workgroup per 2048-slot range
	{
		ulonglong2* lists2;
		CK(hipMalloc(&lists2, n * sizeof(ulonglong2)));
		const uint32_t nr = slots_n >> kRangeLg; // 32768 ranges
		unsigned long long *rcnt, *rcur, *roff_d, *tiles_d;
		CK(hipMalloc(&rcnt, nr * sizeof(unsigned long long)));
		CK(hipMalloc(&rcur, nr * sizeof(unsigned long long)));
		CK(hipMalloc(&roff_d, (nr + 1) * sizeof(unsigned long long)));
		CK(hipMalloc(&tiles_d, (n / 4096 + 256) * sizeof(unsigned long long)));
		const uint32_t rshiftA = lg - 7; // bucket = top 7 bits of the slot index
		for (int rep = 0; rep < 2; rep++) {
			CK(hipMemset(slots, 0, (size_t)slots_n * sizeof(Slot)));
			CK(hipMemset(cnt, 0, 2 * 256 * sizeof(unsigned long long)));
			const float mc = t([&] { k_count<<<cus * 4, 256>>>(mask, rshiftA, n, D, cnt); });
			std::vector<unsigned long long> h(256), off(257, 0);
			CK(hipMemcpy(h.data(), cnt, 256 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
			for (int r = 0; r < 256; r++)
				off[r + 1] = off[r] + h[r];
			CK(hipMemcpy(cnt + 256, off.data(), 256 * sizeof(unsigned long long), hipMemcpyHostToDevice));
			const float ma = t([&] { k_scatter<<<cus * 4, 256>>>(mask, rshiftA, n, D, cnt + 256, lists); });
			// range counts (a host pass in this benchmark: the real kernel counts per tile on the device)
			std::vector<ulonglong2> hl(n);
			CK(hipMemcpy(hl.data(), lists, n * sizeof(ulonglong2), hipMemcpyDeviceToHost));
			std::vector<unsigned long long> rc(nr, 0), ro(nr + 1, 0), tl;
			for (unsigned long long i = 0; i < n; i++)
				rc[((uint32_t)(hl[i].x >> 11) & mask) >> kRangeLg]++;
			for (uint32_t r = 0; r < nr; r++)
				ro[r + 1] = ro[r] + rc[r];
			for (int bk = 0; bk < 128; bk++)
				for (unsigned long long a = off[bk]; a < off[bk + 1]; a += 4096)
					tl.push_back((a << 24) | std::min<unsigned long long>(4096, off[bk + 1] - a));
			CK(hipMemcpy(rcur, ro.data(), nr * sizeof(unsigned long long), hipMemcpyHostToDevice));
			CK(hipMemcpy(roff_d, ro.data(), (nr + 1) * sizeof(unsigned long long), hipMemcpyHostToDevice));
			CK(hipMemcpy(tiles_d, tl.data(), tl.size() * sizeof(unsigned long long), hipMemcpyHostToDevice));
			const float mb = t([&] { k_scatter_b<<<(uint32_t)tl.size(), 256>>>(lists, tiles_d, mask, rcur, lists2); });
			const float mo = t([&] { k_own<<<nr, 256>>>(slots, mask, lists2, roff_d); });
			std::printf("{\"mode\": \"owned\", \"count_ms\": %.3f, \"pass_a_ms\": %.3f, \"pass_b_ms\": %.3f, \"own_ms\": %.3f}\n", mc, ma, mb,
					mo);
		}
	}
	return 0;
}
