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
	return 0;
}
