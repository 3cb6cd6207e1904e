// ebd_measure.hip — the measured HBM read-stream peak that bench.py reports the roofline
// against, beside the 8 TB/s spec ("report against 8.0 TB/s, and also against a
// measured stream-read peak").  Two read-only streams over one device buffer, each the best of
// its shape in tools/ubench_stream.hip:
//   plain  every lane global_load_dwordx4 of consecutive 16 B (1 KiB per wave instruction),
//          8 loads in flight per lane, folded into one word per lane
//   dma    per CU, 2 loader waves copy consecutive 16-KiB tiles into an LDS ring by
//          global_load_lds_dwordx4 (1 KiB per wave instruction), 2 tiles in flight each, and
//          the other waves read each tile once (ds_read_b128) and release it
// Both read every byte once and write one word per thread.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdint>

#include "../../include/ebpf_discovery_amd.h"

namespace {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4u ld16(const uint8_t* a) { return *(const __attribute__((address_space(1))) v4u*)a; }
__device__ __forceinline__ uint32_t fold(v4u v) { return v.x ^ v.y ^ v.z ^ v.w; }

constexpr int kThreads = 1024;

// the block's contiguous share of [0, bytes), 16-byte granular
__device__ __forceinline__ void block_span(uint64_t bytes, uint64_t& lo, uint64_t& hi) {
	const uint64_t units = bytes / 16, per = (units + gridDim.x - 1) / gridDim.x;
	lo = min(units, (uint64_t)blockIdx.x * per) * 16;
	hi = min(units, ((uint64_t)blockIdx.x + 1) * per) * 16;
}

__global__ __launch_bounds__(kThreads) void k_read_plain(const uint8_t* buf, uint64_t bytes, uint32_t* out) {
	uint64_t lo, hi;
	block_span(bytes, lo, hi);
	uint32_t acc = 0;
	constexpr uint64_t kStep = kThreads * 16ull;
	for (uint64_t b = lo + threadIdx.x * 16ull; b < hi; b += 8 * kStep) {
		v4u v[8];
#pragma unroll
		for (int k = 0; k < 8; k++)
			v[k] = ld16(buf + min(b + k * kStep, hi - 16));
#pragma unroll
		for (int k = 0; k < 8; k++)
			acc ^= fold(v[k]);
	}
	out[blockIdx.x * kThreads + threadIdx.x] = acc;
}

constexpr uint32_t kTile = 16384, kRing = 8, kLoaders = 2, kDepth = 2;
constexpr uint32_t kSpinMax = 1u << 24; // every wait is bounded: a broken hand-off ends the kernel
__device__ __forceinline__ uint32_t lds_acq(const uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void lds_rel(uint32_t* p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ uint32_t slot_word(uint32_t t, uint32_t ready) { return ((t + kRing) << 1) | ready; }

__global__ __launch_bounds__(kThreads) void k_read_dma(const uint8_t* buf, uint64_t bytes, uint32_t* out, uint32_t* err) {
	__shared__ __attribute__((aligned(16))) uint8_t ring[kRing][kTile];
	__shared__ uint32_t st[kRing], take;
	const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
	if (threadIdx.x < kRing)
		st[threadIdx.x] = slot_word(threadIdx.x - kRing, 0); // "tile slot - kRing was released"
	if (threadIdx.x == 0)
		take = 0;
	__syncthreads();
	uint64_t lo, hi;
	block_span(bytes, lo, hi);
	const uint32_t ntiles = (uint32_t)((hi - lo + kTile - 1) / kTile);
	uint32_t acc = 0;
	if (wave < kLoaders) {
		uint32_t issued = 0, marked = 0, tl[kDepth];
		for (uint32_t t = wave; t < ntiles; t += kLoaders) {
			const uint32_t s = t % kRing;
			for (uint32_t spins = 0; lds_acq(&st[s]) != slot_word(t - kRing, 0);) {
				if (++spins > kSpinMax) {
					atomicOr(err, 1u);
					goto done;
				}
				__builtin_amdgcn_s_sleep(1);
			}
			const uint64_t base = lo + (uint64_t)t * kTile;
#pragma unroll
			for (uint32_t k = 0; k < kTile / 1024; k++)
				__builtin_amdgcn_global_load_lds((const void*)(buf + min(base + k * 1024u + lane * 16u, hi - 16)),
						(__attribute__((address_space(3))) void*)(&ring[s][k * 1024u]), 16, 0, 0);
			tl[issued % kDepth] = t;
			issued++;
			if (issued - marked == kDepth) { // the oldest tile in flight has landed
				asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kDepth - 1) * (kTile / 1024)) : "memory");
				const uint32_t tt = tl[marked % kDepth];
				lds_rel(&st[tt % kRing], slot_word(tt, 1));
				marked++;
			}
		}
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		for (; marked < issued; marked++) {
			const uint32_t tt = tl[marked % kDepth];
			lds_rel(&st[tt % kRing], slot_word(tt, 1));
		}
	} else {
		for (;;) {
			uint32_t t = 0;
			if (lane == 0)
				t = atomicAdd(&take, 1u);
			t = __builtin_amdgcn_readfirstlane(t);
			if (t >= ntiles)
				break;
			const uint32_t s = t % kRing;
			for (uint32_t spins = 0; lds_acq(&st[s]) != slot_word(t, 1);) {
				if (++spins > kSpinMax) {
					atomicOr(err, 2u);
					goto done;
				}
				__builtin_amdgcn_s_sleep(1);
			}
#pragma unroll
			for (uint32_t k = 0; k < kTile / 1024; k++)
				acc ^= fold(*(const v4u*)&ring[s][k * 1024u + lane * 16u]);
			lds_rel(&st[s], slot_word(t, 0));
		}
	}
done:
	out[blockIdx.x * kThreads + threadIdx.x] = acc;
}

} // namespace

#define MTRY(x)                            \
	do {                                   \
		if ((x) != hipSuccess) {           \
			rc = -EIO;                     \
			goto out;                      \
		}                                  \
	} while (0)

int ebd_measure_read_bandwidth(int device, uint64_t bytes, uint32_t reps, double* plain_gbps, double* dma_gbps) {
	if (bytes < (1u << 24) || reps == 0 || !plain_gbps || !dma_gbps)
		return -EINVAL;
	bytes &= ~(uint64_t)(kTile - 1);
	int rc = 0, cus = 0;
	uint8_t* buf = nullptr;
	uint32_t *out = nullptr, *err = nullptr;
	hipEvent_t e0 = nullptr, e1 = nullptr;
	hipStream_t s = nullptr;
	float ms[2] = {0, 0};
	uint32_t h_err = 0;
	MTRY(hipSetDevice(device));
	MTRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
	MTRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
	MTRY(hipMalloc(&buf, bytes));
	MTRY(hipMalloc(&out, (size_t)cus * kThreads * sizeof(uint32_t)));
	MTRY(hipMalloc(&err, sizeof(uint32_t)));
	MTRY(hipMemsetAsync(buf, 0x41, bytes, s));
	MTRY(hipMemsetAsync(err, 0, sizeof(uint32_t), s));
	MTRY(hipEventCreate(&e0));
	MTRY(hipEventCreate(&e1));
	for (int shape = 0; shape < 2; shape++) {
		for (uint32_t r = 0; r <= reps; r++) { // the first run warms up and is not timed
			if (r == 1)
				MTRY(hipEventRecord(e0, s));
			if (shape == 0)
				hipLaunchKernelGGL(k_read_plain, dim3(cus), dim3(kThreads), 0, s, buf, bytes, out);
			else
				hipLaunchKernelGGL(k_read_dma, dim3(cus), dim3(kThreads), 0, s, buf, bytes, out, err);
			MTRY(hipGetLastError());
		}
		MTRY(hipEventRecord(e1, s));
		MTRY(hipEventSynchronize(e1));
		MTRY(hipEventElapsedTime(&ms[shape], e0, e1));
	}
	MTRY(hipMemcpy(&h_err, err, sizeof(uint32_t), hipMemcpyDeviceToHost));
	if (h_err)
		rc = -EIO; // a hand-off wait ran out: the dma number is not a measurement
	*plain_gbps = (double)bytes * reps / (ms[0] / 1e3) / 1e9;
	*dma_gbps = (double)bytes * reps / (ms[1] / 1e3) / 1e9;
out:
	if (e0)
		(void)hipEventDestroy(e0);
	if (e1)
		(void)hipEventDestroy(e1);
	(void)hipFree(buf);
	(void)hipFree(out);
	(void)hipFree(err);
	if (s)
		(void)hipStreamDestroy(s);
	return rc;
}
