// ubench_mem.hip — read bandwidth of the access patterns a lane-per-event scan can use.
// N events of E bytes (16-B aligned, back to back) in one HBM buffer; each kernel XORs every
// byte it reads into a sink.  Reported: useful GB/s (N * E bytes / time).
//   stream   coalesced: lane t reads 16 B at 16 t (+ grid stride)                 (reference)
//   lane16   lane per event, 16-B loads, 8 per 128-B window, next window in flight
//   quad64   4 lanes per 4 events: each load instruction of the quad reads 64 contiguous
//            bytes of one event (4 x 16 B), then a 4x4 transpose inside the quad (DPP)
//            hands every lane the 64 B of its own event
//   hipcc --offload-arch=gfx950 -O3 -o ubench_mem tools/ubench_mem.hip && ./ubench_mem
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4u ld16(const uint8_t* p) { return *(const __attribute__((address_space(1))) v4u*)p; }

__global__ __launch_bounds__(1024) void k_stream(const uint8_t* buf, size_t bytes, uint32_t* out) {
	v4u acc = {0, 0, 0, 0};
	const size_t stride = (size_t)gridDim.x * blockDim.x * 16;
	for (size_t o = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; o < bytes; o += stride)
		acc ^= ld16(buf + o);
	out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// lane per event: windows of 8 chunks at the event's own 16-B alignment
__global__ __launch_bounds__(1024) void k_lane16(const uint8_t* buf, uint32_t n, uint32_t E, uint32_t* out) {
	v4u acc = {0, 0, 0, 0};
	const uint32_t nch = E / 16;
	for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
		const uint8_t* p = buf + (size_t)e * E;
		for (uint32_t c = 0; c < nch; c += 8) {
			v4u w[8];
#pragma unroll
			for (int k = 0; k < 8; k++)
				w[k] = ld16(p + 16 * min(c + k, nch - 1));
#pragma unroll
			for (int k = 0; k < 8; k++)
				acc ^= w[k];
		}
	}
	out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// quad-cooperative: lane r of quad q loads chunk (c + r) of each of the quad's 4 events, so
// each load instruction reads 16 segments of 64 contiguous bytes.  (A scan would then
// transpose 4x4 inside the quad; that is VALU / permute work, not measured here.)
__global__ __launch_bounds__(1024) void k_quad64(const uint8_t* buf, uint32_t n, uint32_t E, uint32_t* out) {
	v4u acc = {0, 0, 0, 0};
	const uint32_t nch = E / 16;
	const uint32_t r = threadIdx.x & 3;
	const uint32_t quads = (n + 3) / 4;
	for (uint32_t qd = (blockIdx.x * blockDim.x + threadIdx.x) >> 2; qd < quads; qd += (gridDim.x * blockDim.x) >> 2) {
		const uint32_t e0 = qd * 4;
		for (uint32_t c = 0; c < nch; c += 8) {
			v4u g[8];
#pragma unroll
			for (int k = 0; k < 8; k++) { // events e0 + (k & 3), chunks c + r and c + 4 + r
				const uint32_t e = min(e0 + (k & 3), n - 1);
				g[k] = ld16(buf + (size_t)e * E + 16 * min(c + 4 * (k >> 2) + r, nch - 1));
			}
#pragma unroll
			for (int k = 0; k < 8; k++)
				acc ^= g[k];
		}
	}
	out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

int main(int argc, char** argv) {
	hipDeviceProp_t prop;
	(void)hipGetDeviceProperties(&prop, 0);
	const int cus = prop.multiProcessorCount;
	const uint32_t E = argc > 1 ? (uint32_t)atoi(argv[1]) : 256; // multiple of 16
	const uint32_t n = (uint32_t)((5ull << 30) / E); // ~5.4 GB of events
	const size_t bytes = (size_t)n * E;
	uint8_t* buf;
	uint32_t* out;
	if (hipMalloc(&buf, bytes + 4096) != hipSuccess || hipMalloc(&out, (size_t)cus * 16 * 1024 * 4) != hipSuccess)
		return 1;
	(void)hipMemset(buf, 0x5a, bytes + 4096);
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
		printf("E=%u %-8s %8.3f ms  %7.0f GB/s useful\n", E, name, ms, bytes / (ms * 1e-3) / 1e9);
	};
	time("stream", [&] { hipLaunchKernelGGL(k_stream, dim3(cus * 8), dim3(1024), 0, 0, buf, bytes, out); });
	time("lane16", [&] { hipLaunchKernelGGL(k_lane16, dim3(cus * 8), dim3(1024), 0, 0, buf, n, E, out); });
	time("lane16x1", [&] { hipLaunchKernelGGL(k_lane16, dim3(cus), dim3(1024), 0, 0, buf, n, E, out); });
	time("quad64", [&] { hipLaunchKernelGGL(k_quad64, dim3(cus * 8), dim3(1024), 0, 0, buf, n, E, out); });
	return 0;
}
