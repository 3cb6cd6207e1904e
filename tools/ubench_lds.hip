// ubench_lds.hip — microbenchmark of the DFA byte step (table in LDS), no global memory
// in the timed loop.  Measures byte-steps per second chip-wide for:
//   layout 0: u8 table, index (s << 8) | b            (bank = byte bits 2..6)
//   layout 1: u8 table, index (s << 8) | (b ^ ((s & 31) << 2))   (bank depends on s too)
//   layout 2: u8 table, rows 260 B apart, index s * 260 + b' where b' moves the byte's
//             low 5 bits to bits 6..2 (bank = (s + b[4:0]) mod 32; same-state lanes never conflict)
// STATES: random states in [0, 128) or a realistic mix (most lanes in a few states).
// and ILP = 1, 2, 4 independent chains per lane.
//   hipcc --offload-arch=gfx950 -O3 -o ubench_lds tools/ubench_lds.hip && ./ubench_lds
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ uint32_t reorder_word(uint32_t w) {
	const uint32_t hi = __builtin_amdgcn_ubfe(w, 5, 27) & 0x03030303u; // b[6:5] -> bits 1..0
	return ((w << 2) & 0x7c7c7c7cu) | hi | (w & 0x80808080u);
}

template <int LAYOUT, int ILP>
__global__ __launch_bounds__(1024) void k_chain(const uint8_t* gtab, const uint32_t* text, uint32_t nwords, uint32_t iters,
		uint32_t* out) {
	__shared__ __attribute__((aligned(16))) uint8_t T[256 * 260];
	for (uint32_t k = threadIdx.x * 4; k < 256 * 260; k += blockDim.x * 4)
		*(uint32_t*)(T + k) = *(const uint32_t*)(gtab + k);
	__syncthreads();
	uint32_t s[ILP];
	for (int j = 0; j < ILP; j++)
		s[j] = (threadIdx.x * 7 + j * 13) & 127;
	const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
	uint32_t acc = 0;
	// 4 words of "text" per chain, loaded once; each iteration rotates their bytes
	uint32_t w[ILP][4];
	for (int j = 0; j < ILP; j++)
		for (int q = 0; q < 4; q++)
			w[j][q] = text[(gid * 4 * ILP + j * 4 + q) % nwords];
	for (uint32_t it = 0; it < iters; it++) {
		uint32_t wr[ILP][4];
		for (int j = 0; j < ILP; j++)
			for (int q = 0; q < 4; q++) {
				w[j][q] = (w[j][q] >> 8) | (w[j][q] << 24);
				wr[j][q] = LAYOUT == 2 ? reorder_word(w[j][q]) : w[j][q];
			}
#pragma unroll
		for (int k = 0; k < 16; k++) {
#pragma unroll
			for (int j = 0; j < ILP; j++) {
				const uint32_t wk = wr[j][k >> 2];
				uint32_t idx;
				if (LAYOUT == 2) {
					idx = s[j] * 260u + __builtin_amdgcn_ubfe(wk, 8 * (k & 3), 8);
				} else if (LAYOUT == 0) {
					idx = __builtin_amdgcn_perm(s[j], wk, 0x0c0c0400u | (uint32_t)(k & 3));
				} else {
					const uint32_t b = (wk >> (8 * (k & 3))) & 0xff;
					idx = (s[j] << 8) | (b ^ ((s[j] & 31) << 2));
				}
				s[j] = T[idx];
				acc = max(acc, s[j]);
			}
		}
	}
	out[gid] = acc + s[0];
}

template <int LAYOUT, int ILP>
static double run(const uint8_t* dtab, const uint32_t* dtext, uint32_t nwords, uint32_t* dout, int blocks, uint32_t iters,
		size_t pad, int threads = 1024) {
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	hipLaunchKernelGGL((k_chain<LAYOUT, ILP>), dim3(blocks), dim3(threads), pad, 0, dtab, dtext, nwords, iters, dout);
	(void)hipEventRecord(a);
	hipLaunchKernelGGL((k_chain<LAYOUT, ILP>), dim3(blocks), dim3(threads), pad, 0, dtab, dtext, nwords, iters, dout);
	(void)hipEventRecord(b);
	(void)hipEventSynchronize(b);
	float ms = 0;
	(void)hipEventElapsedTime(&ms, a, b);
	const double steps = (double)blocks * threads * ILP * iters * 16;
	return steps / (ms * 1e-3) / 1e9; // G byte-steps / s
}

int main() {
	hipDeviceProp_t prop;
	(void)hipGetDeviceProperties(&prop, 0);
	const int cus = prop.multiProcessorCount;
	// table: random next states in [0, 128)
	// "random": next state uniform in [0, 128).  "sticky": like parsing text, a state keeps
	// itself with probability 7/8 (most lanes sit in a few URL / header-value states).
	const int sticky = getenv("UB_STICKY") ? 1 : 0;
	std::vector<uint8_t> tab(256 * 260);
	uint32_t x = 12345;
	for (int st = 0; st < 256; st++)
		for (int b = 0; b < 260; b++) {
			x = x * 1664525u + 1013904223u;
			uint32_t nx = (x >> 24) & 127;
			if (sticky && ((x >> 8) & 7) != 0)
				nx = st & 127;
			tab[st * 260 + b] = (uint8_t)nx;
		}
	// text: lowercase-heavy bytes like URLs / hosts
	const char* alpha = "abcdefghijklmnopqrstuvwxyz0123456789/.-_=?&abcdeimnorst";
	const uint32_t nwords = 1 << 20;
	std::vector<uint32_t> text(nwords);
	for (auto& w : text) {
		uint32_t v = 0;
		for (int q = 0; q < 4; q++) {
			x = x * 1664525u + 1013904223u;
			v |= (uint32_t)(uint8_t)alpha[(x >> 16) % 55] << (8 * q);
		}
		w = v;
	}
	uint8_t* dtab;
	uint32_t *dtext, *dout;
	(void)hipMalloc(&dtab, 256 * 260);
	(void)hipMalloc(&dtext, nwords * 4);
	(void)hipMalloc(&dout, (size_t)cus * 8 * 1024 * 4);
	(void)hipMemcpy(dtab, tab.data(), 256 * 260, hipMemcpyHostToDevice);
	(void)hipMemcpy(dtext, text.data(), nwords * 4, hipMemcpyHostToDevice);
	const uint32_t iters = 64;
	for (int bpc = 1; bpc <= 2; bpc++) {
		const int blocks = cus * 8;
		const size_t pad = bpc == 1 ? 40 * 1024 : 0; // 104 KB per block -> one block per CU
		printf("sticky=%d blocks/CU=%d  L0/ILP1 %.0f  L0/ILP2 %.0f  L1/ILP1 %.0f  L1/ILP2 %.0f  L2/ILP1 %.0f  L2/ILP2 %.0f  L2/ILP4 %.0f  (G steps/s)\n",
				sticky, bpc, run<0, 1>(dtab, dtext, nwords, dout, blocks, iters, pad), run<0, 2>(dtab, dtext, nwords, dout, blocks, iters, pad),
				run<1, 1>(dtab, dtext, nwords, dout, blocks, iters, pad), run<1, 2>(dtab, dtext, nwords, dout, blocks, iters, pad),
				run<2, 1>(dtab, dtext, nwords, dout, blocks, iters, pad), run<2, 2>(dtab, dtext, nwords, dout, blocks, iters, pad),
				run<2, 4>(dtab, dtext, nwords, dout, blocks, iters, pad));
	}
	// chains per CU: scan lanes of k_fresh (640 = 10 waves) at ILP 1 and 2, one block per CU
	for (int th : {384, 640, 1024}) {
		const size_t pad = 40 * 1024;
		printf("threads=%d  L2/ILP1 %.0f  L2/ILP2 %.0f  L2/ILP4 %.0f (G steps/s)\n", th, run<2, 1>(dtab, dtext, nwords, dout, cus * 8, iters, pad, th),
				run<2, 2>(dtab, dtext, nwords, dout, cus * 8, iters, pad, th), run<2, 4>(dtab, dtext, nwords, dout, cus * 8, iters, pad, th));
	}
	return 0;
}
