// swar_probe.hip — experiment (not part of libebd_amd.so): the byte-parallel fast-path scan
// of DESIGN.md section 9, next step 1, measured beside k_fresh by tools/perf_swar.py.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -I ebpf-discovery_amd/csrc -I include \
//         tools/swar_probe.hip -o tools/libswar_probe.so
//
// One lane per event.  For every 16-byte chunk of its buffer a lane computes, with SWAR
// arithmetic and no table, masks of SP, CR, LF, ':' and of the bytes outside 0x20-0x7e (the
// C-locale VALUE class of HttpRequestParser.cpp:47-65 is exactly 0x20-0x7e), then steps a
// small state machine from delimiter to delimiter: the request line (P:162-262), each header
// key up to ':' (P:264-297), the spaces and the value up to CR (P:299-352), LF, the empty line
// (P:354-364).  The byte classes beyond printable (URL, key, Host and client-IP values) come
// from a 256-byte table read per byte of the chunk, only when some lane of the wave is inside
// such a span.  What the machine does not take (an invalid byte, a space inside a key, a
// header line without ':', a duplicate Host, a request past 8,193 bytes, a buffer that ends
// first) is marked for the DFA path, which stays the spec: tools/perf_swar.py compares every
// event the machine took with k_fresh's result.
#include <hip/hip_runtime.h>

#include "ebd_device.h"
#include "ebd_spec.h"

namespace ebd {

namespace {
constexpr int kSwarThreads = 256;

// 0x80 in each byte of w equal to the byte of b4 (exact per byte: no borrow crosses bytes)
__device__ __forceinline__ uint32_t swar_eq(uint32_t w, uint32_t b4) {
	const uint32_t t = w ^ b4;
	return ~(((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t) & 0x80808080u;
}
// 0x80 in each byte of w outside [0x20, 0x7e]
__device__ __forceinline__ uint32_t swar_np(uint32_t w) {
	const uint32_t lo = w & 0x7f7f7f7fu;
	return (((lo + 0x01010101u) | w) | ~((lo + 0x60606060u) | w)) & 0x80808080u;
}
// bits 7, 15, 23, 31 -> bits 0..3
__device__ __forceinline__ uint32_t swar_pack(uint32_t m) { return (((m >> 7) * 0x00204081u) >> 21) & 0xfu; }

typedef unsigned int v4u_sw __attribute__((ext_vector_type(4)));
typedef v4u_sw v4u_sw_a1 __attribute__((aligned(1)));
__device__ __forceinline__ uint4 gload_u4(const uint8_t* a) { // global_load_dwordx4, any alignment
	const v4u_sw v = *(const __attribute__((address_space(1))) v4u_sw_a1*)a;
	return uint4{v.x, v.y, v.z, v.w};
}

__device__ __forceinline__ uint32_t chunk_byte(const uint4& c, uint32_t k) {
	const uint32_t lo = (k & 4u) ? c.y : c.x, hi = (k & 4u) ? c.w : c.z;
	return (((k & 8u) ? hi : lo) >> (8u * (k & 3u))) & 0xffu;
}

enum : uint32_t { PH_URL, PH_PROTO, PH_KEY, PH_SPV, PH_VAL, PH_LF, PH_END, PH_DONE, PH_FALLBACK };
enum : uint32_t { KY_OTHER, KY_HOST, KY_CIP };

} // namespace

// Per event: status (1 FINISHED, 0 for the DFA path), consumed, the spans and info bits the
// fast path's result holds (cip_off: the raw first client-IP value byte, as k_fresh's).
struct SwarOut {
	uint16_t consumed;
	uint8_t status, info;
	uint16_t url_off, url_len, host_off, host_len, cip_off, pad;
};

__global__ __launch_bounds__(kSwarThreads) void k_swar_scan(const EventRec* ev, const uint32_t* lens, const uint64_t* offs,
		const uint8_t* payload, unsigned long long payload_bytes, uint32_t n, const uint8_t* cls_g, SwarOut* out) {
	__shared__ uint8_t cls[256];
	__shared__ uint32_t s_next;
	const uint32_t per = (n + gridDim.x - 1) / gridDim.x, rb = min(n, blockIdx.x * per), re = min(n, rb + per);
	for (uint32_t k = threadIdx.x; k < 256; k += kSwarThreads)
		cls[k] = cls_g[k];
	if (threadIdx.x == 0)
		s_next = rb + kSwarThreads;
	__syncthreads();
	uint32_t i = rb + threadIdx.x;
	// the lane's event
	uint32_t L = 0, ph = PH_DONE, pos = 0, c = 0, nch = 0;
	const uint8_t* p = payload;
	uint32_t flags = 0, url_start = 0, url_end = 0, host_start = 0, host_end = 0, host_seen = 0, cip_start = 0, cipkey = 0, cip_seen = 0,
			 pidx = 0, ks = 0, klen = 0, ktype = 0, kid = 0;
	unsigned long long k0 = 0, k1 = 0, k2 = 0;
	uint4 cur = uint4{0, 0, 0, 0};
	auto finish = [&](uint32_t status, uint32_t consumed) {
		SwarOut o;
		o.status = (uint8_t)status;
		o.consumed = (uint16_t)consumed;
		o.info = (uint8_t)((url_start == 5 ? EBD_INFO_POST : 0) | ((flags & 16) ? EBD_INFO_HTTPS : 0) | (cip_seen ? EBD_INFO_CIP : 0));
		o.url_off = (uint16_t)url_start;
		o.url_len = (uint16_t)(url_end - url_start);
		o.host_off = (uint16_t)(host_seen ? host_start : 0);
		o.host_len = (uint16_t)(host_seen ? host_end - host_start : 0);
		o.cip_off = (uint16_t)(cip_seen ? cip_start : 0);
		o.pad = 0;
		out[i] = o;
	};
	auto start = [&]() { // the next event of the workgroup's range into the lane
		for (;;) {
			if (i >= re) {
				ph = PH_DONE;
				return;
			}
			const uint32_t fl = ev[i].flags, Li = lens[i];
			const unsigned long long o = offs[i];
			if ((fl & FLAG_NEW) && Li != EBD_NO_BUFFER && Li >= 6 && o + Li <= payload_bytes) {
				flags = fl;
				L = Li;
				p = payload + o;
				c = 0;
				nch = (L + 15u) >> 4;
				cur = gload_u4(p); // unaligned dwordx4
				// the method and the URL's '/': "GET /" or "POST /" (P:162-199)
				const uint32_t w0 = cur.x, b4 = cur.y & 0xffu, b5 = (cur.y >> 8) & 0xffu;
				const bool get = w0 == 0x20544547u && b4 == '/'; // "GET " '/'
				const bool post = w0 == 0x54534f50u && b4 == ' ' && b5 == '/';
				url_start = post ? 5u : 4u;
				url_end = url_start;
				host_seen = cip_seen = cipkey = 0;
				host_start = host_end = cip_start = 0;
				ph = (get || post) ? PH_URL : PH_FALLBACK;
				pos = url_start + 1u;
				pidx = 0;
				if (ph == PH_FALLBACK) {
					finish(0, 0);
					i = atomicAdd(&s_next, 1u);
					continue;
				}
				return;
			}
			finish(0, 0); // not a fresh parse of a buffer this scan takes
			i = atomicAdd(&s_next, 1u);
		}
	};
	start();
	while (__any(ph != PH_DONE)) {
		if (ph != PH_DONE) {
			// masks of the chunk [16c, 16c + 16), bytes past the buffer masked out
			const uint32_t cb = 16u * c;
			const uint32_t valid = cb + 16u <= L ? 0xffffu : ((1u << (L - cb)) - 1u);
			uint32_t msp = 0, mcr = 0, mlf = 0, mcol = 0, mnp = 0;
			const uint32_t wd[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
			for (int q = 0; q < 4; q++) {
				msp |= swar_pack(swar_eq(wd[q], 0x20202020u)) << (4 * q);
				mcr |= swar_pack(swar_eq(wd[q], 0x0d0d0d0du)) << (4 * q);
				mlf |= swar_pack(swar_eq(wd[q], 0x0a0a0a0au)) << (4 * q);
				mcol |= swar_pack(swar_eq(wd[q], 0x3a3a3a3au)) << (4 * q);
				mnp |= swar_pack(swar_np(wd[q])) << (4 * q);
			}
			// the table classes of the chunk, read the first time a span of the chunk needs them
			uint32_t murl = 0, mkey = 0, mhost = 0, mcip = 0;
			bool have_cls = false;
			auto classes = [&]() {
				if (have_cls)
					return;
				have_cls = true;
#pragma unroll
				for (uint32_t k = 0; k < 16; k++) {
					const uint32_t cl = cls[chunk_byte(cur, k)];
					murl |= ((cl & C_URL) ? 1u : 0u) << k;
					mkey |= ((cl & C_KEY) ? 1u : 0u) << k;
					mhost |= ((cl & C_HOST) ? 1u : 0u) << k;
					mcip |= ((cl & C_CIP) ? 1u : 0u) << k;
				}
			};
			const uint32_t cend = min(cb + 16u, L);
			while (pos < cend && ph < PH_DONE) {
				const uint32_t rel = pos - cb, above = valid & (0xffffu << rel);
				if (pos > kMaxRequestLength) { // P:88-91: the DFA path handles the cap
					ph = PH_FALLBACK;
					break;
				}
				if (ph == PH_URL) { // P:201-213
					classes();
					const uint32_t stop = (msp | ~murl) & above;
					if (!stop) {
						pos = cend;
						break;
					}
					const uint32_t q = (uint32_t)__builtin_ctz(stop);
					if (!((msp >> q) & 1u)) {
						ph = PH_FALLBACK;
						break;
					}
					url_end = cb + q;
					pos = cb + q + 1u;
					ph = PH_PROTO;
					pidx = 0;
				} else if (ph == PH_PROTO) { // "HTTP/1.0" or "HTTP/1.1", CR, LF (P:215-262)
					const uint32_t b = chunk_byte(cur, rel);
					bool ok;
					if (pidx < 7)
						ok = b == (uint32_t)"HTTP/1."[pidx];
					else if (pidx == 7)
						ok = b == '0' || b == '1';
					else if (pidx == 8)
						ok = b == '\r';
					else
						ok = b == '\n';
					if (!ok) {
						ph = PH_FALLBACK;
						break;
					}
					pos++;
					if (++pidx == 10) {
						ph = PH_KEY;
						ks = pos;
						klen = 0;
						k0 = k1 = k2 = 0;
					}
				} else if (ph == PH_KEY) { // P:264-297 (no space inside the key on this path)
					classes();
					const uint32_t stop = (mcol | mcr | ~mkey) & above;
					const uint32_t q = stop ? (uint32_t)__builtin_ctz(stop) : 16u;
					const uint32_t e = cb + q < cend ? cb + q : cend;
					for (uint32_t a = pos; a < e; a++, klen++) { // the first 21 bytes, lower-cased
						if (klen < kMaxHeaderKeyLength) {
							const unsigned long long b = to_lower(chunk_byte(cur, a - cb));
							const uint32_t sh = 8u * (klen & 7u);
							if (klen < 8)
								k0 |= b << sh;
							else if (klen < 16)
								k1 |= b << sh;
							else
								k2 |= b << sh;
						}
					}
					if (!stop) {
						pos = cend;
						break;
					}
					const uint32_t at = cb + q;
					if ((mcr >> q) & 1u) {
						if (at != ks) { // a line without ':' (P:266-268): the DFA path
							ph = PH_FALLBACK;
							break;
						}
						ph = PH_END;
						pos = at + 1u;
						continue;
					}
					if (!((mcol >> q) & 1u)) {
						ph = PH_FALLBACK;
						break;
					}
					// the key's type (P:366-372): "host" and the client-IP keys, the 21-byte key kept whole
					ktype = KY_OTHER;
					kid = 0;
					if (klen == 4 && k0 == 0x74736f68ull) // host
						ktype = KY_HOST;
					else if (klen >= 21 && k0 == 0x725f79786f727072ull && k1 == 0x64615f65746f6d65ull && k2 == 0x7373657264ull)
						ktype = KY_CIP, kid = 1; // rproxy_remote_address (a longer key truncated to it: P:283-285)
					else if (klen == 14 && k0 == 0x696c632d65757274ull && k1 == 0x70692d746e65ull)
						ktype = KY_CIP, kid = 2; // true-client-ip
					else if (klen == 11 && k0 == 0x746e65696c632d78ull && k1 == 0x70692dull)
						ktype = KY_CIP, kid = 3; // x-client-ip
					else if (klen == 15 && k0 == 0x726177726f662d78ull && k1 == 0x726f662d646564ull)
						ktype = KY_CIP, kid = 4; // x-forwarded-for
					else if (klen == 16 && k0 == 0x632d707474682d78ull && k1 == 0x70692d746e65696cull)
						ktype = KY_CIP, kid = 5; // x-http-client-ip
					if (ktype == KY_HOST && host_seen) { // P:287-290: a second Host
						ph = PH_FALLBACK;
						break;
					}
					ph = PH_SPV;
					pos = at + 1u;
				} else if (ph == PH_SPV) { // P:299-319
					const uint32_t stop = ~msp & above;
					if (!stop) {
						pos = cend;
						break;
					}
					const uint32_t q = (uint32_t)__builtin_ctz(stop), at = cb + q;
					if ((mnp >> q) & 1u) { // not a VALUE byte (an empty value ends in CR): the DFA path
						ph = PH_FALLBACK;
						break;
					}
					if (ktype == KY_HOST) {
						host_start = at;
						host_seen = 1;
					} else if (ktype == KY_CIP) {
						if (!cipkey)
							cipkey = kid;
						if (kid == cipkey && !cip_seen) {
							cip_start = at;
							cip_seen = 1;
						}
					}
					ph = PH_VAL;
					pos = at + 1u;
				} else if (ph == PH_VAL) { // P:321-352
					if (ktype != KY_OTHER)
						classes();
					const uint32_t bad = ktype == KY_HOST ? ~mhost : ktype == KY_CIP ? ~mcip : 0u;
					const uint32_t stop = (mnp | bad) & above;
					if (!stop) {
						pos = cend;
						break;
					}
					const uint32_t q = (uint32_t)__builtin_ctz(stop), at = cb + q;
					if (!((mcr >> q) & 1u)) {
						ph = PH_FALLBACK;
						break;
					}
					if (ktype == KY_HOST)
						host_end = at;
					ph = PH_LF;
					pos = at + 1u;
				} else if (ph == PH_LF) { // P:248-262
					if (!((mlf >> rel) & 1u)) {
						ph = PH_FALLBACK;
						break;
					}
					pos++;
					ph = PH_KEY;
					ks = pos;
					klen = 0;
					k0 = k1 = k2 = 0;
				} else { // PH_END, P:354-364
					if (!((mlf >> rel) & 1u)) {
						ph = PH_FALLBACK;
						break;
					}
					finish(1, pos + 1u);
					ph = PH_DONE;
					break;
				}
			}
			// the next chunk, or the next event
			if (ph < PH_DONE && pos >= cend && cend == L) // the buffer ended first: unfinished
				ph = PH_FALLBACK;
			if (ph == PH_FALLBACK) {
				finish(0, 0);
				ph = PH_DONE;
			}
			if (ph == PH_DONE) {
				i = atomicAdd(&s_next, 1u);
				start();
			} else {
				c = pos >> 4;
				cur = gload_u4(p + 16u * c);
			}
		}
	}
}

} // namespace ebd

// out: n records of 16 bytes (SwarOut); *ms: the kernel's time (HIP events); blocks: workgroups
extern "C" int swar_scan(const void* ev, const uint32_t* lens, const uint64_t* offs, const uint8_t* payload,
		unsigned long long payload_bytes, uint32_t n, void* out, int blocks, float* ms) {
	static uint8_t* dcls = nullptr;
	if (!dcls) {
		uint8_t h[256];
		for (int c = 0; c < 256; c++)
			h[c] = ebd::byte_class((uint32_t)c);
		if (hipMalloc(&dcls, 256) != hipSuccess || hipMemcpy(dcls, h, 256, hipMemcpyHostToDevice) != hipSuccess)
			return -1;
	}
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	(void)hipEventRecord(a, 0);
	hipLaunchKernelGGL(ebd::k_swar_scan, dim3(blocks), dim3(ebd::kSwarThreads), 0, 0, (const ebd::EventRec*)ev, lens,
			(const uint64_t*)offs, payload, payload_bytes, n, (const uint8_t*)dcls, (ebd::SwarOut*)out);
	(void)hipEventRecord(b, 0);
	if (hipEventSynchronize(b) != hipSuccess)
		return -2;
	(void)hipEventElapsedTime(ms, a, b);
	(void)hipEventDestroy(a);
	(void)hipEventDestroy(b);
	return hipGetLastError() == hipSuccess ? 0 : -3;
}
