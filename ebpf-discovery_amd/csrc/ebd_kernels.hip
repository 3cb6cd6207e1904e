// ebd_kernels.hip — the MI355X kernels of the HTTP per-event parse path.
//
// Batch pipeline (one poll cycle of Discovery::fetchAndHandleEvents, Discovery.cpp:48-90):
//   k_carry_insert  sessions saved by earlier batches join this batch's session set
//   k_fresh         every NEW_DATA buffer through a fresh parser (DFA in LDS, one lane per
//                   event); finished requests get their client class and 128-bit key
//   k_slow_collect  events of sessions that need the sequential path (a fresh parse left
//                   the request unfinished, or the session was saved by an earlier batch)
//   k_walk          one lane per such session, events in order: the exact
//                   handleExistingSession / handleNewSession / handleCloseEvent logic
//                   (Discovery.cpp:112-198) over the generic parser
//   k_agg_fast      Aggregator::newRequest for the single-buffer requests
//   k_reps          first-arrival domain / scheme / endpoint string for new services
#include <hip/hip_runtime.h>

#include "ebd_device.h"
#include "ebd_fresh.h"

namespace ebd {

__device__ __forceinline__ void set_error(const Dev& d, unsigned long long bit) { atomicOr(&d.ctr[CTR_ERRORS], bit); }

__device__ __forceinline__ unsigned long long ld_relaxed(const unsigned long long* p) {
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Coherent reads of words another workgroup publishes during this launch.  A load (even an
// agent-scope one) can be served by a stale line of this XCD's L2; an idempotent RMW such
// as atomicOr(p, 0) may be folded into such a load by the compiler.  A compare-and-swap
// with an impossible comparand is a real memory-side RMW that never changes the word.
__device__ __forceinline__ unsigned long long rmw_read(unsigned long long* p) { return atomicCAS(p, ~0ull, ~0ull); }
__device__ __forceinline__ unsigned int rmw_read(unsigned int* p) { return atomicCAS(p, 0xffffffffu, 0xffffffffu); }

// ---------------------------------------------------------------------------------
// Service table: open addressing on the 64-bit tag, 128-bit key verified.
//
// No lane ever waits for another lane's publication: a same-wave claimer whose publish
// sits on a divergent loop exit would be scheduled after the waiter (SIMT deadlock).
// A claimer CASes the tag and stores the second half; a finder compares the second half
// when it is already visible and otherwise queues (slot, hi) for k_verify, which runs
// after the inserting kernel.  A mismatch there is reported as EBD_ERR_COLLISION.
// ---------------------------------------------------------------------------------
__device__ uint32_t agg_insert(const Dev& d, Hash128 h, unsigned long long seq, uint32_t cls) {
	uint32_t idx = (uint32_t)h.lo & d.slot_mask;
	bool found = false;
	unsigned long long seen_min = 0;
	for (uint32_t probe = 0; probe <= d.slot_mask; probe++) {
		Slot* s = d.slots + idx;
		// One plain load pass over the slot's first 32 bytes.  tag and hi are written once
		// (0 -> value), min_seq only decreases: a stale copy at worst shows 0 (resolved by
		// the CAS below, or the coherent re-read of hi) or a larger min_seq (a redundant
		// atomicMin).  Slot words are only ever written by atomics here, so no dirty line
		// sits in L2 when the next kernel starts.
		const ulonglong2 th = *(const ulonglong2*)&s->tag;
		const ulonglong2 mo = *(const ulonglong2*)&s->min_seq;
		seen_min = mo.x;
		unsigned long long t = th.x;
		bool claimed = false;
		if (t == 0) {
			t = atomicCAS(&s->tag, 0ull, h.lo);
			if (t == 0) {
				atomicExch(&s->hi, h.hi);
				const unsigned long long k = atomicAdd(&d.ctr[CTR_NEW], 1ull);
				if (k < d.new_cap)
					d.new_slots[k] = idx;
				else
					set_error(d, EBD_ERR_TABLE_FULL);
				claimed = true;
				seen_min = ~0ull;
			}
		}
		if (claimed) {
			found = true;
			break;
		}
		if (t == h.lo) {
			unsigned long long hi = th.y;
			if (hi == 0)
				hi = rmw_read(&s->hi);
			if (hi == 0) { // claimer's store not visible yet: verify after this kernel
				const unsigned long long k = atomicAdd(&d.ctr[CTR_VERIFY], 1ull);
				if (k < d.verify_cap) {
					d.verify[k].slot = idx;
					d.verify[k].hi = h.hi;
				} else {
					set_error(d, EBD_ERR_VERIFY_FULL);
				}
				found = true;
				break;
			}
			if (hi == h.hi) {
				found = true;
				break;
			}
			atomicAdd(&d.ctr[CTR_COLLISIONS], 1ull); // same tag, other key: keep probing
		}
		idx = (idx + 1) & d.slot_mask;
	}
	if (!found) {
		set_error(d, EBD_ERR_TABLE_FULL);
		return 0xffffffffu;
	}
	Slot* s = d.slots + idx;
	if (cls == CLS_INTERNAL)
		atomicAdd(&s->internal_clients, 1u);
	else if (cls == CLS_EXTERNAL)
		atomicAdd(&s->external_clients, 1u);
	if (seq < seen_min)
		atomicMin(&s->min_seq, seq);
	return idx;
}

// ---------------------------------------------------------------------------------
// Session set: (pid, fd, sessionID) -> slot.  Claimed by a CAS on the 64-bit tag; the
// full key is stored by the claimer and compared by sset_find in later kernels (a tag
// shared by two keys is reported as EBD_ERR_COLLISION there).
// ---------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long sset_tag(unsigned long long kv, uint32_t sid) {
	return fmix64(kv ^ ((unsigned long long)sid * 0x9E3779B97F4A7C15ull) ^ 0x5bd1e9955bd1e995ull) | 1ull;
}

__device__ int sset_insert(const Dev& d, uint32_t pid, uint32_t fd, uint32_t sid, uint32_t carry) {
	const unsigned long long kv = ((unsigned long long)fd << 32) | pid;
	const unsigned long long tag = sset_tag(kv, sid);
	uint32_t idx = (uint32_t)tag & d.sset_mask;
	int res = -1;
	for (uint32_t probe = 0; probe <= d.sset_mask; probe++) {
		SSlot* s = d.sset + idx;
		unsigned long long t = ld_relaxed(&s->tag);
		if (t == 0) {
			t = atomicCAS(&s->tag, 0ull, tag);
			if (t == 0) {
				s->kv = kv;
				s->sid = sid;
				const unsigned long long k = atomicAdd(&d.ctr[CTR_DIRTY], 1ull);
				d.dirty[k] = idx;
				t = tag;
			}
		}
		if (t == tag) {
			res = (int)idx;
			break;
		}
		idx = (idx + 1) & d.sset_mask;
	}
	if (res < 0) {
		set_error(d, EBD_ERR_SESSION_FULL);
		return -1;
	}
	if (carry)
		d.sset[res].carry = carry;
	return res;
}

// Lookup after the inserting kernels finished (plain loads are coherent then).
__device__ int sset_find(const Dev& d, uint32_t pid, uint32_t fd, uint32_t sid) {
	const unsigned long long kv = ((unsigned long long)fd << 32) | pid;
	const unsigned long long tag = sset_tag(kv, sid);
	uint32_t idx = (uint32_t)tag & d.sset_mask;
	for (uint32_t probe = 0; probe <= d.sset_mask; probe++) {
		const SSlot* s = d.sset + idx;
		const unsigned long long t = s->tag;
		if (t == 0)
			return -1;
		if (t == tag) {
			if (s->kv == kv && s->sid == sid)
				return (int)idx;
			set_error(d, EBD_ERR_COLLISION); // two sessions share a 64-bit tag
		}
		idx = (idx + 1) & d.sset_mask;
	}
	return -1;
}

// ---------------------------------------------------------------------------------
// k_fresh: one lane per event, DFA table in LDS.
//
// A workgroup takes tiles of kTile events and counting-sorts each tile by its number of
// 16-byte chunks (LDS histogram), longest first, so a wave scans 64 buffers of nearly equal
// length and its lanes finish together; waves take groups from an LDS counter.  A lane
// reads its buffer one 128-byte line at a time (8 chunks, the next line in flight).  Per byte:
// one table step (v_mad_u32_u24 + ds_read_u8) and a running maximum; per chunk: the
// branch-free crossing trackers of ebd_fresh.h.
// ---------------------------------------------------------------------------------
// Logical index (s << 8) | b into the LDS image (ebd_dfa.h kLdsRow / lds_col).
struct LdsTable {
	const uint8_t* t;
	__device__ __forceinline__ uint32_t operator[](uint32_t i) const { return t[(i >> 8) * kLdsRow + lds_col(i & 0xffu)]; }
};

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned long long u64a1 __attribute__((aligned(1)));
// 16-byte load through a global (not flat) pointer: global_load_dwordx4
__device__ __forceinline__ Chunk gload16(uintptr_t a) {
	const v4u v = *(const __attribute__((address_space(1))) v4u*)a;
	Chunk c;
	c.w[0] = v.x;
	c.w[1] = v.y;
	c.w[2] = v.z;
	c.w[3] = v.w;
	return c;
}
// 8 bytes at any alignment: global_load_dwordx2 (gfx950 runs in unaligned-access mode)
__device__ __forceinline__ unsigned long long gload8u(const uint8_t* a) {
	return *(const __attribute__((address_space(1))) u64a1*)a;
}

// Buffer access for fresh_finalize on the device.  The payload must stay readable up to
// the next 16-byte boundary after each buffer plus 8 bytes (ebd_api.hip pads it).
struct DevMem {
	const uint8_t* p;
	uintptr_t q; // p rounded down to 16
	uint32_t last; // last chunk index of the buffer
	__device__ __forceinline__ Chunk chunk(uint32_t c) const { return gload16(q + 16 * (uintptr_t)min(c, last)); }
	__device__ __forceinline__ unsigned long long ld8(uint32_t o) const { return gload8u(p + o); }
};

constexpr int kFreshThreads = 1024;
constexpr int kTile = 4096;
constexpr int kBins = 128;

// A chunk word with every byte b replaced by lds_col(b) (5 VALU per 4 bytes).
__device__ __forceinline__ uint32_t lds_cols(uint32_t w) {
#ifndef EBD_LDS_PLAIN
	return ((w << 2) & 0x7c7c7c7cu) | ((w >> 5) & 0x03030303u) | (w & 0x80808080u);
#else
	return w;
#endif
}

// LDS address of entry (s, byte k of the column-mapped word wc).
__device__ __forceinline__ uint32_t tab_index(uint32_t s, uint32_t wc, int k) {
#ifndef EBD_LDS_PLAIN
	return s * kLdsRow + __builtin_amdgcn_ubfe(wc, 8 * (k & 3), 8); // v_bfe + v_mad_u32_u24
#else
	return __builtin_amdgcn_perm(s, wc, 0x0c0c0400u | (uint32_t)(k & 3)); // (s << 8) | byte
#endif
}

// What fresh_event needs of an event, read once (coalesced) while a tile is binned and kept
// in LDS in sorted order, so the scan issues no scattered metadata loads.
struct TileEv {
	unsigned long long off_idx; // buffer offset (bits 0..47), tile-relative event index (48..63)
	uint32_t pid;
	uint16_t len;
	uint8_t flags;
	uint8_t kind; // TE_*
};
static_assert(sizeof(TileEv) == 16, "tile record is 16 bytes");
enum : uint8_t { TE_PARSE = 0, TE_SKIP = 1, TE_BAD = 2 };

// Loads one event's record fields; the bin is its chunk count as fresh_event chunks it.
__device__ __forceinline__ TileEv tile_ev(const Dev& d, uint32_t i, uint32_t t, uint32_t* bin) {
	const uint8_t* evb = (const uint8_t*)(d.ev + i);
	const uint8_t flags = evb[32];
	const uint32_t pid = *(const uint32_t*)evb;
	const uint32_t L = d.len[i];
	const uint64_t off = d.off[i];
	TileEv te;
	te.off_idx = (off & 0xffffffffffffull) | ((unsigned long long)t << 48);
	te.pid = pid;
	te.flags = flags;
	te.len = (uint16_t)(L <= EBD_BUFFER_MAX_DATA_SIZE ? L : 0);
	te.kind = !(flags & FLAG_NEW) || L == EBD_NO_BUFFER ? TE_SKIP
	        : (L > EBD_BUFFER_MAX_DATA_SIZE || off >> 48) ? TE_BAD : TE_PARSE;
	const uint32_t skip = (uint32_t)(off + (uintptr_t)d.payload) & 127u;
	const uint32_t ch = (skip + L + 15) >> 4;
	*bin = te.kind != TE_PARSE ? 0 : (ch < kBins ? ch : kBins - 1);
	return te;
}

// 16 DFA steps over one chunk; m collects the maximum next state.
template <bool kFull>
__device__ __forceinline__ void scan_chunk(const uint8_t* T, const Chunk& w, uint32_t& s, uint32_t& m, uint32_t pos0,
		uint32_t skip, uint32_t end) {
#ifdef EBD_EXP_MEMONLY // experiment: the loads without the DFA (results are wrong)
	m ^= w.w[0] ^ w.w[1] ^ w.w[2] ^ w.w[3];
	return;
#endif
	const uint32_t wc[4] = {lds_cols(w.w[0]), lds_cols(w.w[1]), lds_cols(w.w[2]), lds_cols(w.w[3])};
#pragma unroll
	for (int k = 0; k < 16; k++) {
		const uint32_t sn = T[tab_index(s, wc[k >> 2], k)];
		if (kFull) {
			s = sn;
			if (k & 1)
				m = max(m, s);
			else
				m = max(m, sn); // pairs fold into v_max3
		} else {
			const bool v = pos0 + k >= skip && pos0 + k < end;
			s = v ? sn : s;
			m = max(m, v ? sn : 0u);
		}
	}
}

// Partial chunk (the buffer starts or ends inside it, or lies outside it): the steps at
// positions [lo, hi) of the chunk count, the others leave the state alone.
__device__ __forceinline__ void scan_chunk_masked(const uint8_t* T, const Chunk& w, uint32_t& s, uint32_t& m,
		uint32_t pos0, uint32_t skip, uint32_t end) {
#ifdef EBD_EXP_MEMONLY
	m ^= w.w[0] ^ w.w[1] ^ w.w[2] ^ w.w[3];
	return;
#endif
	const int lo = (int)skip - (int)pos0, hi = (int)end - (int)pos0;
	const uint32_t wc[4] = {lds_cols(w.w[0]), lds_cols(w.w[1]), lds_cols(w.w[2]), lds_cols(w.w[3])};
#pragma unroll
	for (int k = 0; k < 16; k++) {
		const uint32_t sn = T[tab_index(s, wc[k >> 2], k)];
		const bool v = k >= lo && k < hi;
		s = v ? sn : s;
		m = max(m, v ? sn : 0u);
	}
}

__device__ __forceinline__ void fresh_event(const Dev& d, const uint8_t* T, const TileEv& te, uint32_t base) {
	const uint32_t i = base + (uint32_t)(te.off_idx >> 48);
	const uint8_t flags = te.flags;
	const uint32_t L = te.len;
	const uint64_t boff = te.off_idx & 0xffffffffffffull;
	FreshResult fr;
	fr.r.consumed = 0;
	fr.r.status = EBD_STATUS_NONE;
	fr.r.info = 0;
	fr.r.u.session.index = 0;
	fr.r.u.session.pad_[0] = fr.r.u.session.pad_[1] = 0;
	fr.cip = false;
	if (te.kind != TE_SKIP) {
		if (te.kind == TE_BAD) {
			set_error(d, EBD_ERR_BAD_INPUT);
		} else {
			const DfaInfo& di = d.di;
			const uint8_t* p = d.payload + boff;
			const uintptr_t pa = (uintptr_t)p;
			const uintptr_t q = pa & ~(uintptr_t)127; // the buffer's first 128-byte line
			const uint32_t skip = (uint32_t)(pa & 127);
			const uint32_t end = skip + L;
			const uint32_t nch = (end + 15) >> 4;
			ScanRec sr;
			rec_init(di, sr);
			uint32_t s = di.init;
			// The buffer is read line by line: window j is the j-th 128-byte line from the
			// one holding the buffer's first byte (8 chunks), its 8 loads issued back to back.
			// Every 16-B lane load is its own L2 request, and ~32k lanes per XCD keep more
			// lines in flight than the 4 MB L2 holds, so a line must be consumed by the loads
			// issued together: windows that straddle lines re-fetched each line (measured
			// 3.5 L2 misses per line).  The next line is in flight while one is scanned; two
			// register windows keep fixed roles (a register copy of a loaded chunk, or a load
			// behind a branch, would make the wave wait for every load).  Loads past the
			// buffer re-read its last chunk.
			const uint32_t last = nch ? nch - 1 : 0;
			Chunk A[8], B[8];
			auto ldw = [&](Chunk(&w)[8], uint32_t j) {
#pragma unroll
				for (int k = 0; k < 8; k++)
					w[k] = gload16(q + 16 * (uintptr_t)min(8 * j + k, last));
			};
			bool live = nch > 0;
			// One chunk for every lane (a no-op for lanes already done): DFA steps, then the
			// trackers.  The only exits are uniform.
			auto step = [&](const Chunk& w, uint32_t c) {
				uint32_t sx = s, m = 0;
				const bool full = c * 16 >= skip && c * 16 + 16 <= end;
				if (__all(full))
					scan_chunk<true>(T, w, sx, m, c * 16, skip, end);
				else
					scan_chunk_masked(T, w, sx, m, c * 16, skip, end);
				if (live) {
					if (st_terminal(di, sx)) {
						sr.term = (c << 8) | s;
						sr.cseen |= m >= 254 ? 1u : 0u; // sr.cip already names this chunk
						live = false;
					} else {
						chunk_track(di, sr, c, sx, m >= 254);
						live = c + 1 < nch;
					}
					s = sx;
				}
			};
			ldw(A, 0);
			for (uint32_t j = 0;; j += 2) {
				ldw(B, j + 1);
#pragma unroll
				for (int k = 0; k < 8; k++) {
					step(A[k], 8 * j + k);
					if (!__any(live))
						break;
				}
				if (!__any(live))
					break;
				ldw(A, j + 2);
#pragma unroll
				for (int k = 0; k < 8; k++) {
					step(B[k], 8 * (j + 1) + k);
					if (!__any(live))
						break;
				}
				if (!__any(live))
					break;
			}
#ifdef EBD_EXP_SCANONLY // experiment: scan cost alone (results are wrong)
			fr.r.consumed = (uint16_t)s;
			fr.r.u.span.url_off = (uint16_t)(sr.url ^ sr.host ^ sr.hend ^ sr.cip ^ sr.term ^ sr.cseen);
			d.res[i] = fr.r;
			return;
#endif
			fresh_finalize(LdsTable{T}, di, sr, s, DevMem{p, q, last}, skip, L, te.pid, flags, fr);
			if (fr.r.status == EBD_STATUS_FINISHED) {
				d.keys[i] = fr.key;
			} else if (fr.r.status == EBD_STATUS_UNFINISHED) {
				// the session may be saved (Discovery.cpp:148-150): sequential path
				const EventRec& ev = d.ev[i];
				atomicAdd(&d.ctr[CTR_UNFINISHED], 1ull);
				sset_insert(d, ev.pid, ev.fd, ev.sessionID, 0);
			}
		}
	}
	d.res[i] = fr.r;
}

#ifdef EBD_EXP_LB8 // experiment: two workgroups per CU
__global__ __launch_bounds__(kFreshThreads, 8) void k_fresh(Dev d) {
#else
__global__ __launch_bounds__(kFreshThreads) void k_fresh(Dev d) {
#endif
	// static LDS: the table sits at LDS address 0, so a step's index is its address
	__shared__ __attribute__((aligned(16))) uint8_t T[kLdsTableBytes];
	__shared__ TileEv tev[kTile]; // the tile's events in scan order (longest first)
	__shared__ uint32_t hist[kBins];
	__shared__ uint32_t next_group;
	for (uint32_t k = threadIdx.x * 16u; k < kLdsTableBytes; k += kFreshThreads * 16u)
		*(uint4*)(T + k) = *(const uint4*)(d.dfa + k);
	const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
	constexpr int kPer = kTile / kFreshThreads;
	const uint32_t ntiles = (d.n + kTile - 1) / kTile;
	for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
		const uint32_t base = tile * kTile;
		const uint32_t cnt = d.n - base < (uint32_t)kTile ? d.n - base : (uint32_t)kTile;
		__syncthreads(); // previous tile's records fully consumed; table loaded
		if (threadIdx.x < kBins)
			hist[threadIdx.x] = 0;
		if (threadIdx.x == 0)
			next_group = 0;
		__syncthreads();
		uint32_t bin[kPer], rank[kPer];
		TileEv rec[kPer];
#pragma unroll
		for (int k = 0; k < kPer; k++) {
			const uint32_t t = threadIdx.x + k * kFreshThreads;
			rec[k] = tile_ev(d, base + (t < cnt ? t : 0), t, &bin[k]); // unconditional loads, all in flight
		}
#pragma unroll
		for (int k = 0; k < kPer; k++) {
			const uint32_t t = threadIdx.x + k * kFreshThreads;
			bin[k] = t < cnt ? kBins - 1 - bin[k] : 0; // longest buffers first
#ifdef EBD_EXP_NOSORT // experiment: memory order (a wave takes 64 adjacent buffers)
			bin[k] = 0;
#endif
			rank[k] = t < cnt ? atomicAdd(&hist[bin[k]], 1u) : 0;
		}
		__syncthreads();
		if (wave == 0) { // exclusive scan of the 128 bins, two per lane
			const uint32_t a = hist[2 * lane], b = hist[2 * lane + 1];
			uint32_t x = a + b;
#pragma unroll
			for (int o = 1; o < 64; o <<= 1) {
				const uint32_t y = __shfl_up(x, o);
				if ((int)lane >= o)
					x += y;
			}
			const uint32_t excl = x - a - b;
			hist[2 * lane] = excl;
			hist[2 * lane + 1] = excl + a;
		}
		__syncthreads();
#pragma unroll
		for (int k = 0; k < kPer; k++) {
			const uint32_t t = threadIdx.x + k * kFreshThreads;
#ifdef EBD_EXP_NOSORT
			if (t < cnt)
				tev[t] = rec[k];
#else
			if (t < cnt)
				tev[hist[bin[k]] + rank[k]] = rec[k];
#endif
		}
		__syncthreads();
		// groups of 64 in descending length; a wave takes the next one when it is free
		// (longest-first greedy: the short groups at the end even out the waves)
		for (;;) {
			uint32_t g = 0;
			if (lane == 0)
				g = atomicAdd(&next_group, 1u);
			g = __builtin_amdgcn_readfirstlane(g);
			if (g * 64 >= cnt)
				break;
			const uint32_t t = g * 64 + lane;
			if (t < cnt)
				fresh_event(d, T, tev[t], base);
		}
	}
}

// ---------------------------------------------------------------------------------
// Client-IP token and class of a fast-path request that carries a client-IP header
// (HttpRequestParser.cpp:370-407 on the first client-IP value, Aggregator.cpp:50-74 on its
// front token).  k_fresh found where the value starts; the lane copies the value's first
// kCipRaw bytes into its LDS row with 8-byte loads and parses the token there.
// ---------------------------------------------------------------------------------
constexpr int kAggThreads = 256;
constexpr int kCipRaw = 64;
constexpr int kCipStride = kCipRaw + 8; // rows 72 B apart: lanes spread over the banks

__device__ __forceinline__ uint32_t cip_classify(const Dev& d, uint32_t i, ebd_event_result& r, uint8_t* row) {
	const uint8_t* p = d.payload + d.off[i];
	const uint32_t cs = r.u.span.cip_off, lim = r.consumed; // the value ends before the final CRLF
	unsigned long long v[kCipRaw / 8];
#pragma unroll
	for (int h = 0; h < kCipRaw / 8; h++) // past the request: re-read its last byte (stays in the buffer)
		v[h] = gload8u(p + min(cs + 8 * h, lim - 1));
#pragma unroll
	for (int h = 0; h < kCipRaw / 8; h++)
		*(unsigned long long*)(row + 8 * h) = v[h];
	uint32_t tb, te;
	uint8_t cls;
	const uint32_t avail = lim - cs < (uint32_t)kCipRaw ? lim - cs : (uint32_t)kCipRaw; // valid bytes in the row
	uint32_t e = 0;
	while (e < avail && row[e] != ',' && row[e] != '\r')
		e++;
	if (e < avail || avail == lim - cs) {
		cip_token(*d.ifs, [row](uint32_t b) { return (uint32_t)row[b]; }, 0, e, &tb, &te, &cls);
	} else { // a value longer than the copy without ',' or CR in it: parse from the buffer
		cip_token(*d.ifs, [p](uint32_t b) { return (uint32_t)p[b]; }, cs, lim, &tb, &te, &cls);
		tb -= cs;
		te -= cs;
	}
	r.u.span.cip_off = (uint16_t)(cs + tb);
	r.u.span.cip_len = (uint16_t)(te - tb);
	return cls;
}

__global__ void k_carry_insert(Dev d) {
	for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < d.n_carry_in; c += gridDim.x * blockDim.x) {
		const Carry& cr = d.carry_in[c];
		sset_insert(d, cr.pid, cr.fd, cr.sid, c + 1);
	}
}

__global__ void k_slow_collect(Dev d) {
	if (d.ctr[CTR_DIRTY] == 0)
		return; // no session needs the sequential path in this batch
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < d.n; i += gridDim.x * blockDim.x) {
		const EventRec& e = d.ev[i];
		if (!(e.flags & (FLAG_NEW | FLAG_END)))
			continue;
		const int slot = sset_find(d, e.pid, e.fd, e.sessionID);
		if (slot >= 0) {
			const unsigned long long k = atomicAdd(&d.ctr[CTR_SLOW], 1ull);
			d.slow_keys[k] = ((unsigned long long)(uint32_t)slot << 32) | i;
		}
	}
}

// ---------------------------------------------------------------------------------
// k_walk: the sequential session path.  The bytes of the request in progress are the
// carried bytes (if the request started in an earlier batch) followed by the buffers
// of this batch's events from position j0 on.
// ---------------------------------------------------------------------------------
struct Walk {
	const uint8_t* cb; // carried bytes of the request in progress
	uint32_t clen;
	uint32_t j0;       // first sorted position whose buffer belongs to the request
};

__device__ __forceinline__ uint32_t slow_event(const Dev& d, uint32_t j) { return (uint32_t)d.slow_keys[j]; }

__device__ __forceinline__ uint32_t piece_len(const Dev& d, uint32_t j) {
	const uint32_t i = slow_event(d, j);
	const uint32_t L = d.len[i];
	return ((d.ev[i].flags & FLAG_NEW) && L != EBD_NO_BUFFER && L <= EBD_BUFFER_MAX_DATA_SIZE) ? L : 0;
}

// Visits stream bytes [a, a + n) in order; the stream ends at sorted position jend whose
// piece is truncated to cend bytes.  fn(byte) returns false to stop.  Returns bytes visited.
template <typename Fn>
__device__ uint32_t stream_visit(const Dev& d, const Walk& w, uint32_t jend, uint32_t cend, uint32_t a, uint32_t n, Fn fn) {
	uint32_t pos = 0, done = 0;
	const uint32_t b = a + n;
	if (w.clen) {
		for (uint32_t k = a; k < b && k < w.clen; k++) {
			if (!fn(w.cb[k]))
				return done;
			done++;
		}
		pos = w.clen;
	}
	for (uint32_t j = w.j0; j <= jend && pos < b; j++) {
		uint32_t pl = piece_len(d, j);
		if (j == jend)
			pl = cend;
		if (pl == 0)
			continue;
		const uint32_t lo = a > pos ? a : pos, hi = b < pos + pl ? b : pos + pl;
		if (lo < hi) {
			const uint8_t* src = d.payload + d.off[slow_event(d, j)] + (lo - pos);
			for (uint32_t k = 0; k < hi - lo; k++) {
				if (!fn(src[k]))
					return done;
				done++;
			}
		}
		pos += pl;
	}
	return done;
}

// handleSuccessfulParse -> handleNewRequest -> Aggregator::newRequest
// (Discovery.cpp:161-192, 210-212) for a request finished by the session path.
__device__ void emit_session_request(const Dev& d, const Walk& w, uint32_t jend, uint32_t cend, const GenParser& g,
		uint32_t i, ebd_event_result& r) {
	const EventRec& ev = d.ev[i];
	const uint32_t hl = (g.f & GPF_HOST) ? g.host_len : 0, ul = g.url_len;
	uint32_t raw = 0;
	if (g.f & GPF_CIP_FOUND) // the value up to its first ',' is the front token's source
		raw = stream_visit(d, w, jend, cend, g.cip_start, g.cip_len, [](uint8_t c) { return c != ','; });
	const uint32_t total = hl + ul + raw;
	const unsigned long long at = atomicAdd(&d.ctr[CTR_SSTR], (unsigned long long)total);
	uint8_t info = (uint8_t)((g.mcand == 'P' ? EBD_INFO_POST : 0) | ((g.f & GPF_HTTPS) ? EBD_INFO_HTTPS : 0) | EBD_INFO_SESSION);
	uint8_t cls;
	KeyHasher kh;
	kh.init(ev.pid);
	uint32_t tb = 0, te = 0;
	if (at + total > d.sstr_cap) {
		set_error(d, EBD_ERR_ARENA_FULL);
		return;
	}
	uint8_t* dst = d.sstr + at;
	uint32_t k = 0;
	stream_visit(d, w, jend, cend, g.host_start, hl, [&](uint8_t c) {
		dst[k++] = c;
		return true;
	});
	stream_visit(d, w, jend, cend, g.url_start, ul, [&](uint8_t c) {
		dst[k++] = c;
		return true;
	});
	if (raw)
		stream_visit(d, w, jend, cend, g.cip_start, raw, [&](uint8_t c) {
			dst[k++] = c;
			return true;
		});
	if (g.f & GPF_CIP_FOUND) {
		front_token(dst + hl + ul, raw, &tb, &te);
		info |= EBD_INFO_CIP;
		cls = classify_token(*d.ifs, dst + hl + ul + tb, te - tb);
	} else {
		cls = classify_source(*d.ifs, ev.flags, ev.sourceIP);
	}
	info |= (uint8_t)(cls << EBD_INFO_CLASS_SHIFT);
	kh.bytes(dst, hl + ul);
	agg_insert(d, kh.finish(), d.seq_base + i, cls);
	atomicAdd(&d.ctr[CTR_REQUESTS], 1ull);
	const unsigned long long q = atomicAdd(&d.ctr[CTR_SREQ], 1ull);
	SessReq sr;
	sr.seq = d.seq_base + i;
	sr.pid = ev.pid;
	sr.str_off = (uint32_t)at;
	sr.host_len = (uint16_t)hl;
	sr.url_len = (uint16_t)ul;
	sr.cip_off = (uint16_t)(hl + ul + tb);
	sr.cip_len = (uint16_t)(te - tb);
	sr.info = info;
	sr.status = EBD_STATUS_FINISHED;
	sr.pad = 0;
	sr.pad2 = 0;
	d.sreq[q] = sr;
	r.info = info;
	r.u.session.index = (uint32_t)q;
}

__device__ void walk_session(const Dev& d, uint32_t j, uint32_t nslow, uint32_t slot) {
	SSlot* ss = d.sset + slot;
	ss->visited = 1;
	GenParser g;
	bool live = false;
	Walk w{nullptr, 0, j};
	const uint32_t carry = ss->carry;
	if (carry) { // saved session from an earlier batch (LRU entry)
		const Carry& c = d.carry_in[carry - 1];
		g = c.g;
		live = true;
		w.cb = c.bytes;
		w.clen = c.nbytes;
	} else {
		gp_init(g);
	}
	const KeyTrie* trie = d.trie;
	uint32_t jj = j;
	for (; jj < nslow && (uint32_t)(d.slow_keys[jj] >> 32) == slot; jj++) {
		const uint32_t i = slow_event(d, jj);
		const EventRec& ev = d.ev[i];
		const uint8_t flags = ev.flags;
		const uint32_t L = d.len[i];
		ebd_event_result r;
		r.consumed = 0;
		r.status = EBD_STATUS_NONE;
		r.info = EBD_INFO_SESSION;
		r.u.session.index = 0xffffffffu;
		r.u.session.pad_[0] = r.u.session.pad_[1] = 0;
		atomicAdd(&d.ctr[CTR_SESSION_EVENTS], 1ull);
		if ((flags & FLAG_NEW) && L != EBD_NO_BUFFER && L <= EBD_BUFFER_MAX_DATA_SIZE) {
			const uint8_t* buf = d.payload + d.off[i];
			auto at = [buf](uint32_t k) { return (uint32_t)buf[k]; };
			if (live) { // handleExistingSession, Discovery.cpp:123-139
				r.info |= EBD_INFO_EXISTING;
				const uint32_t c = gp_parse(g, trie, at, L, flags);
				r.consumed = (uint16_t)c;
				if (g.state == ST_INVALID) {
					r.status = EBD_STATUS_INVALID;
					atomicAdd(&d.ctr[CTR_KDELETES], 1ull); // bpfDiscoveryDeleteSession
					live = false;
				} else if (g.state == ST_FINISHED) {
					r.status = EBD_STATUS_FINISHED;
					emit_session_request(d, w, jj, c, g, i, r);
					gp_reset(g); // session.reset(); stays saved
					w = Walk{nullptr, 0, jj + 1};
				} else {
					r.status = EBD_STATUS_UNFINISHED;
				}
			} else { // handleNewSession, Discovery.cpp:141-159
				gp_init(g);
				w = Walk{nullptr, 0, jj};
				const uint32_t c = gp_parse(g, trie, at, L, flags);
				r.consumed = (uint16_t)c;
				if (g.state == ST_INVALID) {
					r.status = EBD_STATUS_INVALID;
				} else if (g.state == ST_FINISHED) {
					r.status = EBD_STATUS_FINISHED;
					emit_session_request(d, w, jj, c, g, i, r);
				} else {
					r.status = EBD_STATUS_UNFINISHED;
					if (!(flags & FLAG_END)) {
						live = true; // saveSession
						atomicAdd(&d.ctr[CTR_INSERTS], 1ull);
					}
				}
			}
		}
		if (flags & FLAG_END) // handleCloseEvent, Discovery.cpp:194-198
			live = false;
		d.res[i] = r;
	}
	if (live) { // saved for the next batch, with the bytes of the request in progress
		const unsigned long long c = atomicAdd(&d.ctr[CTR_CARRY_OUT], 1ull);
		if (c >= d.carry_cap) {
			set_error(d, EBD_ERR_LRU_OVERFLOW);
			return;
		}
		Carry& out = d.carry_out[c];
		const EventRec& ev = d.ev[slow_event(d, j)];
		out.pid = ev.pid;
		out.fd = ev.fd;
		out.sid = ev.sessionID;
		out.g = g;
		const uint32_t nb = g.length < kCarryBytes ? g.length : kCarryBytes;
		out.nbytes = nb;
		uint32_t k = 0;
		uint8_t* dst = out.bytes;
		// the request in progress ends with the last event of this session (fully consumed)
		stream_visit(d, w, jj - 1, piece_len(d, jj - 1), 0, nb, [&](uint8_t b) {
			dst[k++] = b;
			return true;
		});
	}
}

__global__ void k_walk(Dev d, uint32_t nslow) {
	for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nslow; j += gridDim.x * blockDim.x) {
		const uint32_t slot = (uint32_t)(d.slow_keys[j] >> 32);
		if (j > 0 && (uint32_t)(d.slow_keys[j - 1] >> 32) == slot)
			continue;
		walk_session(d, j, nslow, slot);
	}
}

// Saved sessions with no event in this batch stay saved unchanged.
__global__ void k_carry_pass(Dev d) {
	for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < d.n_carry_in; c += gridDim.x * blockDim.x) {
		const Carry& cr = d.carry_in[c];
		const int slot = sset_find(d, cr.pid, cr.fd, cr.sid);
		if (slot >= 0 && d.sset[slot].visited)
			continue;
		const unsigned long long k = atomicAdd(&d.ctr[CTR_CARRY_OUT], 1ull);
		if (k >= d.carry_cap) {
			set_error(d, EBD_ERR_LRU_OVERFLOW);
			continue;
		}
		Carry& out = d.carry_out[k];
		out.pid = cr.pid;
		out.fd = cr.fd;
		out.sid = cr.sid;
		out.g = cr.g;
		out.nbytes = cr.nbytes;
		for (uint32_t b = 0; b < cr.nbytes; b++)
			out.bytes[b] = cr.bytes[b];
	}
}

// Aggregator::newRequest for the fast-path requests, in event order (coalesced reads of the
// results, keys and events).  The client class comes from the client-IP header's front token
// when k_fresh found one (cip_classify), else from the session's source address
// (Aggregator.cpp:60-66, 85-88).  Requests are counted per block: one global atomic each.
__global__ __launch_bounds__(kAggThreads) void k_agg_fast(Dev d) {
	__shared__ __attribute__((aligned(8))) uint8_t rows[kAggThreads * kCipStride];
	__shared__ unsigned long long nreq;
	uint8_t* row = rows + threadIdx.x * kCipStride;
	if (threadIdx.x == 0)
		nreq = 0;
	__syncthreads();
	uint32_t cnt = 0;
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < d.n; i += gridDim.x * blockDim.x) {
		ebd_event_result r = d.res[i];
		if (r.status != EBD_STATUS_FINISHED || (r.info & EBD_INFO_SESSION))
			continue;
		uint32_t cls;
		if (r.info & EBD_INFO_CIP) {
			cls = cip_classify(d, i, r, row);
		} else {
			const uint8_t* evb = (const uint8_t*)(d.ev + i);
			const v4u sv = *(const __attribute__((address_space(1))) v4u*)(evb + 16); // sourceIP (4-B aligned)
			uint8_t src[16];
			__builtin_memcpy(src, &sv, 16);
			cls = classify_source(*d.ifs, evb[32], src);
		}
		r.info = (uint8_t)((r.info & ~(3u << EBD_INFO_CLASS_SHIFT)) | (cls << EBD_INFO_CLASS_SHIFT));
		d.res[i] = r;
		agg_insert(d, d.keys[i], d.seq_base + i, cls);
		cnt++;
	}
	atomicAdd(&nreq, (unsigned long long)cnt);
	__syncthreads();
	if (threadIdx.x == 0 && nreq)
		atomicAdd(&d.ctr[CTR_REQUESTS], nreq);
}

// First-arrival representative of every service created in this batch (Aggregator.cpp:
// 112-130, 160-167): endpoint string, domain, scheme, pid.
__global__ void k_reps(Dev d) {
	const unsigned long long nn = d.ctr[CTR_NEW];
	const uint32_t n_new = (uint32_t)(nn < d.new_cap ? nn : d.new_cap);
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n_new; k += gridDim.x * blockDim.x) {
		Slot* s = d.slots + d.new_slots[k];
		const unsigned long long seq = s->min_seq;
		const uint32_t e = (uint32_t)(seq - d.seq_base);
		const ebd_event_result r = d.res[e];
		const uint8_t *host, *url;
		uint32_t hl, ul;
		if (r.info & EBD_INFO_SESSION) {
			const SessReq& q = d.sreq[r.u.session.index];
			host = d.sstr + q.str_off;
			hl = q.host_len;
			url = host + hl;
			ul = q.url_len;
		} else {
			const uint8_t* p = d.payload + d.off[e];
			host = p + r.u.span.host_off;
			hl = r.u.span.host_len;
			url = p + r.u.span.url_off;
			ul = r.u.span.url_len;
		}
		const unsigned long long at = atomicAdd(&d.ctr[CTR_SARENA], (unsigned long long)(hl + ul));
		uint32_t doff = 0, dlen = 0;
		host_domain(host, hl, &doff, &dlen);
		s->pid = d.ev[e].pid;
		s->ep_len = hl + ul;
		s->dom = doff | (dlen << 16);
		s->info = ((r.info & EBD_INFO_HTTPS) ? 1u : 0u) | 2u;
		if (at + hl + ul > d.sarena_cap) {
			set_error(d, EBD_ERR_ARENA_FULL);
			s->ep_off = ~0ull;
			continue;
		}
		s->ep_off = at;
		uint8_t* dst = d.sarena + at;
		for (uint32_t b = 0; b < hl; b++)
			dst[b] = host[b];
		for (uint32_t b = 0; b < ul; b++)
			dst[hl + b] = url[b];
	}
}

__global__ void k_verify(Dev d) {
	const unsigned long long nv = d.ctr[CTR_VERIFY];
	const uint32_t n = (uint32_t)(nv < d.verify_cap ? nv : d.verify_cap);
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x)
		if (d.slots[d.verify[k].slot].hi != d.verify[k].hi)
			set_error(d, EBD_ERR_COLLISION);
}

__global__ void k_sset_clear(Dev d) {
	const unsigned long long nd = d.ctr[CTR_DIRTY];
	for (unsigned long long k = blockIdx.x * blockDim.x + threadIdx.x; k < nd; k += gridDim.x * blockDim.x) {
		SSlot* s = d.sset + d.dirty[k];
		s->tag = 0;
		s->kv = 0;
		s->sid = 0;
		s->pad = 0;
		s->carry = 0;
		s->visited = 0;
	}
}

__global__ void k_slots_init(Slot* slots, uint32_t n) {
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		Slot s;
		s.tag = 0;
		s.hi = 0;
		s.min_seq = ~0ull;
		s.ep_off = 0;
		s.pid = 0;
		s.internal_clients = 0;
		s.external_clients = 0;
		s.ep_len = 0;
		s.dom = 0;
		s.info = 0;
		s.pad[0] = s.pad[1] = 0;
		slots[k] = s;
	}
}

__global__ void k_collect(const Slot* slots, uint32_t n, ebd_service* out, unsigned long long* cnt) {
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const Slot& s = slots[k];
		if (s.tag == 0)
			continue;
		const unsigned long long at = atomicAdd(cnt, 1ull);
		ebd_service v;
		v.pid = s.pid;
		v.internal_clients = s.internal_clients;
		v.external_clients = s.external_clients;
		v.https = (uint8_t)(s.info & 1u);
		v.pad_[0] = v.pad_[1] = v.pad_[2] = 0;
		v.endpoint_off = s.ep_off;
		v.endpoint_len = s.ep_len;
		v.domain_off = s.dom & 0xffffu;
		v.domain_len = s.dom >> 16;
		v.pad2_ = 0;
		v.first_seq = s.min_seq;
		v.key_lo = s.tag;
		v.key_hi = s.hi;
		out[at] = v;
	}
}

// ---------------------------------------------------------------------------------
// Synthetic trace generation in HBM (ebd_gen.h).
// ---------------------------------------------------------------------------------
__global__ void k_gen_len(const GenTables* T, uint32_t config, unsigned long long seed, unsigned long long first, uint32_t n,
		uint32_t align, unsigned long long* alen) {
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
		alen[i] = align_up(gen_single(T, config, seed, first + i, nullptr, nullptr), align);
}

__global__ void k_gen_write(const GenTables* T, uint32_t config, unsigned long long seed, unsigned long long first, uint32_t n,
		EventRec* ev, uint32_t* len, const unsigned long long* off, uint8_t* payload) {
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
		EventRec e;
		const uint32_t L = gen_single(T, config, seed, first + i, &e, payload + off[i]);
		ev[i] = e;
		len[i] = L;
	}
}

// ---------------------------------------------------------------------------------
// launch wrappers (called from ebd_api.cpp)
// ---------------------------------------------------------------------------------
static int grid_for(uint64_t items, int block, int cap) {
	uint64_t g = (items + block - 1) / block;
	if (g < 1)
		g = 1;
	return (int)(g > (uint64_t)cap ? cap : g);
}

hipError_t launch_fresh(const Dev& d, hipStream_t st, int cus) {
	const uint32_t ntiles = (d.n + kTile - 1) / kTile;
	const int grid = (int)(ntiles < (uint32_t)cus * 2 ? ntiles : (uint32_t)cus * 2);
	hipLaunchKernelGGL(k_fresh, dim3(grid > 0 ? grid : 1), dim3(kFreshThreads), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_carry_insert(const Dev& d, hipStream_t st) {
	hipLaunchKernelGGL(k_carry_insert, dim3(grid_for(d.n_carry_in, 256, 256)), dim3(256), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_slow_collect(const Dev& d, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_slow_collect, dim3(grid_for(d.n, 256, cus * 8)), dim3(256), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_walk(const Dev& d, uint32_t nslow, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_walk, dim3(grid_for(nslow, 64, cus * 16)), dim3(64), 0, st, d, nslow);
	return hipGetLastError();
}
hipError_t launch_carry_pass(const Dev& d, hipStream_t st) {
	hipLaunchKernelGGL(k_carry_pass, dim3(grid_for(d.n_carry_in, 64, 256)), dim3(64), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_agg_fast(const Dev& d, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_agg_fast, dim3(grid_for(d.n, kAggThreads, cus * 8)), dim3(kAggThreads), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_reps(const Dev& d, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_reps, dim3(cus * 4), dim3(64), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_verify(const Dev& d, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_verify, dim3(cus), dim3(256), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_sset_clear(const Dev& d, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_sset_clear, dim3(cus * 4), dim3(256), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_slots_init(Slot* slots, uint32_t n, hipStream_t st) {
	hipLaunchKernelGGL(k_slots_init, dim3(grid_for(n, 256, 4096)), dim3(256), 0, st, slots, n);
	return hipGetLastError();
}
hipError_t launch_collect(const Slot* slots, uint32_t n, ebd_service* out, unsigned long long* cnt, hipStream_t st) {
	hipLaunchKernelGGL(k_collect, dim3(grid_for(n, 256, 4096)), dim3(256), 0, st, slots, n, out, cnt);
	return hipGetLastError();
}
hipError_t launch_gen_len(const GenTables* T, uint32_t config, uint64_t seed, uint64_t first, uint32_t n, uint32_t align,
		unsigned long long* alen, hipStream_t st) {
	hipLaunchKernelGGL(k_gen_len, dim3(grid_for(n, 256, 8192)), dim3(256), 0, st, T, config, (unsigned long long)seed,
			(unsigned long long)first, n, align, alen);
	return hipGetLastError();
}
hipError_t launch_gen_write(const GenTables* T, uint32_t config, uint64_t seed, uint64_t first, uint32_t n, EventRec* ev,
		uint32_t* len, const unsigned long long* off, uint8_t* payload, hipStream_t st) {
	hipLaunchKernelGGL(k_gen_write, dim3(grid_for(n, 256, 8192)), dim3(256), 0, st, T, config, (unsigned long long)seed,
			(unsigned long long)first, n, ev, len, off, payload);
	return hipGetLastError();
}

} // namespace ebd
