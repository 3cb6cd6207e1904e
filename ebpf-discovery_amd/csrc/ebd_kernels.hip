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

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef v4u v4u_a1 __attribute__((aligned(1)));
typedef unsigned long long u64a1 __attribute__((aligned(1)));
typedef unsigned int u32a1 __attribute__((aligned(1)));
// 8 bytes at any alignment: global_load_dwordx2 (gfx950 runs in unaligned-access mode)
__device__ __forceinline__ unsigned long long gload8u(const uint8_t* a) {
	return *(const __attribute__((address_space(1))) u64a1*)a;
}

// ---------------------------------------------------------------------------------
// Service table: open addressing on the 64-bit tag, 128-bit key verified.
//
// No lane ever waits for another lane's publication: a same-wave claimer whose publish
// sits on a divergent loop exit would be scheduled after the waiter (SIMT deadlock).
// A claimer CASes the tag and stores the second half; a finder compares the second half
// when it is already visible and otherwise queues (slot, hi) for k_verify, which runs
// after the inserting kernel.  A mismatch there is reported as EBD_ERR_COLLISION.
//
// First arrival (Aggregator.cpp:155-168: the request that creates a key fixes its domain
// and scheme): every request offers first = seq << 16 | isHttps << 15 | host length, and
// the slot keeps the minimum (atomicMin), so the earliest request's scheme and host/url
// split win.  The endpoint bytes are the same for every request of a key, so the claimer
// stores them (claim_publish) whoever arrives first.
// ---------------------------------------------------------------------------------
EBD_HD unsigned long long first_word(unsigned long long seq, bool https, uint32_t hl) {
	return (seq << 16) | ((unsigned long long)(https ? 1u : 0u) << 15) | (hl & 0x7fffu);
}

// Returns the slot (kNone when the table is full); *claimed: this call created the service.
// inc_int / inc_ext: the counter increments (one request: its class; a merged record: its counts).
__device__ uint32_t agg_insert(const Dev& d, Hash128 h, unsigned long long first, uint32_t inc_int, uint32_t inc_ext,
		bool* claimed) {
	uint32_t idx = (uint32_t)h.lo & d.slot_mask;
	bool found = false;
	*claimed = false;
	unsigned long long seen_first = 0;
	for (uint32_t probe = 0; probe <= d.slot_mask; probe++) {
		Slot* s = d.slots + idx;
		// One plain load pass over the slot's first 32 bytes.  tag and hi are written once
		// (0 -> value), first only decreases: a stale copy at worst shows 0 (resolved by
		// the CAS below, or the coherent re-read of hi) or a larger first (a redundant
		// atomicMin).  Slot words are only ever written by atomics here, so no dirty line
		// sits in L2 when the next kernel starts.
		const ulonglong2 th = *(const ulonglong2*)&s->tag;
		const ulonglong2 mo = *(const ulonglong2*)&s->first;
		seen_first = mo.x;
		unsigned long long t = th.x;
		if (t == 0) {
			t = atomicCAS(&s->tag, 0ull, h.lo);
			if (t == 0) {
				atomicExch(&s->hi, h.hi);
				*claimed = true;
				seen_first = ~0ull;
				found = true;
				break;
			}
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
		return kNone;
	}
	Slot* s = d.slots + idx;
	if (inc_int)
		atomicAdd(&s->internal_clients, inc_int);
	if (inc_ext)
		atomicAdd(&s->external_clients, inc_ext);
	if (first < seen_first)
		atomicMin(&s->first, first);
	return idx;
}

// Endpoint E = host + url as 8-byte words (ebd_spec.h endpoint_piece) to an 8-byte aligned
// destination: unaligned 8-byte loads (gfx950 runs in unaligned mode; sources are readable
// 8 bytes past their end), aligned stores.
__device__ __forceinline__ void copy_endpoint(unsigned long long* dst, const uint8_t* host, uint32_t hl, const uint8_t* url,
		uint32_t ul) {
	const uint32_t n = hl + ul;
	for (uint32_t oo = 0; oo < n; oo += 8) {
		const unsigned long long A = gload8u(host + (oo < hl ? oo : 0));
		const unsigned long long B = gload8u(url + ((oo > hl && oo - hl < ul) ? oo - hl : 0));
		dst[oo >> 3] = endpoint_piece(hl, n, oo, A, B);
	}
}

// The claimer of slot idx publishes the service's list entry, pid and endpoint bytes.
// list_at: its position in the claimed-slot list; ep_at: its (8-aligned) arena offset.
__device__ void claim_publish(const Dev& d, uint32_t idx, unsigned long long list_at, unsigned long long ep_at, uint32_t pid,
		const uint8_t* host, uint32_t hl, const uint8_t* url, uint32_t ul) {
	Slot* s = d.slots + idx;
	if (list_at < d.new_cap)
		d.new_slots[list_at] = idx;
	else
		set_error(d, EBD_ERR_TABLE_FULL);
	const uint32_t n = hl + ul;
	unsigned long long off = ~0ull;
	if (ep_at + n <= d.sarena_cap) {
		copy_endpoint((unsigned long long*)(d.sarena + ep_at), host, hl, url, ul);
		off = ep_at;
	} else {
		set_error(d, EBD_ERR_ARENA_FULL);
	}
	atomicExch(&s->ep_off, off);
	atomicExch((unsigned long long*)&s->pid, (unsigned long long)pid | ((unsigned long long)n << 32)); // pid, ep_len
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
// k_fresh: one lane per event, DFA table in LDS, events pulled from a workgroup queue.
//
// Memory layout decides this kernel's speed (tools/ubench_mem2.hip): buffers read a 64-B
// window at a time, the four lanes of a quad loading 64 contiguous bytes of one member's
// window per instruction (4 instructions = one window for each member), then a 4x4 block
// transpose inside the quad (DPP) hands every lane its own window.  Each workgroup owns a
// contiguous range of the batch and its lanes take the next event from an LDS counter when
// they finish one, so the chip streams the payload roughly in memory order and no lane waits
// for a longer neighbour.  The next window is loaded while the current one is scanned; it is
// predicted as "the same buffer's next window, or the lane's next event's first window", and
// a buffer that terminates early (POST body, invalid byte) costs one idle window.
//
// Chunks are event-relative (chunk c = bytes [16c, 16c + 16) of the buffer, unaligned loads):
// there is no leading skip.  The last chunk may extend past the buffer; the DFA steps over
// those bytes too, which can only change states at positions >= L: a terminal position >= L
// is an unfinished parse (fresh_finalize), and every other tracked position is < L.
//
// Per byte: one table step (v_mad_u32_u24 + ds_read_u8) and a running maximum; per chunk:
// the branch-free crossing trackers of ebd_fresh.h.  A lane that finishes a buffer appends
// its scan record to the wave's queue in LDS; 64 records are finalized together (rescans,
// spans, key), so the finalize code always runs on a full wave.
// ---------------------------------------------------------------------------------
// Logical index (s << 8) | b into the LDS image (ebd_dfa.h kLdsRow / lds_col).
struct LdsTable {
	const uint8_t* t;
	__device__ __forceinline__ uint32_t operator[](uint32_t i) const { return t[(i >> 8) * kLdsRow + lds_col(i & 0xffu)]; }
};

// One 16-byte chunk as 4 little-endian words.
struct Chunk {
	uint32_t w[4];
};

// 16-byte load through a global (not flat) pointer, any alignment: global_load_dwordx4
__device__ __forceinline__ Chunk gload16(uintptr_t a) {
	const v4u v = *(const __attribute__((address_space(1))) v4u_a1*)a;
	Chunk c;
	c.w[0] = v.x;
	c.w[1] = v.y;
	c.w[2] = v.z;
	c.w[3] = v.w;
	return c;
}

// Buffer access for fresh_finalize on the device: 4 and 8 bytes at any buffer offset.  Every
// offset it reads lies within the buffer's last 16-byte chunk, and the payload stays
// readable EBD_PAYLOAD_PAD bytes past each buffer (ebd_api.hip pads it).
struct DevMem {
	const uint8_t* p;
	__device__ __forceinline__ uint32_t ld4(uint32_t o) const { return *(const __attribute__((address_space(1))) u32a1*)(p + o); }
	__device__ __forceinline__ unsigned long long ld8(uint32_t o) const { return gload8u(p + o); }
};

constexpr int kFreshThreads = 1024;
constexpr int kFreshWaves = kFreshThreads / 64;
#ifndef EBD_SCAN_WAVES
#define EBD_SCAN_WAVES 12
#endif
constexpr int kScanWaves = EBD_SCAN_WAVES; // waves [0, kScanWaves) scan; the others finalize
#ifndef EBD_RING
#define EBD_RING 128
#endif
constexpr uint32_t kRing = EBD_RING; // finalize records in flight per workgroup (power of two)
#ifndef EBD_FINPER
#define EBD_FINPER 0
#endif
// records per finalize lane at a time (0: one record, finalized only by the lanes that hold one)
constexpr int kFinPer = EBD_FINPER > 0 ? EBD_FINPER : 1;

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
#if !defined(EBD_LDS_PLAIN) && !defined(EBD_LDS_COLPERM)
	return s * kLdsRow + __builtin_amdgcn_ubfe(wc, 8 * (k & 3), 8); // v_bfe + v_mad_u32_u24
#else
	return __builtin_amdgcn_perm(s, wc, 0x0c0c0400u | (uint32_t)(k & 3)); // (s << 8) | byte
#endif
}

// 16 DFA steps over one chunk: s advances, m = the maximum next state, qs = the states at
// the quarter starts (s0 | s4 << 8 | s8 << 16 | s12 << 24), qm = running maxima after 4, 8
// and 12 steps (ebd_fresh.h chunk_update).
__device__ __forceinline__ void scan_chunk(const uint8_t* T, const Chunk& w, uint32_t& s, uint32_t& m, uint32_t& qs,
		uint32_t& qm) {
	qs = s;
#ifdef EBD_EXP_MEMONLY // experiment: the loads without the DFA (results are wrong)
	m = w.w[0] ^ w.w[1] ^ w.w[2] ^ w.w[3];
	qm = 0;
	return;
#endif
	const uint32_t wc[4] = {lds_cols(w.w[0]), lds_cols(w.w[1]), lds_cols(w.w[2]), lds_cols(w.w[3])};
	m = 0;
#pragma unroll
	for (int k = 0; k < 16; k++) {
		s = T[tab_index(s, wc[k >> 2], k)];
		m = max(m, s); // pairs fold into v_max3
		if (k == 3) {
			qs |= s << 8;
			qm = m;
		} else if (k == 7) {
			qs |= s << 16;
			qm |= m << 8;
		} else if (k == 11) {
			qs |= s << 24;
			qm |= m << 16;
		}
	}
}

// quad_perm DPP: the value of `v` held by quad lane P's pattern
template <int P>
__device__ __forceinline__ uint32_t qperm(uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, P, 0xf, 0xf, true); }
constexpr int kQX2 = 2 | (3 << 2) | (0 << 4) | (1 << 6); // lane r takes lane r ^ 2
constexpr int kQX1 = 1 | (0 << 2) | (3 << 4) | (2 << 6); // lane r takes lane r ^ 1
template <int K>
__device__ __forceinline__ uint32_t qbcast(uint32_t v) { return qperm<K | (K << 2) | (K << 4) | (K << 6)>(v); }
template <int K>
__device__ __forceinline__ unsigned long long qbcast64(unsigned long long v) {
	return (unsigned long long)qbcast<K>((uint32_t)v) | ((unsigned long long)qbcast<K>((uint32_t)(v >> 32)) << 32);
}

// 4x4 transpose of 16-B blocks among the 4 lanes of a quad: lane r holds X[k] = piece r of
// member k's window; afterwards it holds piece k of its own window.
__device__ __forceinline__ void transpose_quad(Chunk (&X)[4], uint32_t r) {
	const bool lo2 = r < 2, lo1 = (r & 1) == 0;
#pragma unroll
	for (int k = 0; k < 2; k++)
#pragma unroll
		for (int d = 0; d < 4; d++) {
			const uint32_t recv = qperm<kQX2>(lo2 ? X[k + 2].w[d] : X[k].w[d]);
			X[k + 2].w[d] = lo2 ? recv : X[k + 2].w[d];
			X[k].w[d] = lo2 ? X[k].w[d] : recv;
		}
#pragma unroll
	for (int k = 0; k < 4; k += 2)
#pragma unroll
		for (int d = 0; d < 4; d++) {
			const uint32_t recv = qperm<kQX1>(lo1 ? X[k + 1].w[d] : X[k].w[d]);
			X[k + 1].w[d] = lo1 ? recv : X[k + 1].w[d];
			X[k].w[d] = lo1 ? X[k].w[d] : recv;
		}
}

// An event as a lane holds it.  kind: EK_PARSE (a buffer to scan), EK_SKIP (no parse:
// not NEW_DATA or the saved buffer is missing, Discovery.cpp:99-110), EK_BAD (length or
// offset out of range), EK_NONE (the workgroup's range is exhausted).
enum : uint32_t { EK_PARSE = 0, EK_SKIP = 1, EK_BAD = 2, EK_NONE = 3 };
struct LaneEv {
	uint32_t idx;
	uint32_t L;       // buffer length (0 unless EK_PARSE)
	uint32_t kind;
	uint32_t pf;      // pid (the DiscoveryEvent's, Discovery.cpp:136, 157)
	uint32_t flags;
	const uint8_t* p; // buffer (a harmless valid address unless EK_PARSE)
};

__device__ __forceinline__ LaneEv lane_ev(const Dev& d, uint32_t i, uint32_t end) {
	LaneEv e;
	e.idx = i;
	if (i >= end) {
		e.kind = EK_NONE;
		e.L = 0;
		e.pf = e.flags = 0;
		e.p = d.payload;
		return e;
	}
	const uint8_t* evb = (const uint8_t*)(d.ev + i);
	const uint32_t flags = evb[32];
	e.pf = *(const uint32_t*)evb;
	e.flags = flags;
#ifdef EBD_EXP_L2ONLY // experiment: every event parses one of the first 4096 buffers (L2-resident)
	const uint32_t L = d.len[i & 4095];
	const uint64_t off = d.off[i & 4095];
#else
	const uint32_t L = d.len[i];
	const uint64_t off = d.off[i];
#endif
	e.kind = !(flags & FLAG_NEW) || L == EBD_NO_BUFFER ? EK_SKIP : (L > EBD_BUFFER_MAX_DATA_SIZE || off >> 48) ? EK_BAD : EK_PARSE;
	e.L = e.kind == EK_PARSE ? L : 0;
	e.p = e.kind == EK_PARSE ? d.payload + off : d.payload;
	return e;
}

// A finished scan waiting for fresh_finalize (64 B).
struct FinRec {
	unsigned long long pl; // buffer address (bits 0..47) | L << 48
	uint32_t idx, pid;
	uint32_t sf;  // final state | flags << 8 | cseen << 16 | post << 17
	uint32_t cqm;
	uint32_t c01; // url.c | host.c << 16
	uint32_t c23; // hend.c | cip.c << 16
	uint32_t c4;  // term.c
	uint32_t qs[5];
	uint32_t pad[2];
};
static_assert(sizeof(FinRec) == 64, "finalize record is 64 bytes");

__device__ __forceinline__ void write_none(const Dev& d, uint32_t i) {
	ebd_event_result r;
	r.consumed = 0;
	r.status = EBD_STATUS_NONE;
	r.info = 0;
	r.u.session.index = 0;
	r.u.session.pad_[0] = r.u.session.pad_[1] = 0;
	d.res[i] = r;
}

// A NEW_DATA event with an empty buffer: a fresh parser consumes nothing and is left
// unfinished, so the session may be saved (Discovery.cpp:141-159).
__device__ __forceinline__ void write_empty(const Dev& d, uint32_t i) {
	ebd_event_result r;
	r.consumed = 0;
	r.status = EBD_STATUS_UNFINISHED;
	r.info = 0;
	r.u.span.url_off = r.u.span.url_len = r.u.span.host_off = r.u.span.host_len = r.u.span.cip_off = r.u.span.cip_len = 0;
	d.res[i] = r;
	const EventRec& ev = d.ev[i];
	atomicAdd(&d.ctr[CTR_UNFINISHED], 1ull);
	sset_insert(d, ev.pid, ev.fd, ev.sessionID, 0);
}

// fresh_finalize for N records per lane, its steps interleaved so that the records' memory
// round trips overlap: the quarter bytes of every record, then spans, then the endpoint
// pieces of every record, 64 bytes of each per round trip.  have[n]: record n is real.
template <int N>
__device__ __forceinline__ void finalize_recs(const Dev& d, const uint8_t* T, const FinRec (&q)[N], const bool (&have)[N]) {
	const DfaInfo& di = d.di;
	ScanRec sr[N];
	FinLoads f[N];
	const uint8_t* p[N];
	uint32_t L[N];
#pragma unroll
	for (int n = 0; n < N; n++) {
		p[n] = have[n] ? (const uint8_t*)(uintptr_t)(q[n].pl & 0xffffffffffffull) : d.payload;
		L[n] = have[n] ? (uint32_t)(q[n].pl >> 48) : 0;
		sr[n].url = Trk{q[n].c01 & 0xffffu, q[n].qs[0]};
		sr[n].host = Trk{q[n].c01 >> 16, q[n].qs[1]};
		sr[n].hend = Trk{q[n].c23 & 0xffffu, q[n].qs[2]};
		sr[n].cip = Trk{q[n].c23 >> 16, q[n].qs[3]};
		sr[n].term = Trk{q[n].c4, q[n].qs[4]};
		sr[n].cqm = q[n].cqm;
		sr[n].cseen = (q[n].sf >> 16) & 1u;
		if (!have[n])
			rec_init(di, sr[n]); // loads at offset 0 of a valid address
		fresh_loads(di, sr[n], DevMem{p[n]}, f[n]);
	}
	FreshResult fr[N];
#pragma unroll
	for (int n = 0; n < N; n++)
		fresh_spans(LdsTable{T}, di, sr[n], q[n].sf & 0xffu, ((q[n].sf >> 17) & 1u) != 0, f[n], L[n], (uint8_t)(q[n].sf >> 8), fr[n]);
	// keys (ebd_spec.h endpoint_key, groups of 8 pieces, all records' loads issued together)
	constexpr uint32_t kGroup = 8;
	KeyHasher kh[N];
	uint32_t hs[N], hl[N], us[N], ul[N], en[N], nmax = 0;
#pragma unroll
	for (int n = 0; n < N; n++) {
		const bool k = have[n] && fr[n].keyed;
		hs[n] = k ? fr[n].r.u.span.host_off : 0;
		hl[n] = k ? fr[n].r.u.span.host_len : 0;
		us[n] = k ? fr[n].r.u.span.url_off : 0;
		ul[n] = k ? fr[n].r.u.span.url_len : 0;
		en[n] = hl[n] + ul[n];
		nmax = max(nmax, en[n]);
		kh[n].init(d.hkey, q[n].pid);
	}
	for (uint32_t g = 0; g < nmax; g += 8 * kGroup) {
		uint64_t A[N][kGroup], B[N][kGroup];
#pragma unroll
		for (int n = 0; n < N; n++)
#pragma unroll
			for (uint32_t k = 0; k < kGroup; k++) {
				const uint32_t oo = g + 8 * k;
				A[n][k] = gload8u(p[n] + hs[n] + (oo < hl[n] ? oo : 0));
				B[n][k] = gload8u(p[n] + us[n] + ((oo > hl[n] && oo - hl[n] < ul[n]) ? oo - hl[n] : 0));
			}
#pragma unroll
		for (int n = 0; n < N; n++)
#pragma unroll
			for (uint32_t k = 0; k < kGroup; k++) {
				const uint32_t oo = g + 8 * k;
				if (oo < en[n])
					kh[n].word(endpoint_piece(hl[n], en[n], oo, A[n][k], B[n][k]));
			}
	}
#pragma unroll
	for (int n = 0; n < N; n++) {
		if (!have[n])
			continue;
		const uint32_t i = q[n].idx;
		if (fr[n].r.status == EBD_STATUS_FINISHED) {
#ifdef EBD_EXP_NOHASH // experiment: finalize without the key (results are wrong)
			d.keys[i] = Hash128{en[n], 1};
#else
			d.keys[i] = kh[n].finish_words(en[n]);
#endif
		} else if (fr[n].r.status == EBD_STATUS_UNFINISHED) {
			// the session may be saved (Discovery.cpp:148-150): sequential path
			const EventRec& ev = d.ev[i];
			atomicAdd(&d.ctr[CTR_UNFINISHED], 1ull);
			sset_insert(d, ev.pid, ev.fd, ev.sessionID, 0);
		}
		d.res[i] = fr[n].r;
	}
}

// Leading buffer bytes a scan record carries in LDS (window 0 and half of window 1), so that
// finalize reads the request line and usually the Host header from LDS instead of reloading
// lines that left L2 while the lane scanned the rest of the buffer.
#ifndef EBD_STAGE
#define EBD_STAGE 64
#endif
constexpr uint32_t kStage = EBD_STAGE;
static_assert(kStage == 0 || kStage == 64 || kStage == 96 || kStage == 128, "whole or half windows");

// Buffer bytes for fresh_finalize: offsets [0, lim) from the staged LDS copy `s` (4-B aligned,
// readable 4 bytes past lim), the rest from the buffer in global memory.
struct StagedMem {
	const uint8_t* p;
	const uint32_t* s;
	uint32_t lim;
	__device__ __forceinline__ uint32_t lds4(uint32_t o) const {
		return __builtin_amdgcn_alignbyte(s[(o >> 2) + 1], s[o >> 2], o & 3u);
	}
	__device__ __forceinline__ uint32_t ld4(uint32_t o) const {
		if (o + 4 <= lim)
			return lds4(o);
		return *(const __attribute__((address_space(1))) u32a1*)(p + o);
	}
	__device__ __forceinline__ unsigned long long ld8(uint32_t o) const {
		if (o + 8 <= lim)
			return (unsigned long long)lds4(o) | ((unsigned long long)lds4(o + 4) << 32);
		return gload8u(p + o);
	}
};

// fresh_finalize for one record (ebd_fresh.h), run only by the lanes that hold one.  `stage`:
// the record's staged leading bytes (pad[0] of the record = how many are valid).
template <typename Mem>
__device__ __forceinline__ void finalize_rec(const Dev& d, const uint8_t* T, const FinRec& q, const Mem& mem) {
	const uint8_t* p = (const uint8_t*)(uintptr_t)(q.pl & 0xffffffffffffull);
	(void)p; // used by the debug builds below
	const uint32_t L = (uint32_t)(q.pl >> 48);
	const uint32_t i = q.idx;
#ifdef EBD_DBG_CHECK2 // debug build: a record that cannot be real raises bit 60 and is dropped
	if (p < d.payload || p >= d.payload + (1ull << 36) || L > EBD_BUFFER_MAX_DATA_SIZE || i >= d.n) {
		atomicOr(&d.ctr[CTR_ERRORS], 1ull << 60);
		return;
	}
#endif
#ifdef EBD_DBG_CHECK // debug build: a record that cannot be real is reported and dropped
	if (p < d.payload || p >= d.payload + (1ull << 36) || L > EBD_BUFFER_MAX_DATA_SIZE || i >= d.n) {
		printf("EBD_DBG fin: block %u thread %u idx %u n %u L %u p-payload %lld c4 %u sf %x\n", blockIdx.x, threadIdx.x, i, d.n,
				L, (long long)(p - d.payload), q.c4, q.sf);
		return;
	}
#endif
	ScanRec sr;
	sr.url = Trk{q.c01 & 0xffffu, q.qs[0]};
	sr.host = Trk{q.c01 >> 16, q.qs[1]};
	sr.hend = Trk{q.c23 & 0xffffu, q.qs[2]};
	sr.cip = Trk{q.c23 >> 16, q.qs[3]};
	sr.term = Trk{q.c4, q.qs[4]};
	sr.cqm = q.cqm;
	sr.cseen = (q.sf >> 16) & 1u;
	FreshResult fr;
#ifdef EBD_DBG_CHECK
	{
		FinLoads f;
		fresh_loads(d.di, sr, DevMem{p}, f);
		fresh_spans(LdsTable{T}, d.di, sr, q.sf & 0xffu, ((q.sf >> 17) & 1u) != 0, f, L, (uint8_t)(q.sf >> 8), fr);
		const auto& sp = fr.r.u.span;
		if (fr.keyed && (sp.host_off + sp.host_len > L || sp.url_off + sp.url_len > L)) {
			printf("EBD_DBG span: idx %u L %u host %u+%u url %u+%u\n", i, L, sp.host_off, sp.host_len, sp.url_off, sp.url_len);
			return;
		}
		if (16 * sr.term.c >= L + 16 || 16 * sr.url.c >= L + 16 || 16 * sr.host.c >= L + 16 || 16 * sr.cip.c >= L + 16) {
			printf("EBD_DBG trk: idx %u L %u term %u url %u host %u cip %u\n", i, L, sr.term.c, sr.url.c, sr.host.c, sr.cip.c);
			return;
		}
	}
#endif
	fresh_finalize(LdsTable{T}, d.di, sr, q.sf & 0xffu, ((q.sf >> 17) & 1u) != 0, mem, L, d.hkey, q.pid, (uint8_t)(q.sf >> 8), fr);
	if (fr.r.status == EBD_STATUS_FINISHED) {
		d.keys[i] = fr.key;
	} else if (fr.r.status == EBD_STATUS_UNFINISHED) {
		// the session may be saved (Discovery.cpp:148-150): sequential path
		const EventRec& ev = d.ev[i];
		atomicAdd(&d.ctr[CTR_UNFINISHED], 1ull);
		sset_insert(d, ev.pid, ev.fd, ev.sessionID, 0);
	}
	d.res[i] = fr.r;
}

__device__ __forceinline__ uint32_t lds_load_acq(const uint32_t* p) {
	return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store_rel(uint32_t* p, uint32_t v) {
	__hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Workgroup state shared by the scan and finalize waves.
struct FreshShared {
	FinRec ring[kRing];
	uint32_t ready[kRing]; // position + 1 once ring[pos % kRing] is written
	uint32_t freed[kRing]; // position + 1 once ring[pos % kRing] is finalized
#if EBD_STAGE
	uint32_t rdata[kRing * (kStage / 4) + 4];      // staged leading bytes of ring[slot] (+4: lds4 slack)
	uint32_t stage[kScanWaves * 64 * (kStage / 4)]; // a scan lane's current buffer, as scanned
	uint32_t fstage[(kFreshWaves - kScanWaves) * 64 * (kStage / 4) + 4]; // a finalize lane's record's bytes
#endif
	uint32_t next_ev;      // next event of the workgroup's range
	uint32_t tail;         // positions handed out to scan lanes
	uint32_t claim;        // positions handed out to finalize waves
	uint32_t scan_done;    // scan waves that finished
};

__global__ __launch_bounds__(kFreshThreads) void k_fresh(Dev d) {
	// static LDS: the table sits at LDS address 0, so a step's index is its address
	__shared__ __attribute__((aligned(16))) uint8_t T[kLdsTableBytes];
	__shared__ FreshShared sh;
	const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 3;
	// this workgroup's contiguous share of the batch
	const uint32_t per = (uint32_t)(((unsigned long long)d.n + gridDim.x - 1) / gridDim.x);
	const uint32_t rb = min(d.n, blockIdx.x * per), re = min(d.n, rb + per);
	for (uint32_t k = threadIdx.x * 16u; k < kLdsTableBytes; k += kFreshThreads * 16u)
		*(uint4*)(T + k) = *(const uint4*)(d.dfa + k);
	for (uint32_t k = threadIdx.x; k < kRing; k += kFreshThreads)
		sh.ready[k] = sh.freed[k] = 0;
	if (threadIdx.x == 0) {
		sh.next_ev = rb + kScanWaves * 64 * 2;
		sh.tail = sh.claim = sh.scan_done = 0;
	}
	__syncthreads();
	const DfaInfo& di = d.di;

	if (wave >= kScanWaves) {
		// ---- finalize waves: kFinPer x 64 records at a time, in position order ----
		for (;;) {
			uint32_t c = 0;
			if (lane == 0)
				c = atomicAdd(&sh.claim, 64u * kFinPer);
			c = __builtin_amdgcn_readfirstlane(c);
			FinRec q[kFinPer];
			bool have[kFinPer];
#pragma unroll
			for (int j = 0; j < kFinPer; j++) {
				const uint32_t pos = c + 64 * j + lane, slot = pos & (kRing - 1);
				have[j] = false;
				for (;;) {
					if (lds_load_acq(&sh.ready[slot]) == pos + 1) {
						have[j] = true;
						break;
					}
					if (lds_load_acq(&sh.scan_done) == (uint32_t)kScanWaves && pos >= lds_load_acq(&sh.tail))
						break;
					__builtin_amdgcn_s_sleep(2);
				}
				if (have[j]) {
					q[j] = sh.ring[slot];
#if EBD_STAGE && EBD_FINPER == 0
					{ // the staged bytes move to this lane's row, so the slot is free at once
						const uint4* src = (const uint4*)(sh.rdata + slot * (kStage / 4));
						uint4* dst = (uint4*)(sh.fstage + ((wave - kScanWaves) * 64 + lane) * (kStage / 4));
#pragma unroll
						for (uint32_t k = 0; k < kStage / 16; k++)
							dst[k] = src[k];
					}
#endif
					lds_store_rel(&sh.freed[slot], pos + 1);
				} else {
					q[j] = FinRec{};
				}
			}
			if (!__any(have[0]))
				break;
#ifndef EBD_EXP_NOFIN // experiment: scan without finalize (results are wrong)
#if EBD_FINPER == 0
			if (have[0]) {
#if EBD_STAGE
				finalize_rec(d, T, q[0], StagedMem{(const uint8_t*)(uintptr_t)(q[0].pl & 0xffffffffffffull),
						sh.fstage + ((wave - kScanWaves) * 64 + lane) * (kStage / 4), q[0].pad[0]});
#else
				finalize_rec(d, T, q[0], DevMem{(const uint8_t*)(uintptr_t)(q[0].pl & 0xffffffffffffull)});
#endif
			}
#else
			finalize_recs<kFinPer>(d, T, q, have);
#endif
#endif
		}
		return;
	}

	// ---- scan waves ----
	const uint32_t sl = wave * 64 + lane; // scan lane
	constexpr uint32_t kScanLanes = kScanWaves * 64;
	auto grab = [&]() -> uint32_t { return atomicAdd(&sh.next_ev, 1u); };
	// the lane's current event (e0) and the next one (e1, whose record arrives early)
	LaneEv e0 = lane_ev(d, rb + sl, re);
	LaneEv e1 = lane_ev(d, rb + kScanLanes + sl, re);
	uint32_t w0 = 0; // e0's window to scan next
	uint32_t s = di.init, live = 0, post = 0;
	ScanRec sr;
	rec_init(di, sr);

	// Hands e0's scan record to the finalize waves when `done`.
	auto push = [&](bool done) {
		const unsigned long long b = __ballot(done);
		if (b == 0)
			return;
		uint32_t base = 0;
		if (lane == 0)
			base = atomicAdd(&sh.tail, (uint32_t)__popcll(b));
		base = __builtin_amdgcn_readfirstlane(base);
		if (done) {
			const uint32_t pos = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0));
			const uint32_t slot = pos & (kRing - 1);
			if (pos >= kRing) // the slot's previous record must have been taken
				while (lds_load_acq(&sh.freed[slot]) != pos - kRing + 1)
					__builtin_amdgcn_s_sleep(1);
			FinRec t;
#if EBD_STAGE
			{ // staged bytes equal the buffer's up to the scanned windows and the last chunk's end
				const uint4* src = (const uint4*)(sh.stage + sl * (kStage / 4));
				uint4* dst = (uint4*)(sh.rdata + slot * (kStage / 4));
#pragma unroll
				for (uint32_t k = 0; k < kStage / 16; k++)
					dst[k] = src[k];
				const uint32_t scanned = min(64u * w0, kStage), chunks_end = (e0.L + 15u) & ~15u;
				t.pad[0] = min(scanned, chunks_end);
			}
#else
			t.pad[0] = 0;
#endif
			t.pl = (unsigned long long)(uintptr_t)e0.p | ((unsigned long long)e0.L << 48);
			t.idx = e0.idx;
			t.pid = e0.pf;
			t.sf = s | (e0.flags << 8) | (sr.cseen << 16) | (post << 17);
			t.cqm = sr.cqm;
			t.c01 = sr.url.c | (sr.host.c << 16);
			t.c23 = sr.hend.c | (sr.cip.c << 16);
			t.c4 = sr.term.c;
			t.qs[0] = sr.url.qs;
			t.qs[1] = sr.host.qs;
			t.qs[2] = sr.hend.qs;
			t.qs[3] = sr.cip.qs;
			t.qs[4] = sr.term.qs;
			t.pad[1] = 0;
			sh.ring[slot] = t;
			lds_store_rel(&sh.ready[slot], pos + 1);
		}
	};
	// Moves on while e0 needs no scan: such events are resolved here.
	auto resolve = [&]() {
		for (;;) {
			if (e0.kind == EK_SKIP) {
				write_none(d, e0.idx);
			} else if (e0.kind == EK_BAD) {
				set_error(d, EBD_ERR_BAD_INPUT);
				write_none(d, e0.idx);
			} else if (e0.kind == EK_PARSE && e0.L == 0) {
				write_empty(d, e0.idx);
			} else {
				break;
			}
			e0 = e1;
			e1 = lane_ev(d, grab(), re);
		}
		w0 = 0;
		s = di.init;
		post = 0;
		rec_init(di, sr);
		live = e0.kind == EK_PARSE ? 1u : 0u;
	};
	resolve();

	// The window in flight: (tidx, tw) names what W holds for this lane.
	auto nwin = [](uint32_t L) { return (L + 63) >> 6; };
	Chunk W[4];
	uint32_t tidx, tw;
	auto issue = [&](const uint8_t* p, uint32_t L, uint32_t w) {
		// member k's window: pieces p + 16 * min(4w + j, last), j = 0..3; this lane loads piece r
		const uint32_t last = L ? (L - 1) >> 4 : 0;
		const unsigned long long a = (unsigned long long)(uintptr_t)p;
		const uint32_t pc = (w << 2) | (last << 16); // window's first chunk | last chunk
		unsigned long long ak[4];
		uint32_t pk[4];
#ifdef EBD_BPERM_ADDR // experiment: quad broadcast through ds_bpermute instead of DPP
		{
			const int qb = (int)((threadIdx.x & 63u) & ~3u) * 4;
#pragma unroll
			for (int k = 0; k < 4; k++) {
				const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(qb + 4 * k, (int)(uint32_t)a);
				const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(qb + 4 * k, (int)(uint32_t)(a >> 32));
				ak[k] = (unsigned long long)lo | ((unsigned long long)hi << 32);
				pk[k] = (uint32_t)__builtin_amdgcn_ds_bpermute(qb + 4 * k, (int)pc);
			}
		}
#else
		ak[0] = qbcast64<0>(a), pk[0] = qbcast<0>(pc);
		ak[1] = qbcast64<1>(a), pk[1] = qbcast<1>(pc);
		ak[2] = qbcast64<2>(a), pk[2] = qbcast<2>(pc);
		ak[3] = qbcast64<3>(a), pk[3] = qbcast<3>(pc);
#endif
#pragma unroll
		for (int k = 0; k < 4; k++) {
			const uint32_t c = min((pk[k] & 0xffffu) + r, pk[k] >> 16);
#ifdef EBD_DBG_CHECK2
			if (ak[k] - (uintptr_t)d.payload >= (1ull << 36)) {
				atomicOr(&d.ctr[CTR_ERRORS], 1ull << 61);
				ak[k] = (uintptr_t)d.payload;
			}
#endif
#ifdef EBD_DBG_CHECK
			if (ak[k] < (uintptr_t)d.payload || ak[k] >= (uintptr_t)d.payload + (1ull << 36)) {
				printf("EBD_DBG issue: block %u thread %u k %d a-payload %lld c %u\n", blockIdx.x, threadIdx.x, k,
						(long long)(ak[k] - (uintptr_t)d.payload), c);
				ak[k] = (uintptr_t)d.payload;
			}
#endif
			W[k] = gload16((uintptr_t)(ak[k] + 16ull * c));
		}
	};
	tidx = e0.idx;
	tw = 0;
	issue(e0.p, e0.L, 0);

	while (__any(e0.kind != EK_NONE)) {
		// is the window in flight the one e0 needs?
		const bool valid = e0.kind == EK_PARSE && tidx == e0.idx && tw == w0;
		Chunk X[4] = {W[0], W[1], W[2], W[3]};
		// predict and load the next window
		{
			const uint8_t* np;
			uint32_t nL, ni, nw;
			if (!valid) {
				np = e0.p, nL = e0.L, ni = e0.idx, nw = w0;
			} else if (w0 + 1 < nwin(e0.L)) {
				np = e0.p, nL = e0.L, ni = e0.idx, nw = w0 + 1;
			} else {
				np = e1.p, nL = e1.L, ni = e1.idx, nw = 0;
			}
			issue(np, nL, nw);
			tidx = ni;
			tw = nw;
		}
		transpose_quad(X, r);
		bool done = false;
		if (valid) {
			if (w0 == 0)
				post = (X[0].w[0] & 0xffu) == 'P' ? 1u : 0u;
#if EBD_STAGE
			if (64 * w0 < kStage) { // this window's chunks into the lane's staging row
				uint4* st = (uint4*)(sh.stage + sl * (kStage / 4)) + 4 * w0;
#pragma unroll
				for (int k = 0; k < 4; k++)
					if (64 * w0 + 16 * k < kStage)
						st[k] = make_uint4(X[k].w[0], X[k].w[1], X[k].w[2], X[k].w[3]);
			}
#endif
#pragma unroll
			for (int k = 0; k < 4; k++) {
				uint32_t sx = s, m, qs, qm;
				scan_chunk(T, X[k], sx, m, qs, qm);
				if (live) {
					const uint32_t c = 4 * w0 + k;
					chunk_update(di, sr, c, s, qs, qm, m);
					live = !st_terminal(di, sx) && 16 * (c + 1) < e0.L ? 1u : 0u;
					s = sx;
				}
			}
			w0++;
			done = !live;
		}
		push(done);
		if (done) {
			e0 = e1;
			e1 = lane_ev(d, grab(), re);
			resolve();
		}
	}
	if (lane == 0)
		atomicAdd(&sh.scan_done, 1u);
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
	kh.init(d.hkey, ev.pid);
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
	bool claimed;
	const uint32_t slot = agg_insert(d, kh.finish(), first_word(d.seq_base + i, (g.f & GPF_HTTPS) != 0, hl),
			cls == CLS_INTERNAL, cls == CLS_EXTERNAL, &claimed);
	if (claimed) // a rare path: one reservation per claim
		claim_publish(d, slot, atomicAdd(&d.ctr[CTR_SERVICES], 1ull),
				atomicAdd(&d.ctr[CTR_SARENA], (unsigned long long)((hl + ul + 7u) & ~7u)), ev.pid, dst, hl, dst + hl, ul);
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

// Aggregator::newRequest for the fast-path requests (coalesced reads of the results, keys
// and events).  The client class comes from the client-IP header's front token when k_fresh
// found one (cip_classify), else from the session's source address (Aggregator.cpp:60-66,
// 85-88).  A block walks a contiguous range of the batch 256 events at a time.  Requests
// with a client-IP header (~30 % in config 3) are queued in LDS and parsed kAggThreads at a
// time, so the token parse, the longest code path, runs on full waves instead of on the
// few lanes of each wave that have one.  Aggregation is order-free (counters, atomicMin of
// the first-arrival word), so queueing does not change the result.  Services created in a
// step reserve their list entries and arena bytes with one global atomic per block and step
// (a single hot counter serialises at ~12 ns per atomic); requests are counted per block.
constexpr uint32_t kCipQueue = 2 * kAggThreads;

// A service this thread created in the current step, waiting for its reservations.
struct PendingClaim {
	uint32_t slot, pid, hl, ul, li;
	unsigned long long ab;
	const uint8_t *host, *url;
};

struct AggShared {
	uint32_t q[kCipQueue]; // queued client-IP requests
	uint32_t qn;
	uint32_t cn;           // claims of this step (list entries)
	unsigned long long cb; // their arena bytes
	unsigned long long list_base, arena_base;
	unsigned long long nreq;
};

__device__ __forceinline__ void agg_request(const Dev& d, uint32_t i, const ebd_event_result& r, uint32_t cls, AggShared& sh,
		PendingClaim& pc, bool& has) {
	bool claimed;
	const Hash128 key = d.keys[i];
	const uint32_t slot = agg_insert(d, key, first_word(d.seq_base + i, (r.info & EBD_INFO_HTTPS) != 0, r.u.span.host_len),
			cls == CLS_INTERNAL, cls == CLS_EXTERNAL, &claimed);
	if (claimed) {
		const uint8_t* p = d.payload + d.off[i];
		pc.slot = slot;
		pc.pid = d.ev[i].pid;
		pc.host = p + r.u.span.host_off;
		pc.hl = r.u.span.host_len;
		pc.url = p + r.u.span.url_off;
		pc.ul = r.u.span.url_len;
		pc.li = atomicAdd(&sh.cn, 1u);
		pc.ab = atomicAdd(&sh.cb, (unsigned long long)((pc.hl + pc.ul + 7u) & ~7u));
		has = true;
	}
}

__device__ __forceinline__ void agg_cip_one(const Dev& d, uint32_t i, uint8_t* row, AggShared& sh, PendingClaim& pc, bool& has) {
	ebd_event_result r = d.res[i];
	const uint32_t cls = cip_classify(d, i, r, row);
	r.info = (uint8_t)((r.info & ~(3u << EBD_INFO_CLASS_SHIFT)) | (cls << EBD_INFO_CLASS_SHIFT));
	d.res[i] = r;
	agg_request(d, i, r, cls, sh, pc, has);
}

__global__ __launch_bounds__(kAggThreads) void k_agg_fast(Dev d) {
	__shared__ __attribute__((aligned(8))) uint8_t rows[kAggThreads * kCipStride];
	__shared__ AggShared sh;
	uint8_t* row = rows + threadIdx.x * kCipStride;
	if (threadIdx.x == 0) {
		sh.nreq = 0;
		sh.qn = 0;
		sh.cn = 0;
		sh.cb = 0;
	}
	__syncthreads();
	uint32_t cnt = 0;
	const uint32_t steps = (d.n + kAggThreads - 1) / kAggThreads;
	const uint32_t per = (steps + gridDim.x - 1) / gridDim.x;
	const uint32_t s0 = min(steps, blockIdx.x * per), s1 = min(steps, s0 + per);
	for (uint32_t st = s0; st < s1; st++) { // uniform trip count: the barriers below are safe
		PendingClaim pc[2];
		bool has[2] = {false, false};
		const uint32_t i = st * kAggThreads + threadIdx.x;
		if (i < d.n) {
			ebd_event_result r = d.res[i];
			if (r.status == EBD_STATUS_FINISHED && !(r.info & EBD_INFO_SESSION)) {
				cnt++;
				if (r.info & EBD_INFO_CIP) {
					sh.q[atomicAdd(&sh.qn, 1u)] = i;
				} else {
					const uint8_t* evb = (const uint8_t*)(d.ev + i);
					const v4u sv = *(const __attribute__((address_space(1))) v4u*)(evb + 16); // sourceIP (4-B aligned)
					uint8_t src[16];
					__builtin_memcpy(src, &sv, 16);
					const uint32_t cls = classify_source(*d.ifs, evb[32], src);
					r.info = (uint8_t)((r.info & ~(3u << EBD_INFO_CLASS_SHIFT)) | (cls << EBD_INFO_CLASS_SHIFT));
					d.res[i] = r;
					agg_request(d, i, r, cls, sh, pc[0], has[0]);
				}
			}
		}
		__syncthreads();
		const uint32_t m = sh.qn; // < kCipQueue: below kAggThreads before this step, + at most kAggThreads
		__syncthreads();          // every thread has read qn before a push or the drain changes it
		const bool last = st + 1 == s1;
		if (m >= kAggThreads || (last && m > 0)) { // full waves; the block's last step drains the rest
			if (threadIdx.x < min(m, (uint32_t)kAggThreads))
				agg_cip_one(d, sh.q[threadIdx.x], row, sh, pc[1], has[1]);
			__syncthreads();
			if (m >= kAggThreads && threadIdx.x < m - kAggThreads) // [kAggThreads, m) -> [0, m - kAggThreads)
				sh.q[threadIdx.x] = sh.q[kAggThreads + threadIdx.x];
			if (threadIdx.x == 0)
				sh.qn = m >= kAggThreads ? m - kAggThreads : 0;
		}
		__syncthreads();
		// this step's claims: one reservation of list entries and arena bytes for the block
		if (threadIdx.x == 0) {
			const uint32_t cn = sh.cn;
			if (cn) {
				sh.list_base = atomicAdd(&d.ctr[CTR_SERVICES], (unsigned long long)cn);
				sh.arena_base = atomicAdd(&d.ctr[CTR_SARENA], sh.cb);
			}
			sh.cn = 0;
			sh.cb = 0;
		}
		__syncthreads();
#pragma unroll
		for (int k = 0; k < 2; k++)
			if (has[k])
				claim_publish(d, pc[k].slot, sh.list_base + pc[k].li, sh.arena_base + pc[k].ab, pc[k].pid, pc[k].host, pc[k].hl,
						pc[k].url, pc[k].ul);
		__syncthreads(); // list_base / arena_base are read before the next step's reservation
	}
	atomicAdd(&sh.nreq, (unsigned long long)cnt);
	__syncthreads();
	if (threadIdx.x == 0 && sh.nreq)
		atomicAdd(&d.ctr[CTR_REQUESTS], sh.nreq);
}

__global__ void k_verify(Dev d) {
	const unsigned long long nv = d.ctr[CTR_VERIFY];
	const uint32_t n = (uint32_t)(nv < d.verify_cap ? nv : d.verify_cap);
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x)
		if (d.slots[d.verify[k].slot].hi != d.verify[k].hi)
			set_error(d, EBD_ERR_COLLISION);
}

__device__ __forceinline__ Slot empty_slot() {
	Slot s;
	s.tag = 0;
	s.hi = 0;
	s.first = ~0ull;
	s.ep_off = 0;
	s.pid = 0;
	s.ep_len = 0;
	s.internal_clients = 0;
	s.external_clients = 0;
	s.pad[0] = s.pad[1] = s.pad[2] = s.pad[3] = 0;
	return s;
}

// Aggregator::clear (Aggregator.cpp:136-153): every claimed slot back to empty.
__global__ void k_clear_used(const unsigned int* used, const unsigned long long* ctr, Slot* slots) {
	const unsigned long long n = ctr[CTR_SERVICES];
	for (unsigned long long k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x)
		slots[used[k]] = empty_slot();
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
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x)
		slots[k] = empty_slot();
}

// Aggregator::collectServices (Aggregator.cpp:170-181) over the claimed-slot list.  Domain
// and scheme come from the first-arrival word (the earliest request's host length and
// isHttps, Aggregator.cpp:112-130): the domain is "[...]" through the first ']' after the
// host's first '[' (empty without one), else the host up to its first ':'.
__global__ void k_collect(const Slot* slots, const unsigned int* used, const unsigned long long* ctr, const uint8_t* arena,
		ebd_service* out) {
	const unsigned long long n = ctr[CTR_SERVICES];
	for (unsigned long long k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const Slot& s = slots[used[k]];
		const uint32_t hl = (uint32_t)(s.first & 0x7fffu);
		uint32_t doff = 0, dlen = 0;
		if (s.ep_off != ~0ull)
			host_domain(arena + s.ep_off, hl, &doff, &dlen);
		ebd_service v;
		v.pid = s.pid;
		v.internal_clients = s.internal_clients;
		v.external_clients = s.external_clients;
		v.https = (uint8_t)((s.first >> 15) & 1u);
		v.pad_[0] = v.pad_[1] = v.pad_[2] = 0;
		v.endpoint_off = s.ep_off;
		v.endpoint_len = s.ep_len;
		v.domain_off = doff;
		v.domain_len = dlen;
		v.host_len = hl;
		v.first_seq = s.first >> 16;
		v.key_lo = s.tag;
		v.key_hi = s.hi;
		out[k] = v;
	}
}

// ---------------------------------------------------------------------------------
// Cross-GPU merge.  Export: the collected services grouped by owner GPU
// (key_lo % world) with their endpoint bytes; merge: received records inserted into the
// owner's table with agg_insert (counters add, the smallest first word wins).
// ---------------------------------------------------------------------------------
constexpr int kOwnerMax = 64;

// Per owner: records and (8-aligned) string bytes, block histograms in LDS.
__global__ void k_owner_count(const ebd_service* rec, const unsigned long long* ctr, uint32_t world, unsigned long long* cnt,
		unsigned long long* bytes) {
	__shared__ unsigned long long hc[kOwnerMax], hb[kOwnerMax];
	for (uint32_t w = threadIdx.x; w < world; w += blockDim.x)
		hc[w] = hb[w] = 0;
	__syncthreads();
	const unsigned long long n = ctr[CTR_SERVICES];
	for (unsigned long long k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const uint32_t w = (uint32_t)(rec[k].key_lo % world);
		atomicAdd(&hc[w], 1ull);
		atomicAdd(&hb[w], (unsigned long long)((rec[k].endpoint_len + 7u) & ~7u));
	}
	__syncthreads();
	for (uint32_t w = threadIdx.x; w < world; w += blockDim.x) {
		if (hc[w])
			atomicAdd(&cnt[w], hc[w]);
		if (hb[w])
			atomicAdd(&bytes[w], hb[w]);
	}
}

// cur[w] / scur[w]: the next record / string byte of owner w (initialised to the owners'
// segment starts); records land in arbitrary order inside their owner's segment.
__global__ void k_owner_scatter(const ebd_service* rec, const unsigned long long* ctr, uint32_t world, const uint8_t* arena,
		unsigned long long* cur, unsigned long long* scur, const unsigned long long* sbase, ebd_service* out, uint8_t* strings) {
	const unsigned long long n = ctr[CTR_SERVICES];
	for (unsigned long long k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		ebd_service v = rec[k];
		const uint32_t w = (uint32_t)(v.key_lo % world);
		const uint32_t nb = (v.endpoint_len + 7u) & ~7u;
		const unsigned long long at = atomicAdd(&cur[w], 1ull);
		const unsigned long long sat = atomicAdd(&scur[w], (unsigned long long)nb);
		if (v.endpoint_off != ~0ull) {
			const unsigned long long* src = (const unsigned long long*)(arena + v.endpoint_off);
			unsigned long long* dst = (unsigned long long*)(strings + sat);
			for (uint32_t b = 0; b < nb / 8; b++)
				dst[b] = src[b];
			v.endpoint_off = sat - sbase[w];
		}
		out[at] = v;
	}
}

__global__ void k_merge(Dev d, const ebd_service* rec, uint32_t n, const uint8_t* strings) {
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const ebd_service v = rec[k];
		bool claimed;
		const unsigned long long first = (v.first_seq << 16) | ((unsigned long long)(v.https & 1u) << 15) | (v.host_len & 0x7fffu);
		const uint32_t slot = agg_insert(d, Hash128{v.key_lo, v.key_hi}, first, v.internal_clients, v.external_clients, &claimed);
		if (claimed) {
			const uint8_t* ep = strings + (v.endpoint_off == ~0ull ? 0 : v.endpoint_off);
			const uint32_t hl = min(v.host_len, v.endpoint_len);
			claim_publish(d, slot, atomicAdd(&d.ctr[CTR_SERVICES], 1ull),
					atomicAdd(&d.ctr[CTR_SARENA], (unsigned long long)((v.endpoint_len + 7u) & ~7u)), v.pid, ep, hl, ep + hl,
					v.endpoint_len - hl);
		}
	}
}

// ---------------------------------------------------------------------------------
// Synthetic trace generation in HBM (ebd_gen.h).
// ---------------------------------------------------------------------------------
// Pass 1: aligned length of every candidate event (0: another shard's), and whether it is kept.
__global__ void k_gen_len(const GenTables* T, uint32_t config, unsigned long long seed, unsigned long long first, uint32_t n,
		uint32_t align, uint32_t count, uint32_t index, unsigned long long* alen, uint32_t* keep) {
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
		const uint32_t L = gen_single_shard(T, config, seed, first + i, count, index, nullptr, nullptr);
		alen[i] = L ? align_up(L, align) : 0;
		keep[i] = L ? 1u : 0u;
	}
}

// Pass 2: kept candidates written at their scanned positions; gidx (optional) = the trace
// index of each written event.
__global__ void k_gen_write(const GenTables* T, uint32_t config, unsigned long long seed, unsigned long long first, uint32_t n,
		const uint32_t* keep, const uint32_t* pos, const unsigned long long* boff, EventRec* ev, uint32_t* len,
		unsigned long long* off, uint8_t* payload, unsigned long long* gidx) {
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
		if (!keep[i])
			continue;
		EventRec e;
		const uint32_t k = pos[i];
		const uint32_t L = gen_single(T, config, seed, first + i, &e, payload + boff[i]);
		ev[k] = e;
		len[k] = L;
		off[k] = boff[i];
		if (gidx)
			gidx[k] = first + i;
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
	// one workgroup per CU (LDS-bound occupancy), each a contiguous range of the batch
	const uint64_t groups = ((uint64_t)d.n + kFreshThreads * 4 - 1) / (kFreshThreads * 4);
	const int grid = (int)(groups < (uint64_t)cus ? groups : (uint64_t)cus);
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
hipError_t launch_collect(const Slot* slots, const unsigned int* used, const unsigned long long* ctr, const uint8_t* arena,
		ebd_service* out, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_collect, dim3(cus * 8), dim3(256), 0, st, slots, used, ctr, arena, out);
	return hipGetLastError();
}
hipError_t launch_clear_used(const unsigned int* used, const unsigned long long* ctr, Slot* slots, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_clear_used, dim3(cus * 8), dim3(256), 0, st, used, ctr, slots);
	return hipGetLastError();
}
hipError_t launch_gen_len(const GenTables* T, uint32_t config, uint64_t seed, uint64_t first, uint32_t n, uint32_t align,
		uint32_t count, uint32_t index, unsigned long long* alen, uint32_t* keep, hipStream_t st) {
	hipLaunchKernelGGL(k_gen_len, dim3(grid_for(n, 256, 8192)), dim3(256), 0, st, T, config, (unsigned long long)seed,
			(unsigned long long)first, n, align, count, index, alen, keep);
	return hipGetLastError();
}
hipError_t launch_gen_write(const GenTables* T, uint32_t config, uint64_t seed, uint64_t first, uint32_t n,
		const uint32_t* keep, const uint32_t* pos, const unsigned long long* boff, EventRec* ev, uint32_t* len,
		unsigned long long* off, uint8_t* payload, unsigned long long* gidx, hipStream_t st) {
	hipLaunchKernelGGL(k_gen_write, dim3(grid_for(n, 256, 8192)), dim3(256), 0, st, T, config, (unsigned long long)seed,
			(unsigned long long)first, n, keep, pos, boff, ev, len, off, payload, gidx);
	return hipGetLastError();
}

hipError_t launch_owner_count(const ebd_service* rec, const unsigned long long* ctr, uint32_t world, unsigned long long* cnt,
		unsigned long long* bytes, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_owner_count, dim3(cus * 4), dim3(256), 0, st, rec, ctr, world, cnt, bytes);
	return hipGetLastError();
}
hipError_t launch_owner_scatter(const ebd_service* rec, const unsigned long long* ctr, uint32_t world, const uint8_t* arena,
		unsigned long long* cur, unsigned long long* scur, const unsigned long long* sbase, ebd_service* out, uint8_t* strings,
		hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_owner_scatter, dim3(cus * 8), dim3(256), 0, st, rec, ctr, world, arena, cur, scur, sbase, out, strings);
	return hipGetLastError();
}
hipError_t launch_merge(const Dev& d, const ebd_service* rec, uint32_t n, const uint8_t* strings, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_merge, dim3(grid_for(n, 256, cus * 8)), dim3(256), 0, st, d, rec, n, strings);
	return hipGetLastError();
}

} // namespace ebd
