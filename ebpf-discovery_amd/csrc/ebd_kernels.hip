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

#include <hipcub/hipcub.hpp>

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
#ifndef EBD_EXP_AGG_NOATOMIC // experiment: probe only, no counter / first-arrival atomics
	if (inc_int)
		atomicAdd(&s->internal_clients, inc_int);
	if (inc_ext)
		atomicAdd(&s->external_clients, inc_ext);
	if (first < seen_first)
		atomicMin(&s->first, first);
#endif
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
	if (list_at < d.new_cap) {
		d.new_slots[list_at] = idx;
	} else {
		set_error(d, EBD_ERR_TABLE_FULL);
		return;
	}
	const uint32_t n = hl + ul;
	unsigned long long off = ~0ull;
	if (ep_at + n <= d.sarena_cap) {
		copy_endpoint((unsigned long long*)(d.sarena + ep_at), host, hl, url, ul);
		off = ep_at;
	} else {
		set_error(d, EBD_ERR_ARENA_FULL);
	}
	d.list_ep[list_at] = off;
	d.list_pl[list_at] = (unsigned long long)pid | ((unsigned long long)n << 32);
}

// ---------------------------------------------------------------------------------
// Network counters (Aggregator.cpp:89-106, EBD_CFG_NETWORK_COUNTERS): an external client's
// /24 and /16 (IPv4) or 48-bit prefix (IPv6) go into its service's maps, map[prefix] = now.
// A claim is one CAS of the whole 64-bit key, so no second word is ever waited for; the time
// is an atomicMax, and the request that finds the entry erased (time 0) adds one to the
// map's size in the service slot.  A v6 prefix does not fit the key beside the slot, so it
// is first interned in a dictionary whose slot index stands for it.
// ---------------------------------------------------------------------------------
__device__ uint32_t v6d_index(const Dev& d, unsigned long long pfx48) {
	const unsigned long long key = pfx48 | (1ull << 63);
	uint32_t idx = (uint32_t)fmix64(key) & d.v6d_mask;
	for (uint32_t probe = 0; probe <= d.v6d_mask; probe++) {
		unsigned long long t = d.v6d[idx]; // a stale 0 at worst: the CAS decides
		if (t == 0) {
			t = atomicCAS(&d.v6d[idx], 0ull, key);
			if (t == 0) {
				atomicAdd(&d.ctr[CTR_V6D], 1ull);
				return idx;
			}
		}
		if (t == key)
			return idx;
		idx = (idx + 1) & d.v6d_mask;
	}
	set_error(d, EBD_ERR_NET_FULL);
	return kNone;
}

// Claims or finds (kind, slot, value) in `nets` and returns the entry (nullptr: table full).
__device__ NetEnt* net_find_or_claim(const Dev& d, NetEnt* nets, uint32_t mask, unsigned long long key) {
	uint32_t idx = (uint32_t)fmix64(key) & mask;
	for (uint32_t probe = 0; probe <= mask; probe++) {
		NetEnt* e = nets + idx;
		unsigned long long t = e->key;
		if (t == 0) {
			t = atomicCAS(&e->key, 0ull, key);
			if (t == 0) {
				atomicAdd(&d.ctr[CTR_NETS], 1ull);
				return e;
			}
		}
		if (t == key)
			return e;
		idx = (idx + 1) & mask;
	}
	set_error(d, EBD_ERR_NET_FULL);
	return nullptr;
}

__device__ void net_touch(const Dev& d, uint32_t slot, uint32_t kind, uint32_t value) {
	NetEnt* e = net_find_or_claim(d, d.nets, d.net_mask, net_key(kind, slot, value));
	if (e && atomicMax(&e->time, d.now) == 0) // new, or erased by networkCountersCleaning
		atomicAdd(&d.slots[slot].nets[kind - 1], 1u);
}

// incrementServiceClientsNumber's network part for an external client (net: net_pack).
__device__ void agg_nets(const Dev& d, uint32_t slot, unsigned long long net) {
	if (slot == kNone)
		return;
	if (net & kNetV6) {
		const uint32_t v = v6d_index(d, net & 0xffffffffffffull);
		if (v != kNone)
			net_touch(d, slot, NET_V6, v);
	} else {
		net_touch(d, slot, NET_V4_24, (uint32_t)(net & 0xffffffu));
		net_touch(d, slot, NET_V4_16, (uint32_t)(net & 0xffffu));
	}
}

// ---------------------------------------------------------------------------------
// Session set: (pid, fd, sessionID) -> slot.  Claimed by a CAS on the 64-bit tag; the
// full key is stored by the claimer and compared by sset_find in later kernels (a tag
// shared by two keys is reported as EBD_ERR_COLLISION there).
// ---------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long sset_tag(unsigned long long kv, uint32_t sid) {
	return fmix64(kv ^ ((unsigned long long)sid * 0x9E3779B97F4A7C15ull) ^ 0x5bd1e9955bd1e995ull) | 1ull;
}

// ev: the event whose fresh parse was UNFINISHED (kNone for a carried session): the first
// such event of the batch bounds when the session can have entered the LRU (k_lru_delta).
__device__ int sset_insert(const Dev& d, uint32_t pid, uint32_t fd, uint32_t sid, uint32_t carry, uint32_t ev) {
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
	if (ev != kNone)
		atomicMax(&d.sset[res].first_c, ~ev);
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
// k_fresh: every NEW_DATA buffer through a fresh parser (Discovery.cpp:141-159
// handleNewSession): the walk of ebd_fresh.h, the client class and the 128-bit service key.
//
// One workgroup per CU owns a contiguous range of the batch.  The payload of consecutive
// events is (almost always) one contiguous byte range in HBM, so the workgroup streams it in
// tiles: a tile is a run of consecutive events whose buffers lie in one 16-KiB window of the
// payload, copied into an LDS slot by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
// instruction, fully coalesced, no VGPRs in flight).  The lane-per-event window loads of the
// previous design capped the stream at ~2.3 TB/s (tools/ubench_mem2.hip) however little
// work the lanes did; a tile stream has no such cap.  Every later access to the bytes is an
// LDS access: the walk, the span rescans, the key, the client-IP token.  Waves have roles:
//   planner (wave 0)   reads len / off / the event records 64 events per round, 4 rounds
//                      ahead, classifies each source address (Aggregator.cpp:60-66, 85-88),
//                      cuts the events into tiles and writes each tile's event table
//   loaders            DMA a planned tile into its slot, then build the slot's bitmap of
//                      bytes outside [0x20, 0x7e] (SWAR, 16 bytes per lane)
//   walkers            one lane per event: the DFA over 4-byte words from LDS, jumping over
//                      generic header values to the next non-printable byte (the bitmap)
//   finalizers         64 finished walks at a time: spans, key, client-IP token and class,
//                      results; the last finalized event of a tile frees its slot
// A slot's life: FREE -> PLANNED (planner) -> READY (loader) -> FREE (when every event of the
// tile is finished).  Its state word carries the tile number, so a walker whose event lies
// in a later tile can tell "not loaded yet" from "already done and recycled".
// ---------------------------------------------------------------------------------
// The table as k_fresh keeps it in LDS: byte-major rows for bytes 0..127 (a byte >= 0x80 steps
// like 0x7f: both are invalid everywhere, ebd_dfa.cpp checks it).  Logical index (s << 8) | b.
struct LdsTable {
	const uint8_t* t;
	__device__ __forceinline__ uint32_t operator[](uint32_t i) const { return t[min(i & 0xffu, 127u) * kLdsStride + (i >> 8)]; }
};

#ifndef EBD_FRESH_WALKERS
#define EBD_FRESH_WALKERS 6
#endif
#ifndef EBD_FRESH_LOADERS
#define EBD_FRESH_LOADERS 2
#endif
constexpr int kFreshThreads = 768; // 12 waves: 3 per SIMD leave 168 VGPRs to the heaviest role (finalize)
constexpr int kFreshWaves = kFreshThreads / 64;
constexpr int kLoadWaves = EBD_FRESH_LOADERS;
constexpr int kWalkWaves = EBD_FRESH_WALKERS;
constexpr int kFinWaves = kFreshWaves - 1 - kLoadWaves - kWalkWaves;
static_assert(kFinWaves >= 1, "k_fresh: at least one finalize wave");
#ifndef EBD_TILE
#define EBD_TILE 16384
#endif
#ifndef EBD_SLOTS
#define EBD_SLOTS 6
#endif
constexpr uint32_t kTile = EBD_TILE; // payload bytes per slot
constexpr uint32_t kTilePad = 64;    // word / 8-byte reads past a buffer's end stay inside the slot
constexpr uint32_t kSlots = EBD_SLOTS;
#ifndef EBD_TILE_EVENTS
#define EBD_TILE_EVENTS 128
#endif
constexpr uint32_t kTileEvents = EBD_TILE_EVENTS;
constexpr uint32_t kFinRing = 256; // finalize records in flight
static_assert((kFinRing & (kFinRing - 1)) == 0 && kFinRing >= 128, "ring: a power of two >= 2 x 64");
// slot state: code | (tile + kSlots) << 2; code 0: free after that tile, 1: planned, 2: ready
enum : uint32_t { SL_FREE = 0, SL_PLANNED = 1, SL_READY = 2 };
__device__ __forceinline__ uint32_t sl_enc(uint32_t code, uint32_t tile) { return code | ((tile + kSlots) << 2); }
__device__ __forceinline__ int sl_tile(uint32_t st) { return (int)(st >> 2) - (int)kSlots; }

// event kinds in a tile's event table
enum : uint32_t { EK_PARSE = 0, EK_SKIP = 1, EK_BAD = 2, EK_EMPTY = 3 };

// finalize record: structure of arrays in the ring (a wave's 64 lanes touch 64 consecutive words)
enum : uint32_t {
	R_SLOT,  // slot | index in the tile << 8
	R_EV,    // event (range-relative)
	R_SF,    // final state | cseen << 8 | post << 9
	R_URL, R_HOST, R_HEND, R_CIP, R_TERM, // trackers (wtrk)
	R_POS,   // ring position + 1 (checked by finalize)
	R_WORDS
};

struct FreshLds {
	uint8_t T[kLdsTableBytes]; // first: LDS address = table index
	uint8_t tile[kSlots][kTile + kTilePad];
	unsigned long long bm[kSlots][kTile / 64]; // bit b of word j: tile byte 64 j + b is outside [0x20, 0x7e]
	uint4 evt[kSlots][kTileEvents];            // x: buffer offset in the tile | L << 16, y: pid, z: flags | kind << 8 | class << 12
	uint32_t ring[R_WORDS * kFinRing];
	uint32_t ready[kFinRing]; // position + 1 once the slot's record is written
	uint32_t freed[kFinRing]; // position + 1 once the slot's record is taken
	unsigned long long sbase[kSlots]; // payload offset of the tile's first byte (16-aligned)
	uint32_t sst[kSlots], sfirst[kSlots], scnt[kSlots], sspan[kSlots], sdone[kSlots];
	uint32_t load_next, walk_next, ntiles, plan_done, tail, claim, walk_done;
	uint32_t abort; // a wait that cannot end: every role leaves (EBD_ERR_INTERNAL), none hangs
};
// Every wait in k_fresh is bounded: ~2^22 sleeps (far longer than any batch) end the kernel
// with EBD_ERR_INTERNAL instead of hanging the GPU on a protocol fault.
constexpr uint32_t kSpinMax = 1u << 22;
static_assert(sizeof(FreshLds) <= 160 * 1024, "k_fresh LDS fits one CU");
static_assert(offsetof(FreshLds, tile) % 16 == 0 && (kTile + kTilePad) % 16 == 0, "tile rows are 16-byte aligned");

__device__ __forceinline__ uint32_t lds_load_acq(const uint32_t* p) {
	return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store_rel(uint32_t* p, uint32_t v) {
	__hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// One more turn of a wait: false once the wait has lasted too long or another wave gave up.
__device__ __forceinline__ bool keep_waiting(const Dev& d, FreshLds& sh, uint32_t& spins) {
	if (++spins > kSpinMax) {
		set_error(d, EBD_ERR_INTERNAL);
		lds_store_rel(&sh.abort, 1u);
		return false;
	}
	if (lds_load_acq(&sh.abort))
		return false;
	__builtin_amdgcn_s_sleep(2);
	return true;
}

// Bytes of w outside [0x20, 0x7e] as 4 bits.  The borrows and carries of the SWAR tests can
// flag a byte above a flagged one, never below: the lowest flag is always exact, and the walk
// only ever asks for the first non-printable byte.
__device__ __forceinline__ uint32_t nonprint4(uint32_t w) {
	const uint32_t lt = (w - 0x20202020u) & ~w & 0x80808080u;
	const uint32_t ge = ((w + 0x01010101u) | w) & 0x80808080u;
	return ((((lt | ge) >> 7) * 0x204081u) >> 21) & 0xfu;
}

// A byte >= 0x80 becomes 0x7f (the table's last row).
__device__ __forceinline__ uint32_t clamp7f(uint32_t x) {
	const uint32_t m = x & 0x80808080u;
	return (x & 0x7f7f7f7fu) | (m - (m >> 7));
}

// An event's bytes in its tile: 4 and 8 bytes at any buffer offset (LDS, no alignment needed).
struct TileMem {
	const uint8_t* b; // the buffer's first byte in the slot
	__device__ __forceinline__ uint32_t ld4(uint32_t o) const {
		const uintptr_t a = (uintptr_t)(b + o);
		const uint32_t* w = (const uint32_t*)(a & ~(uintptr_t)3);
		return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)a & 3u);
	}
	__device__ __forceinline__ unsigned long long ld8(uint32_t o) const {
		return (unsigned long long)ld4(o) | ((unsigned long long)ld4(o + 4) << 32);
	}
	__device__ __forceinline__ uint32_t at(uint32_t o) const { return b[o]; }
};

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
	sset_insert(d, ev.pid, ev.fd, ev.sessionID, 0, i);
}

// One more event of the slot's tile is finished; the last one frees the slot.
__device__ __forceinline__ void tile_event_done(FreshLds& sh, uint32_t slot) {
	const uint32_t st = sh.sst[slot]; // READY(t): stable until this slot's events are all done
	if (atomicAdd(&sh.sdone[slot], 1u) + 1u == sh.scnt[slot])
		lds_store_rel(&sh.sst[slot], sl_enc(SL_FREE, (uint32_t)sl_tile(st)));
}

// The client-IP front token of a finished request and its class, from the value's bytes in
// LDS (kept out of line: it is the longest code path, and inlined into the finalize it pushed
// the kernel past 128 VGPRs).
__device__ __noinline__ uint32_t tile_cip(const Interfaces& ifs, const uint8_t* b, uint32_t cs, uint32_t consumed, uint32_t* tb,
		uint32_t* te) {
	uint8_t c8;
	cip_token(ifs, [b](uint32_t k) { return (uint32_t)b[k]; }, cs, consumed, tb, te, &c8);
	return c8;
}

// The finalize of one walked event (fresh_finalize + the client class), from LDS only.
__device__ __forceinline__ bool finalize_rec(const Dev& d, FreshLds& sh, const uint32_t (&q)[R_WORDS], uint32_t rb) {
	const uint32_t slot = q[R_SLOT] & 0xffu, j = q[R_SLOT] >> 8;
	if (slot >= kSlots || j >= kTileEvents || rb + q[R_EV] >= d.n) {
		set_error(d, EBD_ERR_INTERNAL); // a record that cannot be real: reported, never followed
		return false;
	}
	const uint4 e = sh.evt[slot][j];
	const uint32_t T0 = e.x & 0xffffu, L = e.x >> 16, pid = e.y, flags = e.z & 0xffu, scls = (e.z >> 12) & 3u;
	const uint32_t i = rb + q[R_EV];
	const TileMem mem{sh.tile[slot] + T0};
	WalkRec wr;
	wr.url = q[R_URL];
	wr.host = q[R_HOST];
	wr.hend = q[R_HEND];
	wr.cip = q[R_CIP];
	wr.term = q[R_TERM];
	wr.cseen = (q[R_SF] >> 8) & 1u;
	FreshResult fr;
	fresh_finalize(LdsTable{sh.T}, d.di, wr, q[R_SF] & 0xffu, ((q[R_SF] >> 9) & 1u) != 0, mem, L, d.hkey, pid, (uint8_t)flags, fr);
	ebd_event_result& r = fr.r;
	if (r.status == EBD_STATUS_FINISHED) {
		uint32_t cls = scls;
		if (fr.cip) { // the first client-IP value's front token decides (Aggregator.cpp:50-74)
			uint32_t tb, te;
			cls = tile_cip(*d.ifs, mem.b, r.u.span.cip_off, r.consumed, &tb, &te);
			r.u.span.cip_off = (uint16_t)tb;
			r.u.span.cip_len = (uint16_t)(te - tb);
		}
		r.info = (uint8_t)(r.info | (cls << EBD_INFO_CLASS_SHIFT));
		d.keys[i] = fr.key;
	} else if (r.status == EBD_STATUS_UNFINISHED) {
		// the session may be saved (Discovery.cpp:148-150): sequential path
		const EventRec& ev = d.ev[i];
		atomicAdd(&d.ctr[CTR_UNFINISHED], 1ull);
		sset_insert(d, ev.pid, ev.fd, ev.sessionID, 0, i);
	}
	d.res[i] = r;
	return true;
}

__global__ __launch_bounds__(kFreshThreads) void k_fresh(Dev d) {
	__shared__ __attribute__((aligned(16))) FreshLds sh;
	const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
	// this workgroup's contiguous share of the batch
	const uint32_t per = (uint32_t)(((unsigned long long)d.n + gridDim.x - 1) / gridDim.x);
	const uint32_t rb = min(d.n, blockIdx.x * per), re = min(d.n, rb + per), nr = re - rb;
	for (uint32_t k = threadIdx.x * 16u; k < kLdsTableBytes; k += kFreshThreads * 16u)
		*(uint4*)(sh.T + k) = *(const uint4*)(d.dfa + k);
	for (uint32_t k = threadIdx.x; k < kFinRing; k += kFreshThreads)
		sh.ready[k] = sh.freed[k] = 0;
	if (threadIdx.x < kSlots)
		sh.sst[threadIdx.x] = sl_enc(SL_FREE, threadIdx.x - kSlots); // "tile slot - kSlots is done"
	if (threadIdx.x == 0)
		sh.load_next = sh.walk_next = sh.ntiles = sh.plan_done = sh.tail = sh.claim = sh.walk_done = sh.abort = 0;
	__syncthreads();
	const DfaInfo& di = d.di;

	if (wave == 0) {
		// ---- planner ----
		constexpr uint32_t kAhead = 4; // rounds of 64 events whose metadata is in flight
		uint32_t mL[kAhead], mPid[kAhead], mFl[kAhead];
		unsigned long long mOff[kAhead];
		v4u mSrc[kAhead];
		auto fetch = [&](uint32_t r, uint32_t k) {
			const uint32_t i = rb + r * 64 + lane;
			if (i < re) {
				const uint8_t* evb = (const uint8_t*)(d.ev + i);
				mL[k] = d.len[i];
				mOff[k] = d.off[i];
				mPid[k] = *(const uint32_t*)evb;
				mSrc[k] = *(const __attribute__((address_space(1))) v4u*)(evb + 16); // 4-byte aligned
				mFl[k] = *(const uint32_t*)(evb + 32);
			}
		};
		const uint32_t rounds = (nr + 63) / 64;
#pragma unroll
		for (uint32_t k = 0; k < kAhead; k++)
			fetch(k, k);
		uint32_t tnum = 0, slot = 0, cnt = 0, first = 0, maxend = 0;
		bool open = false, has_base = false;
		unsigned long long A = 0;
		auto close = [&]() {
			if (lane == 0) {
				sh.sbase[slot] = A;
				sh.sspan[slot] = (maxend + 15u) & ~15u;
				sh.sfirst[slot] = first;
				sh.scnt[slot] = cnt;
				sh.sdone[slot] = 0;
				lds_store_rel(&sh.sst[slot], sl_enc(SL_PLANNED, tnum));
			}
			tnum++;
			open = false;
		};
		for (uint32_t r0 = 0; r0 < rounds; r0 += kAhead) {
#pragma unroll
			for (uint32_t k = 0; k < kAhead; k++) {
				const uint32_t r = r0 + k;
				if (r >= rounds)
					break;
				const uint32_t i = rb + r * 64 + lane;
				const bool valid = i < re;
				const uint32_t L = mL[k], flags = mFl[k] & 0xffu;
				const unsigned long long off = mOff[k];
				const uint32_t kind = !(flags & FLAG_NEW) || L == EBD_NO_BUFFER ? EK_SKIP
						: (L > EBD_BUFFER_MAX_DATA_SIZE || (off >> 40)) ? EK_BAD : L == 0 ? EK_EMPTY : EK_PARSE;
				const bool hasb = valid && kind == EK_PARSE;
				uint8_t src[16];
				__builtin_memcpy(src, &mSrc[k], 16);
				const uint32_t cls = hasb ? classify_source(*d.ifs, (uint8_t)flags, src) : 0u;
				const uint32_t nvalid = min(64u, re - (rb + r * 64));
				const uint4 ent = make_uint4(0u, mPid[k], flags | (kind << 8) | (cls << 12), 0u);
				if (r + kAhead < rounds)
					fetch(r + kAhead, k);
				uint32_t j0 = 0;
				while (j0 < nvalid) {
					if (!open) {
						slot = tnum % kSlots;
						uint32_t spins = 0;
						while (lds_load_acq(&sh.sst[slot]) != sl_enc(SL_FREE, tnum - kSlots))
							if (!keep_waiting(d, sh, spins))
								return;
						open = true;
						has_base = false;
						cnt = 0;
						maxend = 0;
						first = r * 64 + j0;
					}
					if (!has_base) {
						const unsigned long long pb = __ballot(hasb && lane >= j0);
						if (pb) {
							A = __shfl(off, __builtin_ctzll(pb), 64) & ~15ull;
							has_base = true;
						}
					}
					// the longest run of events from j0 that fits the tile
					const bool fit = !hasb || (has_base && off >= A && off + L + 15ull <= A + kTile);
					const unsigned long long nf = __ballot(lane >= j0 && lane < nvalid && !fit);
					uint32_t stop = nf ? (uint32_t)__builtin_ctzll(nf) : nvalid;
					stop = min(stop, j0 + (kTileEvents - cnt));
					if (lane >= j0 && lane < stop) {
						uint4 x = ent;
						x.x = hasb ? (uint32_t)(off - A) | (L << 16) : 0u;
						sh.evt[slot][cnt + lane - j0] = x;
					}
					uint32_t end = (lane >= j0 && lane < stop && hasb) ? (uint32_t)(off + L - A) : 0u;
					for (int o = 32; o > 0; o >>= 1)
						end = max(end, (uint32_t)__shfl_xor((int)end, o, 64));
					maxend = max(maxend, end);
					cnt += stop - j0;
					j0 = stop;
					if (j0 < nvalid || cnt == kTileEvents)
						close();
				}
			}
		}
		if (open && cnt)
			close();
		if (lane == 0) {
			sh.ntiles = tnum;
			lds_store_rel(&sh.plan_done, 1u);
		}
		return;
	}

	if (wave <= (uint32_t)kLoadWaves) {
		// ---- loaders ----
		for (;;) {
			uint32_t t = 0;
			if (lane == 0)
				t = atomicAdd(&sh.load_next, 1u);
			t = __builtin_amdgcn_readfirstlane(t);
			const uint32_t slot = t % kSlots;
			bool have = false;
			uint32_t spins = 0;
			for (;;) {
				if (lds_load_acq(&sh.sst[slot]) == sl_enc(SL_PLANNED, t)) {
					have = true;
					break;
				}
				if (lds_load_acq(&sh.plan_done) && t >= sh.ntiles)
					break;
				if (!keep_waiting(d, sh, spins))
					break;
			}
			if (!have)
				break;
			const unsigned long long A = sh.sbase[slot];
			const uint32_t span = sh.sspan[slot];
			uint8_t* dst = sh.tile[slot];
			for (uint32_t k = 0; k * 1024u < span; k++) {
				const uint32_t o = k * 1024u + lane * 16u;
				if (o < span)
					__builtin_amdgcn_global_load_lds((const void*)(d.payload + A + o),
							(__attribute__((address_space(3))) void*)(dst + k * 1024u), 16, 0, 0);
			}
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			uint16_t* bm16 = (uint16_t*)sh.bm[slot];
			for (uint32_t j = lane; j * 16u < span; j += 64u) {
				const uint4 v = *(const uint4*)(dst + 16u * j);
				bm16[j] = (uint16_t)(nonprint4(v.x) | (nonprint4(v.y) << 4) | (nonprint4(v.z) << 8) | (nonprint4(v.w) << 12));
			}
			lds_store_rel(&sh.sst[slot], sl_enc(SL_READY, t));
		}
		return;
	}

	if (wave >= (uint32_t)(1 + kLoadWaves + kWalkWaves)) {
		// ---- finalizers: 64 consecutive ring positions per wave, each record as it arrives ----
		// A wave cannot wait for all 64: the records that would complete its batch may belong
		// to tiles that are only planned once the slots its own pending records hold are freed.
		for (;;) {
			uint32_t c = 0;
			if (lane == 0)
				c = atomicAdd(&sh.claim, 64u);
			c = __builtin_amdgcn_readfirstlane(c);
			const uint32_t pos = c + lane, rs = pos & (kFinRing - 1);
			bool todo = true; // this lane's position is still to be finalized (or ruled out)
			bool any_rec = false;
			uint32_t spins = 0;
			for (;;) {
				const bool rd = todo && lds_load_acq(&sh.ready[rs]) == pos + 1;
				if (__any(rd)) {
					if (rd) {
						uint32_t q[R_WORDS];
#pragma unroll
						for (uint32_t f = 0; f < R_WORDS; f++)
							q[f] = sh.ring[f * kFinRing + rs];
						lds_store_rel(&sh.freed[rs], pos + 1); // the ring slot may be written again
						if (q[R_POS] != pos + 1)
							set_error(d, EBD_ERR_INTERNAL); // ring protocol violated: reported, not followed
#ifndef EBD_EXP_NOFIN // experiment: records taken, not finalized (results are wrong)
						else if (finalize_rec(d, sh, q, rb))
#else
						else
#endif
							tile_event_done(sh, q[R_SLOT] & 0xffu);
						todo = false;
					}
					any_rec = true;
					spins = 0;
					continue;
				}
				if (!__any(todo))
					break;
				uint32_t done = 0, tail = 0;
				if (lane == 0) {
					done = lds_load_acq(&sh.walk_done);
					tail = lds_load_acq(&sh.tail);
				}
				done = __builtin_amdgcn_readfirstlane(done);
				tail = __builtin_amdgcn_readfirstlane(tail);
				if (done == (uint32_t)kWalkWaves) { // every position below tail was pushed
					if (todo && pos >= tail && lds_load_acq(&sh.ready[rs]) != pos + 1)
						todo = false;
					if (!__any(todo))
						break;
				}
				if (!keep_waiting(d, sh, spins))
					break;
			}
			if (!any_rec || lds_load_acq(&sh.abort)) // the batch began past the last record
				break;
		}
		return;
	}

	// ---- walkers: one lane per event ----
	uint32_t ev = kNone, wt = 0, slot = 0, T0 = 0, L = 0, p = 0, s = di.init, post = 0, j = 0;
	bool over = false, rdy = false;
	uint32_t idle = 0;
	WalkRec wr;
	walk_init(di, wr);
	for (;;) {
		// events for the lanes without one, one LDS atomic per wave
		const bool need = !over && ev == kNone;
		const unsigned long long nb = __ballot(need);
		if (nb) {
			uint32_t base = 0;
			if (lane == 0)
				base = atomicAdd(&sh.walk_next, (uint32_t)__popcll(nb));
			base = __builtin_amdgcn_readfirstlane(base);
			if (need) {
				const uint32_t e = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(nb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)nb, 0));
				if (e < nr) {
					ev = e;
					rdy = false;
				} else {
					over = true;
				}
			}
		}
		if (__all(over))
			break;
		bool worked = false;
		// find the event's tile: tiles are numbered in event order
		if (ev != kNone && !rdy) {
			for (;;) {
				slot = wt % kSlots;
				const uint32_t st = lds_load_acq(&sh.sst[slot]);
				const int tt = sl_tile(st);
				if (tt > (int)wt || (tt == (int)wt && (st & 3u) == SL_FREE)) { // tile wt is done: ev is later
					wt++;
					continue;
				}
				if (tt == (int)wt && (st & 3u) == SL_READY) {
					if (ev >= sh.sfirst[slot] + sh.scnt[slot]) {
						wt++;
						continue;
					}
					rdy = true;
				}
				break; // rdy, or tile wt is not loaded yet
			}
			if (rdy) {
				worked = true;
				j = ev - sh.sfirst[slot];
				const uint4 e = sh.evt[slot][j];
				const uint32_t kind = (e.z >> 8) & 3u;
				if (kind != EK_PARSE) {
					const uint32_t i = rb + ev;
					if (kind == EK_BAD)
						set_error(d, EBD_ERR_BAD_INPUT);
					if (kind == EK_EMPTY)
						write_empty(d, i);
					else
						write_none(d, i);
					tile_event_done(sh, slot);
					ev = kNone;
					rdy = false;
				} else {
					T0 = e.x & 0xffffu;
					L = e.x >> 16;
					p = 0;
					s = di.init;
					walk_init(di, wr);
					post = sh.tile[slot][T0] == 'P' ? 1u : 0u;
#ifdef EBD_EXP_NOWALK // experiment: the tile stream without walks (results are wrong)
					p = L;
#endif
				}
			}
		}
		bool fin = false;
#ifdef EBD_EXP_NOWALK
		if (ev != kNone && rdy && p >= L) {
			fin = true;
		} else
#endif
		if (ev != kNone && rdy) {
			worked = true;
			const uint8_t* b = sh.tile[slot] + T0;
			if (st_skips(di, s)) {
				// jump to the word of the next byte outside [0x20, 0x7e] (none: unfinished at L)
				const uint32_t x0 = T0 + p, xe = T0 + L;
				uint32_t J = x0 >> 6;
				unsigned long long w = sh.bm[slot][J] & (~0ull << (x0 & 63u));
				while (w == 0 && 64u * (J + 1) < xe)
					w = sh.bm[slot][++J];
				const uint32_t qx = w ? 64u * J + (uint32_t)__builtin_ctzll(w) : xe;
				if (qx >= xe) {
					p = L;
					fin = true;
				} else {
					p = (qx - T0) & ~3u;
				}
			}
			if (!fin) {
				const uint32_t x = clamp7f(TileMem{b}.ld4(p));
				const uint32_t s0 = s;
				s = sh.T[__builtin_amdgcn_ubfe(x, 0, 8) * kLdsStride + s];
				uint32_t m = s;
				s = sh.T[__builtin_amdgcn_ubfe(x, 8, 8) * kLdsStride + s];
				m = max(m, s);
				s = sh.T[__builtin_amdgcn_ubfe(x, 16, 8) * kLdsStride + s];
				m = max(m, s);
				s = sh.T[(x >> 24) * kLdsStride + s];
				m = max(m, s);
				word_update(di, wr, p >> 2, s0, m);
				p += 4;
				fin = st_terminal(di, s) || p >= L;
			}
		}
		// hand finished walks to the finalizers
		const unsigned long long fb = __ballot(fin);
		if (fb) {
			uint32_t base = 0;
			if (lane == 0)
				base = atomicAdd(&sh.tail, (uint32_t)__popcll(fb));
			base = __builtin_amdgcn_readfirstlane(base);
			if (fin) {
				const uint32_t pos = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(fb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fb, 0));
				const uint32_t rs = pos & (kFinRing - 1);
				uint32_t spins = 0;
				if (pos >= kFinRing) // the slot's previous record must have been taken
					while (lds_load_acq(&sh.freed[rs]) != pos - kFinRing + 1)
						if (!keep_waiting(d, sh, spins))
							break;
				uint32_t t[R_WORDS];
				t[R_SLOT] = slot | (j << 8);
				t[R_EV] = ev;
				t[R_SF] = s | (wr.cseen << 8) | (post << 9);
				t[R_URL] = wr.url;
				t[R_HOST] = wr.host;
				t[R_HEND] = wr.hend;
				t[R_CIP] = wr.cip;
				t[R_TERM] = wr.term;
				t[R_POS] = pos + 1;
#pragma unroll
				for (uint32_t f = 0; f < R_WORDS; f++)
					sh.ring[f * kFinRing + rs] = t[f];
				lds_store_rel(&sh.ready[rs], pos + 1);
				ev = kNone;
				rdy = false;
			}
		}
		if (!__any(worked)) {
			if (!keep_waiting(d, sh, idle))
				break;
		} else {
			idle = 0;
		}
	}
	if (lane == 0)
		atomicAdd(&sh.walk_done, 1u);
}

// ---------------------------------------------------------------------------------
// The network of an external fast-path client (EBD_CFG_NETWORK_COUNTERS, Aggregator.cpp:89-106):
// k_fresh already chose the client and its class (the client-IP front token, or the source
// address); the maps need the address itself, parsed again here from the token's bytes.
// ---------------------------------------------------------------------------------
constexpr int kAggThreads = 256;

__device__ unsigned long long request_net(const Dev& d, uint32_t i, const ebd_event_result& r) {
	unsigned long long net = 0;
	if (r.info & EBD_INFO_CIP) {
		const uint8_t* t = d.payload + d.off[i] + r.u.span.cip_off;
		struct View {
			const uint8_t* t;
			__device__ uint8_t operator[](uint32_t k) const { return t[k]; }
		};
		classify_token(*d.ifs, View{t}, r.u.span.cip_len, &net);
	} else {
		const uint8_t* evb = (const uint8_t*)(d.ev + i);
		const v4u sv = *(const __attribute__((address_space(1))) v4u*)(evb + 16); // sourceIP (4-B aligned)
		uint8_t src[16];
		__builtin_memcpy(src, &sv, 16);
		classify_source(*d.ifs, evb[32], src, &net);
	}
	return net;
}

__global__ void k_carry_insert(Dev d) {
	for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < d.n_carry_in; c += gridDim.x * blockDim.x) {
		const Carry& cr = d.carry_in[c];
		sset_insert(d, cr.pid, cr.fd, cr.sid, c + 1, kNone);
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
			d.res[i].info |= EBD_INFO_SESSION; // k_walk's, not k_agg_fast's (which may run first)
			atomicMax(&d.sset[slot].last_ev, i + 1);
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
constexpr int kWalkThreads = 256;

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

// Sequential byte reads through a 16-B register window: one aligned dwordx4 load per 16
// bytes instead of one byte load each.  The aligned block holding a valid byte never
// leaves that byte's page, so the over-read cannot fault.
struct ByteWin {
	const uint8_t* base;
	uintptr_t blk;
	uint32_t w0, w1, w2, w3;
	__device__ explicit ByteWin(const uint8_t* b) : base(b), blk(~(uintptr_t)0), w0(0), w1(0), w2(0), w3(0) {}
	__device__ __forceinline__ uint32_t operator()(uint32_t k) {
		const uintptr_t a = (uintptr_t)(base + k), b = a & ~(uintptr_t)15;
		if (b != blk) {
			const uint4 v = *(const uint4*)b;
			w0 = v.x, w1 = v.y, w2 = v.z, w3 = v.w;
			blk = b;
		}
		const uint32_t q = (uint32_t)(a >> 2) & 3u;
		const uint32_t x = q == 0 ? w0 : q == 1 ? w1 : q == 2 ? w2 : w3;
		return (x >> ((uint32_t)(a & 3u) * 8u)) & 0xffu;
	}
};

// Visits stream bytes [a, a + n) in order; the stream ends at sorted position jend whose
// piece is truncated to cend bytes.  fn(byte) returns false to stop.  Returns bytes visited.
template <typename Fn>
__device__ uint32_t stream_visit(const Dev& d, const Walk& w, uint32_t jend, uint32_t cend, uint32_t a, uint32_t n, Fn fn) {
	uint32_t pos = 0, done = 0;
	const uint32_t b = a + n;
	if (w.clen) {
		ByteWin cb(w.cb);
		for (uint32_t k = a; k < b && k < w.clen; k++) {
			if (!fn((uint8_t)cb(k)))
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
			ByteWin src(d.payload + d.off[slow_event(d, j)] + (lo - pos));
			for (uint32_t k = 0; k < hi - lo; k++) {
				if (!fn((uint8_t)src(k)))
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
	unsigned long long net = 0;
	if (g.f & GPF_CIP_FOUND) {
		front_token(dst + hl + ul, raw, &tb, &te);
		info |= EBD_INFO_CIP;
		cls = classify_token(*d.ifs, dst + hl + ul + tb, te - tb, &net);
	} else {
		cls = classify_source(*d.ifs, ev.flags, ev.sourceIP, &net);
	}
	info |= (uint8_t)(cls << EBD_INFO_CLASS_SHIFT);
	kh.bytes(dst, hl + ul);
	bool claimed;
	const uint32_t slot = agg_insert(d, kh.finish(), first_word(d.seq_base + i, (g.f & GPF_HTTPS) != 0, hl),
			cls == CLS_INTERNAL, cls == CLS_EXTERNAL, &claimed);
	if (claimed) // a rare path: one reservation per claim
		claim_publish(d, slot, atomicAdd(&d.ctr[CTR_SERVICES], 1ull),
				atomicAdd(&d.ctr[CTR_SARENA], (unsigned long long)((hl + ul + 7u) & ~7u)), ev.pid, dst, hl, dst + hl, ul);
	if (d.net_on && cls == CLS_EXTERNAL)
		agg_nets(d, slot, net);
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

// A session as the walkers hold it: the parser (Session, Discovery.h), the request in
// progress (Walk), whether it is in the LRU (savedSessions) and when it was last found or
// inserted there (LRU recency; Discovery.cpp:114 find and :215 insert both touch it).
struct SessState {
	GenParser g;
	Walk w;
	unsigned long long stamp;
	uint32_t live;
	uint32_t li; // position in the exact walker's live list
};

enum : uint32_t { OP_NONE = 0, OP_INSERT = 1, OP_ERASE = 2 };

// Event jj (sorted position) of a session: handleNewEvent (Discovery.cpp:92-198) with the
// session's state in S.  Returns the LRU operation it implies; an insert (saveSession,
// Discovery.cpp:148-150) is left to the caller, which may have to evict first.
__device__ uint32_t session_event(const Dev& d, const KeyTrie* trie, SessState& S, uint32_t jj) {
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
	uint32_t op = OP_NONE;
	if ((flags & FLAG_NEW) && L != EBD_NO_BUFFER && L <= EBD_BUFFER_MAX_DATA_SIZE) {
		ByteWin at(d.payload + d.off[i]);
		if (S.live) { // handleExistingSession, Discovery.cpp:123-139 (find touched it)
			S.stamp = d.seq_base + i;
			r.info |= EBD_INFO_EXISTING;
			const uint32_t c = gp_parse(S.g, trie, at, L, flags);
			r.consumed = (uint16_t)c;
			if (S.g.state == ST_INVALID) {
				r.status = EBD_STATUS_INVALID;
				atomicAdd(&d.ctr[CTR_KDELETES], 1ull); // bpfDiscoveryDeleteSession
				S.live = 0;
				op = OP_ERASE;
			} else if (S.g.state == ST_FINISHED) {
				r.status = EBD_STATUS_FINISHED;
				emit_session_request(d, S.w, jj, c, S.g, i, r);
				gp_reset(S.g); // session.reset(); stays saved
				S.w = Walk{nullptr, 0, jj + 1};
			} else {
				r.status = EBD_STATUS_UNFINISHED;
			}
		} else { // handleNewSession, Discovery.cpp:141-159
			gp_init(S.g);
			S.w = Walk{nullptr, 0, jj};
			const uint32_t c = gp_parse(S.g, trie, at, L, flags);
			r.consumed = (uint16_t)c;
			if (S.g.state == ST_INVALID) {
				r.status = EBD_STATUS_INVALID;
			} else if (S.g.state == ST_FINISHED) {
				r.status = EBD_STATUS_FINISHED;
				emit_session_request(d, S.w, jj, c, S.g, i, r);
			} else {
				r.status = EBD_STATUS_UNFINISHED;
				if (!(flags & FLAG_END))
					op = OP_INSERT;
			}
		}
	}
	if ((flags & FLAG_END) && S.live) { // handleCloseEvent, Discovery.cpp:194-198
		S.live = 0;
		op = OP_ERASE;
	}
	d.res[i] = r;
	return op;
}

// The session's state at its first event of the batch (sorted position j).
__device__ void session_begin(const Dev& d, SessState& S, uint32_t j, uint32_t slot) {
	SSlot* ss = d.sset + slot;
	ss->visited = 1;
	S.w = Walk{nullptr, 0, j};
	S.li = kNone;
	const uint32_t carry = ss->carry;
	if (carry) { // saved session from an earlier batch (LRU entry)
		const Carry& c = d.carry_in[carry - 1];
		S.g = c.g;
		S.live = 1;
		S.stamp = c.stamp;
		S.w.cb = c.bytes;
		S.w.clen = c.nbytes;
	} else {
		gp_init(S.g);
		S.live = 0;
		S.stamp = 0;
	}
}

// A session still in the LRU after the batch, with the bytes of its request in progress
// (which ends with the session's last event jlast of the batch, fully consumed).
__device__ void session_carry_out(const Dev& d, const SessState& S, uint32_t j, uint32_t jlast) {
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
	out.stamp = S.stamp;
	out.g = S.g;
	const uint32_t nb = S.g.length < kCarryBytes ? S.g.length : kCarryBytes;
	out.nbytes = nb;
	uint32_t k = 0;
	uint8_t* dst = out.bytes;
	stream_visit(d, S.w, jlast, piece_len(d, jlast), 0, nb, [&](uint8_t b) {
		dst[k++] = b;
		return true;
	});
}

// The parallel session path: one lane per session (k_walk_heads lists them), events in
// order.  Exact while no LRU eviction can happen (run_batch checks an upper bound of the
// live sessions first).  The header-key trie and the byte classes sit in LDS: the walk
// reads them once per byte.
__global__ __launch_bounds__(kWalkThreads) void k_walk(Dev d) {
	__shared__ KeyTrie trie;
	for (uint32_t k = threadIdx.x; k < (uint32_t)sizeof(KeyTrie); k += kWalkThreads)
		((uint8_t*)&trie)[k] = ((const uint8_t*)d.trie)[k];
	__syncthreads();
	const uint32_t nh = (uint32_t)d.ctr[CTR_HEADS], nslow = (uint32_t)d.ctr[CTR_SLOW];
	for (uint32_t h = blockIdx.x * kWalkThreads + threadIdx.x; h < nh; h += gridDim.x * kWalkThreads) {
		const uint32_t j = d.heads[h];
		const uint32_t slot = (uint32_t)(d.slow_keys[j] >> 32);
		SessState S;
		session_begin(d, S, j, slot);
		uint32_t jj = j;
		for (; jj < nslow && (uint32_t)(d.slow_keys[jj] >> 32) == slot; jj++) {
			const uint32_t op = session_event(d, &trie, S, jj);
			if (op == OP_INSERT) {
				S.live = 1; // saveSession: a new key goes to the front (LRUCache.h:54-60)
				S.stamp = d.seq_base + slow_event(d, jj);
				atomicAdd(&d.ctr[CTR_INSERTS], 1ull);
			}
		}
		if (S.live)
			session_carry_out(d, S, j, jj - 1);
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
		out.stamp = cr.stamp;
		out.g = cr.g;
		out.nbytes = cr.nbytes;
		for (uint32_t b = 0; b < cr.nbytes; b++)
			out.bytes[b] = cr.bytes[b];
	}
}

// ---------------------------------------------------------------------------------
// Exact LRU (LRUCache.h:50-89, capacity EBD_MAX_SESSIONS, Discovery.cpp:39).
//
// Eviction couples sessions, so the parallel walker is exact only while the LRU never
// holds more than its capacity.  An upper bound decides: a session can be in the LRU only
// from its first event whose fresh parse was UNFINISHED (the only way in is saveSession
// after such a parse) or from before the batch (carried), until its last event if that one
// closes it.  k_lru_delta marks +1 / -1 at those events, a scan gives the running count,
// and k_lru_peak its maximum.  When carried + peak <= capacity no insert can find the cache
// full; otherwise the batch's session events run through k_walk_lru, which replays them in
// event order with a real LRU: find / insert touch, an insert into a full cache evicts the
// least recently used session (which then parses its next buffer as a new session,
// Discovery.cpp:141), close and INVALID erase.
// ---------------------------------------------------------------------------------
__global__ void k_lru_delta(Dev d, uint32_t nslow, int* delta, uint8_t* minus) {
	for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nslow; j += gridDim.x * blockDim.x) {
		const uint32_t i = slow_event(d, j);
		const SSlot& ss = d.sset[(uint32_t)(d.slow_keys[j] >> 32)];
		const bool carried = ss.carry != 0;
		const uint32_t first = ss.first_c ? ~ss.first_c : kNone;
		const bool plus = !carried && first == i;
		const bool close = (d.ev[i].flags & FLAG_END) && i + 1 == ss.last_ev && (carried || (first != kNone && first <= i));
		delta[i] = (plus ? 1 : 0) - (close ? 1 : 0);
		minus[i] = close ? 1 : 0;
	}
}

// max over events of (running count before the event's close) = scan[i] + minus[i]
__global__ void k_lru_peak(const int* scan, const uint8_t* minus, uint32_t n, unsigned long long* ctr) {
	__shared__ int red[256];
	int m = 0;
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
		m = max(m, scan[i] + (int)minus[i]);
	red[threadIdx.x] = m;
	__syncthreads();
	for (uint32_t s = blockDim.x / 2; s > 0; s >>= 1) {
		if (threadIdx.x < s)
			red[threadIdx.x] = max(red[threadIdx.x], red[threadIdx.x + s]);
		__syncthreads();
	}
	if (threadIdx.x == 0)
		atomicMax(&ctr[CTR_LRU_PEAK], (unsigned long long)red[0] + (1ull << 31));
}

// Event -> sorted position (kNone for events of no session in the set) and each sorted
// position's session head.
__global__ void k_lru_index(Dev d, uint32_t nslow, uint32_t* jpos, uint32_t* head) {
	for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nslow; j += gridDim.x * blockDim.x) {
		jpos[slow_event(d, j)] = j;
		const uint32_t slot = (uint32_t)(d.slow_keys[j] >> 32);
		if (j > 0 && (uint32_t)(d.slow_keys[j - 1] >> 32) == slot)
			continue;
		for (uint32_t jj = j; jj < nslow && (uint32_t)(d.slow_keys[jj] >> 32) == slot; jj++)
			head[jj] = j;
	}
}

constexpr int kLruThreads = 256;

__device__ __forceinline__ void live_add(SessState* S, uint32_t* live, uint32_t& nlive, uint32_t h) {
	S[h].li = nlive;
	live[nlive++] = h;
}
__device__ __forceinline__ void live_remove(SessState* S, uint32_t* live, uint32_t& nlive, uint32_t h) {
	const uint32_t k = S[h].li, last = live[--nlive];
	live[k] = last;
	S[last].li = k;
	S[h].li = kNone;
}

// The exact walker: one workgroup.  Lane 0 replays the session events in event order; at an
// insert into a full cache the workgroup finds the least recently used session together.
__global__ __launch_bounds__(kLruThreads) void k_walk_lru(Dev d, uint32_t nslow, const uint32_t* jpos, const uint32_t* head,
		SessState* S, uint32_t* live, uint32_t cap) {
	__shared__ uint32_t ord[kLruThreads];
	__shared__ uint32_t nord, nlive, k_next, evict_for;
	__shared__ unsigned long long rs[kLruThreads];
	__shared__ uint32_t ri[kLruThreads];
	__shared__ KeyTrie trie;
	const uint32_t t = threadIdx.x;
	for (uint32_t k = t; k < (uint32_t)sizeof(KeyTrie); k += kLruThreads)
		((uint8_t*)&trie)[k] = ((const uint8_t*)d.trie)[k];
	if (t == 0)
		nlive = 0;
	__syncthreads();
	// every session's state at the batch start; the carried ones are in the LRU
	for (uint32_t j = t; j < nslow; j += kLruThreads)
		if (head[j] == j) {
			session_begin(d, S[j], j, (uint32_t)(d.slow_keys[j] >> 32));
			if (S[j].live) {
				const uint32_t k = atomicAdd(&nlive, 1u);
				S[j].li = k;
				live[k] = j;
			}
		}
	__syncthreads();
	// carried sessions without an event in this batch are in the LRU too (handles nslow + c)
	for (uint32_t c = t; c < d.n_carry_in; c += kLruThreads) {
		const Carry& cr = d.carry_in[c];
		const int slot = sset_find(d, cr.pid, cr.fd, cr.sid);
		if (slot >= 0 && d.sset[slot].visited)
			continue;
		SessState& x = S[nslow + c];
		x.live = 1;
		x.stamp = cr.stamp;
		const uint32_t k = atomicAdd(&nlive, 1u);
		x.li = k;
		live[k] = nslow + c;
	}
	__syncthreads();
	for (uint32_t base = 0; base < d.n; base += kLruThreads) {
		// this chunk's session events, in event order
		const uint32_t i = base + t;
		const uint32_t jp = i < d.n ? jpos[i] : kNone;
		if (t == 0)
			nord = 0;
		__syncthreads();
		const unsigned long long b = __ballot(jp != kNone);
		__shared__ uint32_t wcount[kLruThreads / 64];
		if ((t & 63) == 0)
			wcount[t >> 6] = (uint32_t)__popcll(b);
		__syncthreads();
		uint32_t off = 0;
		for (uint32_t w = 0; w < (t >> 6); w++)
			off += wcount[w];
		if (jp != kNone)
			ord[off + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0))] = jp;
		if (t == kLruThreads - 1)
			nord = off + (uint32_t)__popcll(b);
		__syncthreads();
		uint32_t k = 0;
		while (k < nord) { // uniform
			if (t == 0) {
				uint32_t e = kNone;
				for (; k < nord; k++) {
					const uint32_t jj = ord[k], h = head[jj];
					const uint32_t op = session_event(d, &trie, S[h], jj);
					if (op == OP_ERASE && S[h].li != kNone) {
						live_remove(S, live, nlive, h);
					} else if (op == OP_INSERT) {
						if (nlive >= cap) { // LRUCache.h:56-58: pop the tail first
							e = h;
							k++;
							break;
						}
						S[h].live = 1;
						S[h].stamp = d.seq_base + slow_event(d, jj);
						live_add(S, live, nlive, h);
						atomicAdd(&d.ctr[CTR_INSERTS], 1ull);
					}
				}
				k_next = k;
				evict_for = e;
			}
			__syncthreads();
			k = k_next;
			if (evict_for != kNone) { // the least recently used live session
				unsigned long long best = ~0ull;
				uint32_t bi = kNone;
				for (uint32_t x = t; x < nlive; x += kLruThreads) {
					const unsigned long long st = S[live[x]].stamp;
					if (st < best) {
						best = st;
						bi = live[x];
					}
				}
				rs[t] = best;
				ri[t] = bi;
				__syncthreads();
				for (uint32_t s = kLruThreads / 2; s > 0; s >>= 1) {
					if (t < s && rs[t + s] < rs[t]) {
						rs[t] = rs[t + s];
						ri[t] = ri[t + s];
					}
					__syncthreads();
				}
				if (t == 0) {
					const uint32_t v = ri[0], h = evict_for;
					if (v != kNone) {
						S[v].live = 0; // evicted: its next buffer starts a new session
						live_remove(S, live, nlive, v);
						atomicAdd(&d.ctr[CTR_EVICTIONS], 1ull);
					}
					const uint32_t jj = ord[k - 1];
					S[h].live = 1;
					S[h].stamp = d.seq_base + slow_event(d, jj);
					live_add(S, live, nlive, h);
					atomicAdd(&d.ctr[CTR_INSERTS], 1ull);
				}
			}
			__syncthreads();
		}
	}
	// the sessions left in the LRU are saved for the next batch
	for (uint32_t x = t; x < nlive; x += kLruThreads) {
		const uint32_t h = live[x];
		if (h >= nslow) { // untouched carried session: saved unchanged
			const Carry& cr = d.carry_in[h - nslow];
			const unsigned long long c = atomicAdd(&d.ctr[CTR_CARRY_OUT], 1ull);
			if (c >= d.carry_cap) {
				set_error(d, EBD_ERR_LRU_OVERFLOW);
				continue;
			}
			Carry& out = d.carry_out[c];
			out.pid = cr.pid;
			out.fd = cr.fd;
			out.sid = cr.sid;
			out.stamp = cr.stamp;
			out.g = cr.g;
			out.nbytes = cr.nbytes;
			for (uint32_t b = 0; b < cr.nbytes; b++)
				out.bytes[b] = cr.bytes[b];
			continue;
		}
		uint32_t jl = h;
		const uint32_t slot = (uint32_t)(d.slow_keys[h] >> 32);
		while (jl + 1 < nslow && (uint32_t)(d.slow_keys[jl + 1] >> 32) == slot)
			jl++;
		session_carry_out(d, S[h], h, jl);
	}
}

// Aggregator::newRequest for the fast-path requests: coalesced reads of the results and keys
// k_fresh wrote (the client class is already in each result, Aggregator.cpp:50-88), one slot
// probe per request.  A block walks a contiguous range of the batch 256 events at a time, each
// wave its own 64 of them, and the waves never wait for each other: every step of a wave is a
// chain of dependent random accesses (slot probe, claim / counter atomics), and a block-wide
// barrier per step made each step last as long as the slowest of 256 chains.
//
// A service created here only claims its slot: the claim (slot, claiming event) goes to the
// block's own stretch of the claim stage, counted in LDS, with no global atomic.  The
// publication kernels then give every block's claims their list entries and arena bytes from
// a scan of the per-block counts (k_pub_count, k_pub_scan) and copy the endpoint bytes
// (k_publish).  A single global counter serialises at ~12 ns per atomic: reserving per block
// and step cost ~5 ms per 100 M-event batch that creates 30 M services.
struct AggShared {
	uint32_t cn; // claims of this block
	unsigned long long nreq;
};

__device__ __forceinline__ void agg_request(const Dev& d, uint32_t i, const ebd_event_result& r, uint32_t cls, AggShared& sh,
		unsigned long long net) {
	bool claimed;
	const Hash128 key = d.keys[i];
	const uint32_t slot = agg_insert(d, key, first_word(d.seq_base + i, (r.info & EBD_INFO_HTTPS) != 0, r.u.span.host_len),
			cls == CLS_INTERNAL, cls == CLS_EXTERNAL, &claimed);
	if (d.net_on && cls == CLS_EXTERNAL)
		agg_nets(d, slot, net);
	if (claimed) { // at most one claim per event: the block's stretch holds them all
		const uint32_t k = atomicAdd(&sh.cn, 1u);
		const unsigned long long at = (unsigned long long)blockIdx.x * d.cstage_per + k;
		d.cstage_slot[at] = slot;
		d.cstage_ev[at] = i;
	}
}

// Steps (of kAggThreads events) per block; the claim stage holds per * kAggThreads per block.
EBD_HD uint32_t agg_steps_per_block(uint32_t n, uint32_t grid) {
	const uint32_t steps = (n + kAggThreads - 1) / kAggThreads;
	return (steps + grid - 1) / grid;
}

// LDS words written by some lanes of a wave and then read by others: order the accesses.
__device__ __forceinline__ void wave_sync() {
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifndef EBD_AGG_WAVES
#define EBD_AGG_WAVES 8
#endif
__global__ __launch_bounds__(kAggThreads) __attribute__((amdgpu_waves_per_eu(EBD_AGG_WAVES, 8))) void k_agg_fast(Dev d) {
	__shared__ AggShared sh;
	if (threadIdx.x == 0) {
		sh.nreq = 0;
		sh.cn = 0;
	}
	__syncthreads();
	uint32_t cnt = 0;
	const uint32_t steps = (d.n + kAggThreads - 1) / kAggThreads;
	const uint32_t per = agg_steps_per_block(d.n, gridDim.x);
	const uint32_t s0 = min(steps, blockIdx.x * per), s1 = min(steps, s0 + per);
	for (uint32_t st = s0; st < s1; st++) {
		const uint32_t i = st * kAggThreads + threadIdx.x;
		if (i < d.n) {
			const ebd_event_result r = d.res[i];
			if (r.status == EBD_STATUS_FINISHED && !(r.info & EBD_INFO_SESSION)) {
				cnt++;
				const uint32_t cls = (r.info >> EBD_INFO_CLASS_SHIFT) & 3u;
				agg_request(d, i, r, cls, sh, d.net_on && cls == CLS_EXTERNAL ? request_net(d, i, r) : 0ull);
			}
		}
	}
	atomicAdd(&sh.nreq, (unsigned long long)cnt);
	__syncthreads();
	if (threadIdx.x == 0) {
		d.blk_cnt[blockIdx.x] = sh.cn;
		if (sh.nreq)
			atomicAdd(&d.ctr[CTR_REQUESTS], sh.nreq);
	}
}

// ---- publication of the services k_agg_fast created (one block per k_agg_fast block) ----
constexpr int kPubThreads = 256, kPubClaims = kPubThreads / 4;

__device__ __forceinline__ uint32_t claim_bytes(const Dev& d, uint32_t i) {
	const ebd_event_result r = d.res[i];
	return (r.u.span.host_len + r.u.span.url_len + 7u) & ~7u;
}

// Inclusive prefix of x over the block (kPubThreads); `part` is LDS scratch of 4 words.
__device__ __forceinline__ uint32_t block_scan(uint32_t x, uint32_t* part, uint32_t* total) {
	const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
	for (int o = 1; o < 64; o <<= 1) {
		const uint32_t y = __shfl_up(x, o, 64);
		if (lane >= (uint32_t)o)
			x += y;
	}
	if (lane == 63)
		part[wave] = x;
	__syncthreads();
	uint32_t before = 0, t = 0;
	for (uint32_t w = 0; w < kPubThreads / 64; w++) {
		before += w < wave ? part[w] : 0u;
		t += part[w];
	}
	__syncthreads(); // part may be rewritten by the next call
	*total = t;
	return before + x;
}

// The batch's sessions for k_walk: the sorted position of each one's first event.  A block
// takes tiles of kPubThreads * kHeadsPer positions, kHeadsPer consecutive ones per thread,
// and reserves its tile's heads with one atomic.
constexpr uint32_t kHeadsPer = 16;
__global__ __launch_bounds__(kPubThreads) void k_walk_heads(Dev d, uint32_t nslow) {
	__shared__ uint32_t part[kPubThreads / 64];
	__shared__ unsigned long long base;
	const uint64_t tile = (uint64_t)kPubThreads * kHeadsPer;
	for (uint64_t t0 = (uint64_t)blockIdx.x * tile; t0 < nslow; t0 += (uint64_t)gridDim.x * tile) {
		const uint64_t a = t0 + (uint64_t)threadIdx.x * kHeadsPer;
		uint32_t mask = 0;
		if (a < nslow) {
			uint32_t prev = a == 0 ? 0xffffffffu : (uint32_t)(d.slow_keys[a - 1] >> 32);
			for (uint32_t k = 0; k < kHeadsPer && a + k < nslow; k++) {
				const uint32_t s = (uint32_t)(d.slow_keys[a + k] >> 32);
				if (s != prev)
					mask |= 1u << k;
				prev = s;
			}
		}
		const uint32_t cnt = (uint32_t)__popc(mask);
		uint32_t total;
		const uint32_t incl = block_scan(cnt, part, &total);
		if (threadIdx.x == 0)
			base = atomicAdd(&d.ctr[CTR_HEADS], (unsigned long long)total);
		__syncthreads();
		uint32_t at = (uint32_t)base + incl - cnt;
		while (mask) {
			const uint32_t k = (uint32_t)__ffs(mask) - 1u;
			mask &= mask - 1u;
			d.heads[at++] = (uint32_t)(a + k);
		}
		__syncthreads(); // base is rewritten for the next tile
	}
}

// Pass 1: the arena bytes of each block's claims.
__global__ __launch_bounds__(kPubThreads) void k_pub_count(Dev d) {
	__shared__ uint32_t part[kPubThreads / 64];
	const uint32_t b = blockIdx.x, cn = d.blk_cnt[b];
	const unsigned long long at0 = (unsigned long long)b * d.cstage_per;
	unsigned long long sum = 0;
	for (uint32_t j = threadIdx.x; j < cn; j += kPubThreads)
		sum += claim_bytes(d, d.cstage_ev[at0 + j]);
	uint32_t total;
	block_scan((uint32_t)sum, part, &total);
	if (threadIdx.x == 0)
		d.blk_bytes[b] = total;
}

// Pass 2 (one block): each block's first list entry and arena offset; the list and arena grow.
__global__ __launch_bounds__(1024) void k_pub_scan(Dev d, uint32_t nblk) {
	__shared__ unsigned long long cs[1024], bs[1024];
	const uint32_t t = threadIdx.x;
	// nblk <= 2 * 1024: each thread sums two blocks, a Hillis-Steele scan over the pairs
	const uint32_t b0 = 2 * t, b1 = 2 * t + 1;
	const unsigned long long c0 = b0 < nblk ? d.blk_cnt[b0] : 0, c1 = b1 < nblk ? d.blk_cnt[b1] : 0;
	const unsigned long long y0 = b0 < nblk ? d.blk_bytes[b0] : 0, y1 = b1 < nblk ? d.blk_bytes[b1] : 0;
	cs[t] = c0 + c1;
	bs[t] = y0 + y1;
	__syncthreads();
	for (uint32_t o = 1; o < 1024; o <<= 1) {
		const unsigned long long a = t >= o ? cs[t - o] : 0, z = t >= o ? bs[t - o] : 0;
		__syncthreads();
		cs[t] += a;
		bs[t] += z;
		__syncthreads();
	}
	const unsigned long long lbase = d.ctr[CTR_SERVICES], abase = d.ctr[CTR_SARENA];
	const unsigned long long ce = cs[t] - c0 - c1, be = bs[t] - y0 - y1; // exclusive prefix of the pair
	if (b0 < nblk) {
		d.blk_lbase[b0] = lbase + ce;
		d.blk_abase[b0] = abase + be;
	}
	if (b1 < nblk) {
		d.blk_lbase[b1] = lbase + ce + c0;
		d.blk_abase[b1] = abase + be + y0;
	}
	__syncthreads();
	if (t == 0) {
		d.ctr[CTR_SERVICES] = lbase + cs[1023];
		d.ctr[CTR_SARENA] = abase + bs[1023];
	}
}

// Pass 3: list entries and endpoint bytes.  Four lanes per claim copy 8-byte pieces round
// robin (a claim's loads go out together); offset, pid and length go beside the list entry.
// The bytes are the claiming request's host + url: every request of the key has the same.
__global__ __launch_bounds__(kPubThreads) void k_publish(Dev d) {
	__shared__ uint32_t part[kPubThreads / 64];
	const uint32_t b = blockIdx.x, cn = d.blk_cnt[b], r = threadIdx.x & 3;
	const unsigned long long at0 = (unsigned long long)b * d.cstage_per;
	const unsigned long long lbase = d.blk_lbase[b];
	unsigned long long abase = d.blk_abase[b];
	for (uint32_t j0 = 0; j0 < cn; j0 += kPubClaims) { // uniform
		const uint32_t j = j0 + (threadIdx.x >> 2);
		uint32_t i = kNone, slot = 0, hl = 0, ul = 0;
		const uint8_t *host = d.payload, *url = d.payload;
		if (j < cn) {
			i = d.cstage_ev[at0 + j];
			slot = d.cstage_slot[at0 + j];
			const ebd_event_result res = d.res[i];
			const uint8_t* p = d.payload + d.off[i];
			host = p + res.u.span.host_off;
			hl = res.u.span.host_len;
			url = p + res.u.span.url_off;
			ul = res.u.span.url_len;
		}
		const uint32_t n = hl + ul;
		const uint32_t nb = (i != kNone && r == 0) ? ((n + 7u) & ~7u) : 0u; // counted once per claim
		uint32_t total;
		const uint32_t incl = block_scan(nb, part, &total);
		const uint32_t excl = __shfl(incl - nb, (int)((threadIdx.x & 63) & ~3u), 64); // the quad leader's
		if (i != kNone) {
			const unsigned long long ep_at = abase + excl, li = lbase + j;
			const bool fits = ep_at + n <= d.sarena_cap, listed = li < d.new_cap;
			if (fits) {
				unsigned long long* dst = (unsigned long long*)(d.sarena + ep_at);
				for (uint32_t oo = 8 * r; oo < n; oo += 32) {
					const unsigned long long A = gload8u(host + (oo < hl ? oo : 0));
					const unsigned long long B = gload8u(url + ((oo > hl && oo - hl < ul) ? oo - hl : 0));
					dst[oo >> 3] = endpoint_piece(hl, n, oo, A, B);
				}
			}
			if (r == 0) {
				if (!fits)
					set_error(d, EBD_ERR_ARENA_FULL);
				if (listed) {
					d.new_slots[li] = slot;
					d.list_ep[li] = fits ? ep_at : ~0ull;
					d.list_pl[li] = (unsigned long long)d.ev[i].pid | ((unsigned long long)n << 32);
				} else {
					set_error(d, EBD_ERR_TABLE_FULL);
				}
			}
		}
		abase += total;
	}
}

__global__ void k_verify(Dev d) {
	const unsigned long long nv = d.ctr[CTR_VERIFY];
	const uint32_t n = (uint32_t)(nv < d.verify_cap ? nv : d.verify_cap);
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x)
		if (d.slots[d.verify[k].slot].hi != d.verify[k].hi)
			set_error(d, EBD_ERR_COLLISION);
	if (blockIdx.x == 0 && threadIdx.x == 0) // the last kernel of a batch: batch totals into run totals
		d.ctr[CTR_EVICTIONS_TOTAL] += d.ctr[CTR_EVICTIONS];
}

__device__ __forceinline__ Slot empty_slot() {
	Slot s;
	s.tag = 0;
	s.hi = 0;
	s.first = ~0ull;
	s.pad0[0] = s.pad0[1] = 0;
	s.internal_clients = 0;
	s.external_clients = 0;
	s.nets[0] = s.nets[1] = s.nets[2] = 0;
	s.pad = 0;
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
		s->first_c = 0;
		s->carry = 0;
		s->visited = 0;
		s->last_ev = 0;
		s->pad = 0;
		s->pad2 = 0;
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
__global__ void k_collect(Dev d, ebd_service* out) {
	const unsigned long long n = min(d.ctr[CTR_SERVICES], (unsigned long long)d.new_cap);
	for (unsigned long long k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const Slot& s = d.slots[d.new_slots[k]];
		const unsigned long long ep = d.list_ep[k], pl = d.list_pl[k];
		const uint32_t hl = (uint32_t)(s.first & 0x7fffu);
		uint32_t doff = 0, dlen = 0;
		if (ep != ~0ull)
			host_domain(d.sarena + ep, hl, &doff, &dlen);
		ebd_service v;
		v.pid = (uint32_t)pl;
		v.internal_clients = s.internal_clients;
		v.external_clients = s.external_clients;
		v.https = (uint8_t)((s.first >> 15) & 1u);
		v.pad_[0] = v.pad_[1] = v.pad_[2] = 0;
		v.endpoint_off = ep;
		v.endpoint_len = (uint32_t)(pl >> 32);
		v.domain_off = doff;
		v.domain_len = dlen;
		v.host_len = hl;
		v.first_seq = s.first >> 16;
		v.key_lo = s.tag;
		v.key_hi = s.hi;
		v.nets_v4_16 = s.nets[0];
		v.nets_v4_24 = s.nets[1];
		v.nets_v6 = s.nets[2];
		v.pad2_ = 0;
		out[k] = v;
	}
}

// ---------------------------------------------------------------------------------
// Network counters: networkCountersCleaning, the network-counter clear, and the set dump.
// ---------------------------------------------------------------------------------
// Aggregator::networkCountersCleaning (A:182-209): an entry seen retention or more before
// now is erased (signed difference, like the steady_clock durations it restates).
__global__ void k_net_clean(Dev d, unsigned long long now, unsigned long long retention) {
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k <= d.net_mask; k += gridDim.x * blockDim.x) {
		NetEnt& e = d.nets[k];
		const unsigned long long t = e.time;
		if (e.key == 0 || t == 0 || (long long)(now - t) < (long long)retention)
			continue;
		e.time = 0;
		const uint32_t kind = (uint32_t)(e.key >> 62), slot = (uint32_t)(e.key >> 31) & 0x7fffffffu;
		atomicSub(&d.slots[slot].nets[kind - 1], 1u);
	}
}

// Aggregator::clear with network counters (A:138-149), step 1: the services that keep a
// non-empty map are copied out (slot words and endpoint bytes) before the table is emptied
// (step 2, k_clear_used), then re-inserted with zeroed client counters (step 3) and their map
// entries moved to the new slots in a fresh table (step 4).  The others are gone.
__global__ void k_keep_collect(Dev d, KeepRec* keep, unsigned long long* kbytes, unsigned long long kcap) {
	const unsigned long long n = d.ctr[CTR_SERVICES];
	for (unsigned long long k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const uint32_t si = d.new_slots[k];
		const Slot& s = d.slots[si];
		if ((s.nets[0] | s.nets[1] | s.nets[2]) == 0)
			continue;
		KeepRec r;
		r.tag = s.tag;
		r.hi = s.hi;
		r.first = s.first;
		const unsigned long long ep = d.list_ep[k], pl = d.list_pl[k];
		r.pid = (uint32_t)pl;
		r.ep_len = (uint32_t)(pl >> 32);
		r.old_slot = si;
		r.pad = r.pad2 = 0;
		r.nets[0] = s.nets[0];
		r.nets[1] = s.nets[1];
		r.nets[2] = s.nets[2];
		r.ep_off = ~0ull;
		const unsigned long long nb = (r.ep_len + 7u) & ~7u;
		const unsigned long long at = atomicAdd(&d.ctr[CTR_KEEP_BYTES], nb);
		if (ep != ~0ull && at + nb <= kcap) {
			const unsigned long long* src = (const unsigned long long*)(d.sarena + ep);
			for (unsigned long long w = 0; w < nb / 8; w++)
				kbytes[at / 8 + w] = src[w];
			r.ep_off = at;
		} else if (ep != ~0ull) {
			set_error(d, EBD_ERR_ARENA_FULL);
		}
		keep[atomicAdd(&d.ctr[CTR_KEEP], 1ull)] = r;
	}
}

__global__ void k_keep_insert(Dev d, const KeepRec* keep, const uint8_t* kbytes, uint32_t* remap) {
	const unsigned long long n = d.ctr[CTR_KEEP];
	for (unsigned long long k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const KeepRec r = keep[k];
		bool claimed;
		const uint32_t slot = agg_insert(d, Hash128{r.tag, r.hi}, r.first, 0, 0, &claimed);
		if (slot == kNone)
			continue;
		if (claimed) {
			const uint32_t len = r.ep_off == ~0ull ? 0 : r.ep_len;
			const uint8_t* ep = kbytes + (r.ep_off == ~0ull ? 0 : r.ep_off);
			const uint32_t hl = min((uint32_t)(r.first & 0x7fffu), len);
			claim_publish(d, slot, atomicAdd(&d.ctr[CTR_SERVICES], 1ull),
					atomicAdd(&d.ctr[CTR_SARENA], (unsigned long long)((len + 7u) & ~7u)), r.pid, ep, hl, ep + hl, len - hl);
		} else {
			set_error(d, EBD_ERR_INTERNAL); // kept keys are distinct and the table was empty
		}
		Slot& s = d.slots[slot];
		s.nets[0] = r.nets[0];
		s.nets[1] = r.nets[1];
		s.nets[2] = r.nets[2];
		remap[r.old_slot] = slot;
	}
}

// Live entries of the old table into the (zeroed) new one under their services' new slots
// (remap == nullptr: the same slots, a compaction).  Erased entries and the v6 prefixes only
// they used are dropped: a v6 prefix is re-interned from the old dictionary into d.v6d (a
// zeroed one), so neither table keeps more than the live map entries (Aggregator.cpp:182-209
// erases them; the maps hold at most one retention period of prefixes).
__global__ void k_net_remap(Dev d, const NetEnt* old, uint32_t old_mask, const uint32_t* remap,
		const unsigned long long* old_v6d) {
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k <= old_mask; k += gridDim.x * blockDim.x) {
		const NetEnt e = old[k];
		if (e.key == 0 || e.time == 0)
			continue;
		const uint32_t kind = (uint32_t)(e.key >> 62), slot = (uint32_t)(e.key >> 31) & 0x7fffffffu;
		const uint32_t ns = remap ? remap[slot] : slot;
		if (ns == kNone) { // a live entry belongs to a service with a non-empty map: kept
			set_error(d, EBD_ERR_INTERNAL);
			continue;
		}
		uint32_t v = (uint32_t)(e.key & 0x7fffffffu);
		if (kind == NET_V6) {
			v = v6d_index(d, old_v6d[v] & 0xffffffffffffull);
			if (v == kNone)
				continue;
		}
		NetEnt* ne = net_find_or_claim(d, d.nets, d.net_mask, net_key(kind, ns, v));
		if (ne)
			ne->time = e.time;
	}
}

// Every live map entry with its service's key and its prefix bytes (ebd_collect_networks).
__global__ void k_net_dump(Dev d, ebd_service_net* out, uint32_t cap, unsigned long long* count) {
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k <= d.net_mask; k += gridDim.x * blockDim.x) {
		const NetEnt e = d.nets[k];
		if (e.key == 0 || e.time == 0)
			continue;
		const unsigned long long at = atomicAdd(count, 1ull);
		if (at >= cap)
			continue;
		const uint32_t kind = (uint32_t)(e.key >> 62), slot = (uint32_t)(e.key >> 31) & 0x7fffffffu;
		const uint32_t v = (uint32_t)(e.key & 0x7fffffffu);
		unsigned long long pfx = kind == NET_V6 ? (d.v6d[v] & 0xffffffffffffull) : v;
		ebd_service_net r;
		r.key_lo = d.slots[slot].tag;
		r.key_hi = d.slots[slot].hi;
		r.kind = (uint8_t)kind;
		for (int b = 0; b < 6; b++)
			r.prefix[b] = (uint8_t)(pfx >> (8 * b));
		r.pad_ = 0;
		r.time_ns = e.time;
		out[at] = r;
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

// Config 4 (ebd_gen.h conn4_*): one thread per connection task t = slot * J + j.
__global__ void k_gen4_count(unsigned long long seed, uint32_t J, uint32_t* cnt) {
	const uint64_t tasks = (uint64_t)kSlots4 * J;
	for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < tasks; t += (uint64_t)gridDim.x * blockDim.x) {
		Conn4 c;
		conn4(seed, (t % J) * kSlots4 + t / J, c);
		cnt[t] = conn4_events(c);
	}
}

// Aligned piece length at every position < n (DATA_END: 0); st = exclusive scan of cnt.
__global__ void k_gen4_len(const GenTables* T, unsigned long long seed, uint32_t J, unsigned long long n, uint32_t align,
		const uint32_t* st, unsigned long long* alen) {
	const uint64_t tasks = (uint64_t)kSlots4 * J;
	for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < tasks; t += (uint64_t)gridDim.x * blockDim.x) {
		const uint32_t slot = (uint32_t)(t / J), j = (uint32_t)(t % J);
		const uint64_t r0 = st[t] - st[(uint64_t)slot * J];
		conn4_visit(*T, seed, slot, j, r0, n, [&](uint64_t p0, const Conn4&, const Req4* r, uint32_t) {
			if (!r) {
				alen[p0] = 0;
				return;
			}
			for (uint32_t f = 0; f < r->k && p0 + (uint64_t)f * kSlots4 < n; f++)
				alen[p0 + (uint64_t)f * kSlots4] = align_up(r->cut[f + 1] - r->cut[f], align);
		});
	}
}

__global__ void k_gen4_write(const GenTables* T, unsigned long long seed, uint32_t J, unsigned long long n, const uint32_t* st,
		const unsigned long long* boff, EventRec* ev, uint32_t* len, unsigned long long* off, uint8_t* payload,
		unsigned long long* gidx) {
	const uint64_t tasks = (uint64_t)kSlots4 * J;
	for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < tasks; t += (uint64_t)gridDim.x * blockDim.x) {
		const uint32_t slot = (uint32_t)(t / J), j = (uint32_t)(t % J);
		const uint64_t r0 = st[t] - st[(uint64_t)slot * J];
		conn4_visit(*T, seed, slot, j, r0, n, [&](uint64_t p0, const Conn4& c, const Req4* r, uint32_t e) {
			if (!r) {
				conn4_record(c, e, true, ev[p0]);
				len[p0] = EBD_NO_BUFFER;
				off[p0] = boff[p0];
				if (gidx)
					gidx[p0] = p0;
				return;
			}
			uint8_t* dst[4] = {nullptr, nullptr, nullptr, nullptr};
			for (uint32_t f = 0; f < r->k; f++) {
				const uint64_t p = p0 + (uint64_t)f * kSlots4;
				if (p >= n)
					break;
				dst[f] = payload + boff[p];
				conn4_record(c, e + f, false, ev[p]);
				len[p] = r->cut[f + 1] - r->cut[f];
				off[p] = boff[p];
				if (gidx)
					gidx[p] = p;
			}
			write_req4(*r, dst);
		});
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
// k_agg_fast's grid: the blocks that are resident at once (more would run as a second, partial
// round after the first; fewer leave the random-access latency exposed), at most 2048
// (k_pub_scan scans 2 per thread).
static uint32_t agg_blocks_per_cu() {
	static int bpc = 0;
	if (bpc <= 0) {
		int nb = 0;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_agg_fast, kAggThreads, 0) != hipSuccess || nb <= 0)
			nb = 4;
		bpc = nb;
	}
	return (uint32_t)bpc;
}
static uint32_t agg_grid(uint32_t n, int cus) {
	return (uint32_t)grid_for(n, kAggThreads, (int)min((uint32_t)cus * agg_blocks_per_cu(), 2048u));
} // k_pub_scan: <= 2048
uint32_t agg_stage_per_block(uint32_t n, int cus) { return agg_steps_per_block(n, agg_grid(n, cus)) * kAggThreads; }

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
hipError_t launch_lru_bound(const Dev& d, uint32_t nslow, int* delta, uint8_t* minus, int* scan, void* tmp, size_t tmp_bytes,
		hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_lru_delta, dim3(grid_for(nslow, 256, cus * 8)), dim3(256), 0, st, d, nslow, delta, minus);
	hipError_t e = hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, delta, scan, (int)d.n, st);
	if (e != hipSuccess)
		return e;
	hipLaunchKernelGGL(k_lru_peak, dim3(grid_for(d.n, 256, cus * 4)), dim3(256), 0, st, scan, minus, d.n, d.ctr);
	return hipGetLastError();
}
hipError_t launch_walk_lru(const Dev& d, uint32_t nslow, uint32_t* jpos, uint32_t* head, SessState* S, uint32_t* live,
		uint32_t cap, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_lru_index, dim3(grid_for(nslow, 256, cus * 8)), dim3(256), 0, st, d, nslow, jpos, head);
	hipLaunchKernelGGL(k_walk_lru, dim3(1), dim3(kLruThreads), 0, st, d, nslow, (const uint32_t*)jpos, (const uint32_t*)head, S,
			live, cap);
	return hipGetLastError();
}
size_t sess_state_bytes() { return sizeof(SessState); }
hipError_t launch_walk(const Dev& d, uint32_t nslow, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_walk_heads, dim3(grid_for(nslow, kPubThreads * kHeadsPer, cus * 4)), dim3(kPubThreads), 0, st, d, nslow);
	hipLaunchKernelGGL(k_walk, dim3(grid_for(nslow, kWalkThreads, cus * 4)), dim3(kWalkThreads), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_carry_pass(const Dev& d, hipStream_t st) {
	hipLaunchKernelGGL(k_carry_pass, dim3(grid_for(d.n_carry_in, 64, 256)), dim3(64), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_agg_fast(const Dev& d, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_agg_fast, dim3(agg_grid(d.n, cus)), dim3(kAggThreads), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_publish(const Dev& d, hipStream_t st, int cus) {
	const uint32_t g = agg_grid(d.n, cus);
	hipLaunchKernelGGL(k_pub_count, dim3(g), dim3(kPubThreads), 0, st, d);
	hipLaunchKernelGGL(k_pub_scan, dim3(1), dim3(1024), 0, st, d, g);
	hipLaunchKernelGGL(k_publish, dim3(g), dim3(kPubThreads), 0, st, d);
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
hipError_t launch_collect(const Dev& d, ebd_service* out, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_collect, dim3(cus * 8), dim3(256), 0, st, d, out);
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

hipError_t launch_net_clean(const Dev& d, unsigned long long now, unsigned long long retention, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_net_clean, dim3(grid_for((uint64_t)d.net_mask + 1, 256, cus * 8)), dim3(256), 0, st, d, now, retention);
	return hipGetLastError();
}
hipError_t launch_keep_collect(const Dev& d, KeepRec* keep, unsigned long long* kbytes, unsigned long long kcap, hipStream_t st,
		int cus) {
	hipLaunchKernelGGL(k_keep_collect, dim3(cus * 4), dim3(256), 0, st, d, keep, kbytes, kcap);
	return hipGetLastError();
}
hipError_t launch_keep_insert(const Dev& d, const KeepRec* keep, const uint8_t* kbytes, uint32_t* remap, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_keep_insert, dim3(cus * 4), dim3(256), 0, st, d, keep, kbytes, remap);
	return hipGetLastError();
}
hipError_t launch_net_remap(const Dev& d, const NetEnt* old, uint32_t old_mask, const uint32_t* remap,
		const unsigned long long* old_v6d, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_net_remap, dim3(grid_for((uint64_t)old_mask + 1, 256, cus * 8)), dim3(256), 0, st, d, old, old_mask, remap,
			old_v6d);
	return hipGetLastError();
}
hipError_t launch_net_dump(const Dev& d, ebd_service_net* out, uint32_t cap, unsigned long long* count, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_net_dump, dim3(grid_for((uint64_t)d.net_mask + 1, 256, cus * 8)), dim3(256), 0, st, d, out, cap, count);
	return hipGetLastError();
}

hipError_t launch_gen4_count(unsigned long long seed, uint32_t J, uint32_t* cnt, hipStream_t st) {
	hipLaunchKernelGGL(k_gen4_count, dim3(grid_for((uint64_t)kSlots4 * J, 256, 8192)), dim3(256), 0, st, seed, J, cnt);
	return hipGetLastError();
}
hipError_t launch_gen4_len(const GenTables* T, unsigned long long seed, uint32_t J, unsigned long long n, uint32_t align,
		const uint32_t* stt, unsigned long long* alen, hipStream_t st) {
	hipLaunchKernelGGL(k_gen4_len, dim3(grid_for((uint64_t)kSlots4 * J, 256, 8192)), dim3(256), 0, st, T, seed, J, n, align, stt, alen);
	return hipGetLastError();
}
hipError_t launch_gen4_write(const GenTables* T, unsigned long long seed, uint32_t J, unsigned long long n, const uint32_t* stt,
		const unsigned long long* boff, EventRec* ev, uint32_t* len, unsigned long long* off, uint8_t* payload,
		unsigned long long* gidx, hipStream_t st) {
	hipLaunchKernelGGL(k_gen4_write, dim3(grid_for((uint64_t)kSlots4 * J, 256, 8192)), dim3(256), 0, st, T, seed, J, n, stt, boff, ev,
			len, off, payload, gidx);
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
