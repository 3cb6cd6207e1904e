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
#include "ebd_scan.h"

namespace ebd {

__device__ __forceinline__ void set_error(const Dev& d, unsigned long long bit) { atomicOr(&d.ctr[CTR_ERRORS], bit); }

// A saved buffer the kernels may read: at most EBD_BUFFER_MAX_DATA_SIZE long and inside the
// batch's payload.  An event whose buffer is not is handled as one whose buffer is missing
// (Discovery.cpp:103-107); k_fresh reports it as EBD_ERR_BAD_INPUT.
__device__ __forceinline__ bool buf_in(const Dev& d, uint32_t L, unsigned long long off) {
	return L <= EBD_BUFFER_MAX_DATA_SIZE && off <= d.payload_bytes && L <= d.payload_bytes - off;
}

// A global counter bumped by the active lanes of a wave together: one atomic for the wave
// instead of one per lane (a hot counter serialises its atomics at the memory side; the
// session path bumps several per event).  Returns this lane's offset: the counter's value
// before the wave plus the sizes of the active lanes below this one.  Works in divergent
// code: only the lanes active at the call take part.
__device__ __forceinline__ unsigned long long wave_add(unsigned long long* ctr, unsigned long long size) {
	const unsigned long long act = __ballot(1);
	const uint32_t lane = __lane_id(), leader = (uint32_t)__ffsll((long long)act) - 1u;
	unsigned long long pre = 0, tot = 0;
	if (__ballot(size != 1ull) == 0) { // every size 1 (a constant 1 folds to this path): ranks by mbcnt
		pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
		tot = (unsigned long long)__popcll(act);
	} else if (act == ~0ull) { // a full wave: a log-step inclusive scan
		unsigned long long x = size;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			const unsigned long long y = __shfl_up(x, (unsigned)o);
			x += lane >= (uint32_t)o ? y : 0ull;
		}
		pre = x - size;
		tot = __shfl(x, 63);
	} else {
		for (unsigned long long m = act; m; m &= m - 1) { // uniform: the active lanes' sizes, in lane order
			const uint32_t l = (uint32_t)__ffsll((long long)m) - 1u;
			const unsigned long long v = __shfl(size, (int)l);
			pre += l < lane ? v : 0ull;
			tot += v;
		}
	}
	unsigned long long base = 0;
	if (lane == leader)
		base = atomicAdd(ctr, tot);
	return __shfl(base, (int)leader) + pre;
}

// LDS words written by some lanes of a wave and then read by others: order the accesses.
__device__ __forceinline__ void wave_sync() {
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A global list grown by a whole 256-thread block at once: x = this thread's entries; returns
// the index of its first one.  One atomic per call for the block: a list counter takes about
// 88 returning atomics per microsecond (MI355X_MICROARCH.md, dequeue), so a wave_add per wave
// and step held k_slow_collect at that rate (1.25 M atomics, 15 ms per 80 M-event poll cycle).
// Every thread of the block calls it (barriers); part: LDS scratch of 4 words.
__device__ __forceinline__ unsigned long long block_reserve(unsigned long long* ctr, uint32_t x, uint32_t* part,
		unsigned long long* base) {
	const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
	uint32_t incl = x;
	for (int o = 1; o < 64; o <<= 1) {
		const uint32_t y = __shfl_up(incl, o, 64);
		if (lane >= (uint32_t)o)
			incl += y;
	}
	if (lane == 63)
		part[wave] = incl;
	__syncthreads();
	uint32_t before = 0, total = 0;
	for (uint32_t w = 0; w < 4; w++) {
		before += w < wave ? part[w] : 0u;
		total += part[w];
	}
	if (threadIdx.x == 0)
		*base = total ? atomicAdd(ctr, (unsigned long long)total) : 0ull;
	__syncthreads();
	return *base + before + incl - x; // base and part are rewritten only after the next call's first barrier
}

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
typedef unsigned short u16a1 __attribute__((aligned(1)));
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

// The next slot of a probe: linear, wrapping inside the key's range of probe_mask + 1 slots (the
// whole table, or the 2048-slot range one k_own workgroup holds in LDS).
__device__ __forceinline__ uint32_t probe_next(const Dev& d, uint32_t idx) {
	return (idx & ~d.probe_mask) | ((idx + 1) & d.probe_mask);
}

// Returns the slot (kNone when the table is full); *claimed: this call created the service.
// inc_int / inc_ext: the counter increments (one request: its class; a merged record: its counts).
__device__ uint32_t agg_insert(const Dev& d, Hash128 h, unsigned long long first, uint32_t inc_int, uint32_t inc_ext,
		bool* claimed) {
	uint32_t idx = (uint32_t)h.lo & d.slot_mask;
	bool found = false;
	*claimed = false;
	unsigned long long seen_first = 0;
	for (uint32_t probe = 0; probe <= d.probe_mask; probe++) {
		Slot* s = d.slots + idx;
		// One plain load pass over the slot's first 32 bytes.  tag and hi are written once
		// (0 -> value), first only decreases: a stale copy at worst shows 0 (resolved by
		// the CAS below, or the coherent re-read of hi) or a larger first (a redundant
		// atomicMin).  Slot words are only ever written by atomics here, so no dirty line
		// sits in L2 when the next kernel starts.
		const ulonglong2 th = *(const ulonglong2*)&s->tag;
		const ulonglong2 mo = *(const ulonglong2*)&s->nfirst;
		seen_first = ~mo.x;
		unsigned long long t = th.x;
		if (t == 0) {
			t = atomicCAS(&s->tag, 0ull, h.lo);
			if (t == 0) {
				atomicExch(&s->hi, h.hi); // (a write-through store instead was slower: DESIGN.md round 5)
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
		idx = probe_next(d, idx);
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
		atomicMax(&s->nfirst, ~first); // the slot keeps ~first: an empty slot is all zeros
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

__device__ void net_touch(const Dev& d, uint32_t slot, uint32_t kind, uint32_t value, unsigned long long now) {
	NetEnt* e = net_find_or_claim(d, d.nets, d.net_mask, net_key(kind, slot, value));
	if (e && atomicMax(&e->time, now) == 0) // new, or erased by networkCountersCleaning
		atomicAdd(&d.slots[slot].nets[kind - 1], 1u);
}

// incrementServiceClientsNumber's network part for an external client (net: net_pack).
// Aggregator::getCurrentTime of the request finished by event i: the event's own reading when
// the batch carries them (ebd_set_event_clock), else the batch's.
// A map entry's time 0 means "erased", so a reading of 0 counts as 1 (the batch clock is >= 1 too).
__device__ __forceinline__ unsigned long long request_time(const Dev& d, uint32_t i) {
	return d.times ? max(d.times[i], 1ull) : d.now;
}

__device__ void agg_nets(const Dev& d, uint32_t slot, unsigned long long net, unsigned long long now) {
	if (slot == kNone)
		return;
	if (net & kNetV6) {
		const uint32_t v = v6d_index(d, net & 0xffffffffffffull);
		if (v != kNone)
			net_touch(d, slot, NET_V6, v, now);
	} else {
		net_touch(d, slot, NET_V4_24, (uint32_t)(net & 0xffffffu), now);
		net_touch(d, slot, NET_V4_16, (uint32_t)(net & 0xffffu), now);
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
// *claimed: the slot this call claimed (for the dirty list), else kNone.
__device__ int sset_insert(const Dev& d, uint32_t pid, uint32_t fd, uint32_t sid, uint32_t carry, uint32_t ev, uint32_t* claimed) {
	const unsigned long long kv = ((unsigned long long)fd << 32) | pid;
	const unsigned long long tag = sset_tag(kv, sid);
	const uint32_t mask = *d.sset_mask;
	uint32_t idx = (uint32_t)tag & mask;
	int res = -1;
	for (uint32_t probe = 0; probe <= mask; probe++) {
		SSlot* s = d.sset + idx;
		unsigned long long t = ld_relaxed(&s->tag);
		if (t == 0) {
			t = atomicCAS(&s->tag, 0ull, tag);
			if (t == 0) {
				s->kv = kv;
				s->sid = sid;
				*claimed = idx;
				t = tag;
			}
		}
		if (t == tag) {
			res = (int)idx;
			break;
		}
		idx = (idx + 1) & mask;
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
	const uint32_t mask = *d.sset_mask;
	uint32_t idx = (uint32_t)tag & mask;
	for (uint32_t probe = 0; probe <= mask; probe++) {
		const SSlot* s = d.sset + idx;
		const unsigned long long t = s->tag;
		if (t == 0)
			return -1;
		if (t == tag) {
			if (s->kv == kv && s->sid == sid)
				return (int)idx;
			set_error(d, EBD_ERR_COLLISION); // two sessions share a 64-bit tag
		}
		idx = (idx + 1) & mask;
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
// Logical index (s << 8) | b into the LDS image (ebd_dfa.h: byte-major, kLdsStride).
struct LdsTable {
	const uint8_t* t;
	__device__ __forceinline__ uint32_t operator[](uint32_t i) const { return t[min(i & 0xffu, kLdsCols - 1) * kLdsStride + (i >> 8)]; }
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

#ifndef EBD_FRESH_THREADS
#define EBD_FRESH_THREADS 1024
#endif
#ifndef EBD_FRESH_WGS
#define EBD_FRESH_WGS 1 // workgroups per CU
#endif
constexpr int kFreshThreads = EBD_FRESH_THREADS;
constexpr int kFreshWaves = kFreshThreads / 64;
#ifndef EBD_SCAN_WAVES
#define EBD_SCAN_WAVES 12
#endif
// waves [0, kScanWaves) scan; the others finalize.  The split balances the scan against the
// finalize batches (which wait on the words past the staged bytes that the record does not
// carry).  Round 5 (finalize also classified the source address): 11 + 5 took 2.84 ms per 20 M
// config-3 events against 3.03 for 10 + 6, 3.20 for 9 + 7 and 3.14 for 12 + 4.  Round 6, with
// the class moved to k_agg_fast: 12 + 4 2.69-2.72 ms against 2.84-2.86 for 11 + 5, 2.96 for
// 10 + 6 and 3.10-3.16 for 13 + 3 (config 4's poll cycle: 5.13 against 5.04 ms).
constexpr int kScanWaves = EBD_SCAN_WAVES;
constexpr int kPfWaves = 0;
constexpr int kFinWaves = kFreshWaves - kScanWaves - kPfWaves;
constexpr uint32_t kScanLanes = kScanWaves * 64, kFinLanes = kFinWaves * 64;
#ifndef EBD_RING
#define EBD_RING 128
#endif
constexpr uint32_t kRing = EBD_RING; // finalize records in flight per workgroup
// A push covers up to 64 consecutive positions and a finalize wave frees its 64 only when
// all are ready: a ring of fewer than 2 x 64 slots can leave a push waiting on a slot whose
// finalize wave waits on that same push.  Slots are pos & (kRing - 1).
static_assert(kRing >= 128 && (kRing & (kRing - 1)) == 0, "ring: a power of two of at least 128 slots");

// LDS address of entry (s, byte k of word x): v_bfe (off the state chain) + v_mad_u32_u24.
__device__ __forceinline__ uint32_t tab_index(uint32_t s, uint32_t x, int k) {
	return min(__builtin_amdgcn_ubfe(x, 8 * (k & 3), 8), kLdsCols - 1) * kLdsStride + s;
}

// Every byte of w in [0x20, 0x7e] (SWAR: no byte < 0x20, none >= 0x7f; exact tests).
__device__ __forceinline__ bool printable4(uint32_t w) {
	const uint32_t lt = (w - 0x20202020u) & ~w & 0x80808080u;
	const uint32_t ge = ((w + 0x01010101u) | w) & 0x80808080u;
	return (lt | ge) == 0;
}

// 16 DFA steps over one chunk: s advances, m = the maximum next state, qs = the states at
// the quarter starts (s0 | s4 << 8 | s8 << 16 | s12 << 24), qm = running maxima after 4, 8
// and 12 steps (ebd_fresh.h chunk_update).  (Skipping a printable quarter in a generic
// header-value state was measured slower: exec-masked, the wave still waits for the lanes
// that step)
__device__ __forceinline__ void scan_chunk(const uint8_t* T, const Chunk& w, uint32_t& s, uint32_t& m, uint32_t& qs, uint32_t& qm) {
	qs = s;
	m = 0;
#pragma unroll
	for (int q = 0; q < 4; q++) {
		const uint32_t x = w.w[q];
#pragma unroll
		for (int k = 0; k < 4; k++) {
			s = T[tab_index(s, x, k)];
			m = max(m, s);
		}
		if (q < 3) {
			qs |= s << (8 * (q + 1));
			qm = q == 0 ? m : (qm | (m << (8 * q)));
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
// The buffer is read in 64-byte windows.  A 16-byte aligned buffer's windows lie on the 64-byte
// grid of the address space (each a whole half line, measured 4.3 TB/s against 3.6 TB/s for
// buffer-relative windows with a trivial consumer, tools/ubench_stream.hip): window w holds
// the pieces [4w, 4w + 4) counted from `base` = the buffer's 64-byte line half, of which
// the first j0 precede the buffer.  Other buffers use buffer-relative windows (j0 = 0).
struct LaneEv {
	uint32_t idx;
	uint32_t L;  // buffer length (0 unless EK_PARSE)
	uint32_t pf; // pid (the DiscoveryEvent's, Discovery.cpp:136, 157)
	uint32_t m;  // kind | j0 << 2 | flags << 8; j0 = pieces of window 0 before the buffer
	unsigned long long base; // window 0's first byte (a harmless valid address unless EK_PARSE)
	__device__ __forceinline__ uint32_t kind() const { return m & 3u; }
	__device__ __forceinline__ uint32_t j0() const { return (m >> 2) & 3u; }
	__device__ __forceinline__ uint32_t flags() const { return m >> 8; }
	// the buffer's last piece, counted from base
	__device__ __forceinline__ uint32_t lastp() const { return L ? (16u * j0() + L - 1u) >> 4 : 0u; }
	__device__ __forceinline__ const uint8_t* p() const { return (const uint8_t*)(uintptr_t)(base + 16u * j0()); }
};

// An event's words as loaded (lane_ev decodes them).  Decoding the next event only where it
// is first needed (a window later) was measured slower: 3.02 against 2.90 ms per 20 M config-3
// events, same box.  The source address is not carried: finalize reads it from the event.
struct LaneRaw {
	uint32_t idx, pf, flags, len, past; // past: beyond the workgroup's range (no event)
	unsigned long long off;
};

// Branch-free: an index past the range loads event 0's words (and is marked so), so every call
// issues the same four loads and the scan loop's memory counter waits stay exact.
__device__ __forceinline__ LaneRaw lane_load(const Dev& d, uint32_t i, uint32_t end) {
	LaneRaw r;
	r.idx = i;
	const uint32_t j = i < end ? i : 0u;
	const uint8_t* evb = (const uint8_t*)(d.ev + j);
	r.past = i < end ? 0u : 1u; // kept apart from the loaded words: nothing here waits for them
	r.flags = evb[32];
	r.pf = *(const uint32_t*)evb;
	r.len = d.len[j];
	r.off = d.off[j];
	return r;
}

__device__ __forceinline__ LaneEv lane_ev(const Dev& d, const LaneRaw& r) {
	LaneEv e;
	e.idx = r.idx;
	if (r.past) {
		e.m = EK_NONE;
		e.L = 0;
		e.pf = 0;
		e.base = (unsigned long long)(uintptr_t)d.payload;
		return e;
	}
	const uint32_t flags = r.flags;
	e.pf = r.pf;
	const uint32_t L = r.len;
	const uint64_t off = r.off;
	const uint32_t kind = !(flags & FLAG_NEW) || L == EBD_NO_BUFFER ? EK_SKIP : !buf_in(d, L, off) ? EK_BAD : EK_PARSE;
	e.L = kind == EK_PARSE ? L : 0;
	const uint8_t* p = kind == EK_PARSE ? d.payload + off : d.payload;
	// the 64-byte grid when the buffer is 16-byte aligned and its line half stays inside the
	// readable allocation (from the 16-byte boundary at or below payload, ebpf_discovery_amd.h)
	const unsigned long long a = (unsigned long long)(uintptr_t)p, a64 = a & ~63ull;
	const bool grid = (a & 15u) == 0 && a64 >= ((unsigned long long)(uintptr_t)d.payload & ~15ull);
	const uint32_t j0 = grid ? (uint32_t)((a & 63u) >> 4) : 0u;
	e.base = grid ? a64 : a;
	e.m = kind | (j0 << 2) | (flags << 8);
	return e;
}

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
	d.ev_slot[wave_add(&d.ctr[CTR_UNFINISHED], 1ull)] = i; // k_sset_build inserts its session
	(void)ev;
}

// A finished scan waiting for fresh_finalize: 16 words, kept in the ring as 16 arrays of
// kRing words (structure of arrays), so the 64 lanes of a push or of a finalize wave, which
// hold consecutive ring positions, touch consecutive words: no LDS bank conflicts (a 64-B
// record per lane made every access 16-way conflicted).
enum : uint32_t {
	R_PLO,  // buffer address bits 0..31
	R_PHI,  // buffer address bits 32..47 | L << 16
	R_IDX,  // event index
	R_PID,
	R_SF,   // final state | flags << 8 | cseen << 16 | post << 17
	R_CQM,
	R_C01,  // url.c | host.c << 16
	R_C23,  // hend.c | cip.c << 16
	R_C4,   // term.c
	R_QS,   // qs[0..4] (url, host, hend, cip, term)
	R_LIM = R_QS + 5, // staged leading bytes that are valid
	R_POS,  // ring position + 1 (checked by finalize)
	R_TW,   // the 4 bytes the terminal tracker's rescan needs, from the scan lane's registers
	R_WORDS
};
static_assert(R_WORDS == 17, "finalize record is 17 words");

// Leading buffer bytes a scan lane stages (window 0), carried to finalize in LDS so that it
// reads the request line and usually the Host header from LDS instead of reloading lines
// that left L2 while the lane scanned the rest of the buffer.  Rows are structure of
// arrays too: word j of the row of lane (or slot) l at [j * stride + l], one row of slack.
#ifndef EBD_STAGE
#define EBD_STAGE 96 // window 0 and the first half of window 1 (the request line and, mostly, Host)
#endif
constexpr uint32_t kStage = EBD_STAGE, kStageWords = kStage / 4;
static_assert(kStage >= 64 && kStage <= 128 && kStage % 16 == 0, "staging: window 0 plus whole chunks of window 1");

// Buffer bytes for fresh_finalize: offsets [0, lim) from the staged copy (word j at
// s[j * kFinLanes]), the rest from the buffer in global memory.
struct StagedMem {
	const uint8_t* p;
	const uint32_t* s;
	uint32_t lim;
	uint32_t two, tw; // the word at buffer offset two, carried in the record (R_TW)
	__device__ __forceinline__ uint32_t lds4(uint32_t o) const {
		return __builtin_amdgcn_alignbyte(s[((o >> 2) + 1) * kFinLanes], s[(o >> 2) * kFinLanes], o & 3u);
	}
	__device__ __forceinline__ uint32_t ld4(uint32_t o) const {
		if (o == two)
			return tw;
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

__device__ __forceinline__ uint32_t lds_load_acq(const uint32_t* p) {
	return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store_rel(uint32_t* p, uint32_t v) {
	__hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Workgroup state shared by the scan and finalize waves.
struct FreshShared {
	uint32_t ring[R_WORDS * kRing];
	uint32_t ready[kRing]; // position + 1 once the slot's record is written
	uint32_t freed[kRing]; // position + 1 once the slot's record is taken
	uint32_t rdata[(kStageWords + 1) * kRing];      // staged bytes of each slot's record
	uint32_t stage[kStageWords * kScanLanes];       // a scan lane's current buffer, as scanned
	uint32_t fstage[(kStageWords + 1) * kFinLanes]; // a finalize lane's record's bytes
	uint32_t unf[kFinWaves][128];                   // each finalize wave's UNFINISHED events not yet listed
	uint32_t next_ev;   // next event of the workgroup's range
	uint32_t tail;      // positions handed out to scan lanes
	uint32_t claim;     // positions handed out to finalize waves
	uint32_t scan_done; // scan waves that finished
};
static_assert(sizeof(FreshShared) + kLdsTableBytes <= 160 * 1024, "k_fresh LDS fits one CU");

// fresh_finalize (ebd_fresh.h) for the record in the lane's registers; the lane's staged
// bytes are at fs (word j at fs[j * kFinLanes]).
// Returns true for an UNFINISHED parse: its session may be saved (Discovery.cpp:148-150), and
// the caller lists the event for k_sset_build.
__device__ __forceinline__ bool finalize_rec(const Dev& d, const uint8_t* T, const uint32_t (&q)[R_WORDS], const uint32_t* fs) {
	const uint8_t* p = (const uint8_t*)(uintptr_t)((unsigned long long)q[R_PLO] | ((unsigned long long)(q[R_PHI] & 0xffffu) << 32));
	const uint32_t L = q[R_PHI] >> 16;
	const uint32_t i = q[R_IDX];
	if (i >= d.n || L > EBD_BUFFER_MAX_DATA_SIZE || (unsigned long long)(p - d.payload) >> 40) {
		set_error(d, EBD_ERR_INTERNAL); // a record that cannot be real: reported, never followed
		return false;
	}
	ScanRec sr;
	sr.url = Trk{q[R_C01] & 0xffffu, q[R_QS + 0]};
	sr.host = Trk{q[R_C01] >> 16, q[R_QS + 1]};
	sr.hend = Trk{q[R_C23] & 0xffffu, q[R_QS + 2]};
	sr.cip = Trk{q[R_C23] >> 16, q[R_QS + 3]};
	sr.term = Trk{q[R_C4], q[R_QS + 4]};
	sr.cqm = q[R_CQM];
	sr.cseen = (q[R_SF] >> 16) & 1u;
	FreshResult fr;
	// the terminal tracker's word travels in the record: it lies at the end of the request,
	// past the staged bytes, where a reload from HBM cost one line per event
	const uint32_t two = 16 * sr.term.c + 4 * flip_quarter<RS_TERM>(d.di, sr.term, 0);
	fresh_finalize(LdsTable{T}, d.di, sr, q[R_SF] & 0xffu, ((q[R_SF] >> 17) & 1u) != 0, StagedMem{p, fs, q[R_LIM], two, q[R_TW]}, L,
			d.hkey, q[R_PID], (uint8_t)(q[R_SF] >> 8), fr);
	// the client's class (source address or client-IP token) is k_agg_fast's: it reads the
	// event records in event order, whole lines, where a read here came back from HBM
	if (fr.r.status == EBD_STATUS_FINISHED)
		d.keys[i] = fr.key;
	d.res[i] = fr.r;
	return fr.r.status == EBD_STATUS_UNFINISHED;
}

// The table first: LDS address = table index, so a step's read needs no base add.
struct FreshLds {
	uint8_t T[kLdsTableBytes];
	FreshShared sh;
};

__global__ __launch_bounds__(kFreshThreads)
#if EBD_FRESH_WGS > 1
__attribute__((amdgpu_waves_per_eu(EBD_FRESH_WGS * kFreshThreads / 256, 8)))
#endif
void k_fresh(Dev d) {
	__shared__ __attribute__((aligned(16))) FreshLds lds;
	uint8_t* T = lds.T;
	FreshShared& sh = lds.sh;
	const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 3;
	// this workgroup's contiguous share of the batch
	const uint32_t per = (uint32_t)(((unsigned long long)d.n + gridDim.x - 1) / gridDim.x);
	const uint32_t rb = min(d.n, blockIdx.x * per), re = min(d.n, rb + per);
	for (uint32_t k = threadIdx.x * 16u; k < kLdsTableBytes; k += kFreshThreads * 16u)
		*(uint4*)(T + k) = *(const uint4*)(d.dfa + k);
	for (uint32_t k = threadIdx.x; k < kRing; k += kFreshThreads)
		sh.ready[k] = sh.freed[k] = 0;
	if (threadIdx.x == 0) {
		sh.next_ev = rb + kScanLanes * 2;
		sh.tail = sh.claim = sh.scan_done = 0;
	}
	__syncthreads();
	const DfaInfo& di = d.di;


	if (wave >= kScanWaves) {
		// ---- finalize waves: 64 records at a time, in position order ----
		const uint32_t fl = (wave - kScanWaves) * 64 + lane; // finalize lane
		uint32_t* fs = sh.fstage + fl;
		// UNFINISHED events go to ev_slot 64 at a time, one atomic each (a wave_add per batch of
		// records held config-4 poll cycles, ~30 % of them UNFINISHED, at the counter's rate)
		uint32_t* ust = sh.unf[wave - kScanWaves];
		uint32_t uh = 0, un = 0; // wave-uniform: ring head and entries
		for (;;) {
			uint32_t c = 0;
			if (lane == 0)
				c = atomicAdd(&sh.claim, 64u);
			c = __builtin_amdgcn_readfirstlane(c);
			const uint32_t pos = c + lane, slot = pos & (kRing - 1);
			// 0: waiting, 1: the record is ready, 2: the scan ended before this position.
			// The wave polls as a whole (a uniform loop): one conflict-free LDS read per lane
			// and one lane reading the scan counters, then a sleep.
			uint32_t st = 0;
			for (;;) {
				if (st == 0 && lds_load_acq(&sh.ready[slot]) == pos + 1)
					st = 1;
				if (__all(st != 0))
					break;
				uint32_t done = 0, tail = 0;
				if (lane == 0) {
					done = lds_load_acq(&sh.scan_done);
					tail = lds_load_acq(&sh.tail);
				}
				done = __builtin_amdgcn_readfirstlane(done);
				tail = __builtin_amdgcn_readfirstlane(tail);
				if (done == (uint32_t)kScanWaves) { // every position below tail was pushed
					if (st == 0 && pos >= tail)
						st = 2;
					if (__all(st != 0))
						break;
				}
				__builtin_amdgcn_s_sleep(4);
			}
			if (!__any(st == 1))
				break;
			uint32_t q[R_WORDS];
			if (st == 1) {
#pragma unroll
				for (uint32_t f = 0; f < R_WORDS; f++)
					q[f] = sh.ring[f * kRing + slot];
#pragma unroll
				for (uint32_t j = 0; j < kStageWords; j++) // the staged bytes move to this lane's row
					fs[j * kFinLanes] = sh.rdata[j * kRing + slot];
				lds_store_rel(&sh.freed[slot], pos + 1); // the slot may be written again
			}
			bool unf = false;
			if (st == 1) {
				if (q[R_POS] != pos + 1)
					set_error(d, EBD_ERR_INTERNAL); // ring protocol violated: reported, not followed
				else
					unf = finalize_rec(d, T, q, fs);
			}
			const unsigned long long b = __ballot(unf);
			if (unf)
				ust[(uh + un + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0))) & 127u] = q[R_IDX];
			un += (uint32_t)__popcll(b);
			if (un >= 64) {
				wave_sync();
				unsigned long long at = 0;
				if (lane == 0)
					at = atomicAdd(&d.ctr[CTR_UNFINISHED], 64ull);
				at = __shfl(at, 0);
				d.ev_slot[at + lane] = ust[(uh + lane) & 127u];
				uh += 64;
				un -= 64;
				wave_sync(); // the words just read may be rewritten
			}
		}
		wave_sync();
		if (un) {
			unsigned long long at = 0;
			if (lane == 0)
				at = atomicAdd(&d.ctr[CTR_UNFINISHED], (unsigned long long)un);
			at = __shfl(at, 0);
			if (lane < un)
				d.ev_slot[at + lane] = ust[(uh + lane) & 127u];
		}
		return;
	}

	// ---- scan waves ----
	const uint32_t sl = wave * 64 + lane; // scan lane
	uint32_t* stg = sh.stage + sl;        // this lane's staging row (word j at stg[j * kScanLanes])
	auto grab = [&]() -> uint32_t { return atomicAdd(&sh.next_ev, 1u); };
	// The lane's current event (e0) and the next one (e1, decoded: its first window is loaded
	// while e0's last one is scanned).  Holding a third event's words as loaded, decoded only at
	// the next hand-off so that a hand-off never waits for the loads it issues, was measured
	// neutral: 2.97-3.02 against 2.98 ms per 20 M config-3 events (round 5, same box).
	LaneEv e0 = lane_ev(d, lane_load(d, rb + sl, re));
	LaneEv e1 = lane_ev(d, lane_load(d, rb + kScanLanes + sl, re));
	uint32_t w0 = 0; // e0's window to scan next
	uint32_t s = di.init, live = 0;
	ScanRec sr;
	rec_init(di, sr);

	// Hands e0's scan record to the finalize waves when `done`; tw: the terminal tracker's word.
	auto push = [&](bool done, uint32_t tw) {
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
			// staged bytes equal the buffer's up to the loaded windows and the last chunk's end
			const uint32_t scanned = min(64u * w0 - 16u * e0.j0(), kStage), chunks_end = (e0.L + 15u) & ~15u;
			const uint32_t post = (stg[0] & 0xffu) == 'P' ? 1u : 0u; // the method's first byte
			const unsigned long long a = (unsigned long long)(uintptr_t)e0.p();
			uint32_t t[R_WORDS];
			t[R_PLO] = (uint32_t)a;
			t[R_PHI] = ((uint32_t)(a >> 32) & 0xffffu) | (e0.L << 16);
			t[R_IDX] = e0.idx;
			t[R_PID] = e0.pf;
			t[R_SF] = s | (e0.flags() << 8) | (sr.cseen << 16) | (post << 17);
			t[R_CQM] = sr.cqm;
			t[R_C01] = sr.url.c | (sr.host.c << 16);
			t[R_C23] = sr.hend.c | (sr.cip.c << 16);
			t[R_C4] = sr.term.c;
			t[R_QS + 0] = sr.url.qs;
			t[R_QS + 1] = sr.host.qs;
			t[R_QS + 2] = sr.hend.qs;
			t[R_QS + 3] = sr.cip.qs;
			t[R_QS + 4] = sr.term.qs;
			t[R_LIM] = min(scanned, chunks_end);
			t[R_POS] = pos + 1;
			t[R_TW] = tw;
#pragma unroll
			for (uint32_t f = 0; f < R_WORDS; f++)
				sh.ring[f * kRing + slot] = t[f];
#pragma unroll
			for (uint32_t j = 0; j < kStageWords; j++)
				sh.rdata[j * kRing + slot] = stg[j * kScanLanes];
			lds_store_rel(&sh.ready[slot], pos + 1);
		}
	};
	// Moves on while e0 needs no scan: such events are resolved here.
	auto resolve = [&]() {
		for (;;) {
			if (e0.kind() == EK_SKIP) {
				write_none(d, e0.idx);
			} else if (e0.kind() == EK_BAD) {
				set_error(d, EBD_ERR_BAD_INPUT);
				write_none(d, e0.idx);
			} else if (e0.kind() == EK_PARSE && e0.L == 0) {
				write_empty(d, e0.idx);
			} else {
				break;
			}
			e0 = e1;
			e1 = lane_ev(d, lane_load(d, grab(), re));
		}
		w0 = 0;
		s = di.init;
		rec_init(di, sr);
		live = e0.kind() == EK_PARSE ? 1u : 0u;
	};
	resolve();

	// The window in flight: (tidx, tw) names what W holds for this lane.
	auto nwin = [](const LaneEv& e) { return e.L ? (e.lastp() >> 2) + 1u : 0u; };
	Chunk W[4];
	uint32_t tidx, tw;
	auto issue = [&](unsigned long long a, uint32_t last, uint32_t w) {
		// member k's window: pieces base + 16 * min(4w + j, last), j = 0..3; this lane loads piece r
		const uint32_t pc = (w << 2) | (last << 16); // window's first piece | last piece
		unsigned long long ak[4];
		uint32_t pk[4];
		ak[0] = qbcast64<0>(a), pk[0] = qbcast<0>(pc);
		ak[1] = qbcast64<1>(a), pk[1] = qbcast<1>(pc);
		ak[2] = qbcast64<2>(a), pk[2] = qbcast<2>(pc);
		ak[3] = qbcast64<3>(a), pk[3] = qbcast<3>(pc);
#pragma unroll
		for (int k = 0; k < 4; k++) {
			const uint32_t c = min((pk[k] & 0xffffu) + r, pk[k] >> 16);
			W[k] = gload16((uintptr_t)(ak[k] + 16ull * c));
		}
	};
	tidx = e0.idx;
	tw = 0;
	issue(e0.base, e0.lastp(), 0);

	while (__any(e0.kind() != EK_NONE)) {
		// is the window in flight the one e0 needs?
		const bool valid = e0.kind() == EK_PARSE && tidx == e0.idx && tw == w0;
		Chunk X[4] = {W[0], W[1], W[2], W[3]};
		// predict and load the next window
		{
			unsigned long long na;
			uint32_t nl, ni, nw;
			if (!valid) {
				na = e0.base, nl = e0.lastp(), ni = e0.idx, nw = w0;
			} else if (w0 + 1 < nwin(e0)) {
				na = e0.base, nl = e0.lastp(), ni = e0.idx, nw = w0 + 1;
			} else {
				na = e1.base, nl = e1.lastp(), ni = e1.idx, nw = 0;
			}
			issue(na, nl, nw);
			tidx = ni;
			tw = nw;
		}
		transpose_quad(X, r);
		bool done = false;
		if (valid) {
			// slot k holds the buffer's chunk c = 4 w0 + k - j0 (slots before the buffer: c < 0)
#pragma unroll
			for (int k = 0; k < 4; k++) { // the buffer's first kStage bytes into the lane's staging row
				const int c = (int)(4 * w0 + k) - (int)e0.j0();
				if (c >= 0 && c < (int)(kStage / 16))
#pragma unroll
					for (int j = 0; j < 4; j++)
						stg[(4 * c + j) * kScanLanes] = X[k].w[j];
			}
#pragma unroll
			for (int k = 0; k < 4; k++) {
				uint32_t sx = s, m, qs, qm;
				scan_chunk(T, X[k], sx, m, qs, qm);
				const int ci = (int)(4 * w0 + k) - (int)e0.j0();
				if (live && ci >= 0) {
					const uint32_t c = (uint32_t)ci;
					chunk_update(di, sr, c, s, qs, qm, m);
					live = !st_terminal(di, sx) && 16 * (c + 1) < e0.L ? 1u : 0u;
					s = sx;
				}
			}
			w0++;
			done = !live;
		}
		uint32_t tw = 0;
		if (done) { // the last chunk scanned is the terminal tracker's, in this window's registers
			const uint32_t k = (sr.term.c + e0.j0()) & 3u, qt = flip_quarter<RS_TERM>(di, sr.term, 0);
			uint32_t w4[4];
#pragma unroll
			for (int j = 0; j < 4; j++)
				w4[j] = k == 0 ? X[0].w[j] : k == 1 ? X[1].w[j] : k == 2 ? X[2].w[j] : X[3].w[j];
			tw = qt == 0 ? w4[0] : qt == 1 ? w4[1] : qt == 2 ? w4[2] : w4[3];
		}
		push(done, tw);
		if (done) {
			e0 = e1;
			e1 = lane_ev(d, lane_load(d, grab(), re));
			resolve();
		}
	}
	if (lane == 0)
		atomicAdd(&sh.scan_done, 1u);
}

// ---------------------------------------------------------------------------------
// k_fresh_scan: the structural scan (ebd_scan.h) over LDS tiles of whole buffers (EBD_CFG_FRESH_SCAN;
// k_fresh, the projected DFA, is the default: section 8 of DESIGN.md has both measured).
//
// Every workgroup is one wave with a contiguous range of the batch and no partner: it never
// waits for another wave.  Per tile:
//   1. the next up-to-64 events' words are in the lanes (loaded one tile ahead); a prefix sum
//      of their 16-byte piece counts takes the events whose buffers fit kTileBytes;
//   2. the buffers land in the wave's LDS tile in one LDS-DMA stream (global_load_lds, 16 B
//      per lane, consecutive: the whole-line read shape) when they lie back to back in the
//      payload, as a batch from the ring buffer does; other layouts are copied buffer by buffer;
//   3. lanes over pieces: the piece bitmap of bytes outside [0x20, 0x7e] (nv4 + __ballot), the
//      key / Host / client-IP class bitmaps (class table + v_dot4_u32_u8), and the list of
//      every LF + 1 in the tile (a wave prefix sum places each lane's LFs);
//   4. lanes over buffers: the request line (scan_reqline);
//   5. lanes over lines: each listed line parsed on its own (scan_line) against the buffer it
//      lies in (a bitmap of buffer-start pieces and its prefix counts);
//   6. lanes over buffers: the line records folded in order (scan_fold), the key and client
//      class; result and key go out in event order (16-B rows of consecutive lanes: whole
//      lines), UNFINISHED events to the session list through an LDS ring, 64 at a time.
// The payload is read once, from HBM, in lines; everything after the DMA is LDS traffic.
// ---------------------------------------------------------------------------------
#ifndef EBD_SCAN_TILE
#define EBD_SCAN_TILE 11264
#endif
#ifndef EBD_SCAN_WGS
#define EBD_SCAN_WGS 8 // one-wave workgroups per CU (LDS-bound: 8 x 19.4 KiB)
#endif
#ifndef EBD_SCAN_LINES
#define EBD_SCAN_LINES 320
#endif
constexpr uint32_t kTileBytes = EBD_SCAN_TILE, kTilePieces = kTileBytes / 16, kTileWords = kTilePieces / 64;
static_assert(kTilePieces % 64 == 0 && kTilePieces >= (EBD_BUFFER_MAX_DATA_SIZE + 30) / 16, "a tile holds any one buffer");
static_assert(kTileBytes + 64 < 65536, "tile positions fit the 16-bit line records");
constexpr uint32_t kLines = EBD_SCAN_LINES; // lines a tile lists (a buffer with more goes to scan_event)
constexpr uint32_t kUnfRing = 128;          // UNFINISHED events waiting to be listed (a flush takes 64)

struct ScanLds {
	uint8_t tile[kTileBytes + 64]; // + reads a few bytes past the last buffer (key words, protocol)
	uint16_t cm[CB_N][kTilePieces]; // class bitmaps: bit i of cm[c][pc] = byte 16 pc + i not in class c
	unsigned long long nvw[kTileWords];
	unsigned long long evb[kTileWords]; // bit j of word w: piece 64 w + j starts a buffer of the tile
	uint16_t evpre[kTileWords];         // buffers starting before word w
	uint16_t evq[64], evend[64], evfirst[64]; // per buffer (by rank): first header line, end, its record
	LineRec lrec[kLines];
	uint8_t ncls[256]; // ~byte_class (ebd_scan.h NB_*)
	uint32_t unf[kUnfRing];
};

// scan_event's source: the wave's tile in LDS.
struct TileSrc {
	const uint8_t* t;
	const unsigned long long* nv;
	const uint8_t* nc;
	const uint16_t (*cm)[kTilePieces];
	__device__ __forceinline__ uint32_t byte(uint32_t p) const { return t[p]; }
	__device__ __forceinline__ uint32_t dw(uint32_t p) const {
		const uint32_t* a = (const uint32_t*)(t + (p & ~3u));
		return __builtin_amdgcn_alignbyte(a[1], a[0], p & 3u);
	}
	__device__ __forceinline__ unsigned long long ld8(uint32_t p) const {
		const uint32_t* a = (const uint32_t*)(t + (p & ~3u));
		const uint32_t x0 = a[0], x1 = a[1], x2 = a[2];
		return (unsigned long long)__builtin_amdgcn_alignbyte(x1, x0, p & 3u) |
				((unsigned long long)__builtin_amdgcn_alignbyte(x2, x1, p & 3u) << 32);
	}
	__device__ __forceinline__ void piece(uint32_t pc, uint32_t (&w)[4]) const {
		const uint4 v = *(const uint4*)(t + 16 * pc);
		w[0] = v.x;
		w[1] = v.y;
		w[2] = v.z;
		w[3] = v.w;
	}
	__device__ __forceinline__ unsigned long long nvword(uint32_t j) const { return nv[j]; }
	__device__ __forceinline__ uint32_t ncls(uint32_t b) const { return nc[b]; }
	__device__ __forceinline__ unsigned long long clsword(uint32_t c, uint32_t a) const { return ((const unsigned long long*)cm[c])[a]; }
};

// An event's words as a lane of k_fresh_scan holds them (Discovery.cpp:92-110: flags, pid, the
// saved buffer).
struct ScanMeta {
	uint32_t L, pid, fw, valid; // fw: the event's word at byte 32 (flags in its low byte)
	unsigned long long off;
};

// Branch-free: a position past the range loads event rb's words (marked invalid), so every
// call issues the same loads.
__device__ __forceinline__ ScanMeta scan_meta(const Dev& d, uint32_t i, uint32_t rb, uint32_t re) {
	ScanMeta m;
	m.valid = i < re ? 1u : 0u;
	const uint32_t j = i < re ? i : rb;
	const uint8_t* e = (const uint8_t*)(d.ev + j);
	m.pid = *(const uint32_t*)e;
	m.fw = *(const uint32_t*)(e + 32);
	m.L = d.len[j];
	m.off = d.off[j];
	return m;
}

// scan_event (and the generic parser for a key with a space) for the buffers the line records
// leave: a call, so that its loops do not take registers from the straight-line path.
__device__ __attribute__((noinline)) void scan_exact(const uint8_t* t, const unsigned long long* nv, const uint8_t* nc,
		const uint16_t (*cm)[kTilePieces], const KeyTrie* trie, uint32_t B, uint32_t L, ScanOut& o) {
	const TileSrc src{t, nv, nc, cm};
	scan_event(src, B, L, o);
	if (o.slow)
		scan_slow(src, trie, B, L, o);
}

__device__ __forceinline__ uint32_t lane_rank(unsigned long long b) {
	return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
}

__global__ __launch_bounds__(64) void k_fresh_scan(Dev d) {
	__shared__ __attribute__((aligned(16))) ScanLds lds;
	const uint32_t lane = threadIdx.x;
	const uint32_t per = (uint32_t)(((unsigned long long)d.n + gridDim.x - 1) / gridDim.x);
	const uint32_t rb = min(d.n, blockIdx.x * per), re = min(d.n, rb + per);
	((uint32_t*)lds.ncls)[lane] = ~((const uint32_t*)d.trie->cls)[lane] & 0x1f1f1f1fu;
	const TileSrc src{lds.tile, lds.nvw, lds.ncls, lds.cm};
	uint32_t uh = 0, un = 0; // the UNFINISHED ring: head and entries (wave-uniform)
	uint32_t base = rb;
	ScanMeta m = scan_meta(d, base + lane, rb, re);
	while (base < re) {
		const uint32_t flags = m.fw & 0xffu;
		const bool has = m.valid && (flags & FLAG_NEW) && m.L != EBD_NO_BUFFER; // Discovery.cpp:92-110
		const bool bad = has && !buf_in(d, m.L, m.off);
		const bool parse = has && !bad && m.L > 0;
		const unsigned long long a = (unsigned long long)(uintptr_t)(d.payload + (parse ? m.off : 0ull));
		const uint32_t np = parse ? (uint32_t)(((a & 15u) + m.L + 15u) >> 4) : 0u;
		uint32_t S = np; // inclusive prefix of the piece counts
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			const uint32_t y = __shfl_up(S, (unsigned)o, 64);
			S += lane >= (uint32_t)o ? y : 0u;
		}
		const uint32_t k = (uint32_t)__popcll(__ballot(m.valid && S <= kTilePieces)); // >= 1: a buffer fits alone
		const bool mine = lane < k, mp = mine && parse;
		const uint32_t P = S - np; // the buffer's first tile piece
		const uint32_t N = __shfl(S, (int)k - 1);
		const ScanMeta nm = scan_meta(d, base + k + lane, rb, re); // the next tile's events
		if (N > 0) {
			const unsigned long long a16 = a & ~15ull, g = a16 - 16ull * P;
			const unsigned long long act = __ballot(mine && np > 0);
			const unsigned long long g0 = __shfl(g, __ffsll((long long)act) - 1);
			if (__ballot(mine && np > 0 && g != g0) == 0) { // back to back: one stream of N pieces
				for (uint32_t j0 = 0; j0 < N; j0 += 64)
					if (j0 + lane < N)
						__builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(uintptr_t)(g0 + 16ull * (j0 + lane)),
								(__attribute__((address_space(3))) void*)(lds.tile + 16 * j0), 16, 0, 0);
			} else { // buffer by buffer, through registers
				uint32_t mx = mine ? np : 0u;
#pragma unroll
				for (int o = 32; o > 0; o >>= 1)
					mx = max(mx, (uint32_t)__shfl_xor(mx, o, 64));
				for (uint32_t q = 0; q < mx; q += 4) {
					Chunk c[4];
#pragma unroll
					for (uint32_t t = 0; t < 4; t++)
						if (mine && q + t < np)
							c[t] = gload16((uintptr_t)(a16 + 16ull * (q + t)));
#pragma unroll
					for (uint32_t t = 0; t < 4; t++)
						if (mine && q + t < np)
							*(uint4*)(lds.tile + 16 * (P + q + t)) = make_uint4(c[t].w[0], c[t].w[1], c[t].w[2], c[t].w[3]);
				}
			}
		}
		if (lane < kTileWords)
			lds.evb[lane] = 0ull;
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		wave_sync();
		// the buffers of the tile, by rank: where they start and end
		const uint32_t rank = lane_rank(__ballot(mp));
		const uint32_t B = 16 * P + (uint32_t)(a & 15u), E = B + (mp ? m.L : 0u);
		if (mp) {
			atomicOr(&lds.evb[P >> 6], 1ull << (P & 63u));
			lds.evend[rank] = (uint16_t)E;
			lds.evfirst[rank] = 0xffffu;
		}
		// lanes over pieces: the bitmaps and the line list (every LF + 1, in tile order)
		uint32_t nl = 0;
		for (uint32_t j0 = 0; j0 < N; j0 += 64) {
			const uint32_t j = min(j0 + lane, N - 1);
			const uint4 v = *(const uint4*)(lds.tile + 16 * j);
			const uint32_t w[4] = {v.x, v.y, v.z, v.w};
			uint32_t cmk[CB_N];
			piece_classes(src, w, cmk);
			const unsigned long long b = __ballot((nv4(v.x) | nv4(v.y) | nv4(v.z) | nv4(v.w)) != 0u);
			if (lane == 0)
				lds.nvw[j0 >> 6] = b;
#pragma unroll
			for (uint32_t c = 0; c < CB_N; c++)
				lds.cm[c][j] = (uint16_t)cmk[c];
			const bool own = j0 + lane < N;
			unsigned long long z0 = own ? (lf4(v.x) | ((unsigned long long)lf4(v.y) << 32)) : 0ull;
			unsigned long long z1 = own ? (lf4(v.z) | ((unsigned long long)lf4(v.w) << 32)) : 0ull;
			const uint32_t c = (uint32_t)(__popcll(z0) + __popcll(z1));
			uint32_t x = c; // inclusive prefix over the lanes
#pragma unroll
			for (int o = 1; o < 64; o <<= 1) {
				const uint32_t y = __shfl_up(x, (unsigned)o, 64);
				x += lane >= (uint32_t)o ? y : 0u;
			}
			uint32_t at = nl + x - c;
			for (; z0; z0 &= z0 - 1, at++)
				if (at < kLines)
					lds.lrec[at].a = (16 * j + ((uint32_t)__builtin_ctzll(z0) >> 3) + 1) << 16;
			for (; z1; z1 &= z1 - 1, at++)
				if (at < kLines)
					lds.lrec[at].a = (16 * j + 8 + ((uint32_t)__builtin_ctzll(z1) >> 3) + 1) << 16;
			nl += __shfl(x, 63);
		}
		const uint32_t nlines = min(nl, kLines);
		wave_sync();
		if (lane < kTileWords) { // buffers starting before each word of evb
			const uint32_t c = (uint32_t)__popcll(lds.evb[lane]);
			uint32_t x = c;
#pragma unroll
			for (int o = 1; o < 16; o <<= 1) {
				const uint32_t y = __shfl_up(x, (unsigned)o, 64);
				x += lane >= (uint32_t)o ? y : 0u;
			}
			lds.evpre[lane] = (uint16_t)(x - c);
		}
		static_assert(kTileWords <= 16, "evpre scan covers 16 words");
		// lanes over buffers: the request lines (P:162-262)
		ReqOut rq;
		rq.dec = SF_UNF;
		if (mp) {
			rq = scan_reqline(src, B, m.L);
			lds.evq[rank] = (uint16_t)(rq.dec == SF_GO && rq.q < E ? rq.q : 0xffffu);
		}
		wave_sync();
		// lanes over lines: each listed line against the buffer it lies in (P:264-352)
		for (uint32_t l0 = 0; l0 < nlines; l0 += 64) {
			const uint32_t l = l0 + lane;
			if (l < nlines) {
				const uint32_t q = lds.lrec[l].a >> 16, pc = min(q >> 4, N - 1), wi = pc >> 6;
				const uint32_t e = lds.evpre[wi] + (uint32_t)__popcll(lds.evb[wi] & ((2ull << (pc & 63u)) - 1ull)) - 1u;
				const LineRec r = scan_line(src, q, lds.evend[e]);
				lds.lrec[l] = r;
				if (q == lds.evq[e])
					lds.evfirst[e] = (uint16_t)l;
			}
		}
		wave_sync();
		bool unf = false;
		if (mine) {
			const uint32_t i = base + lane;
			ebd_event_result r;
			Hash128 key{0, 0};
			if (parse) {
				ScanOut o;
				const uint32_t l0 = lds.evfirst[rank];
				scan_init(o, m.L);
				if (!scan_fold(rq, [&](uint32_t l) { return lds.lrec[l < kLines ? l : 0]; }, l0, nlines, B, m.L, o))
					scan_exact(lds.tile, lds.nvw, lds.ncls, lds.cm, d.trie, B, m.L, o); // rare shapes (ebd_scan.h)
				r = scan_result(o, (uint8_t)flags);
				if (o.status == EBD_STATUS_FINISHED) {
					key = endpoint_key<2>(d.hkey, m.pid, o.host_off, o.host_len, o.url_off, o.url_len,
							[&](uint32_t x) { return src.ld8(B + x); }); // the client's class is k_agg_fast's
				}
				unf = o.status == EBD_STATUS_UNFINISHED;
			} else {
				// an empty buffer: a fresh parser consumes nothing and waits (Discovery.cpp:148-150);
				// no buffer (or one out of range): no parse at all
				if (bad)
					set_error(d, EBD_ERR_BAD_INPUT);
				unf = has && !bad;
				r.consumed = 0;
				r.status = unf ? EBD_STATUS_UNFINISHED : EBD_STATUS_NONE;
				r.info = 0;
				r.u.span.url_off = r.u.span.url_len = r.u.span.host_off = r.u.span.host_len = r.u.span.cip_off = r.u.span.cip_len = 0;
			}
			d.res[i] = r;
			d.keys[i] = key;
		}
		// UNFINISHED events to the session-set list (k_sset_build), 64 per counter atomic
		const unsigned long long ub = __ballot(unf);
		if (unf)
			lds.unf[(uh + un + lane_rank(ub)) & (kUnfRing - 1)] = base + lane;
		un += (uint32_t)__popcll(ub);
		if (un >= kUnfRing / 2) { // (un < kUnfRing / 2 + 64 <= kUnfRing entries)
			wave_sync();
			unsigned long long at = 0;
			if (lane == 0)
				at = atomicAdd(&d.ctr[CTR_UNFINISHED], (unsigned long long)(kUnfRing / 2));
			at = __shfl(at, 0);
			for (uint32_t t = 0; t < kUnfRing / 2; t += 64)
				d.ev_slot[at + t + lane] = lds.unf[(uh + t + lane) & (kUnfRing - 1)];
			uh += kUnfRing / 2;
			un -= kUnfRing / 2;
			wave_sync();
		}
		base += k;
		m = nm;
		wave_sync(); // the next tile's DMA rewrites what this one's lanes read
	}
	wave_sync();
	if (un) {
		unsigned long long at = 0;
		if (lane == 0)
			at = atomicAdd(&d.ctr[CTR_UNFINISHED], (unsigned long long)un);
		at = __shfl(at, 0);
		for (uint32_t t = 0; t < un; t += 64)
			if (t + lane < un)
				d.ev_slot[at + t + lane] = lds.unf[(uh + t + lane) & (kUnfRing - 1)];
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

__device__ __forceinline__ uint32_t cip_classify(const Dev& d, uint32_t i, ebd_event_result& r, uint8_t* row,
		unsigned long long* net) {
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
		cip_token(*d.ifs, [row](uint32_t b) { return (uint32_t)row[b]; }, 0, e, &tb, &te, &cls, net);
	} else { // a value longer than the copy without ',' or CR in it: parse from the buffer
		cip_token(*d.ifs, [p](uint32_t b) { return (uint32_t)p[b]; }, cs, lim, &tb, &te, &cls, net);
		tb -= cs;
		te -= cs;
	}
	r.u.span.cip_off = (uint16_t)(cs + tb);
	r.u.span.cip_len = (uint16_t)(te - tb);
	return cls;
}

// The session set of the batch, sized to what it holds: the sessions carried from earlier
// batches and those of the fresh parses k_fresh left unfinished (k_fresh lists them in
// ev_slot).  Its mask is chosen on the device (no host round trip) at a load of at most 1/2
// of the sessions it can hold, so the probes of k_slow_collect (one per event of the batch)
// land in a table of a few times the live sessions instead of one sized for every event.
__global__ void k_sset_size(Dev d, uint32_t cap) {
	const unsigned long long want = 2ull * (d.ctr[CTR_UNFINISHED] + d.n_carry_in);
	uint32_t m = cap < 1024u ? cap : 1024u; // never past the allocation (cap: a power of two)
	while (m < want && m < cap)
		m <<= 1;
	*d.sset_mask = m - 1u;
}
// Tiles of 256 x kSetPer inserts per block; the claimed slots join the dirty list with one
// atomic per tile (block_reserve).
constexpr uint32_t kSetPer = 8;
__global__ __launch_bounds__(256) void k_sset_build(Dev d) {
	__shared__ uint32_t part[4];
	__shared__ unsigned long long base;
	const uint32_t nu = (uint32_t)d.ctr[CTR_UNFINISHED], total = d.n_carry_in + nu, tile = 256u * kSetPer;
	for (uint32_t t0 = blockIdx.x * tile; t0 < total; t0 += gridDim.x * tile) { // uniform
		uint32_t cl[kSetPer], cnt = 0;
#pragma unroll
		for (uint32_t u = 0; u < kSetPer; u++) {
			const uint32_t k = t0 + u * 256u + threadIdx.x;
			cl[u] = kNone;
			if (k < d.n_carry_in) {
				const Carry& cr = d.carry_in[k];
				sset_insert(d, cr.pid, cr.fd, cr.sid, k + 1, kNone, &cl[u]);
			} else if (k < total) {
				const uint32_t i = d.ev_slot[k - d.n_carry_in];
				const EventRec& ev = d.ev[i];
				sset_insert(d, ev.pid, ev.fd, ev.sessionID, 0, i, &cl[u]);
			}
			cnt += cl[u] != kNone ? 1u : 0u;
		}
		unsigned long long at = block_reserve(&d.ctr[CTR_DIRTY], cnt, part, &base);
#pragma unroll
		for (uint32_t u = 0; u < kSetPer; u++)
			if (cl[u] != kNone)
				d.dirty[at++] = cl[u];
	}
}

// Tiles of 256 x kCollectPer events per block, one atomic per tile for the list (block_reserve).
constexpr uint32_t kCollectPer = 8;
__global__ __launch_bounds__(256) void k_slow_collect(Dev d) {
	__shared__ uint32_t part[4];
	__shared__ unsigned long long base;
	if (d.ctr[CTR_DIRTY] == 0)
		return; // no session needs the sequential path in this batch
	const uint32_t tile = 256u * kCollectPer;
	for (uint64_t t0 = (uint64_t)blockIdx.x * tile; t0 < d.n; t0 += (uint64_t)gridDim.x * tile) { // uniform
		uint32_t has = 0;
#pragma unroll
		for (uint32_t u = 0; u < kCollectPer; u++) {
			const uint64_t i = t0 + u * 256u + threadIdx.x;
			if (i >= d.n)
				continue;
			// every event's key at its own index (~0: not on the session path), so that the keys
			// enter the sort in event order and the sort (stable) orders only the group bits
			unsigned long long key = ~0ull;
			const EventRec& e = d.ev[i];
			const int slot = (e.flags & (FLAG_NEW | FLAG_END)) ? sset_find(d, e.pid, e.fd, e.sessionID) : -1;
			if (slot >= 0) {
				d.res[i].info |= EBD_INFO_SESSION; // k_walk's, not k_agg_fast's (which may run first)
				// grouped by session, sessions in the order of their first UNFINISHED fresh parse
				// (carried ones first): the lanes of a walker wave then follow sessions that started
				// together, whose events lie close together in the batch (L2 / TLB locality), where
				// the session-set slot order (a hash) sent them all over the batch
				const SSlot& ss = d.sset[slot];
				const uint32_t grp = ss.carry ? ss.carry - 1 : d.carry_cap + ~ss.first_c;
				key = ((unsigned long long)grp << 32) | i;
				has |= 1u << u;
				d.ev_slot[i] = (uint32_t)slot;
			}
			d.slow_keys[i] = key;
		}
		(void)block_reserve(&d.ctr[CTR_SLOW], (uint32_t)__popc(has), part, &base); // the count
	}
}

// ---------------------------------------------------------------------------------
// k_walk: the sequential session path.  The bytes of the request in progress are the
// carried bytes (if the request started in an earlier batch) followed by the buffers
// of this batch's events from position j0 on.
// ---------------------------------------------------------------------------------
constexpr int kWalkThreads = 256;
#ifndef EBD_WALK_REFILL
#define EBD_WALK_REFILL 60
#endif
constexpr int kWalkRefill = EBD_WALK_REFILL; // lanes of a wave waiting before it ends and starts events
#ifndef EBD_WALK_BLOCKS
#define EBD_WALK_BLOCKS 4 // k_walk blocks per CU (EBD_WALK_WPE waves per SIMD)
#endif
constexpr int kWalkDryBlocks = 3; // k_walk_dry blocks per CU (3 waves per SIMD at its register count)

struct Walk {
	const uint8_t* cb; // carried bytes of the request in progress
	uint32_t clen;
	uint32_t j0;       // first sorted position whose buffer belongs to the request
};

__device__ __forceinline__ uint32_t slow_event(const Dev& d, uint32_t j) { return (uint32_t)d.slow_keys[j]; }

__device__ __forceinline__ uint32_t piece_len(const Dev& d, uint32_t j) {
	const uint32_t i = slow_event(d, j);
	const uint32_t L = d.len[i];
	return ((d.ev[i].flags & FLAG_NEW) && L != EBD_NO_BUFFER && buf_in(d, L, d.off[i])) ? L : 0;
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

// The session path's tables in LDS: the DFA image (byte-major, LdsTable) and the attribute
// byte of each state (DfaTable::attr).
struct SessTabs {
	const uint8_t* T;
	const uint8_t* A;
};
struct ByteTab {
	const uint8_t* t;
	__device__ __forceinline__ uint32_t operator[](uint32_t i) const { return t[i]; }
};

// dfa_parse (ebd_fresh.h) over one buffer on the device: 16-byte aligned blocks, the next
// one loaded while the current one is walked, dfa_walk_block per block (a byte is valid
// when its buffer offset is below the bytes the request may take).  The
// aligned block holding a valid byte never leaves that byte's page, so the over-read cannot
// fault.  The walk stops after the block in which the state became terminal.
__device__ uint32_t dfa_parse_dev(GenParser& g, const SessTabs& tb, const DfaInfo& di, const uint8_t* p, uint32_t n, uint8_t flags) {
	const LdsTable T{tb.T};
	const ByteTab A{tb.A};
	DfaWalk w;
	dfa_walk_load(g, A[g.ds], w);
	const uint32_t pos0 = w.pos, ne = dfa_allow(pos0, n);
	if (ne) {
		const uintptr_t a0 = (uintptr_t)p, b0 = a0 & ~(uintptr_t)15;
		const uint32_t k0 = (uint32_t)(a0 & 15u), nb = (k0 + ne + 15u) >> 4;
		uint4 cur = *(const uint4*)b0;
		for (uint32_t bi = 0; bi < nb && w.tpos == kNone; bi++) {
			const uint4 nx = bi + 1 < nb ? *(const uint4*)(b0 + 16u * (bi + 1)) : cur;
			const uint32_t wd[4] = {cur.x, cur.y, cur.z, cur.w};
			const uint32_t base = 16u * bi - k0; // buffer offset of the block's byte 0 (wraps below 0)
			dfa_walk_block(T, A, w, wd, base, pos0 + base, ne);
			cur = nx;
		}
	}
	return dfa_walk_store(di, w, pos0, ne, n, flags, g);
}

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

// Copies the stream bytes of three spans, [a[k], a[k] + n[k]) to dst[k], in one pass over the
// request's pieces (each piece's event is looked up once, not once per span): 8-byte loads
// and stores inside each piece, byte stores for a piece's last < 8 bytes (the next span's or
// request's bytes follow dst[k]'s in the arena).
__device__ void stream_copy3(const Dev& d, const Walk& w, uint32_t jend, uint32_t cend, const uint32_t (&a)[3], const uint32_t (&n)[3],
		uint8_t* const (&dst)[3]) {
	uint32_t b = 0;
#pragma unroll
	for (int k = 0; k < 3; k++)
		b = n[k] && a[k] + n[k] > b ? a[k] + n[k] : b;
	if (b == 0)
		return;
	// 32 bytes at a time: the four 8-byte loads are issued before any store (one memory round
	// trip per 32 bytes; a load-store pair per 8 bytes and a byte loop for the tail waited on
	// every load), at in-span offsets (a source is readable 8 bytes past its end); the tail is
	// stored in 4-, 2- and 1-byte pieces
	auto copy = [](const uint8_t* src, uint8_t* out, uint32_t len) {
		for (uint32_t k = 0; k < len; k += 32) {
			unsigned long long v[4];
#pragma unroll
			for (uint32_t m = 0; m < 4; m++)
				v[m] = gload8u(src + min(k + 8u * m, len - 1u));
#pragma unroll
			for (uint32_t m = 0; m < 4; m++) {
				const uint32_t o = k + 8u * m;
				if (o + 8u <= len) {
					*(u64a1*)(out + o) = v[m];
				} else if (o < len) {
					uint8_t* p = out + o;
					unsigned long long x = v[m];
					const uint32_t t = len - o;
					if (t & 4u) {
						*(u32a1*)p = (uint32_t)x;
						p += 4;
						x >>= 32;
					}
					if (t & 2u) {
						*(u16a1*)p = (uint16_t)x;
						p += 2;
						x >>= 16;
					}
					if (t & 1u)
						*p = (uint8_t)x;
				}
			}
		}
	};
	// the spans' parts inside piece [pos, pos + pl), whose bytes start at src
	auto piece = [&](const uint8_t* src, uint32_t pos, uint32_t pl) {
#pragma unroll
		for (int k = 0; k < 3; k++) {
			const uint32_t lo = a[k] > pos ? a[k] : pos, hi = a[k] + n[k] < pos + pl ? a[k] + n[k] : pos + pl;
			if (lo < hi)
				copy(src + (lo - pos), dst[k] + (lo - a[k]), hi - lo);
		}
	};
	uint32_t pos = 0;
	if (w.clen) {
		piece(w.cb, 0, w.clen);
		pos = w.clen;
	}
	// the walker's records of the pieces (one line for a request's pieces), four loaded at a time
	for (uint32_t j = w.j0; j <= jend && pos < b; j += 4) {
		unsigned long long pc[4];
#pragma unroll
		for (uint32_t m = 0; m < 4; m++)
			pc[m] = d.pieces[min(j + m, jend)];
#pragma unroll
		for (uint32_t m = 0; m < 4; m++) {
			uint32_t pl = (uint32_t)(pc[m] & 0xffffffu);
			if (j + m == jend)
				pl = cend;
			if (j + m > jend || pos >= b || pl == 0)
				continue;
			piece(d.payload + (pc[m] >> 24), pos, pl);
			pos += pl;
		}
	}
}

// handleSuccessfulParse -> handleNewRequest -> Aggregator::newRequest
// (Discovery.cpp:161-192, 210-212) for a request finished by the session path.
// A request the session path finished, from the walker to k_emit: everything the emission
// needs, in the session-request slot it will occupy (32 bytes: SessReq's size).  The walker
// only records it, so the emission (span copies, client class, key, service table) runs
// for all of the batch's session requests at once in k_emit, on full waves, instead of
// for the few lanes of a walker wave whose event happened to finish a request.
struct EmitRec {
	uint32_t i, jend, j0; // finishing event, its sorted position, the request's first
	uint32_t cc;          // carried bytes (1 + index, bits 0-23; ebd_ctx_create bounds the LRU) | cend bits 8-13 << 24
	uint16_t host_start, host_len, url_start, url_len, cip_start, cip_len;
	uint8_t f, mcand, info, cend_lo; // GenParser::f and mcand; the result's info bits so far; cend bits 0-7
	// the bytes event i's parse consumed (its piece's end in the request), carried here so that
	// k_emit needs no read of the event's result
	__device__ __forceinline__ uint32_t carry() const { return cc & 0xffffffu; }
	__device__ __forceinline__ uint32_t cend() const { return (uint32_t)cend_lo | ((cc >> 24) << 8); }
};
static_assert(sizeof(EmitRec) == sizeof(SessReq), "an emission record fills a session-request slot");

__device__ void defer_emit(const Dev& d, const Walk& w, uint32_t jend, const GenParser& g, uint32_t i, ebd_event_result& r) {
	const unsigned long long q = wave_add(&d.ctr[CTR_SREQ], 1ull); // CTR_REQUESTS: k_sess_tally adds CTR_SREQ
	EmitRec e;
	e.i = i;
	e.jend = jend;
	e.j0 = w.j0;
	const uint32_t carry = w.cb ? (uint32_t)(((const uint8_t*)w.cb - (const uint8_t*)d.carry_in) / sizeof(Carry)) + 1u : 0u;
	const uint32_t cend = r.consumed; // at most EBD_BUFFER_MAX_DATA_SIZE: 14 bits
	e.cc = carry | ((cend >> 8) << 24);
	e.cend_lo = (uint8_t)cend;
	e.host_start = (uint16_t)g.host_start;
	e.host_len = (uint16_t)g.host_len;
	e.url_start = (uint16_t)g.url_start;
	e.url_len = (uint16_t)g.url_len;
	e.cip_start = (uint16_t)g.cip_start;
	e.cip_len = (uint16_t)g.cip_len;
	e.f = g.f;
	e.mcand = g.mcand;
	e.info = r.info;
	*(EmitRec*)(d.sreq + q) = e;
	r.u.session.index = (uint32_t)q;
}

// handleSuccessfulParse -> handleNewRequest -> Aggregator::newRequest
// (Discovery.cpp:161-192, 210-212) for the session path's request q.
#ifndef EBD_EMIT_BLOCKS
#define EBD_EMIT_BLOCKS 8 // k_emit workgroups per CU
#endif
__global__ __launch_bounds__(256) void k_emit(Dev d) {
	__shared__ __attribute__((aligned(8))) uint8_t rows[256 * kCipStride];
	uint8_t* row = rows + threadIdx.x * kCipStride; // this lane's client-IP value, parsed from LDS
	const uint32_t nq = (uint32_t)d.ctr[CTR_SREQ], stride = gridDim.x * blockDim.x;
	const uint32_t q0 = blockIdx.x * blockDim.x + threadIdx.x;
	// the lane's next record is loaded while the current one is emitted
	EmitRec en = *(const EmitRec*)(d.sreq + (q0 < nq ? q0 : 0u));
	for (uint32_t q = q0; q < nq; q += stride) {
		const EmitRec e = en;
		en = *(const EmitRec*)(d.sreq + (q + stride < nq ? q + stride : q));
		const uint32_t i = e.i;
		const uint32_t carry = e.carry();
		const Walk w{carry ? d.carry_in[carry - 1].bytes : nullptr, carry ? d.carry_in[carry - 1].nbytes : 0u, e.j0};
		const uint32_t cend = e.cend();
		const EventRec& ev = d.ev[i];
		const uint32_t hl = (e.f & GPF_HOST) ? e.host_len : 0, ul = e.url_len;
		const uint32_t cl = (e.f & GPF_CIP_FOUND) ? e.cip_len : 0; // the whole first client-IP value
		const uint32_t total = hl + ul + cl;
		const unsigned long long at = wave_add(&d.ctr[CTR_SSTR], (unsigned long long)total);
		uint8_t info = (uint8_t)(e.info | (e.mcand == 'P' ? EBD_INFO_POST : 0) | ((e.f & GPF_HTTPS) ? EBD_INFO_HTTPS : 0));
		SessReq sr;
		sr.seq = d.seq_base + i;
		sr.pid = ev.pid;
		sr.status = EBD_STATUS_FINISHED;
		sr.pad = 0;
		sr.pad2 = 0;
		if (at + total > d.sstr_cap) {
			// no room for its strings: the request is not aggregated, is marked so, and is not
			// counted (k_sess_tally adds CTR_SREQ to CTR_REQUESTS)
			set_error(d, EBD_ERR_ARENA_FULL);
			atomicAdd(&d.ctr[CTR_REQUESTS], ~0ull);
			sr.str_off = 0;
			sr.host_len = sr.url_len = sr.cip_off = sr.cip_len = 0;
			sr.info = (uint8_t)(info | EBD_INFO_DROPPED);
			d.sreq[q] = sr;
			d.res[i].info = sr.info;
			continue;
		}
		uint8_t* dst = d.sstr + at;
		const uint32_t sa[3] = {e.host_start, e.url_start, e.cip_start}, sn[3] = {hl, ul, cl};
		uint8_t* const sd[3] = {dst, dst + hl, dst + hl + ul};
		stream_copy3(d, w, e.jend, cend, sa, sn, sd);
		unsigned long long net = 0;
		uint8_t cls;
		uint32_t tb = 0, te = 0;
		if (e.f & GPF_CIP_FOUND) {
			// the value (just copied to the arena) goes to the lane's LDS row with 8-byte loads
			// (the arena has 64 bytes of slack), so the byte-serial parse below reads LDS
			const uint8_t* cv = dst + hl + ul;
			if (cl <= (uint32_t)kCipRaw) {
#pragma unroll
				for (uint32_t h = 0; h < (uint32_t)kCipRaw / 8; h++)
					if (8 * h < cl)
						*(unsigned long long*)(row + 8 * h) = gload8u(cv + 8 * h);
				cv = row;
			}
			uint32_t raw = 0; // the value up to its first ',' is the front token's source
			while (raw < cl && cv[raw] != ',')
				raw++;
			front_token(cv, raw, &tb, &te);
			info |= EBD_INFO_CIP;
			cls = classify_token(*d.ifs, cv + tb, te - tb, &net);
		} else {
			cls = classify_source(*d.ifs, ev.flags, ev.sourceIP, &net);
		}
		info |= (uint8_t)(cls << EBD_INFO_CLASS_SHIFT);
		// the endpoint's key in block form over its copy (the arena has 64 bytes of slack)
		const Hash128 key = endpoint_key(d.hkey, ev.pid, 0, hl, hl, ul, [dst](uint32_t o) { return gload8u(dst + o); });
		bool claimed;
		const uint32_t slot = agg_insert(d, key, first_word(d.seq_base + i, (e.f & GPF_HTTPS) != 0, hl),
				cls == CLS_INTERNAL, cls == CLS_EXTERNAL, &claimed);
		if (claimed)
			claim_publish(d, slot, wave_add(&d.ctr[CTR_SERVICES], 1ull),
					wave_add(&d.ctr[CTR_SARENA], (unsigned long long)((hl + ul + 7u) & ~7u)), ev.pid, dst, hl, dst + hl, ul);
		if (d.net_on && cls == CLS_EXTERNAL)
			agg_nets(d, slot, net, request_time(d, i));
		sr.str_off = (uint32_t)at;
		sr.host_len = (uint16_t)hl;
		sr.url_len = (uint16_t)ul;
		sr.cip_off = (uint16_t)(hl + ul + tb);
		sr.cip_len = (uint16_t)(te - tb);
		sr.info = info;
		d.sreq[q] = sr;
		d.res[i].info = info;
	}
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

// The LRU operation of one event (the exact-LRU rounds record them, k_lru_*): none (no find:
// no buffer to parse, or the session is not saved), insert (saveSession), erase (close or a
// saved session's INVALID), access (a saved session's buffer: find touched it, it stays).
enum : uint32_t { OP_NONE = 0, OP_INSERT = 1, OP_ERASE = 2, OP_ACCESS = 3 };

// Event jj (sorted position) of a session: handleNewEvent (Discovery.cpp:92-198) with the
// session's state in S.  Returns the LRU operation it implies; an insert (saveSession,
// Discovery.cpp:148-150) is left to the caller, which may have to evict first.
// An event of the session path from the start to the end of its parse (Discovery.cpp:92-198).
enum : uint32_t { EV_PARSE = 256, EV_EXISTING = 512 };
struct EvCtx {
	uint32_t i, jj, L;
	uint32_t flags; // the event's flags | EV_PARSE | EV_EXISTING
};

// handleNewEvent up to parse(): whether the event's buffer is parsed, and with which parser
// (the saved session's, or a fresh one for a session not in the LRU).
__device__ __forceinline__ bool ev_begin(const Dev& d, SessState& S, uint32_t jj, uint32_t i, uint32_t flags, uint32_t L,
		unsigned long long off, EvCtx& e) {
	e.i = i;
	e.jj = jj;
	e.L = L;
	e.flags = flags;
	if (!(flags & FLAG_NEW) || L == EBD_NO_BUFFER || !buf_in(d, L, off))
		return false;
	e.flags |= EV_PARSE;
	if (S.live) { // handleExistingSession, Discovery.cpp:123-139 (find touched it)
		S.stamp = d.seq_base + i;
		e.flags |= EV_EXISTING;
	} else { // handleNewSession, Discovery.cpp:141-159
		gp_init(S.g);
		S.w = Walk{nullptr, 0, jj};
	}
	return true;
}

// handleNewEvent after parse() consumed c bytes: the outcome, the request (FINISHED), the
// kernel-side delete (INVALID of a saved session), the close.  Returns the LRU operation
// it implies; an insert (saveSession, Discovery.cpp:148-150) is left to the caller, which
// may have to evict first.
template <bool DRY = false>
__device__ __forceinline__ uint32_t ev_end(const Dev& d, SessState& S, const EvCtx& e, uint32_t c) {
	ebd_event_result r;
	r.consumed = 0;
	r.status = EBD_STATUS_NONE;
	r.info = EBD_INFO_SESSION;
	r.u.session.index = 0xffffffffu;
	r.u.session.pad_[0] = r.u.session.pad_[1] = 0;
	uint32_t op = OP_NONE; // CTR_SESSION_EVENTS: the walkers count the events they replay
	if (e.flags & EV_PARSE) {
		r.consumed = (uint16_t)c;
		if (e.flags & EV_EXISTING) {
			r.info |= EBD_INFO_EXISTING;
			op = OP_ACCESS;
			if (S.g.state == ST_INVALID) {
				r.status = EBD_STATUS_INVALID;
				if (!DRY)
					atomicAdd(&d.ctr[CTR_KDELETES], 1ull); // bpfDiscoveryDeleteSession
				S.live = 0;
				op = OP_ERASE;
			} else if (S.g.state == ST_FINISHED) {
				r.status = EBD_STATUS_FINISHED;
				if (!DRY)
					defer_emit(d, S.w, e.jj, S.g, e.i, r);
				gp_reset(S.g); // session.reset(); stays saved
				S.w = Walk{nullptr, 0, e.jj + 1};
			} else {
				r.status = EBD_STATUS_UNFINISHED;
			}
		} else {
			if (S.g.state == ST_INVALID) {
				r.status = EBD_STATUS_INVALID;
			} else if (S.g.state == ST_FINISHED) {
				r.status = EBD_STATUS_FINISHED;
				if (!DRY)
					defer_emit(d, S.w, e.jj, S.g, e.i, r);
			} else {
				r.status = EBD_STATUS_UNFINISHED;
				if (!(e.flags & FLAG_END))
					op = OP_INSERT;
			}
		}
	}
	if ((e.flags & FLAG_END) && S.live) { // handleCloseEvent, Discovery.cpp:194-198
		S.live = 0;
		op = OP_ERASE;
	}
	if (!DRY)
		d.res[e.i] = r;
	return op;
}

// Event jj (sorted position) of a session: handleNewEvent (Discovery.cpp:92-198) with the
// session's state in S, the whole buffer at once (the exact LRU walker's form).
// The piece record of sorted position jj (Dev::pieces): k_emit copies a request's spans from them.
__device__ __forceinline__ void piece_record(const Dev& d, uint32_t jj, uint32_t fl, uint32_t L, unsigned long long off) {
	uint32_t pl = ((fl & FLAG_NEW) && L != EBD_NO_BUFFER && buf_in(d, L, off)) ? L : 0; // piece_len
	if (pl > 0xffffffu || (off >> 40)) { // beyond the record's fields (a buffer is at most 8 KiB): reported
		set_error(d, EBD_ERR_BAD_INPUT);
		pl = 0;
	}
	d.pieces[jj] = (off << 24) | pl;
}

__device__ uint32_t session_event(const Dev& d, const SessTabs& tb, SessState& S, uint32_t jj) {
	const uint32_t i = slow_event(d, jj);
	piece_record(d, jj, d.ev[i].flags, d.len[i], d.off[i]);
	EvCtx e;
	uint32_t c = 0;
	if (ev_begin(d, S, jj, i, d.ev[i].flags, d.len[i], d.off[i], e))
		c = dfa_parse_dev(S.g, tb, d.di, d.payload + d.off[i], e.L, (uint8_t)e.flags);
	return ev_end(d, S, e, c);
}

// The session's state at its first event of the batch (sorted position j); carry: its
// session-set slot's carry word (1 + carried index, 0: none).
__device__ __forceinline__ void session_begin_c(const Dev& d, SessState& S, uint32_t j, uint32_t slot, uint32_t carry) {
	d.sset[slot].visited = 1;
	S.w = Walk{nullptr, 0, j};
	S.li = kNone;
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
__device__ __forceinline__ void session_begin(const Dev& d, SessState& S, uint32_t j, uint32_t slot) {
	session_begin_c(d, S, j, slot, d.sset[slot].carry);
}

// A session still in the LRU after the batch, with the bytes of its request in progress
// (which ends with the session's last event jlast of the batch, fully consumed).
__device__ __forceinline__ void session_carry_out(const Dev& d, const SessState& S, uint32_t j, uint32_t jlast) {
	const unsigned long long c = wave_add(&d.ctr[CTR_CARRY_OUT], 1ull);
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
// live sessions first), or with the evictions the exact-LRU rounds derived, by event: evf[i]
// bit 0 = the session was evicted before its event i (it parses that buffer as a new
// session), bit 1 at a session's first event = evicted after its last event (not carried out).  DRY (the
// rounds' walks): no outputs, only each event's LRU operation in ops[j].  The header-key trie
// and the byte classes sit in LDS: the walk reads them once per byte.
// The exact-LRU rounds' walks (DRY): a list entry is the sorted position a session's walk
// starts at (its first event, or where its flags changed, from the snapshot of its state
// there); the walk stops before the first event at or past the horizon hz and leaves where
// it stopped in wto (kNone: the session's end); the state before each event it walks goes to
// snap, the event's LRU operation to opt (by event).
struct DryWalk {
	const uint32_t* head; // sorted position -> its session's first position
	SessState* snap;
	uint32_t* wto;
	uint8_t* opt;
	const LruCtrl* ctl;   // the round's horizon (ctl->tend); nothing to do once ctl->done
	unsigned long long* stat; // EBD_LRU_TRACE: events and bytes walked, the longest lane's bytes (summed over rounds)
};

// k_walk's LDS tables: the DFA image (LdsTable's byte-major layout) with one more column,
// kWalkIdCol, in which every state steps to itself, then the state attributes.  A byte outside
// the parse (before the buffer in its first block, past the allowed bytes in its last) reads the
// identity column, so the state chain carries no select: one v_mad_u32_u24 and one ds_read_u8
// per byte.
constexpr uint32_t kWalkIdCol = kLdsCols;
constexpr uint32_t kWalkAttrOff = ((kLdsCols + 1) * kLdsStride + 15u) & ~15u;
// Sessions of the batch walk are handed out in chunks of kWalkChunk: chunk 0 of each workgroup
// is fixed (blockIdx.x), the later ones are claimed from a global counter (d.ctr[CTR_COUNT],
// zeroed before each launch) by the lane that draws their first ticket.  A fixed share per
// workgroup had the walk end with its slowest workgroups: with the same sessions, events and
// bytes each, some took twice the median's time (80 M config-4 events, tools/walk_balance.py).
constexpr uint32_t kWalkChunk = kWalkThreads, kWalkSlots = 8; // chunk bases kept in LDS
constexpr uint32_t kWalkLdsBytes = kWalkAttrOff + 256 + 16 + 8 * kWalkSlots; // + ticket counter, chunk bases and tags

// dfa_walk_block (ebd_fresh.h) on k_walk's tables: the same walk, with the valid bytes' count
// computed once per block, and the attribute changes found from the packed attributes (four
// bytes per word) instead of a compare per byte.
__device__ __forceinline__ void walk_block(const uint8_t* tabs, DfaWalk& w, const uint32_t (&wd)[4], uint32_t base, uint32_t pbase,
		uint32_t ne) {
	const uint32_t a0 = w.a;
	uint32_t s = w.s;
	uint32_t P[4] = {0u, 0u, 0u, 0u}; // the attribute after each byte
#pragma unroll
	for (int k = 0; k < 16; k++) {
		const uint32_t b = (wd[k >> 2] >> (8 * (k & 3))) & 0xffu;
		const uint32_t col = base + (uint32_t)k < ne ? min(b, kLdsCols - 1) : kWalkIdCol;
		s = tabs[col * kLdsStride + s];
		P[k >> 2] |= (uint32_t)tabs[kWalkAttrOff + s] << (8 * (k & 3));
	}
	// valid bytes: base + k < ne, consecutive (base wraps below 0 in a buffer's first block)
	const uint32_t nv = (int)base < 0 ? min(16u - min(0u - base, 16u), ne) : base < ne ? min(16u, ne - base) : 0u;
	uint32_t chg = 0, prev = a0 << 24;
#pragma unroll
	for (int q = 0; q < 4; q++) { // bytes whose attribute differs from the one before
		const uint32_t x = P[q] ^ __builtin_amdgcn_alignbyte(P[q], prev, 3u);
		const uint32_t nz = (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
		chg |= ((((nz >> 7) * 0x00204081u) >> 21) & 0xfu) << (4 * q);
		prev = P[q];
	}
	if (nv) {
		if (w.pos == 0) // P:162: handleCharMethod: the request's first byte is the method candidate
			w.mcand = blk_byte(wd[0], wd[1], wd[2], wd[3], 0u - pbase);
		if ((a0 & A_TERM) && w.tpos == kNone)
			w.tpos = w.pos + 1;
	}
	for (uint32_t m = chg; m; m &= m - 1u) {
		const uint32_t k = (uint32_t)__builtin_ctz(m);
		dfa_walk_change(w, k ? blk_byte(P[0], P[1], P[2], P[3], k - 1u) : a0, blk_byte(P[0], P[1], P[2], P[3], k), pbase + k);
	}
	w.s = s;
	w.a = prev >> 24;
	w.pos += nv;
}

// Waves per SIMD the walker's register budget must allow (0: the compiler's choice).  At 4
// (128 VGPRs, a few spills outside the byte loop; 4 workgroups per CU) k_walk took 20.1-20.4 ms
// per 80 M config-4 events against 21.3-21.4 at 3 (150 VGPRs).
#ifndef EBD_WALK_WPE
#define EBD_WALK_WPE 4
#endif
#if EBD_WALK_WPE
#define EBD_WALK_ATTR __attribute__((amdgpu_waves_per_eu(EBD_WALK_WPE, 8)))
#else
#define EBD_WALK_ATTR
#endif
template <bool DRY>
__device__ __forceinline__ void walk_sessions(const Dev& d, const uint8_t* evf, const DryWalk& dw, const uint32_t* hlist,
		const uint32_t* hcount) {
	if (DRY && dw.ctl->done) // the rounds have settled: later rounds' kernels do nothing
		return;
	if (DRY && blockIdx.x * kWalkThreads >= *hcount)
		return; // a round walks few sessions: the workgroups past them skip the table load
	const uint32_t hz = DRY ? dw.ctl->tend : 0u;
	__shared__ __attribute__((aligned(16))) uint8_t tabs[kWalkLdsBytes];
	uint32_t* s_next = (uint32_t*)(tabs + kWalkAttrOff + 256); // the workgroup's next ticket
	// chunk c's first session, at c % kWalkSlots: c << 32 | base in one 64-bit word, so that a
	// reader sees the chunk and its base together (a tag seen, then a base already rewritten by
	// chunk c + kWalkSlots, cannot happen)
	unsigned long long* s_cb = (unsigned long long*)(s_next + 4);
	// the sessions to walk: every one (k_walk_heads), or the exact-LRU round's list
	const uint32_t* heads = hlist ? hlist : d.heads;
	const uint32_t nh = hlist ? *hcount : (uint32_t)d.ctr[CTR_HEADS], nslow = (uint32_t)d.ctr[CTR_SLOW];
	const uint32_t stride = gridDim.x * kWalkThreads;
	// Sessions: the rounds' walks (DRY, a few per lane at most) take every stride-th; the batch
	// walk gives each workgroup a contiguous share and its lanes take the next one from an LDS
	// counter when they start a session, so that a lane with long sessions takes fewer of them
	// (striding had the slowest lanes of a workgroup at 1.7x its mean).
	for (uint32_t k = threadIdx.x * 16u; k < kLdsTableBytes; k += kWalkThreads * 16u)
		*(uint4*)(tabs + k) = *(const uint4*)(d.dfa + k);
	if (threadIdx.x < kLdsStride)
		tabs[kWalkIdCol * kLdsStride + threadIdx.x] = (uint8_t)threadIdx.x; // the identity column
	if (threadIdx.x < 256 / 16)
		*(uint4*)(tabs + kWalkAttrOff + 16u * threadIdx.x) = *(const uint4*)(d.dfa + kLdsTableBytes + 16u * threadIdx.x);
	if (threadIdx.x < kWalkSlots)
		s_cb[threadIdx.x] = 0ull; // chunk 0 is never looked up
	if (threadIdx.x == 0)
		*s_next = kWalkThreads; // the lanes' first sessions are chunk 0
	__syncthreads();
	const ByteTab A{tabs + kWalkAttrOff};
	// A lane walks its sessions one 64-byte window (four 16-byte blocks) per iteration.  A lane
	// whose event ended waits until 60 of the 64 lanes have (or none is still parsing); then the
	// wave ends those events and starts the next ones together: one buffer per lane and step
	// made each wave step as long as its longest buffer, while ending and starting events one
	// lane at a time ran the long end-of-event path (outcome, emission, next event's loads) for
	// a few lanes at a time.
	// Every iteration every lane issues the loads of the window it will need next (its event's
	// next window, else its session's next event's first) and walks the window loaded the
	// iteration before, so the loads' latency hides behind a window's walk.  They are issued
	// unconditionally and in the same order each iteration: with a load issued only on some
	// paths (a 16-byte block rotated through registers), the compiler waited for every load in
	// flight before each block, and each block then cost a memory round trip (clock stamps:
	// 5,600 cycles per block).
	// The next session for a lane of the batch walk (kNone: none left).  The claim precedes the
	// wait in every call, so a lane never waits for a claim by a lane of its own wave that has
	// not run; a claim by another wave is one global atomic away.
	auto take = [&]() -> uint32_t {
		const uint32_t t = atomicAdd(s_next, 1u);
		const uint32_t c = t / kWalkChunk, o = t % kWalkChunk, k = c % kWalkSlots;
		if (o == 0) {
			const uint32_t b = gridDim.x * kWalkChunk + (uint32_t)atomicAdd(d.ctr + CTR_COUNT, (unsigned long long)kWalkChunk);
			__hip_atomic_store(&s_cb[k], ((unsigned long long)c << 32) | b, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
		}
		unsigned long long cb;
		for (uint32_t spins = 0; ((cb = __hip_atomic_load(&s_cb[k], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) >> 32) != c;
				spins++) {
			// a later chunk in the slot (kWalkSlots chunks claimed while this lane waited), or the
			// claimer never storing: neither can happen; reported, never followed or hung on
			if ((cb >> 32) > c || spins > (1u << 22)) {
				set_error(d, EBD_ERR_INTERNAL);
				return kNone;
			}
			__builtin_amdgcn_s_sleep(1);
		}
		const uint32_t hh = (uint32_t)cb + o;
		return hh < nh ? hh : kNone;
	};
	const uint32_t h0 = blockIdx.x * kWalkThreads + threadIdx.x;
	uint32_t h = DRY ? h0 : (h0 < nh ? h0 : kNone);
	bool have = false, in_ev = false, ended = false;
	SessState S;
	uint32_t grp = 0, jj = 0, jhead = 0;
	EvCtx e;
	DfaWalk w;
	uint32_t pos0 = 0, ne = 0, k0 = 0, nb = 0, wi = 0;
	uintptr_t b0 = 0;
	// the window in flight: event tag_i's window tag_w (kNone: nothing useful)
	uint4 Wv[4] = {uint4{0u, 0u, 0u, 0u}, uint4{0u, 0u, 0u, 0u}, uint4{0u, 0u, 0u, 0u}, uint4{0u, 0u, 0u, 0u}};
	uint32_t tag_i = kNone, tag_w = 0;
	uint32_t pf_j = kNone, pf_i = 0, pf_fl = 0, pf_L = 0; // the session's next event, prefetched
	unsigned long long pf_off = 0, nk1 = ~0ull;           // and the sort key after it
	// the lane's next session, one dependent load per refill while the current one is walked,
	// so that starting it waits for nothing: its head position, sort key, first event's words,
	// the key after it, its session-set slot (or, DRY, its first position) and the slot's carry
	uint32_t nx_h = kNone, nx_st = 0, nx_jj = 0, nx_fl = 0, nx_L = 0, nx_slot = 0, nx_carry = 0;
	// the batch walk reads the head record k_walk_heads wrote (two stages); the rounds' walks
	// follow their own list in four (head, key, event words and slot)
	constexpr uint32_t kNxStages = DRY ? 4u : 2u;
	unsigned long long nx_key = 0, nx_k1 = 0, nx_off = 0;
	uint32_t inserts = 0; // CTR_INSERTS: one atomic per wave when it ends
	uint32_t st_ev = 0, st_by = 0; // DRY with dw.stat: this lane's events and bytes walked
	for (;;) {
		const unsigned long long busy = __ballot(in_ev), wait = __ballot(!in_ev && (ended || h < nh));
		if (busy == 0 && wait == 0)
			break;
		if (busy == 0 || __popcll(wait) >= kWalkRefill) {
			if (ended) {
				const uint32_t c = dfa_walk_store(d.di, w, pos0, ne, e.L, (uint8_t)e.flags, S.g);
				const uint32_t op = ev_end<DRY>(d, S, e, c);
				if (op == OP_INSERT) {
					S.live = 1; // saveSession: a new key goes to the front (LRUCache.h:54-60)
					S.stamp = d.seq_base + e.i;
					inserts++;
				}
				if (DRY)
					dw.opt[e.i] = (uint8_t)op;
				ended = false;
			}
			if (have && nx_h < nh && nx_st < kNxStages) { // the next session's pipeline: one stage per refill
				if (!DRY && nx_st == 0) { // its head record (k_walk_heads): position, first event, slot, group
					const uint4 r = d.hrec[nx_h];
					nx_jj = r.x;
					nx_key = ((unsigned long long)r.w << 32) | r.y;
					nx_slot = r.z;
				} else if (!DRY) { // its first event's words, the key after it, the slot's carry word
					const uint32_t i0 = (uint32_t)nx_key;
					nx_fl = d.ev[i0].flags;
					nx_L = d.len[i0];
					nx_off = d.off[i0];
					nx_k1 = nx_jj + 1 < nslow ? d.slow_keys[nx_jj + 1] : ~0ull;
					nx_carry = d.sset[nx_slot].carry;
				} else if (nx_st == 0) {
					nx_jj = heads[nx_h];
				} else if (nx_st == 1) {
					nx_key = d.slow_keys[nx_jj];
				} else if (nx_st == 2) {
					const uint32_t i0 = (uint32_t)nx_key;
					nx_fl = d.ev[i0].flags;
					nx_L = d.len[i0];
					nx_off = d.off[i0];
					nx_k1 = nx_jj + 1 < nslow ? d.slow_keys[nx_jj + 1] : ~0ull;
					nx_slot = dw.head[nx_jj];
				}
				nx_st++;
			}
			while (!in_ev && h < nh) { // the next event that needs a parse, finishing the others
				if (!have) {
					const bool ready = nx_h == h && nx_st == kNxStages;
					unsigned long long key;
					if (ready) {
						jj = nx_jj;
						key = nx_key;
						nk1 = nx_k1;
					} else {
						jj = heads[h];
						key = d.slow_keys[jj];
						nk1 = jj + 1 < nslow ? d.slow_keys[jj + 1] : ~0ull;
					}
					jhead = jj;
					grp = (uint32_t)(key >> 32);
					if (DRY)
						jhead = ready ? nx_slot : dw.head[jj];
					if (jj == jhead) {
						if (!DRY && ready)
							session_begin_c(d, S, jj, nx_slot, nx_carry);
						else
							session_begin(d, S, jj, d.ev_slot[(uint32_t)key]);
					} else {
						S = dw.snap[jj]; // the state before event jj, as the last walk left it
					}
					pf_j = jj; // the first event's words
					pf_i = (uint32_t)key;
					if (ready) {
						pf_fl = nx_fl, pf_L = nx_L, pf_off = nx_off;
					} else {
						pf_fl = d.ev[pf_i].flags, pf_L = d.len[pf_i], pf_off = d.off[pf_i];
					}
					have = true;
					if (DRY) {
						nx_h = h + stride;
					} else {
						nx_h = take();
					}
					nx_st = 0;
				}
				if (pf_j == jj) { // the session's next event (pf_j is set only inside its group)
					const uint32_t i = pf_i, fl = pf_fl, L = pf_L;
					const unsigned long long off = pf_off;
					// the session's next event: its loads (and the sort key after it) travel while
					// this one is walked
					pf_j = kNone;
					const unsigned long long k2 = nk1;
					if (jj + 1 < nslow && (uint32_t)(k2 >> 32) == grp) {
						pf_j = jj + 1;
						pf_i = (uint32_t)k2;
						pf_fl = d.ev[pf_i].flags;
						pf_L = d.len[pf_i];
						pf_off = d.off[pf_i];
						nk1 = jj + 2 < nslow ? d.slow_keys[jj + 2] : ~0ull;
					}
					if (DRY) {
						dw.snap[jj] = S; // the state before event jj: a later walk may start here
						if (i >= hz) { // past the round's horizon: a later round continues here
							dw.wto[jhead] = jj;
							have = false;
							h += stride;
							continue;
						}
					}
					if (!DRY)
						piece_record(d, jj, fl, L, off);
					if (evf && (evf[i] & 1u))
						S.live = 0; // evicted since its previous event: find() misses
					if (ev_begin(d, S, jj, i, fl, L, off, e)) {
						dfa_walk_load(S.g, A[S.g.ds], w);
						pos0 = w.pos;
						ne = dfa_allow(pos0, e.L);
						if (DRY) {
							st_ev++;
							st_by += ne;
						}
						const uintptr_t p = (uintptr_t)(d.payload + off);
						b0 = p & ~(uintptr_t)15;
						k0 = (uint32_t)(p & 15u);
						nb = ne ? (k0 + ne + 15u) >> 4 : 0u;
						wi = 0;
						in_ev = true;
					} else {
						const uint32_t op = ev_end<DRY>(d, S, e, 0);
						if (DRY)
							dw.opt[i] = (uint8_t)op;
					}
					jj++;
				} else {
					if (!DRY && S.live && !(evf && (evf[slow_event(d, jhead)] & 2u)))
						session_carry_out(d, S, jhead, jj - 1);
					if (DRY)
						dw.wto[jhead] = kNone; // walked to its end
					have = false;
					h = DRY ? h + stride : nx_h;
				}
			}
		}
		// the window loaded last iteration (the copy waits for those loads only)
		const uint4 X[4] = {Wv[0], Wv[1], Wv[2], Wv[3]};
		const bool valid = in_ev && (nb == 0 || (tag_i == e.i && tag_w == wi)); // nb = 0: nothing to walk
		{ // the next window: this event's next one, or the session's next event's first
			uintptr_t nbase = (uintptr_t)d.payload;
			uint32_t nlast = 0, ni = kNone, nw = 0;
			if (in_ev && (!valid || 4u * (wi + 1) < nb)) {
				nbase = b0;
				nlast = nb ? nb - 1u : 0u;
				ni = e.i;
				nw = valid ? wi + 1 : wi;
			} else if (pf_j != kNone && (pf_fl & FLAG_NEW) && pf_L != EBD_NO_BUFFER && pf_L && buf_in(d, pf_L, pf_off)) {
				const uintptr_t pp = (uintptr_t)(d.payload + pf_off);
				nbase = pp & ~(uintptr_t)15;
				nlast = ((uint32_t)(pp & 15u) + pf_L - 1u) >> 4;
				ni = pf_i;
				nw = 0;
			}
#pragma unroll
			for (uint32_t k = 0; k < 4; k++) { // global (not flat) loads: counted by vmcnt alone
				const v4u v = *(const __attribute__((address_space(1))) v4u*)(nbase + 16u * min(4u * nw + k, nlast));
				Wv[k] = uint4{v.x, v.y, v.z, v.w};
			}
			tag_i = ni;
			tag_w = nw;
		}
		if (valid) {
#pragma unroll
			for (uint32_t k = 0; k < 4; k++) { // dfa_parse_dev's blocks
				const uint32_t bk = 4u * wi + k;
				if (bk < nb && w.tpos == kNone) {
					const uint32_t wd[4] = {X[k].x, X[k].y, X[k].z, X[k].w};
					const uint32_t base = 16u * bk - k0;
					walk_block(tabs, w, wd, base, pos0 + base, ne);
				}
			}
			wi++;
			if (4u * wi >= nb || w.tpos != kNone) {
				in_ev = false;
				ended = true;
			}
		}
	}
	if (!DRY) { // the loop ends for the whole wave at once
		for (int o = 32; o > 0; o >>= 1)
			inserts += __shfl_xor(inserts, o, 64);
		if ((threadIdx.x & 63) == 0 && inserts)
			atomicAdd(&d.ctr[CTR_INSERTS], (unsigned long long)inserts);
	} else if (dw.stat) {
		uint32_t mx = st_by;
		for (int o = 32; o > 0; o >>= 1) {
			st_ev += __shfl_xor(st_ev, o, 64);
			st_by += __shfl_xor(st_by, o, 64);
			mx = max(mx, (uint32_t)__shfl_xor(mx, o, 64));
		}
		if ((threadIdx.x & 63) == 0) {
			atomicAdd(&dw.stat[0], (unsigned long long)st_ev);
			atomicAdd(&dw.stat[1], (unsigned long long)st_by);
			atomicMax(&dw.stat[3], (unsigned long long)mx);
		}
	}
}

// The batch walk (with output) and the exact-LRU rounds' dry walks: one body, two kernels, so
// that the register budget (EBD_WALK_WPE) binds the batch walk alone; the dry walk kept at the
// compiler's budget was faster (1 M-event exact LRU: 83 against 87 ms per batch).
__global__ __launch_bounds__(kWalkThreads) EBD_WALK_ATTR void k_walk(Dev d, const uint8_t* evf, DryWalk dw, const uint32_t* hlist,
		const uint32_t* hcount) {
	walk_sessions<false>(d, evf, dw, hlist, hcount);
}
__global__ __launch_bounds__(kWalkThreads) void k_walk_dry(Dev d, const uint8_t* evf, DryWalk dw, const uint32_t* hlist,
		const uint32_t* hcount) {
	walk_sessions<true>(d, evf, dw, hlist, hcount);
}

// After a walker: every sorted session event was replayed once (Discovery::handleNewEvent)
// and every session request counted once (the walkers bump no per-event counter).
__global__ void k_sess_tally(Dev d) {
	d.ctr[CTR_SESSION_EVENTS] += d.ctr[CTR_SLOW];
	d.ctr[CTR_REQUESTS] += d.ctr[CTR_SREQ];
}

// Saved sessions with no event in this batch stay saved unchanged.
__global__ void k_carry_pass(Dev d, const uint8_t* cevf) {
	for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < d.n_carry_in; c += gridDim.x * blockDim.x) {
		if (cevf && cevf[c])
			continue; // evicted (the exact-LRU rounds)
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
// Everything but the close flag comes from the sort key: a session's group is its carry index
// (carried) or carry_cap + its first UNFINISHED event (k_slow_collect), and its last event of
// the batch is the last of its group.  Only a session's entry and close events write (delta
// and minus are zeroed before), and only a session's last event reads its event record.
__global__ void k_lru_delta(Dev d, uint32_t nslow, int* delta, uint8_t* minus) {
	for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nslow; j += gridDim.x * blockDim.x) {
		const unsigned long long key = d.slow_keys[j];
		const uint32_t grp = (uint32_t)(key >> 32), i = (uint32_t)key;
		const bool carried = grp < d.carry_cap;
		const uint32_t first = carried ? kNone : grp - d.carry_cap;
		const bool plus = !carried && first == i;
		const bool last = j + 1 == nslow || (uint32_t)(d.slow_keys[j + 1] >> 32) != grp;
		const bool close = last && (carried || first <= i) && (d.ev[i].flags & FLAG_END);
		if (plus != close)
			delta[i] = plus ? 1 : -1;
		if (close)
			minus[i] = 1;
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
	__shared__ unsigned long long rs[kLruThreads / 64];
	__shared__ uint32_t ri[kLruThreads / 64];
	__shared__ __attribute__((aligned(16))) uint8_t tabs[kLdsTableBytes + 256];
	const uint32_t t = threadIdx.x;
	for (uint32_t k = t * 16u; k < kLdsTableBytes + 256; k += kLruThreads * 16u)
		*(uint4*)(tabs + k) = *(const uint4*)(d.dfa + k);
	const SessTabs tb{tabs, tabs + kLdsTableBytes};
	if (t == 0)
		nlive = 0;
	__syncthreads();
	// every session's state at the batch start; the carried ones are in the LRU
	for (uint32_t j = t; j < nslow; j += kLruThreads)
		if (head[j] == j) {
			session_begin(d, S[j], j, d.ev_slot[slow_event(d, j)]);
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
		if (t >= 64) {
			// waves 1-3 pull the chunk's session state, event metadata and first payload lines
			// into L2 while lane 0 walks it (its chain of dependent loads then hits L2, not HBM)
			uint32_t sink = 0;
			for (uint32_t q = t - 64; q < nord; q += kLruThreads - 64) {
				const uint32_t jj = ord[q], h = head[jj], i = slow_event(d, jj);
				const volatile uint32_t* sp = (const volatile uint32_t*)(S + h);
				sink ^= sp[0] ^ sp[sizeof(SessState) / 4 - 1];
				const uint32_t L = d.len[i];
				const unsigned long long po = d.off[i];
				if ((d.ev[i].flags & FLAG_NEW) && L != 0 && buf_in(d, L, po)) {
					const unsigned long long pe = po + min(L, 512u);
					for (unsigned long long o = po & ~127ull; o < pe; o += 128)
						sink ^= *(const volatile uint32_t*)(d.payload + o); // inside the buffer's page
				}
			}
			if (sink == 0x9e3779b9u && d.n == 0xffffffffu) // never: keeps the loads
				set_error(d, EBD_ERR_INTERNAL);
		}
		uint32_t k = 0;
		while (k < nord) { // uniform
			if (t == 0) {
				uint32_t e = kNone;
				for (; k < nord; k++) {
					const uint32_t jj = ord[k], h = head[jj];
					const uint32_t op = session_event(d, tb, S[h], jj);
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
				for (uint32_t m = 32; m > 0; m >>= 1) { // the wave's minimum (stamps are unique)
					const unsigned long long ob = __shfl_xor(best, (int)m);
					const uint32_t oi = __shfl_xor(bi, (int)m);
					if (ob < best) {
						best = ob;
						bi = oi;
					}
				}
				if ((t & 63) == 0) {
					rs[t >> 6] = best;
					ri[t >> 6] = bi;
				}
				__syncthreads();
				if (t == 0) {
					for (uint32_t x = 1; x < kLruThreads / 64; x++)
						if (rs[x] < rs[0]) {
							rs[0] = rs[x];
							ri[0] = ri[x];
						}
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

// ---------------------------------------------------------------------------------
// Exact LRU in rounds (the parallel form of k_walk_lru).  A world is a set of evictions, as
// flags on the session events at which a session finds itself evicted (k_walk's evf).  A
// round walks sessions in the current world without output (k_walk_dry), which gives every
// session event its LRU operation, then derives the evictions those operations imply:
//  * the LRU's size after each event follows from the operation types alone: an insert makes
//    it min(cap, L + 1) (a full cache evicts first, LRUCache.h:54-60), an erase L - 1.  Maps
//    x -> min(a, x + b) compose within their family, so the sizes come from a scan over event
//    order (k_lru_scan_*), and an insert evicts exactly when the size before it is cap;
//  * an eviction removes the least recently used session.  Every insert or access starts a
//    "marker" (the session's recency) that lasts until the session's next find; the evicted
//    session is the oldest marker still alive, and since evictions only ever take the oldest,
//    they take markers in position order: one merge of the markers (carried sessions first,
//    by recency) with the eviction times (k_lru_greedy).
// The victim's next find (where its absence shows) gets the eviction flag.  If the walked
// flags first differ from the sequential ones at event T, the operations before T are the
// sequential ones, so are the evictions before T, their victims, and every derived flag up
// to T: each round settles at least one more event, and a round that derives the world it
// walked has found the sequential execution (tests/test_lru_rounds.py restates the rounds and
// checks them against a sequential LRU).  A victim's absence shows at its next find, about one
// inter-event gap of a session later, so that is how far a round moves the settled frontier F.
// A round therefore only derives the evictions in a window [F, F + H) (the greedy resumes at
// F from its saved state) and only walks again the sessions whose flags changed.
// ---------------------------------------------------------------------------------
constexpr int kScT = 1024, kScPer = 4;
constexpr uint32_t kLsBlk = kScT * kScPer; // events per scan block
// x -> min(a, x + b) in 32 bits: sizes stay below 2^30 (the LRU capacity and the carried
// sessions, checked on the host), a block's b within +-kLsBlk
constexpr int kLInf = 1 << 30;
struct LFn {
	int a, b;
};
__device__ __forceinline__ LFn lfn_id() { return LFn{kLInf, 0}; }
__device__ __forceinline__ LFn lfn_op(uint32_t op, uint32_t cap) {
	return op == OP_INSERT ? LFn{(int)cap, 1} : op == OP_ERASE ? LFn{kLInf, -1} : lfn_id();
}
__device__ __forceinline__ LFn lfn_then(LFn f, LFn g) { return LFn{min(g.a, f.a + g.b), f.b + g.b}; } // g after f
__device__ __forceinline__ int lfn_apply(LFn f, int x) { return min(f.a, x + f.b); }
__device__ __forceinline__ bool op_marks(uint32_t op) { return op == OP_INSERT || op == OP_ACCESS; }

// Once per batch: each session event's next find (Discovery.cpp:114 for a buffer, :195 for a
// close) in mend (by event), and per carried session its first find and first sorted
// position (cm_end, cm_head: kNone before).
__global__ void k_lru_static(Dev d, uint32_t nslow, uint32_t* mend, uint32_t* cm_end, uint32_t* cm_head) {
	for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nslow; j += gridDim.x * blockDim.x) {
		const unsigned long long key = d.slow_keys[j];
		const uint32_t grp = (uint32_t)(key >> 32), i = (uint32_t)key;
		auto next_find = [&](uint32_t from) {
			for (uint32_t q = from; q < nslow && (uint32_t)(d.slow_keys[q] >> 32) == grp; q++) {
				const uint32_t iq = (uint32_t)d.slow_keys[q], fl = d.ev[iq].flags, L = d.len[iq];
				if ((fl & FLAG_END) || ((fl & FLAG_NEW) && L != EBD_NO_BUFFER && buf_in(d, L, d.off[iq])))
					return iq;
			}
			return kNone;
		};
		mend[i] = next_find(j + 1);
		const bool headj = j == 0 || (uint32_t)(d.slow_keys[j - 1] >> 32) != grp;
		if (headj && grp < d.carry_cap) { // a carried session (its group is its carry index)
			cm_head[grp] = j;
			cm_end[grp] = next_find(j);
		}
	}
}

// The carried sessions' markers, least recently used first (stamps are unique event positions).
__global__ void k_lru_carry_rank(Dev d, const uint32_t* cm_end, uint32_t* mk_ref, uint32_t* mk_e) {
	const uint32_t nc = d.n_carry_in;
	for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < nc; c += gridDim.x * blockDim.x) {
		const unsigned long long st = d.carry_in[c].stamp;
		uint32_t rank = 0;
		for (uint32_t o = 0; o < nc; o++) {
			const unsigned long long so = d.carry_in[o].stamp;
			rank += (so < st || (so == st && o < c)) ? 1u : 0u;
		}
		mk_ref[rank] = 0x80000000u | c;
		mk_e[rank] = cm_end[c];
	}
}

// The round's walks: per session (k_walk_heads' list), from its first changed position if
// that lies in the part walked before (cpos; cleared here), else from where the last walk
// stopped (wto) if that event comes before the horizon.  Entries are start positions.
// zc, zn: the round's carried-session flags (ncf), cleared on the way.
__global__ void k_lru_walklist(Dev d, uint32_t* cpos, const uint32_t* wto, const LruCtrl* ctl, uint32_t* rlist, uint32_t* tot,
		uint8_t* zc, uint32_t zn) {
	if (ctl->done)
		return;
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < zn; k += gridDim.x * blockDim.x)
		zc[k] = 0;
	const uint32_t hz = ctl->tend;
	const uint32_t nh = (uint32_t)d.ctr[CTR_HEADS];
	for (uint32_t h = blockIdx.x * blockDim.x + threadIdx.x; h < nh; h += gridDim.x * blockDim.x) {
		const uint32_t jh = d.heads[h], c = cpos[jh], wt = wto[jh];
		uint32_t start = kNone;
		if (c != kNone) {
			cpos[jh] = kNone;
			if (wt == kNone || c < wt)
				start = c;
		}
		if (wt != kNone && (uint32_t)d.slow_keys[wt] < hz)
			start = min(start, wt);
		if (start != kNone)
			rlist[atomicAdd(&tot[3], 1u)] = start;
	}
}

// The scan blocks a round derives: from the frontier's to the horizon's (the operations before
// the frontier are settled, so are the earlier blocks' markers, evictions and start states
// from the round that last derived them; nothing past the horizon is used).
struct LsSpan {
	uint32_t first, last; // scan blocks, inclusive
};
__device__ __forceinline__ LsSpan lru_span(const LruCtrl* ctl, uint32_t n) {
	const uint32_t nb = (n + kLsBlk - 1) / kLsBlk, tend = ctl->tend;
	const uint32_t first = min(ctl->front, n ? n - 1 : 0u) / kLsBlk;
	const uint32_t last = tend < n ? tend / kLsBlk : (nb ? nb - 1 : 0u);
	return LsSpan{first, last};
}

// Phases 1-5 in one workgroup over the span (about window / kLsBlk + 1 blocks), up to
// kScChunk blocks per pass, each thread a run of consecutive events: the LRU's size before
// each event (maps x -> min(a, x + b) scanned in event order from the span's start state), the
// evictions (an insert that finds the cache full), and the markers (event, end) and eviction
// times in order, numbered on from the start state; evc[i] = the evictions before event i;
// bs[b] = the state at each block start passed.  tot[5] = the evictions before the frontier,
// tot[6] / tot[7] = the markers / evictions before the horizon, tot[1] = the evictions up to
// the span's end.  The outputs gather in LDS and leave in coalesced rows (one workgroup's
// scattered 4-byte stores were what the kernel spent its time on).
constexpr uint32_t kScChunk = 2, kScEv = kScChunk * kLsBlk; // events per pass
__device__ __forceinline__ LFn lfn_shfl_up(LFn f, uint32_t o) { return LFn{__shfl_up(f.a, o, 64), __shfl_up(f.b, o, 64)}; }
__global__ __launch_bounds__(kScT) void k_lru_scan(const uint8_t* opt, const uint32_t* mend, uint32_t n, uint32_t cap, LsState* bs,
		uint32_t* mk_ref, uint32_t* mk_e, uint32_t* ev_t, uint32_t* evc, uint32_t* tot, const LruCtrl* ctl) {
	if (ctl->done)
		return;
	constexpr uint32_t kW = kScT / 64, kPer = kScPer * kScChunk;
	const LsSpan sp = lru_span(ctl, n);
	const uint32_t front = ctl->front, tend = ctl->tend;
	// one LDS object: [evc | marker events | marker ends | eviction times] of a pass, then the
	// waves' totals
	__shared__ uint32_t lds[4 * kScEv + 4 * kW];
	uint32_t* s_evc = lds;
	uint32_t* s_mref = lds + kScEv;
	uint32_t* s_me = lds + 2 * kScEv;
	uint32_t* s_ev = lds + 3 * kScEv;
	LFn* wf = (LFn*)(lds + 4 * kScEv);
	uint32_t* wm = lds + 4 * kScEv + 2 * kW;
	uint32_t* we = lds + 4 * kScEv + 3 * kW;
	const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
	LsState st = bs[sp.first];
	for (uint32_t b0 = sp.first; b0 <= sp.last; b0 += kScChunk) {
		const uint32_t nbk = min(kScChunk, sp.last + 1 - b0), per = kScPer * nbk; // events per thread
		const uint32_t ib = b0 * kLsBlk, i0 = ib + t * per;
		uint32_t ow[kScChunk]; // the thread's operations, 4 per word (OP_NONE past the batch)
#pragma unroll
		for (uint32_t q = 0; q < kScChunk; q++) {
			const uint32_t iq = i0 + 4 * q;
			ow[q] = 0;
			if (q < nbk) {
				if (iq + 4 <= n) {
					ow[q] = *(const uint32_t*)(opt + iq);
				} else {
					for (uint32_t k = 0; k < 4; k++)
						if (iq + k < n)
							ow[q] |= (uint32_t)opt[iq + k] << (8 * k);
				}
			}
		}
		// the markers' ends (loads in flight across the scans)
		uint32_t me[kPer];
#pragma unroll
		for (uint32_t k = 0; k < kPer; k++)
			me[k] = k < per && i0 + k < n && op_marks((ow[k >> 2] >> (8 * (k & 3u))) & 0xffu) ? mend[i0 + k] : 0u;
		LFn f = lfn_id();
		uint32_t mk = 0;
#pragma unroll
		for (uint32_t q = 0; q < kScChunk; q++)
#pragma unroll
			for (uint32_t k = 0; k < 4; k++) {
				const uint32_t op = (ow[q] >> (8 * k)) & 0xffu;
				f = lfn_then(f, lfn_op(op, cap));
				mk += op_marks(op) ? 1u : 0u;
			}
		LFn fi = f; // inclusive over the wave
		uint32_t mi = mk;
#pragma unroll
		for (uint32_t o = 1; o < 64; o <<= 1) {
			const LFn g = lfn_shfl_up(fi, o);
			const uint32_t mg = __shfl_up(mi, o, 64);
			if (lane >= o) {
				fi = lfn_then(g, fi);
				mi += mg;
			}
		}
		if (lane == 63) {
			wf[wv] = fi;
			wm[wv] = mi;
		}
		__syncthreads();
		LFn pre = lfn_id();
		uint32_t ml = 0; // markers of the pass before the thread's
		for (uint32_t w = 0; w < wv; w++) {
			pre = lfn_then(pre, wf[w]);
			ml += wm[w];
		}
		const LFn fx = lfn_shfl_up(fi, 1);
		const uint32_t mx_ = __shfl_up(mi, 1, 64);
		if (lane) {
			pre = lfn_then(pre, fx);
			ml += mx_;
		}
		const int x0 = lfn_apply(pre, st.x);
		int x = x0;
		uint32_t evs = 0, ne = 0; // the thread's evictions, bit k = its event k
#pragma unroll
		for (uint32_t q = 0; q < kScChunk; q++)
#pragma unroll
			for (uint32_t k = 0; k < 4; k++) {
				const uint32_t op = (ow[q] >> (8 * k)) & 0xffu;
				const bool ev = op == OP_INSERT && x >= (int)cap;
				evs |= (ev ? 1u : 0u) << (4 * q + k);
				ne += ev ? 1u : 0u;
				x = lfn_apply(lfn_op(op, cap), x);
			}
		uint32_t ni = ne;
#pragma unroll
		for (uint32_t o = 1; o < 64; o <<= 1) {
			const uint32_t g = __shfl_up(ni, o, 64);
			if (lane >= o)
				ni += g;
		}
		if (lane == 63)
			we[wv] = ni;
		__syncthreads();
		uint32_t el = ni - ne; // evictions of the pass before the thread's
		for (uint32_t w = 0; w < wv; w++)
			el += we[w];
		x = x0;
#pragma unroll
		for (uint32_t k = 0; k < kPer; k++) {
			const uint32_t i = i0 + k;
			if (k >= per || i >= n)
				continue;
			const uint32_t op = (ow[k >> 2] >> (8 * (k & 3u))) & 0xffu;
			if ((i & (kLsBlk - 1u)) == 0)
				bs[i / kLsBlk] = LsState{x, st.m + ml, st.e + el, 0u}; // a block start: a later round may start there
			if (i == front)
				tot[5] = st.e + el;
			if (i == tend) {
				tot[6] = st.m + ml;
				tot[7] = st.e + el;
			}
			s_evc[i - ib] = st.e + el;
			if (op_marks(op)) {
				s_mref[ml] = i;
				s_me[ml] = me[k];
				ml++;
			}
			if ((evs >> k) & 1u)
				s_ev[el++] = i;
			x = lfn_apply(lfn_op(op, cap), x);
		}
		LFn tf = lfn_id();
		uint32_t pm = 0, pe = 0;
		for (uint32_t w = 0; w < kW; w++) {
			tf = lfn_then(tf, wf[w]);
			pm += wm[w];
			pe += we[w];
		}
		__syncthreads();
		const uint32_t nev_pass = min(nbk * kLsBlk, n - ib);
		for (uint32_t k = t; k < nev_pass; k += kScT)
			evc[ib + k] = s_evc[k];
		for (uint32_t k = t; k < pm; k += kScT) {
			mk_ref[st.m + k] = s_mref[k];
			mk_e[st.m + k] = s_me[k];
		}
		for (uint32_t k = t; k < pe; k += kScT)
			ev_t[st.e + k] = s_ev[k];
		st.x = lfn_apply(tf, st.x);
		st.m += pm;
		st.e += pe;
		__syncthreads(); // the LDS is reused
	}
	if (t == 0) {
		if (tend >= n) {
			tot[6] = st.m;
			tot[7] = st.e;
		}
		tot[1] = st.e;
	}
}

// Phase 6: the window's evictions [j0, jend) (those from the frontier to the horizon) take the
// oldest marker alive at their time, in order (LRUCache.h:54-60's evict-the-back in the
// sequential walk).  The merge resumes at qf, after the victim of eviction j0 - 1 (that
// victim and every earlier marker is taken or dead by then), and only markers born before the
// horizon can be victims (a later one would be an inconsistency k_lru_victims reports).  Taken
// from the markers' side: marker m (in order) goes to eviction A, the evictions done so far,
// when it is alive then, i.e. A < c_m = the window's evictions before its end e_m, and A += 1.
// The map A -> A + [A < c] composes over a block of 64 markers into A -> A + #{k : A < X_k}
// with one threshold per marker (marker k of the block is taken iff the block starts at
// A < X_k), so k_lru_thresh derives every block's thresholds in parallel and k_lru_take
// chains the blocks, one compare and popcount each, listing the victims (vict[j] = eviction
// j's marker).  tot[2] = the window's end (first eviction not processed); cnt[1] = 1: the
// operations are inconsistent (a full cache with no victim).
constexpr uint32_t kThT = 256;
__device__ __forceinline__ uint32_t lru_queue_front(const uint32_t* tot, const uint32_t* vict) {
	const uint32_t j0 = tot[5];
	return j0 ? vict[j0 - 1] + 1u : 0u;
}
// c_m from evc (the evictions before the marker's end).  The thresholds: with S the block's
// positive thresholds so far (distinct; ms of them), the map A -> A + #{S > A} rises by one
// at every A not in S, so X_k = the (c_k - ms)-th positive integer not in S (0 when
// c_k <= ms: the markers before take c_k evictions from any start).  S is kept sorted in the
// lanes: that integer is r + #{s_j : s_j - j < r} (one ballot), and it goes in at that rank
// (a wave shift by one lane).
__global__ __launch_bounds__(kThT) void k_lru_thresh(const uint32_t* mk_e, const uint32_t* evc, const uint32_t* tot, const LruCtrl* ctl,
		const uint32_t* vict, uint32_t* mx) {
	if (ctl->done)
		return;
	const uint32_t j0 = tot[5], jend = tot[7], mend = tot[6], qf = lru_queue_front(tot, vict), tend = ctl->tend;
	if (jend <= j0 || qf >= mend)
		return;
	const uint32_t nj = jend - j0, nbk = (mend - qf + 63u) / 64u, wpb = kThT / 64u;
	const uint32_t lane = threadIdx.x & 63u;
	for (uint32_t bk = blockIdx.x * wpb + (threadIdx.x >> 6); bk < nbk; bk += gridDim.x * wpb) {
		const uint32_t m = qf + 64u * bk + lane;
		uint32_t c = 0; // the window's evictions before the marker's end
		if (m < mend) {
			const uint32_t e = mk_e[m];
			if (e >= tend) {
				c = nj; // kNone (never found again) included
			} else {
				const uint32_t eb = evc[e];
				c = eb > j0 ? min(eb, jend) - j0 : 0u;
			}
		}
		uint32_t S = 0, X = 0, ms = 0;
		for (unsigned long long live = __ballot(c > 0); live; live &= live - 1) {
			const uint32_t k = (uint32_t)__builtin_ctzll(live);
			const uint32_t ck = (uint32_t)__builtin_amdgcn_readlane((int)c, (int)k);
			if (ck <= ms)
				continue;
			const uint32_t r = ck - ms;
			const uint32_t i = (uint32_t)__popcll(__ballot(lane < ms && S < r + lane + 1u));
			const uint32_t xk = r + i;
			const uint32_t sh = (uint32_t)__builtin_amdgcn_update_dpp((int)S, (int)S, 0x138, 0xf, 0xf, false); // wave_shr:1
			S = lane > i ? sh : lane == i ? xk : S;
			ms++;
			if (lane == k)
				X = xk;
		}
		if (m < mend)
			mx[m - qf] = X;
	}
}

constexpr uint32_t kTkM = 16384; // thresholds staged in LDS at a time
__global__ __launch_bounds__(kThT) void k_lru_take(const uint32_t* mx, uint32_t* tot, const LruCtrl* ctl, uint32_t* vict,
		unsigned long long* cnt) {
	if (ctl->done)
		return;
	const uint32_t j0 = tot[5], jend = tot[7], mend = tot[6], nev = tot[1], qf = lru_queue_front(tot, vict);
	const uint32_t nj = jend - j0, nm = mend > qf ? mend - qf : 0u;
	__shared__ uint32_t sx[kTkM];
	__shared__ uint32_t s_x;
	const uint32_t t = threadIdx.x, lane = t & 63u;
	if (t == 0)
		s_x = 0;
	__syncthreads();
	for (uint32_t c0 = 0; c0 < nm && s_x < nj; c0 += kTkM) {
		const uint32_t cn = min(kTkM, nm - c0);
		for (uint32_t k0 = 0; k0 < kTkM; k0 += kThT * 16) {
			uint32_t v[16];
#pragma unroll
			for (uint32_t u = 0; u < 16; u++) {
				const uint32_t k = k0 + u * kThT + t;
				v[u] = k < cn ? mx[c0 + k] : 0u;
			}
#pragma unroll
			for (uint32_t u = 0; u < 16; u++)
				sx[k0 + u * kThT + t] = v[u];
		}
		__syncthreads();
		if (t < 64) {
			uint32_t x = s_x;
			for (uint32_t b = 0; b < cn && x < nj; b += 8 * 64) {
				uint32_t xv[8];
#pragma unroll
				for (uint32_t u = 0; u < 8; u++)
					xv[u] = sx[b + 64u * u + lane]; // past cn: 0, never taken
#pragma unroll
				for (uint32_t u = 0; u < 8; u++) {
					const unsigned long long tk = __ballot(x < xv[u]);
					if (x < xv[u])
						vict[j0 + x + __builtin_amdgcn_mbcnt_hi((uint32_t)(tk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)tk, 0))] =
								qf + c0 + b + 64u * u + lane;
					x += (uint32_t)__popcll(tk);
				}
			}
			if (t == 0)
				s_x = x;
		}
		__syncthreads();
	}
	if (t == 0) {
		const uint32_t x = s_x;
		tot[2] = j0 + x; // jend unless the markers ran out
		cnt[0] = nev;
		if (x < nj)
			atomicOr((uint32_t*)&cnt[1], 1u); // a full cache and no live marker
	}
}

// Phase 6b: the world the evictions before the window's end imply, by event in nf (zero
// before): 1 at the victim's next find; for a victim with none, 2 at its session's first event
// (evicted after its last event: not carried out), or for a carried session with no event in
// the batch ncf (zeroed before).  Every position gets at most one of them: a marker's next
// find follows it in its session, so it is never a batch session's first event, and only a
// session's last marker has none.
__global__ void k_lru_victims(Dev d, const uint32_t* tot, const uint32_t* vict, const uint32_t* mk_ref, const uint32_t* mk_e,
		const uint32_t* ev_t, const uint32_t* jpos, const uint32_t* head, const uint32_t* cm_head, uint8_t* nf, uint8_t* ncf,
		unsigned long long* cnt, const LruCtrl* ctl) {
	if (ctl->done)
		return;
	const uint32_t ne = tot[2];
	for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < ne; j += gridDim.x * blockDim.x) {
		const uint32_t q = vict[j], vr = mk_ref[q], ve = mk_e[q];
		if (!(vr & 0x80000000u) && vr >= ev_t[j])
			atomicOr((uint32_t*)&cnt[1], 1u); // the oldest live marker is not older than the insert
		if (ve != kNone) {
			nf[ve] = 1; // find() misses at the session's next find
		} else if (vr & 0x80000000u) {
			const uint32_t c = vr & 0x7fffffffu;
			if (cm_head[c] != kNone)
				nf[(uint32_t)d.slow_keys[cm_head[c]]] = 2;
			else
				ncf[c] = 1;
		} else {
			nf[(uint32_t)d.slow_keys[head[jpos[vr]]]] = 2;
		}
	}
}

// Phase 7 (by event, coalesced): how many flags the round changed (cnt[2], carried ones
// included), the first event whose eviction bit changed (cnt[3]: the new frontier), and where
// each session's walk must start again (cpos).  The walked world f is cleared behind the read:
// it is the next round's zeroed target.
__global__ void k_lru_diff(uint32_t n, uint8_t* f, const uint8_t* nf, const uint8_t* cf, const uint8_t* ncf, uint32_t ncc,
		const uint32_t* jpos, const uint32_t* head, uint32_t* cpos, unsigned long long* cnt, const LruCtrl* ctl) {
	if (ctl->done)
		return;
	uint32_t x = 0, first = kNone;
	const uint32_t n4 = n / 4u;
	for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n4 + ncc; q += gridDim.x * blockDim.x) {
		if (q < n4) {
			const uint32_t o4 = ((const uint32_t*)f)[q], v4 = ((const uint32_t*)nf)[q];
			if (o4)
				((uint32_t*)f)[q] = 0;
			if (o4 == v4)
				continue;
			for (uint32_t k = 0; k < 4; k++) {
				const uint32_t o = (o4 >> (8 * k)) & 0xffu, v = (v4 >> (8 * k)) & 0xffu, i = 4 * q + k;
				x += o != v ? 1u : 0u;
				if ((o ^ v) & 1u) { // the walk changes only with bit 0
					const uint32_t j = jpos[i];
					atomicMin(&cpos[head[j]], j); // its session walks again from here
					first = i < first ? i : first;
				}
			}
		} else {
			x += cf[q - n4] != ncf[q - n4] ? 1u : 0u;
		}
	}
	if (blockIdx.x == 0 && threadIdx.x < n - 4u * n4) { // the last events (n % 4)
		const uint32_t i = 4u * n4 + threadIdx.x;
		const uint8_t o = f[i], v = nf[i];
		f[i] = 0;
		x += o != v ? 1u : 0u;
		if ((o ^ v) & 1u) {
			const uint32_t j = jpos[i];
			atomicMin(&cpos[head[j]], j);
			first = i < first ? i : first;
		}
	}
	if (__any(x != 0))
		wave_add(&cnt[2], (unsigned long long)x);
	if (first != kNone)
		atomicMin(&cnt[3], (unsigned long long)first);
}

// Aggregator::newRequest for the fast-path requests (coalesced reads of the results, keys
// and events).  The client class comes from the client-IP header's front token when k_fresh
// found one (cip_classify), else from the session's source address (Aggregator.cpp:60-66,
// 85-88).  A block walks a contiguous range of the batch 256 events at a time, each wave
// its own 64 of them, and the waves never wait for each other: every step of a wave is a
// chain of dependent random accesses (result, key, slot probe, claim / counter atomics), and
// a block-wide barrier per step made each step last as long as the slowest of 256 chains.
// Requests with a client-IP header (~30 % in config 3) go to the wave's own LDS ring and are
// parsed 64 at a time, so the token parse, the longest code path, runs on full waves instead
// of on the few lanes of each wave that have one.  Aggregation is order-free (counters,
// atomicMin of the first-arrival word), so queueing does not change the result.
//
// A service created here only claims its slot: the claim (slot, claiming event) goes to the
// block's own stretch of the claim stage, counted in LDS, with no global atomic.  The
// publication kernels then give every block's claims their list entries and arena bytes from
// a scan of the per-block counts (k_pub_count, k_pub_scan) and copy the endpoint bytes
// (k_publish).  A single global counter serialises at ~12 ns per atomic: reserving per block
// and step cost ~5 ms per 100 M-event batch that creates 30 M services.
constexpr uint32_t kAggWaves = kAggThreads / 64;
constexpr uint32_t kCipRing = 128; // per wave: < 64 waiting + at most 64 new per step

struct AggShared {
	uint32_t q[kAggWaves][kCipRing]; // each wave's queued client-IP requests (a ring)
	uint32_t cn;                     // claims of this block
	unsigned long long nreq;
};

__device__ __forceinline__ void agg_request(const Dev& d, uint32_t i, const ebd_event_result& r, uint32_t cls, AggShared& sh,
		unsigned long long net) {
	bool claimed;
	const Hash128 key = d.keys[i];
	const uint32_t slot = agg_insert(d, key, first_word(d.seq_base + i, (r.info & EBD_INFO_HTTPS) != 0, r.u.span.host_len),
			cls == CLS_INTERNAL, cls == CLS_EXTERNAL, &claimed);
	if (d.net_on && cls == CLS_EXTERNAL)
		agg_nets(d, slot, net, request_time(d, i));
	if (claimed) { // at most one claim per event: the block's stretch holds them all
		const uint32_t k = atomicAdd(&sh.cn, 1u);
		const unsigned long long at = (unsigned long long)blockIdx.x * d.cstage_per + k;
		ClaimRec cr;
		cr.slot = slot;
		cr.pid = d.ev[i].pid;
		cr.host_off = r.u.span.host_off;
		cr.host_len = r.u.span.host_len;
		cr.url_off = r.u.span.url_off;
		cr.url_len = r.u.span.url_len;
		cr.off = d.off[i];
		d.cstage[at] = cr;
	}
}

__device__ __forceinline__ void agg_cip_one(const Dev& d, uint32_t i, uint8_t* row, AggShared& sh) {
	ebd_event_result r = d.res[i];
	unsigned long long net = 0;
	const uint32_t cls = cip_classify(d, i, r, row, &net);
	r.info = (uint8_t)((r.info & ~(3u << EBD_INFO_CLASS_SHIFT)) | (cls << EBD_INFO_CLASS_SHIFT));
	d.res[i] = r;
	agg_request(d, i, r, cls, sh, net);
}

// Steps (of kAggThreads events) per block; the claim stage holds per * kAggThreads per block.
EBD_HD uint32_t agg_steps_per_block(uint32_t n, uint32_t grid) {
	const uint32_t steps = (n + kAggThreads - 1) / kAggThreads;
	return (steps + grid - 1) / grid;
}

// 6 waves per SIMD: the compiler fits the kernel in 80 VGPRs without spilling (91 unbounded, 5 waves)
#ifndef EBD_AGG_WAVES
#define EBD_AGG_WAVES 6
#endif
__global__ __launch_bounds__(kAggThreads) __attribute__((amdgpu_waves_per_eu(EBD_AGG_WAVES, 8))) void k_agg_fast(Dev d) {
	__shared__ __attribute__((aligned(8))) uint8_t rows[kAggThreads * kCipStride];
	__shared__ AggShared sh;
	const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
	uint8_t* row = rows + threadIdx.x * kCipStride;
	uint32_t* q = sh.q[wave];
	if (threadIdx.x == 0) {
		sh.nreq = 0;
		sh.cn = 0;
	}
	__syncthreads();
	uint32_t cnt = 0;
	uint32_t qh = 0, qn = 0; // wave-uniform: ring head and queued requests
	const uint32_t steps = (d.n + kAggThreads - 1) / kAggThreads;
	const uint32_t per = agg_steps_per_block(d.n, gridDim.x);
	const uint32_t s0 = min(steps, blockIdx.x * per), s1 = min(steps, s0 + per);
	for (uint32_t st = s0; st < s1; st++) {
		const uint32_t i = st * kAggThreads + wave * 64 + lane;
		bool queue = false;
		if (i < d.n) {
			ebd_event_result r = d.res[i];
			if (r.status == EBD_STATUS_FINISHED && !(r.info & EBD_INFO_SESSION)) {
				cnt++;
				if (r.info & EBD_INFO_CIP) {
					queue = true;
				} else { // the client is the session's source address (Aggregator.cpp:57-63)
					const uint8_t* evb = (const uint8_t*)(d.ev + i);
					const v4u sv = *(const __attribute__((address_space(1))) v4u*)(evb + 16); // sourceIP (4-B aligned)
					uint8_t src[16];
					__builtin_memcpy(src, &sv, 16);
					unsigned long long net = 0;
					const uint32_t cls = classify_source(*d.ifs, evb[32], src, &net);
					r.info = (uint8_t)(r.info | (cls << EBD_INFO_CLASS_SHIFT));
					if (cls) // the class k_fresh leaves out, into the result's info byte (byte 3)
						((uint8_t*)(d.res + i))[3] = r.info;
					agg_request(d, i, r, cls, sh, net);
				}
			}
		}
		const unsigned long long b = __ballot(queue);
		if (queue)
			q[(qh + qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0))) & (kCipRing - 1)] = i;
		qn += (uint32_t)__popcll(b);
		if (qn >= 64) { // a full wave of client-IP requests
			wave_sync();
			agg_cip_one(d, q[(qh + lane) & (kCipRing - 1)], row, sh);
			qh += 64;
			qn -= 64;
			wave_sync(); // the ring words just read may be rewritten by the next step
		}
	}
	wave_sync();
	if (lane < qn) // what is left in the ring
		agg_cip_one(d, q[(qh + lane) & (kCipRing - 1)], row, sh);
	atomicAdd(&sh.nreq, (unsigned long long)cnt);
	__syncthreads();
	if (threadIdx.x == 0) {
		d.blk_cnt[blockIdx.x] = sh.cn;
		if (sh.nreq)
			atomicAdd(&d.ctr[CTR_REQUESTS], sh.nreq);
	}
}

// ---------------------------------------------------------------------------------
// Owned aggregation: Aggregator::newRequest (Aggregator.cpp:44-130, 155-168) for the fast-path
// requests with the service table taken one range of kOwnSlots slots per workgroup, in LDS.
//
// k_agg_fast is bound by memory-side atomics: a probe read, a counter add and a first-arrival
// max per request, plus a CAS and a store per new service, land on random 64-B lines at about
// 20 G atomics/s chip-wide whatever the table's size (tools/ubench_regions.hip: the same work
// one Infinity-Cache-sized region at a time is no faster).  Here the counted requests are
// bucketed by the range of their first slot instead, in two passes of coalesced tile writes
// with exact offsets (the requests of a service share its range, so the counts follow the
// services' popularity and cannot be bounded in advance):
//   k_own_count  per event its range (own_rid) and per-bucket counts;   k_own_scan_a  offsets;
//   k_own_emit   the entries (key, class, claim fields) into their buckets (ownA, own_sub);
//   k_own_bcount per-range counts from own_sub;                         k_own_scan_b  offsets;
//   k_own_part   the entries into their ranges (ownB);
//   k_own        one workgroup per range: its slots into LDS, its requests against them with
//                LDS atomics, the changed slots back to the table.
// Probing wraps inside the range (probe_next) for every other user of the table too.  Claims go
// to the range's stretch of the claim stage (kOwnSlots per range: a claim takes a slot), so the
// publication kernels run unchanged over one stretch per range.
// ---------------------------------------------------------------------------------
constexpr uint32_t kOwnLg = 11, kOwnSlots = 1u << kOwnLg;
constexpr uint32_t kOwnTile = 4096;                  // events or entries per block tile
constexpr unsigned long long kOwnLocked = 2;         // an LDS tag while its claimer writes hi (tags are odd)
constexpr uint16_t kOwnNone = 0xffff;

__device__ __forceinline__ uint32_t own_range(const Dev& d, unsigned long long lo) { return ((uint32_t)lo & d.slot_mask) >> kOwnLg; }

__device__ __forceinline__ bool own_counted(const ebd_event_result& r) {
	return r.status == EBD_STATUS_FINISHED && !(r.info & EBD_INFO_SESSION); // what k_agg_fast aggregates
}

// Per event: k_agg_fast's selection and client class (the class written into the result), its
// range, and per tile the bucket counts (one atomic per bucket and tile).  Requests with a client-IP
// header are queued per wave and their tokens parsed 64 at a time on full waves, as in k_agg_fast.
__device__ __forceinline__ void own_cip_one(const Dev& d, uint32_t i, uint8_t* row) {
	ebd_event_result r = d.res[i];
	unsigned long long net = 0;
	const uint32_t cls = cip_classify(d, i, r, row, &net);
	r.info = (uint8_t)((r.info & ~(3u << EBD_INFO_CLASS_SHIFT)) | (cls << EBD_INFO_CLASS_SHIFT));
	d.res[i] = r;
}

__global__ __launch_bounds__(256) void k_own_count(Dev d) {
	__shared__ __attribute__((aligned(8))) uint8_t rows[256 * kCipStride];
	__shared__ uint32_t cq[4][kCipRing];
	__shared__ uint32_t hist[256];
	__shared__ unsigned long long nreq;
	const uint32_t nb = 1u << d.own_abits, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
	uint8_t* row = rows + threadIdx.x * kCipStride;
	uint32_t* q = cq[wave];
	uint32_t qh = 0, qn = 0; // wave-uniform: ring head and queued requests
	if (threadIdx.x == 0)
		nreq = 0;
	uint32_t cnt = 0;
	for (unsigned long long t0 = (unsigned long long)blockIdx.x * kOwnTile; t0 < d.n; t0 += (unsigned long long)gridDim.x * kOwnTile) {
		for (uint32_t b = threadIdx.x; b < nb; b += 256)
			hist[b] = 0;
		__syncthreads();
#pragma unroll 1
		for (uint32_t j = 0; j < kOwnTile / 256; j++) {
			const unsigned long long ii = t0 + j * 256 + threadIdx.x;
			bool queue = false;
			if (ii < d.n) {
				const uint32_t i = (uint32_t)ii;
				const ebd_event_result r = d.res[i];
				uint16_t rid = kOwnNone;
				if (own_counted(r)) {
					cnt++;
					rid = (uint16_t)own_range(d, d.keys[i].lo);
					atomicAdd(&hist[rid >> d.own_bbits], 1u);
					if (r.info & EBD_INFO_CIP) { // the client is clientIp.front() (Aggregator.cpp:50-56)
						queue = true;
					} else { // the session's source address (Aggregator.cpp:57-63)
						const uint8_t* evb = (const uint8_t*)(d.ev + i);
						const v4u sv = *(const __attribute__((address_space(1))) v4u*)(evb + 16);
						uint8_t src[16];
						__builtin_memcpy(src, &sv, 16);
						const uint32_t cls = classify_source(*d.ifs, evb[32], src);
						if (cls)
							((uint8_t*)(d.res + i))[3] = (uint8_t)(r.info | (cls << EBD_INFO_CLASS_SHIFT));
					}
				}
				d.own_rid[i] = rid;
			}
			const unsigned long long bq = __ballot(queue);
			if (queue)
				q[(qh + qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(bq >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bq, 0))) & (kCipRing - 1)] =
						(uint32_t)ii;
			qn += (uint32_t)__popcll(bq);
			if (qn >= 64) { // a full wave of client-IP requests
				wave_sync();
				own_cip_one(d, q[(qh + lane) & (kCipRing - 1)], row);
				qh += 64;
				qn -= 64;
				wave_sync(); // the ring words just read may be rewritten
			}
		}
		__syncthreads();
		for (uint32_t b = threadIdx.x; b < nb; b += 256)
			if (hist[b])
				atomicAdd(&d.own_ctl->acnt[b], (unsigned long long)hist[b]);
		__syncthreads();
	}
	wave_sync();
	if (lane < qn) // what is left in the ring
		own_cip_one(d, q[(qh + lane) & (kCipRing - 1)], row);
	atomicAdd(&nreq, (unsigned long long)cnt);
	__syncthreads();
	if (threadIdx.x == 0 && nreq)
		atomicAdd(&d.ctr[CTR_REQUESTS], nreq);
}

// One thread: the buckets' starts, cursors and tile counts.
__global__ void k_own_scan_a(Dev d) {
	if (blockIdx.x != 0 || threadIdx.x != 0)
		return;
	OwnCtl& c = *d.own_ctl;
	const uint32_t nb = 1u << d.own_abits;
	unsigned long long s = 0;
	uint32_t t = 0;
	for (uint32_t b = 0; b < nb; b++) {
		c.aoff[b] = c.acur[b] = s;
		c.tcum[b] = t;
		s += c.acnt[b];
		t += (uint32_t)((c.acnt[b] + kOwnTile - 1) / kOwnTile);
	}
	c.aoff[nb] = s;
	c.tcum[nb] = t;
}

// The bucket tile a block takes: bucket b and entries [*e0, *e1) of ownA; false past the last tile.
__device__ __forceinline__ bool own_tile(const Dev& d, uint32_t k, uint32_t* b, unsigned long long* e0, unsigned long long* e1) {
	const OwnCtl& c = *d.own_ctl;
	const uint32_t nb = 1u << d.own_abits;
	if (k >= c.tcum[nb])
		return false;
	uint32_t lo = 0, hi = nb - 1; // the last bucket whose tiles start at or before k
	while (lo < hi) {
		const uint32_t mid = (lo + hi + 1) >> 1;
		if (c.tcum[mid] <= k)
			lo = mid;
		else
			hi = mid - 1;
	}
	*b = lo;
	*e0 = c.aoff[lo] + (unsigned long long)(k - c.tcum[lo]) * kOwnTile;
	*e1 = c.aoff[lo + 1] < *e0 + kOwnTile ? c.aoff[lo + 1] : *e0 + kOwnTile;
	return true;
}

// Pass A: each counted request as an OwnEnt at its bucket's next places (the result already holds
// its class); one reservation per bucket and tile.
__global__ __launch_bounds__(256) void k_own_emit(Dev d) {
	__shared__ uint32_t hist[256];
	__shared__ unsigned long long base[256];
	const uint32_t nb = 1u << d.own_abits, smask = (1u << d.own_bbits) - 1u;
	for (unsigned long long t0 = (unsigned long long)blockIdx.x * kOwnTile; t0 < d.n; t0 += (unsigned long long)gridDim.x * kOwnTile) {
		for (uint32_t b = threadIdx.x; b < nb; b += 256)
			hist[b] = 0;
		__syncthreads();
		uint32_t pk[kOwnTile / 256]; // rank in the bucket << 16 | range
#pragma unroll
		for (uint32_t j = 0; j < kOwnTile / 256; j++) {
			const unsigned long long i = t0 + j * 256 + threadIdx.x;
			pk[j] = ~0u;
			const uint32_t rid = i < d.n ? d.own_rid[i] : kOwnNone;
			if (rid != kOwnNone)
				pk[j] = (atomicAdd(&hist[rid >> d.own_bbits], 1u) << 16) | rid;
		}
		__syncthreads();
		for (uint32_t b = threadIdx.x; b < nb; b += 256)
			if (hist[b])
				base[b] = atomicAdd(&d.own_ctl->acur[b], (unsigned long long)hist[b]);
		__syncthreads();
#pragma unroll
		for (uint32_t j = 0; j < kOwnTile / 256; j++) {
			if (pk[j] == ~0u)
				continue;
			const uint32_t i = (uint32_t)(t0 + j * 256 + threadIdx.x), rid = pk[j] & 0xffffu;
			const ebd_event_result r = d.res[i];
			const Hash128 key = d.keys[i];
			OwnEnt e;
			e.lo = key.lo;
			e.hi = key.hi;
			e.i = i;
			e.w = ((r.info >> EBD_INFO_CLASS_SHIFT) & 3u) | ((r.info & EBD_INFO_HTTPS) ? 4u : 0u) | ((uint32_t)r.u.span.host_len << 3);
			e.pid = d.ev[i].pid;
			e.host_off = r.u.span.host_off;
			e.host_len = r.u.span.host_len;
			e.url_off = r.u.span.url_off;
			e.url_len = r.u.span.url_len;
			e.pad = 0;
			e.off = d.off[i];
			const unsigned long long pos = base[rid >> d.own_bbits] + (pk[j] >> 16);
			d.ownA[pos] = e;
			d.own_sub[pos] = (uint8_t)(rid & smask);
		}
		__syncthreads(); // hist and base are rewritten by the next tile
	}
}

// Per bucket tile: its entries' counts per range (one atomic per range and tile).
__global__ __launch_bounds__(256) void k_own_bcount(Dev d) {
	__shared__ uint32_t hist[256];
	uint32_t bk;
	unsigned long long e0, e1;
	if (!own_tile(d, blockIdx.x, &bk, &e0, &e1))
		return;
	const uint32_t nsub = 1u << d.own_bbits;
	for (uint32_t x = threadIdx.x; x < nsub; x += 256)
		hist[x] = 0;
	__syncthreads();
	for (unsigned long long k = e0 + threadIdx.x; k < e1; k += 256)
		atomicAdd(&hist[d.own_sub[k]], 1u);
	__syncthreads();
	for (uint32_t x = threadIdx.x; x < nsub; x += 256)
		if (hist[x])
			atomicAdd(&d.own_bcnt[(bk << d.own_bbits) | x], hist[x]);
}

// One block: the ranges' starts (exclusive scan of own_bcnt) and cursors; every thread scans a
// run of consecutive ranges, the runs' totals are scanned across the block.
__global__ __launch_bounds__(1024) void k_own_scan_b(Dev d) {
	__shared__ unsigned long long part[1024];
	const uint32_t nr = 1u << (d.own_abits + d.own_bbits), per = (nr + 1023) / 1024;
	const uint32_t r0 = threadIdx.x * per, r1 = min(nr, r0 + per);
	unsigned long long s = 0;
	for (uint32_t r = r0; r < r1; r++)
		s += d.own_bcnt[r];
	part[threadIdx.x] = s;
	__syncthreads();
	for (uint32_t o = 1; o < 1024; o <<= 1) {
		const unsigned long long a = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
		__syncthreads();
		part[threadIdx.x] += a;
		__syncthreads();
	}
	unsigned long long at = part[threadIdx.x] - s;
	for (uint32_t r = r0; r < r1; r++) {
		d.own_boff[r] = d.own_bcur[r] = at;
		at += d.own_bcnt[r];
	}
	if (threadIdx.x == 1023)
		d.own_boff[nr] = part[1023];
}

// Pass B: one bucket tile's entries to their ranges' next places in ownB.
__global__ __launch_bounds__(256) void k_own_part(Dev d) {
	__shared__ uint32_t hist[256];
	__shared__ unsigned long long base[256];
	uint32_t bk;
	unsigned long long e0, e1;
	if (!own_tile(d, blockIdx.x, &bk, &e0, &e1))
		return;
	const uint32_t nsub = 1u << d.own_bbits;
	for (uint32_t x = threadIdx.x; x < nsub; x += 256)
		hist[x] = 0;
	__syncthreads();
	uint32_t pk[kOwnTile / 256]; // rank in the range << 8 | range within the bucket
#pragma unroll
	for (uint32_t j = 0; j < kOwnTile / 256; j++) {
		const unsigned long long k = e0 + j * 256 + threadIdx.x;
		pk[j] = ~0u;
		if (k < e1) {
			const uint32_t sub = d.own_sub[k];
			pk[j] = (atomicAdd(&hist[sub], 1u) << 8) | sub;
		}
	}
	__syncthreads();
	for (uint32_t x = threadIdx.x; x < nsub; x += 256)
		if (hist[x])
			base[x] = atomicAdd(&d.own_bcur[(bk << d.own_bbits) | x], (unsigned long long)hist[x]);
	__syncthreads();
#pragma unroll
	for (uint32_t j = 0; j < kOwnTile / 256; j++)
		if (pk[j] != ~0u)
			d.ownB[base[pk[j] & 0xffu] + (pk[j] >> 8)] = d.ownA[e0 + j * 256 + threadIdx.x];
}

// A range's slot as k_own holds it in LDS: the fields newRequest changes (Slot's first 24 bytes
// and its two client counters).
struct OwnSlot {
	unsigned long long tag, hi, nfirst;
	uint32_t ic, ec;
};

// Pass C: one workgroup per range.  A claim takes an empty slot in two steps (CAS 0 -> kOwnLocked,
// hi, then the tag with release), all inside one loop iteration of the claiming lane, so a lane
// that reads kOwnLocked only re-reads the slot: its claimer is either a lane of the same wave in
// the same iteration or another wave, and neither waits for it.
__global__ __launch_bounds__(256) void k_own(Dev d) {
	__shared__ OwnSlot ls[kOwnSlots];
	__shared__ uint8_t dirty[kOwnSlots];
	__shared__ uint32_t nclaim;
	const uint32_t rg = blockIdx.x;
	Slot* g = d.slots + ((size_t)rg << kOwnLg);
	for (uint32_t k = threadIdx.x; k < kOwnSlots; k += 256) {
		const ulonglong2 th = *(const ulonglong2*)&g[k].tag;
		ls[k].tag = th.x;
		ls[k].hi = th.y;
		ls[k].nfirst = g[k].nfirst;
		ls[k].ic = g[k].internal_clients;
		ls[k].ec = g[k].external_clients;
		dirty[k] = 0;
	}
	if (threadIdx.x == 0)
		nclaim = 0;
	__syncthreads();
	const unsigned long long b = d.own_boff[rg], e = d.own_boff[rg + 1];
	OwnEnt nx;
	if (b + threadIdx.x < e)
		nx = d.ownB[b + threadIdx.x];
	for (unsigned long long j = b + threadIdx.x; j < e; j += 256) {
		const OwnEnt q = nx;
		if (j + 256 < e) // the next entry's load goes out before this one's probe
			nx = d.ownB[j + 256];
		uint32_t idx = (uint32_t)q.lo & (kOwnSlots - 1u);
		bool claimed = false, found = false;
		for (uint32_t p = 0; p < kOwnSlots;) {
			const unsigned long long t = __hip_atomic_load(&ls[idx].tag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
			if (t == 0) {
				unsigned long long want = 0;
				if (__hip_atomic_compare_exchange_strong(&ls[idx].tag, &want, kOwnLocked, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
							__HIP_MEMORY_SCOPE_WORKGROUP)) {
					ls[idx].hi = q.hi;
					__hip_atomic_store(&ls[idx].tag, q.lo, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
					claimed = found = true;
					break;
				}
				continue; // another lane took it: read it again
			}
			if (t == kOwnLocked)
				continue; // its claimer finishes within its own iteration
			if (t == q.lo) {
				if (ls[idx].hi == q.hi) {
					found = true;
					break;
				}
				atomicAdd(&d.ctr[CTR_COLLISIONS], 1ull); // same tag, other key: keep probing
			}
			idx = (idx + 1u) & (kOwnSlots - 1u);
			p++;
		}
		if (!found) {
			set_error(d, EBD_ERR_TABLE_FULL);
			continue;
		}
		const uint32_t cls = q.w & 3u;
		if (cls == CLS_INTERNAL)
			atomicAdd(&ls[idx].ic, 1u);
		else if (cls == CLS_EXTERNAL)
			atomicAdd(&ls[idx].ec, 1u);
		const unsigned long long nf = ~first_word(d.seq_base + q.i, (q.w & 4u) != 0, q.w >> 3); // the slot keeps ~first
		if (nf > ls[idx].nfirst)
			atomicMax(&ls[idx].nfirst, nf);
		dirty[idx] = 1;
		if (claimed) { // at most one claim per slot: the range's stretch holds them all
			ClaimRec cr;
			cr.slot = (rg << kOwnLg) | idx;
			cr.pid = q.pid;
			cr.host_off = q.host_off;
			cr.host_len = q.host_len;
			cr.url_off = q.url_off;
			cr.url_len = q.url_len;
			cr.off = q.off;
			d.cstage[(unsigned long long)rg * kOwnSlots + atomicAdd(&nclaim, 1u)] = cr;
		}
	}
	__syncthreads();
	for (uint32_t k = threadIdx.x; k < kOwnSlots; k += 256) {
		if (!dirty[k])
			continue;
		*(ulonglong2*)&g[k].tag = make_ulonglong2(ls[k].tag, ls[k].hi);
		g[k].nfirst = ls[k].nfirst;
		g[k].internal_clients = ls[k].ic;
		g[k].external_clients = ls[k].ec;
	}
	if (threadIdx.x == 0)
		d.blk_cnt[rg] = nclaim;
}

// ---------------------------------------------------------------------------------
// Device-wide primitives of the library's own (the scans, the compaction and the stable radix sort
// the session path, the exports and the generator use; no vendor library on these paths):
//   scan:    reduce-then-scan over chunks of kPrimChunk elements (k_scan_reduce, one block scans the
//            chunk totals, k_scan_down rescans each chunk from its prefix);
//   select:  stable compaction of the keys that are not ~0 (the session path's keys when few);
//   sort:    stable LSD radix sort of 64-bit keys on bits [lo, hi), 8 bits per pass: per tile
//            digit counts stored digit-major, one scan of them, then a scatter in which every wave
//            ranks its 64 keys by digit with 8 ballots (stable: waves in tile order, keys in lane
//            order), so keys with equal digits keep their input order.
// ---------------------------------------------------------------------------------
constexpr uint32_t kPrimThreads = 256, kPrimPer = 16, kPrimChunk = kPrimThreads * kPrimPer;

// Block-wide exclusive scan of one value per thread (256 threads, 4 waves); *total gets the sum.
template <typename T>
__device__ __forceinline__ T prim_block_excl(T x, T* part, T* total) {
	const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
	T incl = x;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const T y = (T)__shfl_up(incl, (unsigned)o, 64);
		incl += lane >= (uint32_t)o ? y : (T)0;
	}
	if (lane == 63)
		part[w] = incl;
	__syncthreads();
	T before = 0, all = 0;
	for (uint32_t k = 0; k < kPrimThreads / 64; k++) {
		before += k < w ? part[k] : (T)0;
		all += part[k];
	}
	__syncthreads(); // part may be rewritten by the caller's next round
	*total = all;
	return before + incl - x;
}

template <typename T>
__global__ __launch_bounds__(kPrimThreads) void k_scan_reduce(const T* in, unsigned long long n, T* bsum) {
	__shared__ T part[kPrimThreads / 64];
	const unsigned long long b = (unsigned long long)blockIdx.x * kPrimChunk;
	T s = 0;
	for (uint32_t k = threadIdx.x; k < kPrimChunk; k += kPrimThreads)
		if (b + k < n)
			s += in[b + k];
	T total;
	prim_block_excl<T>(s, part, &total);
	if (threadIdx.x == 0)
		bsum[blockIdx.x] = total;
}

// One block of 1024 threads: the chunk totals (nb of them) to their exclusive prefix, in place.
template <typename T>
__global__ __launch_bounds__(1024) void k_scan_top(T* bsum, uint32_t nb) {
	__shared__ T part[1024];
	const uint32_t per = (nb + 1023) / 1024, r0 = threadIdx.x * per, r1 = min(nb, r0 + per);
	T s = 0;
	for (uint32_t r = r0; r < r1; r++)
		s += bsum[r];
	part[threadIdx.x] = s;
	__syncthreads();
	for (uint32_t o = 1; o < 1024; o <<= 1) {
		const T a = threadIdx.x >= o ? part[threadIdx.x - o] : (T)0;
		__syncthreads();
		part[threadIdx.x] += a;
		__syncthreads();
	}
	T at = part[threadIdx.x] - s;
	for (uint32_t r = r0; r < r1; r++) {
		const T v = bsum[r];
		bsum[r] = at;
		at += v;
	}
}

// Each chunk again, thread t its kPrimPer consecutive elements, from the chunk's prefix.
template <typename T>
__global__ __launch_bounds__(kPrimThreads) void k_scan_down(const T* in, T* out, unsigned long long n, const T* bsum, int incl) {
	__shared__ T part[kPrimThreads / 64];
	const unsigned long long b = (unsigned long long)blockIdx.x * kPrimChunk + (unsigned long long)threadIdx.x * kPrimPer;
	T v[kPrimPer];
	T s = 0;
#pragma unroll
	for (uint32_t k = 0; k < kPrimPer; k++) {
		v[k] = b + k < n ? in[b + k] : (T)0;
		s += v[k];
	}
	T total;
	T at = bsum[blockIdx.x] + prim_block_excl<T>(s, part, &total);
#pragma unroll
	for (uint32_t k = 0; k < kPrimPer; k++) {
		if (b + k < n)
			out[b + k] = incl ? at + v[k] : at;
		at += v[k];
	}
}

template <typename T>
static hipError_t prim_scan(const T* in, T* out, unsigned long long n, int incl, void* tmp, hipStream_t st) {
	if (n == 0)
		return hipSuccess;
	const uint32_t nb = (uint32_t)((n + kPrimChunk - 1) / kPrimChunk);
	T* bsum = (T*)tmp;
	hipLaunchKernelGGL(k_scan_reduce<T>, dim3(nb), dim3(kPrimThreads), 0, st, in, n, bsum);
	hipLaunchKernelGGL(k_scan_top<T>, dim3(1), dim3(1024), 0, st, bsum, nb);
	hipLaunchKernelGGL(k_scan_down<T>, dim3(nb), dim3(kPrimThreads), 0, st, in, out, n, (const T*)bsum, incl);
	return hipGetLastError();
}

// Stable compaction of the keys that are not ~0 (in order), the count to *cnt.
__global__ __launch_bounds__(kPrimThreads) void k_sel_count(const unsigned long long* in, unsigned long long n, unsigned int* bsum) {
	__shared__ unsigned int part[kPrimThreads / 64];
	const unsigned long long b = (unsigned long long)blockIdx.x * kPrimChunk;
	unsigned int s = 0;
	for (uint32_t k = threadIdx.x; k < kPrimChunk; k += kPrimThreads)
		if (b + k < n && in[b + k] != ~0ull)
			s++;
	unsigned int total;
	prim_block_excl<unsigned int>(s, part, &total);
	if (threadIdx.x == 0)
		bsum[blockIdx.x] = total;
}
__global__ __launch_bounds__(kPrimThreads) void k_sel_scatter(const unsigned long long* in, unsigned long long* out, unsigned long long n,
		const unsigned int* bsum, uint32_t nb, int* cnt) {
	__shared__ unsigned int part[kPrimThreads / 64];
	const unsigned long long b = (unsigned long long)blockIdx.x * kPrimChunk + (unsigned long long)threadIdx.x * kPrimPer;
	unsigned long long v[kPrimPer];
	unsigned int s = 0;
#pragma unroll
	for (uint32_t k = 0; k < kPrimPer; k++) {
		v[k] = b + k < n ? in[b + k] : ~0ull;
		s += v[k] != ~0ull ? 1u : 0u;
	}
	unsigned int total;
	unsigned int at = bsum[blockIdx.x] + prim_block_excl<unsigned int>(s, part, &total);
#pragma unroll
	for (uint32_t k = 0; k < kPrimPer; k++)
		if (v[k] != ~0ull)
			out[at++] = v[k];
	if (blockIdx.x == nb - 1 && threadIdx.x == 0)
		*cnt = (int)(bsum[blockIdx.x] + total);
}

// Radix sort: per tile of kPrimChunk keys, the counts of each digit, digit-major
// (cnt[d * ntiles + t]).  Digits of up to kRsMaxBits bits: the passes split the sorted bits evenly
// (the session keys' 27 group bits: 3 passes of 9 bits took less than 4 of 8).
constexpr uint32_t kRsMaxBits = 10, kRsMaxBins = 1u << kRsMaxBits;
// 16,384-key tiles of 16 waves: a digit's run inside a tile is then about 32 keys for 9-bit digits,
// written by neighbouring waves (per 80 M-key sort: 2.42 ms, against 2.60 at 8,192 and 3.08 at 4,096)
#ifndef EBD_RS_THREADS
#define EBD_RS_THREADS 1024
#endif
constexpr uint32_t kRsThreads = EBD_RS_THREADS, kRsTile = kRsThreads * kPrimPer; // keys per tile
__global__ __launch_bounds__(kRsThreads) void k_rs_hist(const unsigned long long* in, unsigned long long n, uint32_t sh, uint32_t db,
		uint32_t ntiles, unsigned int* cnt) {
	__shared__ unsigned int h[kRsMaxBins];
	const uint32_t nbin = 1u << db, m = nbin - 1u;
	for (uint32_t x = threadIdx.x; x < nbin; x += kRsThreads)
		h[x] = 0;
	__syncthreads();
	const unsigned long long b = (unsigned long long)blockIdx.x * kRsTile;
	for (uint32_t k = threadIdx.x; k < kRsTile; k += kRsThreads)
		if (b + k < n)
			atomicAdd(&h[(uint32_t)(in[b + k] >> sh) & m], 1u);
	__syncthreads();
	for (uint32_t x = threadIdx.x; x < nbin; x += kRsThreads)
		cnt[(unsigned long long)x * ntiles + blockIdx.x] = h[x];
}

// The tile's keys to their places: wave w takes the tile's w-th quarter in order, 64 keys at a time,
// and ranks them among the wave's keys of the same digit with one ballot per digit bit.
__global__ __launch_bounds__(kRsThreads) void k_rs_scatter(const unsigned long long* in, unsigned long long* out, unsigned long long n,
		uint32_t sh, uint32_t db, uint32_t ntiles, const unsigned int* off) {
	__shared__ unsigned int wh[kRsThreads / 64][kRsMaxBins];
	const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63, nbin = 1u << db, m = nbin - 1u;
	const unsigned long long tb = (unsigned long long)blockIdx.x * kRsTile, q = kRsTile / (kRsThreads / 64);
	const unsigned long long b = tb + w * q, e = min(n, b + q);
	for (uint32_t x = lane; x < nbin; x += 64)
		wh[w][x] = 0;
	__syncthreads();
	for (unsigned long long j = b + lane; j < e; j += 64)
		atomicAdd(&wh[w][(uint32_t)(in[j] >> sh) & m], 1u);
	__syncthreads();
	for (uint32_t dg = threadIdx.x; dg < nbin; dg += kRsThreads) { // the tile's offset, then each wave's quarter after the earlier's
		unsigned int s = off[(unsigned long long)dg * ntiles + blockIdx.x];
		for (uint32_t k = 0; k < kRsThreads / 64; k++) {
			const unsigned int c = wh[k][dg];
			wh[k][dg] = s;
			s += c;
		}
	}
	__syncthreads();
	const unsigned long long lt = (1ull << lane) - 1ull;
	for (unsigned long long j0 = b; j0 < e; j0 += 64) { // wave-uniform
		const unsigned long long j = j0 + lane;
		const bool valid = j < e;
		const unsigned long long key = valid ? in[j] : 0ull;
		const uint32_t dg = (uint32_t)(key >> sh) & m;
		unsigned long long peers = __ballot(valid);
		for (uint32_t bit = 0; bit < db; bit++) {
			const unsigned long long bb = __ballot((dg >> bit) & 1u);
			peers &= ((dg >> bit) & 1u) ? bb : ~bb;
		}
		const uint32_t rank = (uint32_t)__popcll(peers & lt);
		const unsigned int base = wh[w][dg]; // read by every lane before the group's leader moves it
		if (valid)
			out[base + rank] = key;
		wave_sync();
		if (valid && rank == 0)
			wh[w][dg] = base + (unsigned int)__popcll(peers);
		wave_sync();
	}
}

// Stable sort of n keys on bits [lo, hi) between a and b; *sorted says where the result is.
static hipError_t prim_sort(unsigned long long* a, unsigned long long* b, unsigned long long n, uint32_t lo, uint32_t hi, void* tmp,
		unsigned long long** sorted, hipStream_t st) {
	*sorted = a;
	if (n == 0 || hi <= lo)
		return hipSuccess;
	const uint32_t ntiles = (uint32_t)((n + kRsTile - 1) / kRsTile);
	const uint32_t bits = hi - lo, passes = (bits + kRsMaxBits - 1) / kRsMaxBits, db = (bits + passes - 1) / passes;
	unsigned int* cnt = (unsigned int*)tmp;                              // 2^db * ntiles
	void* stmp = (void*)(cnt + ((unsigned long long)kRsMaxBins) * ntiles); // the scan's chunk totals
	unsigned long long* src = a;
	unsigned long long* dst = b;
	for (uint32_t sh = lo; sh < hi; sh += db) {
		const uint32_t d = min(db, hi - sh);
		hipLaunchKernelGGL(k_rs_hist, dim3(ntiles), dim3(kRsThreads), 0, st, src, n, sh, d, ntiles, cnt);
		hipError_t e = prim_scan<unsigned int>(cnt, cnt, (unsigned long long)(1u << d) * ntiles, 0, stmp, st);
		if (e != hipSuccess)
			return e;
		hipLaunchKernelGGL(k_rs_scatter, dim3(ntiles), dim3(kRsThreads), 0, st, src, dst, n, sh, d, ntiles, (const unsigned int*)cnt);
		unsigned long long* t = src;
		src = dst;
		dst = t;
	}
	*sorted = src;
	return hipGetLastError();
}

// The scratch bytes prim_sort needs for n keys (and prim_scan for 256 * tiles elements).
size_t prim_sort_tmp_bytes(unsigned long long n) {
	const unsigned long long ntiles = (n + kRsTile - 1) / kRsTile, m = (unsigned long long)kRsMaxBins * ntiles;
	return (size_t)(m * 4 + ((m + kPrimChunk - 1) / kPrimChunk) * 4 + 256);
}
size_t prim_scan_tmp_bytes(unsigned long long n, size_t elem) { return (size_t)(((n + kPrimChunk - 1) / kPrimChunk) * elem + 256); }
hipError_t prim_scan_u32(const unsigned int* in, unsigned int* out, unsigned long long n, int incl, void* tmp, hipStream_t st) {
	return prim_scan<unsigned int>(in, out, n, incl, tmp, st);
}
hipError_t prim_scan_u64(const unsigned long long* in, unsigned long long* out, unsigned long long n, int incl, void* tmp, hipStream_t st) {
	return prim_scan<unsigned long long>(in, out, n, incl, tmp, st);
}
hipError_t prim_scan_i32(const int* in, int* out, unsigned long long n, int incl, void* tmp, hipStream_t st) {
	return prim_scan<int>(in, out, n, incl, tmp, st);
}
hipError_t prim_sort_keys(unsigned long long* a, unsigned long long* b, unsigned long long n, uint32_t lo, uint32_t hi, void* tmp,
		unsigned long long** sorted, hipStream_t st) {
	return prim_sort(a, b, n, lo, hi, tmp, sorted, st);
}
// Stable compaction of the keys that are not ~0 from in to out; the count to *cnt (device).
hipError_t prim_select_keys(const unsigned long long* in, unsigned long long* out, unsigned long long n, int* cnt, void* tmp, hipStream_t st) {
	if (n == 0)
		return hipMemsetAsync(cnt, 0, sizeof(int), st);
	const uint32_t nb = (uint32_t)((n + kPrimChunk - 1) / kPrimChunk);
	unsigned int* bsum = (unsigned int*)tmp;
	hipLaunchKernelGGL(k_sel_count, dim3(nb), dim3(kPrimThreads), 0, st, in, n, bsum);
	hipLaunchKernelGGL(k_scan_top<unsigned int>, dim3(1), dim3(1024), 0, st, bsum, nb);
	hipLaunchKernelGGL(k_sel_scatter, dim3(nb), dim3(kPrimThreads), 0, st, in, out, n, (const unsigned int*)bsum, nb, cnt);
	return hipGetLastError();
}

// ---- publication of the services k_agg_fast created (one block per k_agg_fast block) ----
constexpr int kPubThreads = 256, kPubClaims = kPubThreads / 4;

__device__ __forceinline__ uint32_t claim_bytes(const ClaimRec& c) { return (c.host_len + c.url_len + 7u) & ~7u; }

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
				const uint32_t s = (uint32_t)(d.slow_keys[a + k] >> 32); // the session group
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
			if (d.hrec) { // what k_walk's next-session prefetch would otherwise load in two dependent steps
				const unsigned long long key = d.slow_keys[a + k];
				const uint32_t i0 = (uint32_t)key;
				d.hrec[at] = uint4{(uint32_t)(a + k), i0, d.ev_slot[i0], (uint32_t)(key >> 32)};
			}
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
		sum += claim_bytes(d.cstage[at0 + j]);
	uint32_t total;
	block_scan((uint32_t)sum, part, &total);
	if (threadIdx.x == 0)
		d.blk_bytes[b] = total;
}

// Pass 2 (one block): each block's first list entry and arena offset; the list and arena grow.
// 2048 blocks per round (two per thread, a Hillis-Steele scan over the pairs), a carry between.
__global__ __launch_bounds__(1024) void k_pub_scan(Dev d, uint32_t nblk) {
	__shared__ unsigned long long cs[1024], bs[1024];
	const uint32_t t = threadIdx.x;
	unsigned long long lbase = d.ctr[CTR_SERVICES], abase = d.ctr[CTR_SARENA]; // the same in every thread
	for (uint32_t r0 = 0; r0 < nblk; r0 += 2048) {
		const uint32_t b0 = r0 + 2 * t, b1 = b0 + 1;
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
		const unsigned long long ce = cs[t] - c0 - c1, be = bs[t] - y0 - y1; // exclusive prefix of the pair
		if (b0 < nblk) {
			d.blk_lbase[b0] = lbase + ce;
			d.blk_abase[b0] = abase + be;
		}
		if (b1 < nblk) {
			d.blk_lbase[b1] = lbase + ce + c0;
			d.blk_abase[b1] = abase + be + y0;
		}
		lbase += cs[1023];
		abase += bs[1023];
		__syncthreads(); // cs and bs are rewritten by the next round
	}
	if (t == 0) {
		d.ctr[CTR_SERVICES] = lbase;
		d.ctr[CTR_SARENA] = abase;
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
		uint32_t i = kNone, slot = 0, hl = 0, ul = 0, pid = 0;
		const uint8_t *host = d.payload, *url = d.payload;
		if (j < cn) {
			const ClaimRec cr = d.cstage[at0 + j];
			i = 0;
			slot = cr.slot;
			pid = cr.pid;
			const uint8_t* p = d.payload + cr.off;
			host = p + cr.host_off;
			hl = cr.host_len;
			url = p + cr.url_off;
			ul = cr.url_len;
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
					d.list_pl[li] = (unsigned long long)pid | ((unsigned long long)n << 32);
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
	if (blockIdx.x == 0 && threadIdx.x == 0) { // the last kernel of a batch: batch totals into run totals,
		// consumed, so a later k_verify (key merges, ebd_aggregate_requests) adds nothing twice
		d.ctr[CTR_EVICTIONS_TOTAL] += d.ctr[CTR_EVICTIONS];
		d.ctr[CTR_EVICTIONS] = 0;
	}
}

__device__ __forceinline__ Slot empty_slot() {
	Slot s;
	s.tag = 0;
	s.hi = 0;
	s.nfirst = 0; // first = ~0: no request yet
	s.pad0[0] = s.pad0[1] = 0;
	s.internal_clients = 0;
	s.external_clients = 0;
	s.nets[0] = s.nets[1] = s.nets[2] = 0;
	s.pad = 0;
	return s;
}

// Aggregator::clear (Aggregator.cpp:136-153): every claimed slot back to empty.
// Aggregator::clear's table reset.  Few services: their slots only, from the claimed-slot list
// (random 64-B writes).  At least a quarter of the slots used: the whole table as a stream of
// 16-B stores instead, which moves 4x the bytes at several times the rate of random writes
// (30 M services in 2^26 slots: 1.8 ms the sparse way).
__global__ void k_clear_used(const unsigned int* used, const unsigned long long* ctr, Slot* slots, uint32_t slot_cap) {
	const unsigned long long n = ctr[CTR_SERVICES];
	const unsigned long long t0 = blockIdx.x * blockDim.x + threadIdx.x, nt = (unsigned long long)gridDim.x * blockDim.x;
	if (4 * n < slot_cap) {
		for (unsigned long long k = t0; k < n; k += nt)
			slots[used[k]] = empty_slot();
	} else { // an empty slot is all zeros: a plain fill, 4 stores in flight per lane
		uint4* w = (uint4*)slots;
		const unsigned long long nw = 4ull * slot_cap;
		for (unsigned long long k = t0; k < nw; k += 4 * nt) {
#pragma unroll
			for (unsigned long long u = 0; u < 4; u++)
				if (k + u * nt < nw)
					w[k + u * nt] = make_uint4(0u, 0u, 0u, 0u);
		}
	}
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
		const unsigned long long first = ~s.nfirst;
		const uint32_t hl = (uint32_t)(first & 0x7fffu);
		uint32_t doff = 0, dlen = 0;
		if (ep != ~0ull)
			host_domain(d.sarena + ep, hl, &doff, &dlen);
		ebd_service v;
		v.pid = (uint32_t)pl;
		v.internal_clients = s.internal_clients;
		v.external_clients = s.external_clients;
		v.https = (uint8_t)((first >> 15) & 1u);
		v.pad_[0] = v.pad_[1] = v.pad_[2] = 0;
		v.endpoint_off = ep;
		v.endpoint_len = (uint32_t)(pl >> 32);
		v.domain_off = doff;
		v.domain_len = dlen;
		v.host_len = hl;
		v.first_seq = first >> 16;
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
		r.first = ~s.nfirst;
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

// The slot of the service with key (lo, hi), kNone if the table has none (find only).
__device__ uint32_t slot_find(const Dev& d, unsigned long long lo, unsigned long long hi) {
	uint32_t idx = (uint32_t)lo & d.slot_mask;
	for (uint32_t probe = 0; probe <= d.probe_mask; probe++) {
		Slot* s = d.slots + idx;
		unsigned long long t = s->tag;
		if (t == 0) // a plain load may see a stale line: the memory-side word decides
			t = rmw_read(&s->tag);
		if (t == 0)
			return kNone;
		if (t == lo) {
			unsigned long long h = s->hi;
			if (h != hi)
				h = rmw_read(&s->hi);
			if (h == hi)
				return idx;
		}
		idx = probe_next(d, idx);
	}
	return kNone;
}

// Network-map entries of other GPUs (ebd_service_net, k_net_dump's records) into the maps of
// this context's services: the entry's service is found by its key, the entry is claimed or
// found like a request's (net_touch), its last-seen time is the later one, and an entry new
// to the map (or erased there) adds one to the map's size (Aggregator.cpp:89-106 across GPUs).
__global__ void k_net_merge(Dev d, const ebd_service_net* rec, uint32_t n) {
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const ebd_service_net r = rec[k];
		const uint32_t slot = slot_find(d, r.key_lo, r.key_hi);
		if (slot == kNone || r.kind < NET_V4_16 || r.kind > NET_V6 || r.time_ns == 0) {
			set_error(d, EBD_ERR_INTERNAL); // not what an export of merged services sends
			continue;
		}
		unsigned long long pfx = 0;
		for (int b = 0; b < 6; b++)
			pfx |= (unsigned long long)r.prefix[b] << (8 * b);
		const uint32_t v = r.kind == NET_V6 ? v6d_index(d, pfx) : (uint32_t)pfx;
		if (v == kNone)
			continue;
		NetEnt* e = net_find_or_claim(d, d.nets, d.net_mask, net_key(r.kind, slot, v));
		if (e && atomicMax(&e->time, r.time_ns) == 0)
			atomicAdd(&d.slots[slot].nets[r.kind - 1], 1u);
	}
}

// ---------------------------------------------------------------------------------
// Cross-GPU merge.  Export: the collected services grouped by owner GPU
// (owner_of(key_lo)) with their endpoint bytes; merge: received records inserted into the
// owner's table with agg_insert (counters add, the smallest first word wins).
// ---------------------------------------------------------------------------------
constexpr int kOwnerMax = 64;

// The GPU that owns a service in the cross-GPU merge: the key's high word mod world.  (Its low
// bit is always set, the used-slot mark, so key_lo mod world would leave every even GPU
// without services.)
__device__ __forceinline__ uint32_t owner_of(unsigned long long key_lo, uint32_t world) {
	return (uint32_t)(key_lo >> 32) % world;
}

// Per owner: records and (8-aligned) string bytes, block histograms in LDS.
__global__ void k_owner_count(const ebd_service* rec, const unsigned long long* ctr, uint32_t world, unsigned long long* cnt,
		unsigned long long* bytes) {
	__shared__ unsigned long long hc[kOwnerMax], hb[kOwnerMax];
	for (uint32_t w = threadIdx.x; w < world; w += blockDim.x)
		hc[w] = hb[w] = 0;
	__syncthreads();
	const unsigned long long n = ctr[CTR_SERVICES];
	for (unsigned long long k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const uint32_t w = owner_of(rec[k].key_lo, world);
		atomicAdd(&hc[w], 1ull);
		atomicAdd(&hb[w], rec[k].endpoint_off == ~0ull ? 0ull : (unsigned long long)((rec[k].endpoint_len + 7u) & ~7u));
	}
	__syncthreads();
	for (uint32_t w = threadIdx.x; w < world; w += blockDim.x) {
		if (hc[w])
			atomicAdd(&cnt[w], hc[w]);
		if (hb[w])
			atomicAdd(&bytes[w], hb[w]);
	}
}

// Records to their owners' segments (cur[w]: the next record of owner w, initialised to the
// segment starts; arbitrary order inside a segment), as wire records; srcoff[at] keeps the
// endpoint's arena offset for k_wire_copy.
__global__ void k_owner_scatter(const ebd_service* rec, const unsigned long long* ctr, uint32_t world, unsigned long long* cur,
		ebd_wire_service* out, unsigned long long* srcoff) {
	const unsigned long long n = ctr[CTR_SERVICES];
	for (unsigned long long k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const ebd_service v = rec[k];
		const uint32_t w = owner_of(v.key_lo, world);
		const unsigned long long at = atomicAdd(&cur[w], 1ull);
		ebd_wire_service o;
		o.key_lo = v.key_lo;
		o.key_hi = v.key_hi;
		o.first = (v.first_seq << 16) | ((unsigned long long)(v.https & 1u) << 15) | (v.host_len & 0x7fffu);
		o.pid = v.pid;
		o.internal_clients = v.internal_clients;
		o.external_clients = v.external_clients;
		o.endpoint_len = v.endpoint_off == ~0ull ? (v.endpoint_len | EBD_WIRE_NO_BYTES) : v.endpoint_len;
		out[at] = o;
		srcoff[at] = v.endpoint_off;
	}
}

// The segment starts of the owner-grouped export (an exclusive scan of the per-owner record counts,
// world <= kOwnerMax): one thread, so that the export needs no host read of the counts.
__global__ void k_owner_prefix(const unsigned long long* cnt, uint32_t world, unsigned long long* cur) {
	if (blockIdx.x == 0 && threadIdx.x == 0) {
		unsigned long long s = 0;
		for (uint32_t w = 0; w < world; w++) {
			cur[w] = s;
			s += cnt[w];
		}
	}
}

// Bytes each wire record's endpoint takes in the strings (the exclusive scan of this is its offset).
// nptr (device, optional): the records that exist; entries from there to n get 0.
__global__ void k_wire_bytes(const ebd_wire_service* rec, uint32_t n, const unsigned long long* nptr, unsigned long long* nb) {
	const unsigned long long m = nptr ? *nptr : n;
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x)
		nb[k] = k < m ? EBD_WIRE_BYTES(rec[k].endpoint_len) : 0ull;
}

// Per segment of records (segment s: seg[s] consecutive records, in order), the bytes of the
// records that are on (need[k] != 0, or dst[k] != ~0 when need is null): the exchange's byte
// counts per owner (source side) or per source (owner side), with no host read.
__global__ void k_wire_seg_bytes(const ebd_wire_service* rec, uint32_t n, const uint8_t* need, const unsigned long long* dst,
		const unsigned long long* seg, uint32_t world, unsigned long long* out) {
	__shared__ unsigned long long pre[kOwnerMax + 1], acc[kOwnerMax];
	if (threadIdx.x == 0) {
		unsigned long long s = 0;
		for (uint32_t w = 0; w < world; w++) {
			pre[w] = s;
			s += seg[w];
		}
		pre[world] = s;
	}
	for (uint32_t w = threadIdx.x; w < world; w += blockDim.x)
		acc[w] = 0;
	__syncthreads();
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const bool on = need ? need[k] != 0 : dst[k] != ~0ull;
		if (!on || k >= pre[world])
			continue;
		uint32_t lo = 0, hi = world - 1; // the last segment that starts at or before k
		while (lo < hi) {
			const uint32_t mid = (lo + hi + 1) >> 1;
			if (pre[mid] <= k)
				lo = mid;
			else
				hi = mid - 1;
		}
		atomicAdd(&acc[lo], (unsigned long long)EBD_WIRE_BYTES(rec[k].endpoint_len));
	}
	__syncthreads();
	for (uint32_t w = threadIdx.x; w < world; w += blockDim.x)
		if (acc[w])
			atomicAdd(&out[w], acc[w]);
}

// Export: each record's endpoint bytes from the arena to its scanned place in the strings.
__global__ void k_wire_copy(const ebd_wire_service* rec, uint32_t n, const unsigned long long* nptr, const unsigned long long* offs,
		const unsigned long long* srcoff, const uint8_t* arena, uint8_t* strings) {
	if (nptr && *nptr < n)
		n = (uint32_t)*nptr;
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const uint32_t nb = EBD_WIRE_BYTES(rec[k].endpoint_len);
		const unsigned long long* src = (const unsigned long long*)(arena + srcoff[k]);
		unsigned long long* dst = (unsigned long long*)(strings + offs[k]);
		for (uint32_t b = 0; b < nb / 8; b++)
			dst[b] = src[b];
	}
}

// Merge: received records inserted with agg_insert (counters add, the smallest first word
// wins); the claimer publishes the endpoint from the strings (offs: the scan of k_wire_bytes).
__global__ void k_merge(Dev d, const ebd_wire_service* rec, uint32_t n, const uint8_t* strings, unsigned long long strlen,
		const unsigned long long* offs) {
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const ebd_wire_service v = rec[k];
		const uint32_t len = v.endpoint_len & ~EBD_WIRE_NO_BYTES;
		const unsigned long long at = offs[k];
		if (at + EBD_WIRE_BYTES(v.endpoint_len) > strlen || len > 0xffffu) { // not what an export writes
			set_error(d, EBD_ERR_INTERNAL);
			continue;
		}
		bool claimed;
		const uint32_t slot = agg_insert(d, Hash128{v.key_lo, v.key_hi}, v.first, v.internal_clients, v.external_clients, &claimed);
		if (claimed) {
			const uint32_t hl = min((uint32_t)(v.first & 0x7fffu), len);
			const unsigned long long list_at = atomicAdd(&d.ctr[CTR_SERVICES], 1ull);
			if (v.endpoint_len & EBD_WIRE_NO_BYTES) { // the source had no bytes: none here either
				set_error(d, EBD_ERR_ARENA_FULL);
				claim_publish(d, slot, list_at, ~0ull - len, v.pid, strings, hl, strings, len - hl);
			} else {
				const uint8_t* ep = strings + at;
				claim_publish(d, slot, list_at, atomicAdd(&d.ctr[CTR_SARENA], (unsigned long long)((len + 7u) & ~7u)), v.pid, ep, hl,
						ep + hl, len - hl);
			}
		}
	}
}

// Two-round merge (ebd_merge_service_keys_device / ebd_merge_service_bytes_device): the key
// round inserts the records as k_merge does, but the claimer of a new service only reserves
// its list entry and arena bytes: dst[k] = the reserved arena offset (~0: record k's bytes are
// not needed, the owner already has the key or the source had none).  The sources then send
// the bytes of exactly the records with dst != ~0 (k_wire_compact), in record order, and
// k_merge_bytes copies them to their reserved places.
__global__ void k_merge_keys(Dev d, const ebd_wire_service* rec, uint32_t n, unsigned long long* dst) {
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const ebd_wire_service v = rec[k];
		const uint32_t len = v.endpoint_len & ~EBD_WIRE_NO_BYTES;
		unsigned long long at = ~0ull;
		if (len > 0xffffu) { // not what an export writes
			set_error(d, EBD_ERR_INTERNAL);
			dst[k] = at;
			continue;
		}
		bool claimed;
		const uint32_t slot = agg_insert(d, Hash128{v.key_lo, v.key_hi}, v.first, v.internal_clients, v.external_clients, &claimed);
		if (claimed) {
			const unsigned long long list_at = atomicAdd(&d.ctr[CTR_SERVICES], 1ull);
			if (list_at >= d.new_cap) {
				set_error(d, EBD_ERR_TABLE_FULL);
			} else {
				if (v.endpoint_len & EBD_WIRE_NO_BYTES) {
					set_error(d, EBD_ERR_ARENA_FULL); // the source had no bytes: none here either
				} else {
					const unsigned long long ep = atomicAdd(&d.ctr[CTR_SARENA], (unsigned long long)((len + 7u) & ~7u));
					if (ep + len <= d.sarena_cap)
						at = ep;
					else
						set_error(d, EBD_ERR_ARENA_FULL);
				}
				d.new_slots[list_at] = slot;
				d.list_ep[list_at] = at;
				d.list_pl[list_at] = (unsigned long long)v.pid | ((unsigned long long)len << 32);
			}
		}
		dst[k] = at;
	}
}

// Bytes each record sends in the bytes round: its endpoint's (8-padded) when needed, else 0.
__global__ void k_wire_bytes_needed(const ebd_wire_service* rec, uint32_t n, const uint8_t* need, const unsigned long long* dst,
		unsigned long long* nb) {
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const bool on = need ? need[k] != 0 : dst[k] != ~0ull;
		nb[k] = on ? EBD_WIRE_BYTES(rec[k].endpoint_len) : 0ull;
	}
}

// Source side: the needed records' bytes (at soff[k] in the export's strings) packed in record
// order at doff[k] (the scan of k_wire_bytes_needed).
__global__ void k_wire_compact(const ebd_wire_service* rec, uint32_t n, const uint8_t* need, const unsigned long long* soff,
		const unsigned long long* doff, const uint8_t* strings, unsigned long long strlen, uint8_t* out, unsigned long long outcap,
		unsigned long long* ctr) {
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		if (!need[k])
			continue;
		const uint32_t nb = EBD_WIRE_BYTES(rec[k].endpoint_len);
		if (soff[k] + nb > strlen || doff[k] + nb > outcap) {
			atomicOr(&ctr[CTR_ERRORS], (unsigned long long)EBD_ERR_INTERNAL);
			continue;
		}
		const unsigned long long* src = (const unsigned long long*)(strings + soff[k]);
		unsigned long long* o = (unsigned long long*)(out + doff[k]);
		for (uint32_t b = 0; b < nb / 8; b++)
			o[b] = src[b];
	}
}

// Owner side: received bytes (at offs[k], the scan of k_wire_bytes_needed over dst) to the
// arena offsets the key round reserved.
__global__ void k_merge_bytes(Dev d, const ebd_wire_service* rec, uint32_t n, const unsigned long long* dst, const unsigned long long* offs,
		const uint8_t* strings, unsigned long long strlen) {
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const unsigned long long at = dst[k];
		if (at == ~0ull)
			continue;
		const uint32_t nb = EBD_WIRE_BYTES(rec[k].endpoint_len);
		if (offs[k] + nb > strlen || at + nb > d.sarena_cap + 64) {
			set_error(d, EBD_ERR_INTERNAL);
			continue;
		}
		const unsigned long long* src = (const unsigned long long*)(strings + offs[k]);
		unsigned long long* o = (unsigned long long*)(d.sarena + at);
		for (uint32_t b = 0; b < nb / 8; b++)
			o[b] = src[b];
	}
}

// service::Aggregator::newRequest (Aggregator.cpp:155-168) for requests parsed elsewhere
// (ebd_aggregate_requests): the service key over (pid, host + url), the client class of
// clientIp.front() or of the session's source address (Aggregator.cpp:50-88), the
// first-arrival word and the network maps, as k_emit does for a session request.
static_assert(sizeof(ebd_request) == 40, "ebd_request is 40 bytes");
__global__ void k_agg_requests(Dev d, const ebd_request* rq, uint32_t n, const uint8_t* strings) {
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const ebd_request q = rq[k];
		const uint8_t* h = strings + q.str_off;
		const uint32_t hl = q.host_len, ul = q.url_len;
		unsigned long long net = 0;
		const uint8_t cls = q.cip_len != EBD_NO_CLIENT_IP ? classify_token(*d.ifs, h + hl + ul, q.cip_len, &net)
		                                                  : classify_source(*d.ifs, q.flags, q.source_ip, &net);
		const Hash128 key = endpoint_key(d.hkey, q.pid, 0, hl, hl, ul, [h](uint32_t o) { return gload8u(h + o); });
		bool claimed;
		const uint32_t slot = agg_insert(d, key, first_word(d.seq_base + k, q.is_https != 0, hl), cls == CLS_INTERNAL,
				cls == CLS_EXTERNAL, &claimed);
		if (claimed)
			claim_publish(d, slot, wave_add(&d.ctr[CTR_SERVICES], 1ull), wave_add(&d.ctr[CTR_SARENA], (unsigned long long)((hl + ul + 7u) & ~7u)),
					q.pid, h, hl, h + hl, ul);
		if (d.net_on && cls == CLS_EXTERNAL)
			agg_nets(d, slot, net, d.now);
		wave_add(&d.ctr[CTR_REQUESTS], 1ull);
	}
}

// ---------------------------------------------------------------------------------
// httpparser::HttpRequestParser one stream at a time (ebd_parse_streams): the generic state
// machine gp_step (HttpRequestParser.cpp:124-364) over the bytes of one chunk per call, plus
// what HttpRequest holds beyond the aggregator's needs: every value of a header whose key is
// result.clientIPKey, split into result.clientIp's tokens at its newline (P:248-262, 381-409).
// ---------------------------------------------------------------------------------

// parseClientIPValue (P:392-409): boost::split(token_compress_on) on ',' then each token's trim
// and IPv4 port / IPv6 bracket handling (front_token); tokens appended in order.
__device__ void stream_split_value(StreamParser& sp, const uint8_t* s, uint32_t a, uint32_t e) {
	uint32_t b = a;
	for (;;) {
		uint32_t t = b;
		while (t < e && s[t] != ',')
			t++;
		uint32_t tb, te;
		front_token(s + b, t - b, &tb, &te);
		if (sp.ntok < EBD_PARSE_MAX_TOKENS) {
			sp.tok[sp.ntok][0] = b + tb;
			sp.tok[sp.ntok][1] = b + te;
			sp.ntok++;
		} else {
			sp.dropped = 1;
		}
		if (t >= e)
			break;
		b = t;
		while (b < e && s[b] == ',') // adjacent separators are one (token_compress_on)
			b++;
		if (b >= e) { // a trailing separator leaves an empty last token
			if (sp.ntok < EBD_PARSE_MAX_TOKENS) {
				sp.tok[sp.ntok][0] = sp.tok[sp.ntok][1] = e;
				sp.ntok++;
			} else {
				sp.dropped = 1;
			}
			break;
		}
	}
}

__global__ void k_parse_streams(const KeyTrie* trie, ebd_parse_call* calls, uint32_t n, const uint8_t* data) {
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		ebd_parse_call& c = calls[k];
		StreamParser sp;
		__builtin_memcpy(&sp, &c.state, sizeof(sp));
		// the host checked the state (ebd_parse_streams -> stream_state_ok); kept in bounds here too,
		// so that no state indexes past the token list or the key trie
		sp.ntok = min(sp.ntok, (uint32_t)EBD_PARSE_MAX_TOKENS);
		sp.g.key = sp.g.key < kTrieNodes ? sp.g.key : kTrieDead;
		GenParser& g = sp.g;
		const uint8_t* s = data + c.data_off; // stream position p is s[p]
		const uint32_t end = c.data_len;
		uint32_t i = g.length; // the chunk: the stream from the parser's position
		const uint32_t i0 = i;
		while (i < end) { // P:85-106
			if (g.length > kMaxRequestLength) {
				g.state = ST_INVALID;
				break;
			}
			const uint32_t ch = s[i], st0 = g.state, kt = gp_key_type(trie, g.key);
			gp_step(g, trie, ch, g.length);
			if (st0 == ST_SP_VAL && g.state == ST_HDR_VAL && kt >= KT_CLIENT0) // the value's first byte (P:311-316)
				sp.vstart = sp.vend = g.length;
			if (st0 == ST_HDR_VAL && g.state == ST_HDR_NL && kt >= KT_CLIENT0) // its CR ends it
				sp.vend = g.length;
			if (st0 == ST_HDR_NL && g.state == ST_HDR_KEY && kt >= KT_CLIENT0 && key_client_id((uint8_t)kt) == g.cipkey)
				stream_split_value(sp, s, sp.vstart, sp.vend); // P:254-257
			i++;
			g.length++;
			if (gp_done(g)) {
				if (c.flags & 16) // DISCOVERY_FLAG_SESSION_SSL_HTTP (P:97-99)
					g.f |= GPF_HTTPS;
				else
					g.f &= (uint8_t)~GPF_HTTPS;
				break;
			}
		}
		c.consumed = i - i0;
		c.status = g.state == ST_FINISHED ? EBD_PARSER_FINISHED : g.state == ST_INVALID ? EBD_PARSER_INVALID : EBD_PARSER_UNFINISHED;
		c.is_https = (g.f & GPF_HTTPS) ? 1 : 0;
		c.client_ip_key = g.cipkey;
		c.tokens_dropped = (uint8_t)sp.dropped;
		c.method_len = g.mlen;
		c.url_off = g.url_start;
		c.url_len = g.url_len;
		c.protocol_off = g.url_start + g.url_len + 1; // 'H' follows the URL's space (P:215-224)
		c.protocol_len = g.plen;
		c.host_off = g.host_start;
		c.host_len = g.host_len;
		c.ntokens = sp.ntok;
		for (uint32_t t = 0; t < sp.ntok; t++) {
			c.tokens[t][0] = sp.tok[t][0];
			c.tokens[t][1] = sp.tok[t][1];
		}
		__builtin_memcpy(&c.state, &sp, sizeof(sp));
	}
}

hipError_t launch_parse_streams(const KeyTrie* trie, ebd_parse_call* calls, uint32_t n, const uint8_t* data, hipStream_t st) {
	hipLaunchKernelGGL(k_parse_streams, dim3((n + 63) / 64), dim3(64), 0, st, trie, calls, n, data);
	return hipGetLastError();
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
	const int grid = (int)(groups < (uint64_t)cus * EBD_FRESH_WGS ? groups : (uint64_t)cus * EBD_FRESH_WGS);
	hipLaunchKernelGGL(k_fresh, dim3(grid > 0 ? grid : 1), dim3(kFreshThreads), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_fresh_scan(const Dev& d, hipStream_t st, int cus) {
	// one-wave workgroups, EBD_SCAN_WGS per CU (LDS-bound), each a contiguous range of at
	// least 256 events
	const uint64_t groups = ((uint64_t)d.n + 255) / 256;
	const int grid = (int)(groups < (uint64_t)cus * EBD_SCAN_WGS ? groups : (uint64_t)cus * EBD_SCAN_WGS);
	hipLaunchKernelGGL(k_fresh_scan, dim3(grid > 0 ? grid : 1), dim3(64), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_sset_build(const Dev& d, uint32_t cap, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_sset_size, dim3(1), dim3(1), 0, st, d, cap);
	hipLaunchKernelGGL(k_sset_build, dim3(cus * 4), dim3(256), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_slow_collect(const Dev& d, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_slow_collect, dim3(grid_for(d.n, 256, cus * 8)), dim3(256), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_lru_bound(const Dev& d, uint32_t nslow, int* delta, uint8_t* minus, int* scan, void* tmp, size_t tmp_bytes,
		hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_lru_delta, dim3(grid_for(nslow, 256, cus * 8)), dim3(256), 0, st, d, nslow, delta, minus);
	(void)tmp_bytes; // prim_scan_tmp_bytes(max_events, 4), ebd_api.hip
	hipError_t e = prim_scan_i32(delta, scan, d.n, 1, tmp, st);
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
// After either walker: the session requests' emission, then the tallies.
hipError_t launch_emit(const Dev& d, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_emit, dim3(cus * EBD_EMIT_BLOCKS), dim3(256), 0, st, d);
	hipLaunchKernelGGL(k_sess_tally, dim3(1), dim3(1), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_walk(const Dev& d, uint32_t nslow, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_walk_heads, dim3(grid_for(nslow, kPubThreads * kHeadsPer, cus * 4)), dim3(kPubThreads), 0, st, d, nslow);
	hipError_t e = hipMemsetAsync(d.ctr + CTR_COUNT, 0, sizeof(unsigned long long), st); // k_walk's chunk counter
	if (e != hipSuccess)
		return e;
	hipLaunchKernelGGL(k_walk, dim3(grid_for(nslow, kWalkThreads, cus * EBD_WALK_BLOCKS)), dim3(kWalkThreads), 0, st, d,
			(const uint8_t*)nullptr, DryWalk{}, (const uint32_t*)nullptr, (const uint32_t*)nullptr);

	return hipGetLastError();
}
// Every session's walk starts at its first event.
__global__ void k_lru_wto_init(Dev d, uint32_t* wto) {
	const uint32_t nh = (uint32_t)d.ctr[CTR_HEADS];
	for (uint32_t h = blockIdx.x * blockDim.x + threadIdx.x; h < nh; h += gridDim.x * blockDim.x)
		wto[d.heads[h]] = d.heads[h];
}

// The exact-LRU rounds' once-per-batch part: heads, event -> sorted position, next finds,
// carried markers, empty operations, every walk at its session's start.
hipError_t launch_lru_init(const Dev& d, uint32_t nslow, const LruRound& w, hipStream_t st, int cus) {
	hipError_t e;
	if ((e = hipMemsetAsync(w.jpos, 0xff, (size_t)d.n * sizeof(uint32_t), st)) != hipSuccess ||
			(e = hipMemsetAsync(w.cm_end, 0xff, (size_t)d.carry_cap * 4, st)) != hipSuccess ||
			(e = hipMemsetAsync(w.cm_head, 0xff, (size_t)d.carry_cap * 4, st)) != hipSuccess ||
			(e = hipMemsetAsync(w.cpos, 0xff, (size_t)nslow * 4, st)) != hipSuccess ||
			(e = hipMemsetAsync(w.opt, 0, d.n, st)) != hipSuccess || (e = hipMemsetAsync(w.f[0], 0, d.n, st)) != hipSuccess ||
			(e = hipMemsetAsync(w.f[1], 0, d.n, st)) != hipSuccess ||
			(e = hipMemsetAsync(w.cf[0], 0, d.carry_cap, st)) != hipSuccess)
		return e;
	hipLaunchKernelGGL(k_walk_heads, dim3(grid_for(nslow, kPubThreads * kHeadsPer, cus * 4)), dim3(kPubThreads), 0, st, d, nslow);
	hipLaunchKernelGGL(k_lru_index, dim3(grid_for(nslow, 256, cus * 8)), dim3(256), 0, st, d, nslow, w.jpos, w.head);
	hipLaunchKernelGGL(k_lru_static, dim3(grid_for(nslow, 256, cus * 8)), dim3(256), 0, st, d, nslow, w.mend, w.cm_end, w.cm_head);
	hipLaunchKernelGGL(k_lru_wto_init, dim3(cus * 4), dim3(256), 0, st, d, w.wto);
	if (d.n_carry_in)
		hipLaunchKernelGGL(k_lru_carry_rank, dim3(grid_for(d.n_carry_in, 256, cus * 4)), dim3(256), 0, st, d, (const uint32_t*)w.cm_end,
				w.mk_ref, w.mk_e);
	return hipGetLastError();
}

// One exact-LRU round in the world f / cf: the walks up to the horizon front + window (from
// where flags changed or the last walk stopped), then the world the evictions before the
// horizon imply in nf / ncf; cnt[1] inconsistency, cnt[2] flags changed, cnt[3] the new
// frontier.
// A round's counters (the walk list tot[3]; cnt: evictions, inconsistency, flags changed,
// first changed event), cleared for the next round by k_lru_advance / k_lru_ctl_init.
__device__ __forceinline__ void lru_round_reset(uint32_t* tot, unsigned long long* cnt) {
	tot[3] = 0;
	cnt[0] = cnt[1] = cnt[2] = 0;
	cnt[3] = ~0ull;
}

// The end of a round (one thread): the world derived is the world walked up to the batch's
// end -> settled in world cur; an inconsistent world -> done, not settled (the one-lane replay
// takes the batch); else the frontier moves past every event the round settled.
__global__ void k_lru_advance(LruCtrl* ctl, unsigned long long* cnt, uint32_t* tot, uint32_t window, uint32_t n, uint32_t cur,
		unsigned long long* stat) {
	if (threadIdx.x != 0 || ctl->done)
		return;
	ctl->rounds++;
	if (stat) { // EBD_LRU_TRACE: the longest lane summed over rounds, the sessions walked
		stat[2] += stat[3];
		stat[3] = 0;
		stat[4] += tot[3];
	}
	const unsigned long long changed = cnt[2], first = cnt[3];
	const unsigned long long wend = (unsigned long long)ctl->front + window;
	if (cnt[1]) { // operations with a full cache and no victim: not a world to walk on
		ctl->done = 1;
		ctl->settled = 0;
		return;
	}
	if (changed == 0 && wend >= n) {
		ctl->done = 1;
		ctl->settled = 1;
		ctl->cur_final = cur ^ 1; // the derived world (equal to the walked one, which k_lru_diff cleared)
		return; // cnt[0] (the evictions) stays for the host
	}
	unsigned long long front = ctl->front;
	if (changed == 0)
		front = wend;
	else if (first != ~0ull) // events before the first changed flag (and the window's end) are settled
		front = first < wend ? first : wend;
	const unsigned long long tend = front + window;
	ctl->front = (uint32_t)front;
	ctl->tend = (uint32_t)(tend < 0xffffffffull ? tend : 0xffffffffull);
	lru_round_reset(tot, cnt);
}

// bs[0]: the batch starts with the carried sessions in the LRU (and their markers first).
__global__ void k_lru_ctl_init(LruCtrl* ctl, uint32_t window, uint32_t* tot, unsigned long long* cnt, LsState* bs, uint32_t nc) {
	if (threadIdx.x == 0) {
		ctl->front = 0;
		ctl->tend = window;
		ctl->done = ctl->settled = ctl->cur_final = ctl->rounds = 0;
		lru_round_reset(tot, cnt);
		bs[0] = LsState{(int)nc, nc, 0u, 0u};
	}
}

hipError_t launch_lru_ctl_init(const Dev& d, const LruRound& w, uint32_t window, hipStream_t st) {
	hipLaunchKernelGGL(k_lru_ctl_init, dim3(1), dim3(64), 0, st, w.ctl, window, w.tot, w.cnt, w.bs, d.n_carry_in);
	return hipGetLastError();
}

hipError_t launch_lru_round(const Dev& d, uint32_t nslow, const LruRound& w, int cur, uint32_t window, hipStream_t st, int cus) {
	const uint32_t n = d.n;
	const uint8_t* f = w.f[cur];
	uint8_t* nf = w.f[cur ^ 1]; // zero: cleared by the last round's k_lru_diff (or launch_lru_init)
	const uint8_t* cf = w.cf[cur];
	uint8_t* ncf = w.cf[cur ^ 1];
	const LruCtrl* ctl = w.ctl;
	hipLaunchKernelGGL(k_lru_walklist, dim3(cus * 4), dim3(256), 0, st, d, w.cpos, (const uint32_t*)w.wto, ctl, w.rlist, w.tot, ncf,
			d.carry_cap);
	hipLaunchKernelGGL(k_walk_dry, dim3(cus * kWalkDryBlocks), dim3(kWalkThreads), 0, st, d, f,
			DryWalk{w.head, (SessState*)w.snap, w.wto, w.opt, ctl, w.stat}, (const uint32_t*)w.rlist, (const uint32_t*)(w.tot + 3));
	hipLaunchKernelGGL(k_lru_scan, dim3(1), dim3(kScT), 0, st, (const uint8_t*)w.opt, (const uint32_t*)w.mend, n, d.carry_cap, w.bs,
			w.mk_ref, w.mk_e, w.ev_t, w.evc, w.tot, ctl);
	hipLaunchKernelGGL(k_lru_thresh, dim3(cus), dim3(kThT), 0, st, (const uint32_t*)w.mk_e, (const uint32_t*)w.evc, (const uint32_t*)w.tot,
			ctl, (const uint32_t*)w.vict, w.mx);
	hipLaunchKernelGGL(k_lru_take, dim3(1), dim3(kThT), 0, st, (const uint32_t*)w.mx, w.tot, ctl, w.vict, w.cnt);
	hipLaunchKernelGGL(k_lru_victims, dim3(cus * 2), dim3(256), 0, st, d, (const uint32_t*)w.tot, (const uint32_t*)w.vict,
			(const uint32_t*)w.mk_ref, (const uint32_t*)w.mk_e, (const uint32_t*)w.ev_t, (const uint32_t*)w.jpos, (const uint32_t*)w.head,
			(const uint32_t*)w.cm_head, nf, ncf, w.cnt, ctl);
	hipLaunchKernelGGL(k_lru_diff, dim3(grid_for(n / 4 + d.carry_cap, 256, cus * 4)), dim3(256), 0, st, n, w.f[cur], (const uint8_t*)nf, cf,
			(const uint8_t*)ncf, d.carry_cap, (const uint32_t*)w.jpos, (const uint32_t*)w.head, w.cpos, w.cnt, ctl);
	hipLaunchKernelGGL(k_lru_advance, dim3(1), dim3(64), 0, st, w.ctl, w.cnt, w.tot, window, n, (uint32_t)cur, w.stat);
	return hipGetLastError();
}
// The final walk of the exact path in the converged world (with output), then the carried
// sessions it did not meet.
hipError_t launch_walk_flags(const Dev& d, uint32_t nslow, const uint8_t* f, const uint8_t* cf, hipStream_t st, int cus) {
	const hipError_t e = hipMemsetAsync(d.ctr + CTR_COUNT, 0, sizeof(unsigned long long), st); // k_walk's chunk counter
	if (e != hipSuccess)
		return e;
	hipLaunchKernelGGL(k_walk, dim3(grid_for(nslow, kWalkThreads, cus * EBD_WALK_BLOCKS)), dim3(kWalkThreads), 0, st, d, f,
			DryWalk{}, (const uint32_t*)nullptr, (const uint32_t*)nullptr);
	if (d.n_carry_in)
		hipLaunchKernelGGL(k_carry_pass, dim3(grid_for(d.n_carry_in, 64, 256)), dim3(64), 0, st, d, cf);
	return hipGetLastError();
}
size_t lru_scan_blocks(uint32_t n) { return (n + kLsBlk - 1) / kLsBlk; }
int lru_size_limit() { return kLInf / 2; }
hipError_t launch_carry_pass(const Dev& d, hipStream_t st) {
	hipLaunchKernelGGL(k_carry_pass, dim3(grid_for(d.n_carry_in, 64, 256)), dim3(64), 0, st, d, (const uint8_t*)nullptr);
	return hipGetLastError();
}
uint32_t own_range_lg() { return kOwnLg; }
// The owned aggregation for a batch (own_ctl and own_bcnt zeroed by the caller).
hipError_t launch_own(const Dev& d, hipStream_t st, int cus) {
	const uint32_t nranges = 1u << (d.own_abits + d.own_bbits);
	const uint64_t tiles = ((uint64_t)d.n + kOwnTile - 1) / kOwnTile;
	const int g = grid_for(tiles, 1, cus * 8);
	const uint32_t btiles = (uint32_t)tiles + (1u << d.own_abits); // bucket tiles: at most one partial per bucket
	hipLaunchKernelGGL(k_own_count, dim3(g), dim3(256), 0, st, d);
	hipLaunchKernelGGL(k_own_scan_a, dim3(1), dim3(64), 0, st, d);
	hipLaunchKernelGGL(k_own_emit, dim3(g), dim3(256), 0, st, d);
	hipLaunchKernelGGL(k_own_bcount, dim3(btiles), dim3(256), 0, st, d);
	hipLaunchKernelGGL(k_own_scan_b, dim3(1), dim3(1024), 0, st, d);
	hipLaunchKernelGGL(k_own_part, dim3(btiles), dim3(256), 0, st, d);
	hipLaunchKernelGGL(k_own, dim3(nranges), dim3(256), 0, st, d);
	return hipGetLastError();
}
hipError_t launch_agg_fast(const Dev& d, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_agg_fast, dim3(agg_grid(d.n, cus)), dim3(kAggThreads), 0, st, d);
	return hipGetLastError();
}
// nblk: the claim stretches (0: k_agg_fast's grid)
hipError_t launch_publish(const Dev& d, uint32_t nblk, hipStream_t st, int cus) {
	const uint32_t g = nblk ? nblk : agg_grid(d.n, cus);
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
hipError_t launch_clear_used(const unsigned int* used, const unsigned long long* ctr, Slot* slots, uint32_t slot_cap,
		hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_clear_used, dim3(cus * 16), dim3(256), 0, st, used, ctr, slots, slot_cap);
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
hipError_t launch_net_merge(const Dev& d, const ebd_service_net* rec, uint32_t n, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_net_merge, dim3(grid_for(n, 256, cus * 8)), dim3(256), 0, st, d, rec, n);
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
hipError_t launch_owner_scatter(const ebd_service* rec, const unsigned long long* ctr, uint32_t world, unsigned long long* cur,
		ebd_wire_service* out, unsigned long long* srcoff, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_owner_scatter, dim3(cus * 8), dim3(256), 0, st, rec, ctr, world, cur, out, srcoff);
	return hipGetLastError();
}
hipError_t launch_owner_prefix(const unsigned long long* cnt, uint32_t world, unsigned long long* cur, hipStream_t st) {
	hipLaunchKernelGGL(k_owner_prefix, dim3(1), dim3(64), 0, st, cnt, world, cur);
	return hipGetLastError();
}
hipError_t launch_wire_bytes(const ebd_wire_service* rec, uint32_t n, const unsigned long long* nptr, unsigned long long* nb, hipStream_t st,
		int cus) {
	hipLaunchKernelGGL(k_wire_bytes, dim3(grid_for(n, 256, cus * 8)), dim3(256), 0, st, rec, n, nptr, nb);
	return hipGetLastError();
}
hipError_t launch_wire_seg_bytes(const ebd_wire_service* rec, uint32_t n, const uint8_t* need, const unsigned long long* dst,
		const unsigned long long* seg, uint32_t world, unsigned long long* out, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_wire_seg_bytes, dim3(grid_for(n, 256, cus * 4)), dim3(256), 0, st, rec, n, need, dst, seg, world, out);
	return hipGetLastError();
}
hipError_t launch_wire_copy(const ebd_wire_service* rec, uint32_t n, const unsigned long long* nptr, const unsigned long long* offs,
		const unsigned long long* srcoff, const uint8_t* arena, uint8_t* strings, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_wire_copy, dim3(grid_for(n, 256, cus * 8)), dim3(256), 0, st, rec, n, nptr, offs, srcoff, arena, strings);
	return hipGetLastError();
}
hipError_t launch_agg_requests(const Dev& d, const ebd_request* rq, uint32_t n, const uint8_t* strings, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_agg_requests, dim3(grid_for(n, 256, cus * 8)), dim3(256), 0, st, d, rq, n, strings);
	return hipGetLastError();
}
hipError_t launch_merge_keys(const Dev& d, const ebd_wire_service* rec, uint32_t n, unsigned long long* dst, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_merge_keys, dim3(grid_for(n, 256, cus * 8)), dim3(256), 0, st, d, rec, n, dst);
	return hipGetLastError();
}
hipError_t launch_wire_bytes_needed(const ebd_wire_service* rec, uint32_t n, const uint8_t* need, const unsigned long long* dst,
		unsigned long long* nb, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_wire_bytes_needed, dim3(grid_for(n, 256, cus * 8)), dim3(256), 0, st, rec, n, need, dst, nb);
	return hipGetLastError();
}
hipError_t launch_wire_compact(const ebd_wire_service* rec, uint32_t n, const uint8_t* need, const unsigned long long* soff,
		const unsigned long long* doff, const uint8_t* strings, unsigned long long strlen, uint8_t* out, unsigned long long outcap,
		unsigned long long* ctr, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_wire_compact, dim3(grid_for(n, 256, cus * 8)), dim3(256), 0, st, rec, n, need, soff, doff, strings, strlen, out,
			outcap, ctr);
	return hipGetLastError();
}
hipError_t launch_merge_bytes(const Dev& d, const ebd_wire_service* rec, uint32_t n, const unsigned long long* dst,
		const unsigned long long* offs, const uint8_t* strings, unsigned long long strlen, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_merge_bytes, dim3(grid_for(n, 256, cus * 8)), dim3(256), 0, st, d, rec, n, dst, offs, strings, strlen);
	return hipGetLastError();
}
hipError_t launch_merge(const Dev& d, const ebd_wire_service* rec, uint32_t n, const uint8_t* strings, unsigned long long strlen,
		const unsigned long long* offs, hipStream_t st, int cus) {
	hipLaunchKernelGGL(k_merge, dim3(grid_for(n, 256, cus * 8)), dim3(256), 0, st, d, rec, n, strings, strlen, offs);
	return hipGetLastError();
}

} // namespace ebd
