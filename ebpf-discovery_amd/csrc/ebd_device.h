// ebd_device.h — device-side data structures shared by the kernels (ebd_kernels.hip).
#pragma once

#include "../../include/ebpf_discovery_amd.h"
#include "ebd_dfa.h"
#include "ebd_gen.h"
#include "ebd_spec.h"

namespace ebd {

// Service table slot (64 B, one cache line half): the Aggregator's
// unordered_map<pair<pid, endpoint>, Service> (Aggregator.h:29-37, Service.h:43-66).
struct Slot {
	unsigned long long tag;    // Hash128.lo of (pid, endpoint); 0 = empty; claimed by CAS
	unsigned long long hi;     // Hash128.hi, published by the claimer
	unsigned long long nfirst; // ~(min over requests of seq << 16 | isHttps << 15 | host length): atomicMax of
	                           // the complement, so that an empty slot is all zeros (a plain fill clears)
	unsigned long long pad0[2]; // (the endpoint's arena offset, pid and length live beside the
	                            //  claimed-slot list, Dev::list_ep / list_pl: written in list order)
	unsigned int internal_clients; // uint32, wraps like Service.h:53-54
	unsigned int external_clients;
	unsigned int nets[3];          // network-map sizes: v4 /16, v4 /24, v6 /48 (Service.h:56-58)
	unsigned int pad;
};
static_assert(sizeof(Slot) == 64, "slot is 64 bytes");

// Session-set slot: (pid, fd, sessionID) of every session that needs the sequential
// path in this batch (Discovery.h:47 LRU key, Types.h:72-86).
struct SSlot {
	unsigned long long tag;
	unsigned long long kv; // fd << 32 | pid
	unsigned int sid;
	unsigned int first_c;  // ~(first event of the batch whose fresh parse was UNFINISHED), 0 = none (atomicMax)
	unsigned int carry;    // 1 + index into the carried-session array, 0 = none
	unsigned int visited;
};
static_assert(sizeof(SSlot) == 32, "session slot is 32 bytes (a probe never straddles two lines)");

constexpr uint32_t kCarryBytes = 8200; // > DISCOVERY_MAX_HTTP_REQUEST_LENGTH + 1

// A saved session that outlives its batch: the LRU entry (Discovery.cpp:148-150) with
// its parser state and the bytes of the request in progress.
struct Carry {
	uint32_t pid, fd, sid, nbytes;
	unsigned long long stamp; // global order of the event that last found or inserted it (LRU recency)
	GenParser g;
	uint8_t bytes[kCarryBytes];
};

// Session-path request (ebd_session_request in the public header).
struct SessReq {
	unsigned long long seq;
	uint32_t pid;
	uint32_t str_off;
	uint16_t host_len, url_len, cip_off, cip_len;
	uint8_t info, status;
	uint16_t pad;
	uint32_t pad2;
};
static_assert(sizeof(SessReq) == 32, "session request is 32 bytes");

// 64-bit counters; [0, CTR_BATCH_END) are reset per batch, the rest persist.
enum Ctr : uint32_t {
	CTR_UNFINISHED = 0, // fresh-UNFINISHED events (session-set inserts)
	CTR_SLOW,           // session-path events
	CTR_SREQ,           // session-path requests
	CTR_SSTR,           // session string bytes
	CTR_NEW,            // service slots claimed in this batch
	CTR_CARRY_OUT,      // sessions saved for the next batch
	CTR_DIRTY,          // session-set slots claimed in this batch
	CTR_INSERTS,        // LRU inserts in this batch
	CTR_VERIFY,         // deferred service-key verifications
	CTR_LRU_PEAK,       // 2^31 + max over the batch of (live sessions - carried), upper bound (k_lru_peak)
	CTR_EVICTIONS,      // LRU evictions in this batch (exact path)
	CTR_HEADS,          // sessions with events in this batch (k_walk_heads)
	CTR_BATCH_END = 12,
	CTR_SARENA = 12,    // service string arena bytes used
	CTR_ERRORS,         // EBD_ERR_* bitmask
	CTR_COLLISIONS,
	CTR_KDELETES,
	CTR_REQUESTS,
	CTR_SESSION_EVENTS,
	CTR_SERVICES,       // length of the claimed-slot list (services in the table)
	CTR_EVICTIONS_TOTAL,
	CTR_KEEP,           // services kept by a network-counter clear
	CTR_KEEP_BYTES,     // their endpoint bytes
	CTR_NETS,           // network-map entries claimed (the table's fill)
	CTR_V6D,            // v6 prefix-dictionary slots claimed
	CTR_COUNT = 24,
};

// Network-counter maps of all services (Service.h:45-58): one open-addressing table of
// (service slot, map, prefix) -> time last seen.  key = kind << 62 | slot << 31 | value, with
// value = the prefix bytes (v4 /16: 2, /24: 3) or, for a v6 48-bit prefix, its index in the
// prefix dictionary (v6d: 48-bit prefix | 1 << 63 per slot).  time = 0: erased (or never set).
enum : uint32_t { NET_V4_16 = 1, NET_V4_24 = 2, NET_V6 = 3 };
struct NetEnt {
	unsigned long long key;
	unsigned long long time;
};
EBD_HD unsigned long long net_key(uint32_t kind, uint32_t slot, uint32_t value) {
	return ((unsigned long long)kind << 62) | ((unsigned long long)slot << 31) | value;
}

// A service kept by a network-counter clear (Aggregator.cpp:138-149): re-inserted into the
// emptied table; its endpoint bytes wait in a side arena.
struct KeepRec {
	unsigned long long tag, hi, first, ep_off;
	uint32_t pid, ep_len, old_slot, pad;
	uint32_t nets[3], pad2;
};

struct VerifyRec {
	unsigned long long hi;
	uint32_t slot, pad;
};

// A service k_agg_fast created, staged for publication (k_pub_count, k_publish): its slot and
// everything publication needs of the claiming request, so publication reads no per-event
// array, only the endpoint bytes.
struct ClaimRec {
	uint32_t slot, pid;
	uint16_t host_off, host_len, url_off, url_len;
	unsigned long long off; // the request's buffer in the payload
};
static_assert(sizeof(ClaimRec) == 24, "claim record is 24 bytes");

// Scratch of the exact-LRU rounds (k_lru_*, ebd_api.hip run_batch): per event (ops by sorted
// position, opt by event, marker ends, eviction flags), the compacted markers and eviction
// times, per carried session, the two worlds of eviction flags, per scan block.
// The exact-LRU rounds' control word, advanced on the device at the end of every round
// (k_lru_advance), so the host enqueues rounds without reading each one's counters: the
// window's first event, the horizon, done (settled, or an inconsistent world), the world the
// walk settled in, and the rounds that ran.  Every round kernel returns at once when done.
struct LruCtrl {
	uint32_t front, tend, done, settled, cur_final, rounds, pad_[2];
};

// A scan block's start state in the exact-LRU rounds: the LRU's size, the markers and the
// evictions before the block.
struct LsState {
	int x;
	uint32_t m, e, pad_;
};
struct LruRound {
	LruCtrl* ctl;
	uint8_t* opt;    // per event: its LRU operation in the walked world
	uint32_t* mend;  // per event: the session's next find
	uint32_t* mk_ref;
	uint32_t* mk_e;
	uint32_t* ev_t;
	uint32_t* evc;   // per event: the evictions before it
	uint32_t* cm_end;
	uint32_t* cm_head;
	uint8_t* f[2];   // the worlds walked / derived, by event (bit 0 evicted before it, bit 1 after the session's last)
	uint8_t* cf[2];  // by carried session: evicted with no event in the batch
	LsState* bs;     // per scan block: its start state
	uint32_t* tot; // 1 evictions (to the span's end), 2 window end, 3 next walk list, 5 evictions before the frontier, 6 markers born before the horizon, 7 evictions before it
	uint32_t* jpos;
	uint32_t* head;
	unsigned long long* cnt;
	uint32_t* vict; // per eviction: its victim marker
	uint32_t* mx;   // per marker from the round's queue front: its threshold (k_lru_thresh)
	uint32_t* cpos;  // per session (first sorted position): its first changed position, kNone
	uint32_t* rlist; // the round's walks: start positions
	uint32_t* wto;   // per session: where its last walk stopped (kNone: at its end)
	void* snap;      // per sorted position: the session's state before it (SessState)
	unsigned long long* stat; // EBD_LRU_TRACE only (else null): the walks' statistics, k_walk<true> / k_lru_advance
};

// ebd_parse_streams' parser (ebd_parser_state's contents): the generic state machine plus
// HttpRequest::clientIp as positions in the request stream (HttpRequestParser.h:28-39).
struct StreamParser {
	GenParser g;
	uint32_t vstart, vend; // the current client-IP header value (stream positions)
	uint32_t ntok, dropped;
	uint32_t tok[EBD_PARSE_MAX_TOKENS][2];
};
static_assert(sizeof(StreamParser) <= sizeof(ebd_parser_state), "stream parser fits ebd_parser_state");

// A caller-owned state k_parse_streams may run: every field that indexes something in range
// (the token list, the key trie, the stream the call sees).  ebd_parse_streams rejects others.
EBD_HD bool stream_state_ok(const StreamParser& sp, uint64_t stream_len) {
	const GenParser& g = sp.g;
	return g.state <= ST_INVALID && g.length <= stream_len && g.key < kTrieNodes && sp.ntok <= EBD_PARSE_MAX_TOKENS &&
			sp.vstart <= sp.vend && sp.vend <= g.length && g.cipkey <= 5;
}

// A fast-path request on its way to the owned aggregation (k_own_emit -> k_own_part -> k_own):
// the service key, the event, w = client class | isHttps << 2 | host length << 3, and what a
// claim publishes (ClaimRec's fields), so that no pass reads the event again.
struct OwnEnt {
	unsigned long long lo, hi;
	uint32_t i, w;
	uint32_t pid;
	uint16_t host_off, host_len, url_off, url_len;
	uint32_t pad;
	unsigned long long off;
};
static_assert(sizeof(OwnEnt) == 48, "owned-aggregation entry is 48 bytes");
// The buckets of one batch (zeroed before it): entries per bucket, their starts and cursors in
// ownA, and the 4096-entry tiles before each bucket (k_own_bcount and k_own_part take one tile
// per block).
struct OwnCtl {
	unsigned long long acnt[256];
	unsigned long long aoff[257];
	unsigned long long acur[256];
	uint32_t tcum[257];
};

struct Dev {
	// immutable tables
	const uint8_t* dfa;
	const uint8_t* attr; // DfaTable::attr (the session path's dfa_parse)
	DfaInfo di;
	const KeyTrie* trie;
	const Interfaces* ifs;
	HashKey hkey; // service-key PRF key (ebd_spec.h KeyHasher)
	// batch
	const EventRec* ev;
	const uint32_t* len;
	const uint64_t* off;
	const uint8_t* payload;
	unsigned long long payload_bytes; // buffers lie in [payload, payload + payload_bytes)
	uint32_t n;
	unsigned long long seq_base;
	// per-event outputs
	ebd_event_result* res;
	Hash128* keys;
	// service table
	Slot* slots;
	uint32_t slot_mask;
	uint32_t probe_mask; // probing wraps inside probe_mask + 1 slots: kOwnSlots when the table is in ranges
	// owned aggregation (k_own_*): the counted requests bucketed by range in two exact passes
	// (2^own_abits buckets of 2^own_bbits ranges), each range then one workgroup's
	uint32_t own_abits, own_bbits;
	struct OwnCtl* own_ctl;
	uint16_t* own_rid;   // per event: its range (0xffff: not a counted request)
	uint8_t* own_sub;    // per bucket-ordered entry: its range within the bucket
	struct OwnEnt* ownA; // entries by bucket
	struct OwnEnt* ownB; // entries by range
	uint32_t* own_bcnt;  // per range: entries
	unsigned long long* own_boff; // per range: first entry in ownB (+ the total)
	unsigned long long* own_bcur; // per range: next free entry
	uint32_t* new_slots;
	unsigned long long* list_ep; // beside new_slots: the endpoint's arena offset (~0: none)
	unsigned long long* list_pl; // beside new_slots: pid | endpoint length << 32
	uint32_t new_cap;
	// k_agg_fast's claims, block b's at [b * cstage_per, + blk_cnt[b]): slot and claiming event;
	// the publication kernels' per-block byte counts and list / arena bases
	struct ClaimRec* cstage;
	uint32_t cstage_per;
	uint32_t* blk_cnt;
	uint32_t* blk_bytes;
	unsigned long long* blk_lbase;
	unsigned long long* blk_abase;
	VerifyRec* verify;
	uint32_t verify_cap;
	uint8_t* sarena;
	unsigned long long sarena_cap;
	// session path
	SSlot* sset;
	uint32_t* sset_mask; // in device memory: k_sset_size picks it per batch
	uint32_t* dirty;
	unsigned long long* slow_keys; // session group << 32 | event (k_slow_collect), sorted
	uint32_t* ev_slot;             // per event: its session's session-set slot (session-path events only)
	uint32_t* heads; // sorted position of each session's first event (k_walk_heads)
	uint4* hrec;     // per head (k_walk_heads): its sorted position, first event, session-set slot, group
	unsigned long long* pieces; // per sorted position: its buffer's payload offset << 24 | the bytes a parse may take (the walkers write it, k_emit reads it)
	Carry* carry_in;
	uint32_t n_carry_in;
	Carry* carry_out;
	uint32_t carry_cap;
	SessReq* sreq;
	uint8_t* sstr;
	unsigned long long sstr_cap;
	// network counters (EBD_CFG_NETWORK_COUNTERS)
	uint32_t net_on;
	unsigned long long now; // Aggregator::getCurrentTime of this batch's requests (>= 1)
	const unsigned long long* times; // or per event (ebd_set_event_clock), nullptr: `now` for all
	NetEnt* nets;
	uint32_t net_mask;
	unsigned long long* v6d;
	uint32_t v6d_mask;
	// counters
	unsigned long long* ctr;
};

} // namespace ebd
