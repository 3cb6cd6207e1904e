// ebd_api.hip — the C ABI (include/ebpf_discovery_amd.h): context, device buffers and the
// per-batch pipeline of ebd_kernels.hip.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <cmath>
#include <mutex>
#include <thread>
#include <sys/random.h>
#include <time.h>
#include <vector>

#include "ebd_device.h"
#include "ebd_fresh.h"
#include "ebd_scan.h"

namespace ebd {
hipError_t launch_fresh(const Dev& d, hipStream_t st, int cus);
hipError_t launch_fresh_scan(const Dev& d, hipStream_t st, int cus);
hipError_t launch_sset_build(const Dev& d, uint32_t cap, hipStream_t st, int cus);
hipError_t launch_slow_collect(const Dev& d, hipStream_t st, int cus);
hipError_t launch_walk(const Dev& d, uint32_t nslow, hipStream_t st, int cus);
hipError_t launch_emit(const Dev& d, hipStream_t st, int cus);
hipError_t launch_net_merge(const Dev& d, const ebd_service_net* rec, uint32_t n, hipStream_t st, int cus);
struct SessState;
hipError_t launch_lru_bound(const Dev& d, uint32_t nslow, int* delta, uint8_t* minus, int* scan, void* tmp, size_t tmp_bytes,
		hipStream_t st, int cus);
hipError_t launch_walk_lru(const Dev& d, uint32_t nslow, uint32_t* jpos, uint32_t* head, SessState* S, uint32_t* live,
		uint32_t cap, hipStream_t st, int cus);
size_t sess_state_bytes();
hipError_t launch_lru_round(const Dev& d, uint32_t nslow, const LruRound& w, int cur, uint32_t window, hipStream_t st, int cus);
hipError_t launch_lru_ctl_init(const Dev& d, const LruRound& w, uint32_t window, hipStream_t st);
int lru_size_limit();
hipError_t launch_lru_init(const Dev& d, uint32_t nslow, const LruRound& w, hipStream_t st, int cus);
hipError_t launch_walk_flags(const Dev& d, uint32_t nslow, const uint8_t* f, const uint8_t* cf, hipStream_t st, int cus);
size_t lru_scan_blocks(uint32_t n);
hipError_t launch_carry_pass(const Dev& d, hipStream_t st);
hipError_t launch_agg_fast(const Dev& d, hipStream_t st, int cus);
hipError_t launch_sset_clear(const Dev& d, hipStream_t st, int cus);
hipError_t launch_verify(const Dev& d, hipStream_t st, int cus);
hipError_t launch_parse_streams(const KeyTrie* trie, ebd_parse_call* calls, uint32_t n, const uint8_t* data, hipStream_t st);
hipError_t launch_publish(const Dev& d, uint32_t nblk, hipStream_t st, int cus);
hipError_t launch_own(const Dev& d, hipStream_t st, int cus);
// the library's own device-wide primitives (ebd_kernels.hip)
size_t prim_sort_tmp_bytes(unsigned long long n);
size_t prim_scan_tmp_bytes(unsigned long long n, size_t elem);
hipError_t prim_scan_u32(const unsigned int* in, unsigned int* out, unsigned long long n, int incl, void* tmp, hipStream_t st);
hipError_t prim_scan_u64(const unsigned long long* in, unsigned long long* out, unsigned long long n, int incl, void* tmp, hipStream_t st);
hipError_t prim_sort_keys(unsigned long long* a, unsigned long long* b, unsigned long long n, uint32_t lo, uint32_t hi, void* tmp,
		unsigned long long** sorted, hipStream_t st);
hipError_t prim_select_keys(const unsigned long long* in, unsigned long long* out, unsigned long long n, int* cnt, void* tmp, hipStream_t st);
uint32_t own_range_lg();
uint32_t agg_stage_per_block(uint32_t n, int cus);
hipError_t launch_slots_init(Slot* slots, uint32_t n, hipStream_t st);
hipError_t launch_collect(const Dev& d, ebd_service* out, hipStream_t st, int cus);
hipError_t launch_clear_used(const unsigned int* used, const unsigned long long* ctr, Slot* slots, uint32_t slot_cap,
		hipStream_t st, int cus);
hipError_t launch_gen_len(const GenTables* T, uint32_t config, uint64_t seed, uint64_t first, uint32_t n, uint32_t align,
		uint32_t count, uint32_t index, unsigned long long* alen, uint32_t* keep, hipStream_t st);
hipError_t launch_gen_write(const GenTables* T, uint32_t config, uint64_t seed, uint64_t first, uint32_t n,
		const uint32_t* keep, const uint32_t* pos, const unsigned long long* boff, EventRec* ev, uint32_t* len,
		unsigned long long* off, uint8_t* payload, unsigned long long* gidx, hipStream_t st);
void build_gen_tables(GenTables* T);
hipError_t launch_owner_count(const ebd_service* rec, const unsigned long long* ctr, uint32_t world, unsigned long long* cnt,
		unsigned long long* bytes, hipStream_t st, int cus);
hipError_t launch_owner_scatter(const ebd_service* rec, const unsigned long long* ctr, uint32_t world, unsigned long long* cur,
		ebd_wire_service* out, unsigned long long* srcoff, hipStream_t st, int cus);
hipError_t launch_owner_prefix(const unsigned long long* cnt, uint32_t world, unsigned long long* cur, hipStream_t st);
hipError_t launch_wire_bytes(const ebd_wire_service* rec, uint32_t n, const unsigned long long* nptr, unsigned long long* nb, hipStream_t st,
		int cus);
hipError_t launch_wire_seg_bytes(const ebd_wire_service* rec, uint32_t n, const uint8_t* need, const unsigned long long* dst,
		const unsigned long long* seg, uint32_t world, unsigned long long* out, hipStream_t st, int cus);
hipError_t launch_wire_copy(const ebd_wire_service* rec, uint32_t n, const unsigned long long* nptr, const unsigned long long* offs,
		const unsigned long long* srcoff,
		const uint8_t* arena, uint8_t* strings, hipStream_t st, int cus);
hipError_t launch_merge(const Dev& d, const ebd_wire_service* rec, uint32_t n, const uint8_t* strings, unsigned long long strlen,
		const unsigned long long* offs, hipStream_t st, int cus);
hipError_t launch_agg_requests(const Dev& d, const ebd_request* rq, uint32_t n, const uint8_t* strings, hipStream_t st, int cus);
hipError_t launch_merge_keys(const Dev& d, const ebd_wire_service* rec, uint32_t n, unsigned long long* dst, hipStream_t st, int cus);
hipError_t launch_wire_bytes_needed(const ebd_wire_service* rec, uint32_t n, const uint8_t* need, const unsigned long long* dst,
		unsigned long long* nb, hipStream_t st, int cus);
hipError_t launch_wire_compact(const ebd_wire_service* rec, uint32_t n, const uint8_t* need, const unsigned long long* soff,
		const unsigned long long* doff, const uint8_t* strings, unsigned long long strlen, uint8_t* out, unsigned long long outcap,
		unsigned long long* ctr, hipStream_t st, int cus);
hipError_t launch_merge_bytes(const Dev& d, const ebd_wire_service* rec, uint32_t n, const unsigned long long* dst,
		const unsigned long long* offs, const uint8_t* strings, unsigned long long strlen, hipStream_t st, int cus);
hipError_t launch_gen4_count(unsigned long long seed, uint32_t J, uint32_t* cnt, hipStream_t st);
hipError_t launch_gen4_len(const GenTables* T, unsigned long long seed, uint32_t J, unsigned long long n, uint32_t align,
		const uint32_t* stt, unsigned long long* alen, hipStream_t st);
hipError_t launch_gen4_write(const GenTables* T, unsigned long long seed, uint32_t J, unsigned long long n, const uint32_t* stt,
		const unsigned long long* boff, EventRec* ev, uint32_t* len, unsigned long long* off, uint8_t* payload,
		unsigned long long* gidx, hipStream_t st);
hipError_t launch_net_clean(const Dev& d, unsigned long long now, unsigned long long retention, hipStream_t st, int cus);
hipError_t launch_keep_collect(const Dev& d, KeepRec* keep, unsigned long long* kbytes, unsigned long long kcap, hipStream_t st,
		int cus);
hipError_t launch_keep_insert(const Dev& d, const KeepRec* keep, const uint8_t* kbytes, uint32_t* remap, hipStream_t st, int cus);
hipError_t launch_net_remap(const Dev& d, const NetEnt* old, uint32_t old_mask, const uint32_t* remap,
		const unsigned long long* old_v6d, hipStream_t st, int cus);
hipError_t launch_net_dump(const Dev& d, ebd_service_net* out, uint32_t cap, unsigned long long* count, hipStream_t st, int cus);
} // namespace ebd

using namespace ebd;

// the layouts the Python binding (ebd/__init__.py) and tests/test_abi.py assume
static_assert(sizeof(ebd_config) == 64, "ebd_config layout");
static_assert(sizeof(ebd_stats) == 104, "ebd_stats layout");
static_assert(sizeof(ebd_event_result) == 16 && sizeof(ebd_service) == 80 && sizeof(ebd_service_net) == 32, "result layouts");
static_assert(sizeof(ebd_request) == 40 && sizeof(ebd_device_batch) == 48, "request / batch layouts");

#define HIP_TRY(x)                                                                                                   \
	do {                                                                                                             \
		hipError_t e_ = (x);                                                                                         \
		if (e_ != hipSuccess) {                                                                                      \
			std::fprintf(stderr, "ebd: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
			return -EIO;                                                                                             \
		}                                                                                                            \
	} while (0)

static constexpr uint32_t kMaxAggBlocks = 2048; // k_agg_fast's grid: at most cus * 8 (k_pub_scan scans 2 per thread)

static uint32_t next_pow2(uint64_t v) {
	uint64_t p = 1;
	while (p < v)
		p <<= 1;
	return p > 0x80000000ull ? 0x80000000u : (uint32_t)p;
}

struct ebd_ctx {
	std::mutex mu;
	int device = 0;
	int cus = 256;
	hipStream_t stream = nullptr;
	ebd_config cfg{};
	HashKey hkey{};
	// tables
	DfaTable* dfa_host = nullptr;
	KeyTrie trie_host{};
	Interfaces ifs_host{};
	uint8_t* d_dfa = nullptr;
	KeyTrie* d_trie = nullptr;
	Interfaces* d_ifs = nullptr;
	GenTables* d_gen = nullptr;
	// services
	Slot* d_slots = nullptr;
	uint32_t slot_cap = 0;
	uint32_t* d_new_slots = nullptr;
	ClaimRec* d_cstage = nullptr; // claim stage: max_events + blocks of slack
	uint64_t cstage_cap = 0;
	uint32_t* d_blk = nullptr;    // blk_cnt, blk_bytes (u32) then blk_lbase, blk_abase (u64), blk_cap each
	uint32_t blk_cap = 0;
	// owned aggregation (k_own_*, ebd_kernels.hip): the table in 2048-slot ranges, one workgroup each
	int own_on = 0;
	uint32_t own_abits = 0, own_bbits = 0;
	uint64_t own_n = 0;          // the batch size the entry buffers hold
	OwnCtl* d_own_ctl = nullptr;
	uint16_t* d_own_rid = nullptr;
	uint8_t* d_own_sub = nullptr;
	OwnEnt* d_ownA = nullptr;
	OwnEnt* d_ownB = nullptr;
	uint32_t* d_own_bcnt = nullptr;
	unsigned long long* d_own_boff = nullptr;
	unsigned long long* d_own_bcur = nullptr;
	unsigned long long* d_list_ep = nullptr;
	unsigned long long* d_list_pl = nullptr;
	uint32_t new_cap = 0;
	VerifyRec* d_verify = nullptr;
	uint32_t verify_cap = 0;
	uint8_t* d_sarena = nullptr;
	uint64_t sarena_cap = 0;
	// per-batch
	uint32_t max_events = 0;
	ebd_event_result* d_res = nullptr;
	Hash128* d_keys = nullptr;
	SSlot* d_sset = nullptr;
	uint32_t sset_cap = 0;
	uint32_t* d_dirty = nullptr;
	uint32_t* d_evslot = nullptr;
	uint32_t* d_smask = nullptr; // the session set's mask for the batch (k_sset_size)
	unsigned long long* d_slow[2] = {nullptr, nullptr};
	unsigned long long* d_pieces = nullptr; // Dev::pieces
	uint4* d_hrec = nullptr;                // Dev::hrec (allocated with the first session-path batch)
	void* d_sort_tmp = nullptr;
	size_t sort_tmp_bytes = 0;
	void* d_sel_tmp = nullptr; // compaction of the session-path keys when they are few
	size_t sel_tmp_bytes = 0;
	int* d_sel_cnt = nullptr;
	Carry* d_carry[2] = {nullptr, nullptr};
	int carry_cur = 0;
	uint32_t n_carry = 0;
	uint32_t carry_cap = 0;
	SessReq* d_sreq = nullptr;
	uint8_t* d_sstr = nullptr;
	uint64_t sstr_cap = 0;
	unsigned long long* d_ctr = nullptr;
	unsigned long long* h_ctr = nullptr; // pinned
	unsigned long long* d_cnt = nullptr;
	ebd_service* d_collect = nullptr;
	// exact LRU (allocated on first need): bound arrays, event -> position, session states
	int* d_lru_delta = nullptr;
	uint8_t* d_lru_minus = nullptr;
	int* d_lru_scan = nullptr;
	void* d_lru_tmp = nullptr;
	size_t lru_tmp_bytes = 0;
	uint32_t* d_lru_jpos = nullptr;
	uint32_t* d_lru_head = nullptr;
	void* d_lru_sess = nullptr;
	uint32_t* d_lru_live = nullptr;
	uint64_t lru_batches_exact = 0;
	uint64_t lru_rounds = 0, lru_sequential = 0;
	uint32_t lru_window = 0; // exact-LRU derivation window (0: EBD_LRU_WINDOW or 8192)
	LruRound lr{};              // the exact-LRU rounds' scratch (allocated on first need)
	void* lr_mem = nullptr;
	unsigned long long* h_lr = nullptr; // pinned: a round's counters
	unsigned long long* h_small = nullptr; // pinned: the counts and totals a C-ABI call waits for (kSmall words)
	uint8_t* h_ps = nullptr;            // pinned: ebd_parse_streams' calls and bytes, both ways
	size_t h_ps_cap = 0;
	uint8_t* d_ps = nullptr;            // their device copy (grown as needed, kept)
	size_t d_ps_cap = 0;
	// device scratch of the C-ABI calls (scratch_get): chunks kept until the context goes, so
	// that no call frees and re-allocates memory a copy of the same stream still reads
	std::vector<std::pair<uint8_t*, size_t>> scr;
	size_t scr_ci = 0, scr_off = 0;
	// network counters (EBD_CFG_NETWORK_COUNTERS): map entries (two tables: a clear rebuilds
	// into the other), the v6 prefix dictionary, and the network-counter clear's scratch
	int net_on = 0;
	NetEnt* d_nets[2] = {nullptr, nullptr};
	int net_cur = 0;
	uint32_t net_cap = 0;
	unsigned long long* d_v6d[2] = {nullptr, nullptr}; // v6 prefix dictionary, swapped with d_nets
	uint32_t v6d_cap = 0;
	uint64_t clock_ns = 0; // ebd_set_clock (0: CLOCK_MONOTONIC per batch)
	const uint64_t* ev_times = nullptr; // ebd_set_event_clock: the next batch's per-event readings (device)
	KeepRec* d_keep = nullptr;
	uint64_t keep_cap = 0;
	unsigned long long* d_kbytes = nullptr;
	uint64_t kbytes_cap = 0;
	uint32_t* d_remap = nullptr;
	ebd_service_net* d_netdump = nullptr;
	// ingest pipeline (ebd_stage_batch / ebd_submit_staged): two device staging slots filled
	// on the copy stream, pinned bounce buffers for pageable sources, results read back on the
	// D2H stream.  Events: up = the slot's upload is done, used = the batch that read the slot
	// is done (the slot may be refilled).
	struct StageSlot {
		EventRec* ev = nullptr;
		uint32_t* len = nullptr;
		uint64_t* off = nullptr;
		uint8_t* payload = nullptr;
		uint64_t pay_cap = 0;
		uint64_t pay_bytes = 0; // the staged batch's payload_bytes
		uint32_t n = 0;
		uint64_t ticket = 0;
		int staged = 0, used_valid = 0;
		hipEvent_t up = nullptr, used = nullptr;
	};
	hipStream_t cstream = nullptr, dstream = nullptr;
	StageSlot stg[2];
	int next_slot = 0;
	uint64_t next_ticket = 1;
	uint8_t* bounce[2] = {nullptr, nullptr};
	hipEvent_t bounce_ev[2] = {nullptr, nullptr};
	int bounce_valid[2] = {0, 0};
	int bounce_next = 0;
	// batch completion: mid = counters after the fresh pass are on the host; end = the
	// session path's counters (h_end) are; batch = every kernel of the last batch finished;
	// res = the async results read-back finished
	hipEvent_t ev_mid = nullptr, ev_end = nullptr, ev_batch = nullptr, ev_res = nullptr;

	int pending_end = 0, res_pending = 0, batch_valid = 0;
	unsigned long long* h_end = nullptr; // pinned
	// bookkeeping
	unsigned long long seq_base = 0;
	uint32_t last_n = 0;
	uint64_t last_sreq = 0, last_sstr = 0;
	int last_slow_ran = 0;
	uint64_t events_total = 0;
	uint64_t max_live = 0;
	// EBD_CFG_TIMING: event pairs around each launch, summed lazily
	struct Timed {
		int kernel;
		hipEvent_t a, b;
	};
	std::vector<Timed> pending;
	std::vector<hipEvent_t> free_events;
	double kt_ms[16] = {0};
	uint64_t kt_n[16] = {0};
};

constexpr size_t kSmall = 256; // ebd_ctx::h_small words

static const char* kKernelNames[] = {"k_fresh", "k_sset_build", "k_slow_collect", "sort", "k_walk", "k_carry_pass",
		"k_agg_fast", "k_publish", "k_sset_clear", "k_verify", "k_clear_used", "k_emit"};
enum { KT_FRESH, KT_CARRY_INSERT, KT_SLOW_COLLECT, KT_SORT, KT_WALK, KT_CARRY_PASS, KT_AGG, KT_PUBLISH, KT_SSET_CLEAR, KT_VERIFY,
	KT_CLEAR, KT_EMIT, KT_N };
static_assert(KT_N <= 16, "kernel timing slots");

static hipEvent_t take_event(ebd_ctx* c) {
	if (!c->free_events.empty()) {
		hipEvent_t e = c->free_events.back();
		c->free_events.pop_back();
		return e;
	}
	hipEvent_t e = nullptr;
	(void)hipEventCreate(&e);
	return e;
}

// Runs `launch` on the context stream, bracketed by HIP events when timing is on.
template <typename F>
static hipError_t timed(ebd_ctx* c, int kernel, F launch) {
	if (!(c->cfg.flags & EBD_CFG_TIMING))
		return launch();
	hipEvent_t a = take_event(c), b = take_event(c);
	(void)hipEventRecord(a, c->stream);
	hipError_t e = launch();
	(void)hipEventRecord(b, c->stream);
	c->pending.push_back({kernel, a, b});
	return e;
}

static void drain_timing(ebd_ctx* c) {
	for (auto& t : c->pending) {
		float ms = 0.f;
		if (hipEventSynchronize(t.b) == hipSuccess && hipEventElapsedTime(&ms, t.a, t.b) == hipSuccess) {
			c->kt_ms[t.kernel] += ms;
			c->kt_n[t.kernel]++;
		}
		c->free_events.push_back(t.a);
		c->free_events.push_back(t.b);
	}
	c->pending.clear();
}

static Dev make_dev(ebd_ctx* c) {
	Dev d{};
	d.dfa = c->d_dfa;
	d.attr = c->d_dfa + kLdsTableBytes;
	d.di = c->dfa_host->info;
	d.trie = c->d_trie;
	d.ifs = c->d_ifs;
	d.hkey = c->hkey;
	d.res = c->d_res;
	d.keys = c->d_keys;
	d.slots = c->d_slots;
	d.slot_mask = c->slot_cap - 1;
	d.probe_mask = c->own_on ? (1u << own_range_lg()) - 1u : d.slot_mask;
	d.own_abits = c->own_abits;
	d.own_bbits = c->own_bbits;
	d.own_ctl = c->d_own_ctl;
	d.own_rid = c->d_own_rid;
	d.own_sub = c->d_own_sub;
	d.ownA = c->d_ownA;
	d.ownB = c->d_ownB;
	d.own_bcnt = c->d_own_bcnt;
	d.own_boff = c->d_own_boff;
	d.own_bcur = c->d_own_bcur;
	d.new_slots = c->d_new_slots;
	d.cstage = c->d_cstage;
	d.cstage_per = 0;
	d.blk_cnt = c->d_blk;
	d.blk_bytes = c->d_blk + c->blk_cap;
	d.blk_lbase = (unsigned long long*)(c->d_blk + 2 * (size_t)c->blk_cap);
	d.blk_abase = d.blk_lbase + c->blk_cap;
	d.list_ep = c->d_list_ep;
	d.list_pl = c->d_list_pl;
	d.new_cap = c->new_cap;
	d.verify = c->d_verify;
	d.verify_cap = c->verify_cap;
	d.sarena = c->d_sarena;
	d.sarena_cap = c->sarena_cap;
	d.sset = c->d_sset;
	d.sset_mask = c->d_smask;
	d.dirty = c->d_dirty;
	d.ev_slot = c->d_evslot;
	d.slow_keys = c->d_slow[0];
	d.pieces = c->d_pieces;
	d.hrec = c->d_hrec;
	d.carry_in = c->d_carry[c->carry_cur];
	d.n_carry_in = c->n_carry;
	d.carry_out = c->d_carry[c->carry_cur ^ 1];
	d.carry_cap = c->carry_cap;
	d.sreq = c->d_sreq;
	d.sstr = c->d_sstr;
	d.sstr_cap = c->sstr_cap;
	d.ctr = c->d_ctr;
	d.seq_base = c->seq_base;
	d.net_on = c->net_on;
	d.nets = c->d_nets[c->net_cur];
	d.net_mask = c->net_cap ? c->net_cap - 1 : 0;
	d.v6d = c->d_v6d[c->net_cur];
	d.v6d_mask = c->v6d_cap ? c->v6d_cap - 1 : 0;
	d.now = 1;
	return d;
}

// Aggregator::getCurrentTime (A:211-213): std::chrono::steady_clock is CLOCK_MONOTONIC.
static uint64_t ctx_now(const ebd_ctx* c) {
	if (c->clock_ns)
		return c->clock_ns;
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	const uint64_t t = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
	return t ? t : 1;
}

// The session-path keys are sorted in place (all n) when at least 1/EBD_SLOW_DENSE of the events
// take the path, else compacted first (0: always compacted, a test build).
#ifndef EBD_SLOW_DENSE
#define EBD_SLOW_DENSE 4
#endif
// A session-path key of k_slow_collect (other events hold ~0).
static void ctx_free(ebd_ctx* c) {
	void* ptrs[] = {c->d_ownA, c->d_ownB, c->d_own_ctl, c->d_own_rid, c->d_own_sub, c->d_own_bcnt, c->d_own_boff, c->d_own_bcur, c->d_dfa, c->d_trie, c->d_ifs, c->d_gen, c->d_slots,
			c->d_new_slots, c->d_cstage, c->d_blk, c->d_list_ep, c->d_list_pl, c->d_verify, c->d_sarena, c->d_res, c->d_keys,
			c->d_sset, c->d_dirty, c->d_evslot, c->d_smask, c->d_slow[0], c->d_slow[1], c->d_pieces, c->d_hrec, c->d_sort_tmp, c->d_sel_tmp, c->d_sel_cnt, c->d_carry[0], c->d_carry[1], c->d_sreq,
			c->d_sstr, c->d_ctr, c->d_cnt, c->d_collect, c->d_lru_delta, c->d_lru_minus,
			c->d_lru_scan, c->d_lru_tmp, c->d_lru_jpos, c->d_lru_head, c->d_lru_sess, c->d_lru_live, c->d_nets[0], c->d_nets[1],
			c->d_v6d[0], c->d_v6d[1], c->d_keep, c->d_kbytes, c->d_remap, c->d_netdump};
	for (void* p : ptrs)
		if (p)
			(void)hipFree(p);
	if (c->h_ctr)
		(void)hipHostFree(c->h_ctr);
	if (c->h_end)
		(void)hipHostFree(c->h_end);
	if (c->lr_mem)
		(void)hipFree(c->lr_mem);
	if (c->lr.stat)
		(void)hipFree(c->lr.stat);
	if (c->h_lr)
		(void)hipHostFree(c->h_lr);
	if (c->h_small)
		(void)hipHostFree(c->h_small);
	if (c->h_ps)
		(void)hipHostFree(c->h_ps);
	if (c->d_ps)
		(void)hipFree(c->d_ps);
	for (auto& ch : c->scr)
		(void)hipFree(ch.first);
	for (int k = 0; k < 2; k++) {
		auto& g = c->stg[k];
		void* sp[] = {g.ev, g.len, g.off, g.payload};
		for (void* p : sp)
			if (p)
				(void)hipFree(p);
		if (g.up)
			(void)hipEventDestroy(g.up);
		if (g.used)
			(void)hipEventDestroy(g.used);
		if (c->bounce[k])
			(void)hipHostFree(c->bounce[k]);
		if (c->bounce_ev[k])
			(void)hipEventDestroy(c->bounce_ev[k]);
	}
	for (hipEvent_t e : {c->ev_mid, c->ev_end, c->ev_batch, c->ev_res})
		if (e)
			(void)hipEventDestroy(e);
	if (c->cstream)
		(void)hipStreamDestroy(c->cstream);
	if (c->dstream)
		(void)hipStreamDestroy(c->dstream);
	for (auto& t : c->pending) {
		(void)hipEventDestroy(t.a);
		(void)hipEventDestroy(t.b);
	}
	for (auto e : c->free_events)
		(void)hipEventDestroy(e);
	if (c->stream)
		(void)hipStreamDestroy(c->stream);
	delete c->dfa_host;
	delete c;
}

extern "C" {

#ifndef EBD_BUILD_ID
#define EBD_BUILD_ID "unknown"
#endif
const char* ebd_build_id(void) { return EBD_BUILD_ID; }

const char* ebd_strerror(int err) {
	switch (-err) {
	case 0: return "success";
	case EINVAL: return "invalid argument";
	case ENOMEM: return "out of device memory";
	case EIO: return "HIP runtime error";
	case ENOSPC: return "capacity exceeded";
	case ENODEV: return "no HIP device";
	default: return "unknown error";
	}
}

int ebd_ctx_create(const ebd_config* cfg, ebd_ctx** out) {
	// lru_capacity: a carried request's index travels in 24 bits (EmitRec); 2^24 carried
	// sessions would be 140 GB of carry buffers
	if (!cfg || !out || cfg->max_events == 0 || cfg->lru_capacity >= (1u << 24))
		return -EINVAL;
	*out = nullptr;
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
		return -ENODEV;
	if (cfg->device < 0 || cfg->device >= ndev)
		return -EINVAL;
	ebd_ctx* c = new ebd_ctx();
	c->cfg = *cfg;
	if (const char* f = std::getenv("EBD_FRESH")) // A/B: EBD_FRESH=scan runs k_fresh_scan, =dfa k_fresh
		c->cfg.flags = std::strcmp(f, "scan") == 0 ? (c->cfg.flags | EBD_CFG_FRESH_SCAN) : (c->cfg.flags & ~EBD_CFG_FRESH_SCAN);
	c->device = cfg->device;
	c->max_events = cfg->max_events;
	if (hipSetDevice(c->device) != hipSuccess) {
		ctx_free(c);
		return -EIO;
	}
	c->hkey = HashKey{cfg->hash_key[0], cfg->hash_key[1]};
	if (c->hkey.k0 == 0 && c->hkey.k1 == 0) {
		uint64_t k[2] = {0, 0};
		if (getrandom(k, sizeof(k), 0) != (ssize_t)sizeof(k)) {
			ctx_free(c);
			return -EIO;
		}
		c->hkey = HashKey{k[0], k[1]};
		c->cfg.hash_key[0] = k[0];
		c->cfg.hash_key[1] = k[1];
	}
	hipDeviceProp_t prop;
	if (hipGetDeviceProperties(&prop, c->device) == hipSuccess && prop.multiProcessorCount > 0)
		c->cus = prop.multiProcessorCount;
	int rc = 0;
	auto fail = [&](int r) {
		ctx_free(c);
		return r;
	};
#define CTX_TRY(x)                                                                                                   \
	do {                                                                                                             \
		hipError_t e_ = (x);                                                                                         \
		if (e_ != hipSuccess) {                                                                                      \
			std::fprintf(stderr, "ebd: %s failed: %s\n", #x, hipGetErrorString(e_));                               \
			return fail(e_ == hipErrorOutOfMemory ? -ENOMEM : -EIO);                                                 \
		}                                                                                                            \
	} while (0)
	CTX_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
	CTX_TRY(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
	CTX_TRY(hipStreamCreateWithFlags(&c->dstream, hipStreamNonBlocking));
	for (hipEvent_t* e : {&c->ev_mid, &c->ev_end, &c->ev_batch, &c->ev_res, &c->stg[0].up, &c->stg[0].used, &c->stg[1].up,
			 &c->stg[1].used, &c->bounce_ev[0], &c->bounce_ev[1]})
		CTX_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
	// tables derived from the parser semantics (ebd_spec.h)
	build_key_trie(&c->trie_host);
	c->dfa_host = new DfaTable();
	rc = build_dfa(&c->trie_host, c->dfa_host);
	if (rc != 0) {
		std::fprintf(stderr, "ebd: DFA construction failed (%d)\n", rc);
		return fail(-EIO);
	}
	std::vector<uint8_t> image(kLdsTableBytes); // the table as k_fresh keeps it in LDS
	build_lds_image(c->dfa_host, image.data());
	image.insert(image.end(), c->dfa_host->attr, c->dfa_host->attr + 256); // dfa_parse's state attributes follow the table
	CTX_TRY(hipMalloc(&c->d_dfa, image.size()));
	CTX_TRY(hipMemcpy(c->d_dfa, image.data(), image.size(), hipMemcpyHostToDevice));
	CTX_TRY(hipMalloc(&c->d_trie, sizeof(KeyTrie)));
	CTX_TRY(hipMemcpy(c->d_trie, &c->trie_host, sizeof(KeyTrie), hipMemcpyHostToDevice));
	std::memset(&c->ifs_host, 0, sizeof(Interfaces));
	CTX_TRY(hipMalloc(&c->d_ifs, sizeof(Interfaces)));
	CTX_TRY(hipMemcpy(c->d_ifs, &c->ifs_host, sizeof(Interfaces), hipMemcpyHostToDevice));
	// service table
	c->slot_cap = next_pow2(cfg->service_capacity ? cfg->service_capacity : (1u << 22));
	CTX_TRY(hipMalloc(&c->d_slots, (size_t)c->slot_cap * sizeof(Slot)));
	CTX_TRY(launch_slots_init(c->d_slots, c->slot_cap, c->stream));
	c->new_cap = c->slot_cap; // claimed-slot list, cumulative until ebd_clear
	CTX_TRY(hipMalloc(&c->d_new_slots, (size_t)c->new_cap * sizeof(uint32_t)));
	// one stretch of per-block capacity per k_agg_fast block: grid * ceil(steps / grid) steps of
	// kAggThreads events, below (steps + grid) * kAggThreads for any batch up to max_events
	c->cstage_cap = (((uint64_t)c->max_events + 255) / 256 + kMaxAggBlocks) * 256;
	c->blk_cap = kMaxAggBlocks;
	{
		// the owned aggregation (opt-in) takes tables of 2^18 to 2^26 slots in ranges of
		// 2^own_range_lg(): 2^own_abits buckets (<= 128) of 2^own_bbits ranges (<= 256); network
		// counters keep k_agg_fast
		uint32_t lg = 0;
		while ((1ull << lg) < c->slot_cap)
			lg++;
		const uint32_t rbits = lg > own_range_lg() ? lg - own_range_lg() : 0;
		const char* agg = getenv("EBD_AGG"); // "own": the owned aggregation (measured slower than k_agg_fast)
		if (agg && !strcmp(agg, "own") && rbits >= 7 && rbits <= 15 && !(cfg->flags & EBD_CFG_NETWORK_COUNTERS)) {
			c->own_on = 1;
			c->own_bbits = rbits < 8 ? rbits : 8;
			c->own_abits = rbits - c->own_bbits;
			const uint64_t nr = 1ull << rbits;
			c->blk_cap = (uint32_t)std::max<uint64_t>(kMaxAggBlocks, nr);
			c->cstage_cap = std::max<uint64_t>(c->cstage_cap, nr << own_range_lg());
			CTX_TRY(hipMalloc(&c->d_own_ctl, sizeof(OwnCtl)));
			CTX_TRY(hipMalloc(&c->d_own_bcnt, nr * sizeof(uint32_t)));
			CTX_TRY(hipMalloc(&c->d_own_boff, (nr + 1) * sizeof(unsigned long long)));
			CTX_TRY(hipMalloc(&c->d_own_bcur, nr * sizeof(unsigned long long)));
		}
	}
	CTX_TRY(hipMalloc(&c->d_cstage, c->cstage_cap * sizeof(ClaimRec)));
	CTX_TRY(hipMalloc(&c->d_blk, (size_t)c->blk_cap * (2 * sizeof(uint32_t) + 2 * sizeof(unsigned long long))));
	CTX_TRY(hipMalloc(&c->d_list_ep, (size_t)c->new_cap * sizeof(unsigned long long)));
	CTX_TRY(hipMalloc(&c->d_list_pl, (size_t)c->new_cap * sizeof(unsigned long long)));
	c->verify_cap = c->max_events;
	CTX_TRY(hipMalloc(&c->d_verify, (size_t)c->verify_cap * sizeof(VerifyRec)));
	c->sarena_cap = cfg->string_arena ? cfg->string_arena : (256ull << 20);
	CTX_TRY(hipMalloc(&c->d_sarena, c->sarena_cap + 64)); // k_reps stores whole 8-byte words
	// per-batch buffers
	const uint64_t n = c->max_events;
	CTX_TRY(hipMalloc(&c->d_res, n * sizeof(ebd_event_result)));
	CTX_TRY(hipMalloc(&c->d_keys, n * sizeof(Hash128)));
	const uint32_t lru = cfg->lru_capacity ? cfg->lru_capacity : EBD_MAX_SESSIONS;
	c->carry_cap = lru;
	c->sset_cap = next_pow2(2 * (n + lru));
	CTX_TRY(hipMalloc(&c->d_sset, (size_t)c->sset_cap * sizeof(SSlot)));
	CTX_TRY(hipMemsetAsync(c->d_sset, 0, (size_t)c->sset_cap * sizeof(SSlot), c->stream));
	CTX_TRY(hipMalloc(&c->d_dirty, (n + lru) * sizeof(uint32_t)));
	CTX_TRY(hipMalloc(&c->d_evslot, (size_t)n * sizeof(uint32_t)));
	CTX_TRY(hipMalloc(&c->d_smask, sizeof(uint32_t)));
	CTX_TRY(hipMalloc(&c->d_slow[0], n * sizeof(unsigned long long)));
	CTX_TRY(hipMalloc(&c->d_slow[1], n * sizeof(unsigned long long)));
	CTX_TRY(hipMalloc(&c->d_pieces, n * sizeof(unsigned long long)));
	c->sort_tmp_bytes = prim_sort_tmp_bytes(n);
	CTX_TRY(hipMalloc(&c->d_sort_tmp, c->sort_tmp_bytes));
	c->sel_tmp_bytes = prim_scan_tmp_bytes(n, sizeof(unsigned int));
	CTX_TRY(hipMalloc(&c->d_sel_tmp, c->sel_tmp_bytes));
	CTX_TRY(hipMalloc(&c->d_sel_cnt, sizeof(int)));
	// + 64: stream_copy3 reads a carried request's bytes up to 8 past their end
	CTX_TRY(hipMalloc(&c->d_carry[0], (size_t)lru * sizeof(Carry) + 64));
	CTX_TRY(hipMalloc(&c->d_carry[1], (size_t)lru * sizeof(Carry) + 64));
	CTX_TRY(hipMalloc(&c->d_sreq, n * sizeof(SessReq)));
	c->sstr_cap = n * 160;
	if (c->sstr_cap < (64ull << 20))
		c->sstr_cap = 64ull << 20;
	if (c->sstr_cap > (4ull << 30))
		c->sstr_cap = 4ull << 30;
	CTX_TRY(hipMalloc(&c->d_sstr, c->sstr_cap + 64)); // k_reps reads whole 8-byte words
	// one word past the counters: k_walk's chunk counter (zeroed before each walk)
	CTX_TRY(hipMalloc(&c->d_ctr, (CTR_COUNT + 1) * sizeof(unsigned long long)));
	CTX_TRY(hipMemsetAsync(c->d_ctr, 0, (CTR_COUNT + 1) * sizeof(unsigned long long), c->stream));
	CTX_TRY(hipMalloc(&c->d_cnt, sizeof(unsigned long long)));
	CTX_TRY(hipHostMalloc(&c->h_ctr, (CTR_COUNT + 1) * sizeof(unsigned long long), hipHostMallocDefault));
	CTX_TRY(hipHostMalloc(&c->h_small, kSmall * sizeof(unsigned long long), hipHostMallocDefault));
	CTX_TRY(hipHostMalloc(&c->h_end, CTR_COUNT * sizeof(unsigned long long), hipHostMallocDefault));
	if (cfg->flags & EBD_CFG_NETWORK_COUNTERS) {
		c->net_on = 1;
		c->net_cap = next_pow2(cfg->net_capacity ? cfg->net_capacity : (1u << 22));
		c->v6d_cap = c->net_cap;
		for (int k = 0; k < 2; k++) {
			CTX_TRY(hipMalloc(&c->d_nets[k], (size_t)c->net_cap * sizeof(NetEnt)));
			CTX_TRY(hipMemsetAsync(c->d_nets[k], 0, (size_t)c->net_cap * sizeof(NetEnt), c->stream));
		}
		for (int k = 0; k < 2; k++) {
			CTX_TRY(hipMalloc(&c->d_v6d[k], (size_t)c->v6d_cap * sizeof(unsigned long long)));
			CTX_TRY(hipMemsetAsync(c->d_v6d[k], 0, (size_t)c->v6d_cap * sizeof(unsigned long long), c->stream));
		}
	}
	CTX_TRY(hipStreamSynchronize(c->stream));
#undef CTX_TRY
	*out = c;
	return 0;
}

int ebd_ctx_destroy(ebd_ctx* c) {
	if (!c)
		return -EINVAL;
	(void)hipSetDevice(c->device);
	(void)hipStreamSynchronize(c->stream);
	ctx_free(c);
	return 0;
}

void* ebd_ctx_stream(ebd_ctx* c) { return c ? (void*)c->stream : nullptr; }

int ebd_get_hash_key(ebd_ctx* c, uint64_t out[2]) {
	if (!c || !out)
		return -EINVAL;
	out[0] = c->hkey.k0;
	out[1] = c->hkey.k1;
	return 0;
}

int ebd_set_interfaces(ebd_ctx* c, const ebd_ipv4_network* v4, uint32_t n4, const ebd_ipv6_network* v6, uint32_t n6) {
	if (!c || n4 > 64 || n6 > 32 || (n4 && !v4) || (n6 && !v6))
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	std::memset(&c->ifs_host, 0, sizeof(Interfaces));
	c->ifs_host.n4 = n4;
	c->ifs_host.n6 = n6;
	for (uint32_t i = 0; i < n4; i++) {
		std::memcpy(c->ifs_host.v4[i], v4[i].addr, 4);
		std::memcpy(c->ifs_host.v4[i] + 4, v4[i].mask, 4);
	}
	for (uint32_t i = 0; i < n6; i++) {
		std::memcpy(c->ifs_host.v6[i], v6[i].addr, 16);
		std::memcpy(c->ifs_host.v6[i] + 16, v6[i].mask, 16);
	}
	HIP_TRY(hipSetDevice(c->device));
	HIP_TRY(hipMemcpyAsync(c->d_ifs, &c->ifs_host, sizeof(Interfaces), hipMemcpyHostToDevice, c->stream));
	HIP_TRY(hipStreamSynchronize(c->stream));
	return 0;
}

// The session path's end-of-batch counters (carried sessions, session requests) of the
// previous batch: read when the next call needs them, not at the end of the batch.
static int finish_pending(ebd_ctx* c) {
	if (!c->pending_end)
		return 0;
	HIP_TRY(hipEventSynchronize(c->ev_end));
	c->pending_end = 0;
	const uint64_t co = c->h_end[CTR_CARRY_OUT];
	c->n_carry = (uint32_t)(co < c->carry_cap ? co : c->carry_cap);
	c->carry_cur ^= 1;
	c->last_sreq = c->h_end[CTR_SREQ];
	c->last_sstr = c->h_end[CTR_SSTR];
	const uint64_t bound = c->n_carry + c->h_end[CTR_INSERTS];
	if (bound > c->max_live)
		c->max_live = bound;
	return 0;
}

// The exact-LRU rounds' scratch, one allocation carved into LruRound's arrays.
static int lru_alloc(ebd_ctx* c) {
	if (c->lr_mem)
		return 0;
	const size_t n = c->max_events, cc = c->carry_cap, nb = lru_scan_blocks(c->max_events) + 1;
	LruRound& w = c->lr;
	struct Part {
		void** p;
		size_t bytes;
	} parts[] = {{(void**)&w.opt, n}, {(void**)&w.mend, 4 * n}, {(void**)&w.mk_ref, 4 * (n + cc)}, {(void**)&w.mk_e, 4 * (n + cc)},
			{(void**)&w.ev_t, 4 * n}, {(void**)&w.evc, 4 * n}, {(void**)&w.cm_end, 4 * cc}, {(void**)&w.cm_head, 4 * cc},
			{(void**)&w.f[0], n}, {(void**)&w.f[1], n}, {(void**)&w.cf[0], cc}, {(void**)&w.cf[1], cc}, {(void**)&w.bs, sizeof(LsState) * (nb + 1)},
			{(void**)&w.ctl, sizeof(LruCtrl)}, {(void**)&w.tot, 32}, {(void**)&w.jpos, 4 * n}, {(void**)&w.head, 4 * n}, {(void**)&w.cnt, 32},
			{(void**)&w.cpos, 4 * n}, {(void**)&w.rlist, 4 * n}, {(void**)&w.vict, 4 * (n + 1)},
			{(void**)&w.mx, 4 * (n + cc + 64)}, {(void**)&w.wto, 4 * n}, {(void**)&w.snap, sess_state_bytes() * n}};
	size_t total = 0;
	for (const Part& q : parts)
		total += (q.bytes + 255) & ~(size_t)255;
	HIP_TRY(hipMalloc(&c->lr_mem, total));
	if (!c->h_lr)
		HIP_TRY(hipHostMalloc(&c->h_lr, 8 * sizeof(unsigned long long), hipHostMallocDefault));
	uint8_t* p = (uint8_t*)c->lr_mem;
	for (const Part& q : parts) {
		*q.p = p;
		p += (q.bytes + 255) & ~(size_t)255;
	}
	return 0;
}

// The exact LRU in rounds (ebd_kernels.hip k_lru_*): walk the sessions in a world of
// evictions without output, derive the evictions the walk's LRU operations imply, repeat
// until the world derived is the world walked; then the walk with output.  Events before the
// frontier are settled; a round derives the evictions of [front, front + window) (and keeps
// the earlier ones) and walks again only the sessions whose flags changed.  *settled = 0: the
// rounds did not settle (the caller replays the batch sequentially instead).
static int run_lru_rounds(ebd_ctx* c, const Dev& d, uint32_t nslow, int* settled) {
	*settled = 0;
	if (c->carry_cap >= (uint32_t)lru_size_limit())
		return 0; // the rounds' 32-bit size maps do not reach: the one-lane replay takes the batch
	if (int rc = lru_alloc(c))
		return rc;
	LruRound& w = c->lr;
	HIP_TRY(launch_lru_init(d, nslow, w, c->stream, c->cus));
	static const bool lru_trace = std::getenv("EBD_LRU_TRACE") != nullptr; // per-round progress on stderr
	// the window trades rounds (a round settles at most the window) against each round's merge
	// work (it re-derives the whole window); EBD_LRU_WINDOW overrides it
	static const uint32_t env_window = [] {
		const char* v = std::getenv("EBD_LRU_WINDOW");
		const long w = v ? std::atol(v) : 0;
		return w > 0 ? (uint32_t)w : 8192u; // 1 M config-4 events, LRU 2048: 2048 -> 523 ms, 4096 -> 394, 8192 -> 347, 16384 -> 387
	}();
	const uint32_t window = c->lru_window ? c->lru_window : env_window;
	// a round settles at least one event and usually most of a window (1 M config-4 events: ~3.3
	// rounds per window), so the cap grows with the windows the batch holds
	const int max_rounds = (int)std::min<unsigned long long>(1ull << 30, 4096ull + 8ull * ((d.n + window - 1) / window));
	// The rounds advance their frontier on the device (k_lru_advance) and stop themselves once
	// settled, so the host enqueues them kRoundChunk at a time and reads the control word once per
	// chunk: no host round trip per round (a settled chunk's remaining rounds exit at once).
	constexpr int kRoundChunk = 8;
	HIP_TRY(launch_lru_ctl_init(d, w, window, c->stream));
	if (lru_trace && !w.stat) {
		HIP_TRY(hipMalloc(&w.stat, 8 * sizeof(unsigned long long)));
		HIP_TRY(hipMemsetAsync(w.stat, 0, 8 * sizeof(unsigned long long), c->stream));
	}
	LruCtrl* h = (LruCtrl*)c->h_lr;
	static_assert(sizeof(LruCtrl) <= 8 * sizeof(unsigned long long), "the control word fits the host read buffer");
	int r = 0;
	for (;;) {
		for (int k = 0; k < kRoundChunk; k++, r++)
			HIP_TRY(timed(c, KT_WALK, [&] { return launch_lru_round(d, nslow, w, r & 1, window, c->stream, c->cus); }));
		HIP_TRY(hipMemcpyAsync(h, w.ctl, sizeof(LruCtrl), hipMemcpyDeviceToHost, c->stream));
		HIP_TRY(hipStreamSynchronize(c->stream));
		if (lru_trace)
			std::fprintf(stderr, "ebd lru rounds %d..%d: front %u, done %u, settled %u, rounds run %u\n", r - kRoundChunk, r - 1, h->front,
					h->done, h->settled, h->rounds);
		if (h->done || r >= max_rounds)
			break;
	}
	c->lru_rounds += h->rounds;
	if (lru_trace) {
		unsigned long long sv[8];
		HIP_TRY(hipMemcpy(sv, w.stat, sizeof(sv), hipMemcpyDeviceToHost));
		std::fprintf(stderr, "ebd lru walks (cumulative): %llu rounds, sessions %llu, events %llu, bytes %llu, longest lane's bytes summed %llu\n",
				(unsigned long long)c->lru_rounds, sv[4], sv[0], sv[1], sv[2]);
	}
	if (!h->done || !h->settled)
		return 0;
	*settled = 1;
	const int cur = (int)h->cur_final;
	HIP_TRY(timed(c, KT_WALK, [&] { return launch_walk_flags(d, nslow, w.f[cur], w.cf[cur], c->stream, c->cus); }));
	HIP_TRY(hipMemcpyAsync(c->d_ctr + CTR_EVICTIONS, w.cnt, sizeof(unsigned long long), hipMemcpyDeviceToDevice, c->stream));
	return 0;
}

// The owned aggregation's per-event and entry buffers for a batch of n events (entries are the
// counted requests, at most one per event), grown when a larger batch comes.
static hipError_t ensure_own(ebd_ctx* c, uint32_t n) {
	if (n <= c->own_n && c->d_ownA)
		return hipSuccess;
	const uint64_t want = std::max<uint64_t>(n, 1u << 16);
	hipError_t e = hipStreamSynchronize(c->stream);
	if (e != hipSuccess)
		return e;
	void** bufs[] = {(void**)&c->d_ownA, (void**)&c->d_ownB, (void**)&c->d_own_rid, (void**)&c->d_own_sub};
	for (void** b : bufs) {
		if (*b)
			(void)hipFree(*b);
		*b = nullptr;
	}
	c->own_n = 0;
	if ((e = hipMalloc(&c->d_ownA, want * sizeof(OwnEnt))) != hipSuccess || (e = hipMalloc(&c->d_ownB, want * sizeof(OwnEnt))) != hipSuccess ||
			(e = hipMalloc(&c->d_own_rid, want * sizeof(uint16_t))) != hipSuccess || (e = hipMalloc(&c->d_own_sub, want)) != hipSuccess)
		return e;
	c->own_n = want;
	return hipSuccess;
}

// One poll cycle on the context stream.  The host waits once, for the counters after the
// fresh pass (is there session work?), while k_agg_fast already runs; a batch without session
// work returns with its kernels still queued, and a batch with some returns once the session
// path is queued (its carried-session count is read by the next call, finish_pending).
static int run_batch(ebd_ctx* c, const EventRec* ev, const uint32_t* len, const uint64_t* off, const uint8_t* payload,
		uint64_t payload_bytes, uint32_t n) {
	if (n > c->max_events)
		return -EINVAL;
	HIP_TRY(hipSetDevice(c->device));
	if (int rc = finish_pending(c))
		return rc;
	if (c->res_pending) { // the previous results are being read back: k_fresh rewrites them
		HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_res, 0));
		c->res_pending = 0;
	}
	Dev d = make_dev(c);
	d.ev = ev;
	d.len = len;
	d.off = off;
	d.payload = payload;
	d.payload_bytes = payload_bytes;
	d.n = n;
	d.now = ctx_now(c);
	d.times = (const unsigned long long*)c->ev_times; // for this batch only
	c->ev_times = nullptr;
	d.cstage_per = agg_stage_per_block(n, c->cus);
	c->last_n = n;
	c->last_slow_ran = 0;
	HIP_TRY(hipMemsetAsync(c->d_ctr, 0, CTR_BATCH_END * sizeof(unsigned long long), c->stream));
	if (n == 0) {
		c->last_sreq = c->last_sstr = 0;
		HIP_TRY(hipEventRecord(c->ev_batch, c->stream));
		c->batch_valid = 1;
		return 0;
	}
	HIP_TRY(timed(c, KT_FRESH, [&] {
		return (c->cfg.flags & EBD_CFG_FRESH_SCAN) ? launch_fresh_scan(d, c->stream, c->cus) : launch_fresh(d, c->stream, c->cus);
	}));
	HIP_TRY(timed(c, KT_CARRY_INSERT, [&] { return launch_sset_build(d, c->sset_cap, c->stream, c->cus); }));
	HIP_TRY(timed(c, KT_SLOW_COLLECT, [&] { return launch_slow_collect(d, c->stream, c->cus); }));
	HIP_TRY(hipMemcpyAsync(c->h_ctr, c->d_ctr, CTR_COUNT * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
	HIP_TRY(hipEventRecord(c->ev_mid, c->stream));
	// Aggregator::newRequest for the fast-path requests: independent of the session path
	// (k_slow_collect marked the session events, counters and first arrival are order-free)
	uint32_t pub_blocks = 0; // the claim stretches the publication walks (0: k_agg_fast's grid)
	if (c->own_on) {
		HIP_TRY(ensure_own(c, n));
		d.own_rid = c->d_own_rid;
		d.own_sub = c->d_own_sub;
		d.ownA = c->d_ownA;
		d.ownB = c->d_ownB;
		d.cstage_per = 1u << own_range_lg();
		pub_blocks = 1u << (c->own_abits + c->own_bbits);
		HIP_TRY(hipMemsetAsync(c->d_own_ctl, 0, sizeof(OwnCtl), c->stream));
		HIP_TRY(hipMemsetAsync(c->d_own_bcnt, 0, ((size_t)1 << (c->own_abits + c->own_bbits)) * sizeof(uint32_t), c->stream));
		HIP_TRY(timed(c, KT_AGG, [&] { return launch_own(d, c->stream, c->cus); }));
	} else {
		HIP_TRY(timed(c, KT_AGG, [&] { return launch_agg_fast(d, c->stream, c->cus); }));
	}
	HIP_TRY(timed(c, KT_PUBLISH, [&] { return launch_publish(d, pub_blocks, c->stream, c->cus); }));
	HIP_TRY(hipEventSynchronize(c->ev_mid));
	const uint64_t nslow = c->h_ctr[CTR_SLOW];
	const uint64_t dirty = c->h_ctr[CTR_DIRTY];
	if (nslow > 0) {
		c->last_slow_ran = 1;
		// session groups (carried index, or carry_cap + first unfinished event) in bits [32,
		// end_bit), every group below the all-ones pattern of the ~0 keys of other events
		int end_bit = 32;
		while ((1ull << (end_bit - 32)) <= (uint64_t)c->carry_cap + c->max_events)
			end_bit++;
		// k_slow_collect left every event's key at its index, so the keys enter the sort in event
		// order and the (stable) radix sort needs only the group bits: 4 passes instead of 8.  When
		// few events take the session path they are compacted first (order kept).
		const bool dense = nslow * EBD_SLOW_DENSE >= n;
		unsigned long long* sorted = nullptr;
		// the library's stable radix sort (prim_sort_keys, 8 bits per pass) and compaction
		HIP_TRY(timed(c, KT_SORT, [&] {
			if (dense)
				return prim_sort_keys(c->d_slow[0], c->d_slow[1], n, 32, (uint32_t)end_bit, c->d_sort_tmp, &sorted, c->stream);
			hipError_t e = prim_select_keys(c->d_slow[0], c->d_slow[1], n, c->d_sel_cnt, c->d_sel_tmp, c->stream);
			if (e != hipSuccess)
				return e;
			return prim_sort_keys(c->d_slow[1], c->d_slow[0], nslow, 32, (uint32_t)end_bit, c->d_sort_tmp, &sorted, c->stream);
		}));
		d.slow_keys = sorted;
		d.heads = (uint32_t*)(sorted == c->d_slow[0] ? c->d_slow[1] : c->d_slow[0]); // the sort's other buffer, free after it
		if (!c->d_hrec)
			HIP_TRY(hipMalloc(&c->d_hrec, (size_t)c->max_events * sizeof(uint4)));
		d.hrec = c->d_hrec;
		// LRU eviction possible?  Only if more sessions than its capacity could be live at once
		// (k_walk_lru's comment): first the cheap count of candidate sessions, then the bound.
		bool exact = false;
		if (dirty > c->carry_cap) {
			const uint64_t nb = (uint64_t)c->max_events;
			if (!c->d_lru_delta) {
				HIP_TRY(hipMalloc(&c->d_lru_delta, nb * sizeof(int)));
				HIP_TRY(hipMalloc(&c->d_lru_minus, nb));
				HIP_TRY(hipMalloc(&c->d_lru_scan, nb * sizeof(int)));
				c->lru_tmp_bytes = prim_scan_tmp_bytes(c->max_events, sizeof(int));
				HIP_TRY(hipMalloc(&c->d_lru_tmp, c->lru_tmp_bytes + 16));
			}
			HIP_TRY(hipMemsetAsync(c->d_lru_delta, 0, (size_t)n * sizeof(int), c->stream));
			HIP_TRY(hipMemsetAsync(c->d_lru_minus, 0, n, c->stream));
			size_t tb = c->lru_tmp_bytes;
			HIP_TRY(launch_lru_bound(d, (uint32_t)nslow, c->d_lru_delta, c->d_lru_minus, c->d_lru_scan, c->d_lru_tmp, tb, c->stream,
					c->cus));
			HIP_TRY(hipMemcpyAsync(c->h_ctr, c->d_ctr, CTR_COUNT * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
			HIP_TRY(hipStreamSynchronize(c->stream));
			const unsigned long long pk = c->h_ctr[CTR_LRU_PEAK];
			const long long peak = pk ? (long long)pk - (1ll << 31) : 0;
			exact = (long long)c->n_carry + peak > (long long)c->carry_cap;
		}
		int settled = 0;
		if (exact) {
			c->lru_batches_exact++;
			if (int rc = run_lru_rounds(c, d, (uint32_t)nslow, &settled))
				return rc;
		}
		if (exact && !settled) {
			c->lru_sequential++;
			if (!c->d_lru_jpos) {
				HIP_TRY(hipMalloc(&c->d_lru_jpos, (size_t)c->max_events * sizeof(uint32_t)));
				HIP_TRY(hipMalloc(&c->d_lru_head, (size_t)c->max_events * sizeof(uint32_t)));
				HIP_TRY(hipMalloc(&c->d_lru_sess, ((size_t)c->max_events + c->carry_cap) * sess_state_bytes()));
				HIP_TRY(hipMalloc(&c->d_lru_live, ((size_t)c->carry_cap + 1) * sizeof(uint32_t)));
			}
			HIP_TRY(hipMemsetAsync(c->d_lru_jpos, 0xff, (size_t)n * sizeof(uint32_t), c->stream));
			HIP_TRY(timed(c, KT_WALK, [&] {
				return launch_walk_lru(d, (uint32_t)nslow, c->d_lru_jpos, c->d_lru_head, (SessState*)c->d_lru_sess, c->d_lru_live,
						c->carry_cap, c->stream, c->cus);
			}));
		} else if (!exact) {
			HIP_TRY(timed(c, KT_WALK, [&] { return launch_walk(d, (uint32_t)nslow, c->stream, c->cus); }));
			if (c->n_carry)
				HIP_TRY(timed(c, KT_CARRY_PASS, [&] { return launch_carry_pass(d, c->stream); }));
		}
		HIP_TRY(timed(c, KT_EMIT, [&] { return launch_emit(d, c->stream, c->cus); }));
	}
	HIP_TRY(timed(c, KT_VERIFY, [&] { return launch_verify(d, c->stream, c->cus); }));
	if (dirty)
		HIP_TRY(timed(c, KT_SSET_CLEAR, [&] { return launch_sset_clear(d, c->stream, c->cus); }));
	if (nslow > 0) {
		HIP_TRY(hipMemcpyAsync(c->h_end, c->d_ctr, CTR_COUNT * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
		HIP_TRY(hipEventRecord(c->ev_end, c->stream));
		c->pending_end = 1;
	} else {
		c->last_sreq = c->last_sstr = 0;
	}
	HIP_TRY(hipEventRecord(c->ev_batch, c->stream));
	c->batch_valid = 1;
	c->seq_base += n;
	c->events_total += n;
	return 0;
}

int ebd_submit_batch_device(ebd_ctx* c, const ebd_device_batch* b) {
	if (!c || !b || (b->n && (!b->events || !b->len || !b->off || !b->payload)))
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	return run_batch(c, (const EventRec*)b->events, b->len, b->off, b->payload, b->payload_bytes, b->n);
}

int ebd_set_seq_base(ebd_ctx* c, uint64_t seq) {
	if (!c)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	c->seq_base = seq;
	return 0;
}

int ebd_kernel_times(ebd_ctx* c, ebd_kernel_time* out, uint32_t cap, uint32_t* n) {
	if (!c || !n)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	(void)hipSetDevice(c->device);
	drain_timing(c);
	*n = KT_N;
	if (!out)
		return 0;
	if (cap < (uint32_t)KT_N)
		return -ENOSPC;
	for (int k = 0; k < KT_N; k++) {
		std::memset(out[k].name, 0, sizeof(out[k].name));
		std::strncpy(out[k].name, kKernelNames[k], sizeof(out[k].name) - 1);
		out[k].launches = c->kt_n[k];
		out[k].total_ms = c->kt_ms[k];
	}
	return 0;
}

int ebd_reset_kernel_times(ebd_ctx* c) {
	if (!c)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	(void)hipSetDevice(c->device);
	drain_timing(c);
	for (int k = 0; k < 16; k++) {
		c->kt_ms[k] = 0;
		c->kt_n[k] = 0;
	}
	return 0;
}

int ebd_sync(ebd_ctx* c) {
	if (!c)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	HIP_TRY(hipSetDevice(c->device));
	HIP_TRY(hipStreamSynchronize(c->cstream));
	HIP_TRY(hipStreamSynchronize(c->stream));
	HIP_TRY(hipStreamSynchronize(c->dstream));
	c->res_pending = 0;
	return finish_pending(c);
}

// ---- ingest pipeline ---------------------------------------------------------------
// Discovery::fetchAndHandleEvents drains the BPF queue and copies every event's 8196-B saved
// buffer (Discovery.cpp:73-110).  Here a host batch is uploaded into one of two device
// staging slots on the copy stream while the compute stream works on the previous batch.
// Pinned sources (ebd_host_alloc, or hipHostRegister'ed) are DMAed directly; pageable ones go
// through two pinned bounce buffers, the CPU copy of one chunk overlapping the DMA of the other.
static constexpr size_t kBounce = 32ull << 20;

static bool host_pinned(const void* p) {
	hipPointerAttribute_t a;
	if (hipPointerGetAttributes(&a, p) != hipSuccess) {
		(void)hipGetLastError();
		return false;
	}
	return a.type == hipMemoryTypeHost;
}

// memcpy with up to 4 threads for large chunks (one core copies ~10 GB/s, below PCIe).
static void par_memcpy(void* dst, const void* src, size_t n) {
	constexpr size_t kPart = 4ull << 20;
	if (n < 2 * kPart) {
		std::memcpy(dst, src, n);
		return;
	}
	const int t = 4;
	const size_t part = (n + t - 1) / t;
	std::thread th[t - 1];
	for (int k = 1; k < t; k++) {
		const size_t a = k * part, z = std::min(n, a + part);
		th[k - 1] = std::thread([=] { std::memcpy((char*)dst + a, (const char*)src + a, z - a); });
	}
	std::memcpy(dst, src, std::min(n, part));
	for (auto& x : th)
		x.join();
}

static int upload(ebd_ctx* c, void* dst, const void* src, size_t bytes) {
	if (!bytes)
		return 0;
	if (host_pinned(src)) {
		HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->cstream));
		return 0;
	}
	for (int k = 0; k < 2; k++)
		if (!c->bounce[k])
			HIP_TRY(hipHostMalloc(&c->bounce[k], kBounce, hipHostMallocDefault));
	for (size_t o = 0; o < bytes; o += kBounce) {
		const size_t m = std::min(kBounce, bytes - o);
		const int b = c->bounce_next;
		c->bounce_next ^= 1;
		if (c->bounce_valid[b]) // its previous chunk has left for the device
			HIP_TRY(hipEventSynchronize(c->bounce_ev[b]));
		par_memcpy(c->bounce[b], (const char*)src + o, m);
		HIP_TRY(hipMemcpyAsync((char*)dst + o, c->bounce[b], m, hipMemcpyHostToDevice, c->cstream));
		HIP_TRY(hipEventRecord(c->bounce_ev[b], c->cstream));
		c->bounce_valid[b] = 1;
	}
	return 0;
}

static int validate_batch(const ebd_ctx* c, const ebd_discovery_event* events, const uint32_t* len, const uint64_t* off,
		const uint8_t* payload, uint64_t payload_bytes, uint32_t n) {
	if (n && (!events || !len || !off || (!payload && payload_bytes)))
		return -EINVAL;
	if (n > c->max_events)
		return -EINVAL;
	for (uint32_t i = 0; i < n; i++) // buffers must lie inside the arena
		if (len[i] != EBD_NO_BUFFER && (len[i] > EBD_BUFFER_MAX_DATA_SIZE || off[i] > payload_bytes || payload_bytes - off[i] < len[i]))
			return -EINVAL;
	return 0;
}

static int stage_locked(ebd_ctx* c, const ebd_discovery_event* events, const uint32_t* len, const uint64_t* off,
		const uint8_t* payload, uint64_t payload_bytes, uint32_t n, uint64_t* ticket) {
	HIP_TRY(hipSetDevice(c->device));
	// any slot not holding a staged batch (tickets may be submitted out of order), next_slot first
	int s = c->next_slot;
	if (c->stg[s].staged)
		s ^= 1;
	auto& g = c->stg[s];
	if (g.staged)
		return -EBUSY; // two batches are already staged and not submitted
	if (!g.ev) {
		HIP_TRY(hipMalloc(&g.ev, (size_t)c->max_events * sizeof(EventRec)));
		HIP_TRY(hipMalloc(&g.len, (size_t)c->max_events * sizeof(uint32_t)));
		HIP_TRY(hipMalloc(&g.off, (size_t)c->max_events * sizeof(uint64_t)));
	}
	const uint64_t need = payload_bytes + EBD_PAYLOAD_PAD;
	if (need > g.pay_cap) {
		if (g.payload) {
			if (g.used_valid)
				HIP_TRY(hipEventSynchronize(g.used));
			HIP_TRY(hipFree(g.payload));
		}
		g.pay_cap = need < c->cfg.max_payload ? c->cfg.max_payload : need;
		HIP_TRY(hipMalloc(&g.payload, g.pay_cap));
	}
	if (g.used_valid) // the batch that last read this slot must be done with it
		HIP_TRY(hipStreamWaitEvent(c->cstream, g.used, 0));
	if (int rc = upload(c, g.ev, events, (size_t)n * sizeof(EventRec)))
		return rc;
	if (int rc = upload(c, g.len, len, (size_t)n * sizeof(uint32_t)))
		return rc;
	if (int rc = upload(c, g.off, off, (size_t)n * sizeof(uint64_t)))
		return rc;
	if (int rc = upload(c, g.payload, payload, payload_bytes))
		return rc;
	HIP_TRY(hipEventRecord(g.up, c->cstream));
	c->next_slot = s ^ 1; // only once the slot is staged
	g.n = n;
	g.pay_bytes = payload_bytes;
	g.staged = 1;
	g.ticket = c->next_ticket++;
	*ticket = g.ticket;
	return 0;
}

static int submit_staged_locked(ebd_ctx* c, uint64_t ticket) {
	int s = -1;
	for (int k = 0; k < 2; k++)
		if (c->stg[k].staged && c->stg[k].ticket == ticket)
			s = k;
	if (s < 0)
		return -EINVAL;
	auto& g = c->stg[s];
	HIP_TRY(hipSetDevice(c->device));
	HIP_TRY(hipStreamWaitEvent(c->stream, g.up, 0)); // the device waits for the upload, not the host
	if (std::getenv("EBD_DEBUG_PTRS")) // fault triage: the device ranges a batch uses
		std::fprintf(stderr, "ebd: batch n=%u payload=[%p, +%llu) ev=%p len=%p off=%p res=%p keys=%p sset=%p carry=%p/%p\n", g.n,
				(void*)g.payload, (unsigned long long)g.pay_cap, (void*)g.ev, (void*)g.len, (void*)g.off, (void*)c->d_res,
				(void*)c->d_keys, (void*)c->d_sset, (void*)c->d_carry[0], (void*)c->d_carry[1]);
	g.staged = 0;
	const int rc = run_batch(c, g.ev, g.len, g.off, g.payload, g.pay_bytes, g.n);
	HIP_TRY(hipEventRecord(g.used, c->stream));
	g.used_valid = 1;
	return rc;
}

int ebd_stage_batch(ebd_ctx* c, const ebd_discovery_event* events, const uint32_t* len, const uint64_t* off,
		const uint8_t* payload, uint64_t payload_bytes, uint32_t n, uint64_t* ticket) {
	if (!c || !ticket)
		return -EINVAL;
	if (int rc = validate_batch(c, events, len, off, payload, payload_bytes, n))
		return rc;
	std::lock_guard<std::mutex> lk(c->mu);
	return stage_locked(c, events, len, off, payload, payload_bytes, n, ticket);
}

int ebd_submit_staged(ebd_ctx* c, uint64_t ticket) {
	if (!c)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	return submit_staged_locked(c, ticket);
}

int ebd_submit_batch(ebd_ctx* c, const ebd_discovery_event* events, const uint32_t* len, const uint64_t* off,
		const uint8_t* payload, uint64_t payload_bytes, uint32_t n) {
	if (!c)
		return -EINVAL;
	if (int rc = validate_batch(c, events, len, off, payload, payload_bytes, n))
		return rc;
	std::lock_guard<std::mutex> lk(c->mu);
	uint64_t t = 0;
	if (int rc = stage_locked(c, events, len, off, payload, payload_bytes, n, &t))
		return rc;
	if (int rc = submit_staged_locked(c, t))
		return rc;
	HIP_TRY(hipStreamSynchronize(c->stream));
	return finish_pending(c);
}

void* ebd_host_alloc(ebd_ctx* c, uint64_t bytes) {
	if (!c || !bytes)
		return nullptr;
	void* p = nullptr;
	if (hipSetDevice(c->device) != hipSuccess || hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
		(void)hipGetLastError();
		return nullptr;
	}
	return p;
}

int ebd_host_free(ebd_ctx* c, void* p) {
	if (!c)
		return -EINVAL;
	if (p)
		HIP_TRY(hipHostFree(p));
	return 0;
}

int ebd_fetch_results_async(ebd_ctx* c, ebd_event_result* out, uint32_t cap, uint32_t* n) {
	if (!c || !n || (cap && !out))
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	*n = c->last_n;
	if (!out)
		return 0; // size query
	if (cap < c->last_n)
		return -ENOSPC;
	HIP_TRY(hipSetDevice(c->device));
	if (!c->last_n)
		return 0;
	if (c->batch_valid)
		HIP_TRY(hipStreamWaitEvent(c->dstream, c->ev_batch, 0));
	HIP_TRY(hipMemcpyAsync(out, c->d_res, (size_t)c->last_n * sizeof(ebd_event_result), hipMemcpyDeviceToHost, c->dstream));
	HIP_TRY(hipEventRecord(c->ev_res, c->dstream));
	c->res_pending = 1;
	return 0;
}

// A read into memory the caller owns (pageable as a rule): the stream is drained first, then one
// blocking hipMemcpy, which returns only once the bytes are in the caller's buffer.  An async copy
// into pageable memory followed by hipStreamSynchronize is the pattern that returned a stale parser
// state from ebd_parse_streams: the runtime stages pageable copies itself,
// and the stream's completion does not cover the host-side end of that staging.
static hipError_t read_out(ebd_ctx* c, void* dst, const void* src, size_t bytes) {
	hipError_t e = hipStreamSynchronize(c->stream);
	if (e != hipSuccess || bytes == 0)
		return e;
	return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
}

int ebd_fetch_results(ebd_ctx* c, ebd_event_result* out, uint32_t cap, uint32_t* n) {
	if (!c || !n || (cap && !out))
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	*n = c->last_n;
	if (!out)
		return 0; // size query
	if (cap < c->last_n)
		return -ENOSPC;
	HIP_TRY(hipSetDevice(c->device));
	HIP_TRY(read_out(c, out, c->d_res, (size_t)c->last_n * sizeof(ebd_event_result)));
	return 0;
}

const ebd_event_result* ebd_results_device(ebd_ctx* c) { return c ? c->d_res : nullptr; }

int ebd_fetch_session_requests(ebd_ctx* c, ebd_session_request* out, uint32_t cap, uint32_t* n, char* strings,
		uint64_t strcap, uint64_t* strlen) {
	if (!c || !n || !strlen)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	if (int rc = finish_pending(c))
		return rc;
	*n = (uint32_t)c->last_sreq;
	*strlen = c->last_sstr < c->sstr_cap ? c->last_sstr : c->sstr_cap;
	if (!out)
		return 0;
	if (cap < *n || strcap < *strlen)
		return -ENOSPC;
	HIP_TRY(hipSetDevice(c->device));
	HIP_TRY(read_out(c, out, c->d_sreq, (size_t)*n * sizeof(SessReq)));
	if (strings)
		HIP_TRY(read_out(c, strings, c->d_sstr, *strlen));
	return 0;
}

int ebd_collect_services(ebd_ctx* c, ebd_service* out, uint32_t cap, uint32_t* n, char* strings, uint64_t strcap,
		uint64_t* strlen) {
	if (!c || !n || !strlen)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	HIP_TRY(hipSetDevice(c->device));
	HIP_TRY(hipMemcpyAsync(c->h_ctr, c->d_ctr, CTR_COUNT * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
	HIP_TRY(hipStreamSynchronize(c->stream));
	uint64_t used = c->h_ctr[CTR_SARENA];
	if (used > c->sarena_cap)
		used = c->sarena_cap;
	const uint64_t cnt = c->h_ctr[CTR_SERVICES];
	*strlen = used;
	*n = (uint32_t)cnt;
	if (!out)
		return 0;
	if (cnt > cap || (used && (!strings || used > strcap)))
		return -ENOSPC;
	if (cnt) {
		if (!c->d_collect)
			HIP_TRY(hipMalloc(&c->d_collect, (size_t)c->slot_cap * sizeof(ebd_service)));
		HIP_TRY(launch_collect(make_dev(c), c->d_collect, c->stream, c->cus));
		HIP_TRY(read_out(c, out, c->d_collect, cnt * sizeof(ebd_service)));
	}
	if (used)
		HIP_TRY(read_out(c, strings, c->d_sarena, used));
	HIP_TRY(hipStreamSynchronize(c->stream));
	return 0;
}

// The live network-map entries move into the other (zeroed) table and their v6 prefixes into the
// other (zeroed) dictionary, under the slots remap gives (nullptr: the same slots).  Erased
// entries and dictionary slots only they used are dropped (ebd_kernels.hip k_net_remap).
static int rebuild_nets(ebd_ctx* c, const uint32_t* remap) {
	const int nxt = c->net_cur ^ 1;
	HIP_TRY(hipMemsetAsync(c->d_nets[nxt], 0, (size_t)c->net_cap * sizeof(NetEnt), c->stream));
	HIP_TRY(hipMemsetAsync(c->d_v6d[nxt], 0, (size_t)c->v6d_cap * sizeof(unsigned long long), c->stream));
	HIP_TRY(hipMemsetAsync(c->d_ctr + CTR_NETS, 0, 2 * sizeof(unsigned long long), c->stream)); // CTR_NETS, CTR_V6D
	Dev dn = make_dev(c);
	dn.nets = c->d_nets[nxt];
	dn.v6d = c->d_v6d[nxt];
	HIP_TRY(launch_net_remap(dn, c->d_nets[c->net_cur], c->net_cap - 1, remap, c->d_v6d[c->net_cur], c->stream, c->cus));
	c->net_cur = nxt;
	return 0;
}

// Aggregator::clear with network counters (A:138-149): the services with a non-empty map
// survive, re-inserted into the emptied table with zeroed client counters; their map entries
// move to a fresh table under the new slots (ebd_kernels.hip k_keep_collect .. k_net_remap).
static int clear_keep_nets(ebd_ctx* c) {
	HIP_TRY(hipMemcpyAsync(c->h_ctr, c->d_ctr, CTR_COUNT * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
	HIP_TRY(hipStreamSynchronize(c->stream));
	const uint64_t nsvc = c->h_ctr[CTR_SERVICES], bytes = c->h_ctr[CTR_SARENA];
	if (nsvc > c->keep_cap) {
		if (c->d_keep)
			HIP_TRY(hipFree(c->d_keep));
		c->keep_cap = nsvc + nsvc / 2 + 1024;
		HIP_TRY(hipMalloc(&c->d_keep, c->keep_cap * sizeof(KeepRec)));
	}
	if (bytes + 64 > c->kbytes_cap) {
		if (c->d_kbytes)
			HIP_TRY(hipFree(c->d_kbytes));
		c->kbytes_cap = bytes + bytes / 2 + 4096;
		HIP_TRY(hipMalloc(&c->d_kbytes, c->kbytes_cap + 64)); // claim_publish reads 8 bytes past
	}
	if (!c->d_remap)
		HIP_TRY(hipMalloc(&c->d_remap, (size_t)c->slot_cap * sizeof(uint32_t)));
	HIP_TRY(hipMemsetAsync(c->d_remap, 0xff, (size_t)c->slot_cap * sizeof(uint32_t), c->stream));
	HIP_TRY(hipMemsetAsync(c->d_ctr + CTR_KEEP, 0, 2 * sizeof(unsigned long long), c->stream));
	Dev d = make_dev(c);
	HIP_TRY(launch_keep_collect(d, c->d_keep, c->d_kbytes, c->kbytes_cap, c->stream, c->cus));
	HIP_TRY(timed(c, KT_CLEAR, [&] { return launch_clear_used(c->d_new_slots, c->d_ctr, c->d_slots, c->slot_cap, c->stream, c->cus); }));
	HIP_TRY(hipMemsetAsync(c->d_ctr + CTR_SARENA, 0, sizeof(unsigned long long), c->stream));
	HIP_TRY(hipMemsetAsync(c->d_ctr + CTR_SERVICES, 0, sizeof(unsigned long long), c->stream));
	HIP_TRY(launch_keep_insert(d, c->d_keep, (const uint8_t*)c->d_kbytes, c->d_remap, c->stream, c->cus));
	return rebuild_nets(c, c->d_remap);
}

int ebd_clear(ebd_ctx* c) {
	if (!c)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	HIP_TRY(hipSetDevice(c->device));
	if (c->net_on)
		return clear_keep_nets(c);
	HIP_TRY(timed(c, KT_CLEAR, [&] { return launch_clear_used(c->d_new_slots, c->d_ctr, c->d_slots, c->slot_cap, c->stream, c->cus); }));
	HIP_TRY(hipMemsetAsync(c->d_ctr + CTR_SARENA, 0, sizeof(unsigned long long), c->stream));
	HIP_TRY(hipMemsetAsync(c->d_ctr + CTR_SERVICES, 0, sizeof(unsigned long long), c->stream));
	return 0;
}

int ebd_set_clock(ebd_ctx* c, uint64_t now_ns) {
	if (!c)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	c->clock_ns = now_ns;
	return 0;
}

int ebd_set_event_clock(ebd_ctx* c, const uint64_t* time_ns) {
	if (!c)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	c->ev_times = time_ns;
	return 0;
}

int ebd_network_counters_cleaning(ebd_ctx* c, uint64_t now_ns) {
	if (!c)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	if (!c->net_on)
		return 0; // every map is empty
	HIP_TRY(hipSetDevice(c->device));
	const uint64_t now = now_ns ? now_ns : ctx_now(c);
	HIP_TRY(launch_net_clean(make_dev(c), now, 3600ull * 1000000000ull, c->stream, c->cus)); // std::chrono::hours(1)
	// Erased entries keep their keys (a later request of the same prefix reuses them), so a
	// daemon that cleans but never clears would fill the table and the v6 dictionary with
	// dead keys: past half full, both are rebuilt from the live entries.
	HIP_TRY(hipMemcpyAsync(c->h_ctr, c->d_ctr, CTR_COUNT * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
	HIP_TRY(hipStreamSynchronize(c->stream));
	if (2 * c->h_ctr[CTR_NETS] > c->net_cap || 2 * c->h_ctr[CTR_V6D] > c->v6d_cap) {
		const int rc = rebuild_nets(c, nullptr);
		if (rc)
			return rc;
		HIP_TRY(hipStreamSynchronize(c->stream));
	}
	return 0;
}

int ebd_collect_networks(ebd_ctx* c, ebd_service_net* out, uint32_t cap, uint32_t* n) {
	if (!c || !n)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	*n = 0;
	if (!c->net_on)
		return 0;
	HIP_TRY(hipSetDevice(c->device));
	if (out && !c->d_netdump)
		HIP_TRY(hipMalloc(&c->d_netdump, (size_t)c->net_cap * sizeof(ebd_service_net)));
	HIP_TRY(hipMemsetAsync(c->d_cnt, 0, sizeof(unsigned long long), c->stream));
	// a size query (out null) only counts: k_net_dump writes nothing at cap 0
	HIP_TRY(launch_net_dump(make_dev(c), out ? c->d_netdump : nullptr, out ? c->net_cap : 0u, c->d_cnt, c->stream, c->cus));
	HIP_TRY(hipMemcpyAsync(c->h_ctr + CTR_COUNT, c->d_cnt, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
	HIP_TRY(hipStreamSynchronize(c->stream));
	const uint64_t cnt = c->h_ctr[CTR_COUNT];
	*n = (uint32_t)cnt;
	if (!out)
		return 0;
	if (cnt > cap)
		return -ENOSPC;
	if (cnt)
		HIP_TRY(hipMemcpy(out, c->d_netdump, cnt * sizeof(ebd_service_net), hipMemcpyDeviceToHost));
	return 0;
}

int ebd_collect_networks_device(ebd_ctx* c, ebd_service_net* out, uint32_t cap, uint32_t* n) {
	if (!c || !n)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	*n = 0;
	if (!c->net_on)
		return 0;
	HIP_TRY(hipSetDevice(c->device));
	HIP_TRY(hipMemsetAsync(c->d_cnt, 0, sizeof(unsigned long long), c->stream));
	// a size query (out null) only counts: k_net_dump writes nothing at cap 0
	HIP_TRY(launch_net_dump(make_dev(c), out, out ? cap : 0u, c->d_cnt, c->stream, c->cus));
	HIP_TRY(hipMemcpyAsync(c->h_ctr + CTR_COUNT, c->d_cnt, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
	HIP_TRY(hipStreamSynchronize(c->stream));
	const uint64_t cnt = c->h_ctr[CTR_COUNT];
	*n = (uint32_t)cnt;
	return out && cnt > cap ? -ENOSPC : 0;
}

int ebd_merge_networks_device(ebd_ctx* c, const ebd_service_net* recs, uint32_t n) {
	if (!c || (n && !recs))
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	if (n == 0)
		return 0;
	if (!c->net_on)
		return -EINVAL; // a context without network counters has no maps to merge into
	HIP_TRY(hipSetDevice(c->device));
	Dev d = make_dev(c);
	d.n = 0;
	HIP_TRY(launch_net_merge(d, recs, n, c->stream, c->cus));
	HIP_TRY(hipStreamSynchronize(c->stream));
	return 0;
}

int ebd_reset_services(ebd_ctx* c) {
	if (!c)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	HIP_TRY(hipSetDevice(c->device));
	HIP_TRY(timed(c, KT_CLEAR, [&] { return launch_clear_used(c->d_new_slots, c->d_ctr, c->d_slots, c->slot_cap, c->stream, c->cus); }));
	HIP_TRY(hipMemsetAsync(c->d_ctr + CTR_SARENA, 0, sizeof(unsigned long long), c->stream));
	HIP_TRY(hipMemsetAsync(c->d_ctr + CTR_SERVICES, 0, sizeof(unsigned long long), c->stream));
	if (c->net_on) {
		HIP_TRY(hipMemsetAsync(c->d_nets[c->net_cur], 0, (size_t)c->net_cap * sizeof(NetEnt), c->stream));
		HIP_TRY(hipMemsetAsync(c->d_v6d[c->net_cur], 0, (size_t)c->v6d_cap * sizeof(unsigned long long), c->stream));
		HIP_TRY(hipMemsetAsync(c->d_ctr + CTR_NETS, 0, 2 * sizeof(unsigned long long), c->stream)); // CTR_NETS, CTR_V6D
	}
	return 0;
}

int ebd_report_json(ebd_ctx* c, char* out, uint64_t cap, uint64_t* len) {
	if (!c || !len)
		return -EINVAL;
	uint32_t n = 0;
	uint64_t sl = 0;
	int rc = ebd_collect_services(c, nullptr, 0, &n, nullptr, 0, &sl);
	if (rc)
		return rc;
	std::vector<ebd_service> svc(n ? n : 1);
	std::vector<char> str(sl ? sl : 1);
	rc = ebd_collect_services(c, svc.data(), n, &n, str.data(), sl, &sl);
	if (rc)
		return rc;
	return ebd_format_services_json(svc.data(), n, str.data(), sl, out, cap, len);
}

// Room to verify every merged record: each may race a claim.
static int ensure_verify(ebd_ctx* c, uint32_t n) {
	if (n <= c->verify_cap)
		return 0;
	HIP_TRY(hipStreamSynchronize(c->stream));
	HIP_TRY(hipFree(c->d_verify));
	c->d_verify = nullptr;
	HIP_TRY(hipMalloc(&c->d_verify, (size_t)n * sizeof(VerifyRec)));
	c->verify_cap = n;
	return 0;
}

// Device scratch for one C-ABI call: pieces carved from the context's chunks in order, the
// carving restarting at every call (ScratchScope).  Every user runs on the context stream, so a
// call may reuse an earlier call's bytes in stream order; chunks are only added (a freed and
// re-allocated stream-ordered buffer had handed ebd_parse_streams a stale result now and then).
static hipError_t scratch_get(ebd_ctx* c, size_t bytes, void** out) {
	bytes = (bytes + 255) & ~(size_t)255;
	while (c->scr_ci < c->scr.size() && c->scr_off + bytes > c->scr[c->scr_ci].second) {
		c->scr_ci++;
		c->scr_off = 0;
	}
	if (c->scr_ci == c->scr.size()) {
		const size_t cap = std::max(bytes, c->scr.empty() ? (size_t)(1 << 20) : 2 * c->scr.back().second);
		uint8_t* p = nullptr;
		hipError_t e = hipMalloc((void**)&p, cap);
		if (e != hipSuccess)
			return e;
		c->scr.emplace_back(p, cap);
		c->scr_off = 0;
	}
	*out = c->scr[c->scr_ci].first + c->scr_off;
	c->scr_off += bytes;
	return hipSuccess;
}
struct ScratchScope {
	explicit ScratchScope(ebd_ctx* c) {
		c->scr_ci = 0;
		c->scr_off = 0;
	}
};

// offs = the exclusive scan of nb (n entries), its scratch from the call's scratch.
static hipError_t excl_scan(ebd_ctx* c, const unsigned long long* nb, unsigned long long* offs, uint32_t n) {
	void* tmp = nullptr;
	hipError_t e = scratch_get(c, prim_scan_tmp_bytes(n, sizeof(unsigned long long)), &tmp);
	return e != hipSuccess ? e : prim_scan_u64(nb, offs, n, 0, tmp, c->stream);
}

// The exclusive scan of each wire record's endpoint bytes (k_wire_bytes) into offs; nb and offs
// are n entries.
static hipError_t wire_offsets(ebd_ctx* c, const ebd_wire_service* recs, uint32_t n, unsigned long long* nb, unsigned long long* offs) {
	hipError_t e = launch_wire_bytes(recs, n, nullptr, nb, c->stream, c->cus);
	return e != hipSuccess ? e : excl_scan(c, nb, offs, n);
}

// A piece of the call's scratch (scratch_get); nothing to free.
struct AsyncBuf {
	ebd_ctx* c;
	void* p = nullptr;
	hipError_t alloc(size_t bytes) { return scratch_get(c, bytes, &p); }
	hipError_t release() { return hipSuccess; }
};

int ebd_export_services_device(ebd_ctx* c, uint32_t world, ebd_wire_service* recs, uint32_t cap, uint8_t* strings, uint64_t strcap,
		uint32_t* counts, uint64_t* str_counts) {
	if (!c || world == 0 || world > 64 || !counts || !str_counts)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	ScratchScope scope(c);
	HIP_TRY(hipSetDevice(c->device));
	if (!c->d_collect)
		HIP_TRY(hipMalloc(&c->d_collect, (size_t)c->slot_cap * sizeof(ebd_service)));
	AsyncBuf own_b{c}; // cnt, bytes, cur: world each
	HIP_TRY(own_b.alloc(3 * 64 * sizeof(unsigned long long)));
	unsigned long long* own = (unsigned long long*)own_b.p;
	HIP_TRY(hipMemsetAsync(own, 0, 2 * 64 * sizeof(unsigned long long), c->stream));
	HIP_TRY(launch_collect(make_dev(c), c->d_collect, c->stream, c->cus));
	HIP_TRY(launch_owner_count(c->d_collect, c->d_ctr, world, own, own + 64, c->stream, c->cus));
	unsigned long long h[3 * 64];
	HIP_TRY(hipMemcpyAsync(c->h_small, own, 2 * 64 * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
	HIP_TRY(hipStreamSynchronize(c->stream));
	std::memcpy(h, c->h_small, 2 * 64 * sizeof(unsigned long long));
	uint64_t total = 0, stotal = 0;
	for (uint32_t w = 0; w < world; w++) {
		counts[w] = (uint32_t)h[w];
		str_counts[w] = h[64 + w];
		h[128 + w] = total; // cur: the owner's first record
		total += h[w];
		stotal += h[64 + w];
	}
	int rc = 0;
	if (recs && total) {
		if (total > cap || stotal > strcap || !strings) {
			rc = -ENOSPC;
		} else {
			// records by owner, then their bytes at the scan of their sizes: owner w's bytes are
			// the str_counts[w] after the earlier owners', in its records' order
			AsyncBuf tmp_b{c}; // srcoff, nb, offs: total each
			HIP_TRY(tmp_b.alloc(3 * total * sizeof(unsigned long long)));
			unsigned long long* tmp = (unsigned long long*)tmp_b.p;
			HIP_TRY(hipMemcpyAsync(own + 128, h + 128, 64 * sizeof(unsigned long long), hipMemcpyHostToDevice, c->stream));
			HIP_TRY(launch_owner_scatter(c->d_collect, c->d_ctr, world, own + 128, recs, tmp, c->stream, c->cus));
			HIP_TRY(wire_offsets(c, recs, (uint32_t)total, tmp + total, tmp + 2 * total));
			HIP_TRY(launch_wire_copy(recs, (uint32_t)total, nullptr, tmp + 2 * total, tmp, c->d_sarena, strings, c->stream, c->cus));
			HIP_TRY(tmp_b.release());
		}
	}
	HIP_TRY(own_b.release());
	HIP_TRY(hipStreamSynchronize(c->stream));
	return rc;
}

int ebd_export_capacity(ebd_ctx* c, uint32_t* records, uint64_t* string_bytes) {
	if (!c || !records || !string_bytes)
		return -EINVAL;
	*records = c->slot_cap;
	*string_bytes = c->sarena_cap + 8;
	return 0;
}

int ebd_export_services_device_sized(ebd_ctx* c, uint32_t world, ebd_wire_service* recs, uint32_t cap, uint8_t* strings, uint64_t strcap,
		uint64_t* sizes) {
	if (!c || world == 0 || world > 64 || !recs || !strings || !sizes)
		return -EINVAL;
	if (cap < c->slot_cap || strcap < c->sarena_cap + 8)
		return -ENOSPC; // the buffers must hold every service the table can have (ebd_export_capacity)
	std::lock_guard<std::mutex> lk(c->mu);
	ScratchScope scope(c);
	HIP_TRY(hipSetDevice(c->device));
	if (!c->d_collect)
		HIP_TRY(hipMalloc(&c->d_collect, (size_t)c->slot_cap * sizeof(ebd_service)));
	AsyncBuf tmp_b{c}; // cur (64), then srcoff, nb, offs (cap each)
	HIP_TRY(tmp_b.alloc((64 + 3 * (size_t)cap) * sizeof(unsigned long long)));
	unsigned long long* cur = (unsigned long long*)tmp_b.p;
	unsigned long long* tmp = cur + 64;
	unsigned long long* sz = (unsigned long long*)sizes;
	const unsigned long long* nsvc = c->d_ctr + CTR_SERVICES; // the record count stays on the device
	HIP_TRY(hipMemsetAsync(sz, 0, 2 * 64 * sizeof(unsigned long long), c->stream));
	HIP_TRY(launch_collect(make_dev(c), c->d_collect, c->stream, c->cus));
	HIP_TRY(launch_owner_count(c->d_collect, c->d_ctr, world, sz, sz + 64, c->stream, c->cus));
	HIP_TRY(launch_owner_prefix(sz, world, cur, c->stream));
	HIP_TRY(launch_owner_scatter(c->d_collect, c->d_ctr, world, cur, recs, tmp, c->stream, c->cus));
	HIP_TRY(launch_wire_bytes(recs, cap, nsvc, tmp + cap, c->stream, c->cus));
	HIP_TRY(excl_scan(c, tmp + cap, tmp + 2 * (size_t)cap, cap));
	HIP_TRY(launch_wire_copy(recs, cap, nsvc, tmp + 2 * (size_t)cap, tmp, c->d_sarena, strings, c->stream, c->cus));
	HIP_TRY(hipStreamSynchronize(c->stream));
	return 0;
}

int ebd_wire_segment_bytes_device(ebd_ctx* c, const ebd_wire_service* recs, uint32_t n, const uint8_t* need, const uint64_t* dst,
		const uint64_t* seg_counts, uint32_t world, uint64_t* out) {
	if (!c || world == 0 || world > 64 || !seg_counts || !out || (n && (!recs || (!need == !dst))))
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	HIP_TRY(hipSetDevice(c->device));
	HIP_TRY(hipMemsetAsync(out, 0, (size_t)world * sizeof(uint64_t), c->stream));
	if (n)
		HIP_TRY(launch_wire_seg_bytes(recs, n, need, (const unsigned long long*)dst, (const unsigned long long*)seg_counts, world,
				(unsigned long long*)out, c->stream, c->cus));
	HIP_TRY(hipStreamSynchronize(c->stream));
	return 0;
}

int ebd_merge_services_device(ebd_ctx* c, const ebd_wire_service* recs, uint32_t n, const uint8_t* strings, uint64_t strlen) {
	if (!c || (n && (!recs || (!strings && strlen))))
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	ScratchScope scope(c);
	HIP_TRY(hipSetDevice(c->device));
	if (n == 0)
		return 0;
	int rc = ensure_verify(c, n);
	if (rc)
		return rc;
	Dev d = make_dev(c);
	d.n = 0;
	AsyncBuf tmp_b{c}; // nb, offs
	HIP_TRY(tmp_b.alloc(2 * (size_t)n * sizeof(unsigned long long)));
	unsigned long long* tmp = (unsigned long long*)tmp_b.p;
	HIP_TRY(wire_offsets(c, recs, n, tmp, tmp + n));
	HIP_TRY(hipMemsetAsync(c->d_ctr + CTR_VERIFY, 0, sizeof(unsigned long long), c->stream));
	HIP_TRY(launch_merge(d, recs, n, strings, strlen, tmp + n, c->stream, c->cus));
	HIP_TRY(launch_verify(d, c->stream, c->cus));
	HIP_TRY(tmp_b.release());
	HIP_TRY(hipStreamSynchronize(c->stream));
	return 0;
}

int ebd_merge_service_keys_device(ebd_ctx* c, const ebd_wire_service* recs, uint32_t n, uint64_t* dst) {
	if (!c || (n && (!recs || !dst)))
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	HIP_TRY(hipSetDevice(c->device));
	if (n == 0)
		return 0;
	int rc = ensure_verify(c, n);
	if (rc)
		return rc;
	Dev d = make_dev(c);
	d.n = 0;
	HIP_TRY(hipMemsetAsync(c->d_ctr + CTR_VERIFY, 0, sizeof(unsigned long long), c->stream));
	HIP_TRY(launch_merge_keys(d, recs, n, (unsigned long long*)dst, c->stream, c->cus));
	HIP_TRY(launch_verify(d, c->stream, c->cus));
	HIP_TRY(hipStreamSynchronize(c->stream));
	return 0;
}

int ebd_wire_compact_device(ebd_ctx* c, const ebd_wire_service* recs, uint32_t n, const uint8_t* strings, uint64_t strlen,
		const uint8_t* need, uint8_t* out, uint64_t outcap, uint64_t* out_len) {
	if (!c || (!out_len && (!out || outcap < strlen)) || (n && (!recs || !need || (!strings && strlen))))
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	ScratchScope scope(c);
	HIP_TRY(hipSetDevice(c->device));
	if (out_len)
		*out_len = 0;
	if (n == 0)
		return 0;
	AsyncBuf tmp_b{c}; // nb, soff, nbn, doff
	HIP_TRY(tmp_b.alloc(4 * (size_t)n * sizeof(unsigned long long)));
	unsigned long long* tmp = (unsigned long long*)tmp_b.p;
	HIP_TRY(wire_offsets(c, recs, n, tmp, tmp + n));
	HIP_TRY(launch_wire_bytes_needed(recs, n, need, nullptr, tmp + 2 * (size_t)n, c->stream, c->cus));
	HIP_TRY(excl_scan(c, tmp + 2 * (size_t)n, tmp + 3 * (size_t)n, n));
	if (!out_len) { // no size query: out holds all the strings, so it holds the needed ones
		HIP_TRY(launch_wire_compact(recs, n, need, tmp + n, tmp + 3 * (size_t)n, strings, strlen, out, outcap, c->d_ctr, c->stream, c->cus));
		HIP_TRY(hipStreamSynchronize(c->stream));
		return 0;
	}
	unsigned long long* last = c->h_small; // the last record's needed bytes and offset: the total
	HIP_TRY(hipMemcpyAsync(&last[0], tmp + 3 * (size_t)n - 1, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
	HIP_TRY(hipMemcpyAsync(&last[1], tmp + 4 * (size_t)n - 1, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
	HIP_TRY(hipStreamSynchronize(c->stream));
	const uint64_t total = last[0] + last[1];
	int rc = 0;
	if (out) {
		if (total > outcap)
			rc = -ENOSPC;
		else
			HIP_TRY(launch_wire_compact(recs, n, need, tmp + n, tmp + 3 * (size_t)n, strings, strlen, out, outcap, c->d_ctr, c->stream,
					c->cus));
	}
	HIP_TRY(tmp_b.release());
	HIP_TRY(hipStreamSynchronize(c->stream));
	*out_len = total;
	return rc;
}

int ebd_merge_service_bytes_device(ebd_ctx* c, const ebd_wire_service* recs, uint32_t n, const uint64_t* dst, const uint8_t* strings,
		uint64_t strlen) {
	if (!c || (n && (!recs || !dst || (!strings && strlen))))
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	ScratchScope scope(c);
	HIP_TRY(hipSetDevice(c->device));
	if (n == 0)
		return 0;
	Dev d = make_dev(c);
	d.n = 0;
	AsyncBuf tmp_b{c}; // nb, offs
	HIP_TRY(tmp_b.alloc(2 * (size_t)n * sizeof(unsigned long long)));
	unsigned long long* tmp = (unsigned long long*)tmp_b.p;
	HIP_TRY(launch_wire_bytes_needed(recs, n, nullptr, (const unsigned long long*)dst, tmp, c->stream, c->cus));
	HIP_TRY(excl_scan(c, tmp, tmp + n, n));
	HIP_TRY(launch_merge_bytes(d, recs, n, (const unsigned long long*)dst, tmp + n, strings, strlen, c->stream, c->cus));
	HIP_TRY(tmp_b.release());
	HIP_TRY(hipStreamSynchronize(c->stream));
	return 0;
}

int ebd_aggregate_requests(ebd_ctx* c, const ebd_request* reqs, uint32_t n, const char* strings, uint64_t strings_len) {
	if (!c || (n && (!reqs || (!strings && strings_len))))
		return -EINVAL;
	for (uint32_t k = 0; k < n; k++) { // the strings of every request inside the buffer
		const ebd_request& q = reqs[k];
		const uint64_t need = (uint64_t)q.host_len + q.url_len + (q.cip_len == EBD_NO_CLIENT_IP ? 0u : q.cip_len);
		if (q.host_len + q.url_len > EBD_MAX_HTTP_REQUEST_LENGTH ||
				(q.cip_len != EBD_NO_CLIENT_IP && q.cip_len > EBD_MAX_HTTP_REQUEST_LENGTH) || q.str_off > strings_len ||
				need > strings_len - q.str_off)
			return -EINVAL;
	}
	std::lock_guard<std::mutex> lk(c->mu);
	ScratchScope scope(c);
	HIP_TRY(hipSetDevice(c->device));
	if (int rc = finish_pending(c))
		return rc;
	if (n == 0)
		return 0;
	Dev d = make_dev(c);
	d.n = 0;
	d.now = ctx_now(c);
	ebd_request* drq = nullptr;
	uint8_t* dstr = nullptr; // 16 bytes of slack: the key reads 8-byte pieces
	HIP_TRY(scratch_get(c, (size_t)n * sizeof(ebd_request), (void**)&drq));
	HIP_TRY(scratch_get(c, (size_t)strings_len + 16, (void**)&dstr));
	hipError_t e = hipMemcpyAsync(drq, reqs, (size_t)n * sizeof(ebd_request), hipMemcpyHostToDevice, c->stream);
	if (e == hipSuccess && strings_len)
		e = hipMemcpyAsync(dstr, strings, (size_t)strings_len, hipMemcpyHostToDevice, c->stream);
	if (e == hipSuccess)
		e = hipMemsetAsync(dstr + strings_len, 0, 16, c->stream);
	if (e == hipSuccess)
		e = hipMemsetAsync(c->d_ctr + CTR_VERIFY, 0, sizeof(unsigned long long), c->stream);
	if (e == hipSuccess)
		e = launch_agg_requests(d, drq, n, dstr, c->stream, c->cus);
	if (e == hipSuccess)
		e = launch_verify(d, c->stream, c->cus);
	HIP_TRY(e);
	HIP_TRY(hipStreamSynchronize(c->stream));
	c->seq_base += n;
	return 0;
}

int ebd_get_stats(ebd_ctx* c, ebd_stats* s) {
	if (!c || !s)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	HIP_TRY(hipSetDevice(c->device));
	if (int rc = finish_pending(c))
		return rc;
	HIP_TRY(hipMemcpyAsync(c->h_ctr, c->d_ctr, CTR_COUNT * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
	HIP_TRY(hipStreamSynchronize(c->stream));
	std::memset(s, 0, sizeof(*s));
	s->events = c->events_total;
	s->requests = c->h_ctr[CTR_REQUESTS];
	s->session_events = c->h_ctr[CTR_SESSION_EVENTS];
	s->kernel_deletes = c->h_ctr[CTR_KDELETES];
	s->live_sessions = c->n_carry;
	s->max_live_sessions = c->max_live;
	s->hash_collisions = c->h_ctr[CTR_COLLISIONS];
	s->lru_evictions = c->h_ctr[CTR_EVICTIONS_TOTAL];
	s->lru_exact_batches = c->lru_batches_exact;
	s->lru_rounds = c->lru_rounds;
	s->lru_sequential = c->lru_sequential;
	s->services = c->h_ctr[CTR_SERVICES];
	s->errors = c->h_ctr[CTR_ERRORS];
	return 0;
}

// --------------------------------------------------------------------------------------
// synthetic traces
// --------------------------------------------------------------------------------------
static std::mutex g_tables_mu;
static GenTables* g_tables = nullptr;
static const GenTables* host_tables() {
	std::lock_guard<std::mutex> lk(g_tables_mu);
	if (!g_tables) {
		g_tables = new GenTables();
		build_gen_tables(g_tables);
	}
	return g_tables;
}

static bool single_config(uint32_t cfg) { return cfg == 1 || cfg == 11 || cfg == 2 || cfg == 3 || cfg == 5; }
static bool trace_ok(const ebd_trace_config* t) {
	if (t && t->config == 4) // a whole trace from position 0, unsharded (its connections interleave)
		return t->first == 0 && t->shard_count <= 1 && !(t->align & (t->align - 1));
	return t && single_config(t->config) && !(t->align & (t->align - 1)) && (t->shard_count <= 1 || t->shard_index < t->shard_count);
}

// Config 4 (ebd_gen.h): connections per slot that cover ceil(n / kSlots4) rounds (>= 3 events each).
static uint32_t gen4_J(uint64_t n) { return (uint32_t)(((n + kSlots4 - 1) / kSlots4) / 3 + 2); }

// Config 4 on the host: the device passes in order (per-slot first rounds, piece lengths,
// offsets, bytes).  ev == nullptr: sizes only.
static int gen4_host(const ebd_trace_config* t, EventRec* ev, uint32_t* len, uint64_t* off, uint8_t* payload, uint64_t cap,
		uint64_t* gidx, uint64_t* total_out) {
	const GenTables* T = host_tables();
	const uint64_t n = t->n;
	const uint32_t a = t->align ? t->align : 1, J = gen4_J(n);
	std::vector<uint32_t> r0((size_t)kSlots4 * J);
	for (uint32_t slot = 0; slot < kSlots4; slot++) {
		uint32_t acc = 0;
		for (uint32_t j = 0; j < J; j++) {
			Conn4 c;
			conn4(t->seed, (uint64_t)j * kSlots4 + slot, c);
			r0[(size_t)slot * J + j] = acc;
			acc += conn4_events(c);
		}
	}
	std::vector<uint64_t> boff(n + 1, 0);
	for (uint32_t slot = 0; slot < kSlots4; slot++)
		for (uint32_t j = 0; j < J; j++)
			conn4_visit(*T, t->seed, slot, j, r0[(size_t)slot * J + j], n, [&](uint64_t p0, const Conn4&, const Req4* r, uint32_t) {
				if (!r)
					return;
				for (uint32_t f = 0; f < r->k && p0 + (uint64_t)f * kSlots4 < n; f++)
					boff[p0 + (uint64_t)f * kSlots4] = align_up(r->cut[f + 1] - r->cut[f], a);
			});
	uint64_t acc = 0;
	for (uint64_t p = 0; p <= n; p++) {
		const uint64_t x = boff[p];
		boff[p] = acc;
		acc += x;
	}
	*total_out = boff[n];
	if (!ev)
		return 0;
	if (boff[n] > cap)
		return -ENOSPC;
	for (uint32_t slot = 0; slot < kSlots4; slot++)
		for (uint32_t j = 0; j < J; j++)
			conn4_visit(*T, t->seed, slot, j, r0[(size_t)slot * J + j], n, [&](uint64_t p0, const Conn4& c, const Req4* r, uint32_t e) {
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
	return 0;
}
// config 5 is config 3's distribution, sharded by connection
static uint32_t gen_config(uint32_t c) { return c == 5 ? 3 : c; }

int ebd_trace_size(const ebd_trace_config* t, uint32_t* n_events, uint64_t* payload_bytes) {
	if (!trace_ok(t) || !payload_bytes)
		return -EINVAL;
	if (t->config == 4) {
		if (n_events)
			*n_events = t->n;
		return gen4_host(t, nullptr, nullptr, nullptr, nullptr, 0, nullptr, payload_bytes);
	}
	const GenTables* T = host_tables();
	const uint32_t a = t->align ? t->align : 1;
	uint64_t total = 0;
	uint32_t kept = 0;
	for (uint32_t i = 0; i < t->n; i++) {
		const uint32_t L = gen_single_shard(T, gen_config(t->config), t->seed, t->first + i, t->shard_count, t->shard_index,
				nullptr, nullptr);
		if (L || t->shard_count <= 1) {
			total += align_up(L, a);
			kept++;
		}
	}
	*payload_bytes = total;
	if (n_events)
		*n_events = kept;
	return 0;
}

int ebd_trace_generate_host(const ebd_trace_config* t, ebd_discovery_event* events, uint32_t* len, uint64_t* off,
		uint8_t* payload, uint64_t payload_cap, uint64_t* gidx) {
	if (!trace_ok(t) || (t->n && (!events || !len || !off || !payload)))
		return -EINVAL;
	if (t->config == 4) {
		uint64_t total = 0;
		return gen4_host(t, (EventRec*)events, len, off, payload, payload_cap, gidx, &total);
	}
	const GenTables* T = host_tables();
	const uint32_t a = t->align ? t->align : 1;
	uint64_t at = 0;
	uint32_t k = 0;
	for (uint32_t i = 0; i < t->n; i++) {
		const uint32_t L = gen_single_shard(T, gen_config(t->config), t->seed, t->first + i, t->shard_count, t->shard_index,
				nullptr, nullptr);
		if (!L && t->shard_count > 1)
			continue;
		if (at + L > payload_cap)
			return -ENOSPC;
		EventRec e;
		gen_single(T, gen_config(t->config), t->seed, t->first + i, &e, payload + at);
		std::memcpy(&events[k], &e, sizeof(e));
		len[k] = L;
		off[k] = at;
		if (gidx)
			gidx[k] = t->first + i;
		k++;
		at = align_up(at + L, a);
	}
	return 0;
}

static int ensure_gen_tables(ebd_ctx* c) {
	if (!c->d_gen) {
		HIP_TRY(hipMalloc(&c->d_gen, sizeof(GenTables)));
		HIP_TRY(hipMemcpy(c->d_gen, host_tables(), sizeof(GenTables), hipMemcpyHostToDevice));
	}
	return 0;
}

// Both device passes share the length pass and its scans; `out` == nullptr: sizes only.
struct GenOut {
	EventRec* ev;
	uint32_t* len;
	uint64_t* off;
	uint8_t* payload;
	uint64_t cap;
	uint64_t* gidx;
};

static int trace_device4(ebd_ctx* c, const ebd_trace_config* t, const GenOut* out, uint32_t* n_events, uint64_t* bytes) {
	const uint64_t n = t->n;
	const uint32_t a = t->align ? t->align : 1, J = gen4_J(n);
	const uint64_t tasks = (uint64_t)kSlots4 * J;
	ScratchScope scope(c);
	uint32_t *cnt = nullptr, *st = nullptr;
	unsigned long long *alen = nullptr, *boff = nullptr;
	HIP_TRY(scratch_get(c, tasks * 4 + 4, (void**)&cnt));
	HIP_TRY(scratch_get(c, tasks * 4 + 4, (void**)&st));
	HIP_TRY(scratch_get(c, n * 8 + 8, (void**)&alen));
	HIP_TRY(scratch_get(c, n * 8 + 8, (void**)&boff));
	HIP_TRY(launch_gen4_count(t->seed, J, cnt, c->stream));
	const size_t b1 = prim_scan_tmp_bytes(tasks, 4), b2 = prim_scan_tmp_bytes(n + 1, 8);
	void* tmp = nullptr;
	HIP_TRY(scratch_get(c, (b1 > b2 ? b1 : b2) + 16, &tmp));
	HIP_TRY(prim_scan_u32(cnt, st, tasks, 0, tmp, c->stream)); // wraps mod 2^32: differences stay exact
	HIP_TRY(hipMemsetAsync(alen, 0, n * 8 + 8, c->stream));
	HIP_TRY(launch_gen4_len(c->d_gen, t->seed, J, n, a, st, alen, c->stream));
	HIP_TRY(prim_scan_u64(alen, boff, n + 1, 0, tmp, c->stream));
	HIP_TRY(hipMemcpyAsync(c->h_small, boff + n, 8, hipMemcpyDeviceToHost, c->stream));
	HIP_TRY(hipStreamSynchronize(c->stream));
	const unsigned long long total = c->h_small[0];
	int rc = 0;
	if (out) {
		if (total > out->cap)
			rc = -ENOSPC;
		else
			HIP_TRY(launch_gen4_write(c->d_gen, t->seed, J, n, st, boff, out->ev, out->len, (unsigned long long*)out->off,
					out->payload, (unsigned long long*)out->gidx, c->stream));
	}
	HIP_TRY(hipStreamSynchronize(c->stream)); // the scratch is the next call's
	if (n_events)
		*n_events = (uint32_t)n;
	if (bytes)
		*bytes = total;
	return rc;
}

static int trace_device(ebd_ctx* c, const ebd_trace_config* t, const GenOut* out, uint32_t* n_events, uint64_t* bytes) {
	HIP_TRY(hipSetDevice(c->device));
	int rc = ensure_gen_tables(c);
	if (rc)
		return rc;
	if (t->config == 4)
		return trace_device4(c, t, out, n_events, bytes);
	const uint32_t n = t->n, a = t->align ? t->align : 1, cfg = gen_config(t->config);
	ScratchScope scope(c);
	unsigned long long *alen = nullptr, *boff = nullptr;
	uint32_t *keep = nullptr, *pos = nullptr;
	HIP_TRY(scratch_get(c, (size_t)n * 8 + 8, (void**)&alen));
	HIP_TRY(scratch_get(c, (size_t)n * 8 + 8, (void**)&boff));
	HIP_TRY(scratch_get(c, (size_t)n * 4 + 4, (void**)&keep));
	HIP_TRY(scratch_get(c, (size_t)n * 4 + 4, (void**)&pos));
	HIP_TRY(launch_gen_len(c->d_gen, cfg, t->seed, t->first, n, a, t->shard_count, t->shard_index, alen, keep, c->stream));
	if (t->shard_count <= 1) // every candidate is kept (a kept event may be empty only here)
		HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)keep, 1, n, c->stream));
	const size_t b1 = prim_scan_tmp_bytes((unsigned long long)n + 1, 8);
	void* tmp = nullptr;
	HIP_TRY(scratch_get(c, b1 + 16, &tmp));
	// the (n+1)-th entries become the totals
	HIP_TRY(hipMemsetAsync(alen + n, 0, 8, c->stream));
	HIP_TRY(hipMemsetAsync(keep + n, 0, 4, c->stream));
	HIP_TRY(prim_scan_u64(alen, boff, (unsigned long long)n + 1, 0, tmp, c->stream));
	HIP_TRY(prim_scan_u32(keep, pos, (unsigned long long)n + 1, 0, tmp, c->stream));
	HIP_TRY(hipMemcpyAsync(c->h_small, boff + n, 8, hipMemcpyDeviceToHost, c->stream));
	HIP_TRY(hipMemcpyAsync(c->h_small + 1, pos + n, 4, hipMemcpyDeviceToHost, c->stream));
	HIP_TRY(hipStreamSynchronize(c->stream));
	const unsigned long long total = c->h_small[0];
	const uint32_t kept = (uint32_t)c->h_small[1];
	rc = 0;
	if (out) {
		if (total > out->cap)
			rc = -ENOSPC;
		else
			HIP_TRY(launch_gen_write(c->d_gen, cfg, t->seed, t->first, n, keep, pos, boff, out->ev, out->len,
					(unsigned long long*)out->off, out->payload, (unsigned long long*)out->gidx, c->stream));
	}
	HIP_TRY(hipStreamSynchronize(c->stream)); // the scratch is the next call's
	if (n_events)
		*n_events = kept;
	if (bytes)
		*bytes = total;
	return rc;
}

int ebd_trace_size_device(ebd_ctx* c, const ebd_trace_config* t, uint32_t* n_events, uint64_t* payload_bytes) {
	if (!c || !trace_ok(t) || !payload_bytes || t->n == 0)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	return trace_device(c, t, nullptr, n_events, payload_bytes);
}

int ebd_trace_generate_device(ebd_ctx* c, const ebd_trace_config* t, ebd_discovery_event* events, uint32_t* len, uint64_t* off,
		uint8_t* payload, uint64_t payload_cap, uint64_t* gidx) {
	if (!c || !trace_ok(t) || t->n == 0 || !events || !len || !off || !payload)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	const GenOut o{(EventRec*)events, len, off, payload, payload_cap, gidx};
	return trace_device(c, t, &o, nullptr, nullptr);
}

// --------------------------------------------------------------------------------------
// host-side hooks for CPU tests of the shared semantics (no GPU needed)
// --------------------------------------------------------------------------------------
int ebd_host_dfa_info(uint32_t* info, uint32_t n) {
	static KeyTrie trie;
	static DfaTable* t = nullptr;
	if (!t) {
		build_key_trie(&trie);
		t = new DfaTable();
		if (build_dfa(&trie, t) != 0)
			return -EIO;
	}
	const uint32_t v[13] = {t->info.nstates, t->info.url_id, t->info.g2, t->info.g3, t->info.g4, t->info.hvc0, t->info.hvh,
			t->info.fin0, t->info.fin1, t->info.inv, t->info.init, t->info.vl0, t->info.vl1};
	(void)t->info.hvc1;
	for (uint32_t k = 0; k < n && k < 13; k++)
		info[k] = v[k];
	return 0;
}

static const DfaTable* host_dfa(const KeyTrie** trie_out);

int ebd_host_dfa_next(uint8_t* out, uint32_t cap) {
	const KeyTrie* trie;
	const DfaTable* t = host_dfa(&trie);
	if (!t || !out || cap < 256u * 256u)
		return -EINVAL;
	std::memcpy(out, t->next, 256u * 256u);
	return (int)t->info.nstates;
}

static const DfaTable* host_dfa(const KeyTrie** trie_out) {
	static KeyTrie trie;
	static DfaTable* t = nullptr;
	static std::mutex mu;
	std::lock_guard<std::mutex> lk(mu);
	if (!t) {
		build_key_trie(&trie);
		DfaTable* x = new DfaTable();
		if (build_dfa(&trie, x) != 0) {
			delete x;
			return nullptr;
		}
		t = x;
	}
	*trie_out = &trie;
	return t;
}

static void fill_ifs(Interfaces& ifs, const ebd_ipv4_network* v4, uint32_t n4, const ebd_ipv6_network* v6, uint32_t n6) {
	std::memset(&ifs, 0, sizeof(ifs));
	ifs.n4 = n4 > 64 ? 64 : n4;
	ifs.n6 = n6 > 32 ? 32 : n6;
	for (uint32_t i = 0; i < ifs.n4; i++) {
		std::memcpy(ifs.v4[i], v4[i].addr, 4);
		std::memcpy(ifs.v4[i] + 4, v4[i].mask, 4);
	}
	for (uint32_t i = 0; i < ifs.n6; i++) {
		std::memcpy(ifs.v6[i], v6[i].addr, 16);
		std::memcpy(ifs.v6[i] + 16, v6[i].mask, 16);
	}
}

struct HostTab {
	const uint8_t* t;
	uint32_t operator[](uint32_t i) const { return t[i]; }
};

// Bytes past a buffer as the host emulation sees them.  The device reads whatever follows
// the buffer; "\r\n" repeated is the most hostile filler (it can complete a request), so
// the host twin uses it to show that nothing past L leaks into a result.
struct HostPast {
	uint32_t operator()(uint32_t k) const { return (k & 1) ? '\n' : '\r'; }
};

// fresh_finalize's buffer access on the host (bytes past the buffer: HostPast).
struct HostMem {
	const uint8_t* p;
	uint32_t L;
	uint32_t at(uint32_t o) const { return o < L ? p[o] : HostPast{}(o - L); }
	uint32_t ld4(uint32_t o) const {
		uint32_t v = 0;
		for (uint32_t b = 0; b < 4; b++)
			v |= at(o + b) << (8 * b);
		return v;
	}
	unsigned long long ld8(uint32_t o) const {
		unsigned long long v = 0;
		for (uint32_t b = 0; b < 8; b++)
			v |= (unsigned long long)at(o + b) << (8 * b);
		return v;
	}
};

int ebd_host_fresh(const uint8_t* buf, uint32_t len, uint32_t pid, uint8_t flags, const uint8_t* src16,
		const ebd_ipv4_network* v4, uint32_t n4, const ebd_ipv6_network* v6, uint32_t n6, const uint64_t hash_key[2],
		ebd_event_result* out, uint64_t key[2]) {
	const KeyTrie* trie;
	const DfaTable* t = host_dfa(&trie);
	if (!t || !out || !hash_key || (len && !buf) || len > EBD_BUFFER_MAX_DATA_SIZE)
		return -EINVAL;
	static Interfaces ifs;
	fill_ifs(ifs, v4, n4, v6, n6);
	ScanRec sr;
	const uint32_t s = fresh_scan_host(HostTab{t->next}, t->info, buf, len, HostPast{}, sr);
	FreshResult fr;
	std::memset(&fr, 0, sizeof(fr));
	uint8_t zero[16] = {0};
	const bool post = len > 0 && buf[0] == 'P';
	fresh_finalize(HostTab{t->next}, t->info, sr, s, post, HostMem{buf, len}, len, HashKey{hash_key[0], hash_key[1]}, pid, flags, fr);
	if (fr.r.status == EBD_STATUS_FINISHED && !fr.cip) // what k_agg_fast does for this event
		fr.r.info = (uint8_t)(fr.r.info | (classify_source(ifs, flags, src16 ? src16 : zero) << EBD_INFO_CLASS_SHIFT));
	if (fr.cip) { // what k_agg_fast (cip_classify) does for this event
		uint32_t tb, te;
		uint8_t cls;
		cip_token(ifs, [buf](uint32_t b) { return (uint32_t)buf[b]; }, fr.r.u.span.cip_off, fr.r.consumed, &tb, &te, &cls);
		fr.r.u.span.cip_off = (uint16_t)tb;
		fr.r.u.span.cip_len = (uint16_t)(te - tb);
		fr.r.info = (uint8_t)(fr.r.info | (cls << EBD_INFO_CLASS_SHIFT));
	}
	*out = fr.r;
	if (key) {
		key[0] = fr.key.lo;
		key[1] = fr.key.hi;
	}
	return 0;
}

// scan_event's source on the host: the buffer at byte `shift` of a tile whose other bytes
// are "\r\n" filler (the most hostile bytes to find past a buffer: they can end a request),
// with the tile's piece bitmap computed as k_fresh's wave computes it.
struct HostTile {
	std::vector<uint8_t> t;
	std::vector<unsigned long long> nv;
	std::vector<uint16_t> cm[CB_N];
	uint8_t nc[256];
	uint32_t byte(uint32_t p) const { return t[p]; }
	uint32_t dw(uint32_t p) const {
		uint32_t v = 0;
		for (uint32_t b = 0; b < 4; b++)
			v |= (uint32_t)t[p + b] << (8 * b);
		return v;
	}
	unsigned long long ld8(uint32_t p) const { return (unsigned long long)dw(p) | ((unsigned long long)dw(p + 4) << 32); }
	void piece(uint32_t pc, uint32_t (&w)[4]) const {
		for (uint32_t k = 0; k < 4; k++)
			w[k] = dw(16 * pc + 4 * k);
	}
	unsigned long long nvword(uint32_t j) const { return nv[j]; }
	uint32_t ncls(uint32_t b) const { return nc[b & 0xffu]; }
	unsigned long long clsword(uint32_t c, uint32_t a) const {
		unsigned long long v = 0;
		for (uint32_t k = 0; k < 4; k++)
			v |= (unsigned long long)(4 * a + k < cm[c].size() ? cm[c][4 * a + k] : 0xffffu) << (16 * k);
		return v;
	}
};

int ebd_host_scan(const uint8_t* buf, uint32_t len, uint32_t shift, uint32_t pid, uint8_t flags, const uint8_t* src16,
		const ebd_ipv4_network* v4, uint32_t n4, const ebd_ipv6_network* v6, uint32_t n6, const uint64_t hash_key[2],
		ebd_event_result* out, uint64_t key[2]) {
	const KeyTrie* trie;
	if (!host_dfa(&trie) || !out || !hash_key || (len && !buf) || len > EBD_BUFFER_MAX_DATA_SIZE || shift > 15)
		return -EINVAL;
	static Interfaces ifs;
	fill_ifs(ifs, v4, n4, v6, n6);
	HostTile s;
	const uint32_t pieces = (shift + len + 15) / 16 + 4;
	s.t.assign(16 * pieces, 0);
	for (uint32_t k = 0; k < s.t.size(); k++)
		s.t[k] = (k & 1) ? '\n' : '\r';
	if (len)
		std::memcpy(s.t.data() + shift, buf, len);
	for (uint32_t b = 0; b < 256; b++)
		s.nc[b] = (uint8_t)(~trie->cls[b] & 0x1fu);
	s.nv.assign((pieces + 63) / 64, 0ull);
	for (uint32_t c = 0; c < CB_N; c++)
		s.cm[c].assign(pieces, 0);
	for (uint32_t pc = 0; pc < pieces; pc++) {
		uint32_t w[4], m[CB_N];
		s.piece(pc, w);
		if (nv4(w[0]) | nv4(w[1]) | nv4(w[2]) | nv4(w[3]))
			s.nv[pc >> 6] |= 1ull << (pc & 63);
		piece_classes(s, w, m);
		for (uint32_t c = 0; c < CB_N; c++)
			s.cm[c][pc] = (uint16_t)m[c];
	}
	ScanOut o;
	int path = 0; // 0: request line + line records (scan_fold), 2: scan_event, 1: the generic parser
	// as k_fresh runs them: every LF of the tile starts a line, each line parsed on its own
	const ReqOut rq = scan_reqline(s, shift, len);
	std::vector<uint32_t> starts;
	std::vector<LineRec> recs;
	for (uint32_t p = 0; p < s.t.size(); p++)
		if (s.t[p] == '\n' && p + 1 < s.t.size()) {
			starts.push_back(p + 1);
			recs.push_back(scan_line(s, p + 1, shift + len));
		}
	uint32_t l0 = (uint32_t)starts.size();
	for (uint32_t l = 0; l < starts.size(); l++)
		if (starts[l] == rq.q)
			l0 = l;
	auto lines = [&](uint32_t l) { return l < recs.size() ? recs[l] : LineRec{LN_SLOW, 0}; };
	if (!scan_fold(rq, lines, l0, (uint32_t)starts.size(), shift, len, o)) {
		path = 2;
		scan_event(s, shift, len, o);
		if (o.slow) {
			path = 1;
			scan_slow(s, trie, shift, len, o);
		}
	}
	ebd_event_result r = scan_result(o, flags);
	Hash128 h{0, 0};
	if (r.status == EBD_STATUS_FINISHED) {
		const auto& sp = r.u.span;
		h = endpoint_key<2>(HashKey{hash_key[0], hash_key[1]}, pid, sp.host_off, sp.host_len, sp.url_off, sp.url_len,
				[&](uint32_t o8) { return s.ld8(shift + o8); });
		uint8_t zero[16] = {0};
		if (!(r.info & EBD_INFO_CIP)) { // what k_fresh does for this event
			r.info = (uint8_t)(r.info | (classify_source(ifs, flags, src16 ? src16 : zero) << EBD_INFO_CLASS_SHIFT));
		} else { // what k_agg_fast (cip_classify) does for this event
			uint32_t tb, te;
			uint8_t cls;
			cip_token(ifs, [buf](uint32_t b) { return (uint32_t)buf[b]; }, r.u.span.cip_off, r.consumed, &tb, &te, &cls);
			r.u.span.cip_off = (uint16_t)tb;
			r.u.span.cip_len = (uint16_t)(te - tb);
			r.info = (uint8_t)(r.info | (cls << EBD_INFO_CLASS_SHIFT));
		}
	}
	*out = r;
	if (key) {
		key[0] = h.lo;
		key[1] = h.hi;
	}
	return path;
}

int ebd_host_gp_parse(const uint8_t* data, const uint32_t* chunk_len, uint32_t nchunks, uint8_t flags, int reset_between,
		uint32_t* consumed, uint32_t* out8) {
	const KeyTrie* trie;
	if (!host_dfa(&trie) || !consumed || !out8)
		return -EINVAL;
	GenParser g;
	gp_init(g);
	uint64_t at = 0;
	for (uint32_t k = 0; k < nchunks; k++) {
		const uint8_t* p = data + at;
		consumed[k] = gp_parse(g, trie, [p](uint32_t i) { return (uint32_t)p[i]; }, chunk_len[k], flags);
		at += chunk_len[k];
		if (reset_between && gp_done(g) && k + 1 < nchunks)
			gp_reset(g);
	}
	const uint32_t v[12] = {g.state, g.url_start, g.url_len, (g.f & GPF_HOST) ? g.host_start : 0,
			(g.f & GPF_HOST) ? g.host_len : 0, g.cip_start, g.cip_len, g.f, g.cipkey, g.mcand, g.mlen,
			(uint32_t)g.plen | ((uint32_t)g.pminor << 8)};
	for (int k = 0; k < 12; k++)
		out8[k] = v[k];
	return 0;
}

// The session path's DFA walker (dfa_parse) over the same chunks: out8 as ebd_host_gp_parse's
// (method and protocol prefix lengths are not kept by the walker: 0).
int ebd_host_dfa_parse(const uint8_t* data, const uint32_t* chunk_len, uint32_t nchunks, uint8_t flags, int reset_between,
		uint32_t* consumed, uint32_t* out8) {
	const KeyTrie* trie;
	const DfaTable* t = host_dfa(&trie);
	if (!t || !consumed || !out8)
		return -EINVAL;
	GenParser g;
	gp_init(g);
	uint64_t at = 0;
	for (uint32_t k = 0; k < nchunks; k++) {
		const uint8_t* p = data + at;
		consumed[k] = dfa_parse(g, HostTab{t->next}, HostTab{t->attr}, t->info, [p](uint32_t i) { return (uint32_t)p[i]; },
				chunk_len[k], flags);
		at += chunk_len[k];
		if (reset_between && gp_done(g) && k + 1 < nchunks)
			gp_reset(g);
	}
	const uint32_t v[12] = {g.state, g.url_start, g.url_len, (g.f & GPF_HOST) ? g.host_start : 0,
			(g.f & GPF_HOST) ? g.host_len : 0, g.cip_start, g.cip_len, g.f, g.cipkey, g.mcand, 0, 0};
	for (int k = 0; k < 12; k++)
		out8[k] = v[k];
	return 0;
}

int ebd_host_classify(const uint8_t* token, uint32_t len, int is_source, uint8_t flags, const ebd_ipv4_network* v4,
		uint32_t n4, const ebd_ipv6_network* v6, uint32_t n6) {
	static Interfaces ifs;
	fill_ifs(ifs, v4, n4, v6, n6);
	if (is_source)
		return classify_source(ifs, flags, token);
	uint32_t tb, te;
	front_token(token, len, &tb, &te);
	return classify_token(ifs, token + tb, te - tb);
}

int ebd_host_endpoint_key(const uint64_t hash_key[2], uint32_t pid, const uint8_t* endpoint, uint32_t len, uint64_t key[2]) {
	if (!hash_key || !key || (len && !endpoint))
		return -EINVAL;
	KeyHasher kh;
	kh.init(HashKey{hash_key[0], hash_key[1]}, pid);
	kh.bytes(endpoint, len);
	const Hash128 h = kh.finish();
	key[0] = h.lo;
	key[1] = h.hi;
	return 0;
}

int ebd_parser_init(ebd_parser_state* st) {
	if (!st)
		return -EINVAL;
	std::memset(st, 0, sizeof(*st));
	GenParser g;
	gp_init(g);
	std::memcpy(st, &g, sizeof(g)); // no client-IP value, no tokens
	return 0;
}

int ebd_parser_state_check(const ebd_parser_state* st, uint64_t stream_len) {
	if (!st)
		return -EINVAL;
	StreamParser sp;
	std::memcpy(&sp, st, sizeof(sp));
	return stream_state_ok(sp, stream_len) ? 0 : -EINVAL;
}

int ebd_parser_reset(ebd_parser_state* st) {
	if (!st)
		return -EINVAL;
	GenParser g;
	std::memcpy(&g, st, sizeof(g));
	gp_reset(g); // keeps result.clientIPKey (P:374-379)
	std::memset(st, 0, sizeof(*st));
	std::memcpy(st, &g, sizeof(g));
	return 0;
}

const char* ebd_client_ip_key_name(uint32_t id) {
	static const char* names[6] = {"", "rproxy_remote_address", "true-client-ip", "x-client-ip", "x-forwarded-for", "x-http-client-ip"};
	return id < 6 ? names[id] : "";
}

int ebd_parse_streams(ebd_ctx* c, ebd_parse_call* calls, uint32_t n, const uint8_t* data, uint64_t data_len) {
	if (!c || (n && (!calls || (!data && data_len))))
		return -EINVAL;
	for (uint32_t k = 0; k < n; k++) { // every stream inside data, every state one this ABI wrote
		const ebd_parse_call& q = calls[k];
		StreamParser sp;
		std::memcpy(&sp, &q.state, sizeof(sp));
		if (q.data_off > data_len || q.data_len > data_len - q.data_off || !stream_state_ok(sp, q.data_len))
			return -EINVAL;
	}
	if (n == 0)
		return 0;
	std::lock_guard<std::mutex> lk(c->mu);
	HIP_TRY(hipSetDevice(c->device));
	// both directions through one pinned buffer of this context (copies from and to pageable
	// memory are left to the runtime's staging otherwise, and the caller's buffers are not
	// ours to pin)
	const size_t cb = (size_t)n * sizeof(ebd_parse_call), need = cb + (size_t)data_len;
	if (c->h_ps_cap < need) {
		if (c->h_ps)
			HIP_TRY(hipHostFree(c->h_ps));
		c->h_ps = nullptr;
		c->h_ps_cap = 0;
		HIP_TRY(hipHostMalloc((void**)&c->h_ps, need, hipHostMallocDefault));
		c->h_ps_cap = need;
	}
	// a device buffer kept by the context (stream-ordered allocations freed and reused every
	// call returned another call's results now and then: 1 fresh process in 7 saw a stale state)
	const size_t dneed = cb + (size_t)data_len + 16;
	if (c->d_ps_cap < dneed) {
		HIP_TRY(hipStreamSynchronize(c->stream));
		if (c->d_ps)
			HIP_TRY(hipFree(c->d_ps));
		c->d_ps = nullptr;
		c->d_ps_cap = 0;
		HIP_TRY(hipMalloc((void**)&c->d_ps, dneed));
		c->d_ps_cap = dneed;
	}
	std::memcpy(c->h_ps, calls, cb);
	if (data_len)
		std::memcpy(c->h_ps + cb, data, (size_t)data_len);
	ebd_parse_call* dcalls = (ebd_parse_call*)c->d_ps;
	const uint8_t* ddata = c->d_ps + cb;
	HIP_TRY(hipMemcpyAsync(c->d_ps, c->h_ps, cb + (size_t)data_len, hipMemcpyHostToDevice, c->stream));
	HIP_TRY(launch_parse_streams(c->d_trie, dcalls, n, ddata, c->stream));
	HIP_TRY(hipMemcpyAsync(c->h_ps, dcalls, cb, hipMemcpyDeviceToHost, c->stream));
	HIP_TRY(hipStreamSynchronize(c->stream));
	std::memcpy(calls, c->h_ps, cb);
	return 0;
}

int ebd_testing_set_lru_window(ebd_ctx* c, uint32_t window) {
	if (!c)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(c->mu);
	c->lru_window = window;
	return 0;
}

int ebd_host_pton(int af6, const uint8_t* text, uint32_t len, uint8_t* out) {
	return af6 ? (inet_pton6(text, len, out) ? 1 : 0) : (inet_pton4(text, len, out) ? 1 : 0);
}

} // extern "C"
