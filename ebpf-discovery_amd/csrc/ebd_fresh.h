// ebd_fresh.h — fast path for one event parsed by a fresh parser (Discovery.cpp:141-159
// handleNewSession), written once for the GPU kernel (k_fresh) and its host emulation.
//
// The walk runs the projected DFA (ebd_dfa.h) over the buffer one 4-byte word at a time,
// word w = bytes [4w, 4w + 4).  The last word may run past the buffer; the walk steps over
// those bytes too, which only changes states at positions >= L, so a terminal position >= L
// is an unfinished parse and every other tracked position is < L.
//
// Jumps.  In a generic header-value state (vl0 / vl1: the value of a header that is neither
// Host nor a client-IP key; they step to themselves on every byte in [0x20, 0x7e], checked
// when the table is built) the parser only waits for the first byte outside [0x20, 0x7e]:
// the CR that ends the value, or an invalid byte (HttpRequestParser.cpp:304-330).  So when a
// word starts in such a state, the walk jumps to the word holding the next non-printable
// byte (the kernel finds it in a bitmap of the tile), or to L when there is none.  No
// predicate below changes inside a skipped stretch, so every flip still lies in a walked word.
//
// Per walked word the walk keeps the word's maximum next state (a state >= hvc0 is a
// client-IP value state).  Along a fresh parse these predicates of the state are monotone
// (false ... false, true ... true; ebd_dfa.h phase groups):
//   URL   s > url_id                        the URL has ended
//   HOST  Host seen                          the first Host value byte was consumed
//   HEND  Host seen and s != HV(host)        the Host value has ended
//   TERM  FINISHED / INVALID                 parse() returns
// A tracker keeps the last walked word whose start state still fails its predicate, with that
// start state; so it names the word in which the predicate flips.  The client-IP value start
// (first byte whose next state is >= hvc0) is tracked the same way, until a word has reached
// such a state.  Finalize re-runs the DFA over the tracker's 4 bytes from the stored state:
// the steps before the flip give the exact position.
#pragma once

#include "../../include/ebpf_discovery_amd.h"
#include "ebd_dfa.h"
#include "ebd_spec.h"

namespace ebd {

constexpr uint32_t kNone = 0xffffffffu;

// A walked word and the state at its start, packed: w | s0 << 16 (w < 2^14: L <= 8192).
EBD_HD uint32_t wtrk(uint32_t w, uint32_t s0) { return w | (s0 << 16); }
EBD_HD uint32_t wtrk_w(uint32_t t) { return t & 0xffffu; }
EBD_HD uint32_t wtrk_s(uint32_t t) { return t >> 16; }

struct WalkRec {
	uint32_t url, host, hend, cip, term; // wtrk; term: the last walked word
	uint32_t cseen;                      // a client-IP value state was reached (the cip tracker is frozen)
};

enum { RS_URL, RS_HOST, RS_HEND, RS_TERM, RS_CIP };

EBD_HD bool st_terminal(const DfaInfo& di, uint32_t s) { return s - di.g4 < 3u; }
EBD_HD bool st_host_seen(const DfaInfo& di, uint32_t s) {
	return (s - di.g3 < di.g4 - di.g3) || s == di.fin1 || s == di.hvc1;
}
template <int W>
EBD_HD bool st_pred(const DfaInfo& di, uint32_t s) {
	if (W == RS_URL)
		return s > di.url_id;
	if (W == RS_HOST)
		return st_host_seen(di, s);
	if (W == RS_HEND)
		return st_host_seen(di, s) && s != di.hvh;
	return st_terminal(di, s);
}
// a word starting in this state may be jumped over up to the next non-printable byte
EBD_HD bool st_skips(const DfaInfo& di, uint32_t s) { return s == di.vl0 || s == di.vl1; }

EBD_HD void walk_init(const DfaInfo& di, WalkRec& r) {
	const uint32_t t = wtrk(0, di.init);
	r.url = r.host = r.hend = r.cip = r.term = t;
	r.cseen = 0;
}

// After walked word w with start state s0 and maximum next state m.
EBD_HD void word_update(const DfaInfo& di, WalkRec& r, uint32_t w, uint32_t s0, uint32_t m) {
	const uint32_t t = wtrk(w, s0);
	r.url = st_pred<RS_URL>(di, s0) ? r.url : t;
	r.host = st_pred<RS_HOST>(di, s0) ? r.host : t;
	r.hend = st_pred<RS_HEND>(di, s0) ? r.hend : t;
	r.cip = r.cseen ? r.cip : t;
	r.cseen |= m >= di.hvc0 ? 1u : 0u;
	r.term = t;
}

// Byte k of a packed word.
EBD_HD uint32_t byte_of(uint32_t w, uint32_t k) { return (w >> (8 * k)) & 0xffu; }

// Steps over the 4 bytes of `w` from state s before W's predicate holds (RS_CIP: before the
// first step whose next state is >= hvc0); 4 if it never does.
template <int W, typename Tab>
EBD_HD uint32_t rescan4(const Tab& T, const DfaInfo& di, uint32_t s, uint32_t w) {
	uint32_t before = 0, hit = 0;
#pragma unroll
	for (int k = 0; k < 4; k++) {
		s = T[(s << 8) | byte_of(w, (uint32_t)k)];
		const bool p = W == RS_CIP ? s >= di.hvc0 : st_pred<W>(di, s);
		hit |= p ? 1u : 0u;
		before += hit ? 0u : 1u;
	}
	return before;
}

// Position (in the buffer) of the first byte after which W's predicate holds; word4 = the
// tracker word's 4 bytes.
template <int W, typename Tab>
EBD_HD uint32_t flip_pos(const Tab& T, const DfaInfo& di, uint32_t t, uint32_t word4) {
	return 4 * wtrk_w(t) + rescan4<W>(T, di, wtrk_s(t), word4);
}

// Host emulation of the device walk.  byte(k): buffer byte k for any k (past L: whatever
// follows the buffer); next_np(p): the first byte >= p below L outside [0x20, 0x7e], or L.
template <typename Tab, typename Byte, typename NextNp>
inline uint32_t fresh_walk_host(const Tab& T, const DfaInfo& di, Byte byte, uint32_t L, NextNp next_np, WalkRec& r) {
	walk_init(di, r);
	uint32_t s = di.init, p = 0;
	while (p < L && !st_terminal(di, s)) {
		if (st_skips(di, s)) {
			const uint32_t q = next_np(p);
			if (q >= L)
				break; // printable to the end: still waiting for the CR, unfinished
			p = q & ~3u;
		}
		const uint32_t s0 = s;
		uint32_t m = 0;
		for (uint32_t k = 0; k < 4; k++) {
			s = T[(s << 8) | byte(p + k)];
			m = m > s ? m : s;
		}
		word_update(di, r, p >> 2, s0, m);
		p += 4;
	}
	return s;
}

struct FreshResult {
	ebd_event_result r;
	Hash128 key;
	bool cip;  // client class pending: decided from the client-IP front token (cip_token)
	bool keyed; // FINISHED: the key over (pid, host + url) is still to be computed
};

// The 4 buffer bytes each tracker's rescan needs.
struct FinLoads {
	uint32_t wt, wu, wh, we, wc;
};

// Mem supplies ld4(off) (4 bytes at buffer offset off, any alignment) and ld8(off).
template <typename Mem>
EBD_HD void fresh_loads(const WalkRec& r, const Mem& mem, FinLoads& f) {
	f.wt = mem.ld4(4 * wtrk_w(r.term));
	f.wu = mem.ld4(4 * wtrk_w(r.url));
	f.wh = mem.ld4(4 * wtrk_w(r.host));
	f.we = mem.ld4(4 * wtrk_w(r.hend));
	f.wc = mem.ld4(4 * wtrk_w(r.cip));
}

// Turns a walk into the per-event result (the client class is decided after: the client-IP
// front token if there is one, else the source address).  `post`: the buffer's first byte is
// 'P'.  flags come from the DiscoveryEvent (Discovery.cpp:136, 157).  A FINISHED result leaves
// out.keyed set: the key is endpoint_key over its spans; out.cip: cip_off is the raw value start.
template <typename Tab>
EBD_HD void fresh_spans(const Tab& T, const DfaInfo& di, const WalkRec& wr, uint32_t s_final, bool post, const FinLoads& f,
		uint32_t L, uint8_t flags, FreshResult& out) {
	ebd_event_result& r = out.r;
	r.info = 0;
	r.u.span.url_off = r.u.span.url_len = r.u.span.host_off = r.u.span.host_len = r.u.span.cip_off = r.u.span.cip_len = 0;
	out.key.lo = out.key.hi = 0;
	out.cip = false;
	out.keyed = false;
	const uint32_t consumed = flip_pos<RS_TERM>(T, di, wr.term, f.wt) + 1;
	if (!st_terminal(di, s_final) || consumed > L) {
		// not terminal, or terminal only past the buffer's last byte: parse() stops at L
		// (HttpRequestParser.cpp:85-106), unfinished
		r.status = EBD_STATUS_UNFINISHED;
		r.consumed = (uint16_t)L;
		return;
	}
	r.consumed = (uint16_t)consumed;
	const bool fin = s_final != di.inv, host = s_final == di.fin1, cip = fin && wr.cseen;
	if (!fin) {
		r.status = EBD_STATUS_INVALID;
		return;
	}
	r.status = EBD_STATUS_FINISHED;
	const uint32_t url_start = post ? 5 : 4;
	const uint32_t url_len = flip_pos<RS_URL>(T, di, wr.url, f.wu) - url_start;
	uint32_t host_start = 0, host_len = 0;
	if (host) {
		host_start = flip_pos<RS_HOST>(T, di, wr.host, f.wh);
		host_len = flip_pos<RS_HEND>(T, di, wr.hend, f.we) - host_start;
	}
	uint8_t info = (uint8_t)((post ? EBD_INFO_POST : 0) | ((flags & 16) ? EBD_INFO_HTTPS : 0));
	if (cip) {
		r.u.span.cip_off = (uint16_t)flip_pos<RS_CIP>(T, di, wr.cip, f.wc); // raw value start
		info |= EBD_INFO_CIP;
		out.cip = true;
	} // else the class comes from the source address
	r.info = info;
	r.u.span.url_off = (uint16_t)url_start;
	r.u.span.url_len = (uint16_t)url_len;
	r.u.span.host_off = (uint16_t)host_start;
	r.u.span.host_len = (uint16_t)host_len;
	out.keyed = true;
}

// The whole finalize for one event but the client class.  pid: the DiscoveryEvent's
// (Discovery.cpp:136, 157).
template <typename Tab, typename Mem>
EBD_HD void fresh_finalize(const Tab& T, const DfaInfo& di, const WalkRec& wr, uint32_t s_final, bool post, const Mem& mem,
		uint32_t L, const HashKey& key, uint32_t pid, uint8_t flags, FreshResult& out) {
	FinLoads f;
	fresh_loads(wr, mem, f);
	fresh_spans(T, di, wr, s_final, post, f, L, flags, out);
	if (out.keyed) {
		const auto& sp = out.r.u.span;
		out.key = endpoint_key<2>(key, pid, sp.host_off, sp.host_len, sp.url_off, sp.url_len, [&](uint32_t o) { return mem.ld8(o); });
	}
}

// Client-IP pass for one event (HttpRequestParser.cpp:370-407 parseClientIPValue on the
// first client-IP header's value, Aggregator.cpp:50-74 on its front token): the raw value
// runs from `cs` to the first ',' or the value's CR (value bytes are C-class, so a CR ends
// it; the request's final CRLF bounds the search).  `at(k)` yields buffer byte k.
template <typename At>
EBD_HD void cip_token(const Interfaces& ifs, At at, uint32_t cs, uint32_t consumed, uint32_t* tb, uint32_t* te, uint8_t* cls,
		unsigned long long* net = nullptr) {
	uint32_t e = cs;
	while (e < consumed && at(e) != ',' && at(e) != '\r')
		e++;
	// front_token / classify_token over the raw value, through the accessor
	struct View {
		At at;
		uint32_t base;
		EBD_HD uint8_t operator[](uint32_t k) const { return (uint8_t)at(base + k); }
	} v{at, cs};
	uint32_t b, en;
	front_token(v, e - cs, &b, &en);
	*tb = cs + b;
	*te = cs + en;
	*cls = classify_token(ifs, View{at, cs + b}, en - b, net);
}

} // namespace ebd
