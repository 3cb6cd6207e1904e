// ebd_fresh.h — fast path for one event parsed by a fresh parser (Discovery.cpp:141-159
// handleNewSession), written once for the GPU kernel and its host emulation.
//
// The byte scan runs the projected DFA (ebd_dfa.h) over the buffer in 16-byte chunks.
// Per byte it only does the table step and keeps the chunk's maximum state (a state
// >= 254 is a client-IP value state).  Along a fresh parse these predicates of the state
// are monotone (false ... false, true ... true; ebd_dfa.h phase groups):
//   URL   s > url_id                        the URL has ended
//   HOST  Host seen                          the first Host value byte was consumed
//   HEND  Host seen and s != HV(host)        the Host value has ended
//   TERM  FINISHED / INVALID                 parse() returns
// so a tracker that keeps "(next chunk << 8) | state at its start" while its predicate is
// still false ends up naming the chunk in which the predicate flips.  The client-IP value
// start (first byte whose next state is >= 254) is tracked the same way with a sticky
// "seen" bit.  Finalize re-runs the DFA over each named chunk (16 bytes, from registers)
// and counts the steps before the flip: that count is the exact position.
#pragma once

#include "../../include/ebpf_discovery_amd.h"
#include "ebd_dfa.h"
#include "ebd_spec.h"

namespace ebd {

constexpr uint32_t kNone = 0xffffffffu;

struct ScanRec {
	uint32_t url, host, hend, cip, term; // (chunk << 8) | state at the chunk's start
	uint32_t cseen;                      // a client-IP value byte was seen
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

EBD_HD void rec_init(const DfaInfo& di, ScanRec& r) {
	r.url = r.host = r.hend = r.cip = r.term = di.init;
	r.cseen = 0;
}

// After chunk c (ended in s1; hit = some byte's next state was >= 254), not terminal.
EBD_HD void chunk_track(const DfaInfo& di, ScanRec& r, uint32_t c, uint32_t s1, bool hit) {
	const uint32_t nxt = ((c + 1) << 8) | s1;
	r.url = st_pred<RS_URL>(di, s1) ? r.url : nxt;
	r.host = st_pred<RS_HOST>(di, s1) ? r.host : nxt;
	r.hend = st_pred<RS_HEND>(di, s1) ? r.hend : nxt;
	r.cseen |= hit ? 1u : 0u;
	r.cip = r.cseen ? r.cip : nxt;
}

// Host emulation of the device scan: identical chunking (skip = buffer address mod 16).
template <typename Tab>
inline uint32_t fresh_scan_host(const Tab& T, const DfaInfo& di, const uint8_t* p, uint32_t skip, uint32_t L, ScanRec& r) {
	rec_init(di, r);
	uint32_t s = di.init;
	const uint32_t nch = (skip + L + 15) / 16;
	for (uint32_t c = 0; c < nch; c++) {
		const uint32_t s0 = s;
		uint32_t m = 0;
		for (uint32_t k = 0; k < 16; k++) {
			const int pos = (int)(c * 16 + k) - (int)skip;
			if (pos < 0 || (uint32_t)pos >= L)
				continue;
			s = T[(s << 8) | p[pos]];
			m = m > s ? m : s;
		}
		if (st_terminal(di, s)) {
			r.term = (c << 8) | s0;
			r.cseen |= m >= 254 ? 1u : 0u; // r.cip already names this chunk
			break;
		}
		chunk_track(di, r, c, s, m >= 254);
	}
	return s;
}

// One 16-byte chunk as 4 little-endian words.
struct Chunk {
	uint32_t w[4];
};

EBD_HD uint32_t chunk_byte(const Chunk& ch, int k) { return (ch.w[k >> 2] >> (8 * (k & 3))) & 0xffu; }

// Position (relative to the buffer) of the first byte in the recorded chunk whose next
// state satisfies W's predicate (RS_CIP: is a client-IP value state).
template <int W, typename Tab>
EBD_HD uint32_t rescan(const Tab& T, const DfaInfo& di, uint32_t rec, const Chunk& ch, uint32_t skip, uint32_t L) {
	const uint32_t c = rec >> 8;
	uint32_t s = rec & 0xffu;
	uint32_t before = 0, seen = 0;
	for (int k = 0; k < 16; k++) {
		const int pos = (int)(c * 16 + k) - (int)skip;
		const bool valid = pos >= 0 && (uint32_t)pos < L;
		const uint32_t sn = valid ? (uint32_t)T[(s << 8) | chunk_byte(ch, k)] : s;
		if (W == RS_CIP) {
			seen |= (valid && sn >= 254) ? 1u : 0u;
			before += seen ? 0u : 1u;
		} else {
			before += st_pred<W>(di, sn) ? 0u : 1u;
		}
		s = sn;
	}
	return c * 16 + before - skip;
}

struct FreshResult {
	ebd_event_result r;
	Hash128 key;
	bool cip; // client class pending: decided from the client-IP token (k_agg_fast, cip_classify)
};

// Turns a scan into the per-event result and the service key (the client class is decided
// later by k_agg_fast: the client-IP front token if there is one, else the source address).  Mem supplies
// chunk(c) (the buffer's c-th aligned 16-byte chunk) and ld8(off) (8 bytes at buffer
// offset off, any alignment; bytes past a span are masked by the caller).
// pid / flags come from the DiscoveryEvent (Discovery.cpp:136, 157).
template <typename Tab, typename Mem>
EBD_HD void fresh_finalize(const Tab& T, const DfaInfo& di, const ScanRec& sr, uint32_t s_final, const Mem& mem, uint32_t skip,
		uint32_t L, uint32_t pid, uint8_t flags, FreshResult& out) {
	ebd_event_result& r = out.r;
	r.info = 0;
	r.u.span.url_off = r.u.span.url_len = r.u.span.host_off = r.u.span.host_len = r.u.span.cip_off = r.u.span.cip_len = 0;
	out.key.lo = out.key.hi = 0;
	out.cip = false;
	if (!st_terminal(di, s_final)) {
		r.status = EBD_STATUS_UNFINISHED;
		r.consumed = (uint16_t)L;
		return;
	}
	const bool fin = s_final != di.inv, host = s_final == di.fin1, cip = fin && sr.cseen;
	// every chunk finalize may need, loaded unconditionally before any is used
	const Chunk wt = mem.chunk(sr.term >> 8), wu = mem.chunk(sr.url >> 8), wh = mem.chunk(sr.host >> 8),
	            we = mem.chunk(sr.hend >> 8), wc = mem.chunk(sr.cip >> 8);
	const uint32_t consumed = rescan<RS_TERM>(T, di, sr.term, wt, skip, L) + 1;
	if (consumed > L) {
		// the device scans whole chunks: a terminal state reached only past the buffer's
		// last byte is an unfinished parse (HttpRequestParser.cpp:85-106 stops at L)
		r.status = EBD_STATUS_UNFINISHED;
		r.consumed = (uint16_t)L;
		return;
	}
	r.consumed = (uint16_t)consumed;
	if (!fin) {
		r.status = EBD_STATUS_INVALID;
		return;
	}
	r.status = EBD_STATUS_FINISHED;
	const bool post = (mem.ld8(0) & 0xff) == 'P';
	const uint32_t url_start = post ? 5 : 4;
	const uint32_t url_len = rescan<RS_URL>(T, di, sr.url, wu, skip, L) - url_start;
	uint32_t host_start = 0, host_len = 0;
	if (host) {
		host_start = rescan<RS_HOST>(T, di, sr.host, wh, skip, L);
		host_len = rescan<RS_HEND>(T, di, sr.hend, we, skip, L) - host_start;
	}
	uint8_t info = (uint8_t)((post ? EBD_INFO_POST : 0) | ((flags & 16) ? EBD_INFO_HTTPS : 0));
	if (cip) {
		// raw value start of the first client-IP header; token and class: k_agg_fast
		r.u.span.cip_off = (uint16_t)rescan<RS_CIP>(T, di, sr.cip, wc, skip, L);
		info |= EBD_INFO_CIP;
		out.cip = true;
	} // else the class comes from the source address (k_agg_fast reads the event)
	r.info = info;
	r.u.span.url_off = (uint16_t)url_start;
	r.u.span.url_len = (uint16_t)url_len;
	r.u.span.host_off = (uint16_t)host_start;
	r.u.span.host_len = (uint16_t)host_len;
#ifdef EBD_EXP_NOHASH // experiment: finalize without the key (results are wrong)
	out.key.lo = host_len * 31 + url_len;
	out.key.hi = 1;
#else
	out.key = endpoint_key(pid, host_start, host_len, url_start, url_len, [&](uint32_t o) { return mem.ld8(o); });
#endif
}

// Client-IP pass for one event (HttpRequestParser.cpp:370-407 parseClientIPValue on the
// first client-IP header's value, Aggregator.cpp:50-74 on its front token): the raw value
// runs from `cs` to the first ',' or the value's CR (value bytes are C-class, so a CR ends
// it; the request's final CRLF bounds the search).  `at(k)` yields buffer byte k.
template <typename At>
EBD_HD void cip_token(const Interfaces& ifs, At at, uint32_t cs, uint32_t consumed, uint32_t* tb, uint32_t* te, uint8_t* cls) {
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
	*cls = classify_token(ifs, View{at, cs + b}, en - b);
}

} // namespace ebd
