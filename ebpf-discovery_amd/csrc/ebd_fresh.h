// ebd_fresh.h — fast path for one event parsed by a fresh parser (Discovery.cpp:141-159
// handleNewSession), written once for the GPU kernel and its host emulation.
//
// The byte scan runs the projected DFA (ebd_dfa.h) over the buffer in 16-byte chunks,
// chunk c = bytes [16c, 16c + 16) of the buffer.  The last chunk may run past the buffer;
// the scan steps over those bytes too, which only changes states at positions >= L, so a
// terminal position >= L is an unfinished parse and every other tracked position is < L.
// Per byte the scan only does the table step and keeps the chunk's maximum next state (a
// state >= hvc0 is a client-IP value state).  Along a fresh parse these predicates of the
// state are monotone (false ... false, true ... true; ebd_dfa.h phase groups):
//   URL   s > url_id                        the URL has ended
//   HOST  Host seen                          the first Host value byte was consumed
//   HEND  Host seen and s != HV(host)        the Host value has ended
//   TERM  FINISHED / INVALID                 parse() returns
// A tracker keeps the last chunk whose start state still fails its predicate, so it ends
// up naming the chunk in which the predicate flips, together with the states at the
// starts of that chunk's four 4-byte quarters.  The client-IP value start (first byte
// whose next state is >= hvc0) is tracked the same way, with the running maxima after 4, 8
// and 12 steps, until a chunk has seen such a state.  Finalize picks the quarter in which
// the predicate flips from those states and re-runs the DFA over its 4 bytes: the steps
// before the flip give the exact position.
#pragma once

#include "../../include/ebpf_discovery_amd.h"
#include "ebd_dfa.h"
#include "ebd_spec.h"

namespace ebd {

constexpr uint32_t kNone = 0xffffffffu;

// The chunk in which a predicate flips, and the states at the starts of its quarters
// (qs = s0 | s4 << 8 | s8 << 16 | s12 << 24).
struct Trk {
	uint32_t c, qs;
};

struct ScanRec {
	Trk url, host, hend, cip, term; // term: the last chunk scanned
	uint32_t cqm;                   // cip chunk: running max next state after 4, 8, 12 steps (bytes 0..2)
	uint32_t cseen;                 // a client-IP value state was reached (the cip tracker is frozen)
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
	const Trk t{0, di.init * 0x01010101u};
	r.url = r.host = r.hend = r.cip = r.term = t;
	r.cqm = 0;
	r.cseen = 0;
}

// After chunk c: s0 = its start state, qs = its quarter-start states, qm = running maxima
// after 4/8/12 steps, m = the chunk's maximum next state.
EBD_HD void chunk_update(const DfaInfo& di, ScanRec& r, uint32_t c, uint32_t s0, uint32_t qs, uint32_t qm, uint32_t m) {
	const Trk t{c, qs};
	r.url = st_pred<RS_URL>(di, s0) ? r.url : t;
	r.host = st_pred<RS_HOST>(di, s0) ? r.host : t;
	r.hend = st_pred<RS_HEND>(di, s0) ? r.hend : t;
	const bool open = r.cseen == 0;
	r.cip = open ? t : r.cip;
	r.cqm = open ? qm : r.cqm;
	r.cseen |= m >= di.hvc0 ? 1u : 0u;
	r.term = t;
}

// Byte k of a packed word.
EBD_HD uint32_t byte_of(uint32_t w, uint32_t k) { return (w >> (8 * k)) & 0xffu; }

// Quarter of the tracker's chunk in which W's predicate flips (3 when no quarter start
// after the first satisfies it).
template <int W>
EBD_HD uint32_t flip_quarter(const DfaInfo& di, const Trk& t, uint32_t cqm) {
	if (W == RS_CIP)
		return byte_of(cqm, 0) >= di.hvc0 ? 0u : byte_of(cqm, 1) >= di.hvc0 ? 1u : byte_of(cqm, 2) >= di.hvc0 ? 2u : 3u;
	return st_pred<W>(di, byte_of(t.qs, 1)) ? 0u : st_pred<W>(di, byte_of(t.qs, 2)) ? 1u : st_pred<W>(di, byte_of(t.qs, 3)) ? 2u : 3u;
}

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

// Position (in the buffer) of the first byte after which W's predicate holds.
template <int W, typename Tab>
EBD_HD uint32_t flip_pos(const Tab& T, const DfaInfo& di, const Trk& t, uint32_t q, uint32_t w4) {
	return 16 * t.c + 4 * q + rescan4<W>(T, di, byte_of(t.qs, q), w4);
}

// Host emulation of the device scan: the same chunks, and bytes past the buffer taken from
// `past(k)` (the device reads whatever follows the buffer).
template <typename Tab, typename Past>
inline uint32_t fresh_scan_host(const Tab& T, const DfaInfo& di, const uint8_t* p, uint32_t L, Past past, ScanRec& r) {
	rec_init(di, r);
	uint32_t s = di.init;
	const uint32_t nch = (L + 15) / 16;
	for (uint32_t c = 0; c < nch; c++) {
		const uint32_t s0 = s;
		uint32_t m = 0, qs = s0, qm = 0;
		for (uint32_t k = 0; k < 16; k++) {
			const uint32_t pos = c * 16 + k;
			s = T[(s << 8) | (pos < L ? p[pos] : past(pos - L))];
			m = m > s ? m : s;
			if (k == 3 || k == 7 || k == 11) {
				qs |= s << (8 * ((k + 1) / 4));
				qm |= m << (8 * (k / 4));
			}
		}
		chunk_update(di, r, c, s0, qs, qm, m);
		if (st_terminal(di, s))
			break;
	}
	return s;
}

struct FreshResult {
	ebd_event_result r;
	Hash128 key;
	bool cip;  // client class pending: decided from the client-IP token (k_agg_fast, cip_classify)
	bool keyed; // FINISHED: the key over (pid, host + url) is still to be computed
};

// The flip quarter of every tracker and the 4 buffer bytes a rescan of it needs.
struct FinLoads {
	uint32_t qt, qu, qh, qe, qc;
	uint32_t wt, wu, wh, we, wc;
};

// Mem supplies ld4(off) (4 bytes at buffer offset off, any alignment) and ld8(off); every
// load is issued before any is used.
template <typename Mem>
EBD_HD void fresh_loads(const DfaInfo& di, const ScanRec& sr, const Mem& mem, FinLoads& f) {
	f.qt = flip_quarter<RS_TERM>(di, sr.term, 0);
	f.qu = flip_quarter<RS_URL>(di, sr.url, 0);
	f.qh = flip_quarter<RS_HOST>(di, sr.host, 0);
	f.qe = flip_quarter<RS_HEND>(di, sr.hend, 0);
	f.qc = flip_quarter<RS_CIP>(di, sr.cip, sr.cqm);
	f.wt = mem.ld4(16 * sr.term.c + 4 * f.qt);
	f.wu = mem.ld4(16 * sr.url.c + 4 * f.qu);
	f.wh = mem.ld4(16 * sr.host.c + 4 * f.qh);
	f.we = mem.ld4(16 * sr.hend.c + 4 * f.qe);
	f.wc = mem.ld4(16 * sr.cip.c + 4 * f.qc);
}

// Turns a scan into the per-event result (the client class is decided later by k_agg_fast:
// the client-IP front token if there is one, else the source address).  `post`: the
// buffer's first byte is 'P'.  flags come from the DiscoveryEvent (Discovery.cpp:136, 157).
// A FINISHED result leaves out.keyed set: the key is endpoint_key over its spans.
template <typename Tab>
EBD_HD void fresh_spans(const Tab& T, const DfaInfo& di, const ScanRec& sr, uint32_t s_final, bool post, const FinLoads& f,
		uint32_t L, uint8_t flags, FreshResult& out) {
	ebd_event_result& r = out.r;
	r.info = 0;
	r.u.span.url_off = r.u.span.url_len = r.u.span.host_off = r.u.span.host_len = r.u.span.cip_off = r.u.span.cip_len = 0;
	out.key.lo = out.key.hi = 0;
	out.cip = false;
	out.keyed = false;
	const uint32_t consumed = flip_pos<RS_TERM>(T, di, sr.term, f.qt, f.wt) + 1;
	if (!st_terminal(di, s_final) || consumed > L) {
		// not terminal, or terminal only past the buffer's last byte: parse() stops at L
		// (HttpRequestParser.cpp:85-106), unfinished
		r.status = EBD_STATUS_UNFINISHED;
		r.consumed = (uint16_t)L;
		return;
	}
	r.consumed = (uint16_t)consumed;
	const bool fin = s_final != di.inv, host = s_final == di.fin1, cip = fin && sr.cseen;
	if (!fin) {
		r.status = EBD_STATUS_INVALID;
		return;
	}
	r.status = EBD_STATUS_FINISHED;
	const uint32_t url_start = post ? 5 : 4;
	const uint32_t url_len = flip_pos<RS_URL>(T, di, sr.url, f.qu, f.wu) - url_start;
	uint32_t host_start = 0, host_len = 0;
	if (host) {
		host_start = flip_pos<RS_HOST>(T, di, sr.host, f.qh, f.wh);
		host_len = flip_pos<RS_HEND>(T, di, sr.hend, f.qe, f.we) - host_start;
	}
	uint8_t info = (uint8_t)((post ? EBD_INFO_POST : 0) | ((flags & 16) ? EBD_INFO_HTTPS : 0));
	if (cip) {
		// raw value start of the first client-IP header; token and class: k_agg_fast
		r.u.span.cip_off = (uint16_t)flip_pos<RS_CIP>(T, di, sr.cip, f.qc, f.wc);
		info |= EBD_INFO_CIP;
		out.cip = true;
	} // else the class comes from the source address (k_agg_fast reads the event)
	r.info = info;
	r.u.span.url_off = (uint16_t)url_start;
	r.u.span.url_len = (uint16_t)url_len;
	r.u.span.host_off = (uint16_t)host_start;
	r.u.span.host_len = (uint16_t)host_len;
	out.keyed = true;
}

// The whole finalize for one event (the host twin; the device interleaves the steps of
// several events).  pid: the DiscoveryEvent's (Discovery.cpp:136, 157).
template <typename Tab, typename Mem>
EBD_HD void fresh_finalize(const Tab& T, const DfaInfo& di, const ScanRec& sr, uint32_t s_final, bool post, const Mem& mem,
		uint32_t L, const HashKey& key, uint32_t pid, uint8_t flags, FreshResult& out) {
	FinLoads f;
	fresh_loads(di, sr, mem, f);
	fresh_spans(T, di, sr, s_final, post, f, L, flags, out);
	if (out.keyed) {
		const auto& sp = out.r.u.span;
		out.key = endpoint_key(key, pid, sp.host_off, sp.host_len, sp.url_off, sp.url_len, [&](uint32_t o) { return mem.ld8(o); });
	}
}

// ---------------------------------------------------------------------------------
// The session path's parser: HttpRequestParser::parse (P:85-106) continued across the
// buffers of a session (Discovery.cpp:123-139 handleExistingSession), as the projected DFA
// plus the few fields the request needs.  The DFA is exact for a continued parse too: its
// projection keeps everything that decides a future transition, whatever the sticky
// clientIPKey (ebd_dfa.cpp checks every state against variants with it set).  What the DFA
// forgets is which client-IP key a value belongs to, so the walker keeps the client id of
// the last header-key state it left (DfaTable::attr bits 0-2) and applies P:309-316 itself:
// the first client-IP value sets clientIPKey when none is set (it stays set across reset,
// P:374-379), and only the first header whose key equals it is the client address.
// The walk goes 16 bytes at a time (dfa_walk_block): the state chain first (one table read
// and one attribute read per byte), then the bookkeeping only at the bytes whose state
// attribute differs from the previous state's (a few per request: URL, Host and client-IP
// value edges, header keys), since no field changes anywhere else.  Terminal states step to
// themselves, so bytes after the end change nothing but the position.
// Spans are request-stream positions, as gp_step's.
// ---------------------------------------------------------------------------------
struct DfaWalk {
	uint32_t s, a, kid, pos, f, cipkey, mcand, tpos, lcp;
	uint32_t url_start, url_end, host_start, host_end, cip_start, cip_end;
};

EBD_HD void dfa_walk_load(const GenParser& g, uint32_t attr_s, DfaWalk& w) {
	w.s = g.ds;
	w.a = attr_s;
	w.kid = g.kid;
	w.pos = g.length;
	w.f = g.f;
	w.cipkey = g.cipkey;
	w.mcand = g.mcand;
	w.tpos = kNone;
	w.lcp = kNone;
	w.url_start = g.url_start;
	w.url_end = g.url_start + g.url_len;
	w.host_start = g.host_start;
	w.host_end = g.host_start + g.host_len;
	w.cip_start = g.cip_start;
	w.cip_end = g.cip_start + g.cip_len;
}

// The byte at request position pos moved the walk from a state with attribute ao to one with
// attribute an != ao.  gp_step's per-byte rules reduced to such bytes: the client id of the
// last header-key state (kid) is that of the state before the byte, which has not changed
// since the previous such byte (dfa_walk_store applies the final state's at the end).
EBD_HD void dfa_walk_change(DfaWalk& w, uint32_t ao, uint32_t an, uint32_t pos) {
	const uint32_t x = an ^ ao, en = an & x, lv = ao & x, ko = ao & 7u;
	w.kid = ko != kKcKeep ? ko : w.kid;
	w.url_start = (en & A_URL) ? pos : w.url_start; // P:190-199: the URL starts with its '/'
	w.url_end = (lv & A_URL) ? pos : w.url_end;     // P:201-213: it ends before the space
	w.host_start = (en & A_HVH) ? pos : w.host_start; // P:309-310: the first Host value byte
	w.host_end = (lv & A_HVH) ? pos : w.host_end;
	w.f |= (en & A_HVH) ? (uint32_t)GPF_HOST : 0u;
	// P:311-316: the first byte of a client-IP value; its key is the last key state's
	const bool ce = (en & A_HVC) != 0;
	const uint32_t ck = w.cipkey ? w.cipkey : w.kid;
	w.cipkey = ce ? ck : w.cipkey;
	const bool take = ce && w.kid == ck && !(w.f & (GPF_CIP_FOUND | GPF_IN_CIP));
	w.cip_start = take ? pos : w.cip_start;
	w.f |= take ? (uint32_t)GPF_IN_CIP : 0u;
	const bool cl = (lv & A_HVC) && (w.f & GPF_IN_CIP); // the value's CR (P:248-257 parses it)
	w.cip_end = cl ? pos : w.cip_end;
	w.f = cl ? ((w.f & ~(uint32_t)GPF_IN_CIP) | GPF_CIP_FOUND) : w.f;
	w.tpos = (en & A_TERM) && w.tpos == kNone ? pos + 1 : w.tpos;
	w.lcp = pos;
}

// Byte k (0..15) of a 16-byte block held as four words.
EBD_HD uint32_t blk_byte(uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3, uint32_t k) {
	const uint32_t lo = (k & 4u) ? v1 : v0, hi = (k & 4u) ? v3 : v2; // selects (an indexed array went to scratch)
	return (((k & 8u) ? hi : lo) >> (8u * (k & 3u))) & 0xffu;
}

// One 16-byte block of a parse: byte k (of the words wd) is valid when base + k < ne (base:
// the buffer offset of byte 0, wrapping below 0 for a buffer that starts inside the block)
// and lies at request position pbase + k; valid bytes are consecutive.  w.tpos = the bytes of
// the request up to and including the byte that made the state terminal (a parse() on an
// ended parser takes one byte).
template <typename Tab, typename At>
EBD_HD void dfa_walk_block(const Tab& T, const At& A, DfaWalk& w, const uint32_t (&wd)[4], uint32_t base, uint32_t pbase, uint32_t ne) {
	const uint32_t a0 = w.a;
	uint32_t s = w.s, a = a0, chg = 0, nv = 0;
	uint32_t P[4] = {0u, 0u, 0u, 0u}; // the attribute after each byte
#pragma unroll
	for (int k = 0; k < 16; k++) {
		const uint32_t b = (wd[k >> 2] >> (8 * (k & 3))) & 0xffu;
		const bool v = base + (uint32_t)k < ne;
		// the read is unconditional (every index is valid): a read inside the condition made the
		// device code branch per byte and wait for both table reads before the next byte's
		const uint32_t t = (uint32_t)T[(s << 8) | b];
		const uint32_t ns = v ? t : s;
		const uint32_t an = A[ns];
		chg |= an != a ? 1u << k : 0u;
		P[k >> 2] |= an << (8 * (k & 3));
		nv += v ? 1u : 0u;
		s = ns;
		a = an;
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
	w.a = a;
	w.pos += nv;
}

// The end of a parse() call that walked `ne` of the buffer's `n` bytes (ne < n: the request
// reached the length cap, P:88-91): the walk back into the session's GenParser.  Returns the
// bytes consumed.  A parse that ended takes isHttps from the event's flags (P:94-103).
EBD_HD uint32_t dfa_walk_store(const DfaInfo& di, DfaWalk& w, uint32_t pos0, uint32_t ne, uint32_t n, uint8_t flags,
		GenParser& g) {
	uint32_t consumed = ne, f = w.f;
	bool done = false;
	if (w.pos != pos0 && w.lcp != w.pos - 1u) { // the bytes after the last change: kid of the final state
		const uint32_t ko = w.a & 7u;
		w.kid = ko != kKcKeep ? ko : w.kid;
	}
	if (w.tpos != kNone) {
		consumed = w.tpos - pos0;
		done = true;
	} else if (ne < n) {
		w.s = di.inv;
		done = true;
	}
	g.ds = (uint8_t)w.s;
	g.kid = (uint8_t)w.kid;
	g.length = pos0 + consumed;
	g.cipkey = (uint8_t)w.cipkey;
	g.mcand = (uint8_t)w.mcand;
	g.url_start = w.url_start;
	g.url_len = w.url_end - w.url_start;
	g.host_start = w.host_start;
	g.host_len = w.host_end - w.host_start;
	g.cip_start = w.cip_start;
	g.cip_len = w.cip_end - w.cip_start;
	if (done) {
		g.state = w.s == di.inv ? ST_INVALID : ST_FINISHED;
		f = (flags & 16) ? (f | GPF_HTTPS) : (f & ~(uint32_t)GPF_HTTPS);
	}
	g.f = (uint8_t)f;
	return consumed;
}

// Bytes of this buffer the request may still take before the length cap (P:88-91: a byte
// is refused once more than kMaxRequestLength bytes were parsed).
EBD_HD uint32_t dfa_allow(uint32_t pos, uint32_t n) {
	const uint32_t allow = pos <= kMaxRequestLength ? kMaxRequestLength + 1 - pos : 0;
	return n < allow ? n : allow;
}

// P:85-106 parse() of one buffer with the DFA, 16 bytes at a time: returns the bytes consumed
// (the host twin of the device walker).
template <typename Tab, typename At, typename ByteAt>
EBD_HD uint32_t dfa_parse(GenParser& g, const Tab& T, const At& A, const DfaInfo& di, ByteAt at, uint32_t n, uint8_t flags) {
	DfaWalk w;
	dfa_walk_load(g, A[g.ds], w);
	const uint32_t pos0 = w.pos, ne = dfa_allow(pos0, n);
	for (uint32_t base = 0; base < ne && w.tpos == kNone; base += 16) {
		uint32_t wd[4] = {0u, 0u, 0u, 0u};
		for (uint32_t k = 0; k < 16 && base + k < ne; k++)
			wd[k >> 2] |= (at(base + k) & 0xffu) << (8 * (k & 3));
		dfa_walk_block(T, A, w, wd, base, pos0 + base, ne);
	}
	return dfa_walk_store(di, w, pos0, ne, n, flags, g);
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
