// ebd_gen.h — synthetic capture traces, host == device.
//
// Every event is a pure function of (config, seed, event index) through Philox4x32-10
// and integer CDF tables, so any shard or sample regenerates bit-identically on the
// CPU (parity tests) and on the GPU (benchmark data generated in HBM).  The request
// layout follows what the kernel-side filter admits (libebpfdiscoveryskel/src/
// DataFunctions.h:45-50: first buffer starts "GET /" or "POST /", >= 16 bytes) and the
// saved-buffer limit (TrackedSession.h:159-170: <= 8192 bytes).
#pragma once

#include "ebd_spec.h"

namespace ebd {

struct Philox {
	EBD_HD static void mulhilo(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
		const uint64_t p = (uint64_t)a * b;
		hi = (uint32_t)(p >> 32);
		lo = (uint32_t)p;
	}
	// Philox4x32-10 (Salmon et al., SC'11)
	EBD_HD static void gen(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1, uint32_t out[4]) {
		for (int r = 0; r < 10; r++) {
			uint32_t hi0, lo0, hi1, lo1;
			mulhilo(0xD2511F53u, c0, hi0, lo0);
			mulhilo(0xCD9E8D57u, c2, hi1, lo1);
			const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
			c0 = n0;
			c1 = lo1;
			c2 = n2;
			c3 = lo0;
			k0 += 0x9E3779B9u;
			k1 += 0xBB67AE85u;
		}
		out[0] = c0;
		out[1] = c1;
		out[2] = c2;
		out[3] = c3;
	}
};

constexpr uint32_t kLenMin = 32, kLenMax = 1024, kLenN = kLenMax - kLenMin + 1;
constexpr uint32_t kPaths = 100000, kHosts = 1000, kPids = 64;

// Integer CDF tables (built on the host with basic IEEE operations only, copied to HBM).
struct GenTables {
	uint32_t len_cdf[kLenN];
	uint32_t host_cdf[kHosts];
	uint32_t path_cdf[kPaths];
};

EBD_HD uint32_t cdf_sample(const uint32_t* cdf, uint32_t n, uint32_t u) {
	uint32_t lo = 0, hi = n - 1; // smallest k with u < cdf[k]; cdf[n-1] = 0xffffffff
	while (lo < hi) {
		const uint32_t mid = (lo + hi) >> 1;
		if (u < cdf[mid])
			hi = mid;
		else
			lo = mid + 1;
	}
	return lo;
}

// Byte sink: counts (w == nullptr) or writes.
struct Sink {
	uint8_t* w;
	uint32_t n;
	EBD_HD void put(uint32_t c) {
		if (w)
			w[n] = (uint8_t)c;
		n++;
	}
	EBD_HD void str(const char* s) {
		while (*s)
			put((uint8_t)*s++);
	}
	EBD_HD void dec(uint32_t v) {
		char b[10];
		int k = 0;
		do {
			b[k++] = (char)('0' + v % 10);
			v /= 10;
		} while (v);
		while (k)
			put((uint8_t)b[--k]);
	}
	EBD_HD void hex(uint32_t v) {
		char b[8];
		int k = 0;
		do {
			b[k++] = "0123456789abcdef"[v & 15];
			v >>= 4;
		} while (v);
		while (k)
			put((uint8_t)b[--k]);
	}
};

struct GenDraws {
	uint32_t u[16];
};

EBD_HD void gen_draws(uint64_t seed, uint32_t config, uint64_t idx, uint32_t stream, GenDraws& d) {
	for (uint32_t k = 0; k < 4; k++)
		Philox::gen((uint32_t)idx, (uint32_t)(idx >> 32), stream * 4 + k, config, (uint32_t)seed, (uint32_t)(seed >> 32), d.u + 4 * k);
}

// fixed 64-byte GET, one endpoint.
template <typename Out>
EBD_HD void compose_fixed64(Out& s) { s.str("GET /index.html HTTP/1.1\r\nHost: 10.0.0.1:8080\r\nAccept: */*xx\r\n\r\n"); }

EBD_HD const char* path_segment(uint32_t k) {
	switch (k & 15) {
	case 0: return "api";
	case 1: return "v1";
	case 2: return "v2";
	case 3: return "users";
	case 4: return "orders";
	case 5: return "static";
	case 6: return "img";
	case 7: return "search";
	case 8: return "cart";
	case 9: return "auth";
	case 10: return "assets";
	case 11: return "docs";
	case 12: return "blog";
	case 13: return "shop";
	case 14: return "media";
	default: return "feed";
	}
}

template <typename Out>
EBD_HD void put_path(Out& s, uint32_t k) {
	s.put('/');
	s.str(path_segment(k));
	s.put('/');
	s.str(path_segment(k >> 4));
	s.str("/item");
	s.dec(k);
	if (k % 3 == 0) {
		s.str("?id=");
		s.dec((k * 7) % 1000);
	}
}

template <typename Out>
EBD_HD void put_host(Out& s, uint32_t j) {
	switch (j & 3) {
	case 0:
		s.str("svc");
		s.dec(j);
		s.str(".example.com");
		break;
	case 1:
		s.str("svc");
		s.dec(j);
		s.str(".example.com:8080");
		break;
	case 2:
		s.str("10.");
		s.dec(j >> 8);
		s.put('.');
		s.dec(j & 255);
		s.str(".7:");
		s.dec(8000 + j % 100);
		break;
	default:
		s.str("[fd00::");
		s.hex(j);
		s.str("]:8443");
		break;
	}
}

template <typename Out>
EBD_HD void put_v4(Out& s, uint32_t r) {
	// first octet from a mix of internal (10, 172.16, 192.168, 127) and external ranges
	// {10, 172, 192, 127, 8, 34, 52, 81, 93, 104, 151, 185, 203, 66, 23, 100} packed by byte
	const uint64_t lo = 0x51342208'7fc0ac0aull, hi = 0x641742cb'b997685dull;
	const uint32_t sel = r & 15;
	const uint32_t f = (uint32_t)(((sel < 8 ? lo : hi) >> (8 * (sel & 7))) & 255);
	uint32_t b = (r >> 4) & 255;
	if (f == 172)
		b = 16 + (b & 15);
	if (f == 192)
		b = 168;
	s.dec(f);
	s.put('.');
	s.dec(b);
	s.put('.');
	s.dec((r >> 12) & 255);
	s.put('.');
	s.dec((r >> 20) & 255);
}

template <typename Out>
EBD_HD void put_v6(Out& s, uint32_t r) {
	switch (r & 3) {
	case 0: s.str("2001:db8:"); break;
	case 1: s.str("fd00:"); break;
	case 2: s.str("2606:4700:"); break;
	default: s.str("fe80:"); break;
	}
	s.put(':');
	s.hex((r >> 2) & 0xffff);
	s.put(':');
	s.hex(r >> 18);
}

// Client-IP header value forms (HttpRequestParserTest.cpp:75-150 shapes).
template <typename Out>
EBD_HD void put_cip_value(Out& s, uint32_t r0, uint32_t r1) {
	switch (r0 % 7) {
	case 0: put_v4(s, r1); break;
	case 1:
		put_v4(s, r1);
		s.put(':');
		s.dec(1024 + (r0 >> 8) % 50000);
		break;
	case 2: put_v6(s, r1); break;
	case 3:
		s.put('[');
		put_v6(s, r1);
		s.str("]:");
		s.dec(1024 + (r0 >> 8) % 50000);
		break;
	case 4:
		s.put('[');
		put_v6(s, r1);
		s.put(']');
		break;
	case 5:
		put_v4(s, r1);
		s.str(", ");
		put_v4(s, r1 * 2654435761u);
		break;
	default: // a leading-zero octet: inet_pton rejects it (no count)
		s.str("01.");
		s.dec(r1 & 255);
		s.str(".1.1");
		break;
	}
}

EBD_HD const char* cip_key(uint32_t k, bool title) {
	switch (k % 5) {
	case 0: return title ? "Rproxy_Remote_Address" : "rproxy_remote_address";
	case 1: return title ? "True-Client-IP" : "true-client-ip";
	case 2: return title ? "X-Client-IP" : "x-client-ip";
	case 3: return title ? "X-Forwarded-For" : "x-forwarded-for";
	default: return title ? "X-HTTP-Client-IP" : "x-http-client-ip";
	}
}

struct MixedReq {
	uint32_t target, path, host, pid, post, cip, cipkey, ciptitle, cipr0, cipr1, body, inval, invpos;
};

EBD_HD void mixed_params(const GenTables& T, const GenDraws& d, MixedReq& q) {
	q.target = kLenMin + cdf_sample(T.len_cdf, kLenN, d.u[0]);
	q.post = (d.u[1] % 100) < 10;
	q.path = cdf_sample(T.path_cdf, kPaths, d.u[2]);
	q.host = cdf_sample(T.host_cdf, kHosts, d.u[3]);
	q.pid = 2000 + d.u[4] % kPids;
	q.cip = (d.u[5] % 100) < 30;
	q.cipkey = (d.u[5] >> 8) % 5;
	q.ciptitle = (d.u[5] >> 12) & 1;
	q.cipr0 = d.u[6];
	q.cipr1 = d.u[7];
	q.body = q.post ? 16 + d.u[14] % 48 : 0;
	q.inval = (d.u[13] % 1000) < 10;
	q.invpos = d.u[13] >> 10;
}

// SURVEY 8(d) config 3 request: request line, Host, optional client-IP header,
// User-Agent padding to the sampled length, Accept, end of headers, POST body.
template <typename Out>
EBD_HD void compose_mixed(Out& s, const MixedReq& q) {
	const uint32_t start = s.n;
	s.str(q.post ? "POST " : "GET ");
	put_path(s, q.path);
	s.str(" HTTP/1.1\r\nHost: ");
	put_host(s, q.host);
	s.str("\r\n");
	if (q.cip) {
		s.str(cip_key(q.cipkey, q.ciptitle));
		s.str(": ");
		put_cip_value(s, q.cipr0, q.cipr1);
		s.str("\r\n");
	}
	s.str("User-Agent: ");
	// fixed part after the UA value: "\r\nAccept: */*\r\n\r\n" (17) + body
	const uint32_t used = s.n - start + 17 + q.body;
	const uint32_t ua = q.target > used + 1 ? q.target - used : 1;
	const char* pat = "Mozilla/5.0 (X11; Linux x86_64) AppleWebKit/537.36 Chrome/120.0 Safari/537.36 "; // 78 chars
	for (uint32_t k = 0; k < ua; k++)
		s.put((uint8_t)pat[k % 78]);
	s.str("\r\nAccept: */*\r\n\r\n");
	for (uint32_t k = 0; k < q.body; k++)
		s.put((uint8_t)('a' + k % 26));
}

constexpr uint8_t FLAG4 = 2, FLAG6 = 4, FLAG_PLAIN = 8, FLAG_SSL = 16, FLAG_NEW = 32, FLAG_END = 64;

struct EventRec { // mirrors ebd_discovery_event (36 bytes)
	uint32_t pid, fd, sessionID, bufferSeq;
	uint8_t sourceIP[16];
	uint8_t flags;
	uint8_t pad[3];
};
static_assert(sizeof(EventRec) == 36, "DiscoveryEvent is 36 bytes");

EBD_HD void mixed_event(const GenDraws& d, const MixedReq& q, uint64_t idx, EventRec& e) {
	e.pid = q.pid;
	e.fd = 5 + (uint32_t)(idx % 1000);
	e.sessionID = (uint32_t)(idx + 1);
	e.bufferSeq = 1;
	const bool v6 = (d.u[8] % 100) < 20;
	const bool ssl = ((d.u[8] >> 8) % 100) < 15;
	e.flags = (uint8_t)((v6 ? FLAG6 : FLAG4) | (ssl ? FLAG_SSL : FLAG_PLAIN) | FLAG_NEW);
	for (int k = 0; k < 16; k++)
		e.sourceIP[k] = 0;
	const uint32_t w[4] = {d.u[9], d.u[10], d.u[11], d.u[12]};
	if (!v6) {
		for (int k = 0; k < 4; k++)
			e.sourceIP[k] = (uint8_t)(w[0] >> (8 * k));
	} else {
		for (int k = 0; k < 16; k++)
			e.sourceIP[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
		const uint32_t sel = d.u[15] & 3; // fd00::/8 (internal), 2001:db8 (external), ::ffff:a.b.c.d, fe80::/10
		if (sel == 0)
			e.sourceIP[0] = 0xfd;
		else if (sel == 1) {
			e.sourceIP[0] = 0x20;
			e.sourceIP[1] = 0x01;
		} else if (sel == 2) {
			for (int k = 0; k < 10; k++)
				e.sourceIP[k] = 0;
			e.sourceIP[10] = e.sourceIP[11] = 0xff;
		} else {
			e.sourceIP[0] = 0xfe;
			e.sourceIP[1] = (uint8_t)(0x80 | (e.sourceIP[1] & 0x3f));
		}
	}
	e.pad[0] = e.pad[1] = e.pad[2] = 0;
}

// Single-buffer configs: 1 (35-B literal), 11 (its 31-B variant), 2 (fixed 64 B), 3 (mixed).
// Returns the buffer length; writes bytes when out != nullptr.
EBD_HD uint32_t gen_single(const GenTables* T, uint32_t config, uint64_t seed, uint64_t idx, EventRec* ev, uint8_t* out) {
	Sink s{out, 0};
	if (config == 1 || config == 11) {
		s.str(config == 1 ? "GET / HTTP/1.1\r\nHost: 127.0.0.1\r\n\r\n" : "GET / HTTP/1.1\r\nHost: 127.0.0.1");
		if (ev) {
			*ev = EventRec{};
			ev->pid = 1000;
			ev->fd = 5;
			ev->sessionID = (uint32_t)(idx + 1);
			ev->bufferSeq = 1;
			ev->flags = FLAG4 | FLAG_PLAIN | FLAG_NEW;
			ev->sourceIP[0] = 127;
			ev->sourceIP[3] = 1;
		}
		return s.n;
	}
	GenDraws d;
	gen_draws(seed, config, idx, 0, d);
	if (config == 2) {
		compose_fixed64(s);
		if (ev) {
			*ev = EventRec{};
			ev->pid = 4242;
			ev->fd = 5;
			ev->sessionID = (uint32_t)(idx + 1);
			ev->bufferSeq = 1;
			ev->flags = FLAG4 | FLAG_PLAIN | FLAG_NEW;
			for (int k = 0; k < 4; k++)
				ev->sourceIP[k] = (uint8_t)(d.u[0] >> (8 * k));
		}
		return s.n;
	}
	MixedReq q;
	mixed_params(*T, d, q);
	compose_mixed(s, q);
	if (out && q.inval) { // ~1 % of requests get an invalid byte in the header section
		const uint32_t hdr = s.n - q.body;
		out[q.invpos % hdr] = 0x01;
	}
	if (ev)
		mixed_event(d, q, idx, *ev);
	return s.n;
}

EBD_HD uint64_t align_up(uint64_t x, uint32_t a) { return (x + a - 1) & ~(uint64_t)(a - 1); }

// ---------------------------------------------------------------------------------
// config-3 requests (seed 4) cut into 2-4 consecutive recv() events
// (the first >= 16 bytes, so it still starts "GET /" or "POST /", DataFunctions.h:45-50; a
// POST body stays in the last piece), 1-8 keep-alive requests per connection, then a
// DATA_END event.  kSlots4 connections are open at a time and interleaved round robin:
// event position p = round * kSlots4 + slot, each slot running its connections j = 0, 1, ...
// back to back.  So at most kSlots4 (<= 8192) sessions are ever live and the LRU never
// evicts.  Connection j of a slot is cid = j * kSlots4 + slot (independent of the trace
// length, so a longer trace extends a shorter one).
// ---------------------------------------------------------------------------------
constexpr uint32_t kSlots4 = 4096, kMaxReq4 = 8;

struct Conn4 {
	uint32_t nreq, flags, pid, fd, sid;
	uint32_t kfrag[kMaxReq4];
	uint8_t src[16];
};

EBD_HD void conn4(uint64_t seed, uint64_t cid, Conn4& c) {
	GenDraws d;
	gen_draws(seed, 4, cid, 8, d); // stream 8: connection draws (streams 0.. are per request)
	c.nreq = 1 + d.u[0] % kMaxReq4;
	const bool v6 = (d.u[1] % 100) < 20, ssl = ((d.u[1] >> 8) % 100) < 15;
	c.flags = (v6 ? FLAG6 : FLAG4) | (ssl ? FLAG_SSL : FLAG_PLAIN);
	c.pid = 2000 + d.u[2] % kPids;
	c.fd = 5 + (uint32_t)(cid % 1000);
	c.sid = (uint32_t)(cid + 1);
	for (int k = 0; k < 16; k++)
		c.src[k] = 0;
	if (!v6) {
		for (int k = 0; k < 4; k++)
			c.src[k] = (uint8_t)(d.u[3] >> (8 * k));
	} else {
		for (int k = 0; k < 16; k++)
			c.src[k] = (uint8_t)(d.u[3 + (k >> 2)] >> (8 * (k & 3)));
		if (d.u[15] & 1) { // half external 2001:db8::/32, half internal fd00::/8
			c.src[0] = 0x20;
			c.src[1] = 0x01;
			c.src[2] = 0x0d;
			c.src[3] = 0xb8;
		} else {
			c.src[0] = 0xfd;
		}
	}
	for (uint32_t q = 0; q < kMaxReq4; q++)
		c.kfrag[q] = 2 + d.u[7 + q] % 3;
}

EBD_HD uint32_t conn4_events(const Conn4& c) {
	uint32_t e = 1; // DATA_END
	for (uint32_t q = 0; q < c.nreq; q++)
		e += c.kfrag[q];
	return e;
}

// Request q of connection cid: its config-3 content, its length and its cut points
// cut[0] = 0 < cut[1] < ... < cut[k] = length.
struct Req4 {
	MixedReq m;
	uint32_t len, hdr, k;
	uint32_t cut[5];
};

EBD_HD void req4(const GenTables& T, uint64_t seed, uint64_t cid, uint32_t q, uint32_t kfrag, Req4& r) {
	GenDraws d;
	gen_draws(seed, 4, cid * kMaxReq4 + q, 0, d);
	mixed_params(T, d, r.m);
	Sink s{nullptr, 0};
	compose_mixed(s, r.m);
	r.len = s.n;
	r.hdr = s.n - r.m.body; // header section: the cuts stay in it
	const uint32_t span = r.hdr > 16 ? r.hdr - 16 : 0;
	r.k = kfrag; // span >= 50 > 4: every request carries its request line, Host, User-Agent and Accept
	r.cut[0] = 0;
	for (uint32_t f = 1; f < r.k; f++) { // one cut per k-th of [16, hdr), jittered inside it
		const uint32_t seg = span / r.k;
		r.cut[f] = 16 + (span * f) / r.k - (seg ? d.u[15 - f] % seg : 0) / 2;
	}
	r.cut[r.k] = r.len;
}

// Writes the request's bytes into its pieces: byte b of the request goes to piece f with
// cut[f] <= b < cut[f + 1], at dst[f] + (b - cut[f]).
struct SplitSink {
	uint8_t* dst[4];
	uint32_t cut[5];
	uint32_t k, n;
	EBD_HD void put(uint32_t c) {
		uint32_t f = 0;
		while (f + 1 < k && n >= cut[f + 1])
			f++;
		if (dst[f]) // a piece past the trace's end is not written
			dst[f][n - cut[f]] = (uint8_t)c;
		n++;
	}
	EBD_HD void str(const char* s) {
		while (*s)
			put((uint8_t)*s++);
	}
	EBD_HD void dec(uint32_t v) {
		char b[10];
		int m = 0;
		do {
			b[m++] = (char)('0' + v % 10);
			v /= 10;
		} while (v);
		while (m)
			put((uint8_t)b[--m]);
	}
	EBD_HD void hex(uint32_t v) {
		char b[8];
		int m = 0;
		do {
			b[m++] = "0123456789abcdef"[v & 15];
			v >>= 4;
		} while (v);
		while (m)
			put((uint8_t)b[--m]);
	}
};

// The request's pieces into their buffers (dst[f], length cut[f + 1] - cut[f]); ~1 % of
// requests carry an invalid byte in the header section, as in config 3.
EBD_HD void write_req4(const Req4& r, uint8_t* const* dst) {
	SplitSink s;
	for (uint32_t f = 0; f < 4; f++)
		s.dst[f] = f < r.k ? dst[f] : nullptr;
	for (uint32_t f = 0; f <= r.k; f++)
		s.cut[f] = r.cut[f];
	s.k = r.k;
	s.n = 0;
	compose_mixed(s, r.m);
	if (r.m.inval) {
		const uint32_t b = r.m.invpos % r.hdr;
		uint32_t f = 0;
		while (f + 1 < r.k && b >= r.cut[f + 1])
			f++;
		if (dst[f])
			dst[f][b - r.cut[f]] = 0x01;
	}
}

// Event e (0-based) of connection cid: request q and piece f of it, or the DATA_END event
// (q = nreq).  bufferSeq counts the connection's data events from 1 (Handlers.h:121-125).
EBD_HD void conn4_event(const Conn4& c, uint32_t e, uint32_t* q, uint32_t* f) {
	uint32_t at = 0;
	for (uint32_t k = 0; k < c.nreq; k++) {
		if (e < at + c.kfrag[k]) {
			*q = k;
			*f = e - at;
			return;
		}
		at += c.kfrag[k];
	}
	*q = c.nreq;
	*f = 0;
}

// Visits the events of connection task t = slot * J + j (slot-major, so that a scan of the
// per-task event counts gives each connection's first round): fn(position, conn, request
// (nullptr for DATA_END), piece, event number).  r0: the connection's first round.
template <typename Fn>
EBD_HD void conn4_visit(const GenTables& T, uint64_t seed, uint32_t slot, uint32_t j, uint64_t r0, uint64_t n, Fn fn) {
	Conn4 c;
	const uint64_t cid = (uint64_t)j * kSlots4 + slot;
	conn4(seed, cid, c);
	uint64_t e = 0;
	for (uint32_t q = 0; q < c.nreq; q++) {
		const uint64_t p0 = (r0 + e) * kSlots4 + slot;
		if (p0 >= n)
			return;
		Req4 r;
		req4(T, seed, cid, q, c.kfrag[q], r);
		fn(p0, c, &r, (uint32_t)e);
		e += r.k;
	}
	const uint64_t pe = (r0 + e) * kSlots4 + slot;
	if (pe < n)
		fn(pe, c, (const Req4*)nullptr, (uint32_t)e);
}

EBD_HD void conn4_record(const Conn4& c, uint32_t e, bool end, EventRec& ev) {
	ev.pid = c.pid;
	ev.fd = c.fd;
	ev.sessionID = c.sid;
	ev.bufferSeq = end ? e : e + 1;
	for (int k = 0; k < 16; k++)
		ev.sourceIP[k] = end ? 0 : c.src[k];
	ev.flags = (uint8_t)(end ? FLAG_END : (c.flags | FLAG_NEW));
	ev.pad[0] = ev.pad[1] = ev.pad[2] = 0;
}

// Shard of a connection (pid, fd, sessionID) among `count` GPUs: every
// event of a connection lands on one GPU, so parser sessions never cross GPUs.  Same
// function as ebd/shard.py connection_hash.
EBD_HD uint32_t conn_shard(uint32_t pid, uint32_t fd, uint32_t sid, uint32_t count) {
	const uint64_t kv = (uint64_t)pid | ((uint64_t)fd << 32);
	return count <= 1 ? 0u : (uint32_t)(fmix64(kv ^ ((uint64_t)sid * 0x9E3779B97F4A7C15ull)) % count);
}

// Event `idx` of a single-buffer config kept by shard `index` of `count`?  Its length when
// kept (0 when not: a kept event is never empty).
EBD_HD uint32_t gen_single_shard(const GenTables* T, uint32_t config, uint64_t seed, uint64_t idx, uint32_t count,
		uint32_t index, EventRec* ev, uint8_t* out) {
	if (count <= 1)
		return gen_single(T, config, seed, idx, ev, out);
	EventRec e;
	const uint32_t L = gen_single(T, config, seed, idx, &e, nullptr);
	if (conn_shard(e.pid, e.fd, e.sessionID, count) != index)
		return 0;
	if (ev || out)
		gen_single(T, config, seed, idx, ev, out);
	return L;
}

} // namespace ebd
