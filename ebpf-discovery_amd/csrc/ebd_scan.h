// ebd_scan.h — the fast path as a structural scan: HttpRequestParser::parse of one buffer by
// a fresh parser (Discovery.cpp:141-159 handleNewSession), computed from delimiter positions
// instead of a byte-at-a-time state machine.  Written once for the GPU kernel (k_fresh: the
// buffer sits in an LDS tile, ebd_kernels.hip) and its host twin (ebd_host_scan).
//
// A fresh parse of a buffer is a short sequence of spans, each with one byte class
// (P = libhttpparser/src/HttpRequestParser.cpp):
//   "GET /" | "POST /"                        P:162-199  (any other byte: INVALID there)
//   URL bytes, then ' '                        P:201-213  class U (C_URL)
//   "HTTP/1.0" | "HTTP/1.1", CR, LF            P:215-262
//   per header line:  key ':' SP* value CR LF  P:264-352  key class K, value V / H / C
//   CR LF                                      P:264-267, P:354-364
// so the result is fixed by the first byte of each span that leaves the span's class.  The
// scan finds those bytes span by span:
//   * header values of other keys (the bulk of a request: User-Agent, Accept ...) need only
//     the first byte outside [0x20, 0x7e] (class V is exactly the printable bytes, P:33).
//     Those bytes are located once per 16-byte piece for the whole tile, by every lane of the
//     wave over consecutive pieces (nv4 + __ballot: one bit per piece, `nvword`), so a value
//     of any length costs one bitmap word and one piece;
//   * the short spans (URL, keys, Host and client-IP values) are tested against per-byte class
//     bitmaps, also built once per tile by the whole wave (a class-table lookup per byte and
//     v_dot4_u32_u8 to gather the bits), so a span of up to 64 bytes costs one bitmap word.
// The spans are taken in stream order and each search ends at the first byte outside its
// class, so the first such byte of the whole request is the one the reference stops at: the
// result is exact.  One shape is left to the generic parser (scan_slow): a header key that
// holds a space (P:268-270 skips it, which changes the key the Host / client-IP tests see).
#pragma once

#include "../../include/ebpf_discovery_amd.h"
#include "ebd_spec.h"

namespace ebd {

// SWAR over 4 bytes: bit 7 of every byte outside [0x20, 0x7e], the bytes that are not C_VAL
// (P:33, P:47-65 in the C locale; bytes >= 0x80 are in no class).  Exact per byte: the low 7
// bits plus 0x60 (0x01) carry into bit 7 exactly when they are >= 0x20 (== 0x7f).
EBD_HD uint32_t nv4(uint32_t w) {
	const uint32_t y = w & 0x7f7f7f7fu;
	return (w | ~(y + 0x60606060u) | (y + 0x01010101u)) & 0x80808080u;
}

// First flagged byte at or after byte lo of a 16-byte piece given as four nv4 words; 16 if none.
EBD_HD uint32_t first_flag16(uint32_t f0, uint32_t f1, uint32_t f2, uint32_t f3, uint32_t lo) {
	unsigned long long a = f0 | ((unsigned long long)f1 << 32), b = f2 | ((unsigned long long)f3 << 32);
	a &= lo >= 8 ? 0ull : (~0ull << (8 * lo));
	b &= lo <= 8 ? ~0ull : (~0ull << (8 * (lo - 8)));
	return a ? ((uint32_t)__builtin_ctzll(a) >> 3) : b ? 8u + ((uint32_t)__builtin_ctzll(b) >> 3) : 16u;
}

// Bit numbers of the classes in the inverted class table (ncls[b] = ~byte_class(b)).
enum : uint32_t { NB_URL = 0, NB_KEY = 1, NB_VAL = 2, NB_HOST = 3, NB_CIP = 4 };
static_assert(C_URL == 1u << NB_URL && C_KEY == 1u << NB_KEY && C_VAL == 1u << NB_VAL && C_HOST == 1u << NB_HOST &&
				C_CIP == 1u << NB_CIP,
		"class bits");

// The source of a scan (tile coordinates: the buffer is bytes [B, B + L)):
//   byte(p), dw(p) (4 bytes at any p), ld8(p), piece(pc, w) (bytes [16 pc, 16 pc + 16)),
//   nvword(j) (bit i: piece 64 j + i holds a byte outside [0x20, 0x7e]), ncls(b),
//   clsword(c, a) (the class bitmaps below).
// Bytes past the buffer are whatever the tile holds there; every search is bounded by E.

// Class bitmaps of the tile: bit b of word clsword(c, a) is set where tile byte 64 a + b is
// NOT in class c (c = CB_KEY, CB_HOST, CB_CIP; the URL, one span per buffer, is looked up
// byte by byte: class_search).  They are built once per tile by every
// lane over consecutive pieces (class_masks16), so a search costs one word per 64 bytes.
enum : uint32_t { CB_KEY = 0, CB_HOST = 1, CB_CIP = 2, CB_N = 3 };

// The 16-bit "not in class" masks of one 16-byte piece for the four classes, from the inverted
// class bytes packed four to a word (f[j] byte i = ncls of piece byte 4 j + i): bit n of the
// class's byte goes to bit 4 j + i by v_dot4_u32_u8 against the weights 1, 2, 4, 8 (and 16 ..
// 128 for the next word).
EBD_HD uint32_t dot4u8(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
	return __builtin_amdgcn_udot4(a, b, c, false);
#else
	for (int i = 0; i < 4; i++)
		c += ((a >> (8 * i)) & 0xffu) * ((b >> (8 * i)) & 0xffu);
	return c;
#endif
}
EBD_HD uint32_t class_mask16(const uint32_t (&f)[4], uint32_t nb) {
	const uint32_t sel = 0x01010101u << nb;
	const uint32_t lo = dot4u8(f[0] & sel, 0x08040201u, dot4u8(f[1] & sel, 0x80402010u, 0u));
	const uint32_t hi = dot4u8(f[2] & sel, 0x08040201u, dot4u8(f[3] & sel, 0x80402010u, 0u));
	return (lo | (hi << 8)) >> nb;
}

// A piece's class masks (mask bit i: piece byte i is not in the class), from its words.
template <typename Src>
EBD_HD void piece_classes(const Src& s, const uint32_t (&w)[4], uint32_t (&m)[CB_N]) {
	uint32_t f[4];
#pragma unroll
	for (uint32_t j = 0; j < 4; j++) {
		const uint32_t x = w[j];
		f[j] = s.ncls(x & 0xffu) | (s.ncls((x >> 8) & 0xffu) << 8) | (s.ncls((x >> 16) & 0xffu) << 16) | (s.ncls(x >> 24) << 24);
	}
	m[CB_KEY] = class_mask16(f, NB_KEY);
	m[CB_HOST] = class_mask16(f, NB_HOST);
	m[CB_CIP] = class_mask16(f, NB_CIP);
}

// First position in [p, e) whose byte is not in class c; e if none (P:47-65).
template <typename Src>
EBD_HD uint32_t first_not(const Src& s, uint32_t p, uint32_t e, uint32_t c) {
	if (p >= e)
		return e;
	uint32_t a = p >> 6;
	unsigned long long w = s.clsword(c, a) & (~0ull << (p & 63u));
	while (!w) {
		a++;
		if (64 * a >= e)
			return e;
		w = s.clsword(c, a);
	}
	const uint32_t r = 64 * a + (uint32_t)__builtin_ctzll(w);
	return r < e ? r : e;
}

// First position in [p, e) whose byte is outside [0x20, 0x7e]; e if none.  Pieces without
// such a byte are skipped 64 at a time through the tile's piece bitmap.
template <typename Src>
EBD_HD uint32_t first_nv(const Src& s, uint32_t p, uint32_t e) {
	uint32_t pc = p >> 4;
	while (16 * pc < e) {
		const uint32_t j = pc >> 6;
		const unsigned long long wd = s.nvword(j) & (~0ull << (pc & 63u));
		if (!wd) {
			pc = (j + 1) << 6;
			continue;
		}
		pc = (j << 6) + (uint32_t)__builtin_ctzll(wd);
		if (16 * pc >= e)
			break;
		uint32_t w[4];
		s.piece(pc, w);
		const uint32_t f = first_flag16(nv4(w[0]), nv4(w[1]), nv4(w[2]), nv4(w[3]), 16 * pc < p ? (p & 15u) : 0u);
		if (f < 16) {
			const uint32_t r = 16 * pc + f;
			return r < e ? r : e;
		}
		pc++;
	}
	return e;
}

// First byte at or after p not in class nb (ncls bit), from the class table byte by byte over
// at most NP pieces: r (<= e).  False: none in them and the buffer goes on past them.
template <uint32_t NP, typename Src>
EBD_HD bool class_search(const Src& s, uint32_t p, uint32_t e, uint32_t nb, uint32_t& r) {
	const uint32_t sel = 0x01010101u << nb;
	uint32_t pc = p >> 4, lo = p & 15u;
#pragma unroll
	for (uint32_t i = 0; i < NP; i++) {
		uint32_t w[4], f[4];
		s.piece(pc, w);
#pragma unroll
		for (uint32_t j = 0; j < 4; j++) {
			const uint32_t x = w[j];
			f[j] = (s.ncls(x & 0xffu) | (s.ncls((x >> 8) & 0xffu) << 8) | (s.ncls((x >> 16) & 0xffu) << 16) |
						   (s.ncls(x >> 24) << 24)) &
					sel;
		}
		const uint32_t k = first_flag16(f[0], f[1], f[2], f[3], lo);
		if (k < 16) {
			const uint32_t x = 16 * pc + k;
			r = x < e ? x : e;
			return true;
		}
		pc++;
		lo = 0;
		if (16 * pc >= e) {
			r = e;
			return true;
		}
	}
	r = e;
	return false;
}

// 4 bytes of a literal (little-endian), and its letter bytes (0x20 each): a key byte b
// matches a lower-case letter c iff (b | 0x20) == c (P:280 lower-cases with tolower, which
// only changes 'A'..'Z'), and any other literal byte only by itself.
constexpr uint32_t lit_word(const char* s, uint32_t n, uint32_t i) {
	uint32_t w = 0;
	for (uint32_t k = 0; k < 4; k++)
		if (4 * i + k < n)
			w |= (uint32_t)(uint8_t)s[4 * i + k] << (8 * k);
	return w;
}
constexpr uint32_t lit_letters(const char* s, uint32_t n, uint32_t i) {
	uint32_t m = 0;
	for (uint32_t k = 0; k < 4; k++)
		if (4 * i + k < n && s[4 * i + k] >= 'a' && s[4 * i + k] <= 'z')
			m |= 0x20u << (8 * k);
	return m;
}
constexpr uint32_t lit_valid(uint32_t n, uint32_t i) {
	return 4 * i + 4 <= n ? 0xffffffffu : 4 * i >= n ? 0u : (0xffffffffu >> (8 * (4 * i + 4 - n)));
}

// The first n bytes of the key (kd: its first 24 bytes) equal the lower-case literal s.
template <uint32_t N>
EBD_HD bool key_is(const uint32_t (&kd)[6], const char (&s)[N]) {
	constexpr uint32_t n = N - 1;
	uint32_t x = 0;
#pragma unroll
	for (uint32_t i = 0; i < (n + 3) / 4; i++)
		x |= ((kd[i] | lit_letters(s, n, i)) ^ lit_word(s, n, i)) & lit_valid(n, i);
	return x == 0;
}

enum : uint32_t { SK_OTHER = 0, SK_HOST = 1, SK_CLIENT = 2 };

// currentHeader.key lower-cased and cut at 21 bytes (P:276-281, kMaxHeaderKeyLength P:44)
// against "host" (P:366-368) and the client-IP keys (P:43, P:370-372).  The key has no space
// here (scan_event leaves such keys to scan_slow), so it is bytes [q, q + n); only a key of
// a matching length reads its words.
template <typename Src>
EBD_HD uint32_t key_type(const Src& s, uint32_t q, uint32_t n) {
	uint32_t kd[6];
	if (n == 4) {
		kd[0] = s.dw(q);
		return key_is(kd, "host") ? SK_HOST : SK_OTHER;
	}
	if (n != 11 && (n < 14 || n > 16) && n < kMaxHeaderKeyLength)
		return SK_OTHER;
#pragma unroll
	for (uint32_t i = 0; i < 4; i++)
		kd[i] = s.dw(q + 4 * i);
	bool c;
	if (n < kMaxHeaderKeyLength) {
		c = n == 11 ? key_is(kd, "x-client-ip")
				: n == 14 ? key_is(kd, "true-client-ip")
				: n == 15 ? key_is(kd, "x-forwarded-for")
						  : key_is(kd, "x-http-client-ip");
	} else { // truncated to 21: only the 21-byte key can match
		kd[4] = s.dw(q + 16);
		kd[5] = s.dw(q + 20);
		c = key_is(kd, "rproxy_remote_address");
	}
	return c ? SK_CLIENT : SK_OTHER;
}

// The outcome of a fresh parse of one buffer (positions relative to the buffer).
struct ScanOut {
	uint32_t status;   // EBD_STATUS_UNFINISHED / FINISHED / INVALID
	uint32_t consumed; // HttpRequestParser::parse's return (P:85-106)
	uint32_t url_off, url_len, host_off, host_len, cip_off;
	uint32_t info; // EBD_INFO_POST | EBD_INFO_CIP of a FINISHED request
	uint32_t slow; // a header key holds a space: scan_slow decides
};

EBD_HD void scan_init(ScanOut& o, uint32_t L) {
	o.status = EBD_STATUS_UNFINISHED;
	o.consumed = L;
	o.url_off = o.url_len = o.host_off = o.host_len = o.cip_off = 0;
	o.info = 0;
	o.slow = 0;
}

// P:85-106 for a fresh parser over bytes [B, B + L) (L <= 8192, so the 8193-byte cap at
// P:88-91 cannot trigger).  INVALID consumes the byte that failed, FINISHED the final LF,
// an unfinished parse the whole buffer.  The request line and Host/URL spans of a FINISHED
// request are filled in; a request with a client-IP header gets the raw value start of the
// first one (P:309-316: for a fresh parser the first client-IP key sets clientIPKey, so its
// header is the one parsed into clientIp; the token is k_agg_fast's, as on the DFA path).
template <typename Src>
EBD_HD void scan_event(const Src& s, uint32_t B, uint32_t L, ScanOut& o) {
	scan_init(o, L);
	if (L == 0)
		return;
	const uint32_t E = B + L;
	// P:162-199: the method must stay a prefix of GET / POST until its space, then '/'
	const bool post = s.byte(B) == 'P';
	const uint32_t nm = post ? 6u : 5u; // "POST /" | "GET /"
	{
		const unsigned long long x = (unsigned long long)s.dw(B) | ((unsigned long long)s.dw(B + 4) << 32);
		const unsigned long long lit = post ? 0x2f2054534f50ull : 0x2f20544547ull;
		const unsigned long long d = (x ^ lit) & (nm == 6 ? 0xffffffffffffull : 0xffffffffffull);
		const uint32_t k = d ? ((uint32_t)__builtin_ctzll(d) >> 3) : nm;
		if (k < nm && k < L) {
			o.status = EBD_STATUS_INVALID;
			o.consumed = k + 1;
			return;
		}
		if (L < nm)
			return;
	}
	// P:201-213: URL bytes until the space
	const uint32_t u0 = B + nm - 1; // the '/'
	uint32_t ue = E;
	for (uint32_t p = u0 + 1; p < E;) { // the URL: class_search 4 pieces at a time
		if (class_search<4>(s, p, E, NB_URL, ue))
			break;
		p = ((p >> 4) + 4) << 4;
	}
	if (ue >= E)
		return;
	if (s.byte(ue) != ' ') {
		o.status = EBD_STATUS_INVALID;
		o.consumed = ue - B + 1;
		return;
	}
	// P:215-262: "HTTP/1.0" | "HTTP/1.1", CR, LF
	uint32_t q = ue + 1;
	{
		const unsigned long long x = (unsigned long long)s.dw(q) | ((unsigned long long)s.dw(q + 4) << 32);
		const unsigned long long dx = (x ^ 0x302e312f50545448ull) & ~(1ull << 56); // '0' / '1' differ in bit 0
		const uint32_t dy = (s.dw(q + 8) ^ 0x0a0du) & 0xffffu;
		const uint32_t k = dx ? ((uint32_t)__builtin_ctzll(dx) >> 3) : dy ? 8u + ((uint32_t)__builtin_ctz(dy) >> 3) : 10u;
		const uint32_t avail = E - q;
		if (k < 10 && k < avail) {
			o.status = EBD_STATUS_INVALID;
			o.consumed = q + k - B + 1;
			return;
		}
		if (avail < 10)
			return;
	}
	q += 10;
	bool host_seen = false, cip_seen = false;
	uint32_t host_off = 0, host_len = 0, cip_off = 0;
	for (;;) {
		if (q >= E)
			return;
		// P:264-297 HEADER_KEY: key bytes up to ':' (a CR first ends the headers, P:265-267)
		const uint32_t ke = s.byte(q) == '\r' ? q : first_not(s, q, E, CB_KEY);
		if (ke >= E)
			return;
		const uint32_t ck = s.byte(ke);
		if (ck == '\r') { // P:354-364 HEADERS_END: LF finishes the request
			if (ke + 1 >= E)
				return;
			if (s.byte(ke + 1) != '\n') {
				o.status = EBD_STATUS_INVALID;
				o.consumed = ke + 1 - B + 1;
				return;
			}
			o.status = EBD_STATUS_FINISHED;
			o.consumed = ke + 1 - B + 1;
			o.url_off = nm - 1;
			o.url_len = ue - u0;
			o.host_off = host_off;
			o.host_len = host_len;
			o.cip_off = cip_off;
			o.info = (post ? EBD_INFO_POST : 0u) | (cip_seen ? EBD_INFO_CIP : 0u);
			return;
		}
		if (ck == ' ') { // P:268-270 skips it: the key is not its bytes
			o.slow = 1;
			return;
		}
		if (ck != ':') {
			o.status = EBD_STATUS_INVALID;
			o.consumed = ke - B + 1;
			return;
		}
		const uint32_t kt = key_type(s, q, ke - q);
		if (kt == SK_HOST && host_seen) { // P:282-287: a second Host
			o.status = EBD_STATUS_INVALID;
			o.consumed = ke - B + 1;
			return;
		}
		// P:299-319 SP_BEFORE_VALUE: spaces skipped, then a C_VAL byte (a CR fails: empty value)
		uint32_t v = ke + 1;
		{
			const uint32_t x = s.dw(v) ^ 0x20202020u; // the first non-space of the next 4 bytes
			if (x)
				v += (uint32_t)__builtin_ctz(x) >> 3;
			else
				for (v += 4; v < E && s.byte(v) == ' ';)
					v++;
		}
		if (v >= E)
			return;
		if ((s.ncls(s.byte(v)) >> NB_VAL) & 1u) {
			o.status = EBD_STATUS_INVALID;
			o.consumed = v - B + 1;
			return;
		}
		// P:321-352 HEADER_VALUE up to CR: other keys' bytes are C_VAL, i.e. printable, so their
		// CR is the first byte outside [0x20, 0x7e]; Host (C_HOST) and client-IP (C_CIP) values
		// also fail at their first byte outside their class before it
		const uint32_t w = first_nv(s, v + 1, E);
		if (kt != SK_OTHER) {
			const uint32_t h = first_not(s, v + 1, w, kt == SK_HOST ? CB_HOST : CB_CIP);
			if (h < w) {
				o.status = EBD_STATUS_INVALID;
				o.consumed = h - B + 1;
				return;
			}
		}
		if (w >= E)
			return;
		if (s.byte(w) != '\r') {
			o.status = EBD_STATUS_INVALID;
			o.consumed = w - B + 1;
			return;
		}
		if (w + 1 >= E) // P:248-262 HEADER_NEWLINE
			return;
		if (s.byte(w + 1) != '\n') {
			o.status = EBD_STATUS_INVALID;
			o.consumed = w + 1 - B + 1;
			return;
		}
		if (kt == SK_HOST) {
			host_seen = true;
			host_off = v - B;
			host_len = w - v;
		} else if (kt == SK_CLIENT && !cip_seen) {
			cip_seen = true;
			cip_off = v - B;
		}
		q = w + 2;
	}
}

// v_alignbyte_b32: bytes [k, k + 4) of hi:lo (k = 0..3)
EBD_HD uint32_t align_byte(uint32_t hi, uint32_t lo, uint32_t k) {
#if defined(__HIP_DEVICE_COMPILE__)
	return __builtin_amdgcn_alignbyte(hi, lo, k);
#else
	return (uint32_t)((((unsigned long long)hi << 32) | lo) >> (8 * k));
#endif
}

EBD_HD uint32_t ctz64_or(unsigned long long w, uint32_t none) { return w ? (uint32_t)__builtin_ctzll(w) : none; }

// First flagged byte of class bitmap c at or after p, within the two words from p's: r (<= e).
// False: neither word has one and the buffer goes on past them.
template <typename Src>
EBD_HD bool search2(const Src& s, uint32_t c, uint32_t p, uint32_t e, uint32_t& r) {
	const uint32_t a = p >> 6;
	const unsigned long long w0 = s.clsword(c, a) & (~0ull << (p & 63u)), w1 = s.clsword(c, a + 1);
	const uint32_t x = w0 ? 64 * a + ctz64_or(w0, 64) : 64 * (a + 1) + ctz64_or(w1, 64);
	r = x < e ? x : e;
	return (w0 | w1) != 0 || 64 * (a + 2) >= e;
}

// First byte outside [0x20, 0x7e] at or after p (<= e): the first flagged piece (piece bitmap)
// and, if its flags all lie before p, the next one.  False: not within two bitmap words.
template <typename Src>
EBD_HD bool nv_search2(const Src& s, uint32_t p, uint32_t e, uint32_t& r) {
	const uint32_t pc0 = p >> 4, j = pc0 >> 6;
	unsigned long long wd = s.nvword(j) & (~0ull << (pc0 & 63u));
	uint32_t jb = j;
	if (!wd) {
		jb = j + 1;
		wd = s.nvword(jb);
	}
	if (!wd) {
		r = e;
		return 1024 * (j + 2) >= e;
	}
	uint32_t pc = 64 * jb + (uint32_t)__builtin_ctzll(wd);
	uint32_t w[4];
	s.piece(pc, w);
	uint32_t f = first_flag16(nv4(w[0]), nv4(w[1]), nv4(w[2]), nv4(w[3]), 16 * pc < p ? (p & 15u) : 0u);
	if (f == 16) { // the flags of p's own piece lie before p: the next flagged piece of the word
		const unsigned long long wd2 = wd & (wd - 1);
		if (!wd2) {
			r = e;
			return 16 * (64 * jb + 64) >= e;
		}
		pc = 64 * jb + (uint32_t)__builtin_ctzll(wd2);
		s.piece(pc, w);
		f = first_flag16(nv4(w[0]), nv4(w[1]), nv4(w[2]), nv4(w[3]), 0u);
	}
	const uint32_t x = 16 * pc + f;
	r = x < e ? x : e;
	return true;
}

// Outcomes of a line or a request, first match wins (the order is the reference's byte order).
enum : uint32_t { SF_GO = 0, SF_UNF = 1, SF_FIN = 2, SF_INV = 3, SF_SLOW = 4 };

// ---------------------------------------------------------------------------------
// Lanes over header lines.  k_fresh's per-lane walk of a buffer, line after line, runs for the
// longest buffer of the wave and diverges on every line kind.  Instead the wave enumerates
// every LF of its tile (each one starts a candidate header line, LF + 1), parses each line in
// a lane of its own with straight-line code (scan_line: the P:264-352 handlers of one line),
// and each buffer's lane only parses its request line (scan_reqline) and folds the records
// of its lines in order (scan_fold): the first line that is not a complete "key: value CRLF"
// decides the outcome, and the cross-line rules are applied there: a second Host
// (P:282-287) and the first client-IP header (P:309-316).  Lines that start after a line that
// decided the outcome, or outside the buffer, are parsed but never folded.  A line the
// straight-line code cannot settle (SLOW: a space in its key, three spaces after ':', a key
// or Host / client-IP value longer than its two bitmap words) sends the buffer to scan_event.
// ---------------------------------------------------------------------------------
enum : uint32_t { LN_OK = 0, LN_FIN = 1, LN_INV = 2, LN_UNF = 3, LN_SLOW = 4 };

// A line's record: a = code | kt << 4 | start << 16 (the line's first byte; tile positions
// < 2^16); b = v | w << 16 for LN_OK (the value's first byte and its CR), else pos (the LF of
// LN_FIN, the failing byte of LN_INV).  An LN_OK line's ':' is start + key length, which for
// the one key that needs it (a second Host, P:282-287) is start + 4.
struct LineRec {
	uint32_t a, b;
};

template <typename Src>
EBD_HD LineRec scan_line(const Src& s, uint32_t q, uint32_t E) {
	uint32_t dec = SF_GO, pos = 0;
	auto decide = [&](bool c, uint32_t d, uint32_t p) {
		const bool t = dec == SF_GO && c;
		dec = t ? d : dec;
		pos = t ? p : pos;
	};
	uint32_t ke;
	const bool kok = search2(s, CB_KEY, q, E, ke); // a CR at q is not K: ke = q
	const uint32_t kr = ke < E ? ke : E;
	const uint32_t c4 = s.dw(kr), ck = c4 & 0xffu, c1 = (c4 >> 8) & 0xffu;
	const uint32_t kt = key_type(s, q, ke - q);
	const uint32_t nsp = ctz64_or(((c4 >> 8) ^ 0x202020u) & 0xffffffu, 24) >> 3;
	const uint32_t v = ke + 1 + nsp, bv = (c4 >> (8 * (nsp + 1))) & 0xffu;
	const uint32_t vs = (v < E ? v : E) + 1;
	uint32_t w;
	bool vok;
	if (kt == SK_OTHER)
		vok = nv_search2(s, vs, E, w);
	else
		vok = search2(s, kt == SK_HOST ? CB_HOST : CB_CIP, vs, E, w);
	const uint32_t w4 = s.dw(w < E ? w : E), cw = w4 & 0xffu, cw1 = (w4 >> 8) & 0xffu;
	decide(q >= E, LN_UNF, 0);
	decide(!kok, LN_SLOW, 0);
	decide(ke >= E, LN_UNF, 0);
	// P:265-267, P:354-364: a CR in the key ends the headers; LF finishes the request
	decide(ck == '\r' && ke + 1 >= E, LN_UNF, 0);
	decide(ck == '\r' && c1 == '\n', LN_FIN, ke + 1);
	decide(ck == '\r', LN_INV, ke + 1);
	decide(ck == ' ', LN_SLOW, 0); // P:268-270: the key skips it
	decide(ck != ':', LN_INV, ke);
	// P:299-319: spaces, then a C_VAL byte (bytes ke+1..ke+3 are in c4)
	decide(nsp == 3, LN_SLOW, 0);
	decide(v >= E, LN_UNF, 0);
	decide(bv < 0x20u || bv > 0x7eu, LN_INV, v);
	// P:321-352: the value ends at its first byte outside its class: CR, then LF (P:248-262)
	decide(!vok, LN_SLOW, 0);
	decide(w >= E, LN_UNF, 0);
	decide(cw != '\r', LN_INV, w);
	decide(w + 1 >= E, LN_UNF, 0);
	decide(cw1 != '\n', LN_INV, w + 1);
	const bool ok = dec == SF_GO;
	LineRec r;
	r.a = (ok ? LN_OK : dec) | (kt << 4) | (q << 16);
	r.b = ok ? (v | (w << 16)) : pos;
	return r;
}

// The request line of a buffer (P:162-262): dec SF_GO with the first header line's start q,
// or the outcome.
struct ReqOut {
	uint32_t dec, pos, q, ue, post;
};

template <typename Src>
EBD_HD ReqOut scan_reqline(const Src& s, uint32_t B, uint32_t L) {
	const uint32_t E = B + L;
	uint32_t dec = L == 0 ? SF_UNF : SF_GO, pos = 0;
	auto decide = [&](bool c, uint32_t d, uint32_t p) {
		const bool t = dec == SF_GO && c;
		dec = t ? d : dec;
		pos = t ? p : pos;
	};
	// P:162-199 "GET /" | "POST /"
	const uint32_t m0 = s.dw(B), m1 = s.dw(B + 4);
	const bool post = (m0 & 0xffu) == 'P';
	const uint32_t nm = post ? 6u : 5u;
	const unsigned long long d = (((unsigned long long)m1 << 32 | m0) ^ (post ? 0x2f2054534f50ull : 0x2f20544547ull)) &
			(post ? 0xffffffffffffull : 0xffffffffffull);
	const uint32_t km = d ? ((uint32_t)__builtin_ctzll(d) >> 3) : nm;
	decide(km < nm && km < L, SF_INV, B + km);
	decide(L < nm, SF_UNF, 0);
	// P:201-213 URL bytes, then ' '; P:215-262 "HTTP/1.0" | "HTTP/1.1" CR LF
	uint32_t ue;
	const bool uok = class_search<3>(s, B + nm, E, NB_URL, ue);
	const uint32_t ur = ue < E ? ue : E;
	const uint32_t p0 = s.dw(ur), p1 = s.dw(ur + 4), p2 = s.dw(ur + 8);
	const unsigned long long x = (unsigned long long)align_byte(p1, p0, 1) | ((unsigned long long)align_byte(p2, p1, 1) << 32);
	const unsigned long long dx = (x ^ 0x302e312f50545448ull) & ~(1ull << 56);
	const uint32_t dy = ((p2 >> 8) ^ 0x0a0du) & 0xffffu;
	const uint32_t k = dx ? ((uint32_t)__builtin_ctzll(dx) >> 3) : dy ? 8u + ((uint32_t)__builtin_ctz(dy) >> 3) : 10u;
	const uint32_t avail = E - ur - 1;
	decide(!uok, SF_SLOW, 0);
	decide(ue >= E, SF_UNF, 0);
	decide((p0 & 0xffu) != ' ', SF_INV, ue);
	decide(k < 10 && k < avail, SF_INV, ue + 1 + k);
	decide(avail < 10, SF_UNF, 0);
	ReqOut r;
	r.dec = dec;
	r.pos = pos;
	r.q = ue + 11;
	r.ue = ue;
	r.post = post ? 1u : 0u;
	return r;
}

// Folds a buffer's line records in order (lines(l) -> LineRec, l0 = the index of the
// line that starts at rq.q, n = lines listed).  False: the buffer needs scan_event.
template <typename Lines>
EBD_HD bool scan_fold(const ReqOut& rq, const Lines& lines, uint32_t l0, uint32_t n, uint32_t B, uint32_t L, ScanOut& o) {
	scan_init(o, L);
	const uint32_t E = B + L;
	uint32_t dec = rq.dec, pos = rq.pos;
	bool host_seen = false, cip_seen = false;
	uint32_t host_off = 0, host_len = 0, cip_off = 0;
	uint32_t q = rq.q, l = l0;
	while (dec == SF_GO) {
		if (q >= E) { // the last line ended with the buffer
			dec = SF_UNF;
			break;
		}
		const LineRec r = lines(l);
		if (l >= n || (r.a >> 16) != q) { // not listed (more lines than the tile's list holds)
			dec = SF_SLOW;
			break;
		}
		const uint32_t code = r.a & 15u, kt = (r.a >> 4) & 3u;
		if (code != LN_OK) {
			dec = code == LN_FIN ? SF_FIN : code == LN_INV ? SF_INV : code == LN_UNF ? SF_UNF : SF_SLOW;
			pos = r.b;
			break;
		}
		if (kt == SK_HOST && host_seen) { // P:282-287: a second Host fails at its ':'
			dec = SF_INV;
			pos = q + 4;
			break;
		}
		const uint32_t v = r.b & 0xffffu, w = r.b >> 16;
		if (kt == SK_HOST) {
			host_seen = true;
			host_off = v - B;
			host_len = w - v;
		} else if (kt == SK_CLIENT && !cip_seen) {
			cip_seen = true;
			cip_off = v - B;
		}
		q = w + 2;
		l++;
	}
	if (dec == SF_SLOW)
		return false;
	if (dec == SF_INV || dec == SF_FIN) {
		o.status = dec == SF_FIN ? EBD_STATUS_FINISHED : EBD_STATUS_INVALID;
		o.consumed = pos - B + 1;
	}
	if (dec == SF_FIN) {
		o.url_off = (rq.post ? 6u : 5u) - 1;
		o.url_len = rq.ue - (B + o.url_off);
		o.host_off = host_off;
		o.host_len = host_len;
		o.cip_off = cip_off;
		o.info = (rq.post ? EBD_INFO_POST : 0u) | (cip_seen ? EBD_INFO_CIP : 0u);
	}
	return true;
}

// The LFs of 4 words (16 tile bytes): bit 7 of each byte equal to '\n' (exact per byte).
EBD_HD uint32_t lf4(uint32_t w) {
	const uint32_t t = w ^ 0x0a0a0a0au;
	return ~(((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t) & 0x80808080u;
}

// The generic parser (gp_step, the reference handlers restated) over the same bytes, for the
// buffers scan_event leaves (a header key with a space).
template <typename Src>
EBD_HD void scan_slow(const Src& s, const KeyTrie* trie, uint32_t B, uint32_t L, ScanOut& o) {
	scan_init(o, L);
	GenParser g;
	gp_init(g);
	uint32_t i = 0;
	while (i < L) {
		gp_step(g, trie, s.byte(B + i), i);
		i++;
		if (gp_done(g))
			break;
	}
	if (!gp_done(g))
		return;
	o.consumed = i;
	if (g.state != ST_FINISHED) {
		o.status = EBD_STATUS_INVALID;
		return;
	}
	o.status = EBD_STATUS_FINISHED;
	o.url_off = g.url_start;
	o.url_len = g.url_len;
	if (g.f & GPF_HOST) {
		o.host_off = g.host_start;
		o.host_len = g.host_len;
	}
	const bool cip = (g.f & (GPF_CIP_FOUND | GPF_IN_CIP)) != 0;
	o.cip_off = cip ? g.cip_start : 0u;
	o.info = (s.byte(B) == 'P' ? EBD_INFO_POST : 0u) | (cip ? EBD_INFO_CIP : 0u);
}

// The per-event result of a scan (status, consumed, spans; POST, HTTPS, CIP bits).
EBD_HD ebd_event_result scan_result(const ScanOut& o, uint8_t flags) {
	ebd_event_result r;
	r.consumed = (uint16_t)o.consumed;
	r.status = (uint8_t)o.status;
	const bool fin = o.status == EBD_STATUS_FINISHED;
	r.info = fin ? (uint8_t)(o.info | ((flags & 16) ? EBD_INFO_HTTPS : 0u)) : (uint8_t)0;
	r.u.span.url_off = (uint16_t)(fin ? o.url_off : 0u);
	r.u.span.url_len = (uint16_t)(fin ? o.url_len : 0u);
	r.u.span.host_off = (uint16_t)(fin ? o.host_off : 0u);
	r.u.span.host_len = (uint16_t)(fin ? o.host_len : 0u);
	r.u.span.cip_off = (uint16_t)(fin ? o.cip_off : 0u);
	r.u.span.cip_len = 0;
	return r;
}

} // namespace ebd
