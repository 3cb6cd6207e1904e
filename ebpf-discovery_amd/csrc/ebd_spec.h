// ebd_spec.h — the HTTP per-event parse semantics, written once for host and device.
//
// Everything here is __host__ __device__: the host uses it to derive the fast-path
// DFA table (ebd_dfa.cpp) and for tests, the GPU kernels use it directly.  Reference
// citations: P = libhttpparser/src/HttpRequestParser.cpp, A = libservice/src/Aggregator.cpp,
// IC = libservice/src/IpAddressCheckerImpl.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define EBD_HD __host__ __device__ __forceinline__

namespace ebd {

// ---------------------------------------------------------------------------------
// Parser states (HttpRequestParser.h:55-68)
// ---------------------------------------------------------------------------------
enum : uint8_t {
	ST_METHOD = 0,
	ST_SP_URL,
	ST_URL,
	ST_SP_PROTO,
	ST_PROTO,
	ST_HDR_NL,
	ST_HDR_KEY,
	ST_SP_VAL,
	ST_HDR_VAL,
	ST_HDRS_END,
	ST_FINISHED,
	ST_INVALID,
};

constexpr uint32_t kMaxRequestLength = 8192; // Constants.h:19,23
constexpr uint32_t kMaxHeaderKeyLength = 21; // P:44

// ---------------------------------------------------------------------------------
// C-locale byte classes (P:31-35, P:47-65).  Bytes >= 0x80 are in no class (signed
// char + classic locale).
// ---------------------------------------------------------------------------------
enum : uint8_t { C_URL = 1, C_KEY = 2, C_VAL = 4, C_HOST = 8, C_CIP = 16, C_UPPER = 32 };

EBD_HD bool is_alnum(uint32_t c) { return (c - '0' < 10u) || ((c | 32u) - 'a' < 26u); }
EBD_HD bool is_upper(uint32_t c) { return c - 'A' < 26u; }
EBD_HD uint32_t to_lower(uint32_t c) { return is_upper(c) ? c + 32u : c; }

EBD_HD uint8_t byte_class(uint32_t c) {
	uint8_t m = 0;
	if (is_alnum(c))
		m = C_URL | C_KEY | C_VAL | C_HOST | C_CIP;
	if (is_upper(c))
		m |= C_UPPER;
	switch (c) {
	// "-._~:/?#[]@!$&'()*+,;=%"  (URL)
	// "!#$%&'*+-.^_`|~"          (KEY)
	// "`~!@#$%^&*()-_=+[]{}\|;:'\"<>,.?/ " (VALUE)
	// "-.:[]"                    (HOST)
	// "-.:[], "                  (CLIENT IP)
	case '-': m |= C_URL | C_KEY | C_VAL | C_HOST | C_CIP; break;
	case '.': m |= C_URL | C_KEY | C_VAL | C_HOST | C_CIP; break;
	case '_': m |= C_URL | C_KEY | C_VAL; break;
	case '~': m |= C_URL | C_KEY | C_VAL; break;
	case ':': m |= C_URL | C_VAL | C_HOST | C_CIP; break;
	case '/': m |= C_URL | C_VAL; break;
	case '?': m |= C_URL | C_VAL; break;
	case '#': m |= C_URL | C_KEY | C_VAL; break;
	case '[': m |= C_URL | C_VAL | C_HOST | C_CIP; break;
	case ']': m |= C_URL | C_VAL | C_HOST | C_CIP; break;
	case '@': m |= C_URL | C_VAL; break;
	case '!': m |= C_URL | C_KEY | C_VAL; break;
	case '$': m |= C_URL | C_KEY | C_VAL; break;
	case '&': m |= C_URL | C_KEY | C_VAL; break;
	case '\'': m |= C_URL | C_KEY | C_VAL; break;
	case '(': m |= C_URL | C_VAL; break;
	case ')': m |= C_URL | C_VAL; break;
	case '*': m |= C_URL | C_KEY | C_VAL; break;
	case '+': m |= C_URL | C_KEY | C_VAL; break;
	case ',': m |= C_URL | C_VAL | C_CIP; break;
	case ';': m |= C_URL | C_VAL; break;
	case '=': m |= C_URL | C_VAL; break;
	case '%': m |= C_URL | C_KEY | C_VAL; break;
	case '^': m |= C_KEY | C_VAL; break;
	case '`': m |= C_KEY | C_VAL; break;
	case '|': m |= C_KEY | C_VAL; break;
	case '{': m |= C_VAL; break;
	case '}': m |= C_VAL; break;
	case '\\': m |= C_VAL; break;
	case '"': m |= C_VAL; break;
	case '<': m |= C_VAL; break;
	case '>': m |= C_VAL; break;
	case ' ': m |= C_VAL | C_CIP; break;
	default: break;
	}
	return m;
}

// ---------------------------------------------------------------------------------
// Header-key trie: currentHeader.key lower-cased, spaces skipped, truncated at 21
// (P:264-297), matched against "host" (P:366-368) and the client-IP keys (P:43,
// P:370-372).  Node 0 = empty key, node 1 = a key that can no longer match.  The
// table is built on the host (build_key_trie) and copied to the device.
// ---------------------------------------------------------------------------------
constexpr int kTrieNodes = 80;
constexpr uint8_t kTrieRoot = 0, kTrieDead = 1;
enum : uint8_t { KT_OTHER = 0, KT_HOST = 1, KT_CLIENT0 = 2 }; // client key k -> KT_CLIENT0 + k (k = 0..4)

struct KeyTrie {
	uint8_t next[kTrieNodes][128]; // next node for a lower-cased 7-bit key byte
	uint8_t cls[256];              // byte_class() of every byte (a table the session path keeps in LDS)
	uint8_t type[kTrieNodes];      // KT_*
	uint8_t nodes;
};

EBD_HD uint8_t key_client_id(uint8_t type) { return type >= KT_CLIENT0 ? (uint8_t)(type - KT_CLIENT0 + 1) : 0; }

// ---------------------------------------------------------------------------------
// Generic parser: the reference state machine (P:85-379) over a compact state.
// Spans are in request-stream coordinates (0 = first byte after reset), which is how
// the device session path addresses bytes spread over several buffers.
// ---------------------------------------------------------------------------------
enum : uint8_t { GPF_HOST = 1, GPF_CIP_FOUND = 2, GPF_IN_CIP = 4, GPF_HTTPS = 8 };

struct GenParser {
	uint8_t state;
	uint8_t mlen, mcand;  // method prefix length and first char ('G' / 'P')
	uint8_t plen, pminor; // protocol prefix length and its 8th char
	uint8_t key;          // trie node of currentHeader.key
	uint8_t cipkey;       // sticky result.clientIPKey: 0 none, 1..5 (P:73-80 does not clear it)
	uint8_t f;            // GPF_*
	uint8_t ds;           // the session path's DFA state (dfa_parse, ebd_fresh.h); 0 = reset
	uint8_t kid;          // dfa_parse: client-IP id (0..5) of the last header key it walked
	uint8_t pad_[2];
	uint32_t length;      // bytes since reset (P:88-91)
	uint32_t url_start, url_len, host_start, host_len, cip_start, cip_len;
};

EBD_HD void gp_init(GenParser& g) {
	g.state = ST_METHOD;
	g.mlen = g.mcand = g.plen = g.pminor = 0;
	g.key = kTrieRoot;
	g.cipkey = 0;
	g.f = 0;
	g.ds = 0;
	g.kid = 0;
	g.pad_[0] = g.pad_[1] = 0;
	g.length = 0;
	g.url_start = g.url_len = g.host_start = g.host_len = g.cip_start = g.cip_len = 0;
}

// P:374-379 reset(): clears everything but result.clientIPKey.
EBD_HD void gp_reset(GenParser& g) {
	uint8_t k = g.cipkey;
	gp_init(g);
	g.cipkey = k;
}

EBD_HD uint8_t gp_key_type(const KeyTrie* t, uint8_t node) { return t->type[node]; }

// One byte (P:124-160 and the handlers P:162-364).  pos = request-stream position.
EBD_HD void gp_step(GenParser& g, const KeyTrie* trie, uint32_t c, uint32_t pos) {
	const uint8_t cls = trie->cls[c & 255];
	switch (g.state) {
	case ST_METHOD: // P:162-188
		if (cls & C_UPPER) {
			bool ok;
			if (g.mlen == 0) {
				g.mcand = (uint8_t)c;
				ok = (c == 'G' || c == 'P');
			} else if (g.mcand == 'G') {
				ok = g.mlen < 3 && "GET"[g.mlen] == (char)c;
			} else {
				ok = g.mlen < 4 && "POST"[g.mlen] == (char)c;
			}
			if (g.mlen < 255)
				g.mlen++;
			if (!ok)
				g.state = ST_INVALID;
			return;
		}
		if (c != ' ' || !((g.mcand == 'G' && g.mlen == 3) || (g.mcand == 'P' && g.mlen == 4))) {
			g.state = ST_INVALID;
			return;
		}
		g.state = ST_SP_URL;
		return;
	case ST_SP_URL: // P:190-199
		if (c != '/') {
			g.state = ST_INVALID;
			return;
		}
		g.url_start = pos;
		g.url_len = 1;
		g.state = ST_URL;
		return;
	case ST_URL: // P:201-213
		if (c != ' ') {
			if (!(cls & C_URL)) {
				g.state = ST_INVALID;
				return;
			}
			g.url_len++;
			return;
		}
		g.state = ST_SP_PROTO;
		return;
	case ST_SP_PROTO: // P:215-224
		if (c != 'H') {
			g.state = ST_INVALID;
			return;
		}
		g.plen = 1;
		g.state = ST_PROTO;
		return;
	case ST_PROTO: // P:226-246
		if (c != '\r') {
			bool ok;
			if (g.plen < 7)
				ok = "HTTP/1."[g.plen] == (char)c;
			else if (g.plen == 7) {
				ok = (c == '0' || c == '1');
				g.pminor = (uint8_t)c;
			} else
				ok = false;
			if (g.plen < 255)
				g.plen++;
			if (!ok)
				g.state = ST_INVALID;
			return;
		}
		if (g.plen != 8) {
			g.state = ST_INVALID;
			return;
		}
		g.state = ST_HDR_NL;
		return;
	case ST_HDR_NL: // P:248-262
		if (c != '\n') {
			g.state = ST_INVALID;
			return;
		}
		if (g.f & GPF_IN_CIP) // parseClientIPValue for the first header whose key == clientIPKey
			g.f = (uint8_t)((g.f & ~GPF_IN_CIP) | GPF_CIP_FOUND);
		g.key = kTrieRoot;
		g.state = ST_HDR_KEY;
		return;
	case ST_HDR_KEY: // P:264-297
		if (c == '\r') {
			g.state = ST_HDRS_END;
			return;
		}
		if (c == ' ')
			return;
		if (c != ':') {
			if (!(cls & C_KEY)) {
				g.state = ST_INVALID;
				return;
			}
			g.key = trie->next[g.key][to_lower(c) & 127];
			return;
		}
		if (gp_key_type(trie, g.key) == KT_HOST && (g.f & GPF_HOST)) {
			g.state = ST_INVALID;
			return;
		}
		g.state = ST_SP_VAL;
		return;
	case ST_SP_VAL: { // P:299-319
		if (c == ' ')
			return;
		if (!(cls & C_VAL)) {
			g.state = ST_INVALID;
			return;
		}
		const uint8_t kt = gp_key_type(trie, g.key);
		if (kt == KT_HOST) {
			g.host_start = pos;
			g.host_len = 1;
			g.f |= GPF_HOST;
		} else if (kt >= KT_CLIENT0) {
			const uint8_t id = key_client_id(kt);
			if (g.cipkey == 0)
				g.cipkey = id;
			if (id == g.cipkey && !(g.f & GPF_CIP_FOUND)) {
				g.cip_start = pos;
				g.cip_len = 1;
				g.f |= GPF_IN_CIP;
			}
		}
		g.state = ST_HDR_VAL;
		return;
	}
	case ST_HDR_VAL: { // P:321-352
		if (c == '\r') {
			g.state = ST_HDR_NL;
			return;
		}
		const uint8_t kt = gp_key_type(trie, g.key);
		if (kt == KT_HOST) {
			if (!(cls & C_HOST)) {
				g.state = ST_INVALID;
				return;
			}
			g.host_len++;
			return;
		}
		if (kt >= KT_CLIENT0) {
			if (!(cls & C_CIP)) {
				g.state = ST_INVALID;
				return;
			}
			if (g.f & GPF_IN_CIP)
				g.cip_len++;
			return;
		}
		if (!(cls & C_VAL))
			g.state = ST_INVALID;
		return;
	}
	case ST_HDRS_END: // P:354-364
		g.state = (c == '\n') ? ST_FINISHED : ST_INVALID;
		return;
	default:
		return;
	}
}

EBD_HD bool gp_done(const GenParser& g) { return g.state == ST_FINISHED || g.state == ST_INVALID; }

// P:85-106 parse(): returns the bytes consumed from this buffer.  `at(i)` yields byte i.
template <typename ByteAt>
EBD_HD uint32_t gp_parse(GenParser& g, const KeyTrie* trie, ByteAt at, uint32_t n, uint8_t flags) {
	uint32_t i = 0;
	while (i < n) {
		if (g.length > kMaxRequestLength) {
			g.state = ST_INVALID;
			return i;
		}
		gp_step(g, trie, at(i), g.length);
		i++;
		g.length++;
		if (gp_done(g)) {
			if (flags & 16) // DISCOVERY_FLAG_SESSION_SSL_HTTP
				g.f |= GPF_HTTPS;
			else
				g.f &= (uint8_t)~GPF_HTTPS;
			return i;
		}
	}
	return i;
}

// ---------------------------------------------------------------------------------
// Client address of a finished request (A:44-94 with P:381-409 for the front token).
// ---------------------------------------------------------------------------------
enum : uint8_t { CLS_NONE = 0, CLS_INTERNAL = 1, CLS_EXTERNAL = 2 };

// glibc resolv/inet_pton.c inet_pton4 (the reference calls glibc inet_pton, A:66-74).
// A byte source shifted by `off` (works for pointers and accessor views alike).
template <typename Src>
struct SrcOff {
	const Src& s;
	uint32_t off;
	EBD_HD uint32_t operator[](uint32_t k) const { return (uint32_t)s[off + k]; }
};

template <typename Src>
EBD_HD bool inet_pton4(const Src& s, uint32_t n, uint8_t out[4]) {
	uint32_t saw_digit = 0, octets = 0, k = 0;
	uint32_t tmp[4] = {0, 0, 0, 0};
	for (uint32_t i = 0; i < n; i++) {
		const uint32_t ch = s[i];
		if (ch - '0' < 10u) {
			const uint32_t nw = tmp[k] * 10u + (ch - '0');
			if (saw_digit && tmp[k] == 0)
				return false;
			if (nw > 255)
				return false;
			tmp[k] = nw;
			if (!saw_digit) {
				if (++octets > 4)
					return false;
				saw_digit = 1;
			}
		} else if (ch == '.' && saw_digit) {
			if (octets == 4)
				return false;
			tmp[++k] = 0;
			saw_digit = 0;
		} else
			return false;
	}
	if (octets < 4)
		return false;
	for (int i = 0; i < 4; i++)
		out[i] = (uint8_t)tmp[i];
	return true;
}

EBD_HD int hex_value(uint32_t ch) {
	if (ch - '0' < 10u)
		return (int)(ch - '0');
	if ((ch | 32u) - 'a' < 6u)
		return (int)((ch | 32u) - 'a' + 10);
	return -1;
}

// glibc resolv/inet_pton.c inet_pton6 (glibc >= 2.26 form).
template <typename Src>
EBD_HD bool inet_pton6(const Src& s, uint32_t n, uint8_t out[16]) {
	uint8_t tmp[16];
	for (int i = 0; i < 16; i++)
		tmp[i] = 0;
	int tp = 0, colonp = -1;
	uint32_t i = 0;
	if (n == 0)
		return false;
	if (s[0] == ':') {
		i = 1;
		if (i == n || s[i] != ':')
			return false;
	}
	uint32_t curtok = i;
	uint32_t xdigits = 0, val = 0;
	while (i < n) {
		const uint32_t ch = s[i++];
		const int d = hex_value(ch);
		if (d >= 0) {
			if (xdigits == 4)
				return false;
			val = (val << 4) | (uint32_t)d;
			if (val > 0xffff)
				return false;
			xdigits++;
			continue;
		}
		if (ch == ':') {
			curtok = i;
			if (xdigits == 0) {
				if (colonp >= 0)
					return false;
				colonp = tp;
				continue;
			} else if (i == n)
				return false;
			if (tp + 2 > 16)
				return false;
			tmp[tp++] = (uint8_t)(val >> 8);
			tmp[tp++] = (uint8_t)val;
			xdigits = 0;
			val = 0;
			continue;
		}
		if (ch == '.' && tp + 4 <= 16) {
			uint8_t v4[4];
			if (inet_pton4(SrcOff<Src>{s, curtok}, n - curtok, v4)) {
				for (int k = 0; k < 4; k++)
					tmp[tp++] = v4[k];
				xdigits = 0;
				break;
			}
		}
		return false;
	}
	if (xdigits > 0) {
		if (tp + 2 > 16)
			return false;
		tmp[tp++] = (uint8_t)(val >> 8);
		tmp[tp++] = (uint8_t)val;
	}
	if (colonp >= 0) {
		if (tp == 16)
			return false;
		const int cnt = tp - colonp;
		for (int k = 1; k <= cnt; k++) { // memmove(endp - n, colonp, n) from the back
			tmp[16 - k] = tmp[colonp + cnt - k];
		}
		for (int k = colonp; k < 16 - cnt; k++)
			tmp[k] = 0;
		tp = 16;
	}
	if (tp != 16)
		return false;
	for (int k = 0; k < 16; k++)
		out[k] = tmp[k];
	return true;
}

struct Interfaces {
	uint32_t n4, n6;
	uint8_t v4[64][8];   // {addr[4], mask[4]}
	uint8_t v6[32][32];  // {addr[16], mask[16]}
};

// IC:39-85 (addr in network byte order)
EBD_HD bool v4_external(const Interfaces& ifs, const uint8_t a[4]) {
	const uint32_t h = ((uint32_t)a[0] << 24) | ((uint32_t)a[1] << 16) | ((uint32_t)a[2] << 8) | a[3];
	// RFC 6890 ranges, IC:44-62 (network, mask)
	if ((h & 0xff000000u) == 0x00000000u || (h & 0xff000000u) == 0x0a000000u || (h & 0xffc00000u) == 0x64400000u ||
			(h & 0xff000000u) == 0x7f000000u || (h & 0xffff0000u) == 0xa9fe0000u || (h & 0xfff00000u) == 0xac100000u ||
			(h & 0xffffff00u) == 0xc0000000u || (h & 0xffffff00u) == 0xc0000200u || (h & 0xffffff00u) == 0xc0586300u ||
			(h & 0xffff0000u) == 0xc0a80000u || (h & 0xfffe0000u) == 0xc6120000u || (h & 0xffffff00u) == 0xc6336400u ||
			(h & 0xffffff00u) == 0xcb007100u || (h & 0xf0000000u) == 0xe0000000u || (h & 0xffff0000u) == 0xe9fc0000u ||
			(h & 0xf0000000u) == 0xf0000000u || h == 0xffffffffu)
		return false;
	for (uint32_t i = 0; i < ifs.n4; i++) { // IC:74-82, checkSubnetIpv4 IC:139-145
		bool eq = true;
		for (int k = 0; k < 4; k++)
			eq &= (a[k] & ifs.v4[i][4 + k]) == (ifs.v4[i][k] & ifs.v4[i][4 + k]);
		if (eq)
			return false;
	}
	return true;
}

// IC:146-180
EBD_HD bool v6_external(const Interfaces& ifs, const uint8_t a[16]) {
	bool z80 = true; // bytes 0..9 zero
	for (int k = 0; k < 10; k++)
		z80 &= a[k] == 0;
	// IC:71-88: ::ffff:0:0/96 (bytes 10,11 = ff), ::ffff:0:0:0/96 (bytes 8,9 = ff; 10,11 = 0),
	// 64:ff9b::/96 (00 64 ff 9b then zeros to byte 11)
	const bool mapped = (z80 && a[10] == 0xff && a[11] == 0xff) ||
			(a[0] == 0 && a[1] == 0 && a[2] == 0 && a[3] == 0 && a[4] == 0 && a[5] == 0 && a[6] == 0 && a[7] == 0 &&
					a[8] == 0xff && a[9] == 0xff && a[10] == 0 && a[11] == 0) ||
			(a[0] == 0x00 && a[1] == 0x64 && a[2] == 0xff && a[3] == 0x9b && a[4] == 0 && a[5] == 0 && a[6] == 0 && a[7] == 0 &&
					a[8] == 0 && a[9] == 0 && a[10] == 0 && a[11] == 0);
	if (mapped) // IC:81-88 getMappedIPv4Addr: bytes 12..15 in network order
		return v4_external(ifs, a + 12);
	for (uint32_t i = 0; i < ifs.n6; i++) { // checkSubnet IC:128-137
		bool eq = true;
		for (int k = 0; k < 16; k++)
			eq &= (a[k] & ifs.v6[i][16 + k]) == (ifs.v6[i][k] & ifs.v6[i][16 + k]);
		if (eq)
			return false;
	}
	if ((a[0] & 0xfe) == 0xfc) // fc00::/7
		return false;
	if (a[0] == 0xfe && (a[1] & 0xc0) == 0xc0) // fec0::/10
		return false;
	if (a[0] == 0xfe && (a[1] & 0xc0) == 0x80) // fe80::/10
		return false;
	bool loop = a[15] == 1; // ::1/128
	for (int k = 0; k < 15; k++)
		loop &= a[k] == 0;
	return !loop;
}

// Source-address fallback (A:57-63).  ipv4ToString / ipv6ToString followed by
// inet_pton is the identity on the address bytes (checked against glibc in the tests),
// so the bytes are classified directly.
// The client's networks for the network counters (A:89-106), packed: address bytes 0..5 at
// bits 0..47 (in_addr / in6_addr order), bit 63 set for IPv6.  Meaningful for an external
// client only.
constexpr unsigned long long kNetV6 = 1ull << 63;
EBD_HD unsigned long long net_pack(const uint8_t* a, bool v6) {
	unsigned long long p = 0;
	for (int k = 0; k < (v6 ? 6 : 3); k++)
		p |= (unsigned long long)a[k] << (8 * k);
	return v6 ? (p | kNetV6) : p;
}

EBD_HD uint8_t classify_source(const Interfaces& ifs, uint8_t flags, const uint8_t src[16], unsigned long long* net = nullptr) {
	if (flags & 2) {
		if (net)
			*net = net_pack(src, false);
		return v4_external(ifs, src) ? CLS_EXTERNAL : CLS_INTERNAL;
	}
	if (flags & 4) {
		if (net)
			*net = net_pack(src, true);
		return v6_external(ifs, src) ? CLS_EXTERNAL : CLS_INTERNAL;
	}
	return CLS_NONE;
}

// Front token of a client-IP header value (P:392-409 on the first token only: the
// aggregator uses clientIp.front(), A:52-53).  `raw` = value bytes up to (excluding)
// the first ',' (boost::split token_compress_on: the first token ends at the first
// separator).  Returns the token as [*b, *e) inside raw.
template <typename Src>
EBD_HD void front_token(const Src& raw, uint32_t n, uint32_t* tb, uint32_t* te) {
	uint32_t b = 0, e = n;
	while (b < e && raw[b] == ' ') // boost::trim; only ' ' can occur in a header value
		b++;
	while (e > b && raw[e - 1] == ' ')
		e--;
	bool dot = false;
	for (uint32_t k = b; k < e; k++)
		dot |= raw[k] == '.';
	if (dot) { // IPv4: cut at the last ':' (P:397-400)
		uint32_t colon = 0xffffffffu;
		for (uint32_t k = b; k < e; k++)
			if (raw[k] == ':')
				colon = k;
		if (colon != 0xffffffffu) {
			e = colon;
			while (b < e && raw[b] == ' ')
				b++;
			while (e > b && raw[e - 1] == ' ')
				e--;
		}
	} else if (e > b && raw[b] == '[') { // IPv6: text between brackets (P:381-390, 401-405)
		uint32_t rb = 0xffffffffu;
		for (uint32_t k = b; k < e; k++)
			if (raw[k] == ']')
				rb = k;
		if (rb != 0xffffffffu) {
			uint32_t ib = b + 1, ie = rb;
			while (ib < ie && raw[ib] == ' ')
				ib++;
			while (ie > ib && raw[ie - 1] == ' ')
				ie--;
			b = ib;
			e = ie;
		}
	}
	*tb = b;
	*te = e;
}

// A:50-74 on clientIp.front(): >= 2 ':' selects AF_INET6, parse failure = no count.
template <typename Src>
EBD_HD uint8_t classify_token(const Interfaces& ifs, const Src& t, uint32_t n, unsigned long long* net = nullptr) {
	uint32_t colons = 0;
	for (uint32_t k = 0; k < n; k++)
		colons += t[k] == ':';
	if (colons >= 2) {
		uint8_t a[16];
		if (n > 45 || !inet_pton6(t, n, a)) // longer than any valid text form
			return CLS_NONE;
		if (net)
			*net = net_pack(a, true);
		return v6_external(ifs, a) ? CLS_EXTERNAL : CLS_INTERNAL;
	}
	uint8_t a[4];
	if (n > 15 || !inet_pton4(t, n, a))
		return CLS_NONE;
	if (net)
		*net = net_pack(a, false);
	return v4_external(ifs, a) ? CLS_EXTERNAL : CLS_INTERNAL;
}

// Domain of a host (A:117-125): "[...]" through the first ']' after '[', empty if none;
// otherwise the prefix before the first ':'.
EBD_HD void host_domain(const uint8_t* h, uint32_t n, uint32_t* off, uint32_t* len) {
	uint32_t lb = 0xffffffffu;
	for (uint32_t k = 0; k < n; k++)
		if (h[k] == '[') {
			lb = k;
			break;
		}
	if (lb != 0xffffffffu) {
		for (uint32_t k = lb + 1; k < n; k++)
			if (h[k] == ']') {
				*off = lb;
				*len = k - lb + 1;
				return;
			}
		*off = 0;
		*len = 0;
		return;
	}
	uint32_t c = n;
	for (uint32_t k = 0; k < n; k++)
		if (h[k] == ':') {
			c = k;
			break;
		}
	*off = 0;
	*len = c;
}

// ---------------------------------------------------------------------------------
// 128-bit key of (pid, host + url): a streaming hash over the endpoint bytes so that
// any host/url split of the same endpoint string hashes alike (A:27-29, A:155-158).
// ---------------------------------------------------------------------------------
struct Hash128 {
	uint64_t lo, hi;
};

EBD_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
EBD_HD uint64_t fmix64(uint64_t k) {
	k ^= k >> 33;
	k *= 0xff51afd7ed558ccdull;
	k ^= k >> 33;
	k *= 0xc4ceb9fe1a85ec53ull;
	k ^= k >> 33;
	return k;
}

// The service key is a keyed pseudo-random function of the exact bytes the reference keys
// on (pid, endpoint = host + url; Aggregator.h:29-37): SipHash-1-3 with the 128-bit output
// (Aumasson & Bernstein; the HashDoS-resistant PRF), keyed by a secret 128-bit HashKey
// drawn per context (ebd_config.hash_key, or getrandom).  The message is the 8-byte pid,
// then E = host + url as little-endian 8-byte words (the last one zero-padded), then a word
// holding |E|; so every host/url split of the same endpoint hashes alike, and the encoding
// is injective.  Without the key an adversary cannot construct two endpoints with one key;
// two distinct (pid, endpoint) pairs share a key with probability 2^-128 each.
struct HashKey {
	uint64_t k0, k1;
};

struct KeyHasher {
	uint64_t v0, v1, v2, v3, acc;
	uint32_t total;
	EBD_HD static void round(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& e) {
		a += b;
		b = rotl64(b, 13);
		b ^= a;
		a = rotl64(a, 32);
		c += e;
		e = rotl64(e, 16);
		e ^= c;
		a += e;
		e = rotl64(e, 21);
		e ^= a;
		c += b;
		b = rotl64(b, 17);
		b ^= c;
		c = rotl64(c, 32);
	}
	EBD_HD void word(uint64_t m) { // one message word, c = 1 round
		v3 ^= m;
		round(v0, v1, v2, v3);
		v0 ^= m;
	}
	EBD_HD void init(const HashKey& k, uint32_t pid) {
		v0 = k.k0 ^ 0x736f6d6570736575ull;
		v1 = k.k1 ^ 0x646f72616e646f6dull ^ 0xee; // 128-bit output variant
		v2 = k.k0 ^ 0x6c7967656e657261ull;
		v3 = k.k1 ^ 0x7465646279746573ull;
		acc = 0;
		total = 0;
		word(pid);
	}
	// streaming form (session path, host code)
	EBD_HD void byte(uint32_t b) {
		acc |= (uint64_t)(b & 0xff) << (8 * (total & 7));
		total++;
		if ((total & 7) == 0) {
			word(acc);
			acc = 0;
		}
	}
	EBD_HD void bytes(const uint8_t* p, uint32_t n) {
		for (uint32_t i = 0; i < n; i++)
			byte(p[i]);
	}
	// after the words were fed directly (block form): n = endpoint length; d = 3 rounds
	EBD_HD Hash128 finish_words(uint32_t n) {
		word(((uint64_t)0xe5 << 56) | n);
		v2 ^= 0xee;
		round(v0, v1, v2, v3);
		round(v0, v1, v2, v3);
		round(v0, v1, v2, v3);
		Hash128 r;
		r.lo = (v0 ^ v1 ^ v2 ^ v3) | 1ull; // 0 marks an empty slot
		v1 ^= 0xdd;
		round(v0, v1, v2, v3);
		round(v0, v1, v2, v3);
		round(v0, v1, v2, v3);
		r.hi = (v0 ^ v1 ^ v2 ^ v3) | 1ull;
		return r;
	}
	EBD_HD Hash128 finish() {
		if (total & 7)
			word(acc);
		return finish_words(total);
	}
};

// Mask of the low `k` bytes of a 64-bit piece (k in [0, 8]).
EBD_HD uint64_t low_bytes(uint32_t k) { return k >= 8 ? ~0ull : ((1ull << (8 * k)) - 1ull); }

// The 8-byte piece of E = host + url at E-offset oo, from A = 8 bytes at host offset oo and
// B = 8 bytes at url offset oo - hl (either may be garbage when unused); n = |E|.
EBD_HD uint64_t endpoint_piece(uint32_t hl, uint32_t n, uint32_t oo, uint64_t A, uint64_t B) {
	const int d = (int)hl - (int)oo; // host bytes left at this piece
	const uint64_t x = d >= 8 ? A : (d <= 0 ? B : ((A & low_bytes((uint32_t)d)) | (B << (8 * (d & 7)))));
	return oo < n ? (x & low_bytes(n - oo)) : 0;
}

// Block form over E = buffer[hs, hs + hl) + buffer[us, us + ul), reading 8-byte pieces
// through `ld8(offset)` (any alignment; bytes beyond a span are masked off).  The loads of
// a group of kGroup pieces are all issued before any is used: 8 pieces (64 bytes of E, one
// memory round trip for most endpoints) from HBM, fewer from LDS, where latency is short and
// registers are what limits the kernel.
template <uint32_t kGroup = 8, typename Ld8>
EBD_HD Hash128 endpoint_key(const HashKey& key, uint32_t pid, uint32_t hs, uint32_t hl, uint32_t us, uint32_t ul, Ld8 ld8) {
	KeyHasher kh;
	kh.init(key, pid);
	const uint32_t n = hl + ul;
	for (uint32_t g = 0; g < n; g += 8 * kGroup) {
		uint64_t A[kGroup], B[kGroup];
#pragma unroll
		for (uint32_t k = 0; k < kGroup; k++) {
			const uint32_t oo = g + 8 * k;
			// both candidate loads, unconditionally and at in-span offsets
			A[k] = ld8(hs + (oo < hl ? oo : 0));
			B[k] = ld8(us + ((oo > hl && oo - hl < ul) ? oo - hl : 0));
		}
#pragma unroll
		for (uint32_t k = 0; k < kGroup; k++) {
			const uint32_t oo = g + 8 * k;
			if (oo < n)
				kh.word(endpoint_piece(hl, n, oo, A[k], B[k]));
		}
	}
	return kh.finish_words(n);
}

} // namespace ebd
