/*
 * oracle.c — CPU restatement of the eBPF-Discovery HTTP per-event parse path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Plain C, written from the reference's
 * behaviour; every block cites the reference file:line it restates.
 * Reference paths:
 *   P  = libhttpparser/src/HttpRequestParser.cpp
 *   D  = libebpfdiscovery/src/Discovery.cpp
 *   L  = libebpfdiscovery/headers/ebpfdiscovery/LRUCache.h
 *   A  = libservice/src/Aggregator.cpp
 *   IC = libservice/src/IpAddressCheckerImpl.cpp
 *   IA = libservice/src/IpAddress.cpp
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

#define MAX_HTTP_REQUEST_LENGTH 8192 /* Constants.h:19,23 */

/* ------------------------------------------------------------------------------- */
/* growable byte string (stands for std::string)                                    */
/* ------------------------------------------------------------------------------- */
typedef struct {
	char* p;
	size_t n, cap;
} dstr;

static void ds_reserve(dstr* s, size_t need) {
	if (need <= s->cap)
		return;
	size_t c = s->cap ? s->cap : 16;
	while (c < need)
		c *= 2;
	s->p = (char*)realloc(s->p, c);
	s->cap = c;
}
static void ds_push(dstr* s, char ch) {
	ds_reserve(s, s->n + 1);
	s->p[s->n++] = ch;
}
static void ds_set(dstr* s, const char* d, size_t n) {
	ds_reserve(s, n + 1);
	memcpy(s->p, d, n);
	s->n = n;
}
static void ds_clear(dstr* s) { s->n = 0; }
static void ds_free(dstr* s) {
	free(s->p);
	s->p = NULL;
	s->n = s->cap = 0;
}
static int ds_eq(const dstr* s, const char* lit) {
	size_t n = strlen(lit);
	return s->n == n && (n == 0 || memcmp(s->p, lit, n) == 0);
}
static int ds_eqds(const dstr* a, const dstr* b) { return a->n == b->n && (a->n == 0 || memcmp(a->p, b->p, a->n) == 0); }
static void ds_copy(dstr* dst, const dstr* src) { ds_set(dst, src->p, src->n); }

typedef struct {
	dstr* v;
	size_t n, cap;
} dstr_list;

static void dl_push(dstr_list* l, const char* d, size_t n) {
	if (l->n == l->cap) {
		l->cap = l->cap ? l->cap * 2 : 4;
		l->v = (dstr*)realloc(l->v, l->cap * sizeof(dstr));
	}
	memset(&l->v[l->n], 0, sizeof(dstr));
	ds_set(&l->v[l->n], d, n);
	l->n++;
}
static void dl_clear(dstr_list* l) {
	for (size_t i = 0; i < l->n; i++)
		ds_free(&l->v[i]);
	l->n = 0;
}
static void dl_free(dstr_list* l) {
	dl_clear(l);
	free(l->v);
	l->v = NULL;
	l->cap = 0;
}

/* ------------------------------------------------------------------------------- */
/* C-locale character classes.  The reference passes a (signed) char to std::isalnum */
/* and friends; main never calls setlocale, so the classic "C" locale applies and    */
/* bytes >= 0x80 belong to no class.                                                 */
/* ------------------------------------------------------------------------------- */
static int c_isalnum(unsigned char c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
static int c_isupper(unsigned char c) { return c >= 'A' && c <= 'Z'; }
static unsigned char c_tolower(unsigned char c) { return c_isupper(c) ? (unsigned char)(c + 32) : c; }
static int c_isspace(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r'; }
/* std::string_view::find over a literal: the terminating NUL is not part of the view. */
static int in_set(unsigned char c, const char* set) {
	for (const char* q = set; *q; q++)
		if ((unsigned char)*q == c)
			return 1;
	return 0;
}

/* P:31-35 */
static const char* URL_SPECIAL = "-._~:/?#[]@!$&'()*+,;=%";
static const char* KEY_SPECIAL = "!#$%&'*+-.^_`|~";
static const char* VALUE_SPECIAL = "`~!@#$%^&*()-_=+[]{}\\|;:'\"<>,.?/ ";
static const char* HOST_SPECIAL = "-.:[]";
static const char* CLIENT_IP_SPECIAL = "-.:[], ";

/* P:47-65 */
static int valid_url(unsigned char c) { return c_isalnum(c) || in_set(c, URL_SPECIAL); }
static int valid_key(unsigned char c) { return c_isalnum(c) || in_set(c, KEY_SPECIAL); }
static int valid_value(unsigned char c) { return c_isalnum(c) || in_set(c, VALUE_SPECIAL); }
static int valid_host(unsigned char c) { return c_isalnum(c) || in_set(c, HOST_SPECIAL); }
static int valid_client_ip(unsigned char c) { return c_isalnum(c) || in_set(c, CLIENT_IP_SPECIAL); }

/* P:43 */
static const char* CLIENT_IP_KEYS[5] = {"rproxy_remote_address", "true-client-ip", "x-client-ip", "x-forwarded-for", "x-http-client-ip"};
#define MAX_HEADER_KEY_LENGTH 21 /* P:44 */

/* ------------------------------------------------------------------------------- */
/* HttpRequest / HttpRequestParser                                                  */
/* ------------------------------------------------------------------------------- */
typedef struct {
	dstr method, url, protocol, host, clientIPKey;
	dstr_list clientIp;
	int isHttps;
} orc_request;

struct orc_parser {
	orc_request result;
	int state;
	dstr hkey, hval; /* currentHeader, HttpRequestParser.h:93-98 */
	size_t length;
	int isClientIpRead;
};

/* P:67-71 (constructor) */
static void req_init(orc_request* r) {
	memset(r, 0, sizeof(*r));
	r->isHttps = 0;
}
/* P:73-80 — NB: clientIPKey is NOT cleared */
static void req_clear(orc_request* r) {
	ds_clear(&r->method);
	ds_clear(&r->url);
	ds_clear(&r->protocol);
	ds_clear(&r->host);
	dl_clear(&r->clientIp);
	r->isHttps = 0;
}
static void req_free(orc_request* r) {
	ds_free(&r->method);
	ds_free(&r->url);
	ds_free(&r->protocol);
	ds_free(&r->host);
	ds_free(&r->clientIPKey);
	dl_free(&r->clientIp);
}
static void parser_init(orc_parser* p) {
	memset(p, 0, sizeof(*p));
	req_init(&p->result);
	p->state = ORC_ST_METHOD; /* P:82 */
}
static void parser_destroy(orc_parser* p) {
	req_free(&p->result);
	ds_free(&p->hkey);
	ds_free(&p->hval);
}

/* P:366-368 */
static int key_is_host(const orc_parser* p) { return ds_eq(&p->hkey, "host"); }
/* P:370-372 */
static int key_is_client_ip(const orc_parser* p) {
	for (int i = 0; i < 5; i++)
		if (ds_eq(&p->hkey, CLIENT_IP_KEYS[i]))
			return 1;
	return 0;
}

/* boost::trim (boost 1.83, classic-locale isspace): in place on [b, e) */
static void trim_range(const char* s, size_t* b, size_t* e) {
	while (*b < *e && c_isspace((unsigned char)s[*b]))
		(*b)++;
	while (*e > *b && c_isspace((unsigned char)s[*e - 1]))
		(*e)--;
}

/* P:381-390 getTextBetweenSquareBrackets + P:392-409 parseClientIPValue.
 * boost::split(..., is_any_of(","), token_compress_on) emits the token before every
 * run of separators and always the final token, so "" -> [""], ",a" -> ["","a"],
 * "a,,b" -> ["a","b"], "a," -> ["a",""]. */
static void parse_client_ip_value(orc_request* r, const char* d, size_t n) {
	size_t tok_b = 0, i = 0;
	for (;;) {
		size_t tok_e;
		int last;
		while (i < n && d[i] != ',')
			i++;
		tok_e = i;
		last = (i >= n);
		if (!last) {
			while (i < n && d[i] == ',') /* token_compress_on: a run is one separator */
				i++;
		}
		{
			size_t b = tok_b, e = tok_e;
			trim_range(d, &b, &e); /* P:396 */
			int has_dot = 0;
			for (size_t k = b; k < e; k++)
				if (d[k] == '.')
					has_dot = 1;
			if (has_dot) { /* P:397-400: IPv4 — cut at the LAST ':' */
				size_t colon = (size_t)-1;
				for (size_t k = b; k < e; k++)
					if (d[k] == ':')
						colon = k;
				if (colon != (size_t)-1) {
					e = colon;
					trim_range(d, &b, &e);
				}
			} else { /* P:401-405: IPv6 — bracketed */
				size_t lb = (size_t)-1, rb = (size_t)-1;
				for (size_t k = b; k < e; k++) {
					if (d[k] == '[' && lb == (size_t)-1)
						lb = k;
					if (d[k] == ']')
						rb = k;
				}
				int starts = (e > b && d[b] == '[');
				if (starts && lb != (size_t)-1 && rb != (size_t)-1 && rb >= lb) {
					size_t ib = lb + 1, ie = rb;
					trim_range(d, &ib, &ie);
					b = ib;
					e = ie;
				}
			}
			dl_push(&r->clientIp, d + b, e - b); /* P:408 */
		}
		if (last)
			break;
		tok_b = i;
	}
}

static void set_invalid(orc_parser* p) { p->state = ORC_ST_INVALID; }

/* P:162-188 */
static void h_method(orc_parser* p, unsigned char ch) {
	if (c_isupper(ch)) {
		ds_push(&p->result.method, (char)ch);
		size_t n = p->result.method.n;
		int maybe_get = n <= 3 && memcmp("GET", p->result.method.p, n) == 0;
		int maybe_post = n <= 4 && memcmp("POST", p->result.method.p, n) == 0;
		if (!maybe_get && !maybe_post)
			set_invalid(p);
		return;
	}
	if (ch != ' ') {
		set_invalid(p);
		return;
	}
	if (!ds_eq(&p->result.method, "GET") && !ds_eq(&p->result.method, "POST")) {
		set_invalid(p);
		return;
	}
	p->state = ORC_ST_SPACE_BEFORE_URL;
}
/* P:190-199 */
static void h_space_before_url(orc_parser* p, unsigned char ch) {
	if (ch != '/') {
		set_invalid(p);
		return;
	}
	ds_push(&p->result.url, (char)ch);
	p->state = ORC_ST_URL;
}
/* P:201-213 */
static void h_url(orc_parser* p, unsigned char ch) {
	if (ch != ' ') {
		if (!valid_url(ch)) {
			set_invalid(p);
			return;
		}
		ds_push(&p->result.url, (char)ch);
		return;
	}
	p->state = ORC_ST_SPACE_BEFORE_PROTOCOL;
}
/* P:215-224 */
static void h_space_before_protocol(orc_parser* p, unsigned char ch) {
	if (ch != 'H') {
		set_invalid(p);
		return;
	}
	ds_push(&p->result.protocol, (char)ch);
	p->state = ORC_ST_PROTOCOL;
}
/* P:226-246 */
static void h_protocol(orc_parser* p, unsigned char ch) {
	if (ch != '\r') {
		ds_push(&p->result.protocol, (char)ch);
		size_t n = p->result.protocol.n;
		int m10 = n <= 8 && memcmp("HTTP/1.0", p->result.protocol.p, n) == 0;
		int m11 = n <= 8 && memcmp("HTTP/1.1", p->result.protocol.p, n) == 0;
		if (!m10 && !m11)
			set_invalid(p);
		return;
	}
	if (!ds_eq(&p->result.protocol, "HTTP/1.0") && !ds_eq(&p->result.protocol, "HTTP/1.1")) {
		set_invalid(p);
		return;
	}
	p->state = ORC_ST_HEADER_NEWLINE;
}
/* P:248-262 */
static void h_header_newline(orc_parser* p, unsigned char ch) {
	if (ch != '\n') {
		set_invalid(p);
		return;
	}
	if (key_is_client_ip(p) && ds_eqds(&p->result.clientIPKey, &p->hkey)) {
		p->isClientIpRead = 1;
		parse_client_ip_value(&p->result, p->hval.p, p->hval.n);
	}
	ds_clear(&p->hkey);
	ds_clear(&p->hval);
	p->state = ORC_ST_HEADER_KEY;
}
/* P:264-297 */
static void h_header_key(orc_parser* p, unsigned char ch) {
	if (ch == '\r') {
		p->state = ORC_ST_HEADERS_END;
		return;
	}
	if (ch == ' ')
		return;
	if (ch != ':') {
		if (!valid_key(ch)) {
			set_invalid(p);
			return;
		}
		if (p->hkey.n < MAX_HEADER_KEY_LENGTH)
			ds_push(&p->hkey, (char)c_tolower(ch));
		return;
	}
	if (key_is_host(p) && p->result.host.n != 0) {
		p->state = ORC_ST_INVALID;
		return;
	}
	if (key_is_client_ip(p) && p->hval.n != 0) /* P:292-294 (unreachable: value is empty here) */
		ds_push(&p->hval, ',');
	p->state = ORC_ST_SPACE_BEFORE_HEADER_VALUE;
}
/* P:299-319 */
static void h_space_before_value(orc_parser* p, unsigned char ch) {
	if (ch == ' ')
		return;
	if (!valid_value(ch)) {
		set_invalid(p);
		return;
	}
	if (key_is_host(p)) {
		ds_push(&p->result.host, (char)ch);
	} else if (key_is_client_ip(p)) {
		if (p->result.clientIPKey.n == 0)
			ds_copy(&p->result.clientIPKey, &p->hkey);
		ds_push(&p->hval, (char)ch);
	}
	p->state = ORC_ST_HEADER_VALUE;
}
/* P:321-352 */
static void h_header_value(orc_parser* p, unsigned char ch) {
	if (ch != '\r' && key_is_host(p)) {
		if (!valid_host(ch)) {
			set_invalid(p);
			return;
		}
		ds_push(&p->result.host, (char)ch);
		return;
	}
	if (ch != '\r' && key_is_client_ip(p)) {
		if (!valid_client_ip(ch)) {
			set_invalid(p);
			return;
		}
		ds_push(&p->hval, (char)ch);
		return;
	}
	if (ch != '\r' && !valid_value(ch)) {
		set_invalid(p);
		return;
	}
	if (ch != '\r')
		return;
	p->state = ORC_ST_HEADER_NEWLINE;
}
/* P:354-364 */
static void h_headers_end(orc_parser* p, unsigned char ch) {
	if (ch != '\n') {
		set_invalid(p);
		return;
	}
	p->state = ORC_ST_FINISHED;
}

/* P:124-160 */
static void handle_char(orc_parser* p, unsigned char ch) {
	switch (p->state) {
	case ORC_ST_METHOD: h_method(p, ch); break;
	case ORC_ST_SPACE_BEFORE_URL: h_space_before_url(p, ch); break;
	case ORC_ST_URL: h_url(p, ch); break;
	case ORC_ST_SPACE_BEFORE_PROTOCOL: h_space_before_protocol(p, ch); break;
	case ORC_ST_PROTOCOL: h_protocol(p, ch); break;
	case ORC_ST_HEADER_NEWLINE: h_header_newline(p, ch); break;
	case ORC_ST_HEADER_KEY: h_header_key(p, ch); break;
	case ORC_ST_SPACE_BEFORE_HEADER_VALUE: h_space_before_value(p, ch); break;
	case ORC_ST_HEADER_VALUE: h_header_value(p, ch); break;
	case ORC_ST_HEADERS_END: h_headers_end(p, ch); break;
	default: break;
	}
}

/* P:85-106 */
static size_t parser_parse(orc_parser* p, const uint8_t* data, size_t n, uint8_t flags) {
	size_t i = 0;
	while (i < n) {
		if (p->length > MAX_HTTP_REQUEST_LENGTH) {
			set_invalid(p);
			return i;
		}
		handle_char(p, data[i]);
		i++;
		p->length++;
		if (p->state == ORC_ST_FINISHED || p->state == ORC_ST_INVALID) {
			p->result.isHttps = (flags & ORC_FLAG_SSL) != 0;
			return i;
		}
	}
	return i;
}
static int parser_is_invalid(const orc_parser* p) { return p->state == ORC_ST_INVALID; }                                   /* P:108-110 */
static int parser_is_finished(const orc_parser* p) { return p->state == ORC_ST_FINISHED || p->state == ORC_ST_INVALID; } /* P:112-114 */
/* P:374-379 */
static void parser_reset(orc_parser* p) {
	p->state = ORC_ST_METHOD;
	ds_clear(&p->hkey);
	ds_clear(&p->hval);
	p->length = 0;
	req_clear(&p->result);
}

/* ------------------------------------------------------------------------------- */
/* glibc inet_pton / inet_ntop (resolv/inet_pton.c, inet/inet_ntop.c)               */
/* ------------------------------------------------------------------------------- */
int orc_inet_pton4(const char* src, size_t len, uint8_t out[4]) {
	const char* end = src + len;
	int saw_digit = 0, octets = 0;
	uint8_t tmp[4], *tp;
	*(tp = tmp) = 0;
	while (src < end) {
		int ch = (unsigned char)*src++;
		if (ch >= '0' && ch <= '9') {
			unsigned int nw = *tp * 10u + (unsigned)(ch - '0');
			if (saw_digit && *tp == 0)
				return 0;
			if (nw > 255)
				return 0;
			*tp = (uint8_t)nw;
			if (!saw_digit) {
				if (++octets > 4)
					return 0;
				saw_digit = 1;
			}
		} else if (ch == '.' && saw_digit) {
			if (octets == 4)
				return 0;
			*++tp = 0;
			saw_digit = 0;
		} else
			return 0;
	}
	if (octets < 4)
		return 0;
	memcpy(out, tmp, 4);
	return 1;
}

static int hex_digit_value(int ch) {
	if (ch >= '0' && ch <= '9')
		return ch - '0';
	if (ch >= 'a' && ch <= 'f')
		return ch - 'a' + 10;
	if (ch >= 'A' && ch <= 'F')
		return ch - 'A' + 10;
	return -1;
}

int orc_inet_pton6(const char* src, size_t len, uint8_t out[16]) {
	const char* src_endp = src + len;
	uint8_t tmp[16];
	uint8_t* tp = memset(tmp, 0, 16);
	uint8_t* endp = tp + 16;
	uint8_t* colonp = NULL;
	if (src == src_endp)
		return 0;
	if (*src == ':') {
		++src;
		if (src == src_endp || *src != ':')
			return 0;
	}
	const char* curtok = src;
	size_t xdigits_seen = 0;
	unsigned int val = 0;
	while (src < src_endp) {
		int ch = (unsigned char)*src++;
		int digit = hex_digit_value(ch);
		if (digit >= 0) {
			if (xdigits_seen == 4)
				return 0;
			val <<= 4;
			val |= (unsigned)digit;
			if (val > 0xffff)
				return 0;
			++xdigits_seen;
			continue;
		}
		if (ch == ':') {
			curtok = src;
			if (xdigits_seen == 0) {
				if (colonp)
					return 0;
				colonp = tp;
				continue;
			} else if (src == src_endp)
				return 0;
			if (tp + 2 > endp)
				return 0;
			*tp++ = (uint8_t)(val >> 8);
			*tp++ = (uint8_t)val;
			xdigits_seen = 0;
			val = 0;
			continue;
		}
		if (ch == '.' && ((tp + 4) <= endp) && orc_inet_pton4(curtok, (size_t)(src_endp - curtok), tp) > 0) {
			tp += 4;
			xdigits_seen = 0;
			break;
		}
		return 0;
	}
	if (xdigits_seen > 0) {
		if (tp + 2 > endp)
			return 0;
		*tp++ = (uint8_t)(val >> 8);
		*tp++ = (uint8_t)val;
	}
	if (colonp != NULL) {
		if (tp == endp)
			return 0;
		size_t n = (size_t)(tp - colonp);
		memmove(endp - n, colonp, n);
		memset(colonp, 0, (size_t)(endp - n - colonp));
		tp = endp;
	}
	if (tp != endp)
		return 0;
	memcpy(out, tmp, 16);
	return 1;
}

static char* put_u64(char* o, uint64_t v) {
	char b[24];
	int k = 0;
	do {
		b[k++] = (char)('0' + v % 10);
		v /= 10;
	} while (v);
	while (k)
		*o++ = b[--k];
	return o;
}

static char* put_u(char* o, unsigned v) {
	char b[12];
	int k = 0;
	do {
		b[k++] = (char)('0' + v % 10);
		v /= 10;
	} while (v);
	while (k)
		*o++ = b[--k];
	return o;
}
static char* put_x(char* o, unsigned v) {
	char b[8];
	int k = 0;
	do {
		b[k++] = "0123456789abcdef"[v & 15];
		v >>= 4;
	} while (v);
	while (k)
		*o++ = b[--k];
	return o;
}
void orc_inet_ntop4(const uint8_t in[4], char out[16]) {
	char* o = out;
	for (int i = 0; i < 4; i++) {
		if (i)
			*o++ = '.';
		o = put_u(o, in[i]);
	}
	*o = 0;
}
void orc_inet_ntop6(const uint8_t in[16], char out[46]) {
	unsigned words[8];
	for (int i = 0; i < 8; i++)
		words[i] = ((unsigned)in[2 * i] << 8) | in[2 * i + 1];
	int best_base = -1, best_len = 0, cur_base = -1, cur_len = 0;
	for (int i = 0; i < 8; i++) {
		if (words[i] == 0) {
			if (cur_base == -1) {
				cur_base = i;
				cur_len = 1;
			} else
				cur_len++;
		} else if (cur_base != -1) {
			if (best_base == -1 || cur_len > best_len) {
				best_base = cur_base;
				best_len = cur_len;
			}
			cur_base = -1;
		}
	}
	if (cur_base != -1 && (best_base == -1 || cur_len > best_len)) {
		best_base = cur_base;
		best_len = cur_len;
	}
	if (best_base != -1 && best_len < 2)
		best_base = -1;
	char* tp = out;
	for (int i = 0; i < 8; i++) {
		if (best_base != -1 && i >= best_base && i < best_base + best_len) {
			if (i == best_base)
				*tp++ = ':';
			continue;
		}
		if (i != 0)
			*tp++ = ':';
		if (i == 6 && best_base == 0 && (best_len == 6 || (best_len == 5 && words[5] == 0xffff))) {
			char v4[16];
			orc_inet_ntop4(in + 12, v4);
			size_t l = strlen(v4);
			memcpy(tp, v4, l);
			tp += l;
			break;
		}
		tp = put_x(tp, words[i]);
	}
	if (best_base != -1 && best_base + best_len == 8)
		*tp++ = ':';
	*tp = 0;
}

/* ------------------------------------------------------------------------------- */
/* LRUCache (L:26-107): hashed unique index + sequenced list                        */
/* ------------------------------------------------------------------------------- */
typedef struct lru_node {
	uint32_t k[3];
	struct lru_node *prev, *next; /* sequenced: head = most recently used */
	struct lru_node* hnext;       /* bucket chain */
	void* value;
	int64_t ivalue;
} lru_node;

typedef struct {
	lru_node** buckets;
	uint32_t nb;
	uint32_t size, capacity;
	lru_node *head, *tail;
	uint64_t evictions;
	void (*free_value)(void*);
} lru_t;

static uint32_t key_hash(const uint32_t k[3]) {
	uint64_t h = 1469598103934665603ull;
	for (int i = 0; i < 3; i++) {
		h ^= k[i];
		h *= 1099511628211ull;
		h ^= h >> 29;
	}
	return (uint32_t)h;
}
static void lru_init(lru_t* l, uint32_t cap, void (*fv)(void*)) {
	memset(l, 0, sizeof(*l));
	l->capacity = cap;
	l->nb = 1024;
	while (l->nb < cap * 2u && l->nb < (1u << 24))
		l->nb *= 2;
	l->buckets = (lru_node**)calloc(l->nb, sizeof(lru_node*));
	l->free_value = fv;
}
static lru_node* lru_lookup(lru_t* l, const uint32_t k[3]) {
	for (lru_node* n = l->buckets[key_hash(k) & (l->nb - 1)]; n; n = n->hnext)
		if (n->k[0] == k[0] && n->k[1] == k[1] && n->k[2] == k[2])
			return n;
	return NULL;
}
static void seq_unlink(lru_t* l, lru_node* n) {
	if (n->prev)
		n->prev->next = n->next;
	else
		l->head = n->next;
	if (n->next)
		n->next->prev = n->prev;
	else
		l->tail = n->prev;
	n->prev = n->next = NULL;
}
static void seq_push_front(lru_t* l, lru_node* n) {
	n->prev = NULL;
	n->next = l->head;
	if (l->head)
		l->head->prev = n;
	l->head = n;
	if (!l->tail)
		l->tail = n;
}
static void lru_remove(lru_t* l, lru_node* n) {
	lru_node** pp = &l->buckets[key_hash(n->k) & (l->nb - 1)];
	while (*pp != n)
		pp = &(*pp)->hnext;
	*pp = n->hnext;
	seq_unlink(l, n);
	if (l->free_value && n->value)
		l->free_value(n->value);
	free(n);
	l->size--;
}
/* L:50-63: new key at size >= capacity evicts the tail; existing key moves to front and is overwritten */
static lru_node* lru_insert(lru_t* l, const uint32_t k[3]) {
	lru_node* n = lru_lookup(l, k);
	if (n) {
		seq_unlink(l, n);
		seq_push_front(l, n);
		return n; /* caller overwrites the value (L:61) */
	}
	if (l->size >= l->capacity && l->tail) {
		lru_remove(l, l->tail); /* L:56-58 pop_back */
		l->evictions++;
	}
	n = (lru_node*)calloc(1, sizeof(lru_node));
	memcpy(n->k, k, sizeof(n->k));
	uint32_t b = key_hash(k) & (l->nb - 1);
	n->hnext = l->buckets[b];
	l->buckets[b] = n;
	seq_push_front(l, n);
	l->size++;
	return n;
}
/* L:70-81: find touches (moves to front) */
static lru_node* lru_find(lru_t* l, const uint32_t k[3]) {
	lru_node* n = lru_lookup(l, k);
	if (n) {
		seq_unlink(l, n);
		seq_push_front(l, n);
	}
	return n;
}
static void lru_destroy(lru_t* l) {
	while (l->head)
		lru_remove(l, l->head);
	free(l->buckets);
}

struct orc_lru {
	lru_t l;
};
orc_lru* orc_lru_new(uint32_t capacity) {
	orc_lru* x = (orc_lru*)calloc(1, sizeof(orc_lru));
	lru_init(&x->l, capacity, NULL);
	return x;
}
void orc_lru_free(orc_lru* x) {
	lru_destroy(&x->l);
	free(x);
}
void orc_lru_insert(orc_lru* x, uint32_t key, int64_t value) {
	uint32_t k[3] = {key, 0, 0};
	lru_node* n = lru_insert(&x->l, k);
	n->ivalue = value;
}
int orc_lru_find(orc_lru* x, uint32_t key, int64_t* value) {
	uint32_t k[3] = {key, 0, 0};
	lru_node* n = lru_find(&x->l, k);
	if (!n)
		return 0;
	if (value)
		*value = n->ivalue;
	return 1;
}
int orc_lru_erase(orc_lru* x, uint32_t key) {
	uint32_t k[3] = {key, 0, 0};
	lru_node* n = lru_lookup(&x->l, k);
	if (!n)
		return 0;
	lru_remove(&x->l, n);
	return 1;
}
/* L:83-85: update does not move the entry */
int orc_lru_update(orc_lru* x, uint32_t key, int64_t value) {
	uint32_t k[3] = {key, 0, 0};
	lru_node* n = lru_lookup(&x->l, k);
	if (!n)
		return 0;
	n->ivalue = value;
	return 1;
}
uint32_t orc_lru_size(const orc_lru* x) { return x->l.size; }

/* ------------------------------------------------------------------------------- */
/* Services (Service.h:43-66) and the Aggregator (A:44-168)                         */
/* ------------------------------------------------------------------------------- */
typedef struct svc {
	uint32_t pid;
	dstr endpoint, domain, scheme;
	uint32_t internal, external; /* uint32, wraps like Service.h:53-54 */
	uint64_t first;              /* index of the event whose request created it (first arrival) */
	uint32_t nets[3];            /* sizes of externalIPv4_16ClientNets, _24ClientNets, IPv6ClientsNets (S:56-58) */
	struct svc* hnext;
} svc;

/* One entry of a service's network map (S:45-50: prefix -> time last seen).  The maps of all
 * services live in one open-addressing table keyed by (service, kind, prefix); an erased
 * entry keeps its key (alive = 0) until the next clear rebuilds the table. */
typedef struct {
	svc* s;            /* NULL: empty slot */
	uint8_t kind;      /* 0: v4 /16, 1: v4 /24, 2: v6 48-bit prefix */
	uint8_t prefix[6]; /* address bytes in network order */
	uint8_t alive;
	uint64_t time;     /* steady-clock ns of the last request (A:97-100: map[key] = currentTime) */
} net_ent;

typedef struct {
	uint8_t addr[4], mask[4];
} v4net;
typedef struct {
	uint8_t addr[16], mask[16];
} v6net;

struct orc_ctx {
	lru_t sessions; /* Discovery::savedSessions, D:39 */
	svc** sb;
	uint32_t snb;
	svc** list;
	uint64_t nsvc, listcap;
	v4net* v4;
	uint32_t n4;
	v6net* v6;
	uint32_t n6;
	int* mock;
	uint32_t nmock, imock;
	int use_mock;
	dstr blob;
	orc_stats st;
	uint64_t cur_event; /* index of the event being handled, over all orc_process calls */
	struct {
		uint32_t length;
		uint8_t data[8192 + 16]; /* + the 16 readable pad bytes some callers pass after a buffer */
	} saved;                    /* DiscoverySavedBuffer, Types.h:58-61 */
	int netcounters;    /* Aggregator(..., enableNetworkCounters) A:132-134 */
	uint64_t now;       /* getCurrentTime() (A:211-213) for the next requests */
	net_ent* nt;
	uint64_t ntcap, ntused;
};

static void free_parser_value(void* v) {
	parser_destroy((orc_parser*)v);
	free(v);
}

orc_ctx* orc_create(uint32_t lru_capacity) {
	orc_ctx* c = (orc_ctx*)calloc(1, sizeof(orc_ctx));
	lru_init(&c->sessions, lru_capacity ? lru_capacity : 8192, free_parser_value);
	c->snb = 1u << 16;
	c->sb = (svc**)calloc(c->snb, sizeof(svc*));
	return c;
}

static void svc_free_all(orc_ctx* c) {
	for (uint64_t i = 0; i < c->nsvc; i++) {
		svc* s = c->list[i];
		ds_free(&s->endpoint);
		ds_free(&s->domain);
		ds_free(&s->scheme);
		free(s);
	}
	c->nsvc = 0;
	memset(c->sb, 0, c->snb * sizeof(svc*));
}

static void nets_rebuild(orc_ctx* c, uint64_t cap);
static void svc_reindex(orc_ctx* c);

/* A:136-153.  Network counters off (the default, main.cpp:78): every service goes.  On:
 * services whose three network maps are all empty go, the others stay with their client
 * counters zeroed. */
void orc_clear(orc_ctx* c) {
	if (!c->netcounters) {
		svc_free_all(c);
		return;
	}
	uint64_t k = 0;
	for (uint64_t i = 0; i < c->nsvc; i++) {
		svc* s = c->list[i];
		if (s->nets[0] == 0 && s->nets[1] == 0 && s->nets[2] == 0) {
			ds_free(&s->endpoint);
			ds_free(&s->domain);
			ds_free(&s->scheme);
			free(s);
		} else {
			s->external = 0;
			s->internal = 0;
			c->list[k++] = s;
		}
	}
	c->nsvc = k;
	svc_reindex(c);
	nets_rebuild(c, c->ntcap); /* only live entries (of kept services) survive */
}

void orc_destroy(orc_ctx* c) {
	svc_free_all(c);
	free(c->sb);
	free(c->list);
	lru_destroy(&c->sessions);
	free(c->v4);
	free(c->v6);
	free(c->mock);
	free(c->nt);
	ds_free(&c->blob);
	free(c);
}

void orc_set_interfaces(orc_ctx* c, const uint8_t* v4, uint32_t n4, const uint8_t* v6, uint32_t n6) {
	free(c->v4);
	free(c->v6);
	c->v4 = (v4net*)calloc(n4 ? n4 : 1, sizeof(v4net));
	c->v6 = (v6net*)calloc(n6 ? n6 : 1, sizeof(v6net));
	if (n4)
		memcpy(c->v4, v4, n4 * sizeof(v4net));
	if (n6)
		memcpy(c->v6, v6, n6 * sizeof(v6net));
	c->n4 = n4;
	c->n6 = n6;
}

void orc_set_checker_mock(orc_ctx* c, const int* verdicts, uint32_t n) {
	free(c->mock);
	c->mock = (int*)calloc(n ? n : 1, sizeof(int));
	if (n)
		memcpy(c->mock, verdicts, n * sizeof(int));
	c->nmock = n;
	c->imock = 0;
	c->use_mock = 1;
}

/* IC:39-85 — addr is in network byte order (in_addr.s_addr bytes) */
static int v4_external(orc_ctx* c, const uint8_t a[4]) {
	static const struct {
		uint32_t network, mask;
	} reserved[] = {
			{0x00000000, 0xff000000}, {0x0a000000, 0xff000000}, {0x64400000, 0xffc00000}, {0x7f000000, 0xff000000},
			{0xa9fe0000, 0xffff0000}, {0xac100000, 0xfff00000}, {0xc0000000, 0xffffff00}, {0xc0000200, 0xffffff00},
			{0xc0586300, 0xffffff00}, {0xc0a80000, 0xffff0000}, {0xc6120000, 0xfffe0000}, {0xc6336400, 0xffffff00},
			{0xcb007100, 0xffffff00}, {0xe0000000, 0xf0000000}, {0xe9fc0000, 0xffff0000}, {0xf0000000, 0xf0000000},
			{0xffffffff, 0xffffffff}};
	uint32_t h = ((uint32_t)a[0] << 24) | ((uint32_t)a[1] << 16) | ((uint32_t)a[2] << 8) | a[3]; /* ntohl */
	for (size_t i = 0; i < sizeof(reserved) / sizeof(reserved[0]); i++)
		if ((h & reserved[i].mask) == reserved[i].network)
			return 0;
	for (uint32_t i = 0; i < c->n4; i++) { /* IC:74-82, checkSubnetIpv4 IC:139-145 */
		int eq = 1;
		for (int k = 0; k < 4; k++)
			if ((a[k] & c->v4[i].mask[k]) != (c->v4[i].addr[k] & c->v4[i].mask[k]))
				eq = 0;
		if (eq)
			return 0;
	}
	return 1;
}

/* IC:98-126 isInRange: prefix compare of a range given as (bytes, prefix length) */
static int in_range6(const uint8_t a[16], const uint8_t net[16], int prefix) {
	for (int i = 0; i < 16; i++) {
		uint8_t m;
		if (prefix >= 8) {
			m = 0xff;
			prefix -= 8;
		} else if (prefix > 0) {
			m = (uint8_t)(0xff << (8 - prefix));
			prefix = 0;
		} else
			m = 0;
		if ((a[i] & m) != net[i])
			return 0;
	}
	return 1;
}

/* IC:146-180 */
static int v6_external(orc_ctx* c, const uint8_t a[16]) {
	/* IC:71-88: "::ffff:0:0/96", "::ffff:0:0:0/96", "64:ff9b::/96" (parsed with inet_pton) */
	static const char* mapped[3] = {"::ffff:0:0", "::ffff:0:0:0", "64:ff9b::"};
	for (int r = 0; r < 3; r++) {
		uint8_t net[16];
		orc_inet_pton6(mapped[r], strlen(mapped[r]), net);
		if (in_range6(a, net, 96))
			return v4_external(c, a + 12);
	}
	for (uint32_t i = 0; i < c->n6; i++) { /* checkSubnet IC:128-137 (32-bit words, same as bytes) */
		int eq = 1;
		for (int k = 0; k < 16; k++)
			if ((a[k] & c->v6[i].mask[k]) != (c->v6[i].addr[k] & c->v6[i].mask[k]))
				eq = 0;
		if (eq)
			return 0;
	}
	static const char* internal[4] = {"fc00::", "fec0::", "fe80::", "::1"};
	static const int plen[4] = {7, 10, 10, 128};
	for (int r = 0; r < 4; r++) {
		uint8_t net[16];
		orc_inet_pton6(internal[r], strlen(internal[r]), net);
		if (in_range6(a, net, plen[r]))
			return 0;
	}
	return 1;
}

int orc_is_v4_external(orc_ctx* c, const uint8_t addr[4]) { return v4_external(c, addr); }
int orc_is_v6_external(orc_ctx* c, const uint8_t addr[16]) { return v6_external(c, addr); }

static int checker_v4(orc_ctx* c, const uint8_t a[4]) {
	if (c->use_mock)
		return c->imock < c->nmock ? c->mock[c->imock++] : 0;
	return v4_external(c, a);
}
static int checker_v6(orc_ctx* c, const uint8_t a[16]) {
	if (c->use_mock)
		return c->imock < c->nmock ? c->mock[c->imock++] : 0;
	return v6_external(c, a);
}

static void net_touch(orc_ctx* c, svc* s, uint8_t kind, const uint8_t* pfx, int n);

/* A:44-110 incrementServiceClientsNumber.  Returns ORC_CLASS_*; with network counters on,
 * an external client's networks go into the service's maps (A:89-106). */
static int client_class(orc_ctx* c, svc* sv, const orc_request* r, uint8_t flags, const uint8_t* src) {
	char addr[64];
	size_t alen;
	int is6 = 0;
	dstr tmp = {0};
	const char* s;
	if (r->clientIp.n != 0) { /* A:52-56 */
		s = r->clientIp.v[0].p;
		alen = r->clientIp.v[0].n;
		size_t colons = 0;
		for (size_t i = 0; i < alen; i++)
			if (s[i] == ':')
				colons++;
		if (colons >= 2)
			is6 = 1;
		/* inet_pton reads a NUL-terminated c_str(): stop at an embedded NUL (none can occur) */
		ds_set(&tmp, s, alen);
		tmp.p[alen] = 0;
		alen = strlen(tmp.p);
		s = tmp.p;
	} else if (flags & ORC_FLAG_IPV4) { /* A:57-58: ipv4ToString, IA:21-30 */
		orc_inet_ntop4(src, addr);
		s = addr;
		alen = strlen(addr);
	} else if (flags & ORC_FLAG_IPV6) { /* A:59-61: ipv6ToString, IA:36-45 */
		orc_inet_ntop6(src, addr);
		s = addr;
		alen = strlen(addr);
		is6 = 1;
	} else {
		return ORC_CLASS_NONE; /* A:62-63 */
	}
	int ext, ok;
	uint8_t b[16] = {0};
	if (is6) {
		ok = orc_inet_pton6(s, alen, b);
		ext = ok ? checker_v6(c, b) : 0;
	} else {
		ok = orc_inet_pton4(s, alen, b);
		ext = ok ? checker_v4(c, b) : 0;
	}
	ds_free(&tmp);
	if (!ok)
		return ORC_CLASS_NONE; /* A:66-84: parse failure is swallowed */
	if (ext && c->netcounters) {
		if (is6) {
			net_touch(c, sv, 2, b, 6); /* A:91-94: the first ipv6NetworkPrefixBytesLen (6) bytes, S:41 */
		} else {
			net_touch(c, sv, 1, b, 3); /* A:96-97: s_addr & 0xFFFFFF = the first three bytes */
			net_touch(c, sv, 0, b, 2); /* A:99-100: s_addr & 0xFFFF = the first two */
		}
	}
	return ext ? ORC_CLASS_EXTERNAL : ORC_CLASS_INTERNAL;
}

/* ------------------------------------------------------------------------------- */
/* Network maps (S:45-58; A:89-106 insert, A:182-209 networkCountersCleaning)       */
/* ------------------------------------------------------------------------------- */
static uint64_t net_hash(const svc* s, uint8_t kind, const uint8_t pfx[6]) {
	uint64_t h = (uint64_t)(uintptr_t)s * 0x9E3779B97F4A7C15ull ^ kind;
	for (int i = 0; i < 6; i++)
		h = (h ^ pfx[i]) * 1099511628211ull;
	return h ^ (h >> 29);
}

static net_ent* net_slot(orc_ctx* c, const svc* s, uint8_t kind, const uint8_t pfx[6]) {
	uint64_t i = net_hash(s, kind, pfx) & (c->ntcap - 1);
	for (;;) {
		net_ent* e = &c->nt[i];
		if (!e->s || (e->s == s && e->kind == kind && memcmp(e->prefix, pfx, 6) == 0))
			return e;
		i = (i + 1) & (c->ntcap - 1);
	}
}

/* rehash the live entries into a table of `cap` slots (dead ones are dropped) */
static void nets_rebuild(orc_ctx* c, uint64_t cap) {
	net_ent* old = c->nt;
	uint64_t oc = c->ntcap;
	c->ntcap = cap < 1024 ? 1024 : cap;
	c->nt = (net_ent*)calloc(c->ntcap, sizeof(net_ent));
	c->ntused = 0;
	for (uint64_t i = 0; i < oc; i++)
		if (old[i].s && old[i].alive) {
			*net_slot(c, old[i].s, old[i].kind, old[i].prefix) = old[i];
			c->ntused++;
		}
	free(old);
}

/* map[prefix] = currentTime (A:94, 97, 100): a new or erased key adds one to the map's size */
static void net_touch(orc_ctx* c, svc* s, uint8_t kind, const uint8_t* pfx, int n) {
	if (2 * (c->ntused + 1) > c->ntcap)
		nets_rebuild(c, c->ntcap ? 2 * c->ntcap : 1024);
	uint8_t key[6] = {0};
	memcpy(key, pfx, (size_t)n);
	net_ent* e = net_slot(c, s, kind, key);
	if (!e->s) {
		e->s = s;
		e->kind = kind;
		memcpy(e->prefix, key, 6);
		c->ntused++;
	}
	if (!e->alive) {
		e->alive = 1;
		s->nets[kind]++;
	}
	e->time = c->now;
}

void orc_set_network_counters(orc_ctx* c, int on) { c->netcounters = on; }
void orc_set_time(orc_ctx* c, uint64_t now) { c->now = now; }

/* A:182-209: erase every entry with currentTime - seen >= 1 h (std::chrono::hours(1)) */
void orc_network_counters_cleaning(orc_ctx* c, uint64_t now) {
	const uint64_t retention = 3600ull * 1000000000ull;
	for (uint64_t i = 0; i < c->ntcap; i++) {
		net_ent* e = &c->nt[i];
		if (e->s && e->alive && (int64_t)(now - e->time) >= (int64_t)retention) {
			e->alive = 0;
			e->s->nets[e->kind]--;
		}
	}
}

static uint64_t svc_hash(uint32_t pid, const char* ep, size_t n) {
	uint64_t h = 1469598103934665603ull ^ pid;
	for (size_t i = 0; i < n; i++) {
		h ^= (unsigned char)ep[i];
		h *= 1099511628211ull;
	}
	return h ^ (h >> 31);
}

/* the hash index over c->list after the list changed (clear with network counters) */
static void svc_reindex(orc_ctx* c) {
	memset(c->sb, 0, c->snb * sizeof(svc*));
	for (uint64_t i = 0; i < c->nsvc; i++) {
		svc* s = c->list[i];
		uint32_t h = (uint32_t)svc_hash(s->pid, s->endpoint.p, s->endpoint.n) & (c->snb - 1);
		s->hnext = c->sb[h];
		c->sb[h] = s;
	}
}

static void svc_index_grow(orc_ctx* c) {
	uint32_t nb = c->snb * 2;
	svc** b = (svc**)calloc(nb, sizeof(svc*));
	for (uint64_t i = 0; i < c->nsvc; i++) {
		svc* s = c->list[i];
		uint32_t h = (uint32_t)svc_hash(s->pid, s->endpoint.p, s->endpoint.n) & (nb - 1);
		s->hnext = b[h];
		b[h] = s;
	}
	free(c->sb);
	c->sb = b;
	c->snb = nb;
}

/* A:155-168 newRequest + A:112-130 toService.  Returns the client class. */
static int agg_new_request(orc_ctx* c, const orc_request* r, uint32_t pid, uint8_t flags, const uint8_t* src) {
	dstr ep = {0};
	ds_reserve(&ep, r->host.n + r->url.n + 1); /* A:27-29 getEndpoint = host + url */
	memcpy(ep.p, r->host.p, r->host.n);
	memcpy(ep.p + r->host.n, r->url.p, r->url.n);
	ep.n = r->host.n + r->url.n;
	c->st.requests++;
	uint32_t b = (uint32_t)svc_hash(pid, ep.p, ep.n) & (c->snb - 1);
	for (svc* s = c->sb[b]; s; s = s->hnext) {
		if (s->pid == pid && ds_eqds(&s->endpoint, &ep)) {
			int cls = client_class(c, s, r, flags, src);
			if (cls == ORC_CLASS_EXTERNAL)
				s->external++;
			else if (cls == ORC_CLASS_INTERNAL)
				s->internal++;
			ds_free(&ep);
			return cls;
		}
	}
	svc* s = (svc*)calloc(1, sizeof(svc));
	s->pid = pid;
	s->endpoint = ep;
	s->first = c->cur_event;
	/* A:117-125 domain */
	const char* h = r->host.p;
	size_t hn = r->host.n;
	size_t lb = (size_t)-1;
	for (size_t i = 0; i < hn; i++)
		if (h[i] == '[') {
			lb = i;
			break;
		}
	if (lb != (size_t)-1) {
		size_t rb = (size_t)-1;
		for (size_t i = lb + 1; i < hn; i++)
			if (h[i] == ']') {
				rb = i;
				break;
			}
		if (rb != (size_t)-1)
			ds_set(&s->domain, h + lb, rb - lb + 1);
		else
			ds_set(&s->domain, "", 0);
	} else {
		size_t colon = hn;
		for (size_t i = 0; i < hn; i++)
			if (h[i] == ':') {
				colon = i;
				break;
			}
		ds_set(&s->domain, h, colon);
	}
	if (r->isHttps) /* A:127 */
		ds_set(&s->scheme, "https", 5);
	else
		ds_set(&s->scheme, "http", 4);
	int cls = client_class(c, s, r, flags, src); /* A:128 */
	if (cls == ORC_CLASS_EXTERNAL)
		s->external++;
	else if (cls == ORC_CLASS_INTERNAL)
		s->internal++;
	if (c->nsvc == c->listcap) {
		c->listcap = c->listcap ? c->listcap * 2 : 1024;
		c->list = (svc**)realloc(c->list, c->listcap * sizeof(svc*));
	}
	c->list[c->nsvc++] = s;
	s->hnext = c->sb[b];
	c->sb[b] = s;
	if (c->nsvc > (uint64_t)c->snb)
		svc_index_grow(c);
	return cls;
}

void orc_agg_new_request(orc_ctx* c, uint32_t pid, const char* host, const char* url, const char* cip, uint8_t flags,
		const uint8_t* source_ip16) {
	orc_request r;
	uint8_t zero[16] = {0};
	req_init(&r);
	ds_set(&r.host, host, strlen(host));
	ds_set(&r.url, url, strlen(url));
	if (cip)
		dl_push(&r.clientIp, cip, strlen(cip));
	r.isHttps = (flags & ORC_FLAG_SSL) != 0;
	agg_new_request(c, &r, pid, flags, source_ip16 ? source_ip16 : zero);
	req_free(&r);
}

static int svc_cmp(const void* a, const void* b) {
	const svc* x = *(const svc* const*)a;
	const svc* y = *(const svc* const*)b;
	if (x->pid != y->pid)
		return x->pid < y->pid ? -1 : 1;
	size_t n = x->endpoint.n < y->endpoint.n ? x->endpoint.n : y->endpoint.n;
	int r = n ? memcmp(x->endpoint.p, y->endpoint.p, n) : 0;
	if (r)
		return r;
	return x->endpoint.n < y->endpoint.n ? -1 : (x->endpoint.n > y->endpoint.n);
}

uint64_t orc_service_count(orc_ctx* c) { return c->nsvc; }

static uint64_t services_dump(orc_ctx* c, char* buf, uint64_t cap, int with_first);

uint64_t orc_services_dump(orc_ctx* c, char* buf, uint64_t cap) { return services_dump(c, buf, cap, 0); }
uint64_t orc_services_dump_first(orc_ctx* c, char* buf, uint64_t cap) { return services_dump(c, buf, cap, 1); }
uint64_t orc_services_dump_nets(orc_ctx* c, char* buf, uint64_t cap) { return services_dump(c, buf, cap, 2); }

static uint64_t ds_out(dstr* out, char* buf, uint64_t cap) {
	uint64_t need = out->n;
	if (buf && cap >= need && need)
		memcpy(buf, out->p, need);
	ds_free(out);
	return need;
}

static void ds_puts(dstr* o, const char* p, size_t n) {
	for (size_t k = 0; k < n; k++)
		ds_push(o, p[k]);
}

/* Every live network-map entry: pid \t endpoint \t kind(1 /16, 2 /24, 3 v6) \t prefix hex (6 bytes)
 * \t time \n, unsorted. */
uint64_t orc_nets_dump(orc_ctx* c, char* buf, uint64_t cap) {
	dstr out = {0};
	char num[32];
	static const char hx[] = "0123456789abcdef";
	for (uint64_t i = 0; i < c->ntcap; i++) {
		const net_ent* e = &c->nt[i];
		if (!e->s || !e->alive)
			continue;
		char* q = put_u(num, e->s->pid);
		ds_puts(&out, num, (size_t)(q - num));
		ds_push(&out, '\t');
		ds_puts(&out, e->s->endpoint.p, e->s->endpoint.n);
		ds_push(&out, '\t');
		ds_push(&out, (char)('1' + (e->kind == 0 ? 0 : e->kind == 1 ? 1 : 2)));
		ds_push(&out, '\t');
		for (int k = 0; k < 6; k++) {
			ds_push(&out, hx[e->prefix[k] >> 4]);
			ds_push(&out, hx[e->prefix[k] & 15]);
		}
		ds_push(&out, '\t');
		q = put_u64(num, e->time);
		ds_puts(&out, num, (size_t)(q - num));
		ds_push(&out, '\n');
	}
	return ds_out(&out, buf, cap);
}

/* boost::json::serialize of a string (boost 1.83 serializer: '"' and '\\' escaped, \b \t \n
 * \f \r by name, other bytes below 0x20 as \u00xx with lower-case hex; everything else,
 * bytes >= 0x80 included, as is). */
static void json_string(dstr* o, const char* p, size_t n) {
	static const char hx[] = "0123456789abcdef";
	ds_push(o, '"');
	for (size_t k = 0; k < n; k++) {
		unsigned char ch = (unsigned char)p[k];
		switch (ch) {
		case '"': ds_puts(o, "\\\"", 2); break;
		case '\\': ds_puts(o, "\\\\", 2); break;
		case '\b': ds_puts(o, "\\b", 2); break;
		case '\t': ds_puts(o, "\\t", 2); break;
		case '\n': ds_puts(o, "\\n", 2); break;
		case '\f': ds_puts(o, "\\f", 2); break;
		case '\r': ds_puts(o, "\\r", 2); break;
		default:
			if (ch < 0x20) {
				ds_puts(o, "\\u00", 4);
				ds_push(o, hx[ch >> 4]);
				ds_push(o, hx[ch & 15]);
			} else {
				ds_push(o, (char)ch);
			}
		}
	}
	ds_push(o, '"');
}

/* Discovery::outputServicesToStdout (D:60-71): {"service": value_from(services)} through
 * boost::json::ext::print (Json.h:32-71) and std::endl, services in creation order.  Service
 * fields in BOOST_DESCRIBE_STRUCT order (S:69-80); an empty string or an empty map (null,
 * S:84-98) is skipped, but "," is written before every field but the object's first (J:38-46).
 * No services: nothing (D:62-64). */
uint64_t orc_services_json(orc_ctx* c, char* buf, uint64_t cap) {
	dstr out = {0};
	if (c->nsvc == 0)
		return ds_out(&out, buf, cap);
	char num[32];
	ds_puts(&out, "{\"service\":[", 12);
	for (uint64_t i = 0; i < c->nsvc; i++) {
		const svc* s = c->list[i];
		if (i)
			ds_push(&out, ',');
		ds_push(&out, '{');
		/* field 0 is pid, a number: never skipped, so every later field is preceded by ',' */
		char* q = put_u(num, s->pid);
		ds_puts(&out, "\"pid\":", 6);
		ds_puts(&out, num, (size_t)(q - num));
		const char* names[3] = {"endpoint", "domain", "scheme"};
		const dstr* vals[3] = {&s->endpoint, &s->domain, &s->scheme};
		for (int f = 0; f < 3; f++) {
			if (vals[f]->n == 0)
				continue;
			ds_push(&out, ',');
			json_string(&out, names[f], strlen(names[f]));
			ds_push(&out, ':');
			json_string(&out, vals[f]->p, vals[f]->n);
		}
		const char* cn[5] = {"internalClientsNumber", "externalClientsNumber", "externalIPv4_16ClientNets",
				"externalIPv4_24ClientNets", "externalIPv6ClientsNets"};
		const uint32_t cv[5] = {s->internal, s->external, s->nets[0], s->nets[1], s->nets[2]};
		for (int f = 0; f < 5; f++) {
			if (f >= 2 && cv[f] == 0) /* an empty map is null */
				continue;
			ds_push(&out, ',');
			json_string(&out, cn[f], strlen(cn[f]));
			ds_push(&out, ':');
			q = put_u(num, cv[f]);
			ds_puts(&out, num, (size_t)(q - num));
		}
		ds_push(&out, '}');
	}
	ds_puts(&out, "]}\n", 3);
	return ds_out(&out, buf, cap);
}

static uint64_t services_dump(orc_ctx* c, char* buf, uint64_t cap, int with_first) {
	svc** v = (svc**)malloc((c->nsvc ? c->nsvc : 1) * sizeof(svc*));
	memcpy(v, c->list, c->nsvc * sizeof(svc*));
	qsort(v, c->nsvc, sizeof(svc*), svc_cmp);
	dstr out = {0};
	char num[32];
	for (uint64_t i = 0; i < c->nsvc; i++) {
		svc* s = v[i];
		char* e = put_u(num, s->pid);
		for (char* q = num; q < e; q++)
			ds_push(&out, *q);
		ds_push(&out, '\t');
		for (size_t k = 0; k < s->endpoint.n; k++)
			ds_push(&out, s->endpoint.p[k]);
		ds_push(&out, '\t');
		for (size_t k = 0; k < s->domain.n; k++)
			ds_push(&out, s->domain.p[k]);
		ds_push(&out, '\t');
		for (size_t k = 0; k < s->scheme.n; k++)
			ds_push(&out, s->scheme.p[k]);
		ds_push(&out, '\t');
		e = put_u(num, s->internal);
		for (char* q = num; q < e; q++)
			ds_push(&out, *q);
		ds_push(&out, '\t');
		e = put_u(num, s->external);
		for (char* q = num; q < e; q++)
			ds_push(&out, *q);
		if (with_first & 1) {
			ds_push(&out, '\t');
			e = put_u64(num, s->first);
			for (char* q = num; q < e; q++)
				ds_push(&out, *q);
		}
		if (with_first & 2)
			for (int k = 0; k < 3; k++) {
				ds_push(&out, '\t');
				e = put_u(num, s->nets[k]);
				for (char* q = num; q < e; q++)
					ds_push(&out, *q);
			}
		ds_push(&out, '\n');
	}
	free(v);
	uint64_t need = out.n;
	if (buf && cap >= need && need)
		memcpy(buf, out.p, need);
	ds_free(&out);
	return need;
}

/* ------------------------------------------------------------------------------- */
/* Discovery event handling (D:73-198)                                              */
/* ------------------------------------------------------------------------------- */
static uint64_t blob_put(orc_ctx* c, const char* d, size_t n) {
	uint64_t at = c->blob.n;
	ds_reserve(&c->blob, c->blob.n + n + 1);
	if (n)
		memcpy(c->blob.p + c->blob.n, d, n);
	c->blob.n += n;
	return at;
}

static void fill_finished(orc_ctx* c, orc_event_result* o, const orc_request* r, int cls) {
	o->cls = (uint32_t)cls;
	o->is_https = (uint32_t)r->isHttps;
	o->host_off = blob_put(c, r->host.p, r->host.n);
	o->host_len = (uint32_t)r->host.n;
	o->url_off = blob_put(c, r->url.p, r->url.n);
	o->url_len = (uint32_t)r->url.n;
	if (r->clientIp.n) {
		o->has_cip = 1;
		o->cip_off = blob_put(c, r->clientIp.v[0].p, r->clientIp.v[0].n);
		o->cip_len = (uint32_t)r->clientIp.v[0].n;
	}
}

static uint32_t status_of(const orc_parser* p) {
	if (p->state == ORC_ST_INVALID)
		return ORC_STATUS_INVALID;
	if (p->state == ORC_ST_FINISHED)
		return ORC_STATUS_FINISHED;
	return ORC_STATUS_UNFINISHED;
}

/* D:161-192 handleNewRequest -> Aggregator::newRequest (the LOG_DEBUG has no effect on results) */
static int handle_new_request(orc_ctx* c, const orc_parser* p, const orc_event* ev) {
	return agg_new_request(c, &p->result, ev->pid, ev->flags, ev->sourceIP);
}

/* D:123-139 */
static void handle_existing_session(orc_ctx* c, lru_node* n, const uint8_t* buf, size_t len, const orc_event* ev,
		orc_event_result* o) {
	orc_parser* p = (orc_parser*)n->value;
	o->kind = ORC_KIND_EXISTING;
	o->consumed = (uint32_t)parser_parse(p, buf, len, ev->flags); /* update(): does not move (L:83-85) */
	o->status = status_of(p);
	if (parser_is_invalid(p)) {
		c->st.kernel_deletes++; /* bpfDiscoveryDeleteSession(event.key) D:126 */
		lru_remove(&c->sessions, n);
		return;
	}
	if (!parser_is_finished(p))
		return;
	int cls = handle_new_request(c, p, ev);
	fill_finished(c, o, &p->result, cls);
	parser_reset(p); /* D:138 session.reset(); the session stays saved */
}

/* D:141-159 */
static void handle_new_session(orc_ctx* c, const uint8_t* buf, size_t len, const orc_event* ev, orc_event_result* o) {
	orc_parser* p = (orc_parser*)calloc(1, sizeof(orc_parser));
	parser_init(p);
	o->kind = ORC_KIND_NEW;
	o->consumed = (uint32_t)parser_parse(p, buf, len, ev->flags);
	o->status = status_of(p);
	if (parser_is_invalid(p)) {
		free_parser_value(p);
		return;
	}
	if (!parser_is_finished(p) && !(ev->flags & ORC_FLAG_DATA_END)) {
		uint32_t k[3] = {ev->pid, ev->fd, ev->sessionID};
		lru_node* n = lru_insert(&c->sessions, k); /* saveSession D:214-216 */
		if (n->value && n->value != p)
			free_parser_value(n->value);
		n->value = p;
		return;
	}
	if (!parser_is_finished(p)) {
		free_parser_value(p);
		return;
	}
	int cls = handle_new_request(c, p, ev);
	fill_finished(c, o, &p->result, cls);
	free_parser_value(p);
}

int orc_process(orc_ctx* c, const orc_event* ev, const uint32_t* len, const uint64_t* off, const uint8_t* payload, uint32_t n,
		orc_event_result* out) {
	for (uint32_t i = 0; i < n; i++, c->cur_event++) {
		const orc_event* e = &ev[i];
		orc_event_result* o = &out[i];
		memset(o, 0, sizeof(*o));
		/* D:92-99 handleNewEvent */
		if (e->flags & ORC_FLAG_NEW_DATA) {
			/* D:101-110 handleNewDataEvent: the saved buffer may be missing */
			if (len[i] == UINT32_MAX) {
				c->st.missing_buffers++;
			} else {
				/* D:102-103: bpf_map_lookup_and_delete_elem copies the whole DiscoverySavedBuffer
				 * (4-B length + 8192-B data, Types.h:58-61) into a stack object, whatever the
				 * length: the same copy here keeps the baseline's cost faithful */
				memcpy(c->saved.data, payload + off[i], len[i] <= sizeof(c->saved.data) ? len[i] : sizeof(c->saved.data));
				memset(c->saved.data + (len[i] < sizeof(c->saved.data) ? len[i] : sizeof(c->saved.data)), 0,
						sizeof(c->saved.data) - (len[i] < sizeof(c->saved.data) ? len[i] : sizeof(c->saved.data)));
				c->saved.length = len[i];
				const uint8_t* buf = c->saved.data;
				/* D:112-121 handleBufferLookupSuccess: find() touches the LRU entry */
				uint32_t k[3] = {e->pid, e->fd, e->sessionID};
				lru_node* nd = lru_find(&c->sessions, k);
				if (nd)
					handle_existing_session(c, nd, buf, len[i], e, o);
				else
					handle_new_session(c, buf, len[i], e, o);
			}
		}
		if (e->flags & ORC_FLAG_DATA_END) { /* D:194-198 handleCloseEvent */
			uint32_t k[3] = {e->pid, e->fd, e->sessionID};
			lru_node* nd = lru_find(&c->sessions, k);
			if (nd)
				lru_remove(&c->sessions, nd);
		}
	}
	c->st.lru_evictions = c->sessions.evictions;
	c->st.lru_size = c->sessions.size;
	return 0;
}

void orc_blob(orc_ctx* c, const char** data, uint64_t* size) {
	*data = c->blob.p;
	*size = c->blob.n;
}
void orc_blob_reset(orc_ctx* c) { c->blob.n = 0; }
void orc_get_stats(orc_ctx* c, orc_stats* s) {
	c->st.lru_evictions = c->sessions.evictions;
	c->st.lru_size = c->sessions.size;
	*s = c->st;
}

/* ------------------------------------------------------------------------------- */
/* parser API for the unit-test vectors                                              */
/* ------------------------------------------------------------------------------- */
orc_parser* orc_parser_new(void) {
	orc_parser* p = (orc_parser*)calloc(1, sizeof(orc_parser));
	parser_init(p);
	return p;
}
void orc_parser_free(orc_parser* p) { free_parser_value(p); }
size_t orc_parser_parse(orc_parser* p, const uint8_t* data, size_t len, uint8_t flags) { return parser_parse(p, data, len, flags); }
int orc_parser_state(const orc_parser* p) { return p->state; }
void orc_parser_reset(orc_parser* p) { parser_reset(p); }

static void out_ds(dstr* o, const dstr* s) {
	for (size_t i = 0; i < s->n; i++)
		ds_push(o, s->p[i]);
}
uint64_t orc_parser_result(const orc_parser* p, char* buf, uint64_t cap) {
	dstr o = {0};
	out_ds(&o, &p->result.method);
	ds_push(&o, '\n');
	out_ds(&o, &p->result.url);
	ds_push(&o, '\n');
	out_ds(&o, &p->result.protocol);
	ds_push(&o, '\n');
	out_ds(&o, &p->result.host);
	ds_push(&o, '\n');
	out_ds(&o, &p->result.clientIPKey);
	ds_push(&o, '\n');
	ds_push(&o, p->result.isHttps ? '1' : '0');
	ds_push(&o, '\n');
	for (size_t i = 0; i < p->result.clientIp.n; i++) {
		if (i)
			ds_push(&o, '\x1f');
		out_ds(&o, &p->result.clientIp.v[i]);
	}
	ds_push(&o, '\n');
	uint64_t need = o.n;
	if (buf && cap >= need)
		memcpy(buf, o.p, need);
	ds_free(&o);
	return need;
}

uint64_t orc_parse_client_ip(const char* data, size_t len, char* buf, uint64_t cap, uint32_t* count) {
	orc_request r;
	req_init(&r);
	parse_client_ip_value(&r, data, len);
	dstr o = {0};
	for (size_t i = 0; i < r.clientIp.n; i++) {
		if (i)
			ds_push(&o, '\x1f');
		out_ds(&o, &r.clientIp.v[i]);
	}
	if (count)
		*count = (uint32_t)r.clientIp.n;
	uint64_t need = o.n;
	if (buf && cap >= need && need)
		memcpy(buf, o.p, need);
	ds_free(&o);
	req_free(&r);
	return need;
}

/* Calibration helper: HttpRequestParser::parse only, a fresh parser per buffer
 * (P:85-106), as the survey timed the compiled reference.  Returns the bytes consumed. */
uint64_t orc_parse_only(const uint8_t* payload, const uint64_t* off, const uint32_t* len, uint32_t n) {
	uint64_t total = 0;
	orc_parser p;
	parser_init(&p);
	for (uint32_t i = 0; i < n; i++) {
		if (len[i] == UINT32_MAX)
			continue;
		parser_reset(&p);
		total += parser_parse(&p, payload + off[i], len[i], ORC_FLAG_UNENCRYPTED);
	}
	parser_destroy(&p);
	return total;
}
