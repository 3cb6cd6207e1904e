/*
 * ebpf_discovery_amd_testing.h — host-side hooks of libebd_amd.so.
 *
 * They run the product's own parse semantics (ebd_spec.h / ebd_fresh.h, the same
 * __host__ __device__ code the GPU kernels execute) on the CPU, so the CPU test suite can
 * compare the product logic with the oracle without a GPU.  They are not a fallback:
 * the batch API (ebpf_discovery_amd.h) only ever runs on the GPU.
 */
#ifndef EBPF_DISCOVERY_AMD_TESTING_H
#define EBPF_DISCOVERY_AMD_TESTING_H

#include "ebpf_discovery_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* DFA layout: nstates, url_id, g2, g3, g4, hvc0, hvh, fin0, fin1, inv, init. */
int ebd_host_dfa_info(uint32_t* info, uint32_t n);
/* The DFA's transition table next[s * 256 + byte] (cap >= 65536); returns nstates. */
int ebd_host_dfa_next(uint8_t* out, uint32_t cap);

/* The DFA fast path (k_fresh's per-event logic) for one buffer; key = its service key under
 * hash_key (ebd_config.hash_key). */
int ebd_host_fresh(const uint8_t* buf, uint32_t len, uint32_t pid, uint8_t flags, const uint8_t* src16,
		const ebd_ipv4_network* v4, uint32_t n4, const ebd_ipv6_network* v6, uint32_t n6, const uint64_t hash_key[2],
		ebd_event_result* out, uint64_t key[2]);

/* The structural fast path (k_fresh_scan's per-event logic, ebd_scan.h) for one buffer placed at
 * byte `shift` (0..15) of its LDS tile; the rest of the tile is "\r\n" filler.  Returns the
 * path that decided it: 0 scan_fast, 2 scan_event, 1 the generic parser (a key with a space). */
int ebd_host_scan(const uint8_t* buf, uint32_t len, uint32_t shift, uint32_t pid, uint8_t flags, const uint8_t* src16,
		const ebd_ipv4_network* v4, uint32_t n4, const ebd_ipv6_network* v6, uint32_t n6, const uint64_t hash_key[2],
		ebd_event_result* out, uint64_t key[2]);

/* The generic parser (k_walk's parser) over consecutive chunks of one stream
 * (HttpRequestParser::parse per chunk).  out8[12] = state, url_start, url_len,
 * host_start, host_len, cip_start, cip_len, flags, cipkey, mcand, mlen, plen | pminor << 8. */
int ebd_host_gp_parse(const uint8_t* data, const uint32_t* chunk_len, uint32_t nchunks, uint8_t flags, int reset_between,
		uint32_t* consumed, uint32_t* out8);

/* The session path's DFA walker (dfa_parse, ebd_fresh.h) over the same chunks: out8 as
 * ebd_host_gp_parse's, with mlen and plen 0 (the walker does not keep them). */
int ebd_host_dfa_parse(const uint8_t* data, const uint32_t* chunk_len, uint32_t nchunks, uint8_t flags, int reset_between,
		uint32_t* consumed, uint32_t* out8);

/* Client classification: a client-IP value token (front_token + classify_token) or,
 * with is_source, the 16 source-address bytes under `flags`.  Returns 0/1/2. */
int ebd_host_classify(const uint8_t* token, uint32_t len, int is_source, uint8_t flags, const ebd_ipv4_network* v4,
		uint32_t n4, const ebd_ipv6_network* v6, uint32_t n6);

/* Service key of (pid, endpoint) under hash_key in its streaming form (the session path's):
 * key[0] = lo, key[1] = hi.  The fast path computes the same key word by word from spans. */
int ebd_host_endpoint_key(const uint64_t hash_key[2], uint32_t pid, const uint8_t* endpoint, uint32_t len, uint64_t key[2]);

/* The exact LRU's derivation window in events (0: EBD_LRU_WINDOW or the default 8192), so a
 * test can make one batch span several windows and resumed walks. */
int ebd_testing_set_lru_window(ebd_ctx* ctx, uint32_t window);

/* inet_pton restatement used on the device: 1 = parsed. */
int ebd_host_pton(int af6, const uint8_t* text, uint32_t len, uint8_t* out);

#ifdef __cplusplus
}
#endif

#endif
