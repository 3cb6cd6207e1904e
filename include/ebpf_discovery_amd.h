/*
 * ebpf_discovery_amd.h — C ABI of the MI355X-native HTTP per-event parse path.
 *
 * Drop-in boundary for dynatrace-oss/eBPF-Discovery's event-consumer hot path:
 *   libebpfdiscovery/src/Discovery.cpp:73-198   (drain, per-event dispatch, session LRU)
 *   libhttpparser/src/HttpRequestParser.cpp:85-409 (per-byte request-line / header scanner)
 *   libservice/src/Aggregator.cpp:44-181         (per-(pid, endpoint) client counters)
 *   libservice/src/IpAddressCheckerImpl.cpp:39-180 (internal / external classification)
 * The reference calls HttpRequestParser::parse once per captured buffer and
 * Aggregator::newRequest once per finished request; this ABI takes a whole batch of
 * captured buffers (the packed form of the BPF queue + savedBuffersMap) and runs the
 * same semantics as hand-written HIP kernels on one GPU.  Plain C types only.
 *
 * Errors: 0 on success, a negative errno otherwise (the reference's int convention,
 * Discovery.cpp:48-58).  An HTTP parse failure is data (EBD_STATUS_INVALID), not an
 * error.  Nothing throws across this boundary.
 *
 * Threading: one submitting thread per context (the reference has one poll thread,
 * ServiceDetectionTask.cpp:43-49); ebd_collect_services / ebd_clear may be called from
 * another thread (the reporting thread) and are serialised by the context, like
 * Aggregator.h:66.  Every call on a context is ordered on the context's private HIP
 * stream.
 */
#ifndef EBPF_DISCOVERY_AMD_H
#define EBPF_DISCOVERY_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EBD_ABI_VERSION 1

/* --- wire format (libebpfdiscoveryshared/headers/ebpfdiscoveryshared/Types.h) ----- */

/* DiscoveryEvent, Types.h:201-205 — 36 bytes, byte-identical to the BPF record. */
typedef struct ebd_discovery_event {
	uint32_t pid;       /* DiscoverySavedBufferKey.pid        @0  */
	uint32_t fd;        /* .fd                                @4  */
	uint32_t sessionID; /* .sessionID                         @8  */
	uint32_t bufferSeq; /* .bufferSeq                         @12 */
	uint8_t sourceIP[16]; /* DiscoverySockSourceIP            @16 */
	uint8_t flags;      /* DiscoveryFlags                     @32 */
	uint8_t pad_[3];
} ebd_discovery_event;

/* DiscoveryFlags, Types.h:122-129 */
#define EBD_FLAG_SESSION_IPV4 2
#define EBD_FLAG_SESSION_IPV6 4
#define EBD_FLAG_SESSION_UNENCRYPTED_HTTP 8
#define EBD_FLAG_SESSION_SSL_HTTP 16
#define EBD_FLAG_EVENT_NEW_DATA 32
#define EBD_FLAG_EVENT_DATA_END 64

/* Constants.h:19-24 */
#define EBD_BUFFER_MAX_DATA_SIZE 8192
#define EBD_MAX_SESSIONS 8192
#define EBD_MAX_HTTP_REQUEST_LENGTH 8192

/* len[i] == EBD_NO_BUFFER: the NEW_DATA event's saved buffer is missing
 * (bpf_map_lookup_and_delete_elem failed, Discovery.cpp:103-107). */
#define EBD_NO_BUFFER 0xffffffffu

/* InterfacesReader.h:15-24, addresses and masks in network byte order (in_addr bytes). */
typedef struct ebd_ipv4_network {
	uint8_t addr[4];
	uint8_t mask[4];
} ebd_ipv4_network;
typedef struct ebd_ipv6_network {
	uint8_t addr[16];
	uint8_t mask[16];
} ebd_ipv6_network;

/* --- per-event result (replaces the per-call HttpRequestParser::parse outcome) ------ */

enum {
	EBD_STATUS_NONE = 0,       /* no parse: DATA_END-only event or missing buffer */
	EBD_STATUS_UNFINISHED = 1, /* parser waits for more buffers (Discovery.cpp:131-134) */
	EBD_STATUS_FINISHED = 2,   /* a request was handed to the aggregator */
	EBD_STATUS_INVALID = 3,    /* HttpRequestParser::isInvalidState() */
};
#define EBD_INFO_POST 0x01     /* method POST (else GET) */
#define EBD_INFO_HTTPS 0x02    /* HttpRequest::isHttps (flags & SSL of the finishing event) */
#define EBD_INFO_SESSION 0x04  /* produced by the session path: see ebd_event_result.session */
#define EBD_INFO_CIP 0x08      /* request.clientIp non-empty (cip_* spans the front token) */
#define EBD_INFO_CLASS_SHIFT 4 /* bits 4-5: 0 not counted, 1 internal, 2 external */
#define EBD_INFO_EXISTING 0x40 /* parsed by a saved session (Discovery.cpp:123-139) */
#define EBD_INFO_DROPPED 0x80  /* FINISHED, but not aggregated or counted: a capacity error
                                  (EBD_ERR_ARENA_FULL) left no room for its strings */

/* 16 bytes.  consumed = HttpRequestParser::parse() return value for this buffer.
 * Fast-path (single-buffer) requests: spans are byte offsets inside this event's
 * buffer.  EBD_INFO_SESSION requests (spanning several buffers): `session` indexes the
 * array returned by ebd_fetch_session_requests. */
typedef struct ebd_event_result {
	uint16_t consumed;
	uint8_t status;
	uint8_t info;
	union {
		struct {
			uint16_t url_off, url_len;
			uint16_t host_off, host_len;
			uint16_t cip_off, cip_len;
		} span;
		struct {
			uint32_t index;
			uint32_t pad_[2];
		} session;
	} u;
} ebd_event_result;

/* A request finished by the session path: strings live in the batch's session string
 * buffer (ebd_fetch_session_requests): host at str_off, url right after it, then the
 * client-IP front token. */
typedef struct ebd_session_request {
	uint64_t seq; /* global event order of the finishing event */
	uint32_t pid;
	uint32_t str_off;  /* host bytes, then url bytes */
	uint16_t host_len, url_len;
	uint16_t cip_off;  /* client-IP front token, relative to str_off */
	uint16_t cip_len;
	uint8_t info;      /* EBD_INFO_* */
	uint8_t status;
	uint16_t pad_;
	uint32_t pad2_;
} ebd_session_request; /* 32 bytes */

/* --- services (Service.h:43-66) ------------------------------------------------------ */
typedef struct ebd_service {
	uint32_t pid;
	uint32_t internal_clients; /* uint32, wraps like Service.h:53-54 */
	uint32_t external_clients;
	uint8_t https; /* scheme "https" (1) / "http" (0) of the first request that created the key;
	                  EBD_SCHEME_NONE: no scheme (only ebd_format_services_json reads it) */
	uint8_t pad_[3];
	uint64_t endpoint_off; /* into the caller's string buffer */
	uint32_t endpoint_len;
	uint32_t domain_off; /* relative to endpoint_off */
	uint32_t domain_len;
	uint32_t host_len;   /* the first request's host length (its host/url split of the endpoint) */
	uint64_t first_seq; /* global order of the request that created it (first arrival) */
	uint64_t key_lo, key_hi; /* 128-bit hash of (pid, endpoint): identical on every GPU, so
	                            shards merge and pick owners by it without comparing strings */
	/* Network counters (EBD_CFG_NETWORK_COUNTERS; Service.h:56-58, Aggregator.cpp:89-106): the
	 * sizes of externalIPv4_16ClientNets, externalIPv4_24ClientNets and externalIPv6ClientsNets
	 * (48-bit prefixes), the numbers the JSON report prints (Service.h:84-98).  0 when off. */
	uint32_t nets_v4_16;
	uint32_t nets_v4_24;
	uint32_t nets_v6;
	uint32_t pad2_;
} ebd_service; /* 80 bytes */
#define EBD_SCHEME_NONE 2

/* One entry of a service's network set (ebd_collect_networks): the service's key, the set
 * (EBD_NET_*), the prefix bytes in address order (v4: 2 or 3 bytes of in_addr, v6: 6 bytes
 * of in6_addr; the rest 0) and the steady-clock time it was last seen (ns). */
#define EBD_NET_V4_16 1
#define EBD_NET_V4_24 2
#define EBD_NET_V6_48 3
typedef struct ebd_service_net {
	uint64_t key_lo, key_hi;
	uint8_t kind;
	uint8_t prefix[6];
	uint8_t pad_;
	uint64_t time_ns;
} ebd_service_net; /* 32 bytes */

typedef struct ebd_stats {
	uint64_t events;            /* events submitted */
	uint64_t requests;          /* Aggregator::newRequest equivalents */
	uint64_t session_events;    /* events handled by the session (multi-buffer) path */
	uint64_t kernel_deletes;    /* bpfDiscoveryDeleteSession equivalents, Discovery.cpp:125-129 */
	uint64_t live_sessions;     /* saved (LRU) sessions after the last batch */
	uint64_t max_live_sessions; /* peak saved sessions seen inside any batch */
	uint64_t services;          /* distinct (pid, endpoint) keys */
	uint64_t hash_collisions;   /* 64-bit slot tag matched but the 128-bit key did not */
	uint64_t errors;            /* bitmask of EBD_ERR_* conditions seen */
	uint64_t lru_evictions;     /* sessions evicted from the full LRU (LRUCache.h:56-58) */
	uint64_t lru_exact_batches; /* batches whose session events ran through the exact LRU path */
	uint64_t lru_rounds;        /* walk-and-derive rounds the exact LRU path took (all batches) */
	uint64_t lru_sequential;    /* exact batches that fell back to the one-lane replay (k_walk_lru) */
} ebd_stats;

#define EBD_ERR_TABLE_FULL 1u      /* service table probe limit reached */
#define EBD_ERR_ARENA_FULL 2u      /* string arena exhausted */
#define EBD_ERR_LRU_OVERFLOW 4u    /* more saved sessions than the carry store holds (internal) */
#define EBD_ERR_SESSION_FULL 8u    /* session scratch exhausted */
#define EBD_ERR_VERIFY_FULL 16u    /* deferred key-verification list exhausted */
#define EBD_ERR_BAD_INPUT 32u      /* len > EBD_BUFFER_MAX_DATA_SIZE, bad offsets */
#define EBD_ERR_COLLISION 64u      /* two keys share a 64-bit tag (results not trusted) */
#define EBD_ERR_INTERNAL 128u      /* a kernel-internal consistency check failed (results not trusted) */
#define EBD_ERR_NET_FULL 256u      /* network-counter sets exhausted (ebd_config.net_capacity) */

typedef struct ebd_config {
	int device;                /* HIP device ordinal */
	uint32_t max_events;       /* largest batch; device work buffers are sized for it */
	uint64_t max_payload;      /* largest payload arena (bytes) of a host batch */
	uint32_t service_capacity; /* service hash slots (power of two, 0 = default 1<<22) */
	uint64_t string_arena;     /* bytes for service endpoint strings (0 = default 256 MiB) */
	uint32_t lru_capacity;     /* 0 = EBD_MAX_SESSIONS (Discovery.cpp:39); below 2^24 (-EINVAL) */
	uint32_t flags;            /* EBD_CFG_* */
	/* Secret key of the 128-bit service-key PRF (SipHash-1-3-128 over pid + endpoint bytes).
	 * {0, 0} = draw one from getrandom().  Contexts whose tables are merged (shards of one
	 * trace on several GPUs) must share it: read it back with ebd_get_hash_key. */
	uint64_t hash_key[2];
	uint32_t net_capacity; /* network-counter set entries (power of two, 0 = default 1<<22) */
	uint32_t pad_;
} ebd_config;

#define EBD_CFG_TIMING 2u /* time every kernel launch with HIP events (ebd_kernel_times) */
/* Aggregator(ipChecker, enableNetworkCounters = true) (Aggregator.cpp:132-134; the
 * --enable-network-counters option, main.cpp:78): every external client's /16 and /24 (IPv4)
 * or 48-bit (IPv6) network is kept per service with the time it was last seen. */
#define EBD_CFG_NETWORK_COUNTERS 4u
/* Fresh parses (Discovery.cpp:141-159) through the structural scan (k_fresh_scan: one wave
 * per LDS tile of buffers; lanes over pieces, header lines and buffers) instead of the
 * projected-DFA kernel (k_fresh, one lane per buffer).  Same results; kept for A/B
 * measurement.  The environment variable EBD_FRESH=scan sets it for
 * every context (EBD_FRESH=dfa clears it). */
#define EBD_CFG_FRESH_SCAN 8u

typedef struct ebd_ctx ebd_ctx;

/* Device-resident batch: every pointer is a device (HBM) pointer that stays valid
 * until the next ebd_sync.  Buffer i is [off[i], off[i] + len[i]) of payload and must lie
 * inside [0, payload_bytes); a buffer that does not is not read: the event counts as one
 * with no saved buffer and EBD_ERR_BAD_INPUT is set (the host entry points reject such a
 * batch with -EINVAL instead, ebd_submit_batch).  payload reads are done in aligned 16-byte
 * blocks and 8-byte pieces, so the allocation must be readable from the 16-byte boundary at
 * or below payload to EBD_PAYLOAD_PAD bytes past payload + payload_bytes. */
#define EBD_PAYLOAD_PAD 16u
typedef struct ebd_device_batch {
	const ebd_discovery_event* events;
	const uint32_t* len;
	const uint64_t* off;
	const uint8_t* payload;
	uint64_t payload_bytes;
	uint32_t n;
} ebd_device_batch;

int ebd_ctx_create(const ebd_config* cfg, ebd_ctx** out);
int ebd_ctx_destroy(ebd_ctx* ctx);
/* The context's HIP stream (hipStream_t), for callers that time or order work. */
void* ebd_ctx_stream(ebd_ctx* ctx);
/* The context's service-key PRF key (ebd_config.hash_key as used). */
int ebd_get_hash_key(ebd_ctx* ctx, uint64_t out[2]);

/* IpAddressCheckerImpl's interface list (InterfacesReader::collectAllIpInterfaces,
 * InterfacesReader.cpp:50-78) — injected, because it is host dependent. */
int ebd_set_interfaces(ebd_ctx* ctx, const ebd_ipv4_network* v4, uint32_t n4, const ebd_ipv6_network* v6, uint32_t n6);

/* One poll cycle (Discovery::fetchAndHandleEvents, Discovery.cpp:73-121): events[i] with its
 * saved buffer at payload + off[i], len[i] bytes (len <= 8192, or EBD_NO_BUFFER).  Host
 * memory, uploaded as ebd_stage_batch does.  Blocks until the batch is processed. */
int ebd_submit_batch(ebd_ctx* ctx, const ebd_discovery_event* events, const uint32_t* len, const uint64_t* off,
		const uint8_t* payload, uint64_t payload_bytes, uint32_t n);
/* The same with the batch already in HBM.  The host waits only for the fresh pass's counters
 * (is there session work?); the rest stays queued on the context stream (ebd_sync).
 * DEVICE inputs, here and in every *_device call, are read on the context stream
 * (ebd_ctx_stream), a non-blocking stream: work that produces them on another stream must be
 * ordered before the call (e.g. hipStreamWaitEvent on the context stream). */
int ebd_submit_batch_device(ebd_ctx* ctx, const ebd_device_batch* batch);
/* Waits for every queued upload, batch and read-back of the context. */
int ebd_sync(ebd_ctx* ctx);

/* --- ingest pipeline (Discovery.cpp:73-110: drain, saved-buffer fetch) ------------------
 * ebd_stage_batch uploads a host batch into one of two device staging slots on the context's
 * copy stream and returns without waiting for the DMA; ebd_submit_staged runs it (the compute
 * stream, not the host, waits for the upload).  Staging batch k+1 before submitting batch k
 * overlaps its H2D with batch k's kernels.  Pinned sources (ebd_host_alloc) are DMAed as they
 * are and must stay unchanged until the batch is submitted and synced; pageable sources are
 * copied through pinned bounce buffers (CPU copy overlapping the DMA) and may be reused as
 * soon as the call returns.  At most two batches are staged and not yet submitted (-EBUSY). */
int ebd_stage_batch(ebd_ctx* ctx, const ebd_discovery_event* events, const uint32_t* len, const uint64_t* off,
		const uint8_t* payload, uint64_t payload_bytes, uint32_t n, uint64_t* ticket);
int ebd_submit_staged(ebd_ctx* ctx, uint64_t ticket);
/* Pinned host memory for producers that fill batches in place (no staging copy). */
void* ebd_host_alloc(ebd_ctx* ctx, uint64_t bytes);
int ebd_host_free(ebd_ctx* ctx, void* p);
/* Global order of the next submitted event (default: events submitted so far).  Shards of
 * one trace set it to their first global event index so first-arrival ties resolve in
 * trace order after the cross-GPU merge. */
int ebd_set_seq_base(ebd_ctx* ctx, uint64_t seq);

/* Per-kernel device time over all launches since the last reset (EBD_CFG_TIMING):
 * HIP events recorded on the context stream around each launch. */
typedef struct ebd_kernel_time {
	char name[24];
	uint64_t launches;
	double total_ms;
} ebd_kernel_time;
int ebd_kernel_times(ebd_ctx* ctx, ebd_kernel_time* out, uint32_t cap, uint32_t* n);
int ebd_reset_kernel_times(ebd_ctx* ctx);

/* Per-event results of the last batch (host copy), n <= cap; out == NULL: *n only. */
int ebd_fetch_results(ebd_ctx* ctx, ebd_event_result* out, uint32_t cap, uint32_t* n);
/* The same read back on the context's D2H stream once the batch is done, without blocking
 * (out should be pinned); complete after ebd_sync.  The next batch's kernels wait for it. */
int ebd_fetch_results_async(ebd_ctx* ctx, ebd_event_result* out, uint32_t cap, uint32_t* n);
/* Device pointer to the last batch's per-event results (valid until the next submit). */
const ebd_event_result* ebd_results_device(ebd_ctx* ctx);
/* Session-path requests of the last batch and their strings. */
int ebd_fetch_session_requests(ebd_ctx* ctx, ebd_session_request* out, uint32_t cap, uint32_t* n, char* strings,
		uint64_t strcap, uint64_t* strlen);

/* Aggregator::collectServices (Aggregator.cpp:170-181): services and their strings.
 * Call with out == NULL to get the sizes.  Order is unspecified (unordered_map). */
int ebd_collect_services(ebd_ctx* ctx, ebd_service* out, uint32_t cap, uint32_t* n, char* strings, uint64_t strcap,
		uint64_t* strlen);
/* Aggregator::clear (Aggregator.cpp:136-153).  Network counters off: every service goes.
 * On: a service whose three network sets are all empty goes; the others stay with their
 * client counters zeroed (their domain, scheme and sets are kept). */
int ebd_clear(ebd_ctx* ctx);
/* Every service and every network-map entry goes: the table as ebd_ctx_create left it.
 * The cross-GPU merge starts from it (ebd_clear keeps the services that have network maps,
 * which would then be reported by their owner GPU and by this one). */
int ebd_reset_services(ebd_ctx* ctx);

/* --- network counters (EBD_CFG_NETWORK_COUNTERS) -------------------------------------- */
/* Aggregator::getCurrentTime for the requests of the batches submitted from now on
 * (steady-clock nanoseconds, like std::chrono::steady_clock on Linux).  0 (the default):
 * CLOCK_MONOTONIC is read when each batch is submitted.  The reference reads the clock per
 * request; one reading per poll cycle differs by at most the cycle's length. */
int ebd_set_clock(ebd_ctx* ctx, uint64_t now_ns);
/* Aggregator::getCurrentTime per request, as the reference reads it (Aggregator.cpp:162,165):
 * time_ns is a DEVICE array of the next submitted batch's n events, and the request an event
 * finishes takes that event's reading (the consumer's clock when it handled the event).  It
 * applies to that one batch (NULL: the batch clock of ebd_set_clock).  The array must stay
 * valid until the batch's work is done (ebd_sync). */
int ebd_set_event_clock(ebd_ctx* ctx, const uint64_t* time_ns);
/* Aggregator::networkCountersCleaning (Aggregator.cpp:182-209): every set entry last seen
 * at least one hour before now_ns is erased (0 = the context clock). */
int ebd_network_counters_cleaning(ebd_ctx* ctx, uint64_t now_ns);
/* The network-set entries of every service (out == NULL: count only).  Order unspecified. */
int ebd_collect_networks(ebd_ctx* ctx, ebd_service_net* out, uint32_t cap, uint32_t* n);
/* The same records into a DEVICE array (out == NULL: *n only; -ENOSPC past cap): what a GPU
 * sends to the owners of its services for the cross-GPU merge (owner = (key_lo >> 32) % world). */
int ebd_collect_networks_device(ebd_ctx* ctx, ebd_service_net* out, uint32_t cap, uint32_t* n);
/* Merges n network-map entries (a DEVICE array, ebd_service_net records of other GPUs) into
 * the maps of this context's services, found by key: merge the services first
 * (ebd_merge_services_device); an entry whose service is missing is reported as
 * EBD_ERR_INTERNAL.  An entry new to its map adds one to the map's size; the last-seen time
 * is the later one (Aggregator.cpp:89-106, 182-209 across GPUs).  -EINVAL without network
 * counters. */
int ebd_merge_networks_device(ebd_ctx* ctx, const ebd_service_net* recs, uint32_t n);

/* --- the service report (Discovery::outputServicesToStdout, Discovery.cpp:60-71) ------- */
/* The report text byte for byte: {"service":[...]} through boost::json::ext::print
 * (Json.h:32-71; null and empty-string fields dropped, network sets printed as their
 * sizes, Service.h:69-98) and the std::endl newline; empty (length 0) when there are no
 * services.  Services appear in `s` order (the reference prints its unordered_map order).
 * *len = the text length; out == NULL or cap < *len: nothing is written (-ENOSPC when out
 * is given).  Host-only: needs no GPU. */
int ebd_format_services_json(const ebd_service* s, uint32_t n, const char* strings, uint64_t strings_len, char* out,
		uint64_t cap, uint64_t* len);
/* The context's services (ebd_collect_services) as that report.  Like the reference, the
 * caller clears the aggregator after printing (ebd_clear). */
int ebd_report_json(ebd_ctx* ctx, char* out, uint64_t cap, uint64_t* len);

/* --- cross-GPU merge of per-GPU service tables ------------------------ */
/* A service on the wire (40 B): what the owner's merge needs.  The endpoint bytes are not
 * addressed: record k's bytes follow record k-1's in the strings, each padded to 8 bytes, so
 * concatenated segments (all-to-all output) stay addressable without rebasing. */
typedef struct ebd_wire_service {
	uint64_t key_lo, key_hi;
	uint64_t first;            /* first-arrival word: first_seq << 16 | https << 15 | host_len */
	uint32_t pid;
	uint32_t internal_clients; /* uint32, add modulo 2^32 (Service.h:53-54) */
	uint32_t external_clients;
	uint32_t endpoint_len;     /* EBD_WIRE_NO_BYTES set: no bytes follow (the source arena was full) */
} ebd_wire_service;
#define EBD_WIRE_NO_BYTES 0x80000000u
/* Bytes a wire record's endpoint takes in the strings. */
#define EBD_WIRE_BYTES(len) (((len) & EBD_WIRE_NO_BYTES) ? 0u : (((len) + 7u) & ~7u))

/* The context's services grouped by owner GPU, owner = (key_lo >> 32) % world (key_lo is always
 * odd: its low bit marks a used slot), into DEVICE arrays:
 * recs[] ordered by owner (counts[w] records for owner w), strings[] their endpoint bytes in
 * record order (str_counts[w] bytes for owner w).  counts / str_counts are host arrays of
 * `world` entries.  recs == NULL: sizes only. */
int ebd_export_services_device(ebd_ctx* ctx, uint32_t world, ebd_wire_service* recs, uint32_t cap, uint8_t* strings,
		uint64_t strcap, uint32_t* counts, uint64_t* str_counts);
/* The interval merge with its sizes left on the device (one host read per
 * interval in ebd/shard.py device_exchange_merge):
 *  - ebd_export_capacity: the record and string-byte capacity that always holds the whole table
 *    (every slot, the whole string arena + 8);
 *  - ebd_export_services_device_sized: ebd_export_services_device into buffers of at least those
 *    capacities, with sizes (DEVICE, 128 words) = [64 per-owner record counts][64 per-owner string
 *    bytes] instead of host counts: nothing is read back, so the counts can go straight into the
 *    size all-to-all;
 *  - ebd_wire_segment_bytes_device: out[s] (DEVICE, world words) = the 8-padded endpoint bytes of
 *    the records of segment s (seg_counts: DEVICE, world consecutive segments) whose need byte is
 *    set, or (need NULL) whose dst is not ~0: the bytes round's counts per owner on the source side
 *    and per source on the owner side;
 *  - ebd_wire_compact_device with out_len NULL packs without the size read (outcap >= strlen). */
int ebd_export_capacity(ebd_ctx* ctx, uint32_t* records, uint64_t* string_bytes);
int ebd_export_services_device_sized(ebd_ctx* ctx, uint32_t world, ebd_wire_service* recs, uint32_t cap, uint8_t* strings,
		uint64_t strcap, uint64_t* sizes);
int ebd_wire_segment_bytes_device(ebd_ctx* ctx, const ebd_wire_service* recs, uint32_t n, const uint8_t* need, const uint64_t* dst,
		const uint64_t* seg_counts, uint32_t world, uint64_t* out);
/* Merges n wire records (DEVICE arrays; strings hold their bytes in record order, readable
 * 8 bytes past strlen) into the context's table: counters add (uint32), the record with the
 * smallest first word fixes scheme and host/url split (Aggregator.cpp:155-168 across GPUs),
 * the endpoint bytes are copied in.  Records whose bytes would run past strlen are skipped
 * and reported as EBD_ERR_INTERNAL. */
int ebd_merge_services_device(ebd_ctx* ctx, const ebd_wire_service* recs, uint32_t n, const uint8_t* strings,
		uint64_t strlen);
/* The same merge in two rounds, so that endpoint bytes cross the fabric once per key the owner
 * lacks ("ship endpoint strings once per new key"), not once per sender:
 *  1. keys: the owner merges the records alone (counters, first word) into its table.  A record
 *     that creates a service reserves the service's arena bytes: dst[k] (DEVICE, n entries) =
 *     the reserved offset, or ~0 when record k's bytes are not needed (the key was there, or
 *     the source had none).  Merge the owner's own records first and theirs are the creators.
 *  2. the owner returns need[k] = (dst[k] != ~0) to each record's source;
 *     ebd_wire_compact_device packs the bytes of the needed records (need: DEVICE, one byte per
 *     exported record) in record order; out == NULL: *out_len only; out_len == NULL: no size
 *     read (outcap >= strlen);
 *  3. ebd_merge_service_bytes_device copies the received bytes (in the order of the records
 *     with dst != ~0, readable 8 bytes past strlen) to the reserved places. */
int ebd_merge_service_keys_device(ebd_ctx* ctx, const ebd_wire_service* recs, uint32_t n, uint64_t* dst);
int ebd_wire_compact_device(ebd_ctx* ctx, const ebd_wire_service* recs, uint32_t n, const uint8_t* strings, uint64_t strlen,
		const uint8_t* need, uint8_t* out, uint64_t outcap, uint64_t* out_len);
int ebd_merge_service_bytes_device(ebd_ctx* ctx, const ebd_wire_service* recs, uint32_t n, const uint64_t* dst,
		const uint8_t* strings, uint64_t strlen);
/* --- requests parsed elsewhere (service::Aggregator::newRequest, Aggregator.h:56) -------
 * One httpparser::HttpRequest with its DiscoverySessionMeta (Aggregator.h:40-44): what
 * Aggregator::newRequest reads of them (Aggregator.cpp:44-130, 155-168).  Its strings lie at
 * strings + str_off: host_len bytes of host, url_len bytes of url, then cip_len bytes of
 * clientIp.front() (cip_len = EBD_NO_CLIENT_IP: clientIp is empty, the client is the source
 * address). */
#define EBD_NO_CLIENT_IP 0xffffu
typedef struct ebd_request {
	uint64_t str_off;
	uint32_t pid;          /* DiscoverySessionMeta.pid */
	uint16_t host_len, url_len;
	uint16_t cip_len;
	uint8_t flags;         /* DiscoverySessionMeta.flags (EBD_FLAG_SESSION_*: IPv4 / IPv6 source) */
	uint8_t is_https;      /* HttpRequest::isHttps: the scheme of a service it creates */
	uint8_t source_ip[16]; /* DiscoverySessionMeta.sourceIP */
	uint32_t pad_;
} ebd_request; /* 40 bytes */
/* Aggregator::newRequest for n such requests in order (host memory), as one batch: the same
 * service key, first-arrival scheme and domain, client class and network maps as requests the
 * parse path finishes (they take the next n positions of the global event order).  Blocks
 * until done.  Lengths over EBD_MAX_HTTP_REQUEST_LENGTH, or strings past strings_len: -EINVAL. */
int ebd_aggregate_requests(ebd_ctx* ctx, const ebd_request* reqs, uint32_t n, const char* strings, uint64_t strings_len);

/* --- one request stream at a time (httpparser::HttpRequestParser, HttpRequestParser.h:41-101) ---
 * For callers that drive a parser object per connection, as the reference's tests and
 * handleExistingSession do: parse(std::string_view, flags), isFinished, isInvalidState, reset,
 * result.  The parser state is caller-owned plain data (ebd_parser_state: the generic state
 * machine plus the result's client-IP tokens); ebd_parse_streams runs n such parsers, one chunk
 * each, on the GPU (HttpRequestParser.cpp:85-106 and the handlers :162-409, exactly; the 8192-B
 * cap included).  A call sees the request stream since the parser's last reset, data[data_off,
 * data_off + data_len), and parses the bytes from the parser's position onwards: the chunk the
 * caller appended.  Every span it returns is a position in that stream. */
#define EBD_PARSE_MAX_TOKENS 32
typedef struct ebd_parser_state {
	uint64_t opaque_[40]; /* 320 bytes */
} ebd_parser_state;
enum {
	EBD_PARSER_UNFINISHED = 0, /* waiting for more bytes */
	EBD_PARSER_FINISHED = 1,   /* isFinished() && !isInvalidState() */
	EBD_PARSER_INVALID = 2,    /* isInvalidState() (isFinished() too) */
};
typedef struct ebd_parse_call {
	ebd_parser_state state; /* in: the parser (ebd_parser_init / ebd_parser_reset / a previous call); out: after */
	uint64_t data_off;      /* the stream since reset: data[data_off, data_off + data_len) */
	uint32_t data_len;
	uint8_t flags;          /* DiscoveryFlags of the chunk: EBD_FLAG_SESSION_SSL_HTTP sets isHttps when it ends */
	uint8_t pad_[3];
	/* out: HttpRequestParser::parse's return value and HttpRequest (HttpRequestParser.h:28-39) */
	uint32_t consumed;
	uint8_t status;         /* EBD_PARSER_* */
	uint8_t is_https;       /* result.isHttps (set when the parse ended) */
	uint8_t client_ip_key;  /* result.clientIPKey: 0 none, 1..5 = ebd_client_ip_key_name(id) (sticky across reset) */
	uint8_t tokens_dropped; /* result.clientIp had more than EBD_PARSE_MAX_TOKENS entries (the rest are not listed) */
	uint32_t method_len;    /* result.method = stream[0, method_len) */
	uint32_t url_off, url_len;
	uint32_t protocol_off, protocol_len;
	uint32_t host_off, host_len;
	uint32_t ntokens;       /* result.clientIp[k] = stream[tokens[k][0], tokens[k][1]) */
	uint32_t tokens[EBD_PARSE_MAX_TOKENS][2];
} ebd_parse_call;
/* HttpRequestParser() and reset() (HttpRequestParser.cpp:82-83, 374-379: reset keeps
 * result.clientIPKey).  Host-only: they write the state, nothing runs on the GPU. */
int ebd_parser_init(ebd_parser_state* st);
int ebd_parser_reset(ebd_parser_state* st);
/* 0 if st is a state these calls can have written for a stream of stream_len bytes (its
 * position, client-IP value and token count, key and clientIPKey in range), else -EINVAL.
 * Host-only; ebd_parse_streams applies it to every call and fails with -EINVAL. */
int ebd_parser_state_check(const ebd_parser_state* st, uint64_t stream_len);
/* n parsers, one chunk each (host arrays; data is the calls' streams).  Blocks until done;
 * -EINVAL (nothing runs) if a stream lies outside data or a state fails ebd_parser_state_check. */
int ebd_parse_streams(ebd_ctx* ctx, ebd_parse_call* calls, uint32_t n, const uint8_t* data, uint64_t data_len);
/* HEADER_CLIENT_IP_KEYS[id - 1] (HttpRequestParser.cpp:43) for a client_ip_key id, "" for 0. */
const char* ebd_client_ip_key_name(uint32_t id);

int ebd_get_stats(ebd_ctx* ctx, ebd_stats* out);
const char* ebd_strerror(int err);
/* The measured HBM read-stream peak of `device` over a `bytes` buffer (>= 16 MiB), `reps` timed
 * passes each: plain 16-byte-per-lane loads and LDS-DMA (global_load_lds) tiles, in GB/s.  The
 * roofline's second reference beside the 8 TB/s spec; allocates and frees its
 * own buffer. */
int ebd_measure_read_bandwidth(int device, uint64_t bytes, uint32_t reps, double* plain_gbps, double* dma_gbps);
/* Hash of the sources this library was built from (profiles/ name the build they measured). */
const char* ebd_build_id(void);

/* --- synthetic traces, identical on host and device ---------- */
typedef struct ebd_trace_config {
	uint32_t config; /* 1, 11, 2, 3: single-buffer configs; 5: config 3's distribution, sharded */
	uint64_t seed;
	uint64_t first;  /* first candidate event index of the trace */
	uint32_t n;      /* candidate events [first, first + n) */
	uint32_t align;  /* payload offset alignment (power of two, >= 1) */
	uint32_t shard_count; /* > 1: keep only the events whose connection (pid, fd, sessionID) hashes */
	uint32_t shard_index; /*     to shard_index mod shard_count (ebd/shard.py connection_hash) */
} ebd_trace_config;

/* Events kept and payload bytes of a trace slice. */
int ebd_trace_size(const ebd_trace_config* cfg, uint32_t* n_events, uint64_t* payload_bytes);
/* Host generation into caller arrays (events, len, off, payload; gidx = trace index of each
 * kept event, may be NULL). */
int ebd_trace_generate_host(const ebd_trace_config* cfg, ebd_discovery_event* events, uint32_t* len, uint64_t* off,
		uint8_t* payload, uint64_t payload_cap, uint64_t* gidx);
/* The same sizes, computed on the context's GPU. */
int ebd_trace_size_device(ebd_ctx* ctx, const ebd_trace_config* cfg, uint32_t* n_events, uint64_t* payload_bytes);
/* Device generation straight into HBM (pointers are device pointers; gidx may be NULL). */
int ebd_trace_generate_device(ebd_ctx* ctx, const ebd_trace_config* cfg, ebd_discovery_event* events, uint32_t* len,
		uint64_t* off, uint8_t* payload, uint64_t payload_cap, uint64_t* gidx);

#ifdef __cplusplus
}
#endif

#endif
