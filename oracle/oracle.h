/*
 * oracle.h — CPU restatement of the eBPF-Discovery HTTP per-event parse path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker, never the product: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product path (ebpf-discovery_amd/, libebd_amd.so) never links or calls it.
 *
 * Every function restates reference behaviour and cites the reference file:line
 * it follows (paths relative to the dynatrace-oss/eBPF-Discovery checkout).
 *
 * Pinning: the reference itself is unbuildable in this image (it needs boost 1.83,
 * spdlog/fmt, gtest and libbpf, none of which are installed; building it would need
 * stand-in headers, which this project does not write).  The restatement is pinned
 * instead by the reference's own unit-test vectors, transcribed as data into
 * tests/golden/ JSON files (HttpRequestParserTest.cpp, AggregatorTest.cpp,
 * IpAddressCheckerTest.cpp, IpAddressTest.cpp, LRUCacheTest.cpp), by the survey's
 * probe outputs of the compiled reference (marked
 * [probe]) and, for the glibc dependency (inet_pton / inet_ntop), by the system
 * glibc present in this container.
 */
#pragma once

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Wire record, libebpfdiscoveryshared/headers/ebpfdiscoveryshared/Types.h:201-205
 * (DiscoverySavedBufferKey key @0, DiscoverySockSourceIP sourceIP @16, flags @32). */
typedef struct {
	uint32_t pid, fd, sessionID, bufferSeq;
	uint8_t sourceIP[16];
	uint8_t flags;
	uint8_t pad_[3];
} orc_event;

/* Flags, Types.h:122-129 */
#define ORC_FLAG_IPV4 2
#define ORC_FLAG_IPV6 4
#define ORC_FLAG_UNENCRYPTED 8
#define ORC_FLAG_SSL 16
#define ORC_FLAG_NEW_DATA 32
#define ORC_FLAG_DATA_END 64

/* Parser states, libhttpparser/headers/httpparser/HttpRequestParser.h:55-68 */
enum {
	ORC_ST_METHOD = 0,
	ORC_ST_SPACE_BEFORE_URL,
	ORC_ST_URL,
	ORC_ST_SPACE_BEFORE_PROTOCOL,
	ORC_ST_PROTOCOL,
	ORC_ST_HEADER_NEWLINE,
	ORC_ST_HEADER_KEY,
	ORC_ST_SPACE_BEFORE_HEADER_VALUE,
	ORC_ST_HEADER_VALUE,
	ORC_ST_HEADERS_END,
	ORC_ST_FINISHED,
	ORC_ST_INVALID,
};

/* Per-event outcome of one replayed event. */
enum { ORC_KIND_NONE = 0, ORC_KIND_NEW = 1, ORC_KIND_EXISTING = 2 };
enum { ORC_STATUS_NONE = 0, ORC_STATUS_UNFINISHED = 1, ORC_STATUS_FINISHED = 2, ORC_STATUS_INVALID = 3 };
enum { ORC_CLASS_NONE = 0, ORC_CLASS_INTERNAL = 1, ORC_CLASS_EXTERNAL = 2 };

typedef struct {
	uint32_t kind;     /* ORC_KIND_* : which Discovery handler parsed it */
	uint32_t status;   /* parser state after this event's parse() call */
	uint32_t consumed; /* parse() return value for this event */
	uint32_t cls;      /* client classification of a FINISHED request */
	uint32_t is_https;
	uint32_t has_cip;  /* request.clientIp non-empty */
	uint64_t host_off, url_off, cip_off; /* offsets into the result blob */
	uint32_t host_len, url_len, cip_len; /* cip = request.clientIp.front() */
	uint32_t pad_;
} orc_event_result;

typedef struct {
	uint64_t kernel_deletes;  /* bpfDiscoveryDeleteSession calls, Discovery.cpp:125-129 */
	uint64_t lru_evictions;   /* LRUCache.h:56-58 */
	uint64_t lru_size;        /* live saved sessions at the end */
	uint64_t requests;        /* Aggregator::newRequest calls */
	uint64_t missing_buffers; /* NEW_DATA events whose buffer lookup failed, Discovery.cpp:103-107 */
} orc_stats;

typedef struct orc_ctx orc_ctx;

/* --- Discovery replay (Discovery.cpp:73-198 with Aggregator.cpp:155-168) -------- */
orc_ctx* orc_create(uint32_t lru_capacity);
void orc_destroy(orc_ctx* c);
/* v4: n4 records of {addr[4], mask[4]} (network byte order, like in_addr);
 * v6: n6 records of {addr[16], mask[16]}.  InterfacesReader.h:15-24 */
void orc_set_interfaces(orc_ctx* c, const uint8_t* v4, uint32_t n4, const uint8_t* v6, uint32_t n6);
/* Replay n events.  len[i] == UINT32_MAX marks "no saved buffer" (map lookup fails). */
int orc_process(orc_ctx* c, const orc_event* ev, const uint32_t* len, const uint64_t* off, const uint8_t* payload, uint32_t n,
		orc_event_result* out);
void orc_blob(orc_ctx* c, const char** data, uint64_t* size);
void orc_blob_reset(orc_ctx* c);
void orc_get_stats(orc_ctx* c, orc_stats* s);
/* Services sorted by (pid, endpoint); one line each:
 * pid \t endpoint \t domain \t scheme \t internal \t external \n.  Returns bytes needed. */
uint64_t orc_services_dump(orc_ctx* c, char* buf, uint64_t cap);
/* The same with a 7th column: the index (over all orc_process calls) of the event whose
 * request created the service — the first arrival that fixed its domain and scheme. */
uint64_t orc_services_dump_first(orc_ctx* c, char* buf, uint64_t cap);
uint64_t orc_service_count(orc_ctx* c);
void orc_clear(orc_ctx* c);

/* --- network counters (Aggregator.cpp:43, 89-106, 136-153, 182-209) -------------- */
void orc_set_network_counters(orc_ctx* c, int on);
/* getCurrentTime() (steady-clock ns) for the requests that follow */
void orc_set_time(orc_ctx* c, uint64_t now);
void orc_network_counters_cleaning(orc_ctx* c, uint64_t now);
/* services_dump rows with three more columns: the sizes of the /16, /24 and v6 maps */
uint64_t orc_services_dump_nets(orc_ctx* c, char* buf, uint64_t cap);
/* pid \t endpoint \t kind (1: v4 /16, 2: v4 /24, 3: v6 48-bit) \t prefix as 12 hex digits \t time \n */
uint64_t orc_nets_dump(orc_ctx* c, char* buf, uint64_t cap);
/* Discovery::outputServicesToStdout text (Discovery.cpp:60-71, Json.h:32-71), creation order */
uint64_t orc_services_json(orc_ctx* c, char* buf, uint64_t cap);

/* Aggregator driven directly (AggregatorTest.cpp:53-156).  cip may be NULL.
 * A mock verdict queue, when set, answers the IpAddressChecker calls in order
 * (IpAddressCheckerMock, AggregatorTest.cpp:34-39). */
void orc_agg_new_request(orc_ctx* c, uint32_t pid, const char* host, const char* url, const char* cip, uint8_t flags,
		const uint8_t* source_ip16);
void orc_set_checker_mock(orc_ctx* c, const int* verdicts, uint32_t n);

/* --- HttpRequestParser (HttpRequestParser.cpp) ---------------------------------- */
typedef struct orc_parser orc_parser;
orc_parser* orc_parser_new(void);
void orc_parser_free(orc_parser* p);
size_t orc_parser_parse(orc_parser* p, const uint8_t* data, size_t len, uint8_t flags);
int orc_parser_state(const orc_parser* p);
void orc_parser_reset(orc_parser* p);
/* method \n url \n protocol \n host \n clientIPKey \n isHttps \n ip0 \x1f ip1 ... \n */
uint64_t orc_parser_result(const orc_parser* p, char* buf, uint64_t cap);
/* Calibration: parse() only over n buffers, a reset parser per buffer; returns bytes consumed */
uint64_t orc_parse_only(const uint8_t* payload, const uint64_t* off, const uint32_t* len, uint32_t n);
/* parseClientIPValue (HttpRequestParser.cpp:392-409) on a fresh parser: tokens joined by \x1f */
uint64_t orc_parse_client_ip(const char* data, size_t len, char* buf, uint64_t cap, uint32_t* count);

/* --- glibc inet (resolv/inet_pton.c, inet/inet_ntop.c; glibc 2.35) ---------------- */
int orc_inet_pton4(const char* s, size_t len, uint8_t out[4]);
int orc_inet_pton6(const char* s, size_t len, uint8_t out[16]);
void orc_inet_ntop4(const uint8_t in[4], char out[16]);
void orc_inet_ntop6(const uint8_t in[16], char out[46]);

/* --- IpAddressCheckerImpl (IpAddressCheckerImpl.cpp:39-180) ----------------------- */
int orc_is_v4_external(orc_ctx* c, const uint8_t addr[4]);
int orc_is_v6_external(orc_ctx* c, const uint8_t addr[16]);

/* --- LRUCache (LRUCache.h:26-107) with int keys / int values (LRUCacheTest.cpp) --- */
typedef struct orc_lru orc_lru;
orc_lru* orc_lru_new(uint32_t capacity);
void orc_lru_free(orc_lru* l);
void orc_lru_insert(orc_lru* l, uint32_t key, int64_t value);
/* returns 1 and *value if found (and touches it), else 0 */
int orc_lru_find(orc_lru* l, uint32_t key, int64_t* value);
int orc_lru_erase(orc_lru* l, uint32_t key);
int orc_lru_update(orc_lru* l, uint32_t key, int64_t value);
uint32_t orc_lru_size(const orc_lru* l);

#ifdef __cplusplus
}
#endif
