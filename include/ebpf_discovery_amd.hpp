/*
 * ebpf_discovery_amd.hpp — header-only C++ facade over the C ABI (ebpf_discovery_amd.h)
 * that keeps the reference's consumer-side API shape, so the event-consumer loop and the
 * aggregator's callers change as little as possible:
 *
 *   ebdamd::Aggregator  ~ service::Aggregator      (libservice/headers/service/Aggregator.h:46-68):
 *                         clear, collectServices, networkCountersCleaning, getCurrentTime;
 *                         newEvents takes one poll cycle's captured buffers (HttpRequestParser::parse
 *                         runs inside the same GPU pass), and newRequest(HttpRequest,
 *                         DiscoverySessionMeta) takes requests parsed elsewhere, queued and handed
 *                         to the GPU in batches (ebd_aggregate_requests)
 *   ebdamd::HttpRequest ~ httpparser::HttpRequest  (HttpRequestParser.h:28-39)
 *   ebdamd::HttpRequestParser ~ httpparser::HttpRequestParser (HttpRequestParser.h:41-101): parse,
 *                         isFinished, isInvalidState, reset, result; each parse() is one GPU call
 *                         (ebd_parse_streams) on the parser's own state
 *   ebdamd::DiscoverySessionMeta ~ DiscoverySessionMeta (Aggregator.h:40-44)
 *   ebdamd::Service     ~ service::Service         (Service.h:43-66; the network maps as their sizes,
 *                         which is all the report prints, Service.h:84-98)
 *   ebdamd::Discovery   ~ ebpfdiscovery::Discovery (Discovery.h:33-44): init, fetchAndHandleEvents,
 *                         outputServicesToStdout, networkCountersCleaning, with the BPF maps behind
 *                         an EventSource (the queue, the saved buffers, bpfDiscoveryDeleteSession)
 *
 * Errors: the C ABI returns 0 / -errno and never throws; this facade throws ebdamd::Error where
 * the reference throws (construction and init, Discovery.cpp:42-46) and returns the int
 * convention from fetchAndHandleEvents (Discovery.cpp:48-90).  Needs only the C header and
 * libebd_amd.so: no HIP or torch types appear here.
 */
#ifndef EBPF_DISCOVERY_AMD_HPP
#define EBPF_DISCOVERY_AMD_HPP

#include "ebpf_discovery_amd.h"

#include <algorithm>
#include <cerrno>
#include <cstdint>
#include <cstring>
#include <iostream>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace ebdamd {

class Error : public std::runtime_error {
public:
	Error(const std::string& what, int code) : std::runtime_error(what + ": " + ebd_strerror(code)), code_(code) {}
	int code() const { return code_; }

private:
	int code_;
};

inline void check(int rc, const char* what) {
	if (rc != 0)
		throw Error(what, rc);
}

/* InterfacesReader::collectAllIpInterfaces (InterfacesReader.cpp:50-78) as it feeds
 * IpAddressCheckerImpl: the host's IPv4 / IPv6 networks. */
struct IpInterfaces {
	std::vector<ebd_ipv4_network> v4;
	std::vector<ebd_ipv6_network> v6;
};

/* service::Service (Service.h:43-66). */
struct Service {
	uint32_t pid = 0;
	std::string endpoint;
	std::string domain;
	std::string scheme;
	uint32_t internalClientsNumber = 0;
	uint32_t externalClientsNumber = 0;
	/* sizes of externalIPv4_16ClientNets, externalIPv4_24ClientNets, externalIPv6ClientsNets */
	uint32_t externalIPv4_16ClientNets = 0;
	uint32_t externalIPv4_24ClientNets = 0;
	uint32_t externalIPv6ClientsNets = 0;

	bool operator==(const Service& o) const {
		return pid == o.pid && endpoint == o.endpoint && domain == o.domain && scheme == o.scheme &&
				internalClientsNumber == o.internalClientsNumber && externalClientsNumber == o.externalClientsNumber &&
				externalIPv4_16ClientNets == o.externalIPv4_16ClientNets &&
				externalIPv4_24ClientNets == o.externalIPv4_24ClientNets && externalIPv6ClientsNets == o.externalIPv6ClientsNets;
	}
};

/* httpparser::HttpRequest (HttpRequestParser.h:28-39): the fields a parse fills. */
struct HttpRequest {
	std::string method;
	std::string url;
	std::string protocol;
	std::string host;
	std::string clientIPKey;
	std::vector<std::string> clientIp;
	bool isHttps = false;
	/* not in the reference: the client-IP header had more than EBD_PARSE_MAX_TOKENS entries, so
	 * clientIp lists only the first ones (the reference's vector has them all; the aggregator only
	 * reads clientIp[0], Aggregator.cpp:57-63, so discovery results are unaffected) */
	bool clientIpTruncated = false;

	/* HttpRequest::clear (HttpRequestParser.cpp:67-80) */
	void clear() {
		method.clear();
		url.clear();
		protocol.clear();
		host.clear();
		clientIp.clear();
		isHttps = false;
		clientIpTruncated = false;
	}
};

/* httpparser::HttpRequestParser (HttpRequestParser.h:41-101) over ebd_parse_streams: the state
 * machine runs on the GPU one chunk per parse() call (speed is not the point here: the batch
 * entry points are); the facade keeps the request's bytes since reset() and materialises
 * `result` from the positions the GPU returns, as the reference returns std::string copies.
 * A parser without a context uses one process-wide context on device 0, created on first use
 * and kept until exit (destroying it from a static destructor could outlive the HIP runtime). */
class HttpRequestParser {
public:
	explicit HttpRequestParser(ebd_ctx* ctx = nullptr) : ctx_(ctx ? ctx : sharedContext()) {
		check(ebd_parser_init(&state_), "ebd_parser_init");
	}

	/* HttpRequestParser::parse (HttpRequestParser.cpp:85-106): the bytes of `data` this call
	 * consumed; the rest of a chunk after the request's end is not parsed (no pipelining). */
	size_t parse(std::string_view data, uint8_t discoveryFlags) {
		const size_t base = stream_.size();
		stream_.append(data.data(), data.size());
		ebd_parse_call call{};
		call.state = state_;
		call.data_off = 0;
		call.data_len = (uint32_t)stream_.size();
		call.flags = discoveryFlags;
		const int rc = ebd_parse_streams(ctx_, &call, 1, reinterpret_cast<const uint8_t*>(stream_.data()), stream_.size());
		if (rc != 0) {
			stream_.resize(base);
			throw Error("ebd_parse_streams", rc);
		}
		state_ = call.state;
		status_ = call.status;
		stream_.resize(base + call.consumed);
		fill(call);
		return call.consumed;
	}

	/* HttpRequestParser.cpp:108-114 */
	bool isInvalidState() const { return status_ == EBD_PARSER_INVALID; }
	bool isFinished() const { return status_ != EBD_PARSER_UNFINISHED; }

	/* HttpRequestParser.cpp:374-379: result.clientIPKey survives */
	void reset() {
		check(ebd_parser_reset(&state_), "ebd_parser_reset");
		status_ = EBD_PARSER_UNFINISHED;
		stream_.clear();
		result.clear();
	}

	HttpRequest result;

private:
	static ebd_ctx* sharedContext() {
		static ebd_ctx* ctx = [] {
			ebd_config cfg{};
			cfg.max_events = 1;
			cfg.service_capacity = 1024;
			cfg.string_arena = 1 << 20;
			cfg.lru_capacity = 1;
			ebd_ctx* c = nullptr;
			check(ebd_ctx_create(&cfg, &c), "ebd_ctx_create");
			return c;
		}();
		return ctx;
	}

	std::string span(uint32_t off, uint32_t len) const {
		if (off > stream_.size())
			return std::string();
		return stream_.substr(off, std::min<size_t>(len, stream_.size() - off));
	}

	void fill(const ebd_parse_call& c) {
		result.method = span(0, c.method_len);
		result.url = span(c.url_off, c.url_len);
		result.protocol = c.protocol_len ? span(c.protocol_off, c.protocol_len) : std::string();
		result.host = span(c.host_off, c.host_len);
		result.clientIPKey = ebd_client_ip_key_name(c.client_ip_key);
		result.clientIp.clear();
		for (uint32_t k = 0; k < c.ntokens && k < EBD_PARSE_MAX_TOKENS; k++)
			result.clientIp.push_back(span(c.tokens[k][0], c.tokens[k][1] - c.tokens[k][0]));
		result.isHttps = c.is_https != 0;
		result.clientIpTruncated = c.tokens_dropped != 0;
	}

	ebd_ctx* ctx_;
	ebd_parser_state state_{};
	uint8_t status_ = EBD_PARSER_UNFINISHED;
	std::string stream_; // the request's bytes since reset (what the parser consumed)
};

/* DiscoverySessionMeta (Aggregator.h:40-44): the session a request came in on. */
struct DiscoverySessionMeta {
	uint8_t sourceIP[16] = {}; /* DiscoverySockSourceIP: in_addr or in6_addr bytes */
	uint32_t pid = 0;
	uint8_t flags = 0;         /* DiscoveryFlags (EBD_FLAG_SESSION_IPV4 / _IPV6 select the family) */
};

/* One poll cycle's events with their saved buffers, packed back to back: what
 * Discovery::handleNewEvent sees one event at a time (Discovery.cpp:92-121). */
class EventBatch {
public:
	/* A NEW_DATA and/or DATA_END event; buf == nullptr: the saved buffer is missing
	 * (bpf_map_lookup_and_delete_elem failed, Discovery.cpp:101-107). */
	void add(const ebd_discovery_event& ev, const void* buf, uint32_t len) {
		events_.push_back(ev);
		offsets_.push_back(payload_.size());
		if (!buf) {
			lengths_.push_back(EBD_NO_BUFFER);
			return;
		}
		lengths_.push_back(len);
		const auto* b = static_cast<const uint8_t*>(buf);
		payload_.insert(payload_.end(), b, b + len);
	}
	void clear() {
		events_.clear();
		lengths_.clear();
		offsets_.clear();
		payload_.clear();
	}
	uint32_t size() const { return (uint32_t)events_.size(); }
	bool empty() const { return events_.empty(); }
	const ebd_discovery_event* events() const { return events_.data(); }
	const uint32_t* lengths() const { return lengths_.data(); }
	const uint64_t* offsets() const { return offsets_.data(); }
	const uint8_t* payload() const { return payload_.data(); }
	uint64_t payloadBytes() const { return payload_.size(); }
	const ebd_discovery_event& event(uint32_t i) const { return events_[i]; }

private:
	std::vector<ebd_discovery_event> events_;
	std::vector<uint32_t> lengths_;
	std::vector<uint64_t> offsets_;
	std::vector<uint8_t> payload_;
};

struct Options {
	int device = 0;
	uint32_t maxEvents = 1u << 20;      /* largest poll cycle */
	uint64_t maxPayload = 256ull << 20; /* largest packed payload of a poll cycle */
	uint32_t serviceCapacity = 0;       /* 0: the library default */
	uint32_t lruCapacity = 0;           /* 0: EBD_MAX_SESSIONS (Discovery.cpp:39) */
	uint32_t netCapacity = 0;
};

/* service::Aggregator (Aggregator.h:46-68) with the session parsers of Discovery in front of it:
 * the context keeps the LRU of saved sessions, the service table and the interface list. */
class Aggregator {
public:
	Aggregator(const IpInterfaces& ifaces, bool enableNetworkCounters, const Options& opt = Options{}) {
		ebd_config cfg{};
		cfg.device = opt.device;
		cfg.max_events = opt.maxEvents;
		cfg.max_payload = opt.maxPayload;
		cfg.service_capacity = opt.serviceCapacity;
		cfg.lru_capacity = opt.lruCapacity;
		cfg.net_capacity = opt.netCapacity;
		cfg.flags = enableNetworkCounters ? EBD_CFG_NETWORK_COUNTERS : 0u;
		check(ebd_ctx_create(&cfg, &ctx_), "ebd_ctx_create");
		const int rc = ebd_set_interfaces(ctx_, ifaces.v4.data(), (uint32_t)ifaces.v4.size(), ifaces.v6.data(),
				(uint32_t)ifaces.v6.size());
		if (rc != 0) {
			ebd_ctx_destroy(ctx_);
			ctx_ = nullptr;
			throw Error("ebd_set_interfaces", rc);
		}
	}
	virtual ~Aggregator() {
		if (ctx_)
			ebd_ctx_destroy(ctx_);
	}
	Aggregator(const Aggregator&) = delete;
	Aggregator& operator=(const Aggregator&) = delete;

	/* Aggregator::clear (Aggregator.cpp:136-153) */
	void clear() {
		flush();
		check(ebd_clear(ctx_), "ebd_clear");
	}

	/* Aggregator::newRequest (Aggregator.cpp:155-168) for a request parsed elsewhere.  Batched:
	 * the request is queued with its getCurrentTime() reading, and the queue goes to the GPU as
	 * one ebd_aggregate_requests call when the reading changes, at kMaxQueued requests, on
	 * flush(), and before anything that reads or changes the services (collectServices, report,
	 * stats, clear, networkCountersCleaning, newEvents).  Throws ebdamd::Error when the library
	 * refuses the batch (e.g. host + url longer than EBD_MAX_HTTP_REQUEST_LENGTH). */
	void newRequest(const HttpRequest& request, const DiscoverySessionMeta& meta) {
		const uint64_t now = getCurrentTime();
		if (!queue_.empty() && now != queueClock_)
			flush();
		queueClock_ = now;
		ebd_request q{};
		q.str_off = queueStrings_.size();
		q.pid = meta.pid;
		q.host_len = (uint16_t)std::min<size_t>(request.host.size(), 0xffffu);
		q.url_len = (uint16_t)std::min<size_t>(request.url.size(), 0xffffu);
		q.flags = meta.flags;
		q.is_https = request.isHttps ? 1 : 0;
		std::memcpy(q.source_ip, meta.sourceIP, sizeof(q.source_ip));
		queueStrings_ += request.host;
		queueStrings_ += request.url;
		if (request.clientIp.empty()) { // the source address decides (Aggregator.cpp:60-66, 85-88)
			q.cip_len = EBD_NO_CLIENT_IP;
		} else { // clientIp.front() decides (Aggregator.cpp:50-59)
			q.cip_len = (uint16_t)std::min<size_t>(request.clientIp.front().size(), EBD_NO_CLIENT_IP - 1u);
			queueStrings_ += request.clientIp.front();
		}
		queue_.push_back(q);
		if (queue_.size() >= kMaxQueued)
			flush();
	}

	/* The queued newRequest calls to the GPU now. */
	void flush() {
		if (queue_.empty())
			return;
		if (queueClock_)
			check(ebd_set_clock(ctx_, queueClock_), "ebd_set_clock");
		const int rc = ebd_aggregate_requests(ctx_, queue_.data(), (uint32_t)queue_.size(), queueStrings_.data(), queueStrings_.size());
		queue_.clear();
		queueStrings_.clear();
		check(rc, "ebd_aggregate_requests");
	}

	/* Discovery::handleNewEvent for every event of the batch (Discovery.cpp:92-198), i.e.
	 * HttpRequestParser::parse on each buffer and Aggregator::newRequest on each finished
	 * request (Aggregator.cpp:155-168).  Returns 0 or -errno; the per-event outcomes are in
	 * lastResults(). */
	int newEvents(const EventBatch& batch) {
		flush();
		if (batch.empty())
			return 0;
		if (const uint64_t now = getCurrentTime())
			if (int rc = ebd_set_clock(ctx_, now))
				return rc;
		return ebd_submit_batch(ctx_, batch.events(), batch.lengths(), batch.offsets(), batch.payload(), batch.payloadBytes(),
				batch.size());
	}

	/* HttpRequestParser's outcome per event of the last batch (status, consumed, spans). */
	std::vector<ebd_event_result> lastResults() const {
		uint32_t n = 0;
		check(ebd_fetch_results(ctx_, nullptr, 0, &n), "ebd_fetch_results");
		std::vector<ebd_event_result> out(n);
		check(ebd_fetch_results(ctx_, out.data(), n, &n), "ebd_fetch_results");
		out.resize(n);
		return out;
	}

	/* Aggregator::collectServices (Aggregator.cpp:170-181); order unspecified. */
	std::vector<Service> collectServices() {
		flush();
		uint32_t n = 0;
		uint64_t bytes = 0;
		check(ebd_collect_services(ctx_, nullptr, 0, &n, nullptr, 0, &bytes), "ebd_collect_services");
		std::vector<ebd_service> raw(n ? n : 1);
		std::string strings(bytes ? bytes : 1, '\0');
		check(ebd_collect_services(ctx_, raw.data(), n, &n, &strings[0], strings.size(), &bytes), "ebd_collect_services");
		std::vector<Service> out;
		out.reserve(n);
		for (uint32_t k = 0; k < n; k++) {
			const ebd_service& s = raw[k];
			Service v;
			v.pid = s.pid;
			v.endpoint = strings.substr(s.endpoint_off, s.endpoint_len);
			v.domain = v.endpoint.substr(s.domain_off, s.domain_len);
			v.scheme = s.https ? "https" : "http";
			v.internalClientsNumber = s.internal_clients;
			v.externalClientsNumber = s.external_clients;
			v.externalIPv4_16ClientNets = s.nets_v4_16;
			v.externalIPv4_24ClientNets = s.nets_v4_24;
			v.externalIPv6ClientsNets = s.nets_v6;
			out.push_back(std::move(v));
		}
		return out;
	}

	/* Aggregator::networkCountersCleaning (Aggregator.cpp:182-209) at getCurrentTime(). */
	void networkCountersCleaning() {
		flush();
		check(ebd_network_counters_cleaning(ctx_, getCurrentTime()), "ebd_network_counters_cleaning");
	}

	/* The text Discovery::outputServicesToStdout prints (Discovery.cpp:60-71); "" without services. */
	std::string report() {
		flush();
		uint64_t len = 0;
		check(ebd_report_json(ctx_, nullptr, 0, &len), "ebd_report_json");
		std::string text(len, '\0');
		if (len)
			check(ebd_report_json(ctx_, &text[0], len, &len), "ebd_report_json");
		text.resize(len);
		return text;
	}

	ebd_stats stats() {
		flush();
		ebd_stats s{};
		check(ebd_get_stats(ctx_, &s), "ebd_get_stats");
		return s;
	}

	ebd_ctx* handle() const { return ctx_; }

protected:
	/* Aggregator::getCurrentTime (Aggregator.cpp:211-213): steady-clock ns of the next batch's
	 * requests.  0 lets the library read CLOCK_MONOTONIC itself; tests override it the way
	 * AggregatorMock does (AggregatorTest.cpp:41-46). */
	virtual uint64_t getCurrentTime() const { return 0; }

private:
	static constexpr size_t kMaxQueued = 1u << 16;
	ebd_ctx* ctx_ = nullptr;
	std::vector<ebd_request> queue_;
	std::string queueStrings_;
	uint64_t queueClock_ = 0;
};

/* The BPF side of Discovery (DiscoveryBpf.h; Discovery.cpp:73-110, 125-129, 210-226). */
class EventSource {
public:
	virtual ~EventSource() = default;
	/* bpf_map_lookup_and_delete_elem on eventsToUserspaceQueueMap: 0, -ENOENT when empty, or
	 * another -errno. */
	virtual int popEvent(ebd_discovery_event& ev) = 0;
	/* bpf_map_lookup_and_delete_elem on savedBuffersMap for ev's key: false when missing. */
	virtual bool takeSavedBuffer(const ebd_discovery_event& ev, std::vector<uint8_t>& data) = 0;
	/* bpfDiscoveryDeleteSession: the kernel stops tracking (pid, fd, sessionID). */
	virtual void deleteTrackedSession(uint32_t pid, uint32_t fd, uint32_t sessionID) = 0;
	/* bpfDiscoveryResetConfig / bpfDiscoveryResumeCollecting: 0 or -errno. */
	virtual int resetConfig() { return 0; }
	virtual int resumeCollecting() { return 0; }
};

/* ebpfdiscovery::Discovery (Discovery.h:33-44): one poll cycle drains the queue into a batch
 * and hands it to the GPU in one call. */
class Discovery {
public:
	Discovery(EventSource& source, bool enableNetworkCounters, const IpInterfaces& ifaces = IpInterfaces{},
			const Options& opt = Options{})
			: source_(source), aggregator_(ifaces, enableNetworkCounters, opt), maxEvents_(opt.maxEvents) {}

	/* Discovery.cpp:42-46 */
	void init() {
		if (const int ret = source_.resetConfig(); ret != 0)
			throw std::runtime_error("Could not initialize BPF program configuration: " + std::to_string(ret));
	}

	/* Discovery::fetchAndHandleEvents (Discovery.cpp:48-90): 0, or the first queue error other
	 * than -ENOENT.  A batch is handed over every maxEvents events and at the end. */
	int fetchAndHandleEvents() {
		if (const int ret = source_.resumeCollecting(); ret != 0)
			return ret;
		batch_.clear();
		ebd_discovery_event ev;
		int ret;
		for (;;) {
			ret = source_.popEvent(ev);
			if (ret != 0)
				break;
			if (ev.flags & EBD_FLAG_EVENT_NEW_DATA) {
				if (source_.takeSavedBuffer(ev, buf_))
					batch_.add(ev, buf_.data(), (uint32_t)buf_.size());
				else
					batch_.add(ev, nullptr, 0);
			} else {
				batch_.add(ev, nullptr, 0); // DATA_END only
			}
			if (batch_.size() == maxEvents_)
				if (int rc = handBatch(); rc != 0)
					return rc;
		}
		if (int rc = handBatch(); rc != 0)
			return rc;
		return ret == -ENOENT ? 0 : ret;
	}

	/* Discovery::outputServicesToStdout (Discovery.cpp:60-71): print, then clear. */
	void outputServicesToStdout(std::ostream& out = std::cout) {
		const std::string text = aggregator_.report();
		if (text.empty())
			return;
		out << text << std::flush;
		aggregator_.clear();
	}

	void networkCountersCleaning() { aggregator_.networkCountersCleaning(); }

	Aggregator& aggregator() { return aggregator_; }

private:
	/* The batch through the GPU; then Discovery::handleExistingSession's kernel delete for each
	 * saved session whose parser went INVALID (Discovery.cpp:125-129). */
	int handBatch() {
		if (batch_.empty())
			return 0;
		if (int rc = aggregator_.newEvents(batch_); rc != 0)
			return rc;
		const std::vector<ebd_event_result> res = aggregator_.lastResults();
		for (uint32_t i = 0; i < res.size() && i < batch_.size(); i++)
			if ((res[i].info & EBD_INFO_EXISTING) && res[i].status == EBD_STATUS_INVALID) {
				const ebd_discovery_event& e = batch_.event(i);
				source_.deleteTrackedSession(e.pid, e.fd, e.sessionID);
			}
		batch_.clear();
		return 0;
	}

	EventSource& source_;
	Aggregator aggregator_;
	uint32_t maxEvents_;
	EventBatch batch_;
	std::vector<uint8_t> buf_;
};

} // namespace ebdamd

#endif
