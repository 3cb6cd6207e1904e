// facade_test.cpp — INTEGRATION.md's C++ call sites compiled against include/ebpf_discovery_amd.hpp
// and libebd_amd.so (built by tests/cpp/Makefile; run by tests/test_cpp_facade.py).
//
//   facade_test cpu   no GPU: the batch packing, and the facade's error path (ebd_ctx_create
//                     fails, the constructor throws ebdamd::Error, Discovery.cpp:42-46 style)
//   facade_test gpu   the Discovery poll loop over an in-memory EventSource on cuda:0:
//                     config 1 (35-B and 31-B payloads), a saved session that
//                     goes INVALID (bpfDiscoveryDeleteSession, Discovery.cpp:125-129), the
//                     report and clear of outputServicesToStdout (Discovery.cpp:60-71) and the
//                     network counters with an overridden getCurrentTime (AggregatorTest.cpp:41-46);
//                     AggregatorTest's two scenarios (AggregatorTest.cpp:69-172, 174-285) rebuilt on
//                     Aggregator::newRequest(HttpRequest, DiscoverySessionMeta), the batching adapter;
//                     HttpRequestParserTest.cpp's TestValidRequest / testInvalidRequest cases
//                     (:152-191 over :193-300) on ebdamd::HttpRequestParser, and reset()'s sticky
//                     clientIPKey (HttpRequestParser.cpp:374-379)
// Prints "ok" and exits 0 when every check passes.
#include "ebpf_discovery_amd.hpp"

#include <cstdio>
#include <cstdlib>
#include <deque>
#include <map>
#include <sstream>
#include <tuple>

namespace {

int failures = 0;
#define CHECK(cond)                                                          \
	do {                                                                     \
		if (!(cond)) {                                                       \
			std::fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #cond); \
			failures++;                                                      \
		}                                                                    \
	} while (0)

ebd_discovery_event make_event(uint32_t pid, uint32_t fd, uint32_t sid, uint32_t seq, uint8_t flags, uint8_t src0 = 127,
		uint8_t src3 = 1) {
	ebd_discovery_event e{};
	e.pid = pid;
	e.fd = fd;
	e.sessionID = sid;
	e.bufferSeq = seq;
	e.sourceIP[0] = src0;
	e.sourceIP[3] = src3;
	e.flags = flags;
	return e;
}

// The BPF queue and savedBuffersMap in memory (DiscoveryBpf.h).
class MemorySource : public ebdamd::EventSource {
public:
	using Key = std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>;
	void push(const ebd_discovery_event& e, const std::string* data) {
		queue.push_back(e);
		if (data)
			saved[Key{e.pid, e.fd, e.sessionID, e.bufferSeq}] = std::vector<uint8_t>(data->begin(), data->end());
	}
	int popEvent(ebd_discovery_event& ev) override {
		if (queue.empty())
			return -ENOENT;
		ev = queue.front();
		queue.pop_front();
		return 0;
	}
	bool takeSavedBuffer(const ebd_discovery_event& ev, std::vector<uint8_t>& data) override {
		auto it = saved.find(Key{ev.pid, ev.fd, ev.sessionID, ev.bufferSeq});
		if (it == saved.end())
			return false;
		data = std::move(it->second);
		saved.erase(it);
		return true;
	}
	void deleteTrackedSession(uint32_t pid, uint32_t fd, uint32_t sid) override { deleted.push_back(Key{pid, fd, sid, 0}); }

	std::deque<ebd_discovery_event> queue;
	std::map<Key, std::vector<uint8_t>> saved;
	std::vector<Key> deleted;
};

constexpr uint8_t kV4New = EBD_FLAG_SESSION_IPV4 | EBD_FLAG_SESSION_UNENCRYPTED_HTTP | EBD_FLAG_EVENT_NEW_DATA;

int run_cpu() {
	ebdamd::EventBatch b;
	const std::string req = "GET / HTTP/1.1\r\nHost: h\r\n\r\n";
	b.add(make_event(1, 5, 1, 1, kV4New), req.data(), (uint32_t)req.size());
	b.add(make_event(1, 5, 2, 1, kV4New), nullptr, 0);
	b.add(make_event(1, 5, 3, 1, EBD_FLAG_EVENT_DATA_END), nullptr, 0);
	b.add(make_event(1, 5, 4, 1, kV4New), req.data(), 10);
	CHECK(b.size() == 4);
	CHECK(b.lengths()[0] == req.size() && b.lengths()[1] == EBD_NO_BUFFER && b.lengths()[2] == EBD_NO_BUFFER);
	CHECK(b.offsets()[3] == req.size() && b.lengths()[3] == 10);
	CHECK(b.payloadBytes() == req.size() + 10);
	CHECK(std::memcmp(b.payload() + req.size(), req.data(), 10) == 0);
	// no GPU: the context cannot be created, and the facade throws where the reference does
	bool threw = false;
	try {
		ebdamd::Aggregator agg(ebdamd::IpInterfaces{}, false);
	} catch (const ebdamd::Error& e) {
		threw = e.code() < 0;
	}
	CHECK(threw);
	MemorySource src;
	threw = false;
	try {
		ebdamd::Discovery d(src, true);
	} catch (const ebdamd::Error&) {
		threw = true;
	}
	CHECK(threw);
	return 0;
}

class ClockedAggregator : public ebdamd::Aggregator {
public:
	using ebdamd::Aggregator::Aggregator;
	uint64_t now = 1000000000000ull;

protected:
	uint64_t getCurrentTime() const override { return now; }
};

// ServiceAggregatorTest::makeRequest (AggregatorTest.cpp:48-62).  The reference's tests mock
// IpAddressChecker's verdict per call; here the real checker (no interfaces) classifies the
// session source address, so each request carries an address with the verdict the test mocks:
// external 8.8.8.8 / 2001:4860::8888, internal 10.0.0.1 / ::1.
std::pair<ebdamd::HttpRequest, ebdamd::DiscoverySessionMeta> makeRequest(uint32_t pid, const std::string& host,
		const std::string& url, int flags = -1, bool external = false) {
	ebdamd::HttpRequest request;
	request.host = host;
	request.url = url;
	ebdamd::DiscoverySessionMeta meta;
	if (flags >= 0) {
		request.isHttps = (flags & EBD_FLAG_SESSION_SSL_HTTP) != 0;
		meta.flags = (uint8_t)flags;
	}
	meta.pid = pid;
	if (meta.flags & EBD_FLAG_SESSION_IPV4) {
		const uint8_t a[4] = {8, 8, 8, 8}, b[4] = {10, 0, 0, 1};
		std::memcpy(meta.sourceIP, external ? a : b, 4);
	} else if (meta.flags & EBD_FLAG_SESSION_IPV6) {
		if (external) {
			const uint8_t a[16] = {0x20, 0x01, 0x48, 0x60, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x88, 0x88};
			std::memcpy(meta.sourceIP, a, 16);
		} else {
			meta.sourceIP[15] = 1;
		}
	}
	return {request, meta};
}

ebdamd::Service svc(uint32_t pid, const char* ep, const char* dom, const char* scheme, uint32_t in, uint32_t ex,
		uint32_t n16 = 0, uint32_t n24 = 0, uint32_t n6 = 0) {
	ebdamd::Service s;
	s.pid = pid;
	s.endpoint = ep;
	s.domain = dom;
	s.scheme = scheme;
	s.internalClientsNumber = in;
	s.externalClientsNumber = ex;
	s.externalIPv4_16ClientNets = n16;
	s.externalIPv4_24ClientNets = n24;
	s.externalIPv6ClientsNets = n6;
	return s;
}

bool contains(const std::vector<ebdamd::Service>& v, const ebdamd::Service& s) {
	for (const auto& x : v)
		if (x == s)
			return true;
	std::fprintf(stderr, "missing service pid %u endpoint '%s' domain '%s' scheme '%s' internal %u external %u\n", s.pid,
			s.endpoint.c_str(), s.domain.c_str(), s.scheme.c_str(), s.internalClientsNumber, s.externalClientsNumber);
	return false;
}

void aggregator_test_scenarios() {
	constexpr int V4 = EBD_FLAG_SESSION_IPV4, V6 = EBD_FLAG_SESSION_IPV6, PLAIN = EBD_FLAG_SESSION_UNENCRYPTED_HTTP,
			  SSL = EBD_FLAG_SESSION_SSL_HTTP;
	// ServiceAggregatorTest.aggregate (AggregatorTest.cpp:69-172)
	{
		ebdamd::Aggregator aggregator(ebdamd::IpInterfaces{}, false);
		CHECK(aggregator.collectServices().empty());
		auto add = [&](uint32_t pid, const char* host, const char* url, int flags, bool external) {
			const auto r = makeRequest(pid, host, url, flags, external);
			aggregator.newRequest(r.first, r.second);
		};
		add(100, "host", "/url", V4, true);                                             // Service 1
		add(100, "host", "/url", -1, false);                                            //   no flags: not counted
		add(100, "host", "/url2", V4, false);                                           // Service 2
		add(200, "host", "/url2", V4, true);                                            // Service 3
		add(200, "host", "/url2", V4, false);
		add(200, "host", "/url2", V4, true);
		add(400, "google.com", "/url123", V4 | PLAIN, true);                            // Service 4
		add(500, "8.8.8.8", "/url123", V4 | PLAIN, true);                               // Service 5
		add(600, "dynatrace.com", "/url123", V4 | SSL, true);                           // Service 6
		add(700, "[::1]", "/url123", V6 | PLAIN, false);                                // Service 7
		add(800, "[2001:0db8:85a3:0001:0000:0000:0000:0000]", "/url123", V6 | SSL, true); // Service 8
		add(900, "[2001:0db8:85a3:0001::]", "/url123", V6 | SSL, true);                 // Service 9
		const auto services = aggregator.collectServices();
		CHECK(services.size() == 9);
		CHECK(contains(services, svc(100, "host/url", "host", "http", 0, 1)));
		CHECK(contains(services, svc(100, "host/url2", "host", "http", 1, 0)));
		CHECK(contains(services, svc(200, "host/url2", "host", "http", 1, 2)));
		CHECK(contains(services, svc(400, "google.com/url123", "google.com", "http", 0, 1)));
		CHECK(contains(services, svc(500, "8.8.8.8/url123", "8.8.8.8", "http", 0, 1)));
		CHECK(contains(services, svc(600, "dynatrace.com/url123", "dynatrace.com", "https", 0, 1)));
		CHECK(contains(services, svc(700, "[::1]/url123", "[::1]", "http", 1, 0)));
		CHECK(contains(services, svc(800, "[2001:0db8:85a3:0001:0000:0000:0000:0000]/url123",
				"[2001:0db8:85a3:0001:0000:0000:0000:0000]", "https", 0, 1)));
		CHECK(contains(services, svc(900, "[2001:0db8:85a3:0001::]/url123", "[2001:0db8:85a3:0001::]", "https", 0, 1)));
		CHECK(aggregator.stats().requests == 12);
		aggregator.clear();
		CHECK(aggregator.collectServices().empty());
	}
	// ServiceAggregatorTest.aggregateNetworkCounters (AggregatorTest.cpp:174-285), with the mocked
	// clock's epoch at 1000 s (a map entry's time 0 means erased on the device)
	{
		ClockedAggregator aggregator(ebdamd::IpInterfaces{}, true);
		const uint64_t t0 = aggregator.now, minute = 60ull * 1000000000ull;
		CHECK(aggregator.collectServices().empty());
		const char* clients[] = {"172.143.4.5", "172.143.6.89", "172.199.45.55", "1234:2345:3456:4567:5678:6789:7890:8901",
				"2001:4860:4860:0000:0000:0000:0000:8888"};
		for (uint32_t pid : {100u, 200u})
			for (int k = 0; k < 5; k++) {
				auto r = makeRequest(pid, "host", "/url", (k < 3 ? V4 : V6) | (pid == 100 ? PLAIN : SSL), true);
				r.first.clientIp = {clients[k]};
				aggregator.newRequest(r.first, r.second);
			}
		auto services = aggregator.collectServices();
		CHECK(services.size() == 2);
		CHECK(contains(services, svc(100, "host/url", "host", "http", 0, 5, 2, 3, 2)));
		CHECK(contains(services, svc(200, "host/url", "host", "https", 0, 5, 2, 3, 2)));
		aggregator.now = t0 + 59 * minute;
		aggregator.networkCountersCleaning();
		aggregator.clear();
		services = aggregator.collectServices();
		CHECK(services.size() == 2);
		for (const auto& s : services)
			CHECK(s.externalClientsNumber == 0 && s.externalIPv4_16ClientNets == 2 && s.externalIPv4_24ClientNets == 3 &&
					s.externalIPv6ClientsNets == 2);
		aggregator.now = t0 + 60 * minute;
		aggregator.networkCountersCleaning();
		aggregator.clear();
		CHECK(aggregator.collectServices().empty());
		CHECK(aggregator.stats().errors == 0);
	}
}

// HttpRequestParserTest.cpp:152-191: chunks in order, the bytes parse() consumed in all, then
// isFinished / isInvalidState and the HttpRequest fields.
std::vector<std::string> chunk_string(const std::string& s, size_t n) { // the test's chunkString
	std::vector<std::string> out;
	for (size_t k = 0; k < s.size(); k += n)
		out.push_back(s.substr(k, n));
	return out;
}

struct ValidCase {
	std::vector<std::string> chunks;
	std::string method, url, protocol, host;
	std::vector<std::string> clientIp;
	bool isHttps = false, finished = true;
	size_t total = 0; // 0: every byte
};

void parser_test_cases() {
	const std::string post3 = "POST /example/ HTTP/1.1\r\nHost: example.com\r\nUser-Agent: curl/7.81.0\r\nAccept: */*\r\n"
	                          "X-Forwarded-For: 192.168.0.1:8080, 10.0.0.1, [2001:0db8:85a3::8a2e:0370:7334]\r\n\r\n"
	                          "{\"name\":\"example\"}\r\n";
	const std::vector<ValidCase> valid = {
			{{"GET /example HTTP/1.1\r\nHost: example.com\r\n\r\n"}, "GET", "/example", "HTTP/1.1", "example.com", {}},
			{{"POST /example HTTP/1.0\r\nHOST: example.com\r\n\r\n"}, "POST", "/example", "HTTP/1.0", "example.com", {}},
			{{"GET /example HTTP/1.1\r\nHost: example.com\r\n\r"}, "GET", "/example", "HTTP/1.1", "example.com", {}, false, false},
			{{"GET /Hello%20World/index.html HTTP/1.1\r\nHost:  example.com\r\nx-forwarded-for:  127.0.0.1\r\n\r\n"}, "GET",
					"/Hello%20World/index.html", "HTTP/1.1", "example.com", {"127.0.0.1"}},
			{{"GET / HTTP/1.1\r\n\r\n"}, "GET", "/", "HTTP/1.1", "", {}},
			{chunk_string("GET /example HTTP/1.1\r\nHost: example.com\r\nX-Forwarded-For: 0.0.0.0\r\n\r\n", 1), "GET", "/example",
					"HTTP/1.1", "example.com", {"0.0.0.0"}},
			{{post3}, "POST", "/example/", "HTTP/1.1", "example.com", {"192.168.0.1", "10.0.0.1", "2001:0db8:85a3::8a2e:0370:7334"},
					true, true, 163},
			{chunk_string("GET /example/ HTTP/1.1\r\nHost: example.com\r\nX-Forwarded-For: 10.0.0.1\r\nUser-Agent: curl/7.81.0\r\n"
			              "Accept: */*\r\nx-forwarded-for: 127.0.0.1,[2001:0db8:85a3::8a2e:0370:7335]:1234\r\n\r\n",
					 2),
					"GET", "/example/", "HTTP/1.1", "example.com", {"10.0.0.1", "127.0.0.1", "2001:0db8:85a3::8a2e:0370:7335"}},
			{chunk_string("GET / HTTP/1.1\r\n", 1), "GET", "/", "HTTP/1.1", "", {}, false, false},
			{{"GET /"}, "GET", "/", "", "", {}, false, false},
			{{"", ""}, "", "", "", "", {}, false, false},
	};
	size_t ci = 0;
	for (const ValidCase& c : valid) {
		ebdamd::HttpRequestParser parser;
		size_t total = 0, all = 0;
		for (const std::string& ch : c.chunks) {
			total += parser.parse(ch, c.isHttps ? EBD_FLAG_SESSION_SSL_HTTP : EBD_FLAG_SESSION_UNENCRYPTED_HTTP);
			all += ch.size();
		}
		if (parser.isInvalidState() || total != (c.total ? c.total : all))
			std::fprintf(stderr, "valid case %zu: %zu chunks, total %zu of %zu, host '%s'\n", ci, c.chunks.size(), total, all,
					parser.result.host.c_str());
		ci++;
		CHECK(parser.isFinished() == c.finished);
		CHECK(!parser.isInvalidState());
		CHECK(total == (c.total ? c.total : all));
		CHECK(parser.result.method == c.method);
		CHECK(parser.result.url == c.url);
		CHECK(parser.result.protocol == c.protocol);
		CHECK(parser.result.host == c.host);
		CHECK(parser.result.clientIp == c.clientIp);
		CHECK(parser.result.isHttps == c.isHttps);
	}
	const std::vector<std::pair<std::vector<std::string>, size_t>> invalid = {
			{{"get /example HTTP/1.1\r\nHost: example.com\r\n\r\n"}, 1},
			{{"POST  HTTP/1.1\r\nHost: example.com\r\n\r\n"}, 6},
			{{"GET / HTTP/1.1\r\nHost: \r\n\r\n"}, 23},
			{{"GET / HTTP/1.1 \r\nHost: example.com\r\n\r\n"}, 15},
			{{"GET / HTTP/1.1\nHost: example.con\n\n"}, 15},
			{{"GET /example", "HTTP/1.1\r\nHost: example.com\r\n\r\n"}, 21},
			{{"GET / HTTP/0.0\r\nHost: example.com\r\n\r\n"}, 12},
			{{"GET http://example.com HTTP/1.1\r\nHost: example.com\r\n\r\n"}, 5},
	};
	for (const auto& c : invalid) {
		ebdamd::HttpRequestParser parser;
		size_t total = 0;
		for (const std::string& ch : c.first)
			total += parser.parse(ch, EBD_FLAG_SESSION_UNENCRYPTED_HTTP);
		CHECK(parser.isFinished());
		CHECK(parser.isInvalidState());
		CHECK(total == c.second);
	}
	// reset() keeps result.clientIPKey (HttpRequestParser.cpp:374-379)
	ebdamd::HttpRequestParser parser;
	parser.parse("GET / HTTP/1.1\r\nX-Forwarded-For: 1.2.3.4\r\n\r\n", EBD_FLAG_SESSION_UNENCRYPTED_HTTP);
	CHECK(parser.result.clientIPKey == "x-forwarded-for");
	parser.reset();
	CHECK(parser.result.url.empty() && parser.result.clientIp.empty() && !parser.isFinished());
	parser.parse("GET /b HTTP/1.1\r\nX-Client-IP: 5.6.7.8\r\nX-Forwarded-For: 9.9.9.9\r\n\r\n", EBD_FLAG_SESSION_UNENCRYPTED_HTTP);
	CHECK(parser.isFinished() && !parser.isInvalidState());
	CHECK(parser.result.clientIp == std::vector<std::string>{"9.9.9.9"});
	CHECK(parser.result.clientIPKey == "x-forwarded-for");
	CHECK(!parser.result.clientIpTruncated);
	// more client tokens than EBD_PARSE_MAX_TOKENS: the first ones are listed and the result says so
	{
		std::string many;
		for (int k = 0; k < EBD_PARSE_MAX_TOKENS + 3; k++)
			many += (k ? "," : "") + std::to_string(k + 1) + ".0.0.1";
		ebdamd::HttpRequestParser p;
		p.parse("GET / HTTP/1.1\r\nX-Forwarded-For: " + many + "\r\n\r\n", EBD_FLAG_SESSION_UNENCRYPTED_HTTP);
		CHECK(p.isFinished() && !p.isInvalidState());
		CHECK(p.result.clientIp.size() == EBD_PARSE_MAX_TOKENS);
		CHECK(p.result.clientIp.front() == "1.0.0.1");
		CHECK(p.result.clientIpTruncated);
	}
}

int run_gpu() {
	parser_test_cases();
	// config 1: 1000 x the 35-byte GET, one connection per event
	{
		MemorySource src;
		const std::string req = "GET / HTTP/1.1\r\nHost: 127.0.0.1\r\n\r\n";
		for (uint32_t i = 0; i < 1000; i++)
			src.push(make_event(1000, 5, i + 1, 1, kV4New), &req);
		ebdamd::Options opt;
		opt.maxEvents = 256; // four hand-overs in one poll cycle
		opt.maxPayload = 1 << 20;
		ebdamd::Discovery d(src, false, ebdamd::IpInterfaces{}, opt);
		d.init();
		CHECK(d.fetchAndHandleEvents() == 0);
		const auto svc = d.aggregator().collectServices();
		CHECK(svc.size() == 1);
		if (svc.size() == 1) {
			ebdamd::Service want;
			want.pid = 1000;
			want.endpoint = "127.0.0.1/";
			want.domain = "127.0.0.1";
			want.scheme = "http";
			want.internalClientsNumber = 1000;
			CHECK(svc[0] == want);
			if (!(svc[0] == want))
				std::fprintf(stderr, "got pid %u endpoint '%s' domain '%s' scheme '%s' internal %u external %u\n", svc[0].pid,
						svc[0].endpoint.c_str(), svc[0].domain.c_str(), svc[0].scheme.c_str(), svc[0].internalClientsNumber,
						svc[0].externalClientsNumber);
		}
		std::ostringstream out;
		d.outputServicesToStdout(out);
		CHECK(out.str() == "{\"service\":[{\"pid\":1000,\"endpoint\":\"127.0.0.1/\",\"domain\":\"127.0.0.1\",\"scheme\":\"http\","
						   "\"internalClientsNumber\":1000,\"externalClientsNumber\":0}]}\n");
		CHECK(d.aggregator().collectServices().empty()); // cleared after the report
		std::ostringstream none;
		d.outputServicesToStdout(none);
		CHECK(none.str().empty());
	}
	// the 31-byte variant never finishes: no service, 1000 saved sessions
	{
		MemorySource src;
		const std::string req = "GET / HTTP/1.1\r\nHost: 127.0.0.1";
		for (uint32_t i = 0; i < 1000; i++)
			src.push(make_event(1000, 5, i + 1, 1, kV4New), &req);
		ebdamd::Discovery d(src, false);
		CHECK(d.fetchAndHandleEvents() == 0);
		CHECK(d.aggregator().collectServices().empty());
		CHECK(d.aggregator().stats().live_sessions == 1000);
	}
	// a saved session whose next buffer is invalid: the kernel session is deleted once; a
	// fragmented request across two poll cycles; a missing buffer and a DATA_END event
	{
		MemorySource src;
		const std::string a = "GET /x HTTP/1.1\r\nHo", bad = "st\x01 h\r\n\r\n", f1 = "POST /y HTTP/1.1\r\nHost: ", f2 = "z\r\n\r\n";
		src.push(make_event(7, 9, 1, 1, kV4New), &a);
		src.push(make_event(7, 9, 2, 1, kV4New), &f1);
		src.push(make_event(7, 9, 3, 1, kV4New), nullptr); // saved buffer missing
		ebdamd::Discovery d(src, false);
		CHECK(d.fetchAndHandleEvents() == 0);
		CHECK(src.deleted.empty());
		src.push(make_event(7, 9, 1, 2, kV4New), &bad);
		src.push(make_event(7, 9, 2, 2, kV4New), &f2);
		src.push(make_event(7, 9, 2, 2, EBD_FLAG_EVENT_DATA_END), nullptr);
		CHECK(d.fetchAndHandleEvents() == 0);
		CHECK(src.deleted.size() == 1 && src.deleted[0] == (MemorySource::Key{7, 9, 1, 0}));
		const auto svc = d.aggregator().collectServices();
		CHECK(svc.size() == 1 && svc[0].endpoint == "z/y" && svc[0].internalClientsNumber == 1);
		CHECK(d.aggregator().stats().live_sessions == 0);
	}
	// network counters with the clock overridden (AggregatorMock, AggregatorTest.cpp:41-46)
	{
		ClockedAggregator agg(ebdamd::IpInterfaces{}, true);
		ebdamd::EventBatch b;
		const char* clients[] = {"8.8.8.8", "8.8.9.9", "1.2.3.4", "2001:db8:1::5"};
		std::vector<std::string> bufs;
		for (const char* c : clients)
			bufs.push_back(std::string("GET /n HTTP/1.1\r\nHost: svc\r\nX-Forwarded-For: ") + c + "\r\n\r\n");
		for (uint32_t i = 0; i < bufs.size(); i++)
			b.add(make_event(50, 3, i + 1, 1, kV4New), bufs[i].data(), (uint32_t)bufs[i].size());
		CHECK(agg.newEvents(b) == 0);
		auto svc = agg.collectServices();
		CHECK(svc.size() == 1);
		if (svc.size() == 1) {
			CHECK(svc[0].externalClientsNumber == 4);
			CHECK(svc[0].externalIPv4_16ClientNets == 2 && svc[0].externalIPv4_24ClientNets == 3 &&
					svc[0].externalIPv6ClientsNets == 1);
		}
		agg.now += 59ull * 60 * 1000000000ull;
		agg.networkCountersCleaning();
		CHECK(agg.collectServices()[0].externalIPv4_24ClientNets == 3);
		agg.now += 60ull * 1000000000ull;
		agg.networkCountersCleaning();
		svc = agg.collectServices();
		CHECK(svc.size() == 1 && svc[0].externalIPv4_16ClientNets == 0 && svc[0].externalIPv6ClientsNets == 0);
		agg.clear();
		CHECK(agg.collectServices().empty());
		CHECK(agg.stats().errors == 0);
	}
	aggregator_test_scenarios();
	return 0;
}

} // namespace

int main(int argc, char** argv) {
	const std::string mode = argc > 1 ? argv[1] : "cpu";
	try {
		if (mode == "gpu")
			run_gpu();
		else if (mode == "parser-repeat") // the parser cases many times in one process
			for (int k = 0; k < (argc > 2 ? std::atoi(argv[2]) : 100); k++)
				parser_test_cases();
		else
			run_cpu();
	} catch (const std::exception& e) {
		std::fprintf(stderr, "exception: %s\n", e.what());
		return 2;
	}
	if (failures) {
		std::fprintf(stderr, "%d checks failed\n", failures);
		return 1;
	}
	std::printf("ok\n");
	return 0;
}
