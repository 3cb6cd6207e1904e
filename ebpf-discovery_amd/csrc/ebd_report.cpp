// ebd_report.cpp — the service report text of Discovery::outputServicesToStdout
// (libebpfdiscovery/src/Discovery.cpp:60-71), byte for byte:
//
//   {"service": boost::json::value_from(services)}  printed by boost::json::ext::print
//   (libebpfdiscovery/headers/ebpfdiscovery/Json.h:32-71), then std::endl.
//
// What that printer does with a Service (libservice/headers/service/Service.h:43-98):
//   * fields in BOOST_DESCRIBE_STRUCT order: pid, endpoint, domain, scheme,
//     internalClientsNumber, externalClientsNumber, externalIPv4_16ClientNets,
//     externalIPv4_24ClientNets, externalIPv6ClientsNets;
//   * a null value (an empty network map, Service.h:84-98) or an empty string is skipped,
//     but "," is written before every field that is not the object's first, skipped or not
//     (Json.h:38-46) — pid, a number, is always first and never skipped, so the quirk cannot
//     show in a service object;
//   * a non-empty map prints as its size; numbers in decimal;
//   * strings through boost::json::serialize (boost 1.83): '"' and '\\' escaped, \b \t \n \f \r
//     by name, other bytes below 0x20 as \u00xx (lower-case hex), every other byte as is.
// No services: nothing is printed at all (Discovery.cpp:62-64).
#include <cerrno>
#include <cstdint>
#include <cstring>
#include <string>

#include "../../include/ebpf_discovery_amd.h"

namespace {

void put_string(std::string& o, const char* p, size_t n) {
	static const char hx[] = "0123456789abcdef";
	o.push_back('"');
	for (size_t k = 0; k < n; k++) {
		const unsigned char ch = (unsigned char)p[k];
		switch (ch) {
		case '"': o += "\\\""; break;
		case '\\': o += "\\\\"; break;
		case '\b': o += "\\b"; break;
		case '\t': o += "\\t"; break;
		case '\n': o += "\\n"; break;
		case '\f': o += "\\f"; break;
		case '\r': o += "\\r"; break;
		default:
			if (ch < 0x20) {
				o += "\\u00";
				o.push_back(hx[ch >> 4]);
				o.push_back(hx[ch & 15]);
			} else {
				o.push_back((char)ch);
			}
		}
	}
	o.push_back('"');
}

// One object member: skipped when `present` is false, "," before all but the first member.
struct Members {
	std::string& o;
	bool first = true;
	void key(const char* k) {
		if (!first)
			o.push_back(',');
		first = false;
		put_string(o, k, std::strlen(k));
		o.push_back(':');
	}
	void num(const char* k, uint64_t v, bool present = true) {
		if (!present) { // Json.h:40-42: skipped, yet it counts as "not the first" (it != obj.begin())
			first = false;
			return;
		}
		key(k);
		o += std::to_string(v);
	}
	void str(const char* k, const char* p, size_t n) {
		if (n == 0) {
			first = false;
			return;
		}
		key(k);
		put_string(o, p, n);
	}
};

} // namespace

extern "C" int ebd_format_services_json(const ebd_service* s, uint32_t n, const char* strings, uint64_t strings_len, char* out,
		uint64_t cap, uint64_t* len) {
	if (!len || (n && !s))
		return -EINVAL;
	std::string o;
	if (n) {
		o += "{\"service\":[";
		for (uint32_t i = 0; i < n; i++) {
			const ebd_service& v = s[i];
			const bool have_ep = strings && v.endpoint_off != ~0ull && v.endpoint_off + v.endpoint_len <= strings_len;
			const char* ep = have_ep ? strings + v.endpoint_off : "";
			const uint32_t el = have_ep ? v.endpoint_len : 0;
			const uint32_t dl = have_ep && v.domain_off + v.domain_len <= el ? v.domain_len : 0;
			if (i)
				o.push_back(',');
			o.push_back('{');
			Members m{o};
			m.num("pid", v.pid);
			m.str("endpoint", ep, el);
			m.str("domain", ep + (dl ? v.domain_off : 0), dl);
			if (v.https <= 1)
				m.str("scheme", v.https ? "https" : "http", v.https ? 5 : 4);
			else // EBD_SCHEME_NONE: a Service built without one (JsonTest.cpp:60-62), "" is skipped
				m.str("scheme", "", 0);
			m.num("internalClientsNumber", v.internal_clients);
			m.num("externalClientsNumber", v.external_clients);
			m.num("externalIPv4_16ClientNets", v.nets_v4_16, v.nets_v4_16 != 0);
			m.num("externalIPv4_24ClientNets", v.nets_v4_24, v.nets_v4_24 != 0);
			m.num("externalIPv6ClientsNets", v.nets_v6, v.nets_v6 != 0);
			o.push_back('}');
		}
		o += "]}\n"; // std::endl
	}
	*len = o.size();
	if (!out)
		return 0;
	if (cap < o.size())
		return -ENOSPC;
	std::memcpy(out, o.data(), o.size());
	return 0;
}
