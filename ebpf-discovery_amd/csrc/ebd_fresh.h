// ebd_fresh.h — fast path for one event parsed by a fresh parser (Discovery.cpp:141-159
// handleNewSession), written once for the GPU kernel and its host emulation.
//
// The byte scan runs the projected DFA (ebd_dfa.h) and recovers the spans with
// counters that rely on the phase-group layout of the state ids:
//   c_url  = bytes processed in G0 (METHOD .. URL)      -> url end   = c_url - 1
//   c_pre  = bytes processed before Host was seen       -> host start = c_pre - 1
//   c_hv   = bytes processed in HV(host)                -> host length
//   c_cons = bytes processed before FINISHED / INVALID  -> parse() return value
//   cip    = first position whose next state is HV(client) -> first client-IP value byte
#pragma once

#include "../../include/ebpf_discovery_amd.h"
#include "ebd_dfa.h"
#include "ebd_spec.h"

namespace ebd {

struct FreshScan {
	uint32_t s, c_url, c_pre, c_hv, c_cons, cip;
};

// One byte of the scan.  `v` = the byte belongs to the buffer.
template <typename Tab>
EBD_HD void fresh_byte(const Tab& T, const DfaInfo& di, FreshScan& f, uint32_t b, int pos, bool v) {
	const uint32_t s = f.s;
	const uint32_t sn = T[(s << 8) | b];
	f.c_url += (v && s <= di.url_id);
	f.c_pre += (v && s < di.g3);
	f.c_hv += (v && s == di.hvh);
	f.c_cons += (v && s < di.g4);
	f.cip = (v && (sn - di.hvc0) < 2u && (uint32_t)pos < f.cip) ? (uint32_t)pos : f.cip;
	f.s = v ? sn : s;
}

EBD_HD void fresh_init(const DfaInfo& di, FreshScan& f) {
	f.s = di.init;
	f.c_url = f.c_pre = f.c_hv = f.c_cons = 0;
	f.cip = 0xffffffffu;
}

// Host emulation of the scan: byte at a time.
template <typename Tab>
inline void fresh_scan_bytes(const Tab& T, const DfaInfo& di, const uint8_t* p, uint32_t L, FreshScan& f) {
	fresh_init(di, f);
	for (uint32_t k = 0; k < L; k++) {
		fresh_byte(T, di, f, p[k], (int)k, true);
		if (f.s >= di.g4)
			break;
	}
}

struct FreshResult {
	ebd_event_result r;
	Hash128 key;
};

// Turns a finished scan into the per-event result, the client class and the service key.
// pid / flags / src come from the DiscoveryEvent (Discovery.cpp:136, 157).
EBD_HD void fresh_finalize(const DfaInfo& di, const FreshScan& f, const uint8_t* p, uint32_t pid, uint8_t flags,
		const uint8_t* src, const Interfaces& ifs, FreshResult& out) {
	ebd_event_result& r = out.r;
	r.consumed = (uint16_t)f.c_cons;
	r.info = 0;
	r.u.span.url_off = r.u.span.url_len = r.u.span.host_off = r.u.span.host_len = r.u.span.cip_off = r.u.span.cip_len = 0;
	out.key.lo = out.key.hi = 0;
	if (f.s == di.inv) {
		r.status = EBD_STATUS_INVALID;
		return;
	}
	if (f.s != di.fin0 && f.s != di.fin1) {
		r.status = EBD_STATUS_UNFINISHED;
		return;
	}
	r.status = EBD_STATUS_FINISHED;
	const bool post = p[0] == 'P';
	const uint32_t url_start = post ? 5 : 4;
	const uint32_t url_len = f.c_url - 1 - url_start;
	uint32_t host_start = 0, host_len = 0;
	if (f.s == di.fin1) {
		host_start = f.c_pre - 1;
		host_len = f.c_hv;
	}
	uint8_t info = (uint8_t)((post ? EBD_INFO_POST : 0) | ((flags & 16) ? EBD_INFO_HTTPS : 0));
	uint8_t cls;
	if (f.cip != 0xffffffffu) {
		// first token of the first client-IP header value: up to ',' or the value's CR
		uint32_t e = f.cip;
		while (e < f.c_cons && p[e] != ',' && p[e] != '\r')
			e++;
		uint32_t tb, te;
		front_token(p + f.cip, e - f.cip, &tb, &te);
		r.u.span.cip_off = (uint16_t)(f.cip + tb);
		r.u.span.cip_len = (uint16_t)(te - tb);
		info |= EBD_INFO_CIP;
		cls = classify_token(ifs, p + f.cip + tb, te - tb);
	} else {
		cls = classify_source(ifs, flags, src);
	}
	info |= (uint8_t)(cls << EBD_INFO_CLASS_SHIFT);
	r.info = info;
	r.u.span.url_off = (uint16_t)url_start;
	r.u.span.url_len = (uint16_t)url_len;
	r.u.span.host_off = (uint16_t)host_start;
	r.u.span.host_len = (uint16_t)host_len;
	KeyHasher kh;
	kh.init(pid);
	kh.bytes(p + host_start, host_len);
	kh.bytes(p + url_start, url_len);
	out.key = kh.finish();
}

} // namespace ebd
