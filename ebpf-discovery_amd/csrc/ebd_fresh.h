// ebd_fresh.h — fast path for one event parsed by a fresh parser (Discovery.cpp:141-159
// handleNewSession), written once for the GPU kernel and its host emulation.
//
// The byte scan runs the projected DFA (ebd_dfa.h) over the buffer in 16-byte chunks.
// Per byte it only does the table step and notes whether the next state is a client-IP
// value state (ids 254 / 255).  Per chunk it records the FIRST chunk in which
//   url  : the state left the request-line-up-to-URL group  (URL end)
//   host : the state entered the Host-seen world             (first Host value byte)
//   term : the state became FINISHED / INVALID               (parse() return value)
//   cip  : some byte's next state was a client-IP value       (first client-IP value byte)
// together with the state at that chunk's start.  The phases are monotone (ebd_dfa.h),
// so finalize recovers every exact position by re-running the DFA over one recorded
// chunk (16 bytes).
#pragma once

#include "../../include/ebpf_discovery_amd.h"
#include "ebd_dfa.h"
#include "ebd_spec.h"

namespace ebd {

constexpr uint32_t kNone = 0xffffffffu;

struct ScanRec {
	uint32_t url, host, term, cip; // (chunk << 8) | state at the chunk's start, kNone if not seen
};

EBD_HD void rec_init(ScanRec& r) { r.url = r.host = r.term = r.cip = kNone; }
EBD_HD bool st_terminal(const DfaInfo& di, uint32_t s) { return s - di.g4 < 3u; }
EBD_HD bool st_host_seen(const DfaInfo& di, uint32_t s) {
	return (s - di.g3 < di.g4 - di.g3) || s == di.fin1 || s == di.hvc1;
}

// After chunk c (started in s0, ended in s1; hit = a byte's next state was >= 254).
// Returns true once the parse reached a terminal state.
EBD_HD bool chunk_track(const DfaInfo& di, ScanRec& r, uint32_t c, uint32_t s0, uint32_t s1, bool hit) {
	const uint32_t rec = (c << 8) | s0;
	if (r.url == kNone && s1 > di.url_id)
		r.url = rec;
	if (r.host == kNone && st_host_seen(di, s1))
		r.host = rec;
	if (r.cip == kNone && hit)
		r.cip = rec;
	if (st_terminal(di, s1)) {
		r.term = rec;
		return true;
	}
	return false;
}

// Host emulation of the device scan: identical chunking (skip = buffer address mod 16).
template <typename Tab>
inline uint32_t fresh_scan_host(const Tab& T, const DfaInfo& di, const uint8_t* p, uint32_t skip, uint32_t L, ScanRec& r) {
	rec_init(r);
	uint32_t s = di.init;
	const uint32_t nch = (skip + L + 15) / 16;
	for (uint32_t c = 0; c < nch; c++) {
		const uint32_t s0 = s;
		bool hit = false;
		for (uint32_t k = 0; k < 16; k++) {
			const int pos = (int)(c * 16 + k) - (int)skip;
			if (pos < 0 || (uint32_t)pos >= L)
				continue;
			s = T[(s << 8) | p[pos]];
			hit |= s >= 254;
		}
		if (chunk_track(di, r, c, s0, s, hit))
			break;
	}
	return s;
}

enum { RS_URL, RS_HOST, RS_TERM, RS_CIP };

// First position inside the recorded chunk where the crossing `what` happens.
template <typename Tab>
EBD_HD uint32_t rescan(const Tab& T, const DfaInfo& di, uint32_t rec, const uint8_t* p, uint32_t skip, uint32_t L, int what) {
	const uint32_t c = rec >> 8;
	uint32_t s = rec & 0xffu;
	for (uint32_t k = 0; k < 16; k++) {
		const int pos = (int)(c * 16 + k) - (int)skip;
		if (pos < 0 || (uint32_t)pos >= L)
			continue;
		const uint32_t sn = T[(s << 8) | p[pos]];
		bool hit;
		switch (what) {
		case RS_URL: hit = s <= di.url_id && sn > di.url_id; break;
		case RS_HOST: hit = !st_host_seen(di, s) && st_host_seen(di, sn); break;
		case RS_TERM: hit = st_terminal(di, sn); break;
		default: hit = sn >= 254; break;
		}
		if (hit)
			return (uint32_t)pos;
		s = sn;
	}
	return kNone;
}

struct FreshResult {
	ebd_event_result r;
	Hash128 key;
};

// Turns a scan into the per-event result, the client class and the service key.
// pid / flags / src come from the DiscoveryEvent (Discovery.cpp:136, 157).
template <typename Tab>
EBD_HD void fresh_finalize(const Tab& T, const DfaInfo& di, const ScanRec& sr, uint32_t s_final, const uint8_t* p,
		uint32_t skip, uint32_t L, uint32_t pid, uint8_t flags, const uint8_t* src, const Interfaces& ifs, FreshResult& out) {
	ebd_event_result& r = out.r;
	r.info = 0;
	r.u.span.url_off = r.u.span.url_len = r.u.span.host_off = r.u.span.host_len = r.u.span.cip_off = r.u.span.cip_len = 0;
	out.key.lo = out.key.hi = 0;
	if (!st_terminal(di, s_final)) {
		r.status = EBD_STATUS_UNFINISHED;
		r.consumed = (uint16_t)L;
		return;
	}
	const uint32_t consumed = rescan(T, di, sr.term, p, skip, L, RS_TERM) + 1;
	r.consumed = (uint16_t)consumed;
	if (s_final == di.inv) {
		r.status = EBD_STATUS_INVALID;
		return;
	}
	r.status = EBD_STATUS_FINISHED;
	const bool post = p[0] == 'P';
	const uint32_t url_start = post ? 5 : 4;
	const uint32_t url_len = rescan(T, di, sr.url, p, skip, L, RS_URL) - url_start;
	uint32_t host_start = 0, host_len = 0;
	if (s_final == di.fin1) {
		host_start = rescan(T, di, sr.host, p, skip, L, RS_HOST);
		uint32_t e = host_start;
		while (e < consumed && p[e] != '\r') // Host value bytes are H-class: no CR inside
			e++;
		host_len = e - host_start;
	}
	uint8_t info = (uint8_t)((post ? EBD_INFO_POST : 0) | ((flags & 16) ? EBD_INFO_HTTPS : 0));
	uint8_t cls;
	if (sr.cip != kNone) {
		// first token of the first client-IP header value: up to ',' or the value's CR
		const uint32_t cip = rescan(T, di, sr.cip, p, skip, L, RS_CIP);
		uint32_t e = cip;
		while (e < consumed && p[e] != ',' && p[e] != '\r')
			e++;
		uint32_t tb, te;
		front_token(p + cip, e - cip, &tb, &te);
		r.u.span.cip_off = (uint16_t)(cip + tb);
		r.u.span.cip_len = (uint16_t)(te - tb);
		info |= EBD_INFO_CIP;
		cls = classify_token(ifs, p + cip + tb, te - tb);
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
