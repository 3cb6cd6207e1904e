// ebd_dfa.cpp — host-side construction of the key trie and the fast-path DFA.
#include "ebd_dfa.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <string>
#include <tuple>
#include <vector>

namespace ebd {

// HttpRequestParser.cpp:40,43 — "host" and the client-IP header keys, in list order.
static const char* kKeys[6] = {"host", "rproxy_remote_address", "true-client-ip", "x-client-ip", "x-forwarded-for",
		"x-http-client-ip"};

void build_key_trie(KeyTrie* t) {
	std::memset(t, 0, sizeof(*t));
	std::map<std::string, int> id;
	std::vector<std::string> name;
	id[""] = kTrieRoot;
	name.push_back("");
	id["\001" "dead"] = kTrieDead;
	name.push_back("\001" "dead");
	for (int k = 0; k < 6; k++) {
		std::string s = kKeys[k];
		for (size_t i = 1; i <= s.size(); i++) {
			std::string p = s.substr(0, i);
			if (!id.count(p)) {
				id[p] = (int)name.size();
				name.push_back(p);
			}
		}
	}
	t->nodes = (uint8_t)name.size();
	for (int c = 0; c < 256; c++)
		t->cls[c] = byte_class((uint32_t)c);
	for (int n = 0; n < (int)name.size(); n++) {
		t->type[n] = KT_OTHER;
		for (int k = 0; k < 6; k++)
			if (name[n] == kKeys[k])
				t->type[n] = k == 0 ? KT_HOST : (uint8_t)(KT_CLIENT0 + (k - 1));
		for (int c = 0; c < 128; c++) {
			if (n == kTrieDead) {
				t->next[n][c] = kTrieDead;
				continue;
			}
			// P:283-285: the byte is appended only while the key is shorter than 21
			std::string s = name[n].size() < kMaxHeaderKeyLength ? name[n] + (char)c : name[n];
			auto it = id.find(s);
			t->next[n][c] = it == id.end() ? kTrieDead : (uint8_t)it->second;
		}
	}
}

namespace {

// Projection of GenParser onto what decides a fresh parser's future transitions.
struct AState {
	uint8_t state, mcand, mlen, plen, key, kt, host;
	bool operator<(const AState& o) const {
		return std::tie(state, mcand, mlen, plen, key, kt, host) < std::tie(o.state, o.mcand, o.mlen, o.plen, o.key, o.kt, o.host);
	}
	bool operator==(const AState& o) const { return !(*this < o) && !(o < *this); }
};

uint8_t node_of(const KeyTrie* t, uint8_t kt_wanted) {
	for (int n = 0; n < t->nodes; n++)
		if (t->type[n] == kt_wanted)
			return (uint8_t)n;
	return kTrieRoot;
}

AState project(const KeyTrie* t, const GenParser& g) {
	AState a{};
	a.state = g.state;
	const uint8_t host = (g.f & GPF_HOST) ? 1 : 0;
	switch (g.state) {
	case ST_METHOD:
		a.mcand = g.mcand;
		a.mlen = g.mlen;
		break;
	case ST_PROTO:
		a.plen = g.plen;
		break;
	case ST_HDR_KEY:
		a.key = g.key;
		a.host = host;
		break;
	case ST_SP_VAL:
	case ST_HDR_VAL: {
		uint8_t kt = t->type[g.key];
		a.kt = kt >= KT_CLIENT0 ? (uint8_t)KT_CLIENT0 : kt;
		a.host = host;
		break;
	}
	case ST_HDR_NL:
	case ST_HDRS_END:
	case ST_FINISHED:
		a.host = host;
		break;
	default:
		break;
	}
	return a;
}

// A concrete parser for an abstract state; `variant` picks among the client keys so
// the builder can check that the projection is consistent.
GenParser represent(const KeyTrie* t, const AState& a, int variant) {
	GenParser g;
	gp_init(g);
	g.state = a.state;
	g.mcand = a.mcand;
	g.mlen = a.mlen;
	g.plen = a.plen;
	if (a.state == ST_PROTO && a.plen == 8)
		g.pminor = (variant & 1) ? '1' : '0';
	g.key = a.key;
	if (a.host)
		g.f |= GPF_HOST;
	if (a.state == ST_SP_VAL || a.state == ST_HDR_VAL) {
		g.key = a.kt == KT_CLIENT0 ? node_of(t, (uint8_t)(KT_CLIENT0 + (variant % 5))) : node_of(t, a.kt);
		if (a.kt == KT_OTHER)
			g.key = kTrieDead;
	}
	if (variant & 2)
		g.cipkey = (uint8_t)(1 + (variant % 5));
	if (variant & 4)
		g.f |= GPF_CIP_FOUND;
	return g;
}

} // namespace

void build_lds_image(const DfaTable* t, uint8_t* out) {
	std::memset(out, 0, kLdsTableBytes);
	for (uint32_t st = 0; st < kLdsRows; st++)
		for (uint32_t b = 0; b < kLdsCols; b++)
			out[b * kLdsStride + st] = t->next[st * 256 + b];
}

int build_dfa(const KeyTrie* trie, DfaTable* out) {
	std::map<AState, int> ids;
	std::vector<AState> states;
	GenParser g0;
	gp_init(g0);
	AState a0 = project(trie, g0);
	ids[a0] = 0;
	states.push_back(a0);
	std::vector<std::vector<int>> trans;
	for (size_t i = 0; i < states.size(); i++) {
		std::vector<int> row(256);
		for (int b = 0; b < 256; b++) {
			AState nx{};
			for (int variant = 0; variant < 8; variant++) {
				GenParser g = represent(trie, states[i], variant);
				gp_step(g, trie, (uint32_t)b, 100);
				AState p = project(trie, g);
				if (variant == 0)
					nx = p;
				else if (!(p == nx))
					return -1; // projection inconsistent: the DFA would diverge from gp_step
			}
			auto it = ids.find(nx);
			if (it == ids.end()) {
				it = ids.emplace(nx, (int)states.size()).first;
				states.push_back(nx);
			}
			row[b] = it->second;
		}
		trans.push_back(row);
	}
	const int n = (int)states.size();
	if (n > 256)
		return -2;

	// Lay the states out in phase groups.
	auto group = [&](const AState& a) -> int {
		switch (a.state) {
		case ST_METHOD:
		case ST_SP_URL:
		case ST_URL:
			return 0;
		case ST_SP_PROTO:
		case ST_PROTO:
			return 1;
		case ST_FINISHED:
		case ST_INVALID:
			return 4;
		default:
			return a.host ? 3 : 2;
		}
	};
	auto rank = [&](const AState& a) -> int { // order inside a group
		const bool hvc = a.state == ST_HDR_VAL && a.kt == KT_CLIENT0;
		switch (group(a)) {
		case 0:
			return a.state == ST_URL ? 2 : (a.state == ST_SP_URL ? 1 : 0);
		case 2:
			return hvc ? 1 : 0;
		case 3:
			return hvc ? 0 : 1;
		case 4:
			return a.state == ST_INVALID ? 2 : a.host;
		default:
			return 0;
		}
	};
	std::vector<int> order(n);
	for (int i = 0; i < n; i++)
		order[i] = i;
	std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
		int gx = group(states[x]), gy = group(states[y]);
		if (gx != gy)
			return gx < gy;
		return rank(states[x]) < rank(states[y]);
	});
	// HV(client) states leave their groups for the two ids after the terminal states, so
	// that "s >= hvc0" (one compare) tells a client-IP value state
	std::vector<int> newid(n, -1);
	int next_id = 0, hvc_seen = 0, hvc_idx[2] = {-1, -1};
	for (int i = 0; i < n; i++) {
		const AState& a = states[order[i]];
		if (a.state == ST_HDR_VAL && a.kt == KT_CLIENT0) {
			hvc_idx[a.host ? 1 : 0] = order[i];
			hvc_seen++;
		} else {
			newid[order[i]] = next_id++;
		}
	}
	if (hvc_seen != 2 || hvc_idx[0] < 0 || hvc_idx[1] < 0 || next_id + 2 > (int)kLdsRows)
		return -2;
	const int hvc_base = next_id;
	newid[hvc_idx[0]] = hvc_base;
	newid[hvc_idx[1]] = hvc_base + 1;
	if (newid[0] != 0)
		return -7; // the reset state must be id 0 (GenParser::ds after gp_init / gp_reset)

	std::memset(out, 0, sizeof(*out));
	for (int st = 0; st < 256; st++)
		out->attr[st] = kKcKeep;
	for (int i = 0; i < n; i++)
		if (states[i].state == ST_HDR_KEY)
			out->attr[newid[i]] = key_client_id(trie->type[states[i].key]);
	DfaInfo& in = out->info;
	in.nstates = (uint32_t)hvc_base + 2;
	in.init = (uint32_t)newid[0];
	in.url_id = in.g2 = in.g3 = in.g4 = in.hvh = in.fin0 = in.fin1 = in.inv = 0xffffffffu;
	in.hvc0 = (uint32_t)hvc_base;
	in.hvc1 = (uint32_t)hvc_base + 1;
	for (int i = 0; i < n; i++) {
		const AState& a = states[i];
		const uint32_t id = (uint32_t)newid[i];
		if (id >= in.hvc0)
			continue;
		if (a.state == ST_URL)
			in.url_id = id;
		if (a.state == ST_HDR_VAL && a.kt == KT_HOST && a.host)
			in.hvh = id;
		if (a.state == ST_FINISHED)
			(a.host ? in.fin1 : in.fin0) = id;
		if (a.state == ST_INVALID)
			in.inv = id;
	}
	uint32_t first[5] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
	for (int i = 0; i < n; i++) {
		const uint32_t id = (uint32_t)newid[i];
		if (id >= in.hvc0)
			continue;
		const int g = group(states[i]);
		if (id < first[g])
			first[g] = id;
	}
	in.g2 = first[2];
	in.g3 = first[3];
	in.g4 = first[4];
	if (in.url_id + 1 != first[1] || in.fin0 != in.g4 || in.fin1 != in.g4 + 1 || in.inv != in.g4 + 2 ||
			(uint32_t)next_id != in.g4 + 3 || in.hvh == 0xffffffffu)
		return -3;
	auto group_of_id = [&](int i) {
		const AState& a = states[i];
		return group(a);
	};
	for (int row = 0; row < 256; row++)
		for (int b = 0; b < 256; b++)
			out->next[row * 256 + b] = (uint8_t)in.inv; // unreachable rows
	for (int i = 0; i < n; i++) {
		const int gi = group_of_id(i);
		for (int b = 0; b < 256; b++) {
			const int j = trans[i][b];
			if (group_of_id(j) < gi)
				return -5;
			out->next[newid[i] * 256 + b] = (uint8_t)newid[j];
		}
	}
	// the (at most two) non-terminal states that step to themselves on every byte of
	// [0x20, 0x7e]: the kernel skips such 4-byte words without table reads (k_fresh scan_chunk)
	in.vl0 = in.vl1 = 0xffffffffu;
	int nvl = 0;
	for (uint32_t st = 0; st < in.nstates; st++) {
		if (st - in.g4 < 3u)
			continue;
		bool loop = true;
		for (int b = 0x20; b <= 0x7e; b++)
			loop &= out->next[st * 256 + b] == st;
		if (!loop)
			continue;
		if (nvl == 0)
			in.vl0 = st;
		else if (nvl == 1)
			in.vl1 = st;
		nvl++;
	}
	if (nvl > 2)
		return -6;
	for (uint32_t st = 0; st < 256; st++) // the LDS image's 128 columns (ebd_dfa.h kLdsCols)
		for (uint32_t b = 128; b < 256; b++)
			if (out->next[st * 256 + b] != out->next[st * 256 + 127])
				return -8;
	for (uint32_t st = 0; st < 256; st++) {
		uint32_t a = out->attr[st];
		a |= st == in.url_id ? A_URL : 0u;
		a |= st == in.hvh ? A_HVH : 0u;
		a |= st >= in.hvc0 && st < in.nstates ? A_HVC : 0u;
		a |= st - in.g4 < 3u ? A_TERM : 0u;
		out->attr[st] = (uint8_t)a;
	}
	return 0;
}

} // namespace ebd
