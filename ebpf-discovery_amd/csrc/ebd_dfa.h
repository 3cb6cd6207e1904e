// ebd_dfa.h — fast-path DFA for single-buffer (fresh-parser) events.
//
// The table is not written by hand: ebd_build_dfa() enumerates, by breadth-first
// search, every state the generic parser (ebd_spec.h gp_step, the restatement of
// HttpRequestParser.cpp:124-364) can reach from reset, projected onto what decides
// future transitions of a fresh parser, and records the projected transition for
// every byte value.  State ids are then laid out in "phase groups" so the kernel can
// recover spans with counters:
//   G0 [0, url_id]        METHOD progress, SPACE_BEFORE_URL, URL (url_id last)
//   G1 (url_id, g2)       SPACE_BEFORE_PROTOCOL, PROTOCOL progress
//   G2 [g2, g3)           header section, Host not seen yet; HV(client) last (= hvc0)
//   G3 [g3, g4)           header section, Host seen; HV(client) first (= g3), HV(host) = hvh
//   G4 [g4, nstates)      FINISHED (no host), FINISHED (host), INVALID
// Transitions never go to a lower group.
#pragma once

#include "ebd_spec.h"

namespace ebd {

struct DfaInfo {
	uint32_t nstates;
	uint32_t url_id, g2, g3, g4;
	uint32_t hvc0, hvh;            // HV(client, no host) = g3 - 1, HV(host) in G3
	uint32_t fin0, fin1, inv;
	uint32_t init;                 // reset state (METHOD, empty)
};

struct DfaTable {
	DfaInfo info;
	uint8_t next[256 * 256]; // next[s * 256 + byte]
};

void build_key_trie(KeyTrie* t);
// Returns 0, or a negative value when an internal consistency check fails.
int build_dfa(const KeyTrie* trie, DfaTable* out);

} // namespace ebd
