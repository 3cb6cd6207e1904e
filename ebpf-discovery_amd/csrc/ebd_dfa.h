// ebd_dfa.h — fast-path DFA for single-buffer (fresh-parser) events.
//
// The table is not written by hand: ebd_build_dfa() enumerates, by breadth-first
// search, every state the generic parser (ebd_spec.h gp_step, the restatement of
// HttpRequestParser.cpp:124-364) can reach from reset, projected onto what decides
// future transitions of a fresh parser, and records the projected transition for
// every byte value.  State ids are then laid out in "phase groups" (see DESIGN.md):
//   G0 [0, url_id]        METHOD progress, SPACE_BEFORE_URL, URL (url_id last)
//   G1 (url_id, g2)       SPACE_BEFORE_PROTOCOL, PROTOCOL progress
//   G2 [g2, g3)           header section, Host not seen yet
//   G3 [g3, g4)           header section, Host seen; HV(host) = hvh
//   G4 = [g4, g4 + 3)     FINISHED (no host), FINISHED (host), INVALID
//   hvc0 = g4 + 3, hvc1   HV(client) without / with Host seen: one compare (s >= hvc0)
//                         tells "inside a client-IP header value"; they are the last ids
// Rows past the used ids are unreachable (filled with INVALID).
// Phases are monotone: the group of the state never decreases (HV(client) counts as the
// header group of its world), which lets the kernel find every span from per-chunk
// crossings and a 16-byte rescan.
#pragma once

#include "ebd_spec.h"

namespace ebd {

struct DfaInfo {
	uint32_t nstates;
	uint32_t url_id, g2, g3, g4;
	uint32_t hvc0, hvh;            // HV(client, no host) = g4 + 3, HV(host) in G3
	uint32_t hvc1;                 // HV(client, host seen) = hvc0 + 1 = nstates - 1
	uint32_t fin0, fin1, inv;
	uint32_t init;                 // reset state (METHOD, empty)
	uint32_t vl0, vl1;             // generic header-value states: self-loops on [0x20, 0x7e] (or ~0)
};

struct DfaTable {
	DfaInfo info;
	uint8_t next[256 * 256]; // next[s * 256 + byte]
	// per state, for the session path's walker (dfa_parse, ebd_fresh.h): bits 0-2 the client-IP
	// id (0 none, 1..5) of the header key a HEADER_KEY state has read so far (its trie node),
	// kKcKeep for every other state; then one bit per span boundary the walker records
	uint8_t attr[256];
};
constexpr uint8_t kKcKeep = 7;
enum : uint32_t { A_URL = 8, A_HVH = 16, A_HVC = 32, A_TERM = 64 }; // s == url_id, s == hvh, s >= hvc0, terminal

// The table as the kernel keeps it in LDS: byte-major, entry (s, b) at b * kLdsStride + s.
// A step's address is then one v_mad_u32_u24(b, kLdsStride, s) on the byte as loaded, with
// no per-byte remapping.  kLdsStride = 196 bytes = 49 dwords, an odd count, so the bank of
// (s, b) is (17 b + s / 4) mod 32: lanes reading different bytes in one state spread over the
// banks, and so do lanes in different states on one byte.
constexpr uint32_t kLdsStride = 196;
constexpr uint32_t kLdsRows = kLdsStride; // >= nstates (ebd_build_dfa checks)
// Every byte >= 0x80 steps like 0x7f in every state (no class of the parser holds one;
// build_dfa checks), so the image keeps 128 columns and a step reads column min(b, 127):
// 25 KB of LDS instead of 50 KB, which k_fresh spends on a wider finalize staging.
constexpr uint32_t kLdsCols = 128;
constexpr uint32_t kLdsTableBytes = kLdsCols * kLdsStride;
void build_lds_image(const DfaTable* t, uint8_t* out); // out: kLdsTableBytes

void build_key_trie(KeyTrie* t);
// Returns 0, or a negative value when an internal consistency check fails.
int build_dfa(const KeyTrie* trie, DfaTable* out);

} // namespace ebd
