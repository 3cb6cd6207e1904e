"""The C-ABI library loads and exports every function include/*.h declares (CPU only:
no compute call needs a GPU here)."""
import ctypes as C
import os
import re

import pytest

import ebd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in ("ebpf_discovery_amd.h", "ebpf_discovery_amd_testing.h"):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[\w\s\*]+?\b(ebd_\w+)\s*\(", text, flags=re.M):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    L = ebd.lib()
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in sorted(names) if not hasattr(L, n)]
    assert not missing, missing
    # and the Python binding types every one of them
    assert names <= set(ebd._SIGS), sorted(names - set(ebd._SIGS))


def test_struct_layouts_match_header():
    assert ebd.EVENT_DTYPE.itemsize == 36          # DiscoveryEvent, Types.h:201-205
    assert ebd.RESULT_DTYPE.itemsize == 16
    assert ebd.SESSION_REQ_DTYPE.itemsize == 32
    assert ebd.SERVICE_DTYPE.itemsize == 80
    assert C.sizeof(ebd.Config) == 64  # static_assert in ebd_api.hip
    assert C.sizeof(ebd.Stats) == 104


def test_strerror():
    assert ebd.lib().ebd_strerror(0) == b"success"
    assert ebd.lib().ebd_strerror(-22) == b"invalid argument"


def test_ctx_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(ebd.EbdError):
        ebd.Context(max_events=16)


def test_ctx_create_rejects_an_lru_beyond_the_emission_record():
    """A carried request's index travels in 24 bits of k_emit's record: ebd_ctx_create refuses
    lru_capacity >= 2^24 with -EINVAL before it looks for a device (so this runs on CPU too)."""
    cfg = ebd.Config()
    cfg.max_events = 16
    cfg.lru_capacity = 1 << 24
    h = C.c_void_p()
    assert ebd.lib().ebd_ctx_create(C.byref(cfg), C.byref(h)) == -22
    assert not h.value


def test_parser_state_init_and_reset_keep_the_client_ip_key():
    """ebd_parser_init / ebd_parser_reset are host-only (HttpRequestParser.cpp:82-83, 374-379):
    reset returns the state machine to METHOD with nothing parsed, and keeps clientIPKey."""
    import numpy as np
    import ebd
    st = np.zeros(320, np.uint8)
    assert ebd.lib().ebd_parser_init(ebd._p(st)) == 0
    assert st[6] == 0 and st[12:16].view(np.uint32)[0] == 0  # cipkey, length
    init_state = int(st[0])
    st[0], st[6] = 10, 4                                       # some later state, clientIPKey x-forwarded-for
    st[12:16] = np.frombuffer(np.uint32(77).tobytes(), np.uint8)
    assert ebd.lib().ebd_parser_reset(ebd._p(st)) == 0
    assert st[0] == init_state and st[6] == 4 and st[12:16].view(np.uint32)[0] == 0
    assert ebd.lib().ebd_client_ip_key_name(4) == b"x-forwarded-for"
    assert ebd.lib().ebd_client_ip_key_name(0) == b""


def test_parser_state_check_rejects_corrupted_states():
    """ebd_parse_streams runs caller-owned states; every field that indexes something (the
    token list, the key trie, the stream) is checked before anything runs."""
    import numpy as np
    import ebd
    L = ebd.lib()
    st = np.zeros(320, np.uint8)
    assert L.ebd_parser_init(ebd._p(st)) == 0
    assert L.ebd_parser_state_check(ebd._p(st), 0) == 0

    def bad(edit, stream_len=100):
        s = st.copy()
        edit(s)
        return L.ebd_parser_state_check(ebd._p(s), stream_len) == -22

    u32 = lambda s, off, v: s.__setitem__(slice(off, off + 4), np.frombuffer(np.uint32(v).tobytes(), np.uint8))
    assert bad(lambda s: u32(s, 48, 33))            # ntok > EBD_PARSE_MAX_TOKENS
    assert bad(lambda s: s.__setitem__(5, 200))     # key past the trie
    assert bad(lambda s: s.__setitem__(0, 12))      # no such parser state
    assert bad(lambda s: s.__setitem__(6, 9))       # clientIPKey past the 5 keys
    assert bad(lambda s: u32(s, 12, 101))           # position past the stream
    assert bad(lambda s: (u32(s, 12, 10), u32(s, 40, 5), u32(s, 44, 4)))  # value start after its end
    assert bad(lambda s: (u32(s, 12, 10), u32(s, 40, 5), u32(s, 44, 11)))  # value end past the position
    s = st.copy()
    u32(s, 12, 10), u32(s, 40, 5), u32(s, 44, 9), u32(s, 48, 32)
    assert L.ebd_parser_state_check(ebd._p(s), 10) == 0
