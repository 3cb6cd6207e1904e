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
