"""ebd — Python binding of libebd_amd.so (include/ebpf_discovery_amd.h) over ctypes.

Mirrors the reference's consumer-side surface for the HTTP per-event parse path:
Context.submit ~ Discovery::fetchAndHandleEvents (one poll cycle, Discovery.cpp:48-90),
Context.services ~ Aggregator::collectServices (Aggregator.cpp:170-181),
Context.clear ~ Aggregator::clear (Aggregator.cpp:136-153).

There is no CPU fallback: if libebd_amd.so is missing, importing this module fails.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.dirname(_HERE)
# EBD_LIB selects another build of the same sources (tools/perf_fresh.py experiment variants)
LIB_PATH = os.environ.get("EBD_LIB") or os.path.join(PKG_DIR, "libebd_amd.so")

FLAG_IPV4, FLAG_IPV6, FLAG_UNENCRYPTED, FLAG_SSL, FLAG_NEW_DATA, FLAG_DATA_END = 2, 4, 8, 16, 32, 64
NO_BUFFER = 0xFFFFFFFF
STATUS_NONE, STATUS_UNFINISHED, STATUS_FINISHED, STATUS_INVALID = 0, 1, 2, 3
INFO_POST, INFO_HTTPS, INFO_SESSION, INFO_CIP, INFO_EXISTING, INFO_DROPPED = 0x01, 0x02, 0x04, 0x08, 0x40, 0x80
CLASS_NONE, CLASS_INTERNAL, CLASS_EXTERNAL = 0, 1, 2
ERR_BITS = {1: "TABLE_FULL", 2: "ARENA_FULL", 4: "LRU_OVERFLOW", 8: "SESSION_FULL", 16: "VERIFY_FULL", 32: "BAD_INPUT",
            64: "COLLISION", 128: "INTERNAL", 256: "NET_FULL"}
NET_V4_16, NET_V4_24, NET_V6_48 = 1, 2, 3

EVENT_DTYPE = np.dtype([("pid", "<u4"), ("fd", "<u4"), ("sessionID", "<u4"), ("bufferSeq", "<u4"),
                        ("sourceIP", "u1", (16,)), ("flags", "u1"), ("pad", "u1", (3,))])
RESULT_DTYPE = np.dtype([("consumed", "<u2"), ("status", "u1"), ("info", "u1"), ("url_off", "<u2"),
                         ("url_len", "<u2"), ("host_off", "<u2"), ("host_len", "<u2"), ("cip_off", "<u2"),
                         ("cip_len", "<u2")])
SESSION_REQ_DTYPE = np.dtype([("seq", "<u8"), ("pid", "<u4"), ("str_off", "<u4"), ("host_len", "<u2"),
                              ("url_len", "<u2"), ("cip_off", "<u2"), ("cip_len", "<u2"), ("info", "u1"),
                              ("status", "u1"), ("pad", "<u2"), ("pad2", "<u4")])
SERVICE_DTYPE = np.dtype([("pid", "<u4"), ("internal", "<u4"), ("external", "<u4"), ("https", "u1"),
                          ("pad", "u1", (3,)), ("endpoint_off", "<u8"), ("endpoint_len", "<u4"),
                          ("domain_off", "<u4"), ("domain_len", "<u4"), ("host_len", "<u4"), ("first_seq", "<u8"),
                          ("key_lo", "<u8"), ("key_hi", "<u8"), ("nets_v4_16", "<u4"), ("nets_v4_24", "<u4"),
                          ("nets_v6", "<u4"), ("pad2", "<u4")])
SERVICE_NET_DTYPE = np.dtype([("key_lo", "<u8"), ("key_hi", "<u8"), ("kind", "u1"), ("prefix", "u1", (6,)), ("pad", "u1"),
                              ("time_ns", "<u8")])
# ebd_wire_service: a service on the cross-GPU wire (its endpoint bytes follow the previous
# record's in the strings, each padded to 8 bytes; WIRE_NO_BYTES in endpoint_len: none)
WIRE_DTYPE = np.dtype([("key_lo", "<u8"), ("key_hi", "<u8"), ("first", "<u8"), ("pid", "<u4"), ("internal", "<u4"),
                       ("external", "<u4"), ("endpoint_len", "<u4")])
WIRE_NO_BYTES = 0x80000000
# ebd_request: an HttpRequest + DiscoverySessionMeta parsed elsewhere (ebd_aggregate_requests)
REQUEST_DTYPE = np.dtype([("str_off", "<u8"), ("pid", "<u4"), ("host_len", "<u2"), ("url_len", "<u2"), ("cip_len", "<u2"),
                          ("flags", "u1"), ("is_https", "u1"), ("source_ip", "u1", (16,)), ("pad", "<u4")])
NO_CLIENT_IP = 0xFFFF
assert REQUEST_DTYPE.itemsize == 40
assert WIRE_DTYPE.itemsize == 40
assert EVENT_DTYPE.itemsize == 36 and RESULT_DTYPE.itemsize == 16
assert SESSION_REQ_DTYPE.itemsize == 32 and SERVICE_DTYPE.itemsize == 80 and SERVICE_NET_DTYPE.itemsize == 32
CFG_TIMING = 2
CFG_NETWORK_COUNTERS = 4
CFG_FRESH_SCAN = 8  # k_fresh_scan (the structural scan) instead of the DFA k_fresh
# A fixed service-key PRF key for tests that compare keys across contexts or with the host
# hooks; products leave the key to the library (a fresh random key per context).
TEST_HASH_KEY = (0x0706050403020100, 0x0F0E0D0C0B0A0908)


class Config(C.Structure):
    _fields_ = [("device", C.c_int), ("max_events", C.c_uint32), ("max_payload", C.c_uint64),
                ("service_capacity", C.c_uint32), ("string_arena", C.c_uint64), ("lru_capacity", C.c_uint32),
                ("flags", C.c_uint32), ("hash_key", C.c_uint64 * 2), ("net_capacity", C.c_uint32), ("pad", C.c_uint32)]


class DeviceBatch(C.Structure):
    _fields_ = [("events", C.c_void_p), ("len", C.c_void_p), ("off", C.c_void_p), ("payload", C.c_void_p),
                ("payload_bytes", C.c_uint64), ("n", C.c_uint32)]


PAYLOAD_PAD = 16  # EBD_PAYLOAD_PAD


class Stats(C.Structure):
    _fields_ = [("events", C.c_uint64), ("requests", C.c_uint64), ("session_events", C.c_uint64),
                ("kernel_deletes", C.c_uint64), ("live_sessions", C.c_uint64), ("max_live_sessions", C.c_uint64),
                ("services", C.c_uint64), ("hash_collisions", C.c_uint64), ("errors", C.c_uint64),
                ("lru_evictions", C.c_uint64), ("lru_exact_batches", C.c_uint64),
                ("lru_rounds", C.c_uint64), ("lru_sequential", C.c_uint64)]


class KernelTime(C.Structure):
    _fields_ = [("name", C.c_char * 24), ("launches", C.c_uint64), ("total_ms", C.c_double)]


class TraceConfig(C.Structure):
    _fields_ = [("config", C.c_uint32), ("seed", C.c_uint64), ("first", C.c_uint64), ("n", C.c_uint32),
                ("align", C.c_uint32), ("shard_count", C.c_uint32), ("shard_index", C.c_uint32)]


class Ipv4Network(C.Structure):
    _fields_ = [("addr", C.c_uint8 * 4), ("mask", C.c_uint8 * 4)]


class Ipv6Network(C.Structure):
    _fields_ = [("addr", C.c_uint8 * 16), ("mask", C.c_uint8 * 16)]


# Every function the public headers declare (checked by tests/test_abi.py).
_SIGS = {
    "ebd_ctx_create": (C.c_int, [C.POINTER(Config), C.POINTER(C.c_void_p)]),
    "ebd_ctx_destroy": (C.c_int, [C.c_void_p]),
    "ebd_ctx_stream": (C.c_void_p, [C.c_void_p]),
    "ebd_get_hash_key": (C.c_int, [C.c_void_p, C.c_void_p]),
    "ebd_set_interfaces": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]),
    "ebd_submit_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                   C.c_uint32]),
    "ebd_submit_batch_device": (C.c_int, [C.c_void_p, C.POINTER(DeviceBatch)]),
    "ebd_stage_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32,
                                  C.POINTER(C.c_uint64)]),
    "ebd_submit_staged": (C.c_int, [C.c_void_p, C.c_uint64]),
    "ebd_host_alloc": (C.c_void_p, [C.c_void_p, C.c_uint64]),
    "ebd_host_free": (C.c_int, [C.c_void_p, C.c_void_p]),
    "ebd_fetch_results_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    "ebd_sync": (C.c_int, [C.c_void_p]),
    "ebd_set_seq_base": (C.c_int, [C.c_void_p, C.c_uint64]),
    "ebd_kernel_times": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    "ebd_reset_kernel_times": (C.c_int, [C.c_void_p]),
    "ebd_fetch_results": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    "ebd_results_device": (C.c_void_p, [C.c_void_p]),
    "ebd_fetch_session_requests": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32), C.c_void_p,
                                             C.c_uint64, C.POINTER(C.c_uint64)]),
    "ebd_collect_services": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32), C.c_void_p,
                                       C.c_uint64, C.POINTER(C.c_uint64)]),
    "ebd_clear": (C.c_int, [C.c_void_p]),
    "ebd_reset_services": (C.c_int, [C.c_void_p]),
    "ebd_set_event_clock": (C.c_int, [C.c_void_p, C.c_void_p]),
    "ebd_collect_networks_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    "ebd_merge_networks_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    "ebd_set_clock": (C.c_int, [C.c_void_p, C.c_uint64]),
    "ebd_network_counters_cleaning": (C.c_int, [C.c_void_p, C.c_uint64]),
    "ebd_collect_networks": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    "ebd_format_services_json": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                           C.POINTER(C.c_uint64)]),
    "ebd_report_json": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]),
    "ebd_export_services_device": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64,
                                             C.c_void_p, C.c_void_p]),
    "ebd_export_capacity": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
    "ebd_export_services_device_sized": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64,
                                                   C.c_void_p]),
    "ebd_wire_segment_bytes_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                                C.c_uint32, C.c_void_p]),
    "ebd_merge_services_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64]),
    "ebd_merge_service_keys_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]),
    "ebd_wire_compact_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                          C.c_uint64, C.POINTER(C.c_uint64)]),
    "ebd_merge_service_bytes_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64]),
    "ebd_aggregate_requests": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64]),
    "ebd_get_stats": (C.c_int, [C.c_void_p, C.POINTER(Stats)]),
    "ebd_strerror": (C.c_char_p, [C.c_int]),
    "ebd_build_id": (C.c_char_p, []),
    "ebd_measure_read_bandwidth": (C.c_int, [C.c_int, C.c_uint64, C.c_uint32, C.POINTER(C.c_double),
                                             C.POINTER(C.c_double)]),
    "ebd_trace_size": (C.c_int, [C.POINTER(TraceConfig), C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
    "ebd_trace_generate_host": (C.c_int, [C.POINTER(TraceConfig), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_uint64, C.c_void_p]),
    "ebd_trace_size_device": (C.c_int, [C.c_void_p, C.POINTER(TraceConfig), C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint64)]),
    "ebd_trace_generate_device": (C.c_int, [C.c_void_p, C.POINTER(TraceConfig), C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.c_void_p, C.c_uint64, C.c_void_p]),
    # testing header
    "ebd_host_dfa_info": (C.c_int, [C.c_void_p, C.c_uint32]),
    "ebd_host_dfa_next": (C.c_int, [C.c_void_p, C.c_uint32]),
    "ebd_host_fresh": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint8, C.c_void_p, C.c_void_p, C.c_uint32,
                                 C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]),
    "ebd_host_scan": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint8, C.c_void_p, C.c_void_p,
                                C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]),
    "ebd_host_gp_parse": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint8, C.c_int, C.c_void_p, C.c_void_p]),
    "ebd_host_dfa_parse": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint8, C.c_int, C.c_void_p, C.c_void_p]),
    "ebd_host_classify": (C.c_int, [C.c_void_p, C.c_uint32, C.c_int, C.c_uint8, C.c_void_p, C.c_uint32, C.c_void_p,
                                    C.c_uint32]),
    "ebd_host_pton": (C.c_int, [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p]),
    "ebd_testing_set_lru_window": (C.c_int, [C.c_void_p, C.c_uint32]),
    "ebd_parser_init": (C.c_int, [C.c_void_p]),
    "ebd_parser_reset": (C.c_int, [C.c_void_p]),
    "ebd_parser_state_check": (C.c_int, [C.c_void_p, C.c_uint64]),
    "ebd_parse_streams": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64]),
    "ebd_client_ip_key_name": (C.c_char_p, [C.c_uint32]),
    "ebd_host_endpoint_key": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p]),
}

_lib = None


def lib():
    """Loads libebd_amd.so; raises if it is missing (no fallback path exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libebd_amd.so not built ({LIB_PATH}); run `make -C ebpf-discovery_amd`")
        try:  # torch ships its own HIP runtime under another file name: load it first so that
            import torch  # noqa: F401  libebd_amd.so binds to that one (one runtime per process)
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            if not hasattr(L, name) and os.environ.get("EBD_LIB"):
                continue  # an experiment build (EBD_LIB) from before a later entry point: not bound
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def build_id():
    return lib().ebd_build_id().decode()


def read_bandwidth(device=0, nbytes=4 << 30, reps=10):
    """ebd_measure_read_bandwidth: the device's measured read-stream rates in GB/s,
    {"plain": 16-B loads per lane, "dma": LDS-DMA tiles}."""
    a, b = C.c_double(), C.c_double()
    _check(lib().ebd_measure_read_bandwidth(device, nbytes, reps, C.byref(a), C.byref(b)), "ebd_measure_read_bandwidth")
    return {"plain": a.value, "dma": b.value}


class EbdError(RuntimeError):
    pass


def _check(rc, what):
    if rc != 0:
        raise EbdError(f"{what}: {lib().ebd_strerror(rc).decode()} ({rc})")


def _p(a):
    if a is None:
        return None
    if hasattr(a, "data_ptr"):  # torch tensor
        return C.c_void_p(a.data_ptr())
    return a.ctypes.data_as(C.c_void_p) if a.size else None


def _nets4(v4):
    arr = (Ipv4Network * max(len(v4), 1))()
    for k, (a, m) in enumerate(v4):
        arr[k].addr[:] = list(a)
        arr[k].mask[:] = list(m)
    return arr


def _nets6(v6):
    arr = (Ipv6Network * max(len(v6), 1))()
    for k, (a, m) in enumerate(v6):
        arr[k].addr[:] = list(a)
        arr[k].mask[:] = list(m)
    return arr


class Context:
    """One GPU context: the Discovery consumer state (session LRU) + the Aggregator."""

    def __init__(self, max_events, device=0, max_payload=0, service_capacity=0, string_arena=0, lru_capacity=0,
                 timing=False, hash_key=None, network_counters=False, net_capacity=0, fresh_scan=False):
        cfg = Config(device=device, max_events=max_events, max_payload=max_payload,
                     service_capacity=service_capacity, string_arena=string_arena, lru_capacity=lru_capacity,
                     flags=(CFG_TIMING if timing else 0) | (CFG_NETWORK_COUNTERS if network_counters else 0) |
                     (CFG_FRESH_SCAN if fresh_scan else 0),
                     net_capacity=net_capacity)
        if hash_key is not None:
            cfg.hash_key[0], cfg.hash_key[1] = int(hash_key[0]), int(hash_key[1])
        h = C.c_void_p()
        _check(lib().ebd_ctx_create(C.byref(cfg), C.byref(h)), "ebd_ctx_create")
        self.h = h
        self.max_events = max_events
        self.network_counters = network_counters
        self._held = []  # device tensors the queued work of the context reads or writes (_fence)

    def close(self):
        if getattr(self, "h", None):
            lib().ebd_ctx_destroy(self.h)  # waits for the context's streams
            self.h = None
            self._ext = None
            self._held = []

    def __del__(self):
        self.close()

    @property
    def stream(self):
        return lib().ebd_ctx_stream(self.h)

    @property
    def hash_key(self):
        k = np.zeros(2, np.uint64)
        _check(lib().ebd_get_hash_key(self.h, _p(k)), "ebd_get_hash_key")
        return int(k[0]), int(k[1])

    def set_interfaces(self, v4=(), v6=()):
        v4, v6 = list(v4), list(v6)
        _check(lib().ebd_set_interfaces(self.h, _nets4(v4), len(v4), _nets6(v6), len(v6)), "ebd_set_interfaces")

    def submit(self, events, lens, offs, payload):
        events = np.ascontiguousarray(events, dtype=EVENT_DTYPE)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        _check(lib().ebd_submit_batch(self.h, _p(events), _p(lens), _p(offs), _p(payload), payload.size,
                                      len(events)), "ebd_submit_batch")

    def stage(self, events, lens, offs, payload):
        """ebd_stage_batch: uploads a host batch on the copy stream; returns its ticket."""
        events = np.ascontiguousarray(events, dtype=EVENT_DTYPE)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        t = C.c_uint64()
        _check(lib().ebd_stage_batch(self.h, _p(events), _p(lens), _p(offs), _p(payload), payload.size, len(events),
                                     C.byref(t)), "ebd_stage_batch")
        return t.value

    def submit_staged(self, ticket):
        _check(lib().ebd_submit_staged(self.h, ticket), "ebd_submit_staged")

    def pinned_empty(self, n, dtype):
        """A numpy array over pinned host memory (ebd_host_alloc), freed with the array."""
        import weakref
        dtype = np.dtype(dtype)
        nbytes = max(int(n) * dtype.itemsize, 1)
        p = lib().ebd_host_alloc(self.h, nbytes)
        if not p:
            raise EbdError("ebd_host_alloc failed")
        buf = (C.c_uint8 * nbytes).from_address(p)
        weakref.finalize(buf, lib().ebd_host_free, self.h, C.c_void_p(p))
        return np.frombuffer(buf, dtype=dtype, count=int(n))

    def results_async(self, out):
        """ebd_fetch_results_async into `out` (RESULT_DTYPE, ideally pinned); valid after sync()."""
        n = C.c_uint32()
        _check(lib().ebd_fetch_results_async(self.h, _p(out), out.size, C.byref(n)), "ebd_fetch_results_async")
        return n.value

    def _fence(self, *tensors, hold=True):
        """The context stream waits for the work torch queued for these tensors on its current
        stream (the context stream is a non-blocking stream: it does not order itself after
        torch's).  Raw pointers are the caller's to order.  hold=False: the C call blocks until
        the context stream is done with them, so nothing needs to keep them alive."""
        import torch
        ts = [t for t in tensors if isinstance(t, torch.Tensor) and t.is_cuda]
        if not ts:
            return
        if getattr(self, "_ext", None) is None:
            self._ext = torch.cuda.ExternalStream(lib().ebd_ctx_stream(self.h), device=ts[0].device)
        self._ext.wait_stream(torch.cuda.current_stream(ts[0].device))
        # and the tensors stay referenced until the context's queued work is known done (sync,
        # close): torch's caching allocator may not hand their memory out again before then.
        # (record_stream on the context's stream would outlive it: ebd_ctx_destroy destroys it.)
        if hold:
            self._held.extend(ts)

    def submit_device(self, events, lens, offs, payload, n, payload_bytes=None):
        """Device-resident batch (torch tensors on the context's device or raw pointers).
        payload_bytes: the bytes buffers may occupy; for a payload tensor it defaults to its
        size less the EBD_PAYLOAD_PAD readable bytes the kernels need past the last buffer."""
        if payload_bytes is None:
            if not hasattr(payload, "numel"):
                raise ValueError("submit_device: payload_bytes is required with a raw payload pointer")
            payload_bytes = max(payload.numel() - PAYLOAD_PAD, 0)
        self._fence(events, lens, offs, payload)
        b = DeviceBatch(events=_ptrval(events), len=_ptrval(lens), off=_ptrval(offs), payload=_ptrval(payload),
                        payload_bytes=payload_bytes, n=n)
        _check(lib().ebd_submit_batch_device(self.h, C.byref(b)), "ebd_submit_batch_device")

    def sync(self):
        _check(lib().ebd_sync(self.h), "ebd_sync")
        self._held = []

    def set_seq_base(self, seq):
        _check(lib().ebd_set_seq_base(self.h, seq), "ebd_set_seq_base")

    def kernel_times(self):
        """{kernel: (launches, total_ms)} of the HIP-event timed launches (timing=True)."""
        n = C.c_uint32()
        _check(lib().ebd_kernel_times(self.h, None, 0, C.byref(n)), "ebd_kernel_times")
        arr = (KernelTime * n.value)()
        _check(lib().ebd_kernel_times(self.h, arr, n.value, C.byref(n)), "ebd_kernel_times")
        return {a.name.decode(): (a.launches, a.total_ms) for a in arr}

    def reset_kernel_times(self):
        _check(lib().ebd_reset_kernel_times(self.h), "ebd_reset_kernel_times")

    def results(self):
        n = C.c_uint32()
        lib().ebd_fetch_results(self.h, None, 0, C.byref(n))
        out = np.zeros(n.value, RESULT_DTYPE)
        _check(lib().ebd_fetch_results(self.h, _p(out), n.value, C.byref(n)), "ebd_fetch_results")
        return out

    def session_requests(self):
        n, sl = C.c_uint32(), C.c_uint64()
        _check(lib().ebd_fetch_session_requests(self.h, None, 0, C.byref(n), None, 0, C.byref(sl)), "sreq")
        out = np.zeros(n.value, SESSION_REQ_DTYPE)
        buf = np.zeros(max(sl.value, 1), np.uint8)
        _check(lib().ebd_fetch_session_requests(self.h, _p(out), n.value, C.byref(n), _p(buf), buf.size,
                                                C.byref(sl)), "ebd_fetch_session_requests")
        return out, buf[:sl.value].tobytes()

    def services_raw(self):
        """ebd_collect_services as (SERVICE_DTYPE records, endpoint bytes)."""
        n, sl = C.c_uint32(), C.c_uint64()
        _check(lib().ebd_collect_services(self.h, None, 0, C.byref(n), None, 0, C.byref(sl)), "collect")
        out = np.zeros(max(n.value, 1), SERVICE_DTYPE)
        buf = np.zeros(max(sl.value, 1), np.uint8)
        _check(lib().ebd_collect_services(self.h, _p(out), out.size, C.byref(n), _p(buf), buf.size, C.byref(sl)),
               "ebd_collect_services")
        return out[:n.value].copy(), buf[:sl.value].copy()

    def services(self, with_seq=False, with_nets=False):
        """[(pid, endpoint, domain, scheme, internal, external)] sorted by (pid, endpoint);
        with_seq appends the first-arrival sequence number (for cross-shard merges), with_nets
        the sizes of the /16, /24 and v6 network maps."""
        n, sl = C.c_uint32(), C.c_uint64()
        _check(lib().ebd_collect_services(self.h, None, 0, C.byref(n), None, 0, C.byref(sl)), "collect")
        out = np.zeros(max(n.value, 1), SERVICE_DTYPE)
        buf = np.zeros(max(sl.value, 1), np.uint8)
        _check(lib().ebd_collect_services(self.h, _p(out), out.size, C.byref(n), _p(buf), buf.size, C.byref(sl)),
               "ebd_collect_services")
        s = buf.tobytes()
        res = []
        for r in out[:n.value]:
            o, L = int(r["endpoint_off"]), int(r["endpoint_len"])
            ep = s[o:o + L]
            dom = ep[int(r["domain_off"]):int(r["domain_off"]) + int(r["domain_len"])]
            t = (int(r["pid"]), ep, dom, b"https" if r["https"] else b"http", int(r["internal"]), int(r["external"]))
            if with_seq:
                t += (int(r["first_seq"]),)
            if with_nets:
                t += (int(r["nets_v4_16"]), int(r["nets_v4_24"]), int(r["nets_v6"]))
            res.append(t)
        res.sort(key=lambda t: (t[0], t[1]))
        return res

    def clear(self):
        _check(lib().ebd_clear(self.h), "ebd_clear")

    def reset_services(self):
        """ebd_reset_services: every service and network-map entry goes (the merge's start)."""
        _check(lib().ebd_reset_services(self.h), "ebd_reset_services")

    def networks_device(self, device):
        """ebd_collect_networks_device: the network-map entries as a device uint8 tensor of
        SERVICE_NET_DTYPE records (32 bytes each)."""
        import torch
        n = C.c_uint32()
        _check(lib().ebd_collect_networks_device(self.h, None, 0, C.byref(n)), "ebd_collect_networks_device")
        out = torch.empty(max(n.value, 1) * SERVICE_NET_DTYPE.itemsize, dtype=torch.uint8, device=device)
        self._fence(out)
        _check(lib().ebd_collect_networks_device(self.h, C.c_void_p(out.data_ptr()), max(n.value, 1), C.byref(n)),
               "ebd_collect_networks_device")
        return out[:n.value * SERVICE_NET_DTYPE.itemsize]

    def merge_networks_device(self, recs):
        """ebd_merge_networks_device: SERVICE_NET_DTYPE records (device uint8 tensor) into the
        maps of this table's services (merge the services first)."""
        n = recs.numel() // SERVICE_NET_DTYPE.itemsize
        self._fence(recs)
        _check(lib().ebd_merge_networks_device(self.h, C.c_void_p(recs.data_ptr()) if n else None, n),
               "ebd_merge_networks_device")

    def set_clock(self, now_ns):
        """Aggregator::getCurrentTime (steady-clock ns) of the next batches' requests; 0 = CLOCK_MONOTONIC."""
        _check(lib().ebd_set_clock(self.h, now_ns), "ebd_set_clock")

    def set_event_clock(self, times):
        """ebd_set_event_clock: per-event getCurrentTime readings (a device int64/uint64 tensor
        of the next batch's n events) or None.  The batch's kernels read it after submit
        returns; _fence keeps it referenced until sync()."""
        self._ev_times = times
        if times is not None:
            self._fence(times)
        _check(lib().ebd_set_event_clock(self.h, C.c_void_p(times.data_ptr()) if times is not None else None),
               "ebd_set_event_clock")

    def network_counters_cleaning(self, now_ns=0):
        _check(lib().ebd_network_counters_cleaning(self.h, now_ns), "ebd_network_counters_cleaning")

    def networks_raw(self):
        """ebd_collect_networks: SERVICE_NET_DTYPE records (one per live network-map entry)."""
        n = C.c_uint32()
        _check(lib().ebd_collect_networks(self.h, None, 0, C.byref(n)), "ebd_collect_networks")
        out = np.zeros(max(n.value, 1), SERVICE_NET_DTYPE)
        _check(lib().ebd_collect_networks(self.h, _p(out), out.size, C.byref(n)), "ebd_collect_networks")
        return out[:n.value].copy()

    def report_json(self):
        """Discovery::outputServicesToStdout's text (bytes; b"" without services)."""
        ln = C.c_uint64()
        _check(lib().ebd_report_json(self.h, None, 0, C.byref(ln)), "ebd_report_json")
        buf = C.create_string_buffer(max(ln.value, 1))
        while True:  # the table may not change between the calls, but size the buffer from the answer
            rc = lib().ebd_report_json(self.h, buf, len(buf), C.byref(ln))
            if rc == 0:
                return buf.raw[:ln.value]
            if ln.value <= len(buf):
                _check(rc, "ebd_report_json")
            buf = C.create_string_buffer(ln.value)

    def export_services_device(self, world, device):
        """The services grouped by owner ((key_lo >> 32) % world) in device tensors: (WIRE_DTYPE
        records as uint8 [n * 40], their endpoint bytes uint8, counts[world], str_counts[world])."""
        import torch
        counts = np.zeros(world, np.uint32)
        scounts = np.zeros(world, np.uint64)
        _check(lib().ebd_export_services_device(self.h, world, None, 0, None, 0, _p(counts), _p(scounts)), "export")
        n, sb = int(counts.sum()), int(scounts.sum())
        recs = torch.empty(max(n, 1) * WIRE_DTYPE.itemsize, dtype=torch.uint8, device=device)
        strs = torch.empty(max(sb, 8), dtype=torch.uint8, device=device)
        self._fence(recs, strs, hold=False)  # torch may hand back memory its stream still uses
        _check(lib().ebd_export_services_device(self.h, world, C.c_void_p(recs.data_ptr()), max(n, 1),
                                                C.c_void_p(strs.data_ptr()), strs.numel(), _p(counts), _p(scounts)),
               "ebd_export_services_device")
        return recs[:n * WIRE_DTYPE.itemsize], strs[:sb], counts, scounts

    def export_services_device_sized(self, world, device):
        """ebd_export_services_device_sized: the services grouped by owner into buffers the context
        keeps (capacity: the whole table), with nothing read back.  Returns (records uint8, strings
        uint8, sizes): sizes is a device int64 [2, world] view, row 0 the records and row 1 the
        string bytes per owner; records and strings are the capacity-sized buffers (their first
        sum(sizes[0]) records and sum(sizes[1]) bytes are the export)."""
        import torch
        key = (str(device), world)
        if getattr(self, "_exp_key", None) is None or self._exp_key[0] != key[0]:
            r, sb = C.c_uint32(), C.c_uint64()
            _check(lib().ebd_export_capacity(self.h, C.byref(r), C.byref(sb)), "ebd_export_capacity")
            self._exp_bufs = (torch.empty(r.value * WIRE_DTYPE.itemsize, dtype=torch.uint8, device=device),
                              torch.empty(max(sb.value, 8), dtype=torch.uint8, device=device),
                              torch.empty(128, dtype=torch.int64, device=device))
            self._exp_cap = r.value
        self._exp_key = key
        recs, strs, sizes = self._exp_bufs
        self._fence(recs, strs, sizes, hold=False)
        _check(lib().ebd_export_services_device_sized(self.h, world, C.c_void_p(recs.data_ptr()), self._exp_cap,
                                                      C.c_void_p(strs.data_ptr()), strs.numel(), C.c_void_p(sizes.data_ptr())),
               "ebd_export_services_device_sized")
        return recs, strs, sizes.view(2, 64)[:, :world]

    def wire_segment_bytes_device(self, recs, seg_counts, need=None, dst=None):
        """ebd_wire_segment_bytes_device: per segment (seg_counts: device int64 [world], the
        records of each segment in order) the endpoint bytes of the records whose need byte is set
        (or whose dst is not -1): a device int64 [world] tensor, nothing read back."""
        import torch
        world = seg_counts.numel()
        n = recs.numel() // WIRE_DTYPE.itemsize
        out = torch.empty(world, dtype=torch.int64, device=seg_counts.device)
        seg = seg_counts.to(torch.int64).contiguous()
        self._fence(recs, seg, out, *(t for t in (need, dst) if t is not None), hold=False)
        _check(lib().ebd_wire_segment_bytes_device(self.h, C.c_void_p(recs.data_ptr()) if n else None, n,
                                                   C.c_void_p(need.data_ptr()) if need is not None else None,
                                                   C.c_void_p(dst.data_ptr()) if dst is not None else None,
                                                   C.c_void_p(seg.data_ptr()), world, C.c_void_p(out.data_ptr())),
               "ebd_wire_segment_bytes_device")
        return out

    def merge_services_device(self, recs, strings):
        """Inserts wire records (device uint8 tensors; strings readable 8 bytes past their
        bytes) into this table."""
        n = recs.numel() // WIRE_DTYPE.itemsize
        self._fence(recs, strings, hold=False)
        _check(lib().ebd_merge_services_device(self.h, C.c_void_p(recs.data_ptr()) if n else None, n,
                                               C.c_void_p(strings.data_ptr()) if strings.numel() else None,
                                               strings.numel()), "ebd_merge_services_device")

    def merge_service_keys_device(self, recs, dst):
        """Key round of the two-round merge: wire records (device uint8 tensor) into this
        table; dst (device int64 tensor, one per record) gets the arena offset reserved for
        each record whose bytes are needed, -1 for the others."""
        n = recs.numel() // WIRE_DTYPE.itemsize
        assert dst.dtype == __import__("torch").int64 and dst.numel() == n
        if n == 0:
            return
        self._fence(recs, dst, hold=False)
        _check(lib().ebd_merge_service_keys_device(self.h, C.c_void_p(recs.data_ptr()), n, C.c_void_p(dst.data_ptr())),
               "ebd_merge_service_keys_device")

    def wire_compact_device(self, recs, strings, need, sized=True):
        """Source side of the bytes round: the endpoint bytes of the exported records whose
        need byte is set, packed in record order (a device uint8 tensor).  sized=False: no size
        read; the whole strings-sized buffer comes back, the packed bytes at its start."""
        import torch
        n = recs.numel() // WIRE_DTYPE.itemsize
        assert need.dtype == torch.uint8 and need.numel() == n
        if n == 0:
            return torch.empty(0, dtype=torch.uint8, device=recs.device)
        self._fence(recs, strings, need, hold=False)
        ln = C.c_uint64(0)
        sp = C.c_void_p(strings.data_ptr()) if strings.numel() else None
        if not sized:
            out = torch.empty(max(strings.numel(), 8), dtype=torch.uint8, device=recs.device)
            self._fence(out, hold=False)
            _check(lib().ebd_wire_compact_device(self.h, C.c_void_p(recs.data_ptr()), n, sp, strings.numel(),
                                                 C.c_void_p(need.data_ptr()), C.c_void_p(out.data_ptr()), out.numel(), None),
                   "ebd_wire_compact_device")
            return out
        _check(lib().ebd_wire_compact_device(self.h, C.c_void_p(recs.data_ptr()), n, sp, strings.numel(),
                                             C.c_void_p(need.data_ptr()), None, 0, C.byref(ln)), "ebd_wire_compact_device")
        out = torch.empty(max(int(ln.value), 8), dtype=torch.uint8, device=recs.device)
        self._fence(out, hold=False)
        _check(lib().ebd_wire_compact_device(self.h, C.c_void_p(recs.data_ptr()), n, sp, strings.numel(),
                                             C.c_void_p(need.data_ptr()), C.c_void_p(out.data_ptr()), out.numel(),
                                             C.byref(ln)), "ebd_wire_compact_device")
        return out[:int(ln.value)]

    def merge_service_bytes_device(self, recs, dst, strings):
        """Bytes round of the two-round merge: the received bytes (device uint8, in the order
        of the records with dst >= 0, readable 8 bytes past their end) to their places."""
        n = recs.numel() // WIRE_DTYPE.itemsize
        if n == 0:
            return
        self._fence(recs, dst, strings, hold=False)
        _check(lib().ebd_merge_service_bytes_device(self.h, C.c_void_p(recs.data_ptr()), n, C.c_void_p(dst.data_ptr()),
                                                    C.c_void_p(strings.data_ptr()) if strings.numel() else None,
                                                    strings.numel()), "ebd_merge_service_bytes_device")

    def aggregate_requests(self, reqs):
        """ebd_aggregate_requests: Aggregator::newRequest for requests parsed elsewhere, in order.
        reqs: (pid, host, url, client_ip or None, flags, is_https, source_ip16) tuples, where
        client_ip is HttpRequest::clientIp.front() (None: clientIp empty)."""
        recs = np.zeros(len(reqs), REQUEST_DTYPE)
        strings = bytearray()
        for k, (pid, host, url, cip, flags, https, src) in enumerate(reqs):
            recs[k]["str_off"] = len(strings)
            recs[k]["pid"], recs[k]["flags"], recs[k]["is_https"] = pid, flags, 1 if https else 0
            recs[k]["host_len"], recs[k]["url_len"] = len(host), len(url)
            recs[k]["cip_len"] = NO_CLIENT_IP if cip is None else len(cip)
            recs[k]["source_ip"] = np.frombuffer(bytes(src).ljust(16, b"\0")[:16], np.uint8)
            strings += host + url + (cip or b"")
        sb = np.frombuffer(bytes(strings) or b"\0", np.uint8)
        _check(lib().ebd_aggregate_requests(self.h, _p(recs), len(recs), _p(sb), len(strings)), "ebd_aggregate_requests")

    def set_lru_window(self, window):
        """The exact LRU's derivation window (testing hook; 0 = default)."""
        _check(lib().ebd_testing_set_lru_window(self.h, window), "ebd_testing_set_lru_window")

    def stats(self):
        s = Stats()
        _check(lib().ebd_get_stats(self.h, C.byref(s)), "ebd_get_stats")
        d = {k: getattr(s, k) for k, _ in Stats._fields_}
        d["error_names"] = [v for b, v in ERR_BITS.items() if d["errors"] & b]
        return d


PARSE_MAX_TOKENS = 32
PARSE_CALL_DTYPE = np.dtype([("state", np.uint8, 320), ("data_off", np.uint64), ("data_len", np.uint32), ("flags", np.uint8),
                             ("pad_", np.uint8, 3), ("consumed", np.uint32), ("status", np.uint8), ("is_https", np.uint8),
                             ("client_ip_key", np.uint8), ("tokens_dropped", np.uint8), ("method_len", np.uint32),
                             ("url_off", np.uint32), ("url_len", np.uint32), ("protocol_off", np.uint32),
                             ("protocol_len", np.uint32), ("host_off", np.uint32), ("host_len", np.uint32),
                             ("ntokens", np.uint32), ("tokens", np.uint32, (PARSE_MAX_TOKENS, 2))])
assert PARSE_CALL_DTYPE.itemsize == 632
PARSER_UNFINISHED, PARSER_FINISHED, PARSER_INVALID = 0, 1, 2


class StreamParser:
    """httpparser::HttpRequestParser (HttpRequestParser.h:41-101) over ebd_parse_streams: one GPU
    call per parse(); the request's bytes since reset() are kept here and `result` is
    materialised from the stream positions the GPU returns (the C++ facade's
    ebdamd::HttpRequestParser does the same)."""

    def __init__(self, ctx):
        self.ctx = ctx
        self.call = np.zeros(1, PARSE_CALL_DTYPE)
        _check(lib().ebd_parser_init(_p(self.call["state"][0])), "ebd_parser_init")
        self.stream = b""
        self.status = PARSER_UNFINISHED
        self.result = self._result()

    def parse(self, data: bytes, flags: int) -> int:
        base = len(self.stream)
        buf = np.frombuffer(self.stream + data or b"\0", np.uint8)
        self.call["data_off"], self.call["data_len"], self.call["flags"] = 0, len(self.stream) + len(data), flags
        _check(lib().ebd_parse_streams(self.ctx.h, _p(self.call), 1, _p(buf), len(self.stream) + len(data)), "ebd_parse_streams")
        c = self.call[0]
        self.stream = (self.stream + data)[:base + int(c["consumed"])]
        self.status = int(c["status"])
        self.result = self._result()
        return int(c["consumed"])

    def reset(self):
        _check(lib().ebd_parser_reset(_p(self.call["state"][0])), "ebd_parser_reset")
        self.stream = b""
        self.status = PARSER_UNFINISHED
        self.result = self._result(cleared=True)

    def is_finished(self):
        return self.status != PARSER_UNFINISHED

    def is_invalid(self):
        return self.status == PARSER_INVALID

    def _result(self, cleared=False):
        c = self.call[0]
        s = self.stream
        key = lib().ebd_client_ip_key_name(int(c["client_ip_key"])).decode()
        if cleared or not s and int(c["consumed"]) == 0:
            return {"method": b"", "url": b"", "protocol": b"", "host": b"", "client_ip": [], "client_ip_key": key,
                    "is_https": False}
        sp = lambda o, n: s[int(o):int(o) + int(n)]  # noqa: E731
        return {"method": sp(0, c["method_len"]), "url": sp(c["url_off"], c["url_len"]),
                "protocol": sp(c["protocol_off"], c["protocol_len"]) if c["protocol_len"] else b"",
                "host": sp(c["host_off"], c["host_len"]),
                "client_ip": [s[int(a):int(b)] for a, b in c["tokens"][:int(c["ntokens"])]],
                "client_ip_key": key, "is_https": bool(c["is_https"]), "tokens_dropped": bool(c["tokens_dropped"])}


def format_services_json(records, strings: bytes):
    """ebd_format_services_json (host only): the report text of SERVICE_DTYPE records."""
    records = np.ascontiguousarray(records, dtype=SERVICE_DTYPE)
    sb = np.frombuffer(strings, np.uint8) if strings else np.zeros(1, np.uint8)
    ln = C.c_uint64()
    _check(lib().ebd_format_services_json(_p(records), len(records), _p(sb), len(strings), None, 0, C.byref(ln)), "json")
    buf = C.create_string_buffer(max(ln.value, 1))
    _check(lib().ebd_format_services_json(_p(records), len(records), _p(sb), len(strings), buf, len(buf), C.byref(ln)),
           "ebd_format_services_json")
    return buf.raw[:ln.value]


def _ptrval(x):
    if x is None:
        return None
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    return int(x)


def trace_config(config, seed, first, n, align=1, shard=(1, 0)):
    return TraceConfig(config=config, seed=seed, first=first, n=n, align=align, shard_count=shard[0],
                       shard_index=shard[1])


def trace_size(config, seed, first, n, align=1, shard=(1, 0), with_events=False):
    """Payload bytes (and with_events: kept events) of candidates [first, first + n)."""
    t = trace_config(config, seed, first, n, align, shard)
    v, k = C.c_uint64(), C.c_uint32()
    _check(lib().ebd_trace_size(C.byref(t), C.byref(k), C.byref(v)), "ebd_trace_size")
    return (k.value, v.value) if with_events else v.value


def generate_host(config, seed, first, n, align=1, shard=(1, 0), with_gidx=False):
    """Synthetic trace on the host: (events, lens, offs, payload[, gidx]).
    shard=(count, index) keeps the events of connections hashing to index (config 5)."""
    k, size = trace_size(config, seed, first, n, align, shard, with_events=True)
    ev = np.zeros(k, EVENT_DTYPE)
    lens = np.zeros(k, np.uint32)
    offs = np.zeros(k, np.uint64)
    gidx = np.zeros(k, np.uint64)
    payload = np.zeros(size + 16, np.uint8)
    t = trace_config(config, seed, first, n, align, shard)
    _check(lib().ebd_trace_generate_host(C.byref(t), _p(ev), _p(lens), _p(offs), _p(payload), payload.size, _p(gidx)),
           "ebd_trace_generate_host")
    return (ev, lens, offs, payload, gidx) if with_gidx else (ev, lens, offs, payload)


def trace_size_device(ctx, config, seed, first, n, align=1, shard=(1, 0), with_events=False):
    t = trace_config(config, seed, first, n, align, shard)
    v, k = C.c_uint64(), C.c_uint32()
    _check(lib().ebd_trace_size_device(ctx.h, C.byref(t), C.byref(k), C.byref(v)), "ebd_trace_size_device")
    return (k.value, v.value) if with_events else v.value


def generate_device(ctx, config, seed, first, n, events, lens, offs, payload, payload_cap, align=1, shard=(1, 0),
                    gidx=None):
    t = trace_config(config, seed, first, n, align, shard)
    _check(lib().ebd_trace_generate_device(ctx.h, C.byref(t), _ptrval(events), _ptrval(lens), _ptrval(offs),
                                           _ptrval(payload), payload_cap, _ptrval(gidx)), "ebd_trace_generate_device")


# ---- host hooks (product semantics on the CPU, for tests) -------------------------------
def dfa_info():
    a = np.zeros(13, np.uint32)
    _check(lib().ebd_host_dfa_info(_p(a), 13), "dfa_info")
    keys = ["nstates", "url_id", "g2", "g3", "g4", "hvc0", "hvh", "fin0", "fin1", "inv", "init", "vl0", "vl1"]
    return dict(zip(keys, (int(x) for x in a)))


def _hkey(hash_key):
    return np.array(hash_key if hash_key is not None else TEST_HASH_KEY, np.uint64)


def dfa_next():
    """The fast-path DFA's transitions as an [nstates, 256] uint8 array."""
    t = np.zeros(256 * 256, np.uint8)
    n = lib().ebd_host_dfa_next(_p(t), t.size)
    if n < 0:
        raise EbdError("ebd_host_dfa_next")
    return t.reshape(256, 256)[:n].copy()


def host_fresh(buf: bytes, pid=0, flags=FLAG_IPV4 | FLAG_UNENCRYPTED | FLAG_NEW_DATA, src16=bytes(16), v4=(), v6=(),
               hash_key=None):
    out = np.zeros(1, RESULT_DTYPE)
    hk = _hkey(hash_key)
    key = np.zeros(2, np.uint64)
    b = np.frombuffer(buf, np.uint8) if buf else np.zeros(1, np.uint8)
    s = np.frombuffer(src16, np.uint8)
    v4, v6 = list(v4), list(v6)
    _check(lib().ebd_host_fresh(_p(b), len(buf), pid, flags, _p(s), _nets4(v4), len(v4), _nets6(v6), len(v6),
                                _p(hk), _p(out), _p(key)), "ebd_host_fresh")
    return out[0], (int(key[0]), int(key[1]))


def host_scan(buf: bytes, pid=0, flags=FLAG_IPV4 | FLAG_UNENCRYPTED | FLAG_NEW_DATA, src16=bytes(16), v4=(), v6=(),
              hash_key=None, shift=0, want_slow=False):
    """The structural fast path (k_fresh, ebd_scan.h) for one buffer at byte `shift` of its tile."""
    out = np.zeros(1, RESULT_DTYPE)
    hk = _hkey(hash_key)
    key = np.zeros(2, np.uint64)
    b = np.frombuffer(buf, np.uint8) if buf else np.zeros(1, np.uint8)
    s = np.frombuffer(src16, np.uint8)
    v4, v6 = list(v4), list(v6)
    rc = lib().ebd_host_scan(_p(b), len(buf), shift, pid, flags, _p(s), _nets4(v4), len(v4), _nets6(v6), len(v6),
                             _p(hk), _p(out), _p(key))
    _check(min(rc, 0), "ebd_host_scan")
    res = (out[0], (int(key[0]), int(key[1])))
    return res + (int(rc),) if want_slow else res


def host_gp_parse(chunks, flags=FLAG_UNENCRYPTED, reset_between=False, walker="gp"):
    """The generic parser (walker "gp") or the session path's DFA walker ("dfa") over the chunks."""
    data = b"".join(chunks)
    d = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    cl = np.array([len(c) for c in chunks], np.uint32) if chunks else np.zeros(1, np.uint32)
    cons = np.zeros(max(len(chunks), 1), np.uint32)
    o = np.zeros(12, np.uint32)
    fn = lib().ebd_host_gp_parse if walker == "gp" else lib().ebd_host_dfa_parse
    _check(fn(_p(d), _p(cl), len(chunks), flags, int(reset_between), _p(cons), _p(o)), "ebd_host_%s_parse" % walker)
    keys = ["state", "url_start", "url_len", "host_start", "host_len", "cip_start", "cip_len", "f", "cipkey", "mcand",
            "mlen", "proto"]
    return [int(x) for x in cons[:len(chunks)]], dict(zip(keys, (int(x) for x in o))), data


def host_classify_token(token: bytes, v4=(), v6=()):
    b = np.frombuffer(token, np.uint8) if token else np.zeros(1, np.uint8)
    v4, v6 = list(v4), list(v6)
    return lib().ebd_host_classify(_p(b), len(token), 0, 0, _nets4(v4), len(v4), _nets6(v6), len(v6))


def host_classify_source(src16: bytes, flags, v4=(), v6=()):
    b = np.frombuffer(src16, np.uint8)
    v4, v6 = list(v4), list(v6)
    return lib().ebd_host_classify(_p(b), 16, 1, flags, _nets4(v4), len(v4), _nets6(v6), len(v6))


def host_endpoint_key(pid: int, endpoint: bytes, hash_key=None):
    b = np.frombuffer(endpoint, np.uint8) if endpoint else np.zeros(1, np.uint8)
    key = np.zeros(2, np.uint64)
    hk = _hkey(hash_key)
    _check(lib().ebd_host_endpoint_key(_p(hk), pid, _p(b), len(endpoint), _p(key)), "ebd_host_endpoint_key")
    return int(key[0]), int(key[1])


def host_pton(text: bytes, af6: bool):
    b = np.frombuffer(text, np.uint8) if text else np.zeros(1, np.uint8)
    out = np.zeros(16, np.uint8)
    ok = lib().ebd_host_pton(1 if af6 else 0, _p(b), len(text), _p(out))
    return bytes(out[:16 if af6 else 4]) if ok else None
