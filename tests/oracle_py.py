"""ctypes binding of the CPU oracle (oracle/build/liboracle.so).

Test infrastructure: used only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker, never as the thing measured or shipped.
"""
import ctypes as C
import os
import subprocess
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "build", "liboracle.so")

EVENT_DTYPE = np.dtype([("pid", "<u4"), ("fd", "<u4"), ("sessionID", "<u4"), ("bufferSeq", "<u4"),
                        ("sourceIP", "u1", (16,)), ("flags", "u1"), ("pad", "u1", (3,))])
assert EVENT_DTYPE.itemsize == 36

RESULT_DTYPE = np.dtype([("kind", "<u4"), ("status", "<u4"), ("consumed", "<u4"), ("cls", "<u4"),
                         ("is_https", "<u4"), ("has_cip", "<u4"), ("host_off", "<u8"), ("url_off", "<u8"),
                         ("cip_off", "<u8"), ("host_len", "<u4"), ("url_len", "<u4"), ("cip_len", "<u4"),
                         ("pad", "<u4")])
assert RESULT_DTYPE.itemsize == 64

STATE_NAMES = ["METHOD", "SPACE_BEFORE_URL", "URL", "SPACE_BEFORE_PROTOCOL", "PROTOCOL", "HEADER_NEWLINE",
               "HEADER_KEY", "SPACE_BEFORE_HEADER_VALUE", "HEADER_VALUE", "HEADERS_END", "FINISHED", "INVALID"]


class Stats(C.Structure):
    _fields_ = [("kernel_deletes", C.c_uint64), ("lru_evictions", C.c_uint64), ("lru_size", C.c_uint64),
                ("requests", C.c_uint64), ("missing_buffers", C.c_uint64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(ORACLE_DIR, "oracle.c")
        if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = C.CDLL(LIB_PATH)
        vp, u8p = C.c_void_p, C.POINTER(C.c_uint8)
        L.orc_create.restype = vp
        L.orc_create.argtypes = [C.c_uint32]
        L.orc_destroy.argtypes = [vp]
        L.orc_set_interfaces.argtypes = [vp, vp, C.c_uint32, vp, C.c_uint32]
        L.orc_process.argtypes = [vp, vp, vp, vp, vp, C.c_uint32, vp]
        L.orc_process.restype = C.c_int
        L.orc_blob.argtypes = [vp, C.POINTER(C.c_char_p), C.POINTER(C.c_uint64)]
        L.orc_blob_reset.argtypes = [vp]
        L.orc_get_stats.argtypes = [vp, C.POINTER(Stats)]
        L.orc_services_dump.argtypes = [vp, vp, C.c_uint64]
        L.orc_services_dump.restype = C.c_uint64
        L.orc_services_dump_first.argtypes = [vp, vp, C.c_uint64]
        L.orc_services_dump_first.restype = C.c_uint64
        L.orc_service_count.argtypes = [vp]
        L.orc_service_count.restype = C.c_uint64
        L.orc_clear.argtypes = [vp]
        L.orc_agg_new_request.argtypes = [vp, C.c_uint32, C.c_char_p, C.c_char_p, C.c_char_p, C.c_uint8, vp]
        L.orc_set_checker_mock.argtypes = [vp, vp, C.c_uint32]
        L.orc_parser_new.restype = vp
        L.orc_parser_free.argtypes = [vp]
        L.orc_parser_parse.argtypes = [vp, C.c_char_p, C.c_size_t, C.c_uint8]
        L.orc_parser_parse.restype = C.c_size_t
        L.orc_parser_state.argtypes = [vp]
        L.orc_parser_state.restype = C.c_int
        L.orc_parser_reset.argtypes = [vp]
        L.orc_parser_result.argtypes = [vp, vp, C.c_uint64]
        L.orc_parser_result.restype = C.c_uint64
        L.orc_parse_client_ip.argtypes = [C.c_char_p, C.c_size_t, vp, C.c_uint64, C.POINTER(C.c_uint32)]
        L.orc_parse_client_ip.restype = C.c_uint64
        L.orc_inet_pton4.argtypes = [C.c_char_p, C.c_size_t, vp]
        L.orc_inet_pton6.argtypes = [C.c_char_p, C.c_size_t, vp]
        L.orc_inet_ntop4.argtypes = [vp, vp]
        L.orc_inet_ntop6.argtypes = [vp, vp]
        L.orc_is_v4_external.argtypes = [vp, vp]
        L.orc_is_v6_external.argtypes = [vp, vp]
        L.orc_lru_new.restype = vp
        L.orc_lru_new.argtypes = [C.c_uint32]
        L.orc_lru_free.argtypes = [vp]
        L.orc_lru_insert.argtypes = [vp, C.c_uint32, C.c_int64]
        L.orc_lru_find.argtypes = [vp, C.c_uint32, C.POINTER(C.c_int64)]
        L.orc_lru_erase.argtypes = [vp, C.c_uint32]
        L.orc_lru_update.argtypes = [vp, C.c_uint32, C.c_int64]
        L.orc_lru_size.argtypes = [vp]
        L.orc_lru_size.restype = C.c_uint32
        L.orc_set_network_counters.argtypes = [vp, C.c_int]
        L.orc_set_time.argtypes = [vp, C.c_uint64]
        L.orc_network_counters_cleaning.argtypes = [vp, C.c_uint64]
        for f in ("orc_services_dump_nets", "orc_nets_dump", "orc_services_json"):
            getattr(L, f).argtypes = [vp, vp, C.c_uint64]
            getattr(L, f).restype = C.c_uint64
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None and a.size else None


class Parser:
    """HttpRequestParser (HttpRequestParser.h:41-101) restated."""

    def __init__(self):
        self.h = lib().orc_parser_new()

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_parser_free(self.h)

    def parse(self, data: bytes, flags: int) -> int:
        return lib().orc_parser_parse(self.h, data, len(data), flags)

    @property
    def state(self):
        return STATE_NAMES[lib().orc_parser_state(self.h)]

    def reset(self):
        lib().orc_parser_reset(self.h)

    def result(self):
        n = lib().orc_parser_result(self.h, None, 0)
        buf = C.create_string_buffer(n)
        lib().orc_parser_result(self.h, buf, n)
        f = buf.raw[:n].split(b"\n")
        ips = f[6].split(b"\x1f") if f[6] else []
        return dict(method=f[0], url=f[1], protocol=f[2], host=f[3], client_ip_key=f[4], is_https=f[5] == b"1",
                    client_ip=ips)


def parse_client_ip(value: bytes):
    cnt = C.c_uint32()
    n = lib().orc_parse_client_ip(value, len(value), None, 0, C.byref(cnt))
    buf = C.create_string_buffer(max(n, 1))
    lib().orc_parse_client_ip(value, len(value), buf, n, C.byref(cnt))
    toks = buf.raw[:n].split(b"\x1f")
    assert len(toks) == cnt.value
    return toks


def pton4(text: bytes):
    out = (C.c_uint8 * 4)()
    return bytes(out) if lib().orc_inet_pton4(text, len(text), out) == 1 else None


def pton6(text: bytes):
    out = (C.c_uint8 * 16)()
    return bytes(out) if lib().orc_inet_pton6(text, len(text), out) == 1 else None


def ntop4(b: bytes):
    out = C.create_string_buffer(16)
    lib().orc_inet_ntop4(C.c_char_p(b), out)
    return out.value


def ntop6(b: bytes):
    out = C.create_string_buffer(46)
    lib().orc_inet_ntop6(C.c_char_p(b), out)
    return out.value


class LRU:
    def __init__(self, capacity):
        self.h = lib().orc_lru_new(capacity)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_lru_free(self.h)

    def insert(self, k, v):
        lib().orc_lru_insert(self.h, k, v)

    def find(self, k):
        v = C.c_int64()
        return v.value if lib().orc_lru_find(self.h, k, C.byref(v)) else None

    def erase(self, k):
        return lib().orc_lru_erase(self.h, k)

    def update(self, k, v):
        return lib().orc_lru_update(self.h, k, v)


def parse_services(text: bytes):
    out = []
    for line in text.split(b"\n"):
        if not line:
            continue
        pid, ep, dom, sch, i, e = line.split(b"\t")
        out.append((int(pid), ep, dom, sch, int(i), int(e)))
    return out


class Oracle:
    """Discovery + Aggregator replay (Discovery.cpp:73-198, Aggregator.cpp:155-168)."""

    def __init__(self, lru_capacity=8192, v4_ifaces=None, v6_ifaces=None, network_counters=False):
        self.h = lib().orc_create(lru_capacity)
        self.set_interfaces(v4_ifaces or [], v6_ifaces or [])
        if network_counters:
            lib().orc_set_network_counters(self.h, 1)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_destroy(self.h)

    def set_interfaces(self, v4, v6):
        a4 = np.frombuffer(b"".join(a + m for a, m in v4), np.uint8) if v4 else np.zeros(0, np.uint8)
        a6 = np.frombuffer(b"".join(a + m for a, m in v6), np.uint8) if v6 else np.zeros(0, np.uint8)
        lib().orc_set_interfaces(self.h, _ptr(a4), len(v4), _ptr(a6), len(v6))

    def process(self, events, lens, offs, payload):
        events = np.ascontiguousarray(events, dtype=EVENT_DTYPE)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        n = len(events)
        out = np.zeros(n, RESULT_DTYPE)
        lib().orc_blob_reset(self.h)
        rc = lib().orc_process(self.h, _ptr(events), _ptr(lens), _ptr(offs), _ptr(payload), n, _ptr(out))
        assert rc == 0
        p = C.c_char_p()
        sz = C.c_uint64()
        lib().orc_blob(self.h, C.byref(p), C.byref(sz))
        blob = C.string_at(p, sz.value) if sz.value else b""
        return out, blob

    def services(self):
        n = lib().orc_services_dump(self.h, None, 0)
        buf = C.create_string_buffer(max(n, 1))
        lib().orc_services_dump(self.h, buf, n)
        return parse_services(buf.raw[:n])

    def services_first(self):
        """services() rows with a 7th field: index of the event that created the service."""
        n = lib().orc_services_dump_first(self.h, None, 0)
        buf = C.create_string_buffer(max(n, 1))
        lib().orc_services_dump_first(self.h, buf, n)
        rows = []
        for line in buf.raw[:n].split(b"\n"):
            if not line:
                continue
            f = line.split(b"\t")
            rows.append((int(f[0]), f[1], f[2], f[3], int(f[4]), int(f[5]), int(f[6])))
        return rows

    def _text(self, fn):
        n = fn(self.h, None, 0)
        buf = C.create_string_buffer(max(n, 1))
        fn(self.h, buf, n)
        return buf.raw[:n]

    def services_nets(self):
        """services() rows with the sizes of the /16, /24 and v6 network maps appended."""
        rows = []
        for line in self._text(lib().orc_services_dump_nets).split(b"\n"):
            if line:
                f = line.split(b"\t")
                rows.append((int(f[0]), f[1], f[2], f[3]) + tuple(int(x) for x in f[4:]))
        return rows

    def nets(self):
        """sorted [(pid, endpoint, kind, prefix hex, time)] of every live network-map entry."""
        rows = []
        for line in self._text(lib().orc_nets_dump).split(b"\n"):
            if line:
                f = line.split(b"\t")
                rows.append((int(f[0]), f[1], int(f[2]), f[3].decode(), int(f[4])))
        return sorted(rows)

    def services_json(self):
        return self._text(lib().orc_services_json)

    def set_time(self, now_ns):
        lib().orc_set_time(self.h, now_ns)

    def network_counters_cleaning(self, now_ns):
        lib().orc_network_counters_cleaning(self.h, now_ns)

    def stats(self):
        s = Stats()
        lib().orc_get_stats(self.h, C.byref(s))
        return {k: getattr(s, k) for k, _ in Stats._fields_}

    def clear(self):
        lib().orc_clear(self.h)

    def new_request(self, pid, host, url, cip, flags, src16=None):
        src = (C.c_uint8 * 16)(*(src16 or bytes(16)))
        lib().orc_agg_new_request(self.h, pid, host, url, cip, flags, src)

    def set_mock(self, verdicts):
        a = np.array(verdicts, dtype=np.int32)
        lib().orc_set_checker_mock(self.h, _ptr(a), len(a))

    def is_v4_external(self, b4):
        return bool(lib().orc_is_v4_external(self.h, C.c_char_p(b4)))

    def is_v6_external(self, b16):
        return bool(lib().orc_is_v6_external(self.h, C.c_char_p(b16)))


_TRACE4 = None  # config 4: the trace sample the workers share (generated before the fork)


def _throughput_worker(args):
    config, seed, first, n, budget_s, shard = args
    import ebd
    from ebd import shard as sh
    o = Oracle()
    done, spent, at = 0, 0.0, first
    chunk = 100_000
    if shard is not None:  # config 4: this worker's connections (they interleave in the trace)
        ev, lens, offs, payload = _TRACE4
        keep = sh.shard_indices(ev, shard[0])[shard[1]].astype(np.int64)
        for a in range(0, keep.size, chunk):
            if spent >= budget_s:
                break
            k = keep[a:a + chunk]
            t = time.perf_counter()
            o.process(ev[k], lens[k], offs[k], payload)
            spent += time.perf_counter() - t
            done += k.size
        return done, spent
    while spent < budget_s:
        ev, lens, offs, payload = ebd.generate_host(config, seed, at, chunk)
        t = time.perf_counter()
        o.process(ev, lens, offs, payload)
        spent += time.perf_counter() - t
        done += len(ev)
        at += chunk
    return done, spent


def config4_sample(seed, budget_s, rate=500_000, cap=24_000_000):
    """The first events of the config-4 trace (it can only be generated from position 0):
    enough for budget_s of oracle work at `rate` events/s, at most `cap`."""
    import ebd
    return ebd.generate_host(4, seed, 0, int(min(cap, max(200_000, budget_s * rate))))


def host_cpu():
    """nproc, this process's affinity share and the CPU model of the host."""
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count() or 1, "affinity_share": share, "cpu_model": model}


def parallel_throughput(config, seed, budget_s, threads=None):
    """The oracle on `threads` host processes (default: the host's CPU share, at most 16 —
    the GPU box gives one GPU's job 16 cores), each on its own connection slice of the
    trace (one event per connection in configs 2/3/5, so index slices are connection
    shards) with its own Discovery/Aggregator state; aggregate events/s = total events /
    the slowest worker's busy time.  The per-worker tables would be merged as the GPUs'
    are; the merge is not timed here."""
    import multiprocessing as mp
    host = host_cpu()
    threads = threads or min(16, host["affinity_share"])
    if threads < 2:
        return None
    slice_ = 50_000_000
    if config == 4:  # connections interleave: every worker walks the same trace, keeping its connections
        global _TRACE4
        _TRACE4 = config4_sample(seed, budget_s * threads)
        jobs = [(config, seed, 0, slice_, budget_s, (threads, k)) for k in range(threads)]
        how = f"its own connections (hash(pid, fd, sessionID) mod workers) of the first {len(_TRACE4[0])} events of"
    else:  # one event per connection: index slices are connection shards
        jobs = [(config, seed, k * slice_, slice_, budget_s, None) for k in range(threads)]
        how = "its own connection slice of"
    with mp.get_context("fork").Pool(threads) as pool:
        res = pool.map(_throughput_worker, jobs)
    _TRACE4 = None
    done = sum(r[0] for r in res)
    busy = max(r[1] for r in res)
    return dict(value=done / busy, unit="events/s", cores=threads, kind="port", host=host,
                sample=f"{threads} processes x ~{budget_s:.0f} s, each on {how} the config-{config} "
                       f"trace (seed {seed}), {done} events in all; cores = min(16, affinity share): the GPU box gives "
                       f"one GPU's job 16 cores")
