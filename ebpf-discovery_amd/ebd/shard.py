"""Multi-GPU sharding and the final per-(pid, endpoint) merge.

Parser state lives per connection (pid, fd, sessionID) (Types.h:72-86; the session LRU key,
Discovery.h:47), so a trace shards by connection: every event of a connection goes to the
same GPU, in trace order.  Each GPU runs its own context over its shard with no data-path
collective.  The one exchange is at the end, the Aggregator merge:

  * every service carries its 128-bit key (a keyed PRF of pid + endpoint, the same on every
    GPU because the ranks share the key), its uint32 counters and the trace position of
    its first request with that request's scheme and host/url split;
  * owner = (key_lo >> 32) mod world (key_lo is always odd: its low bit marks a used slot).
    The GPU groups its services by owner on the device
    (ebd_export_services_device) and ONE all_to_all_single of 40-byte wire records and one
    of endpoint bytes ship each service to its owner, over RCCL (xGMI) on GPU tensors.  A
    record's bytes follow the previous record's (8-byte padded), so the received segments
    concatenate into one addressable table with no offsets to rebase;
  * endpoint bytes cross once per key the owner lacks (two rounds): the records go first,
    alone; the owner merges them (its own records first) and answers each source with one
    byte per record, set where that record created a service whose bytes it needs; the
    sources then send exactly those records' bytes (ebd_merge_service_keys_device,
    ebd_wire_compact_device, ebd_merge_service_bytes_device);
  * the owner merges on the device (ebd_merge_services_device): counters add modulo 2^32
    (Service.h:53-54 are uint32), the earliest first request fixes domain and scheme
    (Aggregator.cpp:155-168: the first request of a key creates the service, later ones
    only count).  The owners' tables are disjoint: together they are the merged table.

The same exchange runs over gloo on CPU tensors for the CPU tests, with the merge rule
restated in numpy (ServiceTable.merged) in place of the device kernel.

Inside one shard the events keep their trace order, so a shard's first arrival is its
earliest event; a context's first_seq is mapped to the trace position before the exchange.
"""
import numpy as np

from . import SERVICE_DTYPE, WIRE_DTYPE, WIRE_NO_BYTES

REC = WIRE_DTYPE  # the exchanged record: ebd_wire_service (include/ebpf_discovery_amd.h)
STR_SLACK = 64  # readable bytes past received endpoint strings (k_merge copies 8-byte words)
NO_OFF = np.uint64(0xFFFFFFFFFFFFFFFF)
M32 = np.uint64(0xFFFFFFFF)


def _fmix64(x):
    x = x.astype(np.uint64)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xFF51AFD7ED558CCD)
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xC4CEB9FE1A85EC53)
        x ^= x >> np.uint64(33)
    return x


def connection_hash(events):
    """64-bit hash of each event's connection (pid, fd, sessionID); ebd_gen.h conn_shard."""
    pid = events["pid"].astype(np.uint64)
    fd = events["fd"].astype(np.uint64)
    sid = events["sessionID"].astype(np.uint64)
    with np.errstate(over="ignore"):
        return _fmix64((pid | (fd << np.uint64(32))) ^ (sid * np.uint64(0x9E3779B97F4A7C15)))


def shard_indices(events, world):
    """Per rank, the trace positions of its events (ascending: trace order is kept)."""
    owner = (connection_hash(events) % np.uint64(world)).astype(np.int64)
    return [np.flatnonzero(owner == r).astype(np.uint64) for r in range(world)]


class ServiceTable:
    """Services as ebd_service records plus the endpoint bytes they point into."""

    def __init__(self, rec=None, strings=None):
        self.rec = rec if rec is not None else np.zeros(0, SERVICE_DTYPE)
        self.strings = strings if strings is not None else np.zeros(0, np.uint8)

    @classmethod
    def from_context(cls, ctx, global_index=None, seq_offset=0):
        """The context's services (ebd_collect_services).  A service's first arrival is the
        context's event order of its first request; global_index[local] (or local +
        seq_offset) turns it into a trace position."""
        raw, blob = ctx.services_raw()
        rec = raw.copy()
        local = raw["first_seq"].astype(np.uint64)
        rec["first_seq"] = (np.asarray(global_index, np.uint64)[local] if global_index is not None
                            else local + np.uint64(seq_offset))
        return cls(rec, blob)

    @classmethod
    def from_rows(cls, rows, keys):
        """From (pid, endpoint, domain, scheme, internal, external, first) rows and their
        (key_lo, key_hi) keys (tests build tables from the oracle this way)."""
        rec = np.zeros(len(rows), SERVICE_DTYPE)
        parts, off = [], 0
        for k, (row, key) in enumerate(zip(rows, keys)):
            pid, ep, dom, sch, i, e, first = row
            ep, dom = bytes(ep), bytes(dom)
            d0 = max(ep.find(dom), 0) if dom else 0
            r = rec[k]
            r["pid"], r["internal"], r["external"] = pid, i, e
            r["https"] = sch in (b"https", "https")
            r["endpoint_off"], r["endpoint_len"] = off, len(ep)
            r["domain_off"], r["domain_len"] = d0, len(dom)
            r["host_len"] = d0 + len(dom)  # a host whose domain is this one (host_domain gives it back)
            r["first_seq"], r["key_lo"], r["key_hi"] = first, key[0], key[1]
            rec[k] = r
            parts.append(ep)
            off += len(ep)
        return cls(rec, np.frombuffer(b"".join(parts), np.uint8).copy() if parts else np.zeros(0, np.uint8))

    def merged(self):
        """One record per key: counters summed mod 2^32, the earliest first request's
        fields (the merge rule of k_merge, restated for the CPU path)."""
        r = self.rec
        if r.size == 0:
            return ServiceTable(r.copy(), self.strings)
        order = np.lexsort((r["first_seq"], r["key_hi"], r["key_lo"]))
        r = r[order]
        head = np.ones(r.size, bool)
        head[1:] = (r["key_lo"][1:] != r["key_lo"][:-1]) | (r["key_hi"][1:] != r["key_hi"][:-1])
        starts = np.flatnonzero(head)
        out = r[starts].copy()
        for f in ("internal", "external"):
            out[f] = (np.add.reduceat(r[f].astype(np.uint64), starts) & M32).astype(np.uint32)
        return ServiceTable(out, self.strings)

    def packed(self):
        """A copy whose strings hold exactly its records' endpoints, in record order."""
        r = self.rec.copy()
        lens = r["endpoint_len"].astype(np.int64)
        new_off = np.zeros(r.size, np.int64)
        if r.size:
            new_off[1:] = np.cumsum(lens)[:-1]
        out = np.empty(int(lens.sum()), np.uint8)
        step, k = 1 << 22, 0
        while k < r.size:  # gather in slices so the index array stays small
            j, acc = k, 0
            while j < r.size and (acc == 0 or acc + lens[j] <= step):
                acc += lens[j]
                j += 1
            if acc:
                sl = slice(k, j)
                base = np.repeat(r["endpoint_off"][sl].astype(np.int64) - new_off[sl], lens[sl])
                idx = np.arange(new_off[k], new_off[k] + acc, dtype=np.int64) + base
                out[new_off[k]:new_off[k] + acc] = self.strings[idx]
            k = j
        r["endpoint_off"] = new_off.astype(np.uint64)
        return ServiceTable(r, out)

    def to_wire(self, world):
        """(wire records grouped by owner, their endpoint bytes in record order, each padded
        to 8, counts[world], str_counts[world]): what ebd_export_services_device returns."""
        owner = owner_np(self.rec["key_lo"], world)
        order = np.argsort(owner, kind="stable")
        r, owner = self.rec[order], owner[order]
        w = np.zeros(r.size, REC)
        for f in ("key_lo", "key_hi", "pid", "internal", "external"):
            w[f] = r[f]
        w["first"] = ((r["first_seq"].astype(np.uint64) << np.uint64(16)) | (r["https"].astype(np.uint64) << np.uint64(15))
                      | (r["host_len"].astype(np.uint64) & np.uint64(0x7FFF)))
        has = r["endpoint_off"] != NO_OFF
        w["endpoint_len"] = np.where(has, r["endpoint_len"], r["endpoint_len"] | np.uint32(WIRE_NO_BYTES))
        nb = wire_bytes(w["endpoint_len"])
        out = np.zeros(int(nb.sum()), np.uint8)
        at = 0
        blob = self.strings
        for k in range(r.size):
            if has[k]:
                o, L = int(r["endpoint_off"][k]), int(r["endpoint_len"][k])
                out[at:at + L] = blob[o:o + L]
            at += int(nb[k])
        counts = np.bincount(owner, minlength=world).astype(np.uint32)
        scounts = np.zeros(world, np.uint64)
        np.add.at(scounts, owner, nb)
        return w, out, counts, scounts

    @classmethod
    def from_wire(cls, w, strings):
        """Received wire records (and their bytes) as a table: endpoint offsets from the scan
        of the padded lengths, domain and scheme from the first-arrival word (k_collect)."""
        nb = wire_bytes(w["endpoint_len"])
        offs = np.zeros(w.size, np.uint64)
        if w.size:
            offs[1:] = np.cumsum(nb)[:-1]
        r = np.zeros(w.size, SERVICE_DTYPE)
        for f in ("key_lo", "key_hi", "pid", "internal", "external"):
            r[f] = w[f]
        first = w["first"].astype(np.uint64)
        r["first_seq"] = first >> np.uint64(16)
        r["https"] = ((first >> np.uint64(15)) & np.uint64(1)).astype(np.uint8)
        r["host_len"] = (first & np.uint64(0x7FFF)).astype(np.uint32)
        none = (w["endpoint_len"] & np.uint32(WIRE_NO_BYTES)) != 0
        r["endpoint_len"] = w["endpoint_len"] & np.uint32(~WIRE_NO_BYTES & 0xFFFFFFFF)
        r["endpoint_off"] = np.where(none, NO_OFF, offs)
        s = strings.tobytes() if hasattr(strings, "tobytes") else bytes(strings)
        for k in np.flatnonzero(~none):
            o = int(offs[k])
            hl = min(int(r["host_len"][k]), int(r["endpoint_len"][k]))
            r["domain_off"][k], r["domain_len"][k] = host_domain(s[o:o + hl])
        return cls(r, np.frombuffer(s, np.uint8).copy() if s else np.zeros(0, np.uint8))

    def rows(self):
        """[(pid, endpoint, domain, scheme, internal, external)] sorted by (pid, endpoint)."""
        s = self.strings.tobytes()
        out = []
        for r in self.rec:
            o, L = int(r["endpoint_off"]), int(r["endpoint_len"])
            ep = s[o:o + L]
            dom = ep[int(r["domain_off"]):int(r["domain_off"]) + int(r["domain_len"])]
            out.append((int(r["pid"]), ep, dom, b"https" if r["https"] else b"http", int(r["internal"]),
                        int(r["external"])))
        out.sort(key=lambda t: (t[0], t[1]))
        return out


def concat(tables):
    recs, blobs, base = [], [], 0
    for t in tables:
        r = t.rec.copy()
        r["endpoint_off"] += np.uint64(base)
        recs.append(r)
        blobs.append(t.strings)
        base += t.strings.size
    return ServiceTable(np.concatenate(recs) if recs else np.zeros(0, SERVICE_DTYPE),
                        np.concatenate(blobs) if blobs else np.zeros(0, np.uint8))


def merge_tables(tables):
    return concat(tables).merged()


def exchange(recs, strings, counts, scounts, group=None):
    """One all_to_all_single of the owner-grouped records and one of their endpoint bytes
    (torch uint8 tensors on the group's device: RCCL on GPU tensors, gloo on CPU ones).
    Returns (records, strings) received: segments in source order, addressable as they are."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = recs.device
    # per destination rank: (records, string bytes)
    sizes = torch.tensor(np.stack([counts.astype(np.int64), scounts.astype(np.int64)], axis=1).reshape(-1), device=dev)
    rsizes = torch.empty_like(sizes)
    dist.all_to_all_single(rsizes, sizes, output_split_sizes=[2] * world, input_split_sizes=[2] * world, group=group)
    rs = rsizes.view(world, 2).cpu().numpy()  # per source: (records, string bytes) for me
    rcounts, rscounts = rs[:, 0], rs[:, 1]
    nrec = REC.itemsize
    out_r = torch.empty(int(rcounts.sum()) * nrec, dtype=torch.uint8, device=dev)
    dist.all_to_all_single(out_r, recs, output_split_sizes=[int(c) * nrec for c in rcounts],
                           input_split_sizes=[int(c) * nrec for c in counts], group=group)
    # STR_SLACK bytes past the received strings: the merge copies endpoints in whole 8-byte words
    nstr = int(rscounts.sum())
    out_s = torch.zeros(nstr + STR_SLACK, dtype=torch.uint8, device=dev)
    dist.all_to_all_single(out_s[:nstr], strings, output_split_sizes=[int(c) for c in rscounts],
                           input_split_sizes=[int(c) for c in scounts], group=group)
    return out_r, out_s


def exchange_merge(table, device="cpu", group=None, two_round=True, stats=None):
    """CPU path: owner-partitioned exchange of a ServiceTable, merged by the numpy rule on
    each owner.  Returns this rank's owned part of the merged table.  two_round: the key
    round, the owner's need flags, then only the needed bytes (device_exchange_merge's
    protocol, with claimers() in place of the device claims); stats gets the bytes sent."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    rec, strings, counts, scounts = table.merged().to_wire(world)
    r = torch.from_numpy(rec.view(np.uint8).reshape(-1).copy()).to(device)
    if not two_round:
        s = torch.from_numpy(strings.copy()).to(device)
        out_r, out_s = exchange(r, s, counts, scounts, group)
        mine = ServiceTable.from_wire(out_r.cpu().numpy().view(REC).copy(), out_s.cpu().numpy()[:out_s.numel() - STR_SLACK])
        if stats is not None:
            stats.update(record_bytes=rec.nbytes, string_bytes=int(strings.size), need_bytes=0)
        return mine.merged().packed()
    out_r, rc = exchange_counts(r, counts, REC.itemsize, group)
    got = out_r.cpu().numpy().view(REC).copy()
    need = claimers(got, rc, rank)
    back = return_to_sources(torch.from_numpy(need.astype(np.uint8)).to(device), rc, counts, group)
    mask = back.cpu().numpy().astype(bool)
    nb = wire_bytes(rec["endpoint_len"])
    soff = np.zeros(nb.size, np.int64)
    soff[1:] = np.cumsum(nb.astype(np.int64))[:-1]
    sel = np.flatnonzero(mask)
    sent = np.concatenate([strings[soff[k]:soff[k] + int(nb[k])] for k in sel]) if sel.size else np.zeros(0, np.uint8)
    owner = np.repeat(np.arange(world), counts.astype(np.int64))
    bc = np.bincount(owner[sel], weights=nb[sel].astype(np.float64), minlength=world).astype(np.int64)
    out_s, _ = exchange_counts(torch.from_numpy(sent.astype(np.uint8)).to(device), bc, 1, group)
    if stats is not None:
        stats.update(record_bytes=rec.nbytes, string_bytes=int(sent.size), need_bytes=int(need.size),
                     string_bytes_one_round=int(strings.size))
    return merged_with_bytes(got, need, out_s.cpu().numpy())


def return_to_sources(flags, rc, counts, group=None):
    """One uint8 per received record (rc[s] from source s, in source order) back to the record's
    source, which gets counts[w] flags from owner w in the order it sent them.  Both sides know
    the sizes already (the record exchange's), so nothing is read back to the host."""
    import torch
    import torch.distributed as dist
    out = torch.empty(int(np.sum(counts)), dtype=torch.uint8, device=flags.device)
    dist.all_to_all_single(out, flags, output_split_sizes=[int(c) for c in counts],
                           input_split_sizes=[int(c) for c in rc], group=group)
    return out


def claimers(w, rc, rank):
    """The records whose bytes an owner asks for (received records w, rc[s] from source s in
    source order): per key, the first record that has bytes, the owner's own records first,
    then in source order.  The device path claims in the same spirit (own records merged
    first); which sender's copy it takes does not matter, every copy of a key is the same."""
    n = w.size
    need = np.zeros(n, np.uint8)
    if n == 0:
        return need
    starts = np.concatenate([[0], np.cumsum(rc)[:-1]]).astype(np.int64)
    pref = np.ones(n, np.int64)
    pref[starts[rank]:starts[rank] + int(rc[rank])] = 0
    has = (w["endpoint_len"] & np.uint32(WIRE_NO_BYTES)) == 0
    order = np.lexsort((np.arange(n), pref, ~has, w["key_hi"], w["key_lo"]))
    kl, kh = w["key_lo"][order], w["key_hi"][order]
    head = np.ones(n, bool)
    head[1:] = (kl[1:] != kl[:-1]) | (kh[1:] != kh[:-1])
    first = order[head]
    need[first[has[first]]] = 1
    return need


def merged_with_bytes(w, need, strings):
    """The owner's table from received records and the bytes of the needed ones (in record
    order): one record per key, counters summed mod 2^32, the earliest first request's fields,
    the endpoint from whichever record carried it, the domain from the earliest host length."""
    nb = wire_bytes(w["endpoint_len"]) * need.astype(np.uint64)
    offs = np.zeros(w.size, np.uint64)
    if w.size:
        offs[1:] = np.cumsum(nb)[:-1]
    t = ServiceTable.from_wire(w, np.zeros(0, np.uint8))
    r = t.rec
    r["endpoint_off"] = np.where(need.astype(bool), offs, NO_OFF)
    if r.size == 0:
        return ServiceTable(r, np.zeros(0, np.uint8))
    order = np.lexsort((r["first_seq"], r["key_hi"], r["key_lo"]))
    r = r[order]
    head = np.ones(r.size, bool)
    head[1:] = (r["key_lo"][1:] != r["key_lo"][:-1]) | (r["key_hi"][1:] != r["key_hi"][:-1])
    starts = np.flatnonzero(head)
    out = r[starts].copy()
    for f in ("internal", "external"):
        out[f] = (np.add.reduceat(r[f].astype(np.uint64), starts) & M32).astype(np.uint32)
    out["endpoint_off"] = np.minimum.reduceat(r["endpoint_off"], starts)  # the one carried copy (NO_OFF: none)
    s = strings.tobytes()
    for k in range(out.size):
        o = out["endpoint_off"][k]
        if o == NO_OFF:
            out["domain_off"][k] = out["domain_len"][k] = 0
            continue
        o = int(o)
        hl = min(int(out["host_len"][k]), int(out["endpoint_len"][k]))
        out["domain_off"][k], out["domain_len"][k] = host_domain(s[o:o + hl])
    return ServiceTable(out, np.frombuffer(s, np.uint8).copy() if s else np.zeros(0, np.uint8)).packed()


def gather_rows(table, group=None):
    """Rank 0 receives every rank's rows (for tests and small tables)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    parts = [None] * world
    dist.all_gather_object(parts, table.rows(), group=group)
    rows = [r for p in parts for r in p]
    rows.sort(key=lambda t: (t[0], t[1]))
    return rows


def device_exchange_merge(ctx, device, group=None, map_first=None, two_round=True):
    """GPU path: export by owner on the device, exchange over RCCL, merge on the device into
    this rank's context (reset first).  two_round (default): records alone, the owner's need
    flags back, then only the needed endpoint bytes (module docstring); else one round of
    records and every record's bytes.  With network counters the services' network-map
    entries follow their services to the owner (one more all_to_all of 32-byte records) and
    merge into its maps (union, later last-seen time).  map_first(first_seq int64 tensor) ->
    trace positions, applied before the exchange.

    Host reads (D2H) per interval: the export leaves its per-owner counts on the device, they go
    through the size all-to-all as they are, and ONE read takes both what this rank sends and what
    it receives (records and string bytes).  That is the whole interval for one round.  The two-round
    protocol reads once more: the bytes round's counts exist only after the owner's key merge has
    decided which records it needs, so they are read (one D2H of both sides' counts, made by a
    kernel of the library, ebd_wire_segment_bytes_device) between the two rounds.  Network maps,
    when on, add the read of their record counts.

    Returns {sent, received, record_bytes, string_bytes, need_bytes, string_bytes_one_round,
    net_sent, net_received, export_ms, merge_ms, exchange_ms, host_reads}."""
    import time
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    t0 = time.perf_counter()
    check_same_hash_key(ctx, device, group)  # once per context and group
    recs_all, strs_all, sizes = ctx.export_services_device_sized(world, device)  # sizes: device [2, world]
    nets = ncounts = None
    d2h = 0
    if getattr(ctx, "network_counters", False):
        nets, ncounts = group_by_owner(ctx.networks_device(device), NET_REC_BYTES, world)
        d2h += 2  # the map dump's count and the grouping's counts
    # per destination (records, string bytes); the size all-to-all takes them from the device
    send = sizes.t().contiguous()  # [world, 2]
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    both = torch.cat([send.reshape(-1), recv.reshape(-1)]).cpu().numpy().astype(np.int64)  # the interval's read
    d2h += 1
    counts, scounts = both[0:2 * world:2], both[1:2 * world:2]
    rc, rsc = both[2 * world::2], both[2 * world + 1::2]
    n_out, s_out = int(counts.sum()), int(scounts.sum())
    rb = REC.itemsize
    recs, strs = recs_all[:n_out * rb], strs_all[:s_out]
    if map_first is not None:
        map_wire_first(recs, map_first)
    t_export = time.perf_counter()
    t_merge = 0.0  # the device merges' share (each C call returns when its work is done)
    n_in = int(rc.sum())
    out_r = torch.empty(n_in * rb, dtype=torch.uint8, device=device)
    dist.all_to_all_single(out_r, recs, output_split_sizes=[int(c) * rb for c in rc],
                           input_split_sizes=[int(c) * rb for c in counts], group=group)
    if not two_round:
        ns = int(rsc.sum())
        out_s = torch.zeros(ns + STR_SLACK, dtype=torch.uint8, device=device)
        dist.all_to_all_single(out_s[:ns], strs, output_split_sizes=[int(c) for c in rsc],
                               input_split_sizes=[int(c) for c in scounts], group=group)
        tm = time.perf_counter()
        ctx.reset_services()
        ctx.merge_services_device(out_r, out_s)
        t_merge += time.perf_counter() - tm
        sent_bytes, need_bytes = s_out, 0
    else:
        tm = time.perf_counter()
        ctx.reset_services()
        dst = torch.empty(n_in, dtype=torch.int64, device=device)
        a = int(np.sum(rc[:rank]))
        b = a + int(rc[rank])
        # the owner's own records first: they create its services, and their bytes stay local
        ctx.merge_service_keys_device(out_r[a * rb:b * rb], dst[a:b])
        ctx.merge_service_keys_device(out_r[:a * rb], dst[:a])
        ctx.merge_service_keys_device(out_r[b * rb:], dst[b:])
        t_merge += time.perf_counter() - tm
        need_in = (dst >= 0).to(torch.uint8)
        # one flag per record back to its source: both sides know the sizes (the records' counts)
        need = return_to_sources(need_in, rc, counts, group)
        packed = ctx.wire_compact_device(recs, strs, need, sized=False)
        # the bytes round's counts: per owner here, per source on the owner side, from the device
        # in one read (both made by k_wire_seg_bytes; no count exchange: each side has both records)
        bc = ctx.wire_segment_bytes_device(recs, send[:, 0], need=need)
        rbc = ctx.wire_segment_bytes_device(out_r, recv[:, 0], dst=dst)
        hb = torch.cat([bc, rbc]).cpu().numpy().astype(np.int64)
        d2h += 1
        ns = int(hb[world:].sum())
        out_s = torch.zeros(ns + STR_SLACK, dtype=torch.uint8, device=device)
        dist.all_to_all_single(out_s[:ns], packed[:int(hb[:world].sum())],
                               output_split_sizes=[int(c) for c in hb[world:]],
                               input_split_sizes=[int(c) for c in hb[:world]], group=group)
        tm = time.perf_counter()
        ctx.merge_service_bytes_device(out_r, dst, out_s)
        t_merge += time.perf_counter() - tm
        sent_bytes, need_bytes = int(hb[:world].sum()), need_in.numel()
    out_n = None
    if nets is not None:
        out_n = exchange_fixed(nets, ncounts, NET_REC_BYTES, group)
        d2h += 1
        tm = time.perf_counter()
        ctx.merge_networks_device(out_n)
        t_merge += time.perf_counter() - tm
    t_end = time.perf_counter()
    return {"sent": n_out, "received": n_in,
            "record_bytes": recs.numel(), "string_bytes": sent_bytes, "need_bytes": need_bytes,
            "string_bytes_one_round": s_out,
            "net_sent": int(ncounts.sum()) if ncounts is not None else 0,
            "net_received": out_n.numel() // NET_REC_BYTES if out_n is not None else 0,
            "export_ms": (t_export - t0) * 1e3, "merge_ms": t_merge * 1e3,
            "exchange_ms": (t_end - t_export - t_merge) * 1e3, "host_reads": d2h}


NET_REC_BYTES = 32  # ebd_service_net


def owner_of(key_lo, world):
    """The owner GPU of uint64 keys held in an int64 tensor: (key_lo >> 32) % world (ebd_kernels.hip
    owner_of)."""
    return ((key_lo >> 32) & 0xFFFFFFFF) % world


def owner_np(key_lo, world):
    """owner_of for a numpy uint64 array."""
    return ((np.asarray(key_lo, np.uint64) >> np.uint64(32)) % np.uint64(world)).astype(np.int64)


def group_by_owner(recs, size, world):
    """Records (uint8 tensor of `size`-byte records starting with key_lo) reordered by owner
    (stable); returns (records, counts[world] numpy)."""
    import torch
    n = recs.numel() // size
    if n == 0:
        return recs, np.zeros(world, np.int64)
    key_lo = recs.view(torch.int64).view(n, size // 8)[:, 0]
    own = owner_of(key_lo, world)
    order = torch.argsort(own, stable=True)
    out = recs.view(n, size)[order].reshape(-1)
    return out, torch.bincount(own, minlength=world).cpu().numpy().astype(np.int64)


def exchange_counts(recs, counts, size, group=None, slack=0):
    """exchange_fixed that also returns the counts received from each source (numpy int64);
    the output has `slack` zero bytes past the received ones."""
    import torch
    import torch.distributed as dist
    dev = recs.device
    sizes = torch.tensor(np.asarray(counts, np.int64), device=dev)
    rsizes = torch.empty_like(sizes)
    dist.all_to_all_single(rsizes, sizes, group=group)
    rc = rsizes.cpu().numpy().astype(np.int64)
    nout = int(rc.sum()) * size
    out = torch.zeros(nout + slack, dtype=torch.uint8, device=dev)
    dist.all_to_all_single(out[:nout], recs, output_split_sizes=[int(c) * size for c in rc],
                           input_split_sizes=[int(c) * size for c in counts], group=group)
    return (out if slack else out[:nout]), rc


def exchange_fixed(recs, counts, size, group=None):
    """One all_to_all_single of owner-grouped fixed-size records (counts per destination)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = recs.device
    sizes = torch.tensor(np.asarray(counts, np.int64), device=dev)
    rsizes = torch.empty_like(sizes)
    dist.all_to_all_single(rsizes, sizes, group=group)
    rc = rsizes.cpu().numpy()
    out = torch.empty(int(rc.sum()) * size, dtype=torch.uint8, device=dev)
    dist.all_to_all_single(out, recs, output_split_sizes=[int(c) * size for c in rc],
                           input_split_sizes=[int(c) * size for c in counts], group=group)
    return out


def map_wire_first(recs, fn):
    """In place on device wire records (uint8 tensor): the first-arrival word's sequence
    number (bits 16..63) through fn (int64 tensor -> int64 tensor)."""
    if recs.numel() == 0:
        return
    words = recs.view(torch_int64()).view(-1, REC.itemsize // 8)
    f = words[:, 2]
    words[:, 2] = (fn(f >> 16) << 16) | (f & 0xFFFF)


def wire_bytes(lens):
    """Bytes each wire record's endpoint takes in the strings (EBD_WIRE_BYTES)."""
    lens = np.asarray(lens, np.uint32)
    return np.where((lens & np.uint32(WIRE_NO_BYTES)) != 0, 0, (lens.astype(np.uint64) + 7) & ~np.uint64(7)).astype(np.uint64)


def host_domain(host):
    """(offset, length) of the domain in a Host value (ebd_spec.h host_domain,
    Aggregator.cpp:112-130): "[...]" through the first ']' after the first '[' (empty
    without one), else the host up to its first ':'."""
    lb = host.find(b"[")
    if lb >= 0:
        rb = host.find(b"]", lb + 1)
        return (lb, rb - lb + 1) if rb >= 0 else (0, 0)
    c = host.find(b":")
    return 0, (c if c >= 0 else len(host))


def check_same_hash_key(ctx, device, group=None):
    """Owners come from the key: a rank keyed with another secret would send the same
    (pid, endpoint) to another owner and the merged table would hold it twice.  Raises unless
    every rank's context uses the same service-key secret."""
    import torch
    import torch.distributed as dist
    tag = (id(group), dist.get_world_size(group))
    if getattr(ctx, "_hash_key_checked", None) == tag:  # the key is fixed per context: once per group
        return
    mine = torch.tensor(np.array(ctx.hash_key, np.uint64).view(np.int64), device=device)
    parts = [torch.empty_like(mine) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, mine, group=group)
    if any(not torch.equal(p, mine) for p in parts):
        raise ValueError("device_exchange_merge: ranks key services with different secrets (pass one hash_key)")
    ctx._hash_key_checked = tag


def torch_int64():
    import torch
    return torch.int64
