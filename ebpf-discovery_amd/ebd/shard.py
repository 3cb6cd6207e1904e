"""Multi-GPU sharding and the final per-(pid, endpoint) merge.

Parser state lives per connection (pid, fd, sessionID) (Types.h:72-86; the session LRU key,
Discovery.h:47), so a trace shards by connection: every event of a connection goes to the
same GPU, in trace order.  Each GPU runs its own context over its shard with no data-path
collective.  The one exchange is at the end, the Aggregator merge:

  * every service carries its 128-bit key hash(pid, endpoint) (identical on every GPU), its
    uint32 counters and the trace position of the request that created it;
  * owner = key mod world: one all_to_all_single ships each service (and its endpoint bytes)
    to its owner, over RCCL on GPU tensors or gloo on CPU tensors;
  * the owner merges by key: counters add modulo 2^32 (Service.h:53-54 are uint32), domain
    and scheme come from the earliest creating request (Aggregator.cpp:155-168: the first
    request of a key creates the service, later ones only count);
  * the owners' disjoint tables gather on rank 0.

Inside one shard the events keep their trace order, so a shard's first arrival is its
earliest event; `global_index` maps a context's local event order to the trace position.
"""
import numpy as np

REC = np.dtype([("key_lo", "<u8"), ("key_hi", "<u8"), ("first", "<u8"), ("ep_off", "<u8"), ("pid", "<u4"),
                ("internal", "<u4"), ("external", "<u4"), ("ep_len", "<u4"), ("dom_off", "<u4"), ("dom_len", "<u4"),
                ("https", "u1"), ("pad", "u1", (7,))])
assert REC.itemsize == 64


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
    """64-bit hash of each event's connection (pid, fd, sessionID)."""
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
    """Services as REC records plus the endpoint bytes they point into."""

    def __init__(self, rec=None, strings=None):
        self.rec = rec if rec is not None else np.zeros(0, REC)
        self.strings = strings if strings is not None else np.zeros(0, np.uint8)

    @classmethod
    def from_context(cls, ctx, global_index=None, seq_offset=0):
        """The context's services (ebd_collect_services).  A service's first arrival is the
        context's event order of its creating request; global_index[local] (or local +
        seq_offset) turns it into a trace position."""
        raw, blob = ctx.services_raw()
        rec = np.zeros(raw.size, REC)
        for f in ("key_lo", "key_hi", "pid", "internal", "external"):
            rec[f] = raw[f]
        rec["ep_off"] = raw["endpoint_off"]
        rec["ep_len"] = raw["endpoint_len"]
        rec["dom_off"] = raw["domain_off"]
        rec["dom_len"] = raw["domain_len"]
        rec["https"] = raw["https"]
        local = raw["first_seq"].astype(np.uint64)
        rec["first"] = np.asarray(global_index, np.uint64)[local] if global_index is not None else local + np.uint64(
            seq_offset)
        return cls(rec, blob)

    @classmethod
    def from_rows(cls, rows, keys):
        """From (pid, endpoint, domain, scheme, internal, external, first) rows and their
        (key_lo, key_hi) keys (tests build tables from the oracle this way)."""
        rec = np.zeros(len(rows), REC)
        parts, off = [], 0
        for k, (row, key) in enumerate(zip(rows, keys)):
            pid, ep, dom, sch, i, e, first = row
            ep = bytes(ep)
            dom = bytes(dom)
            d0 = ep.find(dom) if dom else 0
            rec[k] = (key[0], key[1], first, off, pid, i, e, len(ep), max(d0, 0), len(dom), sch in (b"https", "https"),
                      (0,) * 7)
            parts.append(ep)
            off += len(ep)
        return cls(rec, np.frombuffer(b"".join(parts), np.uint8).copy() if parts else np.zeros(0, np.uint8))

    def merged(self):
        """One record per key: counters summed mod 2^32, the earliest creator's fields."""
        r = self.rec
        if r.size == 0:
            return ServiceTable(r.copy(), self.strings)
        order = np.lexsort((r["first"], r["key_hi"], r["key_lo"]))
        r = r[order]
        head = np.ones(r.size, bool)
        head[1:] = (r["key_lo"][1:] != r["key_lo"][:-1]) | (r["key_hi"][1:] != r["key_hi"][:-1])
        starts = np.flatnonzero(head)
        out = r[starts].copy()
        out["internal"] = (np.add.reduceat(r["internal"].astype(np.uint64), starts) & np.uint64(0xFFFFFFFF)).astype(
            np.uint32)
        out["external"] = (np.add.reduceat(r["external"].astype(np.uint64), starts) & np.uint64(0xFFFFFFFF)).astype(
            np.uint32)
        return ServiceTable(out, self.strings)

    def packed(self):
        """A copy whose strings hold exactly its records' endpoints, in record order."""
        r = self.rec.copy()
        lens = r["ep_len"].astype(np.int64)
        total = int(lens.sum())
        out = np.empty(total, np.uint8)
        new_off = np.zeros(r.size, np.int64)
        if r.size:
            new_off[1:] = np.cumsum(lens)[:-1]
        # gather in slices so the index array stays small
        step = 1 << 22
        k = 0
        while k < r.size:
            j = k
            acc = 0
            while j < r.size and (acc == 0 or acc + lens[j] <= step):
                acc += lens[j]
                j += 1
            sl = slice(k, j)
            L = lens[sl]
            if acc:
                base = np.repeat(r["ep_off"][sl].astype(np.int64) - new_off[sl], L)
                idx = np.arange(new_off[k], new_off[k] + acc, dtype=np.int64) + base
                out[new_off[k]:new_off[k] + acc] = self.strings[idx]
            k = j
        r["ep_off"] = new_off.astype(np.uint64)
        return ServiceTable(r, out)

    def rows(self):
        """[(pid, endpoint, domain, scheme, internal, external)] sorted by (pid, endpoint)."""
        s = self.strings.tobytes()
        out = []
        for r in self.rec:
            o, L = int(r["ep_off"]), int(r["ep_len"])
            ep = s[o:o + L]
            dom = ep[int(r["dom_off"]):int(r["dom_off"]) + int(r["dom_len"])]
            out.append((int(r["pid"]), ep, dom, b"https" if r["https"] else b"http", int(r["internal"]),
                        int(r["external"])))
        out.sort(key=lambda t: (t[0], t[1]))
        return out


def concat(tables):
    recs, blobs, base = [], [], 0
    for t in tables:
        r = t.rec.copy()
        r["ep_off"] += np.uint64(base)
        recs.append(r)
        blobs.append(t.strings)
        base += t.strings.size
    return ServiceTable(np.concatenate(recs) if recs else np.zeros(0, REC),
                        np.concatenate(blobs) if blobs else np.zeros(0, np.uint8))


def merge_tables(tables):
    return concat(tables).merged()


def _a2a_bytes(dist, send, splits, device, group):
    """all_to_all_single of a uint8 numpy buffer with per-rank byte splits."""
    import torch
    world = len(splits)
    cnt = torch.tensor(splits, dtype=torch.int64, device=device)
    rcnt = torch.empty_like(cnt)
    dist.all_to_all_single(rcnt, cnt, group=group)
    rsplits = [int(x) for x in rcnt.cpu()]
    out = torch.empty(max(sum(rsplits), 1), dtype=torch.uint8, device=device)
    inp = torch.from_numpy(send if send.size else np.zeros(1, np.uint8)).to(device)
    if sum(splits) == 0:
        inp = inp[:0]
    dist.all_to_all_single(out[:sum(rsplits)], inp, output_split_sizes=rsplits, input_split_sizes=list(splits),
                           group=group)
    assert len(rsplits) == world
    return out[:sum(rsplits)].cpu().numpy(), rsplits


def exchange_merge(table, device="cpu", group=None):
    """Owner-partitioned merge across the process group; returns the merged table on rank 0
    and None on the other ranks."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    t = table.merged()
    owner = (t.rec["key_lo"] % np.uint64(world)).astype(np.int64)
    order = np.argsort(owner, kind="stable")
    t = ServiceTable(t.rec[order], t.strings).packed()
    owner = owner[order]
    counts = np.bincount(owner, minlength=world)
    # endpoint offsets become relative to their owner's slice of the string bytes
    str_bytes = np.zeros(world, np.int64)
    np.add.at(str_bytes, owner, t.rec["ep_len"].astype(np.int64))
    str_start = np.zeros(world, np.int64)
    str_start[1:] = np.cumsum(str_bytes)[:-1]
    t.rec["ep_off"] -= str_start[owner].astype(np.uint64)
    rbytes, rsplit = _a2a_bytes(dist, t.rec.view(np.uint8).reshape(-1), [int(c) * REC.itemsize for c in counts], device,
                                group)
    sbytes, ssplit = _a2a_bytes(dist, t.strings, [int(x) for x in str_bytes], device, group)
    recv = rbytes.view(REC).copy()
    # rebase each source's offsets onto the received string bytes
    src_of = np.repeat(np.arange(world), [s // REC.itemsize for s in rsplit])
    sbase = np.zeros(world, np.int64)
    sbase[1:] = np.cumsum(ssplit)[:-1]
    recv["ep_off"] += sbase[src_of].astype(np.uint64)
    mine = ServiceTable(recv, sbytes).merged().packed()
    # gather the owners' disjoint tables on rank 0
    n = torch.tensor([mine.rec.size, mine.strings.size], dtype=torch.int64, device=device)
    sizes = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [(int(a), int(b)) for a, b in (s.cpu().tolist() for s in sizes)]
    mr = max(s[0] for s in sizes) * REC.itemsize
    ms = max(s[1] for s in sizes)
    payload = np.zeros(mr + ms, np.uint8)
    payload[:mine.rec.size * REC.itemsize] = mine.rec.view(np.uint8).reshape(-1)
    payload[mr:mr + mine.strings.size] = mine.strings
    buf = torch.from_numpy(payload).to(device)
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    if rank != 0:
        return None
    parts = []
    for (nr, ns), o in zip(sizes, outs):
        o = o.cpu().numpy()
        parts.append(ServiceTable(o[:nr * REC.itemsize].view(REC).copy(), o[mr:mr + ns].copy()))
    return concat(parts)
