"""Multi-GPU path on CPU: connection sharding + the owner-partitioned service merge
(ebd.shard) over a world_size-2 gloo group.

Each rank takes its connection shard of a trace (generated sharded, as bench.py does for
config 5: ebd.generate_host(..., shard=(world, rank)), the same events as
ebd.shard.shard_indices), replays it with the oracle (the stand-in for that rank's GPU
context: this test has no GPU), keys its services with the product's 128-bit endpoint key,
and merges through ebd.shard.exchange_merge: the device path's owner grouping and
all_to_all exchange, with the merge rule in numpy in place of k_merge.  The owners' tables
gathered on rank 0 must equal the oracle over the whole trace: (pid, endpoint, domain,
scheme, internal, external), bit-exact.
"""
import datetime
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import ebd
from ebd import shard
import oracle_py as O
import traces


def _trace(kind):
    if kind == "config3":
        return ebd.generate_host(3, 7, 0, 6000)
    if kind == "config5":
        return ebd.generate_host(5, 5, 0, 6000)
    return traces.fragmented_trace(300, seed=9, window=64)


def _shard_table(ev, lens, offs, payload, idx):
    """One rank's services, from the oracle over its shard (trace order kept)."""
    o = O.Oracle()
    o.process(ev[idx], lens[idx], offs[idx], payload)
    rows = []
    for (pid, ep, dom, sch, i, e, first) in o.services_first():
        rows.append((pid, ep, dom, sch, i, e, int(idx[first])))  # local order -> trace position
    keys = [ebd.host_endpoint_key(r[0], r[1]) for r in rows]
    return shard.ServiceTable.from_rows(rows, keys)


def _worker(rank, world, port, kind, out_path, two_round=True):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    try:
        ev, lens, offs, payload = _trace(kind)
        idx = shard.shard_indices(ev, world)[rank]
        if kind == "config5":  # the shard generated directly, as on the GPU
            sev, sl, so, sp, gidx = ebd.generate_host(5, 5, 0, 6000, shard=(world, rank), with_gidx=True)
            assert np.array_equal(gidx, idx) and np.array_equal(sev, ev[idx])
        table = _shard_table(ev, lens, offs, payload, idx)
        stats = {}
        mine = shard.exchange_merge(table, device="cpu", two_round=two_round, stats=stats)
        owner = shard.owner_np(mine.rec["key_lo"], world)
        assert np.all(owner == rank)  # every merged service is on its owner
        rows = shard.gather_rows(mine)
        parts = [None] * world
        dist.all_gather_object(parts, stats)
        if rank == 0:
            with open(out_path, "w") as f:
                json.dump({"rows": [[p, ep.decode("latin-1"), dom.decode("latin-1"), sch.decode(), i, e]
                                    for (p, ep, dom, sch, i, e) in rows], "stats": parts}, f)
    finally:
        dist.destroy_process_group()


def _run_merge(kind, tmp_path, two_round=True, world=2):
    out_path = str(tmp_path / f"merged_{kind}_{int(two_round)}.json")
    mp.start_processes(_worker, args=(world, _free_port(), kind, out_path, two_round), nprocs=world, join=True,
                       start_method="spawn")
    with open(out_path) as f:
        got = json.load(f)
    rows = [(p, ep.encode("latin-1"), dom.encode("latin-1"), sch.encode(), i, e) for p, ep, dom, sch, i, e in got["rows"]]
    return rows, got["stats"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("kind", ["config3", "config5", "fragmented"])
def test_two_rank_merge_equals_whole_trace(kind, tmp_path):
    merged, _ = _run_merge(kind, tmp_path)
    ev, lens, offs, payload = _trace(kind)
    o = O.Oracle()
    o.process(ev, lens, offs, payload)
    want = sorted(o.services(), key=lambda t: (t[0], t[1]))
    assert len(merged) == len(want)
    assert merged == want


def test_two_round_exchange_ships_bytes_once_per_new_key(tmp_path):
    """The key round, the owners' need flags and the bytes round give the one-round table,
    and endpoint bytes cross only for keys their owner lacked: fewer bytes than one round
    (config 3's Zipf keys recur across shards), at most one copy per merged key."""
    two, st2 = _run_merge("config3", tmp_path, two_round=True)
    one, st1 = _run_merge("config3", tmp_path, two_round=False)
    assert two == one
    sent2 = sum(s["string_bytes"] for s in st2)
    sent1 = sum(s["string_bytes"] for s in st1)
    assert sent1 == sum(s["string_bytes_one_round"] for s in st2)
    assert 0 < sent2 < sent1
    # at most one copy of each merged key's endpoint (8-byte padded)
    assert sent2 <= sum((len(ep) + 7) // 8 * 8 for (_, ep, _, _, _, _) in two)


def test_shards_keep_connections_and_order():
    ev, lens, offs, payload = _trace("fragmented")
    parts = shard.shard_indices(ev, 4)
    allidx = np.sort(np.concatenate(parts))
    assert np.array_equal(allidx, np.arange(len(ev), dtype=np.uint64))
    owner = {}
    for r, p in enumerate(parts):
        assert np.all(np.diff(p.astype(np.int64)) > 0)  # trace order inside a shard
        for i in p:
            k = (int(ev["pid"][i]), int(ev["fd"][i]), int(ev["sessionID"][i]))
            assert owner.setdefault(k, r) == r  # a connection lives on one shard


def test_local_merge_rules():
    """Counters add mod 2^32; domain / scheme / pid come from the earliest creator."""
    rows = [(7, b"h:1/a", b"h", b"http", 0xFFFFFFFF, 3, 50),
            (7, b"h:1/a", b"h", b"https", 2, 1, 10),
            (8, b"h:1/a", b"h", b"http", 1, 1, 5)]
    keys = [ebd.host_endpoint_key(r[0], r[1]) for r in rows]
    t = shard.merge_tables([shard.ServiceTable.from_rows(rows[:1], keys[:1]),
                            shard.ServiceTable.from_rows(rows[1:], keys[1:])])
    got = t.packed().rows()
    assert got == [(7, b"h:1/a", b"h", b"https", 1, 4), (8, b"h:1/a", b"h", b"http", 1, 1)]


def test_bench_dry_run_spawns_two_gloo_ranks():
    """bench.py --gpus 2 --dry-run-cpu: the launcher spawns two ranks (no torchrun), each
    generates its config-5 connection shard, and the owner-partitioned merge over gloo
    yields every service of the whole trace exactly once."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run-cpu", "--events",
                          "3000"], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["dry_run"] and line["n_gpus"] == 2
    assert sum(line["events_per_rank"]) == 6000 and min(line["events_per_rank"]) > 0
    ev, lens, offs, payload = ebd.generate_host(5, 5, 0, 6000)
    o = O.Oracle()
    o.process(ev, lens, offs, payload)
    assert line["services_merged"] == len(o.services())


class _KeyOnly:
    """Stands in for a Context where only its service-key secret matters."""

    def __init__(self, key):
        self.hash_key = key


def _key_worker(rank, world, port, same, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    try:
        ctx = _KeyOnly((1, 2) if same or rank == 0 else (1, 3))
        try:
            shard.check_same_hash_key(ctx, "cpu")
            ok = True
        except ValueError:
            ok = False
        # a wire record without endpoint bytes (WIRE_NO_BYTES: the source arena was full) takes
        # no bytes; the others' bytes follow in record order, so the received segments
        # concatenate into one addressable table (no rebasing)
        rec = np.zeros(2, shard.REC)
        rec["endpoint_len"] = [ebd.WIRE_NO_BYTES, 3]
        strings = np.frombuffer(b"ab%d\0\0\0\0\0" % rank, np.uint8).copy()
        counts = np.array([1, 1], np.uint32) if rank == 0 else np.array([2, 0], np.uint32)
        scounts = np.array([0, 8], np.uint64) if rank == 0 else np.array([8, 0], np.uint64)
        r, s = shard.exchange(torch.from_numpy(rec.view(np.uint8).copy()), torch.from_numpy(strings), counts, scounts)
        t = shard.ServiceTable.from_wire(r.numpy().view(shard.REC).copy(), s.numpy()[:s.numel() - shard.STR_SLACK])
        eps = [None if o == 0xFFFFFFFFFFFFFFFF else t.strings[o:o + n].tobytes().decode()
               for o, n in zip(t.rec["endpoint_off"].tolist(), t.rec["endpoint_len"].tolist())]
        nb = s.numel()
        with open(out_path % rank, "w") as f:
            json.dump({"ok": ok, "eps": eps, "nbytes": nb}, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("same", [True, False])
def test_exchange_checks_hash_keys_and_keeps_missing_endpoints(same, tmp_path):
    out_path = str(tmp_path / "r%d.json")
    mp.start_processes(_key_worker, args=(2, _free_port(), same, out_path), nprocs=2, join=True, start_method="spawn")
    r0, r1 = (json.load(open(out_path % k)) for k in (0, 1))
    assert r0["ok"] == r1["ok"] == same
    # rank 0 receives its own first record (no bytes) and rank 1's two; rank 1 rank 0's second
    assert r0["eps"] == [None, None, "ab1"]
    assert r1["eps"] == ["ab0"]
    assert r0["nbytes"] == 8 + shard.STR_SLACK


def _net_worker(rank, world, port, out_path):
    """Network-map records (ebd_service_net, 32 B, key_lo first) grouped by owner and
    exchanged with one all_to_all: every rank must receive exactly the records it owns."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    try:
        rng = np.random.default_rng(40 + rank)
        recs = np.zeros(500 + 37 * rank, ebd.SERVICE_NET_DTYPE)
        recs["key_lo"] = rng.integers(0, 2**64, recs.size, dtype=np.uint64)  # high bit set half the time
        recs["key_hi"] = rng.integers(0, 2**64, recs.size, dtype=np.uint64)
        recs["kind"] = 1 + rank
        recs["time_ns"] = np.arange(recs.size, dtype=np.uint64) + 1000 * rank
        t = torch.from_numpy(recs.view(np.uint8).reshape(-1).copy())
        grouped, counts = shard.group_by_owner(t, shard.NET_REC_BYTES, world)
        got = shard.exchange_fixed(grouped, counts, shard.NET_REC_BYTES).numpy().view(ebd.SERVICE_NET_DTYPE)
        owners = shard.owner_np(got["key_lo"], world).tolist()
        with open(out_path % rank, "w") as f:
            json.dump({"n": int(recs.size), "counts": counts.tolist(), "owners": owners,
                       "sent_own": int(np.sum(shard.owner_np(recs["key_lo"], world) == rank)),
                       "got": sorted([int(x) for x in got["key_lo"]])}, f)
    finally:
        dist.destroy_process_group()


def test_network_records_reach_their_owner(tmp_path):
    """The network-map exchange of device_exchange_merge (shard.group_by_owner's uint64
    owner rule on int64 tensors, shard.exchange_fixed) over a world-2 gloo group."""
    out_path = str(tmp_path / "n%d.json")
    mp.start_processes(_net_worker, args=(2, _free_port(), out_path), nprocs=2, join=True, start_method="spawn")
    r = [json.load(open(out_path % k)) for k in (0, 1)]
    for k in (0, 1):
        assert all(o == k for o in r[k]["owners"])
        assert sum(r[k]["counts"]) == r[k]["n"]
    assert len(r[0]["got"]) + len(r[1]["got"]) == r[0]["n"] + r[1]["n"]
    assert r[0]["counts"][0] == r[0]["sent_own"] and r[1]["counts"][1] == r[1]["sent_own"]


def test_owner_rule_uses_every_rank():
    """Service keys are odd (their low bit marks a used slot), so the owner comes from the
    high word: every rank of 2, 4 and 8 owns about its share of the services."""
    keys = np.array([ebd.host_endpoint_key(1000 + k % 7, b"h%d/p%d" % (k, k * 31))[0] for k in range(4000)], np.uint64)
    assert np.all(keys & np.uint64(1) == 1)
    for world in (2, 4, 8):
        counts = np.bincount(shard.owner_np(keys, world), minlength=world)
        assert counts.size == world and counts.min() > 0.8 * len(keys) / world, (world, counts)
