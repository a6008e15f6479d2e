"""GPU: the multi-GPU exchange -- byte-range shards, local
passes, all-to-all of the partial tables, final per-owner reduce -- checked
bit-exactly against the oracle on the whole corpus.

One GPU box has one GPU, so several ranks share device 0: the RCCL transport is
exercised at world size 1 (self send/recv through RCCL), the multi-rank data
path through the host-staged transport (threads in one process, and separate
processes over gloo).  Both transports move the same packed buffers; only the
copy differs."""
import json
import os
import subprocess
import sys
import threading

import pytest

import coracle
import mox
from mox import corpus
from mox import dist as mdist
from conftest import ROOT

pytestmark = pytest.mark.gpu


def mixed_corpus(n, seed):
    """Zipf text with Unicode tokens and long (> 16 byte) words mixed in."""
    z = corpus.fill(corpus.ZIPF, seed, 0, n).tobytes()
    u = corpus.fill(corpus.UNICODE, seed + 1, 0, n // 8).tobytes()
    extra = b" ".join(b"Supercalifragilistic%dexpialidocious" % (i % 97) for i in range(3000))
    return z[: n // 2] + b" " + u + b"\n" + extra + b" " + z[n // 2:]


def run_ranks(data, world, gather_root=None, lib_path=None, stats=None, flags=0, table_order=False):
    """Each rank: engine on device 0, its shard, exchange over ThreadAlltoall;
    with gather_root, then the gather of every table into that rank's engine
    (out[root] is then the gathered table, the others their own).  lib_path:
    a check build; stats: a list that receives every rank's mox_stats; flags:
    the engines' flags (MOX_F_SORT_BYTES: the sorted exchange); table_order:
    items in the table's own order instead of sorted."""
    x = mdist.ThreadAlltoall(world)
    out, errs = [None] * world, []

    def rank_main(r):
        try:
            lo, hi, ob, oe, at_end = mdist.shard_range(len(data), world, r)
            e = mox.Engine(device=0, lib_path=lib_path, flags=flags)
            try:
                buf = data[lo:hi]
                d = e.alloc(max(1, len(buf)))
                try:
                    if buf:
                        e.h2d(d, buf)
                    e.run_range(d, len(buf), ob, oe, at_end)
                    e.exchange_host(world, r, x.fn(r))
                    if gather_root is not None:
                        e.gather_host(world, r, x.fn(r), root=gather_root)
                    t = e.fetch()
                    out[r] = (list(t.items()) if table_order else t.sorted_items(), t.tokens)
                    t.close()
                    if stats is not None:
                        stats.append(e.stats())
                finally:
                    e.free(d)
            finally:
                e.close()
        except BaseException as ex:  # noqa: BLE001
            errs.append(ex)
            x.barrier.abort()

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    [t.start() for t in ts]
    [t.join(300) for t in ts]
    if errs:
        raise errs[0]
    return out


@pytest.mark.parametrize("world", [2, 3])
def test_host_exchange_threads(world):
    data = mixed_corpus(6 << 20, 40 + world)
    out = run_ranks(data, world)
    merged = mdist.merge_tables([items for items, _ in out])  # also asserts disjoint owners
    want, wtok = coracle.count(data)
    assert sum(tok for _, tok in out) == wtok
    for items, tok in out:
        assert sum(c for _, c in items) == tok
    assert merged == want


def test_host_exchange_empty_and_tiny_shards():
    for data in (b"", b"a", b"a b", b"x " * 5 + b"Y" * 40):
        out = run_ranks(data, 3)
        assert mdist.merge_tables([items for items, _ in out]) == coracle.count(data)[0]


def test_rccl_transport_world1():
    data = mixed_corpus(3 << 20, 9)
    e = mox.Engine(device=0)
    try:
        e.comm_init(1, 0, mox.comm_unique_id())
        d = e.alloc(len(data))
        try:
            e.h2d(d, data)
            e.run_range(d, len(data), 0, len(data), True)
            e.exchange()
            t = e.fetch()
            got = t.sorted_items()
            t.close()
        finally:
            e.free(d)
    finally:
        e.close()
    assert got == coracle.count(data)[0]


def test_host_exchange_gloo_processes(tmp_path):
    """Two processes (torch.distributed gloo) share the GPU; rank 0 gathers."""
    out = tmp_path / "merged.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29561",
           os.path.join(ROOT, "tests", "dist_worker.py"), str(out)]
    r = subprocess.run(cmd, capture_output=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    res = json.loads(out.read_text())
    data = mixed_corpus(4 << 20, 77)
    assert [(bytes.fromhex(w), c) for w, c in res] == coracle.count(data)[0]


def gpu_count():
    import ctypes
    n = ctypes.c_int(0)
    ctypes.CDLL("libamdhip64.so").hipGetDeviceCount(ctypes.byref(n))
    return n.value


def test_rccl_exchange_gather_two_processes(tmp_path):
    """One process per GPU over RCCL at world size 2: the exchange's ncclSend /
    ncclRecv between two ranks and the gather where only the root receives
    (ADVICE r2).  Needs two GPUs; the one-GPU box skips it (RCCL refuses two
    ranks on one device, "Duplicate GPU detected")."""
    if gpu_count() < 2:
        pytest.skip("needs 2 GPUs")
    out = tmp_path / "merged.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29563",
           os.path.join(ROOT, "tests", "dist_worker.py"), str(out), "rccl"]
    r = subprocess.run(cmd, capture_output=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    res = json.loads(out.read_text())
    data = mixed_corpus(4 << 20, 77)
    assert [(bytes.fromhex(w), c) for w, c in res] == coracle.count(data)[0]


def test_gather_requires_an_exchanged_table():
    """mox_gather / mox_gather_host refuse a table that is not the result of an
    exchange (ranks' local tables overlap) and a table that was already
    gathered: MOX_ESTATE on every rank, no transport call."""
    data = mixed_corpus(2 << 20, 61)
    world = 2
    x = mdist.ThreadAlltoall(world)
    codes, errs = [[] for _ in range(world)], []

    def rank_main(r):
        try:
            lo, hi, ob, oe, at_end = mdist.shard_range(len(data), world, r)
            e = mox.Engine(device=0)
            d = e.alloc(hi - lo)
            try:
                e.h2d(d, data[lo:hi])
                e.run_range(d, hi - lo, ob, oe, at_end)
                for step in ("gather_local", "exchange", "gather", "gather_again"):
                    try:
                        if step == "exchange":
                            e.exchange_host(world, r, x.fn(r))
                        else:
                            e.gather_host(world, r, x.fn(r), root=0)
                        codes[r].append((step, 0))
                    except mox.MoxError as ex:
                        codes[r].append((step, ex.code))
            finally:
                e.free(d)
                e.close()
        except BaseException as ex:  # noqa: BLE001
            errs.append(ex)
            x.barrier.abort()

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    [t.start() for t in ts]
    [t.join(300) for t in ts]
    if errs:
        raise errs[0]
    want = [("gather_local", mox.MOX_ESTATE), ("exchange", 0), ("gather", 0), ("gather_again", mox.MOX_ESTATE)]
    assert codes[0] == want and codes[1] == want


def test_host_exchange_high_cardinality():
    """The reduce-only pass over received partials splits mostly-distinct
    partitions too (weighted records only)."""
    from conftest import assert_tables_equal
    import numpy as np
    data = corpus.fill(corpus.HICARD, 91, 0, 96 << 20).tobytes()
    out = run_ranks(data, 2)
    items = [w for part, _ in out for w in part]
    counts = np.array([c for _, c in items], dtype=np.uint64)
    words = [w for w, _ in items]
    offs = np.zeros(len(words) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(w) for w in words])
    wc, wo, wraw, wtok = coracle.count_arrays(np.frombuffer(data, np.uint8), nthreads=16)
    assert sum(tok for _, tok in out) == wtok
    assert_tables_equal((counts, offs, b"".join(words)), (wc, wo, wraw))


def test_host_exchange_zipf_many_records():
    """2 ranks x 48 MiB of Zipf text: ~1e5 received partials per rank go through
    the LDS-aggregated scatter of the reduce-only pass; exact vs the oracle."""
    from conftest import assert_tables_equal
    import numpy as np
    data = corpus.fill(corpus.ZIPF, 92, 0, 96 << 20).tobytes()
    out = run_ranks(data, 2)
    items = [w for part, _ in out for w in part]
    counts = np.array([c for _, c in items], dtype=np.uint64)
    words = [w for w, _ in items]
    offs = np.zeros(len(words) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(w) for w in words])
    wc, wo, wraw, wtok = coracle.count_arrays(np.frombuffer(data, np.uint8), nthreads=16)
    assert sum(tok for _, tok in out) == wtok
    assert_tables_equal((counts, offs, b"".join(words)), (wc, wo, wraw))


def test_host_gather_threads():
    """mox_gather over the host transport: after the exchange every rank's
    table goes to the root, whose table is then the whole corpus's."""
    data = mixed_corpus(6 << 20, 51)
    want, wtok = coracle.count(data)
    for world, root in ((2, 0), (3, 2)):
        out = run_ranks(data, world, gather_root=root)
        items, tok = out[root]
        assert tok == wtok
        assert sorted(items) == want
        others = [o for r, o in enumerate(out) if r != root]
        assert all(sum(c for _, c in it) == t for it, t in others)


def test_rccl_gather_world1():
    data = mixed_corpus(3 << 20, 19)
    e = mox.Engine(device=0, flags=mox.MOX_F_SORT_BYTES)
    try:
        e.comm_init(1, 0, mox.comm_unique_id())
        d = e.alloc(len(data))
        try:
            e.h2d(d, data)
            e.run_range(d, len(data), 0, len(data), True)
            e.exchange()
            e.gather(0)
            t = e.fetch()
            got = list(t.items())  # MOX_F_SORT_BYTES: table order is bytewise
            t.close()
            st = e.stats()
        finally:
            e.free(d)
    finally:
        e.close()
    assert got == coracle.count(data)[0]
    assert st["x_bytes_sent"] > 0 and st["x_bytes_sent"] == st["x_bytes_recv"] and st["gather_bytes"] > 0


def c3_like_corpus(world, per_rank, seed):
    """world x per_rank bytes of Zipf text with Unicode tokens and long words
    mixed in, and at every shard cut (a multiple of the 1 MiB generator block)
    an item straddling the cut: a token, a 3-byte or a 2-byte Unicode
    whitespace, a Greek token with a final sigma, CR LF and VT.  The base text
    is ASCII and planted items never overlap, so the corpus stays valid UTF-8."""
    import numpy as np
    n = world * per_rank
    buf = bytearray(corpus.fill(corpus.ZIPF, seed, 0, n).tobytes())
    rng = np.random.default_rng(seed)
    items = ["日本語ΣΑΣ".encode(), "İstanbul".encode(), "ΟΔΟΣ".encode(), "\u212aelvin".encode(),
             b"Supercalifragilisticexpialidocious", b"Antidisestablishmentarianism_" * 3]
    cuts = {r * per_rank for r in range(1, world)}
    for k in range(n // 4096 - 1):  # one item per 4 KiB slot, away from the cuts
        it = items[int(rng.integers(len(items)))]
        p = k * 4096 + 1 + int(rng.integers(0, 4096 - 200))
        if any(abs(p - c) < 256 for c in cuts):
            continue
        buf[p - 1:p + len(it) + 1] = b" " + it + b"\n"
    plants = [b"xx STRADDLING yy", " a\u3000b ".encode(), " c\u00a0d ".encode(), " ΣΙΣΥΦΟΣ ".encode(),
              b"\r\n\r\nWORD\x0b"]
    for r in range(1, world):
        it = plants[(r - 1) % len(plants)]
        p = r * per_rank - len(it) // 2
        buf[p:p + len(it)] = it
    return bytes(buf)


def test_world8_threads_c3_path():
    """C3's data path at P = 8 (threads sharing device 0, host transport):
    8 x 32 MiB shards cut at 1 MiB generator-block boundaries, with tokens and
    multi-byte whitespace straddling the cuts; part_owner / long_owner /
    owner_first_part at NB = 1024 / 8; exact against the oracle, and the
    gather at rank 0 gives the whole table."""
    world, per = 8, 32 << 20
    data = c3_like_corpus(world, per, 0x5EED0003)
    assert all(mdist.shard_range(len(data), world, r)[2] in (0, 64) for r in range(world))
    out = run_ranks(data, world, gather_root=0)
    want, wtok = coracle.count(data, nthreads=16)
    assert out[0][1] == wtok
    assert out[0][0] == want


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sorted_exchange_threads(world):
    """The sorted exchange (MOX_F_SORT_BYTES at exchange time): words are owned
    by byte range (splitters from every rank's sampled prefixes), every rank
    sorts its own words, and the gather in rank order is the bytewise-sorted
    table.  Before the gather: every rank's table is in bytewise order and the
    ranks' ranges follow each other; after it: the root's table IS the
    oracle's sorted list, without a sort at the root."""
    data = mixed_corpus(6 << 20, 60 + world)
    want, wtok = coracle.count(data)
    out = run_ranks(data, world, flags=mox.MOX_F_SORT_BYTES, table_order=True)
    for items, tok in out:
        assert [w for w, _ in items] == sorted(w for w, _ in items)
        assert sum(c for _, c in items) == tok
    firsts = [items for items, _ in out if items]
    assert all(a[-1][0] < b[0][0] for a, b in zip(firsts, firsts[1:]))  # ranges in rank order, disjoint
    assert len(firsts) >= min(world, 2)  # the splitters spread the words over the ranks
    assert [x for items, _ in out for x in items] == want
    stats = []
    out = run_ranks(data, world, gather_root=0, flags=mox.MOX_F_SORT_BYTES, table_order=True, stats=stats)
    assert out[0] == (want, wtok)
    assert all(st["ms_sort"] > 0 for st in stats)


def test_sorted_exchange_c3_path_world8():
    """The sorted exchange on test_world8_threads_c3_path's corpus (8 x 32 MiB,
    items straddling every cut): the gathered table at rank 0 is the oracle's
    sorted list, in order."""
    world, per = 8, 32 << 20
    data = c3_like_corpus(world, per, 0x5EED0003)
    out = run_ranks(data, world, gather_root=0, flags=mox.MOX_F_SORT_BYTES, table_order=True)
    want, wtok = coracle.count(data, nthreads=16)
    assert out[0][1] == wtok
    assert out[0][0] == want


def test_sorted_exchange_weights_ranks_by_table_size():
    """Splitters weighted by every rank's table size (k_xsplit): rank 0's shard
    holds ~all distinct words (random tokens), the other ranks' shards a few
    hundred repeated words.  With equal sample weights two thirds of the
    samples would come from the small tables and most of rank 0's words would
    land on one rank; weighted, the ranks' final tables stay near an even
    share -- and the gathered table is still the oracle's sorted list."""
    world = 3
    third = 4 << 20
    h = corpus.fill(corpus.HICARD, 71, 0, third).tobytes()
    few = b" ".join(b"w%03d" % (i % 300) for i in range(third // 5))[:third]
    data = h + b" " + few + b" " + few
    want, wtok = coracle.count(data)
    stats = []
    out = run_ranks(data, world, flags=mox.MOX_F_SORT_BYTES, table_order=True, stats=stats)
    sizes = [len(items) for items, _ in out]
    assert [x for items, _ in out for x in items] == want  # still sorted ranges in rank order
    assert all(st["x_ranged"] == 1 for st in stats)  # the sorted exchange ran (no skew fallback)
    assert max(sizes) <= 2.2 * (sum(sizes) / world), sizes
    out = run_ranks(data, world, gather_root=0, flags=mox.MOX_F_SORT_BYTES, table_order=True)
    assert out[0] == (want, wtok)


def test_sorted_exchange_skewed_prefixes_fall_back():
    """words that share their first 8 bytes (URL-like) cannot be
    split by 8-byte prefix splitters: one rank would receive and sort nearly the
    whole table.  k_xsplit flags the skew and every rank falls back to hash
    owners (the ranks' tables are then in engine order), and the gathered,
    fetched table is still the oracle's sorted list."""
    world = 3
    rng = __import__("random").Random(5)
    words = [b"https://www.example.org/" + bytes(rng.choice(b"abcdefghij") for _ in range(rng.randint(3, 9)))
             for _ in range(150000)]  # ~78 % of the distinct words share "https://"
    data = b" ".join(words) + b" " + corpus.fill(corpus.ZIPF, 72, 0, 1 << 20).tobytes()
    want, wtok = coracle.count(data)
    stats = []
    out = run_ranks(data, world, flags=mox.MOX_F_SORT_BYTES, stats=stats)
    assert sorted(x for items, _ in out for x in items) == want
    assert len(stats) == world and all(st["x_ranged"] == 0 for st in stats)  # hash owners on every rank
    out = run_ranks(data, world, gather_root=0, flags=mox.MOX_F_SORT_BYTES)
    assert out[0] == (want, wtok)
