"""GPU: the BASELINE configs at (or near) full size, where a sorted oracle
table is too big to build, checked through size-independent properties.

* C4 at 4 GiB (high cardinality, ~3.5e8 distinct words): the table's
  order-independent digest (distinct words, sum of counts, two 64-bit sums of a
  mix of (FNV-1a(word), count)) equals the oracle's, computed by routing tokens
  to owner threads by hash (oracle/mox_oracle.c, moxo_count_digest).  This size
  crosses the >2 GiB table-bytes fetch and splits partitions to kk >= 10.
* C4 at 16 GiB (1.4e9 distinct): the same digest against the oracle's --
  distinct words == the oracle's distinct count, and a word split over two
  rows (or two words merged) changes the mix sums -- plus sum of counts ==
  tokens, NUL-free words and a spot check of 4,000 random words' counts.
* C5 at 16 GiB (heavy skew, ~1e6 distinct): the full sorted table against the
  oracle's.
Each test holds the corpus, its device copy and the fetched table: tens of GB
of host memory for C4 16 GiB."""
import numpy as np
import pytest

import coracle
import mox
from mox import corpus
from conftest import assert_tables_equal
from mox import dist as mdist

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def gpu_table(data, **kw):
    e = mox.Engine(device=0, reserve_bytes=data.nbytes, **kw)
    d = e.alloc(data.nbytes)
    try:
        e.h2d(d, data)
        e.run_device(d, data.nbytes)
        t = e.fetch()
        counts, offs, raw = t.arrays()
        tokens = t.tokens
        t.close()
        st = e.stats()
    finally:
        e.free(d)
        e.close()
    return counts, offs, raw, tokens, st


def test_c4_4gib_digest():
    cfg = corpus.CONFIGS["C4"]
    data = corpus.fill(cfg["kind"], cfg["seed"], 0, 4 << 30)
    counts, offs, raw, tokens, st = gpu_table(data)
    assert st["split_partitions"] > 900 and st["reduce_units"] > 1024 * 256, st
    assert offs[-1] > (2 << 30)  # the table-bytes fetch crosses 2 GiB
    assert int(counts.sum()) == tokens
    got = coracle.table_digest(counts, offs, raw)
    del counts, offs, raw
    want, wtok = coracle.count_digest(data, nthreads=16)
    assert tokens == wtok
    assert got == want


def spot_check(data, counts, offs, raw, k, seed):
    rng = np.random.default_rng(seed)
    idx = rng.choice(counts.size, size=min(k, counts.size), replace=False)
    words = [raw[offs[i]:offs[i + 1]] for i in idx]
    want = coracle.count_words(data, words, nthreads=16)
    assert want == [int(counts[i]) for i in idx]


def test_c4_full_16gib_digest():
    cfg = corpus.CONFIGS["C4"]
    data = corpus.fill(cfg["kind"], cfg["seed"], 0, cfg["nbytes"])
    counts, offs, raw, tokens, st = gpu_table(data)
    assert int(counts.sum()) == tokens
    assert counts.size > 1_000_000_000 and (counts > 0).all()
    assert np.frombuffer(raw, np.uint8).min() > 0  # C4 words are [a-z0-9]: no NUL, lowercased
    spot_check(data, counts, offs, raw, 4000, 1)
    got = coracle.table_digest(counts, offs, raw)
    del counts, offs, raw
    want, wtok = coracle.count_digest(data, nthreads=16)
    assert tokens == wtok
    assert got[0] == want[0]  # distinct words: every table row is a different word
    assert got == want


def test_c4_full_16gib_device_sorted():
    """The device bytewise sort on C4's 16 GiB table (1.37e9 words, 14.8 GB of
    word bytes: past the 4 GiB the sort took before round 6; its record arrays
    borrow the pass's dead scratch): mox_sort_result must sort it on the GPU
    (it raises rather than falling back), and the fetched table is the oracle's
    (order-independent digest) in bytewise order -- checked on 400 sampled
    windows of 2,000 consecutive rows, every adjacent pair strictly ascending."""
    cfg = corpus.CONFIGS["C4"]
    data = corpus.fill(cfg["kind"], cfg["seed"], 0, cfg["nbytes"])
    e = mox.Engine(device=0, reserve_bytes=data.nbytes, flags=mox.MOX_F_SORT_BYTES)
    d = e.alloc(data.nbytes)
    try:
        e.h2d(d, data)
        e.run_device(d, data.nbytes)
        e.sort_result()  # on the GPU, or MoxError
        st = e.stats()
        t = e.fetch()
        counts, offs, raw = t.arrays()
        tokens = t.tokens
        t.close()
    finally:
        e.free(d)
        e.close()
    assert st["ms_sort"] > 0
    assert int(counts.sum()) == tokens and counts.size > 1_000_000_000
    rng = np.random.default_rng(6)
    n = counts.size
    for s0 in rng.integers(0, n - 2001, size=400):
        ws = [raw[offs[i]:offs[i + 1]] for i in range(int(s0), int(s0) + 2001)]
        assert all(a < b for a, b in zip(ws, ws[1:]))
    for i in (0, n - 2):  # the two ends
        assert raw[offs[i]:offs[i + 1]] < raw[offs[i + 1]:offs[i + 2]]
    got = coracle.table_digest(counts, offs, raw)
    del counts, offs, raw
    want, wtok = coracle.count_digest(data, nthreads=16)
    assert tokens == wtok
    assert got == want


def test_c5_full_16gib_exact():
    cfg = corpus.CONFIGS["C5"]
    data = corpus.fill(cfg["kind"], cfg["seed"], 0, cfg["nbytes"])
    counts, offs, raw, tokens, _ = gpu_table(data)
    assert int(counts.sum()) == tokens
    wc, wo, wraw, wtok = coracle.count_arrays(data, nthreads=16)
    assert tokens == wtok
    assert_tables_equal((counts, offs, raw), (wc, wo, wraw))


def test_c3_group_two_8gib_shards_exact():
    """C3 at its per-GPU size: the engine group (2 members on device 0, copy
    transport) over two 8 GiB byte-range shards of the C3 stream, cut with
    the bench's left context and 64 KiB look-ahead (mox_run_shards), then the
    exchange, per-owner reduce, gather and the device bytewise sort
    (MOX_F_SORT_BYTES).  The gathered table must be the oracle's table of the
    16 GiB: its digest, and row for row in bytewise order."""
    n, per = 2, 8 << 30
    cfg = corpus.CONFIGS["C3"]
    data = corpus.fill(cfg["kind"], cfg["seed"], 0, n * per)
    g = mox.Engine(device=0, n_gpus=n, transport=mox.XPORT_COPY, devices=[0] * n, flags=mox.MOX_F_SORT_BYTES,
                   reserve_bytes=per)
    bufs = []
    try:
        shards = []
        for r in range(n):
            lo, hi, ob, oe, end = mdist.shard_range(n * per, n, r, per_rank=per)
            m = g.member(r)
            d = m.alloc(hi - lo)
            bufs.append((m, d))
            m.h2d(d, data[lo:hi])
            shards.append((d, hi - lo, ob, oe, end))
        g.run_shards(shards)
        st = g.stats()
        t = g.fetch()
        counts, offs, raw = t.arrays()
        tokens = t.tokens
        t.close()
    finally:
        for m, d in bufs:
            m.free(d)
        g.close()
    assert st["n_gpus"] == n and st["ms_sort"] > 0 and st["x_bytes_sent"] > 0
    assert int(counts.sum()) == tokens == st["tokens"]
    want, wtok = coracle.count_digest(data, nthreads=16)
    assert tokens == wtok
    assert coracle.table_digest(counts, offs, raw) == want
    # device bytewise order: the rows ARE the oracle's sorted rows
    wc, wo, wraw, _ = coracle.count_arrays(data, nthreads=16)
    del data
    assert counts.size == wc.size
    assert np.array_equal(counts, wc) and np.array_equal(offs, wo) and raw == wraw


def test_c2_async_bench_mode_exact():
    """The mode the headline bench times, at its full size (bench.py, N = 1):
    K back-to-back asynchronous passes (mox_run_range_async) over the 1 GiB C2
    corpus with MOX_F_TIMING_MAP, each pass's dictionary built on the side
    stream into the dictionary set the previous pass did not use.  Every
    completed pass's tokens and distinct words equal the oracle's, and the last
    pass's table equals the oracle's table."""
    cfg = corpus.CONFIGS["C2"]
    data = corpus.fill(cfg["kind"], cfg["seed"], 0, cfg["nbytes"])
    wc, wo, wraw, wtok = coracle.count_arrays(data, nthreads=16)
    e = mox.Engine(device=0, flags=mox.MOX_F_TIMING_MAP, reserve_bytes=data.nbytes)
    d = e.alloc(data.nbytes)
    try:
        e.h2d(d, data)
        completed = []
        for i in range(6):
            e.run_range_async(d, data.nbytes, 0, data.nbytes, True)
            if i > 0:  # this call completed the previous pass
                st = e.stats()
                completed.append((st["tokens"], st["uniques"], st["ms_map"] > 0))
        e.run_wait()
        st = e.stats()
        completed.append((st["tokens"], st["uniques"], st["ms_map"] > 0))
        assert st["async_reruns"] == 0 and st["async_dropped"] == 0, st
        t = e.fetch()
        counts, offs, raw = t.arrays()
        tokens = t.tokens
        t.close()
    finally:
        e.free(d)
        e.close()
    assert completed == [(wtok, wc.size, True)] * 6
    assert tokens == wtok
    assert_tables_equal((counts, offs, raw), (wc, wo, wraw))
