"""GPU: the engine group (mox_config.n_gpus > 1, include/mox.h) -- one engine
that drives several GPUs from one host thread, as SURVEY.md §8(b) asks for the
drop-in of main.rs:16-22: mox_count / mox_count_file split the input at
whitespace, run the local passes on every member at once, exchange the
partial tables (hash-partitioned all-to-all), reduce per owner and gather on
member 0; mox_run_shards does the same for device-resident shards.

The box has one GPU, so the members share device 0 over the copy transport
(MOX_XPORT_COPY: device-to-device copies); the RCCL transport
(ncclCommInitAll + grouped send/recv) needs distinct devices and runs when
the box has them.  Also here: the device bytewise table sort (MOX_F_SORT_BYTES,
mox_bsort.hip) against Python's bytes order."""
import os
import random
import subprocess
import sys
import json

import numpy as np
import pytest

import coracle
import mox
from mox import corpus
from mox import dist as mdist
from conftest import ROOT, assert_tables_equal

pytestmark = pytest.mark.gpu


def group(n, flags=0, **kw):
    return mox.Engine(device=0, n_gpus=n, transport=mox.XPORT_COPY, devices=[0] * n, flags=flags, **kw)


def mixed(n, seed):
    """test_gpu_exchange's mixed corpus, made valid UTF-8 (its Unicode part is
    cut at a byte count, which can split a character)."""
    import test_gpu_exchange as X
    return X.mixed_corpus(n, seed).decode("utf-8", "ignore").encode()


@pytest.mark.parametrize("n", [2, 3])
def test_group_count_exact(n):
    data = mixed(6 << 20, 70 + n)
    g = group(n)
    try:
        assert g.group_size() == n
        t = g.count(data)
        got = t.sorted_items()
        tokens = t.tokens
        t.close()
        st = g.stats()
    finally:
        g.close()
    want, wtok = coracle.count(data)
    assert tokens == wtok and got == want
    assert st["n_gpus"] == n and st["tokens"] == wtok and st["uniques"] == len(want)
    assert st["x_bytes_sent"] > 0 and st["x_bytes_sent"] == st["x_bytes_recv"]


def test_group_sorted_table_is_the_oracle_list():
    """MOX_F_SORT_BYTES: the gathered table is sorted bytewise on member 0's GPU
    inside the call: the fetched list IS the oracle's sorted list."""
    data = mixed(4 << 20, 81) + " ΣΑΣ İ K ".encode() + b"a\x00b a\x00b " + b"p" * 40 + b" " + b"p" * 39
    g = group(3, flags=mox.MOX_F_SORT_BYTES)
    try:
        t = g.count(data)
        got = list(t.items())
        t.close()
        assert g.stats()["ms_sort"] > 0
    finally:
        g.close()
    assert got == coracle.count(data)[0]


def test_group_count_file_sharded(tmp_path):
    """Every member reads its own byte range of the file (cut at whitespace)."""
    data = corpus.fill(corpus.ZIPF, 82, 0, (40 << 20) + 777)
    f = tmp_path / "c.txt"
    data.tofile(str(f))
    g = group(4)
    try:
        t = g.count_file(str(f))
        got = t.arrays()
        t.close()
        assert g.stats()["ms_h2d"] > 0
        for small in (b"", b"one", b"x" * 100000):
            (tmp_path / "s.txt").write_bytes(small)
            t = g.count_file(str(tmp_path / "s.txt"))
            assert t.sorted_items() == coracle.count(small)[0]
            t.close()
        with pytest.raises(mox.MoxError):
            g.count_file(str(tmp_path / "missing.txt"))
    finally:
        g.close()
    assert_tables_equal(got, coracle.count_arrays(data, nthreads=16)[:3])


def test_group_edges_and_errors():
    g = group(3)
    try:
        for data in (b"", b"a", b"a b", b"   \n\t ", b"Y" * 50000, b"x " * 5 + b"Z" * 40):
            t = g.count(data)
            assert t.sorted_items() == coracle.count(data)[0], data[:20]
            t.close()
        bad = mixed(3 << 20, 83)
        bad = bad[:2_500_000] + b"\xff" + bad[2_500_000:]  # in the last member's range
        with pytest.raises(mox.Utf8Error):
            g.count(bad)
        t = g.count(b"still usable")  # the group stays usable
        assert t.sorted_items() == [(b"still", 1), (b"usable", 1)]
        t.close()
        with pytest.raises(mox.MoxError):  # one buffer for n GPUs: mox_run_shards instead
            g.run_device(0, 0)
    finally:
        g.close()


def test_group_run_shards_high_cardinality():
    """Device-resident shards with halos (the bench's layout), high-cardinality
    text: the members' reduce-only passes split partitions; exact."""
    data = corpus.fill(corpus.HICARD, 84, 0, 64 << 20).tobytes()
    n = 2
    g = group(n)
    bufs = []
    try:
        shards = []
        for r in range(n):
            lo, hi, ob, oe, end = mdist.shard_range(len(data), n, r)
            m = g.member(r)
            d = m.alloc(max(1, hi - lo))
            m.h2d(d, data[lo:hi])
            bufs.append((m, d))
            shards.append((d, hi - lo, ob, oe, end))
        g.run_shards(shards)
        t = g.fetch()
        got = t.arrays()
        t.close()
    finally:
        for m, d in bufs:
            m.free(d)
        g.close()
    assert_tables_equal(got, coracle.count_arrays(np.frombuffer(data, np.uint8), nthreads=16)[:3])


def test_group_rccl_transport():
    """RCCL transport: ncclCommInitAll over distinct devices (needs >= 2 GPUs)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    cnt = ctypes.c_int(0)
    hip.hipGetDeviceCount(ctypes.byref(cnt))
    if cnt.value < 2:
        with pytest.raises(mox.MoxError):  # shared device: RCCL refuses, the engine says so
            mox.Engine(device=0, n_gpus=2, devices=[0, 0])
        pytest.skip("one GPU on this box: RCCL engine group needs two")
    data = mixed(6 << 20, 85)
    g = mox.Engine(n_gpus=2, flags=mox.MOX_F_SORT_BYTES)
    try:
        t = g.count(data)
        got = list(t.items())
        t.close()
    finally:
        g.close()
    assert got == coracle.count(data)[0]


def tricky_words(rng):
    """Words that stress the bytewise sort: shared 16/32/48-byte prefixes
    (tie levels), proper prefixes, NUL bytes, bytes >= 0x80, length 1..90."""
    base = [b"https://example.com/path/", b"internationalization", b"q" * 16, b"abcdefghijklmnop" * 3]
    words = set()
    for _ in range(3000):
        w = rng.choice(base)[: rng.randint(1, 60)] + bytes(rng.choice(b"az\x01\x7f") for _ in range(rng.randint(0, 30)))
        words.add(w)
    words |= {b"a", b"a\x00", b"a\x00\x00", b"ab", "é".encode(), "éa".encode(), b"\x00"}
    return sorted(words)


@pytest.mark.parametrize("checked", [False, True])
def test_device_sort_tie_levels(monkeypatch, checked):
    """mox_reduce_pairs table (words taken verbatim) sorted on the GPU: the
    order equals Python's bytes order, through several 16-byte tie levels --
    with the first tie levels run without a host round trip (default) and with
    every level read back (MOX_BSORT_CHECKED, the mode a run past RUN_LMAX falls
    back to)."""
    if checked:
        monkeypatch.setenv("MOX_BSORT_CHECKED", "1")
    rng = random.Random(99)
    words = tricky_words(rng)
    shuffled = words[:]
    rng.shuffle(shuffled)
    e = mox.Engine(device=0, flags=mox.MOX_F_SORT_BYTES)
    try:
        t = e.reduce_pairs(shuffled, list(range(1, len(shuffled) + 1)))
        got = list(t.items())
        t.close()
    finally:
        e.close()
    assert [w for w, _ in got] == words
    cnt = dict(zip(shuffled, range(1, len(shuffled) + 1)))
    assert all(cnt[w] == c for w, c in got)


def test_device_sort_run_past_the_segment_sort():
    """6,000 words sharing a 20-byte prefix: one tie run longer than k_bs_segsort
    / k_bs_longsort take (RUN_LMAX), met in a level that runs without a host
    round trip; the sort runs again in the checked mode (radix passes over the
    subset) and the order still equals Python's bytes order."""
    rng = random.Random(7)
    words = sorted({b"x" * 20 + bytes(rng.choice(b"abcdefgh") for _ in range(rng.randint(1, 12))) for _ in range(9000)})
    assert len(words) > 4096
    shuffled = words[:]
    rng.shuffle(shuffled)
    e = mox.Engine(device=0, flags=mox.MOX_F_SORT_BYTES)
    try:
        t = e.reduce_pairs(shuffled, list(range(1, len(shuffled) + 1)))
        got = list(t.items())
        t.close()
    finally:
        e.close()
    assert [w for w, _ in got] == words
    cnt = dict(zip(shuffled, range(1, len(shuffled) + 1)))
    assert all(cnt[w] == c for w, c in got)


@pytest.mark.parametrize("checked", [False, True])
def test_device_sort_uniform_digits(monkeypatch, checked):
    """Tables where some radix digits hold the same value for every word: words
    of 1-2 bytes (window bytes 2..6 are zero everywhere) and words behind one
    shared 5-byte prefix.  k_os_pass reads the digit histogram itself and
    copies such a pass instead of ranking it (no host read between the
    histogram and the passes); the order equals Python's bytes order."""
    if checked:
        monkeypatch.setenv("MOX_BSORT_CHECKED", "1")
    rng = random.Random(123)
    letters = b"abcdefghijklmnopqrstuvwxyz0123456789"
    short = sorted({bytes(rng.choice(letters) for _ in range(rng.randint(1, 2))) for _ in range(3000)})
    pref = sorted({b"zzzzz" + bytes(rng.choice(letters) for _ in range(rng.randint(0, 14))) for _ in range(20000)})
    for words in (short, pref):
        shuffled = words[:]
        rng.shuffle(shuffled)
        e = mox.Engine(device=0, flags=mox.MOX_F_SORT_BYTES)
        try:
            t = e.reduce_pairs(shuffled, list(range(1, len(shuffled) + 1)))
            got = list(t.items())
            t.close()
        finally:
            e.close()
        assert [w for w, _ in got] == words
        cnt = dict(zip(shuffled, range(1, len(shuffled) + 1)))
        assert all(cnt[w] == c for w, c in got)


def test_device_sort_large_tables():
    """24 MiB of Zipf text + 48 MiB of C4-like tokens: the device-sorted
    table equals the oracle's sorted table array for array."""
    z = corpus.fill(corpus.ZIPF, 86, 0, 24 << 20)
    h = corpus.fill(corpus.HICARD, 87, 0, 48 << 20)
    data = np.concatenate([z, np.frombuffer(b" \n", np.uint8), h])
    e = mox.Engine(device=0, flags=mox.MOX_F_SORT_BYTES)
    try:
        t = e.count(data.tobytes())
        counts, offs, raw = t.arrays()
        t.close()
    finally:
        e.close()
    wc, wo, wraw, _ = coracle.count_arrays(data, nthreads=16)
    assert np.array_equal(counts, wc) and np.array_equal(offs, wo) and raw == wraw


def test_bench_multi_gpu_without_torchrun():
    """`python3 bench.py --gpus 2 --xport host --device 0` with no torchrun
    environment: one process, an engine group of 2 members on device 0 (copy
    transport); one JSON line with the multi_gpu fields."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--xport", "host", "--device", "0",
           "--steps", "2", "--warmup", "1", "--bytes-per-gpu", str(64 << 20), "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    line = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["check_sum_counts_eq_tokens"]
    mg = line["multi_gpu"]
    assert mg["mode"] == "engine group (one process)" and mg["all_to_all_bytes"] > 0 and mg["gathered_table"]["n"] > 0


def test_group_sort_falls_back_to_the_host(monkeypatch):
    """a gathered table the device sort cannot take (its scratch, or
    MOX_BSORT_MAX_WORDS) is sorted on the host by mox_fetch_table, not lost."""
    data = mixed(2 << 20, 91)
    monkeypatch.setenv("MOX_BSORT_MAX_WORDS", "10")
    g = group(2, flags=mox.MOX_F_SORT_BYTES)
    try:
        t = g.count(data)
        got = list(t.items())
        t.close()
    finally:
        g.close()
    assert got == coracle.count(data)[0]


def test_group_set_flags_reaches_every_member():
    """mox_set_flags on a group applies to every member: with
    MOX_F_TIMING_MAP set after creation, every member times its map kernel."""
    data = mixed(2 << 20, 92)
    g = group(2)
    try:
        g.set_flags(mox.MOX_F_TIMING_MAP)
        t = g.count(data)
        t.close()
        assert all(g.member(i).stats()["ms_map"] > 0 for i in range(2))
        assert g.stats()["ms_map"] > 0
    finally:
        g.close()


def test_group_eight_members_c3_exact():
    """The driver's N = 8 configuration on one GPU: an engine group of 8
    members (copy transport, all on device 0) over 8 byte-range shards of the
    C3 stream (128 MiB each, the bench's left context and 64 KiB look-ahead),
    local passes, exchange, per-owner reduce, gather and the device bytewise
    sort.  The gathered table is the oracle's sorted table, array for array."""
    n, per = 8, 128 << 20
    cfg = corpus.CONFIGS["C3"]
    data = corpus.fill(cfg["kind"], cfg["seed"], 0, n * per)
    g = group(n, flags=mox.MOX_F_SORT_BYTES, reserve_bytes=per)
    bufs = []
    try:
        shards = []
        for r in range(n):
            lo, hi, ob, oe, end = mdist.shard_range(n * per, n, r, per_rank=per, halo=1 << 16)
            m = g.member(r)
            d = m.alloc(hi - lo)
            bufs.append((m, d))
            m.h2d(d, data[lo:hi])
            shards.append((d, hi - lo, ob, oe, end))
        for _ in range(2):  # twice: the second call reuses every member's buffers
            g.run_shards(shards)
            st = g.stats()
            t = g.fetch()
            counts, offs, raw = t.arrays()
            tokens = t.tokens
            t.close()
            wc, wo, wraw, wtok = coracle.count_arrays(data, nthreads=16)
            assert st["n_gpus"] == n and st["x_bytes_sent"] > 0 and st["ms_sort"] > 0
            assert tokens == wtok == st["tokens"]
            assert np.array_equal(counts, wc) and np.array_equal(offs, wo) and raw == wraw
    finally:
        for m, d in bufs:
            m.free(d)
        g.close()


def test_bench_eight_members_without_torchrun():
    """`bench.py --gpus 8 --xport host --device 0`: the bench's multi-GPU step
    with 8 members (engine group, copy transport on one GPU) exits 0 with the
    multi_gpu fields, so that the driver's 8-GPU run can only fail in RCCL."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--xport", "host", "--device", "0",
           "--steps", "2", "--warmup", "1", "--bytes-per-gpu", str(128 << 20), "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    line = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert line["n_gpus"] == 8 and line["value"] > 0 and line["check_sum_counts_eq_tokens"]
    mg = line["multi_gpu"]
    assert mg["all_to_all_bytes"] > 0 and mg["gathered_table"]["n"] > 0
    assert line["phases_ms"]["sort_bytes"] > 0 and line["hash_order"]["value"] > 0


def test_bench_torchrun_processes_host_transport():
    """The driver's multi-GPU launch shape (torch.distributed.run, one process
    per rank, bench.py main()) with 2 ranks sharing device 0 over the host
    transport: exchange, gather and the sort at rank 0 inside the timed step;
    rank 0 prints one JSON line with the multi_gpu fields."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29571", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--xport", "host", "--device", "0", "--steps", "2", "--warmup", "1",
           "--bytes-per-gpu", str(64 << 20)]
    r = subprocess.run(cmd, capture_output=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    line = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["check_sum_counts_eq_tokens"]
    mg = line["multi_gpu"]
    assert mg["all_to_all_bytes"] > 0 and mg["gathered_table"]["n"] > 0 and len(mg["per_rank_tokens"]) == 2
