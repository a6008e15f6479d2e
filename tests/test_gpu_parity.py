"""GPU parity: the HIP path (through the C ABI) vs the oracle, bit-exact.

Word counts are integers, so the bar is exact equality of the (word, count)
multiset after a deterministic bytewise key sort.
"""
import random

import numpy as np
import pytest

import coracle
import mox
from mox import corpus
from conftest import kat_expected

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = mox.Engine(flags=mox.MOX_F_TIMING)
    yield e
    e.close()


@pytest.fixture(scope="module")
def eng_nodict():
    e = mox.Engine(flags=mox.MOX_F_NO_DICT)
    yield e
    e.close()


def gpu_items(e, data):
    try:
        t = e.count(data)
    except mox.Utf8Error:
        return "error"
    try:
        items = t.sorted_items()
        assert sum(c for _, c in items) == t.tokens
        return items
    finally:
        t.close()


def oracle_items(data):
    try:
        return coracle.count(data)[0]
    except coracle.InvalidUtf8:
        return "error"


def test_kats(eng, kat_cases):
    for case in kat_cases:
        data = bytes.fromhex(case["input_hex"])
        assert gpu_items(eng, data) == kat_expected(case), case["name"]


def test_kats_without_dictionary(eng_nodict, kat_cases):
    for case in kat_cases:
        data = bytes.fromhex(case["input_hex"])
        assert gpu_items(eng_nodict, data) == kat_expected(case), case["name"]


ALPH = [b"a", b"B", b"z", b"Q", b"the", b"THE", b" ", b"\t", b"\n", b"\r\n", b"\x0b", b"\x0c", b"\x1c", b"\x00",
        b",", " ".encode(), "　".encode(), " ".encode(), "\u0085".encode(), "​".encode(),
        "Σ".encode(), "σ".encode(), "İ".encode(), "K".encode(), "é".encode(),
        "É".encode(), "́".encode(), "'".encode(), "­".encode(), "日".encode(),
        "\U0001F600".encode(), "Ǆ".encode(), "ß".encode()]


def rand_text(rng, n):
    return b"".join(rng.choice(ALPH) for _ in range(n))


def test_unicode_icu70_kats(eng, eng_nodict):
    """The engine's lowercase + Final_Sigma against ICU 70.1 (Unicode 14.0):
    every probe and hand-picked string of tests/golden/unicode_icu70.json as a
    token, with and without the dictionary, separated by ASCII and by
    multi-byte whitespace."""
    import json
    from collections import Counter
    from test_unicode_pin import FIX, icu_words
    with open(FIX) as f:
        pairs = icu_words(json.load(f))
    want = sorted(Counter(w.encode() for _, w in pairs).items())
    for sep in ("\n", "\u3000", " \u2029"):
        data = sep.join(s for s, _ in pairs).encode()
        assert gpu_items(eng, data) == want, repr(sep)
        assert gpu_items(eng_nodict, data) == want, repr(sep)


def test_fuzz_small(eng):
    rng = random.Random(2024)
    for i in range(300):
        data = rand_text(rng, rng.randint(0, 80))
        if i % 13 == 0 and data:
            k = rng.randrange(len(data))
            data = data[:k] + bytes([rng.choice([0x80, 0xC3, 0xE2, 0xF5, 0xFF])]) + data[k:]
        assert gpu_items(eng, data) == oracle_items(data), data


def test_tile_boundaries(eng):
    """Tokens, multi-byte whitespace and UTF-8 sequences straddling 16 B lanes and 16 KiB tiles."""
    rng = random.Random(77)
    tile = 16 * 1024
    for _ in range(40):
        n = rng.randint(tile - 64, 3 * tile + 64)
        buf = bytearray(rng.choice(b"abcdefghABCDEF  \n") for _ in range(n))
        for _ in range(30):  # plant tricky items at lane / tile edges
            edge = rng.choice([tile, 2 * tile, 16 * rng.randint(1, n // 16 - 1)]) + rng.randint(-3, 2)
            item = rng.choice([b"W" * rng.randint(15, 40), "　".encode(), " ".encode(),
                               "ΣΣ".encode(), "xİy".encode(), b"\x00\x00", b"Q" * 16, b"q" * 17])
            if 0 <= edge and edge + len(item) <= n:
                buf[edge:edge + len(item)] = item
        data = bytes(buf)
        try:
            data.decode("utf-8")
        except UnicodeDecodeError:
            continue
        assert gpu_items(eng, data) == oracle_items(data)


def test_huge_single_token(eng):
    data = b"x" * (3 << 20) + b" tail " + b"Y" * (1 << 20)
    assert gpu_items(eng, data) == oracle_items(data)


@pytest.mark.parametrize("kind", ["zipf", "hicard", "skew", "unicode"])
def test_corpora_exact(eng, kind):
    k = corpus.KINDS[kind]
    data = corpus.fill(k, 0x1234 + k, 0, 24 << 20)
    t = eng.count(data.tobytes())
    got = t.sorted_items()
    tokens = t.tokens
    t.close()
    want, wtok = coracle.count(data, nthreads=16)
    assert tokens == wtok
    assert got == want


def test_dictionary_gate(eng):
    """k_dict_pick builds no dictionary when the sampled words would cover < 5 %
    of the tokens (high-cardinality input); k_map then writes every token as a
    paired cold record.  Zipf text keeps its dictionary.  Both exact."""
    for kind, want_dict in (("hicard", False), ("zipf", True)):
        k = corpus.KINDS[kind]
        data = corpus.fill(k, 0x6A7E + k, 0, 12 << 20)
        t = eng.count(data.tobytes())
        got = t.sorted_items()
        t.close()
        st = eng.stats()
        assert (st["dict_words"] > 1000) == want_dict, (kind, st["dict_words"])
        assert got == coracle.count(data, nthreads=16)[0], kind


def test_misaligned_and_ranges(eng):
    """run_range on a misaligned device pointer and a sub-range equals the oracle's range rule."""
    data = corpus.fill(corpus.UNICODE, 5, 0, 3 << 20).tobytes()
    d = eng.alloc(len(data) + 64)
    try:
        for mis in (0, 1, 7, 13):
            eng.h2d(d + mis, data)
            for a, b in [(0, len(data)), (4, len(data) - 1000), (123457, 2 * 1024 * 1024 + 5)]:
                eng.run_range(d + mis, len(data), a, b, True)
                t = eng.fetch()
                got = t.sorted_items()
                t.close()
                want = coracle.count_range(data, a, b)[0]
                assert got == want, (mis, a, b)
    finally:
        eng.free(d)


def test_shards_merge_to_whole(eng):
    """Byte-range shards with word-boundary fixup sum to the global count."""
    data = corpus.fill(corpus.ZIPF, 11, 0, 8 << 20).tobytes()
    d = eng.alloc(len(data))
    try:
        eng.h2d(d, data)
        cuts = [0, 1 << 20, (3 << 20) + 5, (5 << 20) + 9, len(data)]
        merged = {}
        for a, b in zip(cuts, cuts[1:]):
            eng.run_range(d, len(data), a, b, True)
            t = eng.fetch()
            for w, c in t.items():
                merged[w] = merged.get(w, 0) + c
            t.close()
        assert sorted(merged.items()) == coracle.count(data)[0]
    finally:
        eng.free(d)


def test_dictionary_does_not_change_counts(eng, eng_nodict):
    data = corpus.fill(corpus.SKEW, 3, 0, 8 << 20).tobytes()
    assert gpu_items(eng, data) == gpu_items(eng_nodict, data)


def test_order_is_deterministic(eng):
    data = corpus.fill(corpus.ZIPF, 21, 0, 16 << 20).tobytes()
    t1 = eng.count(data)
    a = t1.arrays()
    t1.close()
    t2 = eng.count(data)
    b = t2.arrays()
    t2.close()
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2]


def test_invalid_utf8_in_big_corpus(eng):
    data = bytearray(corpus.fill(corpus.ZIPF, 8, 0, 4 << 20).tobytes())
    data[3_000_001] = 0xFF
    with pytest.raises(mox.Utf8Error):
        eng.count(bytes(data))
    # the engine stays usable afterwards
    assert gpu_items(eng, b"a b a") == [(b"a", 2), (b"b", 1)]


def test_count_file_and_cli(tmp_path, eng):
    import subprocess
    import os
    from conftest import ROOT
    data = corpus.fill(corpus.ZIPF, 1, 0, 5 << 20).tobytes()  # C1 stand-in for shakes.txt
    (tmp_path / "shakes.txt").write_bytes(data)
    t = eng.count_file(str(tmp_path / "shakes.txt"))
    assert t.sorted_items() == coracle.count(data)[0]
    t.close()
    cli = os.path.join(ROOT, "map-oxidize_amd", "mox", "meduce-gpu")
    r = subprocess.run([cli], cwd=tmp_path, capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.decode().splitlines()
    assert lines[0] == "Top 10 words:" and len(lines) == 11
    # print_top_words (main.rs:184-192): the 10 largest counts, descending;
    # ties may print in any order (the reference's order is HashMap-random)
    want = dict(coracle.count(data)[0])
    top = [line.encode().rsplit(b": ", 1) for line in lines[1:]]
    assert [int(c) for _, c in top] == sorted(want.values(), reverse=True)[:10]
    assert all(want[w] == int(c) for w, c in top)
    final = {}
    for line in (tmp_path / "final_result.txt").read_bytes().split(b"\n"):
        if line:
            w, c = line.rsplit(b" ", 1)
            final[w] = int(c)
    assert sorted(final.items()) == coracle.count(data)[0]


@pytest.mark.slow
def test_full_size_c2(eng):
    """BASELINE config C2 (1 GiB Zipf) exact against the oracle, plus size-independent checks."""
    cfg = corpus.CONFIGS["C2"]
    data = corpus.fill(cfg["kind"], cfg["seed"], 0, cfg["nbytes"])
    d = eng.alloc(data.nbytes)
    try:
        eng.h2d(d, data)
        eng.run_device(d, data.nbytes)
        t = eng.fetch()
        counts, offs, raw = t.arrays()
        tokens = t.tokens
        t.close()
    finally:
        eng.free(d)
    assert int(counts.sum()) == tokens
    wc, wo, wraw, wtok = coracle.count_arrays(data, nthreads=16)
    assert tokens == wtok and counts.size == wc.size
    # sort the GPU table bytewise and compare arrays
    words = [raw[offs[i]:offs[i + 1]] for i in range(counts.size)]
    order = sorted(range(counts.size), key=words.__getitem__)
    assert all(words[j] == wraw[wo[i]:wo[i + 1]] and counts[j] == wc[i] for i, j in enumerate(order))


def _gpu_arrays(e, data):
    t = e.count(data)
    try:
        counts, offs, raw = t.arrays()
        assert int(counts.sum()) == t.tokens
        return counts, offs, raw
    finally:
        t.close()


def test_high_cardinality_split(eng):
    """C4-like input (random 4-16 byte tokens): partitions are mostly distinct, so
    the reduce splits them into sub-bucket units; exact vs oracle."""
    from conftest import assert_tables_equal
    data = corpus.fill(corpus.HICARD, 0x5EED0004, 0, 96 << 20)
    got = _gpu_arrays(eng, data.tobytes())
    st = eng.stats()
    assert st["split_partitions"] > 0 and st["reduce_units"] > 1024, st
    wc, wo, wraw, _ = coracle.count_arrays(data, nthreads=16)
    assert_tables_equal(got, (wc, wo, wraw))


def test_split_mixed_partitions(eng, eng_nodict):
    """Zipf text and high-cardinality tokens in one corpus: split and whole
    partitions side by side, with dictionary words and spills as weighted records."""
    from conftest import assert_tables_equal
    import numpy as np
    z = corpus.fill(corpus.ZIPF, 77, 0, 40 << 20)
    h = corpus.fill(corpus.HICARD, 78, 0, 88 << 20)
    data = np.concatenate([z, np.frombuffer(b" \n", np.uint8), h])
    want = coracle.count_arrays(data, nthreads=16)[:3]
    for e in (eng, eng_nodict):
        assert_tables_equal(_gpu_arrays(e, data.tobytes()), want)
        assert e.stats()["split_partitions"] > 0


def test_split_deterministic_order(eng):
    data = corpus.fill(corpus.HICARD, 5, 0, 96 << 20).tobytes()
    a = _gpu_arrays(eng, data)
    b = _gpu_arrays(eng, data)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2]


def test_count_file_streamed_chunks(tmp_path, eng):
    """mox_count_file reads in 32 MiB chunks through 8 reader threads x 2 pinned
    buffers: a 600 MiB + 12345 byte file exercises buffer reuse and a ragged tail;
    the empty file and a one-word file the edges."""
    from conftest import assert_tables_equal
    import numpy as np
    data = corpus.fill(corpus.ZIPF, 33, 0, (600 << 20) + 12345)
    f = tmp_path / "big.txt"
    data.tofile(str(f))
    t = eng.count_file(str(f))
    got = t.arrays()
    t.close()
    assert eng.stats()["ms_h2d"] > 0
    wc, wo, wraw, _ = coracle.count_arrays(data, nthreads=16)
    assert_tables_equal(got, (wc, wo, wraw))
    for small in (b"", b"Word"):
        g = tmp_path / "small.txt"
        g.write_bytes(small)
        t = eng.count_file(str(g))
        assert t.sorted_items() == coracle.count(small)[0]
        t.close()
    with pytest.raises(mox.MoxError):
        eng.count_file(str(tmp_path / "missing.txt"))


def test_count_file_overlapped_map(tmp_path, eng):
    """Files over 128 MiB: the map runs one launch per 64 MiB range as soon as
    that range and the next have landed, while later chunks are still being
    read (mox_engine.hip run_file_overlapped), and the region counters carry
    over between launches.  Tokens straddling the range ends (a 2-byte UTF-8
    letter, a 5,100-byte long word), a ragged tail, a token longer than the
    look-ahead (falls back to the ordinary pass) and an invalid byte in the
    third range (error offset) must all match the ordinary pass."""
    from conftest import assert_tables_equal
    R = 64 << 20
    n = 3 * R + 777777
    data = bytearray(corpus.fill(corpus.ZIPF, 41, 0, n).tobytes())
    data[R - 4:R + 4] = b" ab\xce\xa3cd "        # "ab\u03a3cd" across the first range end
    data[2 * R - 100:2 * R + 5000] = b"x" * 5100     # a long word across the second
    data[-3:] = b"Zq!"                                # ragged tail ending in a word
    f = tmp_path / "big.txt"
    f.write_bytes(bytes(data))
    t = eng.count_file(str(f))
    got = t.arrays()
    t.close()
    wc, wo, wraw, _ = coracle.count_arrays(np.frombuffer(bytes(data), np.uint8), nthreads=16)
    assert_tables_equal(got, (wc, wo, wraw))
    # a token running past the next range (the look-ahead): ordinary pass on the resident file
    data2 = bytearray(data)
    data2[R - 10:2 * R + 10] = b"y" * (R + 20)
    f.write_bytes(bytes(data2))
    t = eng.count_file(str(f))
    got = t.arrays()
    t.close()
    wc, wo, wraw, _ = coracle.count_arrays(np.frombuffer(bytes(data2), np.uint8), nthreads=16)
    assert_tables_equal(got, (wc, wo, wraw))
    # invalid UTF-8 in the third range: the error names the file offset
    bad = 2 * R + 12345
    data[bad] = 0xFF
    f.write_bytes(bytes(data))
    with pytest.raises(mox.Utf8Error) as ei:
        eng.count_file(str(f))
    assert "byte %d" % bad in str(ei.value)
    assert gpu_items(eng, b"a b a") == [(b"a", 2), (b"b", 1)]


def test_async_passes():
    """mox_run_range_async: back-to-back passes, each completed by the next call
    (or run_wait / fetch); the table is the last pass's; overflow retries and
    errors are handled by the completing call (include/mox.h)."""
    a = corpus.fill(corpus.ZIPF, 21, 0, 6 << 20).tobytes()
    b = corpus.fill(corpus.UNICODE, 22, 0, 3 << 20).tobytes()
    h = corpus.fill(corpus.HICARD, 23, 0, 24 << 20).tobytes()  # grows buffers: retries inside async completion
    bad = a[: 1 << 20] + b"\xc0\x80" + a[1 << 20: 2 << 20]
    want = {k: coracle.count(x)[0] for k, x in (("a", a), ("b", b), ("h", h))}
    e = mox.Engine(device=0, flags=mox.MOX_F_TIMING_MAP)  # fresh: no reserve, so the first passes overflow
    bufs = {}
    try:
        for k, x in (("a", a), ("b", b), ("h", h), ("bad", bad)):
            bufs[k] = e.alloc(len(x))
            e.h2d(bufs[k], x)
        lens = {"a": len(a), "b": len(b), "h": len(h), "bad": len(bad)}

        def run(k):
            e.run_range_async(bufs[k], lens[k], 0, lens[k], True)

        def table():
            t = e.fetch()  # completes pending passes
            try:
                return t.sorted_items()
            finally:
                t.close()

        for seq in (["h", "a"], ["a", "h"], ["a", "b", "a", "b"], ["h", "h", "b"]):
            for k in seq:
                run(k)
            assert table() == want[seq[-1]], seq
        run("a")
        e.run_wait()
        assert e.stats()["ms_map"] > 0
        assert table() == want["a"]
        # an invalid pass reports its error from the call that completes it
        run("bad")
        with pytest.raises(mox.Utf8Error):
            run("b")
        e.run_wait()
        assert table() == want["b"]
    finally:
        for d in bufs.values():
            e.free(d)
        e.close()


def test_sort_bytes_flag():
    """MOX_F_SORT_BYTES: the fetched table is in bytewise order (Rust String
    Ord), i.e. exactly the oracle's list, not only the same multiset."""
    e = mox.Engine(device=0, flags=mox.MOX_F_SORT_BYTES)
    try:
        for data in (corpus.fill(corpus.UNICODE, 7, 0, 3 << 20).tobytes() + b" " + b"z" * 40 + b" " + b"a" * 17,
                     b"b a B \xc3\x89 \x00x x\x00 " + b"k" * 20, b""):
            t = e.count(data)
            got = list(t.items())
            t.close()
            assert got == coracle.count(data)[0]
    finally:
        e.close()


def test_async_side_stream_dictionaries():
    """Async passes build their dictionaries on a side stream during the previous
    pass's reduce tail.  Back-to-back passes over corpora with different hot
    words (Zipf, Unicode, heavy skew, high cardinality: no dictionary), with the
    flags switched between calls (no dictionary, full timing = dictionary on the
    main stream): every completed pass's tokens and distinct words match the
    oracle, and the last table is exact."""
    specs = [(corpus.ZIPF, 31, 6 << 20), (corpus.UNICODE, 32, 3 << 20), (corpus.SKEW, 33, 5 << 20),
             (corpus.HICARD, 34, 4 << 20), (corpus.ZIPF, 35, 2 << 20)]
    datas = [corpus.fill(k, sd, 0, n).tobytes() for k, sd, n in specs]
    want = [coracle.count(x) for x in datas]  # (sorted items, tokens)
    e = mox.Engine(device=0, flags=mox.MOX_F_TIMING_MAP, reserve_bytes=8 << 20)
    try:
        bufs = []
        for x in datas:
            d = e.alloc(len(x))
            e.h2d(d, x)
            bufs.append(d)
        flags = [mox.MOX_F_TIMING_MAP, mox.MOX_F_TIMING_MAP, mox.MOX_F_NO_DICT, mox.MOX_F_TIMING, mox.MOX_F_TIMING_MAP]
        order = [0, 1, 2, 3, 4, 0, 2, 1, 4, 3, 0, 1, 2, 0, 4, 2]
        def check(st, j, i):
            items, tok = want[j]
            assert st["tokens"] == tok and st["uniques"] == len(items), (i, j, st)

        prev, reruns, dropped = None, 0, 0
        for i, j in enumerate(order):
            e.set_flags(flags[i % len(flags)])
            e.run_range_async(bufs[j], len(datas[j]), 0, len(datas[j]), True)
            st = e.stats()
            if st["async_dropped"] != dropped:
                # the previous pass overflowed with this one queued behind it:
                # superseded, not re-run; this one is still pending
                dropped = st["async_dropped"]
                prev = j
                continue
            if st["async_reruns"] != reruns:  # (no pass queued behind an overflowed one)
                reruns = st["async_reruns"]
            if prev is not None:  # this call completed the previous pass
                check(st, prev, i)
            prev = j
        e.run_wait()
        t = e.fetch()
        assert t.sorted_items() == want[order[-1]][0]
        t.close()
        for d in bufs:
            e.free(d)
    finally:
        e.close()


def test_async_overflow_reruns_once():
    """An overflowing async pass with a pass queued behind it is superseded,
    not re-run; the queued pass re-runs at most once if it
    overflowed itself; later passes are not re-run (no cascade)."""
    h = corpus.fill(corpus.HICARD, 23, 0, 24 << 20).tobytes()
    a = corpus.fill(corpus.ZIPF, 24, 0, 4 << 20).tobytes()
    e = mox.Engine(device=0)  # fresh: no reserve, so the first high-cardinality pass overflows
    try:
        dh, da = e.alloc(len(h)), e.alloc(len(a))
        e.h2d(dh, h)
        e.h2d(da, a)
        e.run_range_async(dh, len(h), 0, len(h), True)
        for _ in range(6):
            e.run_range_async(da, len(a), 0, len(a), True)
        e.run_wait()
        st = e.stats()
        # the overflowing first pass is superseded by the one queued behind it
        # (not re-run); that one re-runs at most once itself; no cascade
        assert st["async_reruns"] + st["async_dropped"] <= 2 and st["async_dropped"] <= 1
        t = e.fetch()
        assert t.sorted_items() == coracle.count(a)[0]
        t.close()
        e.free(dh)
        e.free(da)
    finally:
        e.close()


def test_allocation_failure_recovers(monkeypatch):
    """A device allocation failing half-way through a regrow returns MOX_ENOMEM
    and leaves the engine usable: the next call reallocates."""
    monkeypatch.setenv("MOX_TEST_FAIL_ALLOC", "5")
    e = mox.Engine(device=0)
    monkeypatch.delenv("MOX_TEST_FAIL_ALLOC")
    try:
        data = corpus.fill(corpus.ZIPF, 4, 0, 2 << 20).tobytes()
        with pytest.raises(mox.MoxError) as ex:
            e.count(data)
        assert ex.value.code == mox.MOX_ENOMEM
        assert gpu_items(e, data) == oracle_items(data)
    finally:
        e.close()


def test_bounds_check_build():
    """The check build (libmox_check.so, -DMOX_CHECK: every derived index of
    the split / reduce / scatter / table kernels is bounds-checked on the
    device) runs the shapes of the round-1 faults clean: mixed small, big and
    whole reduce units in one k_reduce_small sweep (C4-like text beside Zipf
    text), and a two-rank exchange whose reduce-only pass splits partitions."""
    import os
    import subprocess
    import sys
    from conftest import ROOT
    code = r"""
import sys, threading
sys.path[:0] = [%r, %r, %r]
import numpy as np, coracle, mox
from mox import corpus
from conftest import assert_tables_equal
import test_gpu_exchange as X
z = corpus.fill(corpus.ZIPF, 77, 0, 24 << 20)
h = corpus.fill(corpus.HICARD, 78, 0, 72 << 20)
data = np.concatenate([z, np.frombuffer(b" \n", np.uint8), h])
e = mox.Engine(device=0)
t = e.count(data.tobytes()); got = t.arrays(); t.close()
st = e.stats(); e.close()
assert st["split_partitions"] > 0, st
assert_tables_equal(got, coracle.count_arrays(data, nthreads=16)[:3])
hc = corpus.fill(corpus.HICARD, 91, 0, 48 << 20).tobytes()
out = X.run_ranks(hc, 2)
items = [w for part, _ in out for w in part]
assert sorted(items) == coracle.count(hc, nthreads=16)[0]
print("check build clean")
""" % (os.path.join(ROOT, "map-oxidize_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"))
    env = dict(os.environ, MOX_LIB=os.path.join(ROOT, "map-oxidize_amd", "mox", "libmox_check.so"))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    assert b"check build clean" in r.stdout
