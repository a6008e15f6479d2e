"""Spill-file compatibility (mox/spill.py).

CPU: the host text logic against the reference's rules (tokio lines(),
split_file round-robin, read_map_result's 2-field / usize parser, last wins)
and against oracle/pyoracle.reference_pipeline.  GPU: map files written from
GPU chunk counts, reduce_phase through mox_reduce_pairs, exact vs the oracle.
"""
import os
import random

import pytest

import coracle
import pyoracle
import mox
from mox import corpus, spill


# ---------------------------------------------------------------- CPU (host logic)
def test_lines_like_tokio():
    assert spill.lines(b"") == []
    assert spill.lines(b"a") == [b"a"]
    assert spill.lines(b"a\n") == [b"a"]
    assert spill.lines(b"a\r\nb\r") == [b"a", b"b\r"]  # '\r' dropped only before '\n'
    assert spill.lines(b"a\n\nb\n") == [b"a", b"", b"b"]
    assert spill.lines(b"\r\n") == [b""]
    with pytest.raises(UnicodeDecodeError):
        spill.lines(b"ok\n\xc0\x80\n")


def test_split_file_round_robin():
    rnd = random.Random(5)
    lines = [b"w%d %s" % (i, b"x" * rnd.randrange(5)) for i in range(37)]
    data = b"\r\n".join(lines[:10]) + b"\n" + b"\n".join(lines[10:])
    chunks = spill.split_file(data, 8)
    assert len(chunks) == 8
    for c in range(8):
        assert chunks[c] == b"".join(ln + b"\n" for ln in lines[c::8])


def test_map_file_names_pop_order():
    names = spill.map_file_names(8, 8)
    assert names[7] == "map_0_chunk_7.txt" and names[0] == "map_7_chunk_0.txt"
    assert spill.map_file_names(8, 3)[4] == "map_0_chunk_4.txt"


def test_read_map_result_rules(tmp_path):
    p = tmp_path / "m.txt"
    p.write_bytes(
        "a 1\n"
        "b 1 2\n"           # three fields: skipped
        "c\n"               # one field: skipped
        "d x\n"             # not a usize: skipped
        "e -3\n"            # unsigned: '-' rejected
        "f +5\n"            # Rust usize accepts a leading '+'
        "g 18446744073709551616\n"  # 2^64: overflow, skipped
        "h 18446744073709551615\n"
        "a 7\r\n"           # repeated word: last wins (HashMap::insert); CRLF
        "i　9\n"        # ideographic space separates fields
        "j\x1c 4\n"         # U+001C is not Rust whitespace: part of the word
        "  k   2  \n"
        "l 3".encode()
    )
    got = spill.read_map_result(str(p))
    assert got == {b"a": 7, b"f": 5, b"h": (1 << 64) - 1, b"i": 9, b"j\x1c": 4, b"k": 2, b"l": 3}


class _OracleTable:
    """Stand-in for mox.Table in the host-logic test (counts from the C oracle)."""

    def __init__(self, items):
        self.items = items

    def write_final_result(self, path):
        with open(path, "wb") as f:
            for w, c in self.items:
                f.write(w + b" %d\n" % c)

    def close(self):
        pass


class _OracleEngine:
    def count(self, data):
        return _OracleTable(coracle.count(data)[0])

    def reduce_pairs(self, words, counts):
        tot = {}
        for w, c in zip(words, counts):
            tot[w] = tot.get(w, 0) + c
        return sorted(tot.items())


def test_pipeline_host_logic_matches_reference_pipeline(tmp_path):
    data = corpus.fill(corpus.UNICODE, 3, 0, 64 << 10).tobytes() + b"\r\nTail Words tail"
    paths = spill.map_phase(_OracleEngine(), spill.split_file(data), str(tmp_path))
    assert sorted(os.path.basename(p) for p in paths) == sorted(spill.map_file_names().values())
    got = spill.reduce_phase(_OracleEngine(), paths)
    assert got == pyoracle.sorted_items(pyoracle.reference_pipeline(data))


def test_pack_pairs():
    data, offs, cnt = spill.pack_pairs([b"ab", b"", b"cde"], [1, 2, 3])
    assert data == b"abcde" and list(offs) == [0, 2, 2, 5] and list(cnt) == [1, 2, 3]


# ---------------------------------------------------------------- GPU
def _mixed(n, seed):
    z = corpus.fill(corpus.ZIPF, seed, 0, n).tobytes()
    u = corpus.fill(corpus.UNICODE, seed + 1, 0, n // 8).tobytes()
    extra = b"\n".join(b"Antidisestablishmentarianism%d LONGWORD%dxxxxxxxxxxxxxx" % (i % 53, i % 7) for i in range(2000))
    return z[: n // 2] + b"\n" + u + b"\n" + extra + b"\n" + z[n // 2:]


@pytest.mark.gpu
def test_gpu_spill_pipeline(tmp_path):
    data = _mixed(3 << 20, 21)
    e = mox.Engine(device=0)
    try:
        chunks = spill.split_file(data)
        paths = spill.map_phase(e, chunks, str(tmp_path))
        by_name = {os.path.basename(p): p for p in paths}
        for c, name in spill.map_file_names().items():  # every map file = its chunk's count
            assert sorted(spill.read_map_result(by_name[name]).items()) == coracle.count(chunks[c])[0]
        t = spill.reduce_phase(e, paths)
        got, tokens = t.sorted_items(), t.tokens
        t.close()
    finally:
        e.close()
    want, wtok = coracle.count(data)
    assert got == want
    assert tokens == wtok
    spill.cleanup(paths)
    assert not any(os.path.exists(p) for p in paths)


@pytest.mark.gpu
def test_gpu_reduce_pairs_edge_cases():
    rnd = random.Random(11)
    words = [b"a", b"A", b"abcdefghijklmnop", b"abcdefghijklmnopq", b"x\x00y", b"\x00", b"\xc3\xa9t\xc3\xa9",
             b"Z" * 300, b"z" * 17]
    pairs = [(rnd.choice(words), rnd.randrange(1, 1000)) for _ in range(5000)]
    pairs += [(b"big", (1 << 62)), (b"big", 5)]
    want = {}
    for w, c in pairs:
        want[w] = want.get(w, 0) + c
    e = mox.Engine(device=0)
    try:
        t = e.reduce_pairs([w for w, _ in pairs], [c for _, c in pairs])
        got = t.sorted_items()
        assert t.tokens == sum(c for _, c in pairs)
        t.close()
        t = e.reduce_pairs([], [])
        assert t.n == 0 and t.tokens == 0
        t.close()
        # a normal run still works after a reduce-only pass on the same engine
        t = e.count(b"b a A b")
        assert t.sorted_items() == [(b"a", 2), (b"b", 2)]
        t.close()
    finally:
        e.close()
    assert got == sorted(want.items())


@pytest.mark.gpu
def test_gpu_reduce_pairs_many():
    """2e6 pairs over ~3e5 distinct short words: exact sums through the split/reduce tail."""
    import numpy as np
    rng = np.random.default_rng(4)
    ids = rng.integers(0, 300_000, size=2_000_000)
    cnt = rng.integers(1, 50, size=ids.size)
    words = [b"w%x" % i for i in ids.tolist()]
    e = mox.Engine(device=0)
    try:
        t = e.reduce_pairs(words, cnt.tolist())
        got = t.sorted_items()
        t.close()
    finally:
        e.close()
    sums = np.bincount(ids, weights=cnt, minlength=300_000).astype(np.int64)
    want = sorted((b"w%x" % i, int(s)) for i, s in enumerate(sums) if s)
    assert got == want
