"""CPU: the bytewise table order of MOX_F_SORT_BYTES (mox_table_sort_bytes,
map-oxidize_amd/csrc/mox_table.cpp) -- host code of libmox.so, exercised on
tables built here (no GPU).  The order is Rust `String` Ord: memcmp over the
common length, then the shorter word first."""
import ctypes
import random

import numpy as np

import mox


def sort_via_lib(words, counts):
    n = len(words)
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(w) for w in words])
    cnt = np.array(counts, dtype=np.uint64)
    raw = np.frombuffer(b"".join(words) or b"\0", dtype=np.uint8).copy()
    t = mox._Table()
    t.n = n
    t.tokens = int(cnt.sum())
    t.counts = cnt.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    t.offs = offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    t.bytes = raw.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
    rc = mox.lib().mox_table_sort_bytes(ctypes.byref(t))
    assert rc == 0
    out = [(raw[offs[i]:offs[i + 1]].tobytes(), int(cnt[i])) for i in range(n)]
    return out


def test_sort_matches_python_bytes_order():
    rng = random.Random(5)
    alphabet = [b"a", b"b", b"\x00", b"\xff", b"z", "é".encode(), b"A"]
    words = set()
    while len(words) < 3000:
        words.add(b"".join(rng.choice(alphabet) for _ in range(rng.randint(1, 24))))
    words = list(words)
    rng.shuffle(words)
    counts = [rng.randint(1, 1 << 40) for _ in words]
    got = sort_via_lib(words, counts)
    assert got == sorted(zip(words, counts))


def test_sort_prefixes_and_long_shared_prefix():
    words = [b"abc", b"ab", b"abcdefghij", b"abcdefghi", b"abcdefgh\x00", b"abcdefgh", b"a" * 40, b"a" * 39 + b"b",
             b"the", b"the,", b"the."]
    got = sort_via_lib(words, list(range(1, len(words) + 1)))
    assert [w for w, _ in got] == sorted(words)
    assert dict(got) == dict(zip(words, range(1, len(words) + 1)))


def test_sort_large_parallel_path():
    """> 65,536 entries takes the threaded path."""
    rng = np.random.default_rng(3)
    n = 200_000
    lens = rng.integers(1, 20, n)
    raw = rng.integers(ord("a"), ord("e"), lens.sum(), dtype=np.uint8).tobytes()
    offs = np.concatenate([[0], np.cumsum(lens)])
    words = sorted({raw[offs[i]:offs[i + 1]] for i in range(n)})
    order = list(range(len(words)))
    random.Random(1).shuffle(order)
    shuffled = [words[i] for i in order]
    got = sort_via_lib(shuffled, [i + 1 for i in order])
    assert [w for w, _ in got] == words
    assert [c for _, c in got] == list(range(1, len(words) + 1))


def test_sort_empty_and_single():
    assert sort_via_lib([], []) == []
    assert sort_via_lib([b"x"], [3]) == [(b"x", 3)]
