import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "map-oxidize_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running (large corpora)")


@pytest.fixture(scope="session")
def kat_cases():
    with open(os.path.join(ROOT, "tests", "golden", "kat.json")) as f:
        return json.load(f)["cases"]


def kat_expected(case):
    if "error" in case:
        return "error"
    return [(bytes.fromhex(w), c) for w, c in case["expected"]]


def canon_table(counts, offs, raw):
    """(keys, counts) of a word table sorted bytewise, vectorised with numpy:
    words become fixed-width 'S' strings (zero padded; words hold no NUL byte),
    so big tables compare without building Python objects per word."""
    import numpy as np
    counts = np.asarray(counts, dtype=np.uint64)
    offs = np.asarray(offs, dtype=np.int64)
    n = counts.size
    if n == 0:
        return np.zeros(0, "S1"), counts
    lens = np.diff(offs)
    width = int(lens.max())
    buf = np.frombuffer(raw, dtype=np.uint8)
    assert not (buf == 0).any(), "canon_table needs NUL-free words"
    cols = np.arange(width, dtype=np.int64)
    idx = offs[:-1, None] + cols[None, :]
    mat = np.where(cols[None, :] < lens[:, None], buf[np.minimum(idx, max(buf.size - 1, 0))], 0).astype(np.uint8)
    keys = np.ascontiguousarray(mat).view("S%d" % width).ravel()
    order = np.argsort(keys, kind="stable")
    return keys[order], counts[order]


def split_long(counts, offs, raw, width=64):
    """(short table, long words): words longer than `width` bytes leave the table
    as a sorted list of (bytes, count), so canon_table's fixed-width matrix
    stays narrow when a corpus holds a few very long tokens."""
    import numpy as np
    counts = np.asarray(counts, dtype=np.uint64)
    offs = np.asarray(offs, dtype=np.int64)
    lens = np.diff(offs)
    longi = np.nonzero(lens > width)[0]
    if longi.size == 0:
        return (counts, offs, raw), []
    longw = sorted((raw[offs[i]:offs[i + 1]], int(counts[i])) for i in longi)
    keep = np.nonzero(lens <= width)[0]
    klen = lens[keep]
    koffs = np.zeros(keep.size + 1, np.int64)
    np.cumsum(klen, out=koffs[1:])
    buf = np.frombuffer(raw, np.uint8)
    idx = np.repeat(offs[keep], klen) + (np.arange(int(koffs[-1])) - np.repeat(koffs[:-1], klen))
    return (counts[keep], koffs, buf[idx].tobytes()), longw


def assert_tables_equal(a, b):
    """a, b: (counts, offs, raw) word tables; equal as (word, count) multisets."""
    import numpy as np
    (a, la), (b, lb) = split_long(*a), split_long(*b)
    assert la == lb
    ka, ca = canon_table(*a)
    kb, cb = canon_table(*b)
    assert ka.size == kb.size, (ka.size, kb.size)
    assert np.array_equal(ka, kb)
    assert np.array_equal(ca, cb)
