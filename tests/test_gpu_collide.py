"""GPU: the forced-collision check build (libmox_hc.so).

Every exactness fallback of the engine runs only when two different words
share a hash: the token pass's full-key compare against a dictionary word of
the same hash (k_map),
the long-word table's byte compare behind an equal FNV-1a hash, the one-wave
sort reduce's 64-bit re-sort and its hand-off to k_reduce, and the key
compares of the k_reduce / k_reduce_small tables.  With full hashes these are
rare (C4's natural 23-bit sort-key collisions aside).  The collision build
(-DMOX_HASH_COLLIDE, mox_internal.h) keeps 22 bits of the 32-bit key hash, 2
bits of the order hash and 8 bits of the FNV-1a-64, so they fire constantly;
it also carries the bounds checks (-DMOX_CHECK).  Each test is bit-exact
against the oracle AND asserts, through the build's path counters
(mox_stats.path_hits), that the fallback it targets actually ran."""
import os
import random

import numpy as np
import pytest

import coracle
import mox
from mox import corpus
from conftest import assert_tables_equal, kat_expected

pytestmark = pytest.mark.gpu

HC = mox.HC_LIB_PATH


@pytest.fixture(scope="module")
def hc():
    e = mox.Engine(device=0, lib_path=HC)
    yield e
    e.close()


@pytest.fixture(scope="module")
def hc_nodict():
    e = mox.Engine(device=0, flags=mox.MOX_F_NO_DICT, lib_path=HC)
    yield e
    e.close()


def items(e, data):
    try:
        t = e.count(data)
    except mox.Utf8Error:
        return "error"
    try:
        it = t.sorted_items()
        assert sum(c for _, c in it) == t.tokens
        return it
    finally:
        t.close()


def arrays(e, data):
    t = e.count(data)
    try:
        counts, offs, raw = t.arrays()
        assert int(counts.sum()) == t.tokens
        return counts, offs, raw
    finally:
        t.close()


def hits(e):
    return e.stats()["path_hits"]


def test_hc_build_loaded():
    assert os.path.exists(HC)
    assert mox.lib(HC).mox_abi_version() == mox.lib().mox_abi_version()


def test_kats_collide(hc, hc_nodict, kat_cases):
    for case in kat_cases:
        data = bytes.fromhex(case["input_hex"])
        assert items(hc, data) == kat_expected(case), case["name"]
        assert items(hc_nodict, data) == kat_expected(case), case["name"]


def test_fuzz_collide(hc):
    from test_gpu_parity import rand_text, oracle_items
    rng = random.Random(4242)
    for i in range(120):
        data = rand_text(rng, rng.randint(0, 80))
        assert items(hc, data) == oracle_items(data), data


def test_zipf_dictionary_same_hash_words(hc):
    """Zipf text with the dictionary: with 22-bit key hashes many distinct words
    share their hash (and so both dictionary slots) with a dictionary word; the
    token pass compares the full 16-byte keys, so each such token is counted as
    its own (cold) word, never as the dictionary word."""
    data = corpus.fill(corpus.ZIPF, 0xC011, 0, 24 << 20)
    got = arrays(hc, data.tobytes())
    ph = hits(hc)
    assert hc.stats()["dict_words"] > 1000
    assert ph[mox.PATH_DICT_SAMEHASH] > 0, ph
    assert_tables_equal(got, coracle.count_arrays(data, nthreads=16)[:3])


def test_high_cardinality_sort_fallbacks(hc):
    """C4-like text: split partitions, count-1 units reduced by one wave; keys
    sharing the 23-bit sort key are re-sorted on 64-bit keys, keys sharing
    (h32, hash32b) send their unit to k_reduce, whose table then compares
    keys behind equal tags."""
    data = corpus.fill(corpus.HICARD, 0xC012, 0, 96 << 20)
    got = arrays(hc, data.tobytes())
    st = hc.stats()
    ph = st["path_hits"]
    assert st["split_partitions"] > 0, st
    assert ph[mox.PATH_SORT_RESORT] > 0 and ph[mox.PATH_SORT_TO_RED] > 0 and ph[mox.PATH_RED_TAG] > 0, ph
    assert_tables_equal(got, coracle.count_arrays(data, nthreads=16)[:3])


def test_mixed_small_units(hc, hc_nodict):
    """Zipf + C4-like text in one corpus: split partitions holding dictionary
    totals and spills are reduced by k_reduce_small, whose LDS table compares
    keys behind equal hashes; with and without the dictionary."""
    z = corpus.fill(corpus.ZIPF, 0xC013, 0, 40 << 20)
    h = corpus.fill(corpus.HICARD, 0xC014, 0, 88 << 20)
    data = np.concatenate([z, np.frombuffer(b" \n", np.uint8), h])
    want = coracle.count_arrays(data, nthreads=16)[:3]
    for e in (hc, hc_nodict):
        assert_tables_equal(arrays(e, data.tobytes()), want)
        assert e.stats()["split_partitions"] > 0
    ph = hits(hc)
    assert ph[mox.PATH_SMALL_TAG] > 0 and ph[mox.PATH_RED_TAG] > 0, ph


def long_word_corpus(seed, n_distinct=40000, tokens=300000):
    """Words of 17..48 bytes (ASCII, some capitalised, some with Unicode
    letters that go through the Unicode lane) from a vocabulary of n_distinct,
    with Zipf-like repeats, plus short words between them."""
    rng = np.random.default_rng(seed)
    letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", np.uint8)
    vocab = []
    for i in range(n_distinct):
        L = int(rng.integers(17, 49))
        w = bytes(letters[rng.integers(0, 26, L)])
        if i % 7 == 0:
            w = w.capitalize()
        if i % 11 == 0:
            w = w[:8] + "Σé".encode() + w[8:]
        vocab.append(w)
    ranks = np.minimum((rng.pareto(0.8, tokens) * 3).astype(np.int64), n_distinct - 1)
    short = [b"the", b"of", b"and", b"x", b"longish"]
    out = []
    for k, r in enumerate(ranks):
        out.append(vocab[r])
        out.append(short[k % 5])
    return b" ".join(out) + b"\n"


def test_long_word_equal_hash_byte_compare(hc, hc_nodict):
    """~40,000 distinct words longer than 16 bytes in 256 FNV-1a values: the
    long-word table's inserts meet equal hashes of other words and compare
    bytes (ASCII corpus references and Unicode-lane arena references)."""
    data = long_word_corpus(0xC015)
    want = coracle.count(data, nthreads=16)[0]
    assert items(hc, data) == want
    assert hits(hc)[mox.PATH_LONG_EQHASH] > 0
    assert items(hc_nodict, data) == want


def test_exchange_two_ranks_collide():
    """A 2-rank host-transport exchange and gather in the collision build: the
    received partials are reduced by k_reduce / k_reduce_small / the long table
    under colliding hashes; exact against the oracle."""
    import test_gpu_exchange as X
    data = X.mixed_corpus(6 << 20, 0xC016) + b" " + long_word_corpus(0xC017, 5000, 40000)
    st = []
    out = X.run_ranks(data, 2, gather_root=0, lib_path=HC, stats=st)
    want, wtok = coracle.count(data, nthreads=16)
    assert out[0][1] == wtok
    assert out[0][0] == want
    assert sum(s["path_hits"][mox.PATH_LONG_EQHASH] for s in st) > 0


def test_reduce_pairs_collide(hc):
    """mox_reduce_pairs (spill-file path) with colliding short and long keys:
    duplicate words summed exactly."""
    rng = random.Random(0xC018)
    words, counts = [], []
    base = [b"w%05d" % i for i in range(20000)] + [b"L" * 17 + b"%06d" % i for i in range(3000)]
    for _ in range(60000):
        words.append(rng.choice(base))
        counts.append(rng.randint(1, 1 << 40))
    want = {}
    for w, c in zip(words, counts):
        want[w] = want.get(w, 0) + c
    t = hc.reduce_pairs(words, counts)
    got = t.sorted_items()
    t.close()
    assert got == sorted(want.items())
    assert hits(hc)[mox.PATH_LONG_EQHASH] > 0
