"""CPU: the synthetic corpora are deterministic and block-addressable."""
import numpy as np

from mox import corpus
import coracle


def test_block_addressable():
    whole = corpus.fill(corpus.ZIPF, 42, 0, 5 << 20)
    part = corpus.fill(corpus.ZIPF, 42, 3 * (1 << 20) - 12345, 1 << 20)
    assert np.array_equal(whole[3 * (1 << 20) - 12345: 4 * (1 << 20) - 12345], part)


def test_deterministic_and_seeded():
    a = corpus.fill(corpus.HICARD, 4, 0, 1 << 20, nthreads=1)
    b = corpus.fill(corpus.HICARD, 4, 0, 1 << 20, nthreads=8)
    c = corpus.fill(corpus.HICARD, 5, 0, 1 << 20)
    assert np.array_equal(a, b) and not np.array_equal(a, c)


def test_unicode_kind_is_valid_utf8():
    d = corpus.fill(corpus.UNICODE, 9, 0, 4 << 20)
    d.tobytes().decode("utf-8")  # strict


def test_zipf_shape():
    d = corpus.fill(corpus.ZIPF, 0x5EED0002, 0, 8 << 20)
    words, tokens = coracle.count(d)
    counts = sorted((c for _, c in words), reverse=True)
    assert 5.0 < d.size / tokens < 7.0          # ~6 B per token + delimiter
    assert 0.08 < counts[0] / tokens < 0.16     # top word ~11%
    assert sum(counts[:4096]) / tokens > 0.75   # hot-dictionary coverage


def test_skew_shape():
    d = corpus.fill(corpus.SKEW, 0x5EED0005, 0, 4 << 20)
    words, tokens = coracle.count(d)
    counts = sorted((c for _, c in words), reverse=True)
    assert sum(counts[:10]) / tokens > 0.85
