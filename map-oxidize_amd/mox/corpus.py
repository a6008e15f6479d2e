"""Deterministic synthetic corpora (map-oxidize_amd/csrc/mox_corpus.c).

Benchmark configs (BASELINE.json / SURVEY.md §8(d)):
  C1 shakes.txt stand-in: ZIPF, 5 MiB, seed 1
  C2 1 GiB ZIPF(1.1), seed 0x5EED0002
  C3 64 GiB ZIPF, seed 0x5EED0003, 8 shards
  C4 16 GiB HICARD, seed 0x5EED0004
  C5 16 GiB SKEW, seed 0x5EED0005
"""
import ctypes
import os

import numpy as np

ZIPF, HICARD, SKEW, UNICODE = 1, 2, 3, 4
KINDS = {"zipf": ZIPF, "hicard": HICARD, "skew": SKEW, "unicode": UNICODE}
CONFIGS = {
    "C1": dict(kind=ZIPF, seed=1, nbytes=5 << 20),
    "C2": dict(kind=ZIPF, seed=0x5EED0002, nbytes=1 << 30),
    "C3": dict(kind=ZIPF, seed=0x5EED0003, nbytes=64 << 30),
    "C4": dict(kind=HICARD, seed=0x5EED0004, nbytes=16 << 30),
    "C5": dict(kind=SKEW, seed=0x5EED0005, nbytes=16 << 30),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmox_corpus.so")
        L = ctypes.CDLL(path)
        L.mox_corpus_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                      ctypes.c_void_p, ctypes.c_int]
        L.mox_corpus_fill.restype = ctypes.c_int
        L.mox_corpus_vocab_word.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_int]
        L.mox_corpus_vocab_word.restype = ctypes.c_int
        _lib = L
    return _lib


def fill(kind, seed, offset, nbytes, out=None, nthreads=None):
    """Bytes [offset, offset+nbytes) of corpus (kind, seed) as a uint8 array."""
    if out is None:
        out = np.empty(nbytes, dtype=np.uint8)
    if nthreads is None:
        nthreads = min(16, os.cpu_count() or 1)
    rc = lib().mox_corpus_fill(kind, seed, offset, nbytes, out.ctypes.data, nthreads)
    if rc != 0:
        raise ValueError("bad corpus kind %r" % kind)
    return out


def vocab_word(rank):
    buf = ctypes.create_string_buffer(64)
    n = lib().mox_corpus_vocab_word(rank, buf, 64)
    return buf.raw[:n]
