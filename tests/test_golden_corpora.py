"""Frozen golden corpora (tests/golden/make_corpora.py):
generator bytes pinned by SHA-256, expected word counts committed (full sorted
tables for 1 MiB and the 5 MiB C1 stand-in, a digest for 16 MiB).  The CPU
tests check the generator and the C oracle against the committed files; the
GPU tests compare the engine's tables with the committed files, not with a
live oracle run, so a drift of the generator or the oracle cannot hide."""
import gzip
import hashlib
import json
import os

import numpy as np
import pytest

import coracle
import mox
from mox import corpus
from conftest import ROOT

GOLD = os.path.join(ROOT, "tests", "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "corpora.json")))["corpora"]


def load_counts(fn):
    with gzip.open(os.path.join(GOLD, fn), "rb") as f:
        out = []
        for line in f.read().split(b"\n"):
            if line:
                w, c = line.rsplit(b"\t", 1)
                out.append((w, int(c)))
        return out


def gen(ent):
    return corpus.fill(ent["kind"], ent["seed"], 0, ent["bytes"])


@pytest.mark.parametrize("ent", MANIFEST, ids=[e["name"] for e in MANIFEST])
def test_generator_bytes_pinned(ent):
    assert hashlib.sha256(gen(ent).tobytes()).hexdigest() == ent["sha256"]


@pytest.mark.parametrize("ent", MANIFEST, ids=[e["name"] for e in MANIFEST])
def test_oracle_matches_committed_counts(ent):
    data = gen(ent)
    digest, tokens = coracle.count_digest(data, nthreads=8)
    assert tokens == ent["tokens"] and list(digest) == ent["digest"] and digest[0] == ent["distinct"]
    if "counts_file" in ent:
        items, tok = coracle.count(data, nthreads=8)
        assert items == load_counts(ent["counts_file"])


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, mox.MOX_F_NO_DICT], ids=["dict", "nodict"])
def test_engine_matches_committed_counts(flags):
    e = mox.Engine(device=0, flags=flags | mox.MOX_F_SORT_BYTES)
    try:
        for ent in MANIFEST:
            data = gen(ent).tobytes()
            assert hashlib.sha256(data).hexdigest() == ent["sha256"]
            t = e.count(data)
            try:
                assert t.tokens == ent["tokens"] and t.n == ent["distinct"], ent["name"]
                if "counts_file" in ent:
                    assert list(t.items()) == load_counts(ent["counts_file"]), ent["name"]  # bytewise order
                counts, offs, raw = t.arrays()
                assert list(coracle.table_digest(counts, offs, raw)) == ent["digest"], ent["name"]
            finally:
                t.close()
    finally:
        e.close()
