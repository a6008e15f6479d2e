"""CPU: the C oracle against the golden KATs and the independent Python oracle."""
import os
import random
import subprocess

import pytest

import coracle
import pyoracle
from conftest import ROOT, kat_expected


def c_count(data):
    try:
        return coracle.count(data)[0]
    except coracle.InvalidUtf8:
        return "error"


def py_count(data):
    try:
        return pyoracle.sorted_items(pyoracle.count_words(data))
    except pyoracle.InvalidUtf8:
        return "error"


def test_c_oracle_matches_golden(kat_cases):
    assert len(kat_cases) > 150
    for case in kat_cases:
        data = bytes.fromhex(case["input_hex"])
        assert c_count(data) == kat_expected(case), case["name"]


def test_golden_regenerates_identically(kat_cases):
    # the committed vectors are what the committed generator writes
    for case in kat_cases:
        data = bytes.fromhex(case["input_hex"])
        assert py_count(data) == kat_expected(case), case["name"]


ALPH = [b"a", b"B", b"z", b"Q", b" ", b"\t", b"\n", b"\r", b"\x0b", b"\x0c", b"\x1c", b"\x00", b",", b".",
        " ".encode(), "　".encode(), " ".encode(), "\u0085".encode(), "​".encode(),
        "Σ".encode(), "σ".encode(), "ς".encode(), "İ".encode(), "K".encode(), "é".encode(), "É".encode(),
        "́".encode(), "'".encode(), "­".encode(), "日".encode(), "😀".encode(), "Ǆ".encode(), "ß".encode()]


def rand_text(rng, n):
    return b"".join(rng.choice(ALPH) for _ in range(n))


def test_c_oracle_vs_python_fuzz():
    rng = random.Random(1234)
    for i in range(400):
        data = rand_text(rng, rng.randint(0, 60))
        if i % 17 == 0 and data:  # sprinkle invalid UTF-8
            k = rng.randrange(len(data))
            data = data[:k] + bytes([rng.choice([0x80, 0xC3, 0xE2, 0xF5, 0xFF, 0xED])]) + data[k:]
        assert c_count(data) == py_count(data), data


def test_c_oracle_threads_agree():
    rng = random.Random(7)
    data = b"\n".join(rand_text(rng, 40) for _ in range(2000))
    assert coracle.count(data, nthreads=1)[0] == coracle.count(data, nthreads=8)[0]


def test_reference_pipeline_equals_global_count():
    # main.rs: round-robin line chunks + spill files + 2-field parse + merge == one global count
    rng = random.Random(99)
    for _ in range(50):
        data = b"\n".join(rand_text(rng, rng.randint(0, 30)) for _ in range(rng.randint(0, 20)))
        try:
            a = pyoracle.reference_pipeline(data)
        except pyoracle.InvalidUtf8:
            continue
        assert a == pyoracle.count_words(data)


def test_count_range_partitions_tokens():
    rng = random.Random(5)
    for _ in range(200):
        data = rand_text(rng, rng.randint(1, 80))
        try:
            whole = dict(coracle.count(data)[0])
        except coracle.InvalidUtf8:
            continue
        cuts = sorted(rng.sample(range(len(data) + 1), k=min(3, len(data) + 1)))
        cuts = [0] + [c for c in cuts if c >= 4] + [len(data)]
        merged = {}
        for a, b in zip(cuts, cuts[1:]):
            if a >= b:
                continue
            for w, c in coracle.count_range(data, a, b)[0]:
                merged[w] = merged.get(w, 0) + c
        assert merged == whole, (data, cuts)


def test_meduce_ref_faithful_pipeline(tmp_path):
    """oracle/build/meduce_ref (the CPU baseline) reproduces main.rs's outputs."""
    from mox import corpus
    data = corpus.fill(corpus.ZIPF, 1, 0, 1 << 20).tobytes()
    src = tmp_path / "shakes.txt"
    src.write_bytes(data)
    r = subprocess.run([coracle.MEDUCE_REF, str(src), "--workdir", str(tmp_path)], capture_output=True, check=True)
    lines = r.stdout.decode().splitlines()
    assert lines[0] == "Top 10 words:"
    final = {}
    for line in (tmp_path / "final_result.txt").read_bytes().split(b"\n"):
        if line:
            w, c = line.rsplit(b" ", 1)
            final[w] = int(c)
    expect = dict(coracle.count(data)[0])
    assert final == expect
    top = sorted(expect.values(), reverse=True)[:10]
    assert [int(l.rsplit(": ", 1)[1]) for l in lines[1:11]] == top
    assert sum(1 for l in lines if l.startswith("Successfully deleted: map_")) == 8
    assert not list(tmp_path.glob("map_*_chunk_*.txt"))
    bad = tmp_path / "bad.txt"
    bad.write_bytes(b"ok \xff no")
    r = subprocess.run([coracle.MEDUCE_REF, str(bad), "--workdir", str(tmp_path)], capture_output=True)
    assert r.returncode == 1


def test_canon_table_matches_python_sort():
    """The vectorised table comparison used by the big GPU parity tests."""
    import numpy as np
    from conftest import canon_table
    from mox import corpus
    data = corpus.fill(corpus.HICARD, 3, 0, 1 << 20)
    counts, offs, raw, _ = coracle.count_arrays(data)
    perm = np.random.default_rng(0).permutation(counts.size)
    words = [raw[offs[i]:offs[i + 1]] for i in perm]
    poffs = np.zeros(len(words) + 1, dtype=np.int64)
    poffs[1:] = np.cumsum([len(w) for w in words])
    keys, cs = canon_table(counts[perm], poffs, b"".join(words))
    want = sorted(zip(words, counts[perm].tolist()))
    assert [k for k in keys.tolist()] == [w for w, _ in want]
    assert cs.tolist() == [c for _, c in want]
