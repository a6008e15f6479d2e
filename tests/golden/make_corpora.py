#!/usr/bin/env python3
"""Freeze golden corpora: a 1 MiB and a 16 MiB Zipf sample
and the C1 5 MiB stand-in for the absent shakes.txt, each as
(generator kind, seed, size) + the SHA-256 of its bytes + the expected word
count: the full sorted table (gzip, "word\\tcount" lines -- Zipf tokens hold no
whitespace) for 1 MiB and 5 MiB, the order-independent digest (distinct words,
sum of counts, two 64-bit mixes) for 16 MiB.

Expected counts come from the C oracle (oracle/mox_oracle.c) and are
cross-checked here against the independent Python restatement
(oracle/pyoracle.py) for the sizes it finishes in seconds.  PARITY UNPINNED
against the reference itself (no Rust toolchain, no reference fixtures:
SURVEY.md §8(c)); what these files pin is that the generator, the oracle and
the engine do not drift.

Regenerate: python tests/golden/make_corpora.py
"""
import gzip
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "map-oxidize_amd"), os.path.join(ROOT, "oracle")]
import coracle  # noqa: E402
import pyoracle  # noqa: E402
from mox import corpus  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
SPECS = [
    # name, kind, seed, bytes, full table?
    ("zipf_1mib", corpus.ZIPF, 0x601D, 1 << 20, True),
    ("c1_standin_5mib", corpus.CONFIGS["C1"]["kind"], corpus.CONFIGS["C1"]["seed"], corpus.CONFIGS["C1"]["nbytes"], True),
    ("zipf_16mib", corpus.ZIPF, 0x1601D, 16 << 20, False),
]


def table_lines(items):
    out = bytearray()
    for w, c in items:
        assert b"\t" not in w and b"\n" not in w
        out += w + b"\t" + str(c).encode() + b"\n"
    return bytes(out)


def main():
    manifest = {"note": __doc__.strip().splitlines()[0], "corpora": []}
    for name, kind, seed, nbytes, full in SPECS:
        data = corpus.fill(kind, seed, 0, nbytes)
        raw = data.tobytes()
        ent = {"name": name, "kind": kind, "seed": seed, "bytes": nbytes, "sha256": hashlib.sha256(raw).hexdigest()}
        items, tokens = coracle.count(data, nthreads=8)
        ent["tokens"] = tokens
        ent["distinct"] = len(items)
        ent["digest"] = list(coracle.count_digest(data, nthreads=8)[0])
        if nbytes <= (5 << 20):  # the independent restatement agrees (pure Python: seconds)
            assert pyoracle.sorted_items(pyoracle.count_words(raw)) == items, name
            ent["pyoracle_checked"] = True
        if full:
            fn = "corpus_%s.counts.gz" % name
            with gzip.GzipFile(os.path.join(HERE, fn), "wb", mtime=0) as f:
                f.write(table_lines(items))
            ent["counts_file"] = fn
        manifest["corpora"].append(ent)
        print(name, ent["sha256"][:16], tokens, len(items), flush=True)
    with open(os.path.join(HERE, "corpora.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
