"""Same tables from two engine builds: counts, byte offsets and bytes, in table
order (the key_less order), on high-cardinality, mixed and Zipf corpora.
An A/B variant whose reduce kernels change only how they sort must give the
default build's arrays exactly.

Usage (GPU box): python3 tools/cmp_order.py build/var_NAME/libmox.so [LIB_B]
(LIB_B defaults to the in-tree libmox.so)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "map-oxidize_amd"))
import mox  # noqa: E402
from mox import corpus  # noqa: E402


def arrays(e, data):
    t = e.count(data)
    try:
        c, o, r = t.arrays()
        assert int(c.sum()) == t.tokens
        return c, o, r, e.stats()
    finally:
        t.close()


def main():
    lib_a = sys.argv[1]
    lib_b = sys.argv[2] if len(sys.argv) > 2 else None
    cases = [
        ("hicard 96 MiB", corpus.fill(corpus.HICARD, 0x5EED0004, 0, 96 << 20)),
        ("hicard 256 MiB", corpus.fill(corpus.HICARD, 11, 0, 256 << 20)),
        ("mixed", np.concatenate([corpus.fill(corpus.ZIPF, 77, 0, 40 << 20), np.frombuffer(b" \n", np.uint8),
                                  corpus.fill(corpus.HICARD, 78, 0, 88 << 20)])),
        ("zipf 64 MiB", corpus.fill(corpus.ZIPF, 3, 0, 64 << 20)),
    ]
    bad = 0
    for flags in (0, mox.MOX_F_NO_DICT):
        ea, eb = mox.Engine(flags=flags, lib_path=lib_a), mox.Engine(flags=flags, lib_path=lib_b)
        try:
            for name, data in cases:
                a, b = arrays(ea, data.tobytes()), arrays(eb, data.tobytes())
                same = np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2]
                bad += not same
                print("%-16s flags=%d words=%d units=%d  %s" % (name, flags, a[0].size, a[3].get("reduce_units", -1),
                                                              "identical" if same else "DIFFERENT"), flush=True)
        finally:
            ea.close()
            eb.close()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
