"""Retries of the 96 MiB mixed corpus (24 MiB Zipf + 72 MiB C4-like) with a
given library (MOX_LIB): each run prints the attempts' retry count and the
split statistics, checks the table against the oracle once.
Usage: MOX_LIB=... python tools/split_retry_probe.py RUNS"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "map-oxidize_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import coracle  # noqa: E402
import mox  # noqa: E402
from mox import corpus  # noqa: E402
from conftest import assert_tables_equal  # noqa: E402

z = corpus.fill(corpus.ZIPF, 77, 0, 24 << 20)
h = corpus.fill(corpus.HICARD, 78, 0, 72 << 20)
data = np.concatenate([z, np.frombuffer(b" \n", np.uint8), h])
want = coracle.count_arrays(data, nthreads=16)[:3]
for k in range(int(sys.argv[1])):
    e = mox.Engine(device=0)
    t = e.count(data.tobytes())
    got = t.arrays()
    t.close()
    st = e.stats()
    e.close()
    print("run", k, "retries", st["retries"], "split_partitions", st["split_partitions"], "reduce_units", st["reduce_units"],
          "cold", st["cold_records"], "dict_words", st["dict_words"], flush=True)
    if k == 0:
        assert_tables_equal(got, want)
print("probe ok")
