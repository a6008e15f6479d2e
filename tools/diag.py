"""Diagnostics: compare GPU vs oracle on KATs and corpora, print differences."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "map-oxidize_amd"), os.path.join(ROOT, "oracle")]
import mox
from mox import corpus
import coracle

def g(e, data):
    try:
        t = e.count(data)
    except mox.Utf8Error:
        return "error"
    r = t.sorted_items(); t.close(); return r

def o(data):
    try:
        return coracle.count(data)[0]
    except coracle.InvalidUtf8:
        return "error"

def diff(a, b, lim=20):
    if a == "error" or b == "error":
        return "gpu=%s oracle=%s" % (a if a == "error" else "ok", b if b == "error" else "ok")
    da, db = dict(a), dict(b)
    out = []
    for k in sorted(set(da) | set(db)):
        if da.get(k) != db.get(k):
            out.append((k, da.get(k), db.get(k)))
    return out[:lim], len(out)

for flags in (0, mox.MOX_F_NO_DICT):
    e = mox.Engine(flags=flags)
    print("=== flags", flags)
    cases = json.load(open(os.path.join(ROOT, "tests/golden/kat.json")))["cases"]
    nbad = 0
    for c in cases:
        data = bytes.fromhex(c["input_hex"])
        a, b = g(e, data), o(data)
        if a != b:
            nbad += 1
            if nbad <= 8:
                print("KAT", c["name"], repr(data[:80]), diff(a, b))
    print("KAT failures:", nbad, "of", len(cases))
    for kind in ("zipf", "unicode"):
        for size in (4096, 100000, 2 << 20):
            data = corpus.fill(corpus.KINDS[kind], 1, 0, size).tobytes()
            a, b = g(e, data), o(data)
            if a != b:
                print(kind, size, diff(a, b, 10))
            else:
                print(kind, size, "ok")
    print(e.stats())
    e.close()
