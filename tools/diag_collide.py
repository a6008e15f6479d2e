"""Diagnostics for the forced-collision build (libmox_hc.so): prints where the
GPU table differs from the oracle (KATs, a long-word corpus) and the pass
attempts of a high-cardinality corpus (MOX_VERBOSE)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "map-oxidize_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import json  # noqa: E402

import coracle  # noqa: E402
import mox  # noqa: E402
from mox import corpus  # noqa: E402


def diff(tag, got, want):
    g, w = dict(got), dict(want)
    bad = [(k, g.get(k), w.get(k)) for k in sorted(set(g) | set(w)) if g.get(k) != w.get(k)]
    if bad:
        print(tag, "DIFF", len(bad), bad[:8], flush=True)
    return not bad


def main():
    libs = sys.argv[1:] or [mox.HC_LIB_PATH]
    for lp in libs:
        print("=====", lp, flush=True)
        run(lp, hicard=len(libs) == 1)
    os._exit(0)  # engines of several libraries: skip interpreter-exit destructors


def run(lib_path, hicard):
    e = mox.Engine(device=0, lib_path=lib_path)
    cases = json.load(open(os.path.join(ROOT, "tests", "golden", "kat.json")))["cases"]
    nbad = 0
    for c in cases:
        if "error" in c:
            continue
        data = bytes.fromhex(c["input_hex"])
        t = e.count(data)
        got = t.sorted_items()
        t.close()
        want = [(bytes.fromhex(w), n) for w, n in c["expected"]]
        if not diff("kat " + c["name"], got, want):
            nbad += 1
            print("   stats", {k: v for k, v in e.stats().items() if k in ("tokens", "uniques", "dict_words", "long_tokens", "path_hits")})
    print("kat mismatches", nbad, flush=True)
    from test_gpu_collide import long_word_corpus
    data = long_word_corpus(0xC015, 2000, 20000)
    t = e.count(data)
    got = t.sorted_items()
    t.close()
    diff("long", got, coracle.count(data)[0])
    print("long stats", {k: v for k, v in e.stats().items() if k in ("tokens", "uniques", "retries", "long_tokens", "path_hits")}, flush=True)
    if not hicard:
        return
    os.environ["MOX_VERBOSE"] = "1"
    e2 = mox.Engine(device=0, lib_path=lib_path)
    h = corpus.fill(corpus.HICARD, 0xC012, 0, 96 << 20).tobytes()
    try:
        t = e2.count(h)
        t.close()
        print("hicard ok", e2.stats(), flush=True)
    except mox.MoxError as ex:
        print("hicard error", ex, flush=True)


if __name__ == "__main__":
    main()
