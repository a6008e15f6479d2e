import sys, os, random
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "map-oxidize_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import mox, coracle
from test_gpu_exchange import mixed_corpus
data = mixed_corpus(6 << 20, 42)
e = mox.Engine()
d = e.alloc(len(data) + 64)
e.h2d(d, data)
rng = random.Random(1)
cases = [(0, len(data) // 2, len(data) // 2 + 65536), (len(data) // 2 - 64, len(data), len(data))]
for _ in range(40):
    lo = rng.randrange(0, len(data) - 4096); hi = rng.randrange(lo + 4096, len(data) + 1)
    cases.append((lo, hi, min(len(data), hi + 65536)))
bad = 0
for rep in range(2):
  for (ob, oe, bh) in cases:
    bl = max(0, ob - 64)
    buf_len = bh - bl
    at_end = bh == len(data)
    e.run_range(d + bl, buf_len, ob - bl, oe - bl, at_end)
    t = e.fetch(); got = dict(t.items()); tok = t.tokens; t.close()
    try:
        want, wtok = coracle.count_range(data[bl:bh], ob - bl, oe - bl)
    except coracle.InvalidUtf8:
        continue
    want = dict(want)
    if got != want or tok != wtok:
        bad += 1
        diff = [w for w in set(got) | set(want) if got.get(w, 0) != want.get(w, 0)]
        base0 = (d + ob) & ~15
        print("MISMATCH", rep, ob, oe, bh, "tok", tok, wtok, "ndiff", len(diff), flush=True)
        for w in diff[:4]:
            pos = []
            i = data.find(w, max(0, ob - 40))
            while i != -1 and i < oe + 40 and len(pos) < 6:
                pos.append((i, (i - ob) % 992 if True else 0, ((d + i) & 15)))
                i = data.find(w, i + 1)
            print("   ", w[:40], got.get(w), want.get(w), pos)
print("done bad", bad)
