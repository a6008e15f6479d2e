import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "map-oxidize_amd"), os.path.join(ROOT, "oracle")]
import mox, coracle
from mox import corpus
data = corpus.fill(corpus.UNICODE, 5, 0, 3 << 20).tobytes()
e = mox.Engine()
d = e.alloc(len(data) + 64)
e.h2d(d, data)
for rep in range(3):
  for a, b in [(123457, 2 * 1024 * 1024 + 5), (4, len(data) - 1000), (16, 2000000), (123457, len(data))]:
    e.run_range(d, len(data), a, b, True)
    t = e.fetch(); got = dict(t.items()); t.close()
    want = dict(coracle.count_range(data, a, b)[0])
    bad = sorted(set(got) | set(want), key=lambda w: -abs(got.get(w, 0) - want.get(w, 0)))
    bad = [w for w in bad if got.get(w, 0) != want.get(w, 0)]
    print("range", a, b, "ndiff", len(bad), flush=True)
    for w in bad[:6]:
        pos = [i for i in range(a, b) if data.startswith(w, i)][:5] if len(w) > 3 else []
        print("  ", w, got.get(w), want.get(w), [(p, (p - (a & ~15)) % 1024) for p in pos])
