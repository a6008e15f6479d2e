import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "map-oxidize_amd"), os.path.join(ROOT, "oracle")]
import mox
from mox import corpus
import coracle
os.environ["MOX_VERBOSE"] = "1"
data = corpus.fill(corpus.SKEW, 3, 0, 8 << 20).tobytes()
for flags in (mox.MOX_F_TIMING, mox.MOX_F_TIMING | mox.MOX_F_NO_DICT):
    e = mox.Engine(flags=flags)
    for rep in range(2):
        t0 = time.time(); t = e.count(data); dt = time.time() - t0
        print("flags", flags, "rep", rep, "%.3fs" % dt, e.stats(), flush=True)
        ok = t.sorted_items() == coracle.count(data)[0]; t.close()
        print("parity", ok, flush=True)
    e.close()
