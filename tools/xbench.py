"""Exchange-pass cost on one GPU: RCCL transport at world size 1 (self send/recv),
so everything but the inter-GPU transfer (count, pack, reduce-only pass, syncs)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "map-oxidize_amd"))
import mox
from mox import corpus

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
e = mox.Engine(device=0, flags=mox.MOX_F_TIMING, reserve_bytes=n)
e.comm_init(1, 0, mox.comm_unique_id())
d = e.alloc(n)
e.h2d(d, corpus.fill(corpus.ZIPF, 0x5EED0002, 0, n))
for it in range(6):
    e.synchronize()
    t0 = time.perf_counter()
    e.run_range(d, n, 0, n, True)
    e.synchronize()
    t1 = time.perf_counter()
    e.exchange()
    e.synchronize()
    t2 = time.perf_counter()
    s = e.stats()
    print("run %.3f ms  exchange %.3f ms (stat %.3f ms, pass run %.3f ms reduce %.3f finalize %.3f)" % (
        (t1 - t0) * 1e3, (t2 - t1) * 1e3, s["ms_exchange"], s["ms_run"], s["ms_reduce"], s["ms_finalize"]), flush=True)
e.free(d)
e.close()
