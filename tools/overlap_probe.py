"""Would overlapping passes help?  Throughput of back-to-back async C2 passes
from one engine vs two engines (threads, separate buffers, one GPU) running at
the same time: if two concurrent pass streams beat one, a pass's map can use
resources its predecessor's reduce tail leaves idle.  Prints GB/s for both."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "map-oxidize_amd"))
import mox  # noqa: E402
from mox import corpus  # noqa: E402

N = 1 << 30
STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 20
WARM = int(sys.argv[2]) if len(sys.argv) > 2 else 20  # past the GPU clock transient (bench.py --warmup)


def make():
    e = mox.Engine(device=0, reserve_bytes=N)
    d = e.alloc(N)
    e.h2d(d, corpus.fill(corpus.ZIPF, 0x5EED0002, 0, N))
    for _ in range(WARM):
        e.run_range_async(d, N, 0, N, True)
    e.synchronize()
    return e, d


def run(e, d, steps):
    for _ in range(steps):
        e.run_range_async(d, N, 0, N, True)
    e.synchronize()


engs = [make(), make()]
for rep in range(2):  # one, two, one, two (interleaved)
    run(*engs[0], WARM)
    t = time.perf_counter()
    run(*engs[0], STEPS)
    one = N * STEPS / (time.perf_counter() - t) / 1e9
    ts = [threading.Thread(target=run, args=(e, d, STEPS)) for e, d in engs]
    t = time.perf_counter()
    for x in ts:
        x.start()
    for x in ts:
        x.join()
    two = 2 * N * STEPS / (time.perf_counter() - t) / 1e9
    print("one engine %.1f GB/s, two concurrent engines %.1f GB/s total (%.3fx)" % (one, two, two / one), flush=True)
