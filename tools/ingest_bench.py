"""PCIe-inclusive ingest: mox_count_file on a 1 GiB C2 file in
tmpfs (page cache: the read is a memcpy) and mox_count on a pageable host buffer,
each end to end (read + H2D + pass + table fetch)."""
import os, sys, tempfile, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "map-oxidize_amd"))
import mox
from mox import corpus

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
data = corpus.fill(corpus.ZIPF, 0x5EED0002, 0, n)
d = "/dev/shm" if os.path.isdir("/dev/shm") else None
with tempfile.TemporaryDirectory(dir=d) as td:
    path = os.path.join(td, "shakes.txt")
    data.tofile(path)
    e = mox.Engine(device=0, flags=mox.MOX_F_TIMING, reserve_bytes=n)
    host = data.tobytes()
    for it in range(4):
        t0 = time.perf_counter(); t = e.count_file(path); t1 = time.perf_counter()
        s = e.stats(); t.close()
        t2 = time.perf_counter(); t = e.count(host); t3 = time.perf_counter()
        s2 = e.stats(); t.close()
        print("count_file: %.1f ms total (read+H2D %.1f ms = %.1f GB/s, pass %.2f ms, fetch %.1f ms) -> %.1f GB/s end to end | "
              "count(host buf): %.1f ms total (H2D %.1f ms = %.1f GB/s)" % (
                  (t1 - t0) * 1e3, s["ms_h2d"], n / s["ms_h2d"] / 1e6, s["ms_run"], s["ms_d2h"], n / (t1 - t0) / 1e9,
                  (t3 - t2) * 1e3, s2["ms_h2d"], n / s2["ms_h2d"] / 1e6), flush=True)
    e.close()
