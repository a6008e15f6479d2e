"""Worker of tests/test_gpu_exchange.py::test_host_exchange_gloo_processes:
one rank of a gloo process group, engine on device 0, host-staged exchange
and gather (mox_gather_host); rank 0 writes the gathered table, bytewise
sorted by the engine (MOX_F_SORT_BYTES), as hex words to argv[1]."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "map-oxidize_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import torch.distributed as dist  # noqa: E402

import mox  # noqa: E402
from mox import dist as mdist  # noqa: E402
from test_gpu_exchange import mixed_corpus  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    data = mixed_corpus(4 << 20, 77)
    lo, hi, ob, oe, at_end = mdist.shard_range(len(data), world, rank)
    e = mox.Engine(device=0, flags=mox.MOX_F_SORT_BYTES)
    d = e.alloc(hi - lo)
    e.h2d(d, data[lo:hi])
    e.run_range(d, hi - lo, ob, oe, at_end)
    a2a = mdist.gloo_alltoallv()
    e.exchange_host(world, rank, a2a)
    e.gather_host(world, rank, a2a, root=0)
    if rank == 0:
        t = e.fetch()
        items = list(t.items())
        t.close()
        with open(sys.argv[1], "w") as f:
            json.dump([(w.hex(), c) for w, c in items], f)
    e.free(d)
    e.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
