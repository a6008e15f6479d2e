"""Worker of tests/test_gpu_exchange.py::test_host_exchange_gloo_processes:
one rank of a gloo process group, engine on device 0, host-staged exchange;
rank 0 writes the merged table (hex words) to argv[1]."""
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
    e = mox.Engine(device=0)
    d = e.alloc(hi - lo)
    e.h2d(d, data[lo:hi])
    e.run_range(d, hi - lo, ob, oe, at_end)
    e.exchange_host(world, rank, mdist.gloo_alltoallv())
    t = e.fetch()
    items = t.sorted_items()
    t.close()
    e.free(d)
    e.close()
    merged = mdist.gather_items(items)
    if rank == 0:
        with open(sys.argv[1], "w") as f:
            json.dump([(w.hex(), c) for w, c in merged], f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
