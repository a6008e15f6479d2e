"""Worker of tests/test_gpu_exchange.py: one rank of a gloo process group.
Default: engine on device 0, host-staged exchange and gather
(mox_gather_host).  With argv[2] == "rccl": engine on device LOCAL_RANK, the
RCCL exchange and gather (mox_comm_init, mox_exchange, mox_gather) -- one
process per GPU, needs as many GPUs as ranks.  Rank 0 writes the gathered
table, bytewise sorted by the engine (MOX_F_SORT_BYTES), as hex words to
argv[1]."""
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
    rccl = len(sys.argv) > 2 and sys.argv[2] == "rccl"
    e = mox.Engine(device=int(os.environ.get("LOCAL_RANK", "0")) if rccl else 0, flags=mox.MOX_F_SORT_BYTES)
    d = e.alloc(hi - lo)
    e.h2d(d, data[lo:hi])
    e.run_range(d, hi - lo, ob, oe, at_end)
    if rccl:
        obj = [mox.comm_unique_id() if rank == 0 else b""]
        dist.broadcast_object_list(obj, src=0)
        e.comm_init(world, rank, obj[0])
        e.exchange()
        e.gather(0)
    else:
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
