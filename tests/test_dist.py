"""CPU: host logic of the multi-GPU path -- byte-range shards,
the gloo all-to-all used by the host-staged exchange transport, and the final
gather/merge -- with world_size 2 over gloo.  The device side of the exchange
is covered by tests/test_gpu_exchange.py."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from mox import dist as mdist


def test_shard_ranges_partition_the_corpus():
    for total in (0, 1, 17, 1000, 1 << 20, (1 << 20) + 3):
        for world in (1, 2, 3, 8):
            owned = []
            if total < 4:
                continue
            for r in range(world):
                lo, hi, ob, oe, at_end = mdist.shard_range(total, world, r)
                assert 0 <= lo <= hi <= total
                assert 0 <= ob <= oe <= hi - lo
                assert ob == 0 or ob >= 4, "own_begin needs 4 bytes of left context"
                assert at_end == (hi == total)
                owned.append((lo + ob, lo + oe))
            assert owned[0][0] == 0 and owned[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(owned, owned[1:]))


def test_weak_scaling_shards():
    per = 1 << 20
    for r in range(4):
        lo, hi, ob, oe, _ = mdist.shard_range(4 * per, 4, r, per_rank=per)
        assert (lo + ob, lo + oe) == (r * per, (r + 1) * per)


def test_merge_tables_rejects_shared_words():
    assert mdist.merge_tables([[(b"a", 1), (b"c", 2)], [(b"b", 5)]]) == [(b"a", 1), (b"b", 5), (b"c", 2)]
    with pytest.raises(ValueError):
        mdist.merge_tables([[(b"a", 1)], [(b"a", 2)]])


def test_thread_alltoall():
    import threading

    world = 3
    x = mdist.ThreadAlltoall(world)
    out = [None] * world

    def run(r):
        send = b"".join(bytes([r * 16 + d]) * (r + d + 1) for d in range(world))
        out[r] = x.fn(r)(memoryview(send), [r + d + 1 for d in range(world)], [s + r + 1 for s in range(world)])

    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    for r in range(world):
        assert out[r] == b"".join(bytes([s * 16 + r]) * (s + r + 1) for s in range(world))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a2a = mdist.gloo_alltoallv()
        ss = [rank + d + 1 for d in range(world)]
        send = b"".join(bytes([rank * 16 + d]) * ss[d] for d in range(world))
        rs = [s + rank + 1 for s in range(world)]
        got = a2a(memoryview(send), ss, rs)
        want = b"".join(bytes([s * 16 + rank]) * rs[s] for s in range(world))
        # the gather's transport shape: every rank sends one block to rank 0 only
        blk = b"r%d" % rank * (rank + 3)
        gs = [len(blk) if d == 0 else 0 for d in range(world)]
        sizes = [len(b"r%d" % s * (s + 3)) if rank == 0 else 0 for s in range(world)]
        gathered = a2a(memoryview(blk), gs, sizes)
        q.put((rank, got == want, gathered))
    finally:
        dist.destroy_process_group()


def test_gloo_alltoallv_and_gather_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in ps]
    res = dict((r, (ok, m)) for r, ok, m in (q.get(timeout=120) for _ in range(world)))
    [p.join(60) for p in ps]
    assert all(ok for ok, _ in res.values())
    assert res[0][1] == b"".join(b"r%d" % s * (s + 3) for s in range(world)) and res[1][1] == b""
