"""Host side of the multi-GPU path: byte-range sharding with
word-boundary halos, a gloo all-to-all for the host-staged exchange and
gather transport (mox_exchange_host / mox_gather_host), and a checker-side
merge of per-rank tables.  The gather itself is device side (mox_gather).

The reference runs one process (main.rs:16-22); sharding is this engine's
addition.  Every token belongs to the rank whose byte range holds its first
byte; a rank's buffer carries 64 bytes of left context and HALO bytes of
look-ahead so it can finish its last token (the engine reports MOX_EHALO if a
token runs past the look-ahead).
"""
import heapq

LEFT_CONTEXT = 64
HALO = 1 << 16


def shard_range(total, world, rank, per_rank=None, halo=HALO):
    """(lo, hi, own_begin, own_end, at_end) of rank's shard of a corpus of
    ``total`` bytes: buffer = corpus[lo:hi], owned bytes = [own_begin, own_end)
    relative to lo.  ``per_rank`` fixes the shard size (weak scaling); default
    splits ``total`` evenly."""
    if per_rank is None:
        # >= 4 so that every non-first owned range has the engine's minimum
        # left context (mox_run_range: own_begin is 0 or >= 4)
        per_rank = max(4, (total + world - 1) // world)
    ob = min(total, rank * per_rank)
    oe = min(total, ob + per_rank) if rank < world - 1 else total
    if ob == oe:  # nothing owned: an empty buffer at the corpus end
        return total, total, 0, 0, True
    lo = max(0, ob - LEFT_CONTEXT)
    hi = min(total, oe + halo)
    return lo, hi, ob - lo, oe - lo, hi == total


def gloo_alltoallv(group=None):
    """An ``alltoallv(send, send_sizes, recv_sizes)`` for Engine.exchange_host over
    torch.distributed (CPU tensors; gloo)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    def a2a(send, send_sizes, recv_sizes):
        inp = torch.from_numpy(np.frombuffer(send, dtype=np.uint8).copy()) if sum(send_sizes) else torch.empty(0, dtype=torch.uint8)
        out = torch.empty(sum(recv_sizes), dtype=torch.uint8)
        dist.all_to_all_single(out, inp, list(recv_sizes), list(send_sizes), group=group)
        return out.numpy().tobytes()

    return a2a


def merge_tables(parts):
    """k-way merge of per-rank (word, count) lists, each sorted bytewise, into one
    bytewise-sorted list.  Ranks own disjoint words after the exchange; a word
    seen on two ranks is an error (it would mean a wrong owner mapping)."""
    out = []
    for w, c in heapq.merge(*parts, key=lambda kv: kv[0]):
        if out and out[-1][0] == w:
            raise ValueError("word %r owned by two ranks" % (w,))
        out.append((w, c))
    return out


class ThreadAlltoall:
    """In-process all-to-all between ``world`` threads (one engine per thread),
    for exercising the exchange with several ranks on one GPU without a process
    group.  ``fn(rank)`` is the alltoallv callback of that rank's thread."""

    def __init__(self, world):
        import threading

        self.world = world
        self.barrier = threading.Barrier(world)
        self.slots = [None] * world

    def fn(self, rank):
        def a2a(send, send_sizes, recv_sizes):
            data = bytes(send)
            offs = [0]
            for s in send_sizes:
                offs.append(offs[-1] + s)
            self.slots[rank] = [data[offs[d]:offs[d + 1]] for d in range(self.world)]
            self.barrier.wait()
            out = b"".join(self.slots[s][rank] for s in range(self.world))
            self.barrier.wait()  # every rank has read before the slots are reused
            if len(out) != sum(recv_sizes):
                raise ValueError("size mismatch in ThreadAlltoall")
            return out

        return a2a
