"""CPU: the exchange's send / receive plan (map-oxidize_amd/csrc/mox_multi.hip x_layout,
count_transpose) through the C-ABI test hook mox_debug_exchange_layout.

Both sides of every (sender, receiver) pair must post the same transfer: rank i's
send lengths to rank p are rank p's receive lengths from rank i (the length
matrices are transposes), so a zero-length peer is skipped on both sides
(RcclTransport / group_payloads: `if (len) ncclSend/ncclRecv`), and each rank packs
its blocks back to back in peer order.  Replaces nothing in the reference (its
reduce_phase, main.rs:111-150, merges in one process); this is the multi-GPU
exchange of SURVEY.md §8(e) step 4."""
import ctypes

import numpy as np
import pytest

import mox

WREC, XHDR = 24, 32  # sizeof(WRec), sizeof(XHdr) (mox_internal.h)


def layout(counts):
    P = counts.shape[0]
    L = mox.lib()
    fn = L.mox_debug_exchange_layout
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    c = np.ascontiguousarray(counts, dtype=np.uint64)
    out = np.zeros((P, 8, P), dtype=np.uint64)
    assert fn(P, c.ctypes.data, out.ctypes.data) == 0, mox.lib().mox_last_error()
    return out


def random_counts(rng, P, zero_frac):
    c = rng.integers(0, 5000, size=(P, P, 3), dtype=np.uint64)
    c[..., 1] = rng.integers(0, 50, size=(P, P))
    c[..., 2] = c[..., 1] * rng.integers(17, 40, size=(P, P))  # long words padded to >= 17 bytes
    z = rng.random((P, P)) < zero_frac
    c[z] = 0
    zl = rng.random((P, P)) < zero_frac
    c[zl, 1] = 0
    c[zl, 2] = 0
    return c


@pytest.mark.parametrize("P", [1, 2, 3, 5, 8, 16, 64])
@pytest.mark.parametrize("zero_frac", [0.0, 0.3, 0.9])
def test_send_recv_lengths_are_transposes(P, zero_frac):
    rng = np.random.default_rng(1000 * P + int(10 * zero_frac))
    for _ in range(5):
        c = random_counts(rng, P, zero_frac)
        out = layout(c)
        s_short_off, s_short_len, s_blob_off, s_blob_len = out[:, 0], out[:, 1], out[:, 2], out[:, 3]
        r_short_off, r_short_len, r_blob_off, r_blob_len = out[:, 4], out[:, 5], out[:, 6], out[:, 7]
        # lengths from the counts: WRec records, XHdr headers + padded bytes
        assert np.array_equal(s_short_len, c[..., 0] * WREC)
        assert np.array_equal(s_blob_len, c[..., 1] * XHDR + c[..., 2])
        # what i sends to p is what p receives from i: transposes
        assert np.array_equal(s_short_len, r_short_len.T)
        assert np.array_equal(s_blob_len, r_blob_len.T)
        # so a skipped (zero-length) transfer is skipped on both sides
        assert np.array_equal(s_short_len != 0, r_short_len.T != 0)
        assert np.array_equal(s_blob_len != 0, r_blob_len.T != 0)
        # blocks back to back in peer order (exclusive prefix sums per rank)
        for off, ln in ((s_short_off, s_short_len), (s_blob_off, s_blob_len),
                        (r_short_off, r_short_len), (r_blob_off, r_blob_len)):
            ex = np.zeros_like(ln)
            ex[:, 1:] = np.cumsum(ln, axis=1)[:, :-1]
            assert np.array_equal(off, ex)
        # totals: everything sent is received somewhere
        assert s_short_len.sum() == r_short_len.sum() and s_blob_len.sum() == r_blob_len.sum()


def test_layout_rejects_bad_rank_counts():
    L = mox.lib()
    fn = L.mox_debug_exchange_layout
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    buf = np.zeros(65 * 65 * 8 * 3, dtype=np.uint64)
    assert fn(0, buf.ctypes.data, buf.ctypes.data) != 0
    assert fn(65, buf.ctypes.data, buf.ctypes.data) != 0
