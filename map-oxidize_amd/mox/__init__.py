"""Python binding of the MI355X word-count engine (ctypes over include/mox.h).

Host-side mirror of the reference's hot path (/root/reference/src/main.rs):

* ``count_words(data)`` / ``Engine.count`` -- ``split_file`` + ``map_phase`` +
  ``reduce_phase`` (main.rs:16-22): bytes -> {word: count}.  Invalid UTF-8 raises
  ``Utf8Error`` (the reference's ``io::ErrorKind::InvalidData`` abort, main.rs:44).
* ``Engine.count_file(path)`` -- the same from a file (main.rs:10, :36-51).
* ``write_final_result`` / ``top_words`` -- the reference's output layer
  (main.rs:170-192).

The compute runs in libmox.so (HIP kernels for gfx950).  There is no CPU
fallback: if the library is missing or no GPU is present, calls raise.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmox.so")

MOX_OK = 0
MOX_EINVAL = -1
MOX_EUTF8 = -2
MOX_ENOMEM = -3
MOX_EHIP = -4
MOX_EIO = -5
MOX_ERCCL = -6
MOX_ESTATE = -7
MOX_EHALO = -8

MOX_F_NO_DICT = 0x1
MOX_F_SORT_BYTES = 0x2  # fetch returns the words bytewise ascending (Rust String Ord)
MOX_F_TIMING = 0x4
MOX_F_TIMING_MAP = 0x8  # HIP events around the map kernel only

UNIQUE_ID_BYTES = 128


class MoxError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("mox error %d: %s" % (code, msg))
        self.code = code


class Utf8Error(MoxError):
    """Input is not valid UTF-8 (reference: tokio lines() -> InvalidData)."""


MAX_GPUS = 16
XPORT_RCCL = 0  # engine group: RCCL communicators over xGMI
XPORT_COPY = 1  # engine group: device-to-device copies (members may share a GPU)


class Config(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int),
        ("flags", ctypes.c_uint32),
        ("dict_words", ctypes.c_uint32),
        ("sample_pieces", ctypes.c_uint32),
        ("reserve_bytes", ctypes.c_uint64),
        ("n_gpus", ctypes.c_uint32),
        ("transport", ctypes.c_uint32),
        ("n_devices", ctypes.c_uint32),
        ("devices", ctypes.c_int32 * MAX_GPUS),
        ("reserved", ctypes.c_uint32 * 5),
    ]


class Shard(ctypes.Structure):
    _fields_ = [
        ("d_buf", ctypes.c_void_p),
        ("buf_len", ctypes.c_size_t),
        ("own_begin", ctypes.c_size_t),
        ("own_end", ctypes.c_size_t),
        ("at_corpus_end", ctypes.c_int),
    ]


class _Table(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("tokens", ctypes.c_uint64),
        ("counts", ctypes.POINTER(ctypes.c_uint64)),
        ("offs", ctypes.POINTER(ctypes.c_uint64)),
        ("bytes", ctypes.POINTER(ctypes.c_uint8)),
    ]


class Stats(ctypes.Structure):
    _fields_ = [
        ("bytes", ctypes.c_uint64),
        ("tokens", ctypes.c_uint64),
        ("uniques", ctypes.c_uint64),
        ("dict_words", ctypes.c_uint64),
        ("cold_records", ctypes.c_uint64),
        ("weighted_records", ctypes.c_uint64),
        ("unicode_tokens", ctypes.c_uint64),
        ("long_tokens", ctypes.c_uint64),
        ("chunks", ctypes.c_uint64),
        ("retries", ctypes.c_uint32),
        ("max_subpasses", ctypes.c_uint32),
        ("ms_run", ctypes.c_double),
        ("ms_dict", ctypes.c_double),
        ("ms_map", ctypes.c_double),
        ("ms_lanes", ctypes.c_double),
        ("ms_reduce", ctypes.c_double),
        ("ms_finalize", ctypes.c_double),
        ("ms_h2d", ctypes.c_double),
        ("ms_d2h", ctypes.c_double),
        ("ms_exchange", ctypes.c_double),
        ("reduce_units", ctypes.c_uint64),
        ("split_partitions", ctypes.c_uint32),
        ("async_reruns", ctypes.c_uint32),
        ("x_bytes_sent", ctypes.c_uint64),
        ("x_bytes_recv", ctypes.c_uint64),
        ("gather_bytes", ctypes.c_uint64),
        ("ms_gather", ctypes.c_double),
        ("path_hits", ctypes.c_uint64 * 8),
        ("ms_sort", ctypes.c_double),
        ("ms_local", ctypes.c_double),
        ("n_gpus", ctypes.c_uint32),
        ("async_dropped", ctypes.c_uint32),
        ("x_ranged", ctypes.c_uint32),
        ("x_pad", ctypes.c_uint32),
    ]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["path_hits"] = [int(x) for x in self.path_hits]
        return d


# int (*)(void* user, const void* send, const uint64_t* send_bytes, void* recv, const uint64_t* recv_bytes)
_A2A_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                           ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64))

# exactness-fallback counters (mox_stats.path_hits; collision check build only)
PATH_DICT_SAMEHASH, PATH_LONG_EQHASH, PATH_SORT_RESORT, PATH_SORT_TO_RED, PATH_RED_TAG, PATH_SMALL_TAG = range(6)
HC_LIB_PATH = os.path.join(_HERE, "libmox_hc.so")  # forced-collision check build (Makefile `hc`)
CHECK_LIB_PATH = os.path.join(_HERE, "libmox_check.so")  # bounds-check build (Makefile `check`)

_libs = {}


def lib(path=None):
    """Load libmox.so, or the library at ``path`` (a check build), once per path.
    Fails loudly: there is no fallback path."""
    if path is None:
        path = os.environ.get("MOX_LIB", LIB_PATH)  # diagnostics builds only (tools/)
    _lib = _libs.get(path)
    if _lib is None:
        if not os.path.exists(path):
            raise MoxError(MOX_ESTATE, "%s not built (run `make` or __graft_entry__.build())" % path)
        L = ctypes.CDLL(path)
        P, U64, I, VP = ctypes.POINTER, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p
        sz = ctypes.c_size_t
        sig = {
            "mox_last_error": ([], ctypes.c_char_p),
            "mox_abi_version": ([], I),
            "mox_engine_create": ([P(Config), P(VP)], I),
            "mox_engine_destroy": ([VP], None),
            "mox_set_flags": ([VP, ctypes.c_uint32], I),
            "mox_count": ([VP, VP, sz, P(P(_Table))], I),
            "mox_count_file": ([VP, ctypes.c_char_p, P(P(_Table))], I),
            "mox_table_free": ([P(_Table)], None),
            "mox_table_sort_bytes": ([P(_Table)], I),
            "mox_run_device": ([VP, VP, sz], I),
            "mox_run_range": ([VP, VP, sz, sz, sz, I], I),
            "mox_run_range_async": ([VP, VP, sz, sz, sz, I], I),
            "mox_run_wait": ([VP], I),
            "mox_fetch_table": ([VP, P(P(_Table))], I),
            "mox_sort_result": ([VP], I),
            "mox_get_stats": ([VP, P(Stats)], I),
            "mox_device_alloc": ([VP, sz, P(VP)], I),
            "mox_device_free": ([VP, VP], I),
            "mox_memcpy_h2d": ([VP, VP, VP, sz], I),
            "mox_memcpy_d2h": ([VP, VP, VP, sz], I),
            "mox_synchronize": ([VP], I),
            "mox_comm_unique_id": ([ctypes.c_char_p], I),
            "mox_comm_init": ([VP, I, I, ctypes.c_char_p], I),
            "mox_exchange": ([VP], I),
            "mox_exchange_host": ([VP, I, I, _A2A_FN, VP], I),
            "mox_gather": ([VP, I], I),
            "mox_gather_host": ([VP, I, I, I, _A2A_FN, VP], I),
            "mox_write_final_result": ([P(_Table), ctypes.c_char_p], I),
            "mox_print_top_words": ([P(_Table), sz], I),
            "mox_reduce_pairs": ([VP, VP, VP, VP, U64], I),
            "mox_run_shards": ([VP, P(Shard)], I),
            "mox_group_size": ([VP], I),
            "mox_group_member": ([VP, I], VP),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = _libs[path] = L
    return _lib


def _check(rc, L=None):
    if rc != MOX_OK:
        msg = (L or lib()).mox_last_error().decode("utf-8", "replace")
        if rc == MOX_EUTF8:
            raise Utf8Error(rc, msg)
        raise MoxError(rc, msg)


class Table:
    """Owning wrapper of a mox_table (words are bytes, counts are ints)."""

    def __init__(self, ptr, L=None):
        self._L = L or lib()
        self._p = ptr
        t = ptr.contents
        self.n = int(t.n)
        self.tokens = int(t.tokens)

    def _c(self, rc):
        _check(rc, self._L)

    def _raw(self):
        import numpy as np

        t = self._p.contents
        n = self.n
        counts = np.ctypeslib.as_array(t.counts, shape=(n,)).copy() if n else np.zeros(0, np.uint64)
        offs = np.ctypeslib.as_array(t.offs, shape=(n + 1,)).copy()
        nb = int(offs[-1]) if n else 0
        # (ctypes.string_at takes a C int size: tables above 2 GiB of bytes need numpy)
        data = np.ctypeslib.as_array(t.bytes, shape=(nb,)).tobytes() if nb else b""
        return counts, offs, data

    def arrays(self):
        """(counts uint64[n], offs uint64[n+1], bytes) in table order."""
        return self._raw()

    def items(self):
        counts, offs, data = self._raw()
        for i in range(self.n):
            yield data[offs[i]:offs[i + 1]], int(counts[i])

    def as_dict(self):
        return dict(self.items())

    def sorted_items(self):
        """Deterministic key sort (bytewise, Rust String Ord) used for parity."""
        return sorted(self.items(), key=lambda kv: kv[0])

    def sort_bytes(self):
        """Reorder this table bytewise ascending in place (mox_table_sort_bytes)."""
        self._c(self._L.mox_table_sort_bytes(self._p))
        return self

    def write_final_result(self, path):
        self._c(self._L.mox_write_final_result(self._p, path.encode()))

    def close(self):
        if self._p is not None:
            self._L.mox_table_free(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Engine:
    def __init__(self, device=-1, flags=0, dict_words=0, sample_pieces=0, reserve_bytes=0, lib_path=None,
                 n_gpus=0, transport=XPORT_RCCL, devices=None, _handle=None):
        """lib_path: a check build instead of libmox.so (CHECK_LIB_PATH, HC_LIB_PATH).
        n_gpus > 1: an engine group (include/mox.h) on ``devices`` (default 0..n_gpus-1)
        over ``transport``."""
        self._L = lib(lib_path)
        self._borrowed = _handle is not None
        if _handle is not None:  # a group member's engine: owned by the group
            self._h = ctypes.c_void_p(_handle)
            return
        cfg = Config()
        cfg.device = device
        cfg.flags = flags
        cfg.dict_words = dict_words
        cfg.sample_pieces = sample_pieces
        cfg.reserve_bytes = reserve_bytes
        cfg.n_gpus = n_gpus
        cfg.transport = transport
        if devices is not None:
            cfg.n_devices = len(devices)
            for i, d in enumerate(devices):
                cfg.devices[i] = d
        h = ctypes.c_void_p()
        self._c(self._L.mox_engine_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h

    # -- engine group (mox_config.n_gpus > 1)
    def group_size(self):
        return int(self._L.mox_group_size(self._h))

    def member(self, i):
        """Member i's engine (device allocations / copies for its shard)."""
        h = self._L.mox_group_member(self._h, i)
        if not h:
            raise MoxError(MOX_EINVAL, "no group member %d" % i)
        return Engine(lib_path=self._L._name, _handle=h)

    def run_shards(self, shards):
        """One group call over device-resident shards: [(d_ptr, buf_len, own_begin, own_end, at_end)]
        per member (mox_run_shards)."""
        arr = (Shard * len(shards))()
        for i, (d, n, a, b, end) in enumerate(shards):
            arr[i] = Shard(ctypes.c_void_p(d), n, a, b, 1 if end else 0)
        self._c(self._L.mox_run_shards(self._h, arr))

    def _c(self, rc):
        _check(rc, self._L)

    def set_flags(self, flags):
        self._c(self._L.mox_set_flags(self._h, flags))

    # -- drop-in for main.rs:16-22
    def count(self, data):
        buf = bytes(data)
        t = ctypes.POINTER(_Table)()
        self._c(self._L.mox_count(self._h, buf, len(buf), ctypes.byref(t)))
        return Table(t, self._L)

    def count_file(self, path):
        t = ctypes.POINTER(_Table)()
        self._c(self._L.mox_count_file(self._h, os.fsencode(path), ctypes.byref(t)))
        return Table(t, self._L)

    # -- device-resident path
    def run_device(self, d_ptr, n):
        self._c(self._L.mox_run_device(self._h, ctypes.c_void_p(d_ptr), n))

    def run_range(self, d_ptr, buf_len, own_begin, own_end, at_end):
        self._c(self._L.mox_run_range(self._h, ctypes.c_void_p(d_ptr), buf_len, own_begin, own_end, 1 if at_end else 0))

    def run_range_async(self, d_ptr, buf_len, own_begin, own_end, at_end):
        """Enqueue a pass; completes the previously enqueued one (include/mox.h)."""
        self._c(self._L.mox_run_range_async(self._h, ctypes.c_void_p(d_ptr), buf_len, own_begin, own_end, 1 if at_end else 0))

    def run_wait(self):
        self._c(self._L.mox_run_wait(self._h))

    def fetch(self):
        t = ctypes.POINTER(_Table)()
        self._c(self._L.mox_fetch_table(self._h, ctypes.byref(t)))
        return Table(t, self._L)

    def sort_result(self):
        """Sort the device-resident result bytewise on the GPU (mox_sort_result)."""
        self._c(self._L.mox_sort_result(self._h))

    def stats(self):
        s = Stats()
        self._c(self._L.mox_get_stats(self._h, ctypes.byref(s)))
        return s.as_dict()

    def ms_map(self):
        """Map-kernel milliseconds of the last pass (cheap: for timed loops)."""
        if not hasattr(self, "_st"):
            self._st = Stats()
            self._st_ref = ctypes.byref(self._st)
        self._c(self._L.mox_get_stats(self._h, self._st_ref))
        return self._st.ms_map

    def alloc(self, nbytes):
        p = ctypes.c_void_p()
        self._c(self._L.mox_device_alloc(self._h, nbytes, ctypes.byref(p)))
        return p.value

    def free(self, d_ptr):
        self._c(self._L.mox_device_free(self._h, ctypes.c_void_p(d_ptr)))

    def h2d(self, d_ptr, host_buf, nbytes=None):
        if nbytes is None:
            nbytes = len(host_buf)
        src = ctypes.c_char_p(host_buf) if isinstance(host_buf, bytes) else host_buf
        if hasattr(host_buf, "ctypes"):
            src = ctypes.c_void_p(host_buf.ctypes.data)
        self._c(self._L.mox_memcpy_h2d(self._h, ctypes.c_void_p(d_ptr), src, nbytes))

    def synchronize(self):
        self._c(self._L.mox_synchronize(self._h))

    # -- multi-GPU
    def comm_init(self, nranks, rank, uid):
        self._c(self._L.mox_comm_init(self._h, nranks, rank, uid))

    def exchange(self):
        """RCCL all-to-all exchange + final reduce (after run_range on every rank)."""
        self._c(self._L.mox_exchange(self._h))

    def exchange_host(self, nranks, rank, alltoallv):
        """The same exchange over a host transport.  ``alltoallv(send, send_sizes,
        recv_sizes)`` gets the send bytes (memoryview, blocks for ranks 0..n-1)
        and must return the received bytes (blocks from ranks 0..n-1)."""
        self._host_call(lambda fn: self._L.mox_exchange_host(self._h, nranks, rank, fn, None), nranks, alltoallv)

    def gather(self, root=0):
        """Gather every rank's final table into root's engine over RCCL (mox_gather)."""
        self._c(self._L.mox_gather(self._h, root))

    def gather_host(self, nranks, rank, alltoallv, root=0):
        """mox_gather over a host transport (same callback as exchange_host)."""
        self._host_call(lambda fn: self._L.mox_gather_host(self._h, nranks, rank, root, fn, None), nranks, alltoallv)

    def _host_call(self, call, nranks, alltoallv):
        err = []

        def cb(_user, send, send_bytes, recv, recv_bytes):
            try:
                ss = [int(send_bytes[i]) for i in range(nranks)]
                rs = [int(recv_bytes[i]) for i in range(nranks)]
                buf = (ctypes.c_uint8 * sum(ss)).from_address(send) if sum(ss) else bytearray()
                out = alltoallv(memoryview(buf), ss, rs)
                out = bytes(out)
                if len(out) != sum(rs):
                    raise ValueError("alltoallv returned %d bytes, expected %d" % (len(out), sum(rs)))
                if out:
                    ctypes.memmove(recv, out, len(out))
                return 0
            except Exception as ex:  # reported after the call returns
                err.append(ex)
                return 1

        fn = _A2A_FN(cb)
        rc = call(fn)
        if err:
            raise err[0]
        _check(rc)

    # -- spill files (mox/spill.py): reduce_phase over parsed map files
    def reduce_pairs(self, words, counts):
        """Sum counts by word (bytes, taken verbatim) on the GPU; returns the
        Table (main.rs:111-150 over read_map_result's maps)."""
        from . import spill

        data, offs, cnt = spill.pack_pairs(list(words), list(counts))
        if len(cnt) != len(offs) - 1:
            raise ValueError("words and counts differ in length")
        buf = ctypes.create_string_buffer(data, max(1, len(data)))
        self._c(self._L.mox_reduce_pairs(self._h, buf, ctypes.c_void_p(offs.ctypes.data),
                                      ctypes.c_void_p(cnt.ctypes.data), len(cnt)))
        return self.fetch()

    def close(self):
        if getattr(self, "_h", None):
            if not getattr(self, "_borrowed", False):
                self._L.mox_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id():
    buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
    _check(lib().mox_comm_unique_id(buf))
    return buf.raw


def count_words(data, **kw):
    """One-shot: bytes -> {word(bytes): count} on the GPU."""
    e = Engine(**kw)
    try:
        t = e.count(data)
        try:
            return t.as_dict()
        finally:
            t.close()
    finally:
        e.close()
