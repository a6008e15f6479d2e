"""ORACLE -- test infrastructure only: ctypes binding of oracle/build/libmox_oracle.so
(the C restatement, oracle/mox_oracle.c).  PARITY UNPINNED (see mox_oracle.c)."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "libmox_oracle.so")
MEDUCE_REF = os.path.join(_HERE, "build", "meduce_ref")
EUTF8 = -2


class _T(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("tokens", ctypes.c_uint64),
                ("counts", ctypes.POINTER(ctypes.c_uint64)), ("offs", ctypes.POINTER(ctypes.c_uint64)),
                ("bytes", ctypes.POINTER(ctypes.c_uint8)), ("bytes_len", ctypes.c_uint64),
                ("invalid_at", ctypes.c_int64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(LIB)
        L.moxo_count.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(_T)]
        L.moxo_count.restype = ctypes.c_int
        L.moxo_free.argtypes = [ctypes.POINTER(_T)]
        L.moxo_count_range.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.POINTER(_T)]
        L.moxo_count_range.restype = ctypes.c_int
        L.moxo_utf8_invalid_at.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.moxo_utf8_invalid_at.restype = ctypes.c_int64
        VP, U64, P64 = ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)
        L.moxo_count_digest.argtypes = [VP, U64, ctypes.c_int, VP, P64]
        L.moxo_count_digest.restype = ctypes.c_int
        L.moxo_table_digest.argtypes = [U64, VP, VP, VP, ctypes.c_int, VP]
        L.moxo_table_digest.restype = None
        L.moxo_count_tokens.argtypes = [VP, U64, ctypes.c_int]
        L.moxo_count_tokens.restype = U64
        L.moxo_count_words.argtypes = [VP, U64, ctypes.c_int, VP, VP, U64, VP]
        L.moxo_count_words.restype = None
        L.moxo_lowercase.argtypes = [ctypes.c_char_p, U64, ctypes.c_char_p]
        L.moxo_lowercase.restype = U64
        L.moxo_is_whitespace.argtypes = [ctypes.c_uint32]
        L.moxo_is_whitespace.restype = ctypes.c_int
        _lib = L
    return _lib


def lowercase(word):
    """The oracle's str::to_lowercase of one token (UTF-8 bytes in and out)."""
    out = ctypes.create_string_buffer(2 * len(word) + 8)
    n = lib().moxo_lowercase(word, len(word), out)
    return out.raw[:n]


def is_whitespace(cp):
    return lib().moxo_is_whitespace(cp) != 0


class InvalidUtf8(ValueError):
    pass


def count(data, nthreads=8):
    """Returns (sorted [(word bytes, count)], total tokens); raises InvalidUtf8."""
    import numpy as np
    if isinstance(data, np.ndarray):
        ptr, n = data.ctypes.data, data.nbytes
        keep = data
    else:
        keep = bytes(data)
        ptr, n = ctypes.cast(ctypes.c_char_p(keep), ctypes.c_void_p).value, len(keep)
    t = _T()
    rc = lib().moxo_count(ptr, n, nthreads, ctypes.byref(t))
    del keep
    if rc == EUTF8:
        raise InvalidUtf8(t.invalid_at)
    try:
        nn = t.n
        if nn == 0:
            return [], int(t.tokens)
        counts = np.ctypeslib.as_array(t.counts, shape=(nn,)).copy()
        offs = np.ctypeslib.as_array(t.offs, shape=(nn + 1,)).copy()
        raw = ctypes.string_at(t.bytes, int(offs[-1]))
        return [(raw[offs[i]:offs[i + 1]], int(counts[i])) for i in range(nn)], int(t.tokens)
    finally:
        lib().moxo_free(ctypes.byref(t))


def count_arrays(data, nthreads=8):
    """Like count() but returns numpy arrays (counts, offs, bytes) -- for big inputs."""
    import numpy as np
    t = _T()
    rc = lib().moxo_count(data.ctypes.data, data.nbytes, nthreads, ctypes.byref(t))
    if rc == EUTF8:
        raise InvalidUtf8(t.invalid_at)
    try:
        nn = t.n
        counts = np.ctypeslib.as_array(t.counts, shape=(nn,)).copy() if nn else np.zeros(0, np.uint64)
        offs = np.ctypeslib.as_array(t.offs, shape=(nn + 1,)).copy()
        raw = np.ctypeslib.as_array(ctypes.cast(t.bytes, ctypes.POINTER(ctypes.c_uint8)), shape=(int(offs[-1]),)).tobytes() if nn and offs[-1] else b""
        return counts, offs, raw, int(t.tokens)
    finally:
        lib().moxo_free(ctypes.byref(t))


def count_range(data, own_begin, own_end):
    """Tokens whose first byte lies in [own_begin, own_end) (shard ownership rule)."""
    keep = bytes(data)
    ptr = ctypes.cast(ctypes.c_char_p(keep), ctypes.c_void_p).value
    t = _T()
    rc = lib().moxo_count_range(ptr, len(keep), own_begin, own_end, ctypes.byref(t))
    if rc == EUTF8:
        raise InvalidUtf8(t.invalid_at)
    try:
        import numpy as np
        nn = t.n
        if nn == 0:
            return [], int(t.tokens)
        counts = np.ctypeslib.as_array(t.counts, shape=(nn,)).copy()
        offs = np.ctypeslib.as_array(t.offs, shape=(nn + 1,)).copy()
        raw = ctypes.string_at(t.bytes, int(offs[-1]))
        return [(raw[offs[i]:offs[i + 1]], int(counts[i])) for i in range(nn)], int(t.tokens)
    finally:
        lib().moxo_free(ctypes.byref(t))


def _ptr(data):
    import numpy as np
    if isinstance(data, np.ndarray):
        return data, data.ctypes.data, data.nbytes
    keep = bytes(data)
    return keep, ctypes.cast(ctypes.c_char_p(keep), ctypes.c_void_p).value, len(keep)


def count_digest(data, nthreads=16):
    """(digest tuple (distinct, sum of counts, sum1, sum2), tokens) of the word
    count of ``data`` -- the order-independent fingerprint of the table that
    count() would return, computed without sorting it (for multi-GiB corpora)."""
    import numpy as np
    keep, ptr, n = _ptr(data)
    out = np.zeros(4, np.uint64)
    tok = ctypes.c_uint64()
    rc = lib().moxo_count_digest(ptr, n, nthreads, out.ctypes.data, ctypes.byref(tok))
    del keep
    if rc == EUTF8:
        raise InvalidUtf8(-1)
    return tuple(int(x) for x in out), int(tok.value)


def table_digest(counts, offs, raw, nthreads=16):
    """The same fingerprint of a (counts, offs, bytes) table, e.g. the GPU's."""
    import numpy as np
    counts = np.ascontiguousarray(counts, dtype=np.uint64)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    buf = np.frombuffer(raw, dtype=np.uint8) if len(raw) else np.zeros(1, np.uint8)
    out = np.zeros(4, np.uint64)
    lib().moxo_table_digest(counts.size, counts.ctypes.data, offs.ctypes.data, buf.ctypes.data, nthreads, out.ctypes.data)
    return tuple(int(x) for x in out)


def count_tokens(data, nthreads=16):
    """Token count only (valid UTF-8 assumed): split_whitespace without counting words."""
    keep, ptr, n = _ptr(data)
    r = int(lib().moxo_count_tokens(ptr, n, nthreads))
    del keep
    return r


def count_words(data, words, nthreads=16):
    """Counts of the given distinct lowercased words (bytes) in ``data``."""
    import numpy as np
    words = list(words)
    assert len(set(words)) == len(words), "distinct words only"
    keep, ptr, n = _ptr(data)
    wb = np.frombuffer(b"".join(words) or b"\0", dtype=np.uint8)
    wo = np.zeros(len(words) + 1, np.uint64)
    wo[1:] = np.cumsum([len(w) for w in words])
    out = np.zeros(max(1, len(words)), np.uint64)
    lib().moxo_count_words(ptr, n, nthreads, wb.ctypes.data, wo.ctypes.data, len(words), out.ctypes.data)
    del keep
    return [int(x) for x in out[:len(words)]]
