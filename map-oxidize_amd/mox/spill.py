"""Intermediate (spill) file compatibility, SURVEY.md §8(f) rank 4.

The reference's pipeline goes through files (/root/reference/src/main.rs):

* ``split_file``      main.rs:36-51   lines dealt round-robin into 8 chunks
* ``map_phase``       main.rs:53-92   per chunk: count_words, then
* ``write_map_result`` main.rs:103-109 ``map_{worker}_chunk_{chunk}.txt``, "word count" lines
* ``read_map_result`` main.rs:152-168 lines with exactly 2 whitespace fields
                                      whose 2nd parses as usize; last wins
* ``reduce_phase``    main.rs:111-150 sum of every file's map

Here the counting of each chunk and the final reduce run on the GPU
(``Engine.count`` / ``mox_reduce_pairs``); splitting, file text formatting and
parsing are host text work.  Only callers that consume or produce the spill
files need this module: the in-memory path (``Engine.count``) is the same
result without files.

Worker ids in file names: the reference's workers pop chunk indices from the
end of a shared queue in a racy order (main.rs:66-68,74); here chunk c is
named as if the chunks were handed out in pop order (c = n-1, n-2, ...) to
workers 0, 1, ... in turn, which is one of the orders the reference produces.
"""
import os
import re

import numpy as np

# Rust char::is_whitespace (Unicode White_Space), which split_whitespace uses
_WS = re.compile("[\t\n\x0b\x0c\r \x85\xa0\u1680\u2000-\u200a\u2028\u2029\u202f\u205f\u3000]+")
_USIZE = re.compile(r"\+?[0-9]+\Z")  # Rust usize FromStr: optional '+', ASCII digits
_USIZE_MAX = (1 << 64) - 1


def lines(data):
    """tokio ``AsyncBufReadExt::lines`` on bytes: split at b'\\n' and strip
    one b'\\r' before it (a final line without newline is kept as is); every
    line must be UTF-8 (else UnicodeDecodeError, the reference's InvalidData)."""
    data = bytes(data)
    parts = data.split(b"\n")
    last = parts.pop()  # text after the final b'\n' (b"" when the data ends with one)
    out = []
    for p in parts:
        if p.endswith(b"\r"):
            p = p[:-1]
        p.decode("utf-8")  # validate (strict)
        out.append(p)
    if last:
        last.decode("utf-8")
        out.append(last)
    return out


def split_file(data, num_chunks=8):
    """main.rs:36-51: line i goes to chunk i % num_chunks, '\\n' re-appended."""
    chunks = [[] for _ in range(num_chunks)]
    for i, ln in enumerate(lines(data)):
        chunks[i % num_chunks].append(ln + b"\n")
    return [b"".join(c) for c in chunks]


def map_file_names(num_chunks=8, num_workers=8):
    """{chunk: file name} in the pop order described in the module docstring."""
    names = {}
    for k, c in enumerate(reversed(range(num_chunks))):
        names[c] = "map_%d_chunk_%d.txt" % (k % num_workers, c)
    return names


def map_phase(engine, chunks, out_dir, num_workers=8):
    """main.rs:53-92: count each chunk on the GPU and write its map file.
    Returns the file paths in the order the reference's results vector would
    hold them (completion order of the pop order)."""
    names = map_file_names(len(chunks), num_workers)
    paths = []
    for c in reversed(range(len(chunks))):
        t = engine.count(chunks[c])
        try:
            p = os.path.join(out_dir, names[c])
            t.write_final_result(p)  # the same "{word} {count}\n" format (main.rs:106)
        finally:
            t.close()
        paths.append(p)
    return paths


def read_map_result(path):
    """main.rs:152-168: {word(bytes): count}; lines without exactly two
    whitespace-separated fields, or whose count is not a usize, are skipped;
    a repeated word keeps its last count (HashMap::insert)."""
    with open(path, "rb") as f:
        data = f.read()
    out = {}
    for ln in lines(data):
        parts = [p for p in _WS.split(ln.decode("utf-8")) if p]
        if len(parts) != 2 or not _USIZE.match(parts[1]):
            continue
        v = int(parts[1])
        if v > _USIZE_MAX:
            continue
        out[parts[0].encode("utf-8")] = v
    return out


def reduce_phase(engine, paths):
    """main.rs:111-150: parse every map file, then sum counts by word with the
    GPU reduce (mox_reduce_pairs).  Returns a mox.Table."""
    words, counts = [], []
    for p in paths:
        m = read_map_result(p)
        words.extend(m.keys())
        counts.extend(m.values())
    return engine.reduce_pairs(words, counts)


def cleanup(paths):
    """main.rs:194-202 (file removal; messages are the caller's business)."""
    for p in paths:
        try:
            os.remove(p)
        except OSError:
            pass


def pack_pairs(words, counts):
    """(bytes, offs uint64[n+1], counts uint64[n]) for mox_reduce_pairs."""
    offs = np.zeros(len(words) + 1, dtype=np.uint64)
    if words:
        offs[1:] = np.cumsum([len(w) for w in words], dtype=np.uint64)
    return b"".join(words), offs, np.asarray(counts, dtype=np.uint64).reshape(-1)
