"""Colliding pairs of the 32-bit key-hash folds (old rotate/xor, new multiply/xor)
over the ZIPF vocabulary (each word lowercased, bare and with each trailing mark)
and 3 M distinct HICARD-like keys, against the random-hash expectation.
profiles/r05/hash_fold_collisions.txt is its output."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "map-oxidize_amd"))
from mox import corpus
L = corpus.lib()
V = 1 << 20
buf = ctypes.create_string_buffer(64)
ks = set()
for i in range(V):
    n = L.mox_corpus_vocab_word(i, buf, 64)
    w = buf.raw[:n].lower()
    for m in [b"", b",", b".", b";", b":", b"!", b"?"]:
        if len(w + m) <= 16: ks.add(w + m)
ks = list(ks)
rng = np.random.default_rng(1)
alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", np.uint8)
def pack(keys):
    arr = np.zeros((len(keys), 16), np.uint8)
    for j, k in enumerate(keys): arr[j, :len(k)] = np.frombuffer(k, np.uint8)
    return arr.view("<u4").astype(np.uint64)
hic = set()
while len(hic) < 3_000_000:
    L_ = rng.integers(4, 17, 200000)
    ch = alpha[rng.integers(0, 36, (200000, 16))]
    for l, c in zip(L_, ch): hic.add(c[:l].tobytes())
hic = list(hic)
M = 0xFFFFFFFF
def rotl(x, r): return ((x << r) | (x >> (32 - r))) & M
def fin(a):
    a = (a * 0x9E3779B1) & M; a ^= a >> 15; a = (a * 0x85EBCA6B) & M; a ^= a >> 13; return a
cands = {
 "current": lambda k: fin(k[:, 0] ^ rotl(k[:, 1], 11) ^ rotl(k[:, 2], 21) ^ rotl(k[:, 3], 6)),
 "mul3": lambda k: fin(k[:, 0] ^ ((k[:, 1] * 0x85EBCA77) & M) ^ ((k[:, 2] * 0xC2B2AE3D) & M) ^ ((k[:, 3] * 0x27D4EB2F) & M)),
 "hash32b_new": lambda k: fin(k[:, 1] ^ ((k[:, 0] * 0x2127599B) & M) ^ ((k[:, 3] * 0x165667B1) & M) ^ ((k[:, 2] * 0xD3A2646D) & M)),
 "hash32b_old": lambda k: fin(k[:, 1] ^ rotl(k[:, 0], 7) ^ rotl(k[:, 3], 17) ^ rotl(k[:, 2], 27)),
}
for name, keys in (("zipf vocab", ks), ("hicard", hic)):
    k4 = pack(keys)
    n = len(keys)
    print(name, n, "random expectation ~%.0f colliding pairs" % (n * (n - 1) / 2 / 2**32))
    for cn, f in cands.items():
        h = f(k4)
        u, cnt = np.unique(h, return_counts=True)
        pairs = (cnt * (cnt - 1) // 2).sum()
        print("  %-8s colliding pairs %d" % (cn, pairs))
