"""CPU: the record layout and level scheme of the device bytewise sort
(map-oxidize_amd/csrc/mox_bsort.hip) restated in Python and checked against
Python's bytes order (= Rust String Ord).

Each level sorts records by (run, key) with key = the word's 7-byte window at
that level big-endian in bits 63..8 and aux = min(bytes left, 8) in bits 7..0;
records tied on (run, key) with aux == 8 form runs that the next level
re-sorts on the next window.  The GPU does the per-level sort as an LSD radix
(stable); here a stable sort by the same key stands in for it.  No GPU code
runs here: this pins the key construction and the tie rule the kernels use."""
import random

WIN, AUX_MORE = 7, 8


def window(word, level):
    a = WIN * level
    have = max(0, len(word) - a)
    k = 0
    for j in range(min(have, WIN)):
        k |= word[a + j] << (8 * (7 - j))
    return k | (AUX_MORE if have > WIN else have)


def model_sort(words):
    recs = [(0, window(w, 0), i) for i, w in enumerate(words)]  # (run, key, idx)
    recs.sort(key=lambda r: (r[0], r[1]))
    run_base, level = 1, 1
    while True:
        # tie runs: equal (run, key) with aux == AUX_MORE on both sides
        tied = [False] * len(recs)
        heads = []
        for j in range(1, len(recs)):
            a, b = recs[j - 1], recs[j]
            if (a[1] & 0xFF) == AUX_MORE and a[0] == b[0] and a[1] == b[1]:
                if not tied[j - 1]:
                    heads.append(j - 1)
                tied[j - 1] = tied[j] = True
        if not heads:
            break
        # subset in sorted position order, run id = base + index of its run
        run_of, r = {}, -1
        for j in range(len(recs)):
            if j in heads:
                r += 1
            if tied[j]:
                run_of[j] = run_base + r
        pos = sorted(run_of)
        sub = [(run_of[j], window(words[recs[j][2]], level), recs[j][2]) for j in pos]
        sub.sort(key=lambda x: (x[0], x[1]))
        for j, s in zip(pos, sub):
            recs[j] = s
        run_base += len(heads)
        level += 1
    return [words[r[2]] for r in recs]


def test_model_matches_bytes_order():
    rng = random.Random(7)
    alphabet = b"ab\x01z\xff"
    for trial in range(200):
        n = rng.randint(0, 60)
        words = set()
        base = bytes(rng.choice(alphabet) for _ in range(rng.randint(0, 20)))
        while len(words) < n:
            kind = rng.random()
            if kind < 0.4:  # shared long prefixes: ties over several levels
                w = base[:rng.randint(0, len(base))] + bytes(rng.choice(alphabet) for _ in range(rng.randint(0, 9)))
            else:
                w = bytes(rng.choice(alphabet) for _ in range(rng.randint(1, 30)))
            if w:
                words.add(w)
        words = list(words)
        rng.shuffle(words)
        assert model_sort(words) == sorted(words)


def test_window_prefix_and_length_classes():
    # a proper prefix sorts first; equal windows order by the bytes left
    assert window(b"abc", 0) < window(b"abcd", 0) < window(b"abcdefg", 0) < window(b"abcdefgh", 0)
    assert window(b"abcdefgh", 0) == window(b"abcdefgz", 0)  # both go on past the window: a tie
    assert window(b"abcdefgh", 0) & 0xFF == AUX_MORE and window(b"abcdefg", 0) & 0xFF == 7
    assert window(b"abcdefgh", 1) == (ord("h") << 56) | 1
