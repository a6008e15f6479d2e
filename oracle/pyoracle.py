"""ORACLE -- test infrastructure only; never imported by the product path.

Independent Python restatement of the reference's word count
(/root/reference/src/main.rs), used to cross-check the C oracle
(oracle/mox_oracle.c) and to generate the golden fixtures in tests/golden/.

* ``count_words``  -- the semantic contract:
  strict UTF-8 decode (tokio ``lines()`` -> InvalidData, main.rs:44/16),
  ``split_whitespace`` over the explicit Unicode White_Space set that Rust's
  ``char::is_whitespace`` uses (main.rs:96; NOT Python's ``str.split()``, which
  also splits on U+001C..U+001F), ``str.lower()`` (full mapping + Final_Sigma,
  the same rules as Rust's ``to_lowercase``, main.rs:97), integer counts.
* ``reference_pipeline`` -- the reference's structure step by step: round-robin
  line chunks (main.rs:36-51), per-chunk ``count_words`` (main.rs:94-101), the
  ``"word count\\n"`` spill format (main.rs:103-109), the 2-field parser
  (main.rs:152-168) and the merge (main.rs:132-134).  Used on small inputs to
  show the pipeline equals the global count.

PARITY UNPINNED: no Rust toolchain here and the reference has no tests or
fixtures, so neither restatement is pinned to reference outputs.  Python 3.10's
case tables are Unicode 13.0.0 while the engine and the C oracle follow ICU 70.1
(Unicode 14.0.0); the 398 code points where they differ are listed in
tests/golden/unicode_icu70.json and kept out of this module's test alphabets.
"""
import re
from collections import Counter

RUST_WHITESPACE = (
    "\t\n\x0b\x0c\r \x85\xa0\u1680"
    + "".join(chr(c) for c in range(0x2000, 0x200B))
    + "\u2028\u2029\u202f\u205f\u3000"
)
_WS_RE = re.compile("[" + re.escape(RUST_WHITESPACE) + "]+")


class InvalidUtf8(ValueError):
    pass


def split_whitespace(text):
    """Rust str::split_whitespace: no empty tokens."""
    return [t for t in _WS_RE.split(text) if t]


def count_words(data: bytes) -> Counter:
    try:
        text = data.decode("utf-8", errors="strict")
    except UnicodeDecodeError as e:
        raise InvalidUtf8(e.start) from e
    return Counter(w.lower() for w in split_whitespace(text))


def _tokio_lines(text):
    # AsyncBufReadExt::lines: split on '\n', strip one trailing '\r'
    if not text:
        return []
    parts = text.split("\n")
    if parts[-1] == "":
        parts.pop()
    return [p[:-1] if p.endswith("\r") else p for p in parts]


def reference_pipeline(data: bytes, num_chunks=8):
    try:
        text = data.decode("utf-8", errors="strict")
    except UnicodeDecodeError as e:
        raise InvalidUtf8(e.start) from e
    chunks = [""] * num_chunks
    for i, line in enumerate(_tokio_lines(text)):  # split_file, main.rs:44-48
        chunks[i % num_chunks] += line + "\n"
    final = Counter()
    for chunk in chunks:  # map_phase + write_map_result + read_map_result
        counts = Counter(w.lower() for w in split_whitespace(chunk))
        spill = "".join("%s %d\n" % (w, c) for w, c in counts.items())
        parsed = {}
        for line in _tokio_lines(spill):
            parts = split_whitespace(line)
            if len(parts) == 2 and parts[1].isdigit():
                parsed[parts[0]] = int(parts[1])
        for w, c in parsed.items():  # reduce merge, main.rs:132-134
            final[w] += c
    return final


def sorted_items(counter):
    """Deterministic order: bytewise ascending UTF-8 (Rust String Ord)."""
    return sorted(((w.encode("utf-8"), c) for w, c in counter.items()), key=lambda t: t[0])
