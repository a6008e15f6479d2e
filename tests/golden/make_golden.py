#!/usr/bin/env python3
"""Generate tests/golden/kat.json: known-answer vectors for the word-count contract.

The reference ships no tests, fixtures or outputs and cannot be built here (no
Rust toolchain), so these vectors are PARITY UNPINNED against the reference
itself: expected outputs come from oracle/pyoracle.py (independent Python
restatement of /root/reference/src/main.rs:94-101 + :36-51) and the hand-written
expectations of SURVEY.md §0.1 are asserted on top.

Regenerate: python tests/golden/make_golden.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle  # noqa: E402

CASES = []


def case(name, data, expect=None):
    CASES.append((name, data, expect))


# SURVEY.md §0.1 known-answer table (expectations written by hand)
case("survey_hello", b"Hello hello\tHELLO\nworld", {"hello": 3, "world": 1})
case("survey_vt_ff_cr", b"a\x0bb\x0cc\rd\r\n", {"a": 1, "b": 1, "c": 1, "d": 1})
case("survey_fs_not_ws", b"foo\x1cbar", {"foo\x1cbar": 1})
case("survey_punct", b"The, the. THE", {"the,": 1, "the.": 1, "the": 1})
case("survey_zwsp", "x y x​y".encode(), {"x": 1, "y": 1, "x​y": 1})
case("survey_final_sigma", "ΟΔΟΣ ΣΑ".encode(), {"οδος": 1, "σα": 1})
case("survey_dotted_i_kelvin", "İ K K".encode(), {"i̇": 1, "k": 2})
case("survey_bom", "﻿The the".encode(), {"﻿the": 1, "the": 1})
case("survey_empty", b"", {})
case("survey_invalid", b"ab\xffcd", "error")

# every ASCII byte as a separator candidate
for c in range(0x80):
    case("sep_%02x" % c, b"a" + bytes([c]) + b"b")
# every multi-byte White_Space char, plus near misses
for cp in [0x85, 0xA0, 0x1680] + list(range(0x2000, 0x200B)) + [0x2028, 0x2029, 0x202F, 0x205F, 0x3000,
                                                                 0x200B, 0x200C, 0xFEFF, 0x180E, 0x2060, 0x3001]:
    case("mbws_%04x" % cp, ("Ab" + chr(cp) + "Cd").encode())
case("crlf_lines", b"one two\r\nthree\r\n\r\nfour")
case("no_trailing_newline", b"alpha beta gamma")
case("all_whitespace", b" \t\n\r\x0b\x0c  \n")
case("leading_trailing_ws", b"   x   ")
case("nul_bytes", b"a\x00b a\x00b A\x00B \x00 \x00\x00")
case("len_boundaries", b" ".join(b"W" * k for k in range(1, 40)) + b" " + b" ".join(b"w" * k for k in range(1, 40)))
case("len16_mixed", b"ABCDEFGHIJKLMNOP abcdefghijklmnop AbCdEfGhIjKlMnOp abcdefghijklmnopq ABCDEFGHIJKLMNOPQ")
case("digits_symbols", b"123 123 1-2-3 $$ $$ @x @X")
case("sigma_context", "Σ ΣΣ ΑΣ ΑΣΑ ΑΣ'Σ ΑΣ. a­Σ ΑΣ́ Σ1 1Σ ΑΣ1Α".encode())
case("greek_cyrillic", "Οδυσσέας ΟΔΥΣΣΕΑΣ МОСКВА москва Москва".encode())
case("special_casing", "İSTANBUL İstanbul i̇stanbul ß SS Ǆ ǅ ǆ ǈ".encode())
case("kelvin_long", ("ABCDEFGHIJKLMNOPK abcdefghijklmnopk").encode())
case("cjk_emoji", "日本語 日本語 東京 😀smile 😀SMILE 𝔘𝔫𝔦".encode())
case("combining", "é É é".encode())
case("long_unicode", ("Ä" * 40 + " " + "ä" * 40).encode())
# invalid UTF-8 variants (reference: InvalidData -> exit 1, no output)
for name, data in [("trunc_2", b"ok \xc3"), ("trunc_3", b"ok \xe2\x80"), ("overlong_c0", b"x \xc0\x80 y"),
                   ("overlong_e0", b"\xe0\x80\xaf"), ("surrogate", b"\xed\xa0\x80"), ("f5", b"\xf5\x80\x80\x80"),
                   ("above_max", b"\xf4\x90\x80\x80"), ("lone_cont", b"a \x80 b"), ("bad_cont", b"\xe2\x28\xa1"),
                   ("overlong_f0", b"\xf0\x80\x80\xaf"), ("c1", b"\xc1\xbf")]:
    case("invalid_" + name, data, "error")


def run(data):
    try:
        return dict(pyoracle.count_words(data))
    except pyoracle.InvalidUtf8:
        return "error"


def main():
    out = []
    for name, data, expect in CASES:
        got = run(data)
        if expect is not None:
            if expect == "error":
                assert got == "error", (name, got)
            else:
                assert got == expect, (name, got, expect)
        pipe = "error"
        try:
            pipe = dict(pyoracle.reference_pipeline(data))
        except pyoracle.InvalidUtf8:
            pass
        assert pipe == got, ("pipeline != global count", name)
        entry = {"name": name, "input_hex": data.hex()}
        if got == "error":
            entry["error"] = "utf8"
        else:
            entry["expected"] = [[w.encode().hex(), c] for w, c in sorted(got.items(), key=lambda kv: kv[0].encode())]
        out.append(entry)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat.json")
    with open(path, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "parity": "unpinned (no reference outputs exist)",
                   "cases": out}, f, indent=0)
    print("wrote %d cases to %s" % (len(out), path))


if __name__ == "__main__":
    main()
