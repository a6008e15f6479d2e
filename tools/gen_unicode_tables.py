#!/usr/bin/env python3
"""Generate the Unicode case tables used by the GPU Unicode lane and the C
oracle, and the ICU-pinned known-answer fixture the tests check them with.

The reference lowercases every token with Rust's ``str::to_lowercase``
(/root/reference/src/main.rs:97): the full (SpecialCasing unconditional)
lowercase mapping per char plus the contextual Final_Sigma rule, which reads
the ``Cased`` and ``Case_Ignorable`` derived properties; tokens are split on
``char::is_whitespace`` (the ``White_Space`` property).  Rust is not installed
here, so the data come from ICU 70.1 (Unicode 14.0.0, the system libicuuc):
``tools/icu_case_dump.c`` prints ``u_strToLower`` (root locale) of every code
point alone and its ``UCHAR_CASED`` / ``UCHAR_CASE_IGNORABLE`` /
``UCHAR_WHITE_SPACE`` bits, and lowercases the Final_Sigma probe strings.

Cross-check: this interpreter's ``unicodedata`` (Unicode 13.0.0, CPython 3.10)
is an independent second source.  Every code point where the two disagree must
be either assigned in Unicode 14.0 (``u_charAge``) or listed in
``KNOWN_CHANGES`` with the reason; anything else aborts the generator.  The
disagreements are written to the fixture as KATs with their Unicode version.

Outputs (both committed; regenerate with ``python tools/gen_unicode_tables.py``):
  map-oxidize_amd/csrc/mox_unicode_tables.h   the engine's tables
  tests/golden/unicode_icu70.json             ICU answers: lower map, property
                                              ranges, White_Space, Final_Sigma
                                              probes, CPython-13 differences
"""
import json
import os
import subprocess
import sys
import tempfile
import unicodedata

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIGMA, FINAL, NONFINAL = 0x3A3, 0x3C2, 0x3C3
SPECIAL_I_DOT = 0x110000  # sentinel: U+0130 -> U+0069 U+0307
# Unicode 14.0 changes to code points assigned earlier that touch the case data.
KNOWN_CHANGES = {0x1734: "HANUNOO SIGN PAMUDPOD: General_Category Mn -> Mc in Unicode 14.0, "
                         "so it is no longer Case_Ignorable"}
# Final_Sigma probe templates; X is the probed code point.  Together they
# recover Cased and Case_Ignorable of X from the contextual rule alone.
TEMPLATES = [[0x41, "X", SIGMA], [0x41, SIGMA, "X"], ["X", SIGMA], [0x41, SIGMA, "X", 0x62]]
# Hand-picked strings, lowercased by ICU as a whole.
EXTRA = ["ΌΣΟΣ", "ΣΑΣ'", "A'Σ'", "AΣΣ", "Σ", "ΣΣ", "AΣ.B", "AΣ.", "A.Σ", "ΑΣͅ", "ΑΣͅΒ",
         "İSTANBUL", "AİΣ", "ᾼΣ", "ǅΣ", "ʰΣ", "ΣʰA", "AΣ­B", "A­Σ", "ΑΣ\U0001D165",
         "ΔΣ‍Α", "ΏΣ", "KKΣ", "ẞΣ", "ΣΑΣΑΣ", "𐐀Σ", "Σ𐐀", "ⰯΣ", "AΣⰯ",
         "\U00010570Σ", "A᜴Σ", "AΣ᜴B"]


def dump_icu(tmp):
    exe = os.path.join(tmp, "icu_case_dump")
    subprocess.run(["gcc", "-O2", "-o", exe, os.path.join(ROOT, "tools", "icu_case_dump.c"), "-licuuc"],
                   check=True)
    out = subprocess.run([exe, "--table"], check=True, capture_output=True, text=True).stdout
    head, *lines = out.splitlines()
    _, _, uver, _, icuver = head.split()
    lower, age, cased, ci, ws = {}, {}, set(), set(), set()
    for ln in lines:
        cp, a, lw, fl = ln.split()
        cp = int(cp, 16)
        age[cp] = a
        lw = tuple(int(x, 16) for x in lw.split("."))
        if lw != (cp,):
            lower[cp] = lw
        cased |= {cp} if "C" in fl else set()
        ci |= {cp} if "I" in fl else set()
        ws |= {cp} if "W" in fl else set()
    return exe, uver, icuver, lower, age, cased, ci, ws


def icu_strings(exe, strs):
    inp = "".join(s.encode().hex() + "\n" for s in strs)
    out = subprocess.run([exe, "--strings"], input=inp, check=True, capture_output=True, text=True).stdout
    return [bytes.fromhex(h).decode() for h in out.splitlines()]


def cpython13(cp, c):
    l = c.lower()
    cs = c.islower() or c.isupper() or unicodedata.category(c) == "Lt"
    # Case_Ignorable recovered by probing CPython's own Final_Sigma rule
    if cs:
        ign = ("A" + chr(SIGMA) + c).lower()[1] == chr(FINAL)
    else:
        ign = ("A" + c + chr(SIGMA)).lower()[-1] == chr(FINAL)
    return tuple(map(ord, l)), cs, ign


def ranges(cps):
    out = []
    for cp in sorted(cps):
        if out and cp == out[-1][1] + 1:
            out[-1][1] = cp
        else:
            out.append([cp, cp])
    return out


def lower_str(s, lower):
    return "".join("".join(map(chr, lower.get(ord(ch), (ord(ch),)))) for ch in s)


def main():
    with tempfile.TemporaryDirectory() as tmp:
        exe, uver, icuver, lower, age, cased, ci, ws = dump_icu(tmp)
        # -- cross-check against CPython's Unicode 13.0 ---------------------------------
        diffs = []
        for cp in range(0x110000):
            if 0xD800 <= cp <= 0xDFFF:
                continue
            want = (lower.get(cp, (cp,)), cp in cased, cp in ci)
            got = cpython13(cp, chr(cp))
            for what, a, b in zip(("lower", "cased", "case_ignorable"), want, got):
                if a != b:
                    a_ = list(a) if isinstance(a, tuple) else a
                    b_ = list(b) if isinstance(b, tuple) else b
                    diffs.append({"cp": cp, "age": age.get(cp), "what": what, "icu70": a_, "cpython13": b_})
        unk = [d["cp"] for d in diffs if d["age"] is None]
        if unk:
            out = subprocess.run([exe, "--age"], input="".join("%x\n" % c for c in unk), check=True,
                                 capture_output=True, text=True).stdout.split()
            age.update(zip(unk, out))
            for d in diffs:
                d["age"] = age[d["cp"]]
        bad = [d for d in diffs if d["age"] != uver.rsplit(".", 1)[0] and d["cp"] not in KNOWN_CHANGES]
        if bad:
            sys.exit("ICU 70 and CPython %s disagree outside Unicode %s additions: %s"
                     % (unicodedata.unidata_version, uver, bad[:10]))
        for d in diffs:
            if d["cp"] in KNOWN_CHANGES:
                d["note"] = KNOWN_CHANGES[d["cp"]]
        assert {cp for cp, l in lower.items() if len(l) > 1} == {0x130} and lower[0x130] == (0x69, 0x307)
        assert max(max(l) for l in lower.values()) < 0x110000
        # -- Final_Sigma probes ---------------------------------------------------------------
        probe = sorted((cased | ci | set(lower) | {0x31, 0x2D, 0x5F}) - ws - {SIGMA})
        strs = ["".join(chr(x) if x != "X" else chr(cp) for x in t) for cp in probe for t in TEMPLATES]
        got = icu_strings(exe, strs + EXTRA)
        mask = []
        for i, cp in enumerate(probe):
            m = 0
            for k, t in enumerate(TEMPLATES):
                s, r = strs[4 * i + k], got[4 * i + k]
                pos = lower_str(s[:t.index(SIGMA)], lower)
                fin = r[len(pos)] == chr(FINAL)
                assert r[len(pos)] in (chr(FINAL), chr(NONFINAL)), (hex(cp), k, r)
                # the ICU output is the per-char map with the sigma choice: mask is lossless
                exp = lower_str(s, lower)
                assert r == exp[:len(pos)] + r[len(pos)] + exp[len(pos) + 1:], (hex(cp), k, r, exp)
                m |= fin << k
            mask.append(m)
        extra = [[s.encode().hex(), r.encode().hex()] for s, r in zip(EXTRA, got[len(strs):])]
    # -- header ----------------------------------------------------------------------------------
    lo = sorted(lower)
    dst = [SPECIAL_I_DOT if len(lower[c]) > 1 else lower[c][0] for c in lo]
    cr, cir = ranges(cased), ranges(ci)
    path = os.path.join(ROOT, "map-oxidize_amd", "csrc", "mox_unicode_tables.h")
    with open(path, "w") as f:
        w = f.write
        w("/* GENERATED by tools/gen_unicode_tables.py -- do not edit.\n")
        w(" * Unicode %s case data from ICU %s (u_strToLower, root locale; UCHAR_CASED,\n" % (uver, icuver))
        w(" * UCHAR_CASE_IGNORABLE), cross-checked against CPython unicodedata %s, for Rust\n"
          % unicodedata.unidata_version)
        w(" * str::to_lowercase semantics (/root/reference/src/main.rs:97): per-char full\n")
        w(" * lowercase map and the Cased / Case_Ignorable ranges of the Final_Sigma rule. */\n")
        w("#pragma once\n#include <stdint.h>\n\n")
        w("#define MOX_UNICODE_VERSION \"%s\"\n" % uver)
        w("#define MOX_LOWER_SPECIAL_I_DOT 0x110000u /* U+0130 -> U+0069 U+0307 */\n")
        w("#define MOX_LOWER_N %d\n#define MOX_CASED_N %d\n#define MOX_CI_N %d\n\n" % (len(lo), len(cr), len(cir)))

        def arr(name, vals):
            w("static const uint32_t %s[%d] = {\n" % (name, len(vals)))
            for i in range(0, len(vals), 8):
                w("  " + ", ".join("0x%05x" % v for v in vals[i:i + 8]) + ",\n")
            w("};\n")

        arr("mox_lower_src", lo)
        arr("mox_lower_dst", dst)
        arr("mox_cased_lo", [a for a, _ in cr])
        arr("mox_cased_hi", [b for _, b in cr])
        arr("mox_ci_lo", [a for a, _ in cir])
        arr("mox_ci_hi", [b for _, b in cir])
    # -- fixture ---------------------------------------------------------------------------------
    fx = {
        "source": "ICU %s u_strToLower(root locale) / u_hasBinaryProperty / u_charAge, via "
                  "tools/icu_case_dump.c; generated by tools/gen_unicode_tables.py" % icuver,
        "icu": icuver, "unicode": uver, "cpython_unicode": unicodedata.unidata_version,
        "lower": [[c, list(lower[c])] for c in lo],
        "cased": cr, "case_ignorable": cir, "white_space": sorted(ws),
        "sigma_templates": [[x if x == "X" else x for x in t] for t in TEMPLATES],
        "sigma_probe": probe, "sigma_final_mask": "".join("%x" % m for m in mask),
        "strings": extra,
        "differs_from_cpython13": diffs,
    }
    gpath = os.path.join(ROOT, "tests", "golden", "unicode_icu70.json")
    with open(gpath, "w") as f:
        json.dump(fx, f, separators=(",", ":"))
        f.write("\n")
    print("wrote %s: %d lower, %d cased ranges, %d case-ignorable ranges (Unicode %s, ICU %s)"
          % (path, len(lo), len(cr), len(cir), uver, icuver))
    print("wrote %s: %d probes, %d CPython-%s differences" % (gpath, len(probe), len(diffs),
                                                             unicodedata.unidata_version))


if __name__ == "__main__":
    sys.exit(main())
