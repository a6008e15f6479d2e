"""CPU: the case tables and the C oracle pinned to ICU 70.1 (Unicode 14.0.0).

tests/golden/unicode_icu70.json holds ICU's answers (tools/gen_unicode_tables.py
runs u_strToLower / u_hasBinaryProperty through tools/icu_case_dump.c):
the per-code-point full lowercase map, the Cased and Case_Ignorable ranges,
White_Space, a Final_Sigma mask for 6,857 probe code points under four
templates, hand-picked whole strings, and every code point where ICU 70 and
CPython's Unicode 13.0 disagree (the KATs of the Unicode 14.0 changes).
The GPU engine is checked against the same fixture in
tests/test_gpu_parity.py::test_unicode_icu70_kats."""
import json
import os
import re

import pytest

import coracle
from conftest import ROOT

FIX = os.path.join(ROOT, "tests", "golden", "unicode_icu70.json")
HDR = os.path.join(ROOT, "map-oxidize_amd", "csrc", "mox_unicode_tables.h")


@pytest.fixture(scope="module")
def fx():
    with open(FIX) as f:
        return json.load(f)


def icu_words(fx):
    """(input, ICU lowercase) pairs for every probe string and hand-picked string."""
    lower = {c: "".join(map(chr, d)) for c, d in fx["lower"]}
    low = lambda s: "".join(lower.get(ord(ch), ch) for ch in s)  # noqa: E731
    out = []
    for cp, m in zip(fx["sigma_probe"], fx["sigma_final_mask"]):
        m = int(m, 16)
        for k, t in enumerate(fx["sigma_templates"]):
            parts = [chr(cp) if x == "X" else chr(x) for x in t]
            i = t.index(0x3A3)
            want = low("".join(parts[:i])) + ("ς" if m >> k & 1 else "σ") + low("".join(parts[i + 1:]))
            out.append(("".join(parts), want))
    for a, b in fx["strings"]:
        out.append((bytes.fromhex(a).decode(), bytes.fromhex(b).decode()))
    return out


def header_arrays():
    h = open(HDR).read()

    def arr(name):
        m = re.search(r"%s\[\d+\] = \{(.*?)\};" % name, h, re.S)
        return [int(x, 16) for x in re.findall(r"0x[0-9a-f]+", m.group(1))]

    ver = re.search(r'MOX_UNICODE_VERSION "([0-9.]+)"', h).group(1)
    return ver, arr


def test_header_tables_are_icu70(fx):
    ver, arr = header_arrays()
    assert ver == fx["unicode"] == "14.0.0" and fx["icu"] == "70.1"
    lower = {c: d for c, d in fx["lower"]}
    dst = [0x110000 if len(lower[c]) > 1 else lower[c][0] for c in sorted(lower)]
    assert arr("mox_lower_src") == sorted(lower) and arr("mox_lower_dst") == dst
    assert [list(r) for r in zip(arr("mox_cased_lo"), arr("mox_cased_hi"))] == fx["cased"]
    assert [list(r) for r in zip(arr("mox_ci_lo"), arr("mox_ci_hi"))] == fx["case_ignorable"]


def test_oracle_white_space_is_icu70(fx):
    ws = set(fx["white_space"])
    assert len(ws) == 25
    for cp in range(0x110000):
        if 0xD800 <= cp <= 0xDFFF:
            continue
        assert coracle.is_whitespace(cp) == (cp in ws), hex(cp)


def test_oracle_lowercase_matches_icu70(fx):
    lower = {c: "".join(map(chr, d)) for c, d in fx["lower"]}
    for cp, _ in fx["lower"]:  # each mapped code point alone (Σ alone is not final)
        got = coracle.lowercase(chr(cp).encode())
        assert got == lower[cp].encode(), hex(cp)
    pairs = icu_words(fx)
    assert len(pairs) > 27000
    for s, want in pairs:
        assert coracle.lowercase(s.encode()) == want.encode(), (s, want)


def test_unicode14_changes_are_kats(fx):
    """Every ICU 70 / CPython 13.0 difference is a Unicode 14.0 addition or the
    one 14.0 property change, and the oracle follows ICU on each of them."""
    diffs = fx["differs_from_cpython13"]
    assert len(diffs) == 398
    assert {d["age"] for d in diffs} == {"14.0", "3.2"}
    assert {d["cp"] for d in diffs if d["age"] != "14.0"} == {0x1734}
    lower = {c: "".join(map(chr, d)) for c, d in fx["lower"]}
    for d in diffs:
        c = chr(d["cp"])
        if d["what"] == "lower":
            assert coracle.lowercase(c.encode()) == lower[d["cp"]].encode()
        # 'A' + c + 'Σ' is final iff c is Case_Ignorable or Cased (ICU's answer)
        fin = d["icu70"] if d["what"] != "lower" else None
        if d["what"] == "case_ignorable" and fin:
            assert coracle.lowercase(("A" + c + "Σ").encode()).endswith("ς".encode())
    # U+1734 is no longer Case_Ignorable: it breaks the Final_Sigma look-behind
    assert coracle.lowercase("A᜴Σ".encode()).endswith("σ".encode())
    # a Unicode 14.0 case pair: U+2C2F GLAGOLITIC CAPITAL LETTER CAUDATE CHRIVI
    assert coracle.lowercase("Ⱟ".encode()) == "ⱟ".encode()


def test_oracle_case_header_is_generated_from_the_fixture():
    """The oracle's own case tables (oracle/mox_oracle_case.h, not the product's
    header) are exactly what oracle/gen_case_tables.py writes from the ICU 70.1
    fixture."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_case_tables", os.path.join(ROOT, "oracle", "gen_case_tables.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    assert open(os.path.join(ROOT, "oracle", "mox_oracle_case.h")).read() == gen.build_text()
    src = open(os.path.join(ROOT, "oracle", "mox_oracle.c")).read()
    assert "mox_unicode_tables.h" not in src.replace("mox_unicode_tables.h is", "")
