"""Differential test of the native JSON parser (``native/src/json.hpp``: in-place DOM build,
SSE2 string scans, integer fast path) against Python's ``json``, built with AddressSanitizer +
UndefinedBehaviorSanitizer so reads past the end of a text fail the run.

* every text Python's ``json.loads`` accepts, the native parser accepts with the same value
  (lax and strict; strict also rejects what ``json.loads(strict=True)`` rejects for raw control
  characters inside strings);
* the allocation-free validator (``tt::valid``) accepts exactly what the parser accepts, and
  ``tt::compact`` (16-byte runs) strips exactly the whitespace outside strings;
* arbitrary and truncated byte strings never crash them."""
import json
import os
import random
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
NATIVE = ROOT / "aca_dotnet_workshop_amd" / "native"
CXX = os.environ.get("CXX", "g++")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if shutil.which(CXX) is None:
        pytest.skip("no C++ compiler")
    exe = tmp_path_factory.mktemp("jsonchk") / "json_check"
    cmd = [CXX, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           "-I", str(NATIVE / "src"), str(NATIVE / "tests" / "json_check.cpp"), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "sanitize" in r.stderr and "cannot find" in r.stderr:
        pytest.skip(f"sanitizer runtime unavailable: {r.stderr[-300:]}")
    assert r.returncode == 0, r.stderr[-3000:]

    def run(texts: list[bytes]) -> list[tuple[str, str, str, str]]:
        inp = "".join(t.hex() + "\n" for t in texts)
        p = subprocess.run([str(exe)], input=inp, capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1"))
        assert p.returncode == 0, p.stderr[-3000:]
        assert "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-3000:]
        rows = [tuple(line.split("\t")) for line in p.stdout.split("\n")[:-1]]
        assert len(rows) == len(texts)
        for t, (lax, _strict, ok, comp) in zip(texts, rows):
            assert (ok == "1") == (lax != "ERR"), t  # validator == parser acceptance
            if ok == "1":
                assert bytes.fromhex(comp) == _compact_ref(t), t
        return [r[:2] for r in rows]
    return run


def _compact_ref(t: bytes) -> bytes:
    out, in_str, i = bytearray(), False, 0
    while i < len(t):
        c = t[i]
        if in_str:
            out.append(c)
            if c == 0x5C and i + 1 < len(t):
                i += 1
                out.append(t[i])
            elif c == 0x22:
                in_str = False
        elif c == 0x22:
            in_str = True
            out.append(c)
        elif c not in b" \n\r\t":
            out.append(c)
        i += 1
    return bytes(out)


ALPHABET = "abcXYZ 019_-\"\\/\u00e9\u4e2d\U0001F600\t\n\x01"


def _string(rng):
    return "".join(rng.choice(ALPHABET) for _ in range(rng.choice((0, 1, 3, 15, 16, 17, 40))))


def _value(rng, depth=0):
    k = rng.randrange(9 if depth < 4 else 5)
    if k == 0:
        return None
    if k == 1:
        return rng.random() < 0.5
    if k == 2:
        return rng.randint(-(1 << 53), 1 << 53)
    if k == 3:
        return rng.choice((0.5, -1.25e-7, 3.141592653589793, 1e300, -2.5e-300, rng.uniform(-1e6, 1e6)))
    if k == 4:
        return _string(rng)
    if k in (5, 6):
        return [_value(rng, depth + 1) for _ in range(rng.randrange(6))]
    return {_string(rng): _value(rng, depth + 1) for _ in range(rng.randrange(10))}


def _texts(rng, n):
    out = []
    for _ in range(n):
        v = _value(rng)
        indent = rng.choice((None, None, 0, 2))
        sep = rng.choice(((",", ":"), (", ", ": ")))
        out.append(json.dumps(v, ensure_ascii=rng.random() < 0.5, indent=indent, separators=sep).encode())
    return out


def test_accepts_what_python_accepts_with_equal_values(checker):
    rng = random.Random(20260501)
    texts = _texts(rng, 2500)
    # raw control characters inside strings: lax accepts, strict rejects (json.loads(strict=...))
    texts += [b'{"a":"x\x01y"}', b'["\ttab"]', b'"\x1f"', b'{"k\nnl":1}']
    for t, (lax, strict) in zip(texts, checker(texts)):
        want = json.loads(t.decode(), strict=False)
        assert lax != "ERR", t
        assert json.loads(lax, strict=False) == want, t
        try:
            json.loads(t.decode(), strict=True)
            py_strict = True
        except json.JSONDecodeError:
            py_strict = False
        assert (strict != "ERR") == py_strict, t
        if py_strict:
            assert json.loads(strict) == want, t


def test_numbers(checker):
    cases = [b"0", b"-0", b"7", b"-123456789012345", b"1234567890123456789", b"9007199254740993", b"1.5",
             b"-2.5e-3", b"1E+10", b"[1,-2,3.0]", b"123456789012345678901234567890"]
    for t, (lax, strict) in zip(cases, checker(cases)):
        assert lax == strict != "ERR"
        assert json.loads(lax) == pytest.approx(json.loads(t), rel=1e-15), t
    bad = [b"-", b"1e", b"--1", b"1-", b"[1,]", b"{\"a\" 1}", b"tru", b"nul", b"\"abc", b"[\"\\u12\"]", b"\"\\q\""]
    for t, (lax, strict) in zip(bad, checker(bad)):
        assert lax == strict == "ERR", t


def test_garbage_and_truncations_do_not_crash(checker):
    rng = random.Random(7)
    texts = []
    for t in _texts(rng, 300):
        texts += [t[:i] for i in sorted({rng.randrange(len(t) + 1) for _ in range(6)})]
    texts += [bytes(rng.randrange(256) for _ in range(rng.randrange(1, 64))) for _ in range(500)]
    texts += [b'"' + b"a" * n for n in range(40)] + [b'"' + b"a" * n + b"\\" for n in range(40)]
    rows = checker(texts)
    assert len(rows) == len(texts)
