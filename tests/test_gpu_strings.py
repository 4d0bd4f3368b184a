"""K11 / K13's check of escaped string values (wave_string_ok, kcp_amd/csrc/tokdev.h) on the GPU: whether Go's
decode accepts a string, decided by the whole wave over coalesced loads.  The rule it must give is decode_string's
(tokdev.h; Go 1.16 encoding/json unquote, decode.go): a control byte, an invalid escape or a \\u without four hex
digits is a Go error; invalid UTF-8 Go repairs, and the device leaves it to the host.  go_string_ok restates that
rule; the strings mix escapes, \\u sequences (surrogates included), backslash runs across the 64-byte chunk
boundary, control bytes and UTF-8 valid and not, in documents that are otherwise clean, so the device decides
every document whose string is accepted and defers every other one."""
import random

import pytest

from kcp_amd import gpudiff as G
from kcp_amd import synth as S
from oracle import negotiate_oracle as N
from tests import rollup_cases as C
from tests.test_gpu_rollup import _check as rollup_check

HEX = b"0123456789abcdefABCDEF"


def go_string_ok(raw: bytes, repair: bool = False) -> bool:
    """decode_string(raw) >= 0: the raw bytes between the quotes decode, with no UTF-8 repair.  repair=True: Go's
    own answer (invalid UTF-8 becomes U+FFFD, no error)."""
    i, n = 0, len(raw)
    while i < n:
        c = raw[i]
        if c == 0x5C:
            e = raw[i + 1] if i + 1 < n else None
            if e is not None and e in b'"\\/bfnrt':
                i += 2
                continue
            if e == ord("u"):
                h = raw[i + 2:i + 6]
                if len(h) < 4 or any(x not in HEX for x in h):
                    return False  # (the closing quote, never a hex digit, ends a short one)
                i += 6
                continue
            return False
        if c < 0x20:
            return False
        if c < 0x80:
            i += 1
            continue
        j = i
        while j < n and raw[j] >= 0x80:
            j += 1
        try:
            raw[i:j].decode("utf-8")  # strict: Go's utf8.DecodeRune rejections (overlong, surrogates, > U+10FFFF)
        except UnicodeDecodeError:
            if not repair:
                return False
        i = j
    return True


def _piece(rng):
    k = rng.randrange(20)
    if k == 0:
        return b"x" * rng.randrange(1, 70)
    if k == 1:
        return b"\\" + bytes([rng.choice(b'"\\/bfnrt')])
    if k == 2:
        return b"\\" + bytes([rng.choice(b"xa0'U ")])  # invalid escapes
    if k == 3:
        return b"\\u" + bytes(rng.choice(HEX + b"gG:") for _ in range(4))
    if k == 4:
        return b"\\u" + bytes(rng.choice(HEX) for _ in range(rng.randrange(0, 4)))  # short: the next bytes decide
    if k == 5:
        return bytes([rng.randrange(1, 0x20)])  # a raw control byte
    if k == 6:
        return rng.choice(["é", "€", "😀", "ſ", "K"]).encode()
    if k == 7:
        return rng.choice([b"\xff", b"\xc0\x80", b"\xe2\x82", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\x80"])
    if k == 8:
        return b"\\\\" * rng.randrange(1, 5)  # even backslash runs: nothing escaped after them
    if k == 9:
        return rng.choice([b"\\ud83d\\ude00", b"\\ud83d", b"\\ude00x", b"\\ud83dx"])  # pairs, lone halves
    return b"ok "


def random_strings(n, seed):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        # no piece ends in an unpaired backslash, so the only quotes are escaped ones
        out.append(b"".join(_piece(rng) for _ in range(rng.randrange(1, 8))))
    # escapes straddling the 64-byte chunk boundary (a backslash at byte 63 escapes byte 64)
    for pre in (62, 63, 64, 126, 127):
        for tail in (b'\\"', b"\\\\", b"\\n", b"\\q", b"\\u00e9", b"\\u00g9", b"\\\\\\q", b"\\\\\\n"):
            out.append(b"a" * pre + tail + b"z")
    return out


def _strings_with_flags(n, seed):
    strs = random_strings(n, seed)
    return strs, [go_string_ok(s) for s in strs]


def test_predicate_examples():
    assert go_string_ok(b"plain") and go_string_ok(b'\\"\\\\\\/\\b\\f\\n\\r\\t') and go_string_ok(b"\\u00e9\\uD83D")
    assert not go_string_ok(b"\\x") and not go_string_ok(b"\\u12") and not go_string_ok(b"a\x01")
    assert go_string_ok("é😀".encode()) and not go_string_ok(b"\xff") and not go_string_ok(b"\xed\xa0\x80")


def test_oracle_agrees_with_go_rule():
    """The oracle's parser (oracle/gpudiff_oracle.py _Parser.string) and the host path (rollup.cpp) reject exactly
    the strings Go rejects -- a \\u takes four hex digits, not whitespace, a sign or '_' (Python's int(x, 16) does)."""
    from oracle import rollup_oracle as R
    from tests.test_rollup import _host, _oracle
    for s in (b"\\u245\t", b"\\u 245", b"\\u+245", b"\\u-245", b"\\u2_45", b"\\u0x12"):
        with pytest.raises(R.DecodeError):
            R.extract(b'{"x":"' + s + b'"}')
    strs, _ = _strings_with_flags(1500, 91)
    base, _ = S.rollup_population(1, 1, seed=92)
    for s in strs:
        d = base[1].replace(b"Deployment has minimum availability.", s, 1)
        o = _oracle(d)
        assert (o == C.DECODE) == (not go_string_ok(s, repair=True)), s
        assert _host(d) == o, s


@pytest.mark.gpu
def test_rollup_string_validity():
    strs, ok = _strings_with_flags(1500, 91)
    assert 0.15 < sum(ok) / len(ok) < 0.85  # both outcomes well represented
    base, _ = S.rollup_population(1, 1, seed=92)
    tmpl = base[1]
    assert b"Deployment has minimum availability." in tmpl
    docs = [tmpl.replace(b"Deployment has minimum availability.", s, 1) for s in strs]
    eng = G.Engine(device=0)
    try:
        res = rollup_check(eng, docs)  # groups and sums equal the oracle's, whoever decided each document
        st = res.k11_status.tolist()
        bad = [(i, st[i], strs[i]) for i in range(len(strs)) if (st[i] == G.TOK_OK) != ok[i]]
        assert not bad, (len(bad), bad[:5])
    finally:
        eng.close()


@pytest.mark.gpu
def test_negotiate_string_validity():
    strs, ok = _strings_with_flags(1500, 93)
    pairs, _ = S.negotiate_population(1, seed=94, variants=False)
    old, new = pairs[0]
    assert b'"description":"Ready column"' in new
    mixed = [(old, new.replace(b'"description":"Ready column"', b'"description":"' + s + b'"', 1)) for s in strs]
    eng = G.Engine(device=0)
    try:
        nb = eng.nbatch(mixed)
        try:
            nb.run()
            got = nb.fetch().tolist()
            st = nb.stats()
        finally:
            nb.close()
        want = [N.classify(a, b) for a, b in mixed]
        assert got == want
        # spec strings are read only by N0: an accepted one leaves the pair on the device
        assert st.n_host == len(strs) - sum(ok), (st.n_host, len(strs) - sum(ok))
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["spec", "status"])
def test_upsert_string_decode(mode):
    """K10 decodes escaped strings by the whole wave (wave_decode_string<true>) and re-escapes them: every body equals
    the host path's, and the device emits exactly the bodies whose strings decode without UTF-8 repair."""
    from tests import upsert_cases as UC
    from tests.test_gpu_upsert import _check as upsert_check
    strs, ok = _strings_with_flags(700, 95)
    base, _ = S.rollup_population(1, 1, seed=96)
    if mode == "spec":
        m, old = UC.SPEC, b'"IfNotPresent"'
    else:
        m, old = UC.STATUS, b'"Deployment has minimum availability."'
    assert old in base[1]
    docs = [base[1].replace(old, b'"' + s + b'"', 1) for s in strs]
    eng = G.Engine(device=0)
    try:
        codes = upsert_check(eng, docs, m, must_device=False)
        bad = [(i, codes[i], strs[i]) for i in range(len(strs)) if (codes[i] == G.TOK_OK) != ok[i]]
        assert not bad, (len(bad), bad[:5])
    finally:
        eng.close()
