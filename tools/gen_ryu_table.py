#!/usr/bin/env python3
"""Generates kcp_amd/csrc/ryu_tables.h: the 128-bit power-of-5 tables of the
Ryu shortest float64 -> decimal algorithm (Ulf Adams, PLDI 2018), computed
exactly with Python integers, plus `d2d_model`, an integer-exact Python model
of the same algorithm over the same truncated tables.  `--check N` validates
the model against numpy's shortest representation (Dragon4, unique=True) on N
random doubles -- the model is what the device code (tokdev.h d2d_shortest)
restates line by line.

Table definitions (Ryu d2s, 125-bit variants):
  POW5_SPLIT[i]     = 5^i scaled to 125 bits:  5^i >> (pow5bits(i) - 125)
  POW5_INV_SPLIT[q] = floor(2^(pow5bits(q) - 1 + 125) / 5^q) + 1
"""
import os
import random
import struct
import sys

POW5_INV_BITCOUNT = 125
POW5_BITCOUNT = 125
N_POW5 = 326
N_POW5_INV = 342


def pow5bits(e):
    return ((e * 1217359) >> 19) + 1


def log10pow2(e):
    return (e * 78913) >> 18


def log10pow5(e):
    return (e * 732923) >> 20


def pow5_split(i):
    v = 5 ** i
    s = pow5bits(i) - POW5_BITCOUNT
    return v >> s if s >= 0 else v << -s


def pow5_inv_split(q):
    return (1 << (pow5bits(q) - 1 + POW5_INV_BITCOUNT)) // (5 ** q) + 1


POW5 = [pow5_split(i) for i in range(N_POW5)]
POW5_INV = [pow5_inv_split(q) for q in range(N_POW5_INV)]
assert all(x < (1 << 128) for x in POW5 + POW5_INV)


def pow5_factor(v):
    c = 0
    while v % 5 == 0:
        v //= 5
        c += 1
    return c


def mul_shift(m, mul, j):
    # (m * mul) >> j with the 64x128 -> 192-bit product, as the device does
    return (m * mul) >> j


def d2d_model(bits):
    """-> (digits integer, decimal exponent) of the shortest, closest
    representation (ties to even), for a finite nonzero double."""
    ieee_m = bits & ((1 << 52) - 1)
    ieee_e = (bits >> 52) & 0x7FF
    if ieee_e == 0:
        e2 = 1 - 1023 - 52 - 2
        m2 = ieee_m
    else:
        e2 = ieee_e - 1023 - 52 - 2
        m2 = (1 << 52) | ieee_m
    even = (m2 & 1) == 0
    accept = even
    mv = 4 * m2
    mm_shift = 1 if (ieee_m != 0 or ieee_e <= 1) else 0
    vm_tz = vr_tz = False
    if e2 >= 0:
        q = log10pow2(e2) - (1 if e2 > 3 else 0)
        e10 = q
        k = POW5_INV_BITCOUNT + pow5bits(q) - 1
        i = -e2 + q + k
        mul = POW5_INV[q]
        vr = mul_shift(4 * m2, mul, i)
        vp = mul_shift(4 * m2 + 2, mul, i)
        vm = mul_shift(4 * m2 - 1 - mm_shift, mul, i)
        if q <= 21:
            if mv % 5 == 0:
                vr_tz = pow5_factor(mv) >= q
            elif accept:
                vm_tz = pow5_factor(mv - 1 - mm_shift) >= q
            else:
                vp -= 1 if pow5_factor(mv + 2) >= q else 0
    else:
        q = log10pow5(-e2) - (1 if -e2 > 1 else 0)
        e10 = q + e2
        i = -e2 - q
        k = pow5bits(i) - POW5_BITCOUNT
        j = q - k
        mul = POW5[i]
        vr = mul_shift(4 * m2, mul, j)
        vp = mul_shift(4 * m2 + 2, mul, j)
        vm = mul_shift(4 * m2 - 1 - mm_shift, mul, j)
        if q <= 1:
            vr_tz = True
            if accept:
                vm_tz = mm_shift == 1
            else:
                vp -= 1
        elif q < 63:
            vr_tz = (mv & ((1 << q) - 1)) == 0
    removed = 0
    last = 0
    if vm_tz or vr_tz:
        while vp // 10 > vm // 10:
            vm_tz = vm_tz and vm % 10 == 0
            vr_tz = vr_tz and last == 0
            last = vr % 10
            vr //= 10
            vp //= 10
            vm //= 10
            removed += 1
        if vm_tz:
            while vm % 10 == 0:
                vr_tz = vr_tz and last == 0
                last = vr % 10
                vr //= 10
                vp //= 10
                vm //= 10
                removed += 1
        if vr_tz and last == 5 and vr % 2 == 0:
            last = 4
        out = vr + (1 if ((vr == vm and (not accept or not vm_tz)) or last >= 5) else 0)
    else:
        round_up = False
        if vp // 100 > vm // 100:
            round_up = vr % 100 >= 50
            vr //= 100
            vp //= 100
            vm //= 100
            removed += 2
        while vp // 10 > vm // 10:
            round_up = vr % 10 >= 5
            vr //= 10
            vp //= 10
            vm //= 10
            removed += 1
        out = vr + (1 if (vr == vm or round_up) else 0)
    return out, e10 + removed


def _numpy_digits(f):
    import numpy as np
    s = np.format_float_scientific(abs(f), unique=True, trim="-")
    mant, ex = s.split("e")
    dig = mant.replace(".", "")
    return int(dig), int(ex) - (len(dig) - 1)


def check(n):
    rnd = random.Random(1)
    bad = 0
    vals = [struct.unpack("<Q", struct.pack("<d", rnd.uniform(-1, 1) * 10 ** rnd.randint(-300, 300)))[0]
            for _ in range(n // 2)]
    vals += [rnd.getrandbits(63) for _ in range(n // 2)]
    vals += [1, 0x000FFFFFFFFFFFFF, 0x0010000000000000, 0x7FEFFFFFFFFFFFFF, 0x3FF0000000000000,
             0x4340000000000000, 0x3FB999999999999A]
    for b in vals:
        b &= (1 << 63) - 1
        if (b >> 52) == 0x7FF or b == 0:
            continue
        f = struct.unpack("<d", struct.pack("<Q", b))[0]
        got = d2d_model(b)
        want = _numpy_digits(f)
        if got != want:
            bad += 1
            if bad < 10:
                print("mismatch", hex(b), f, got, want)
    print("checked %d doubles, %d mismatches" % (len(vals), bad))
    return bad


def write_header(path):
    def row(x):
        return "{0x%016xull, 0x%016xull}" % (x & ((1 << 64) - 1), x >> 64)
    with open(path, "w") as f:
        f.write("// Generated by tools/gen_ryu_table.py -- do not edit.\n")
        f.write("// Ryu (Adams, PLDI 2018) power-of-5 tables, 125-bit: {low, high} 64-bit halves.\n")
        f.write("#pragma once\n#include <stdint.h>\n\nnamespace gd {\n\n")
        f.write("constexpr int kRyuPow5InvBits = %d, kRyuPow5Bits = %d;\n" % (POW5_INV_BITCOUNT, POW5_BITCOUNT))
        f.write("static __device__ const uint64_t kRyuPow5InvSplit[%d][2] = {\n" % N_POW5_INV)
        f.write(",\n".join("    " + row(x) for x in POW5_INV) + "};\n\n")
        f.write("static __device__ const uint64_t kRyuPow5Split[%d][2] = {\n" % N_POW5)
        f.write(",\n".join("    " + row(x) for x in POW5) + "};\n\n}  // namespace gd\n")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--check":
        sys.exit(1 if check(int(sys.argv[2])) else 0)
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kcp_amd", "csrc",
                       "ryu_tables.h")
    write_header(out)
    print(out)
