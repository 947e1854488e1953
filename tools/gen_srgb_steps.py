"""Derive tables/srgb_u8_steps.f64: the 255 steps of the reference's linear -> 8-bit channel map.

The reference turns a linear channel l into a byte with gamma_corrected (color.rs:93-101:
max(l, 0); 12.92 l on [0, 0.0031308], else 1.055 * l.powf(1/2.4) - 0.055) followed by
clamp_display_channel (main.rs:461-463: clamp to [0, 0.999], * 256, as u8). That composite is a
monotone step function of l, so it is fully described by its 255 steps:

    X_k = the least double l with byte(l) >= k,  k = 1..255,   byte(l) = #{k : l >= X_k}

This script finds each X_k by bisection over the bit patterns of the non-negative doubles, with
Python's math.pow — glibc's libm pow, the very function Rust's f64::powf calls on Linux. k_finalize
counts the steps at or below l (kernels.hip srgb_byte), so its RGBA8 output is the reference's
for every double, not just within a tolerance; tests/test_finalize_bytes.py re-derives the table
through the oracle's C chain and checks every double within 4096 ulps of every step.

    python tools/gen_srgb_steps.py            # rewrite tables/srgb_u8_steps.f64
    python tools/gen_srgb_steps.py --check    # exit 1 if the committed table differs
"""
import math
import struct
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
TABLE = ROOT / "tables" / "srgb_u8_steps.f64"


def display_byte(l):
    """gamma_corrected + clamp_display_channel of one channel, as the reference evaluates it."""
    if l != l:
        l = 0.0  # f64::max(NaN, 0.0) = 0.0
    l = max(l, 0.0)
    g = 12.92 * l if l <= 0.0031308 else 1.055 * math.pow(l, 1.0 / 2.4) - 0.055
    c = 0.0 if g != g else min(max(g, 0.0), 0.999)
    m = 256.0 * c
    return 255 if m >= 255.0 else int(m)


def _f(b):
    return struct.unpack("<d", struct.pack("<q", b))[0]


def steps():
    lo0, hi0 = 0, struct.unpack("<q", struct.pack("<d", math.inf))[0]
    out = []
    for k in range(1, 256):
        lo, hi = lo0, hi0  # byte(+0.0) = 0 < k <= 255 = byte(+inf)
        while hi - lo > 1:
            mid = (lo + hi) // 2
            if display_byte(_f(mid)) >= k:
                hi = mid
            else:
                lo = mid
        out.append(_f(hi))
    return out


def main():
    vals = steps()
    assert all(a < b for a, b in zip(vals, vals[1:])), "steps must be strictly increasing"
    raw = struct.pack("<255d", *vals)
    if "--check" in sys.argv:
        same = TABLE.exists() and TABLE.read_bytes() == raw
        print("srgb_u8_steps.f64", "matches" if same else "DIFFERS")
        sys.exit(0 if same else 1)
    TABLE.write_bytes(raw)
    print(f"wrote {TABLE} ({len(vals)} steps, X_1 = {vals[0]!r}, X_255 = {vals[-1]!r})")


if __name__ == "__main__":
    main()
