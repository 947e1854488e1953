"""k_finalize's 8-bit output equals the reference's for EVERY double (CPU, no GPU needed).

The reference turns each linear channel l into a byte with gamma_corrected (color.rs:93-101:
max(l, 0); 12.92 l up to 0.0031308, else 1.055 * l.powf(1/2.4) - 0.055, glibc's pow) and
clamp_display_channel (main.rs:461-463). The device has no glibc pow, and the vendor's differs in
the last ulp (an fdlibm twin does too: it was tried and disagrees with glibc on ~55 doubles at the
byte steps). So k_finalize does not evaluate pow at all: it counts the steps at or below l in
tables/srgb_u8_steps.f64, X_k = the least double whose reference byte is >= k (k = 1..255),
derived with glibc's pow by tools/gen_srgb_steps.py. Proof that the count is the reference's byte:

* the table is exactly the reference map's steps: byte(X_k) >= k > byte(X_k - 1 ulp), evaluated
  by the oracle's C chain (oracle.c gamma_channel with glibc's pow + clamp_display_channel);
* every double within 4096 ulps of every step (and of the 0.0031308 branch edge) is compared
  exhaustively;
* away from the steps the reference map is monotone: on the linear segment exactly (one
  multiplication), on the pow segment because glibc's pow is within 1 ulp of x^(1/2.4) (0.52 ulp
  measured below against 200-bit mpmath) and at every window edge the exact power is more than
  64 ulps from the pow value P_k at which the byte steps. So outside the windows the reference
  byte is #{k : l >= X_k}, which is what the table gives.

GPU side (test_gpu_parity.py): the device's byte function over these windows, k_finalize on
rendered frames and on all five BASELINE configs, array_equal with the oracle.
"""
import math
import struct
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib as O

Y = 1.0 / 2.4
EDGE = 0.0031308  # color.rs:95
WIN = 4096


def steps():
    raw = (O.REPO / "tables" / "srgb_u8_steps.f64").read_bytes()
    return np.frombuffer(raw, dtype="<f8").astype(np.float64)


def table_bytes(linear):
    """The device's rule (kernels.hip srgb_byte): the number of steps at or below the value."""
    x = np.asarray(linear, dtype=np.float64)
    n = np.searchsorted(steps(), x, side="right")
    return np.where(np.isnan(x), 0, n).astype(np.uint8)


def _bits(x):
    return struct.unpack("<q", struct.pack("<d", x))[0]


def _u_of_p(p):
    """clamp_display_channel(1.055 * p - 0.055): the byte as a function of the pow value."""
    c = 1.055 * np.asarray(p, dtype=np.float64) - 0.055
    c = np.where(np.isnan(c), 0.0, np.clip(c, 0.0, 0.999))
    return np.minimum(np.floor(256.0 * c), 255).astype(np.int64)


def test_committed_table_is_rederived_by_its_generator():
    r = subprocess.run([sys.executable, str(O.REPO / "tools" / "gen_srgb_steps.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_table_holds_exactly_the_reference_steps():
    T = steps()
    assert T.shape == (255,) and (np.diff(T) > 0).all()
    at = O.display_bytes(T)
    below = O.display_bytes(np.nextafter(T, -np.inf))
    k = np.arange(1, 256)
    assert (at >= k).all() and (below < k).all()


def test_byte_equals_reference_in_every_step_window():
    T = steps()
    centres = [_bits(float(t)) for t in T] + [_bits(EDGE)]
    win = np.concatenate([np.arange(c - WIN, c + WIN + 1, dtype=np.int64) for c in centres]).view(np.float64)
    ref, dev = O.display_bytes(win), table_bytes(win)
    bad = np.flatnonzero(ref != dev)
    assert len(bad) == 0, f"{len(bad)} doubles differ, e.g. {win[bad[:4]].tolist()}"
    # the windows step monotonically under the reference map, too
    for c in centres:
        seg = O.display_bytes(np.arange(c - WIN, c + WIN + 1, dtype=np.int64).view(np.float64))
        assert (np.diff(seg.astype(int)) >= 0).all()


def test_pow_segment_window_edges_are_far_from_the_pow_steps():
    """The margin the proof needs outside the windows (see the module docstring)."""
    hi = _bits(2.0)
    for k, xk in enumerate(steps(), start=1):
        if xk <= EDGE:
            continue  # linear segment: one multiplication, exactly monotone
        lo_b, hi_b = 0, hi
        while hi_b - lo_b > 1:  # P_k: the least pow value whose byte is >= k
            mid = (lo_b + hi_b) // 2
            if _u_of_p(struct.unpack("<d", struct.pack("<q", mid))[0]) >= k:
                hi_b = mid
            else:
                lo_b = mid
        pk = struct.unpack("<d", struct.pack("<q", hi_b))[0]
        for e in (_bits(float(xk)) - WIN, _bits(float(xk)) + WIN):
            x = struct.unpack("<d", struct.pack("<q", e))[0]
            if x > EDGE:
                assert abs(math.pow(x, Y) - pk) > 64 * math.ulp(pk), (k, x)


def test_glibc_pow_is_within_one_ulp_of_exact():
    mpmath = pytest.importorskip("mpmath")
    mpmath.mp.prec = 200
    rng = np.random.default_rng(21)
    worst = 0.0
    for x in np.concatenate([rng.uniform(EDGE, 1.0, 4000), 10.0 ** rng.uniform(0, 3, 500)]):
        ex = mpmath.power(mpmath.mpf(float(x)), mpmath.mpf(Y))
        worst = max(worst, float(abs(mpmath.mpf(math.pow(float(x), Y)) - ex) / math.ulp(float(ex))))
    assert worst < 0.55, worst


def test_byte_equals_reference_on_random_and_special_values():
    rng = np.random.default_rng(22)
    lin = np.concatenate([rng.uniform(-0.1, 1.2, 3_000_000), 10.0 ** rng.uniform(-320, 308, 500_000),
                          -(10.0 ** rng.uniform(-320, 308, 10_000)),
                          [0.0, -0.0, EDGE, np.nextafter(EDGE, 1), np.inf, -np.inf, np.nan, 5e-324, 1.0, 2.0]])
    with np.errstate(all="ignore"):
        np.testing.assert_array_equal(table_bytes(lin), O.display_bytes(lin))
