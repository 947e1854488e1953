"""Pin the oracle (CPU restatement) to the reference's own tests, fixtures and analytic answers.

Every check here is something the reference itself asserts or implies:
  - main.rs:808-828        sanitize_sample_xyz tests
  - color.rs:1988-2006     gamma_corrected tests
  - qbvh.rs:801-817        push_hit_children test
  - qbvh.rs:1168-1246      4-triangle hit fixture (closest = triangle 1, t = 0.954084586)
  - material.rs:178-185    SF66 Sellmeier coefficients -> published N-SF66 indices
  - color.rs:12            CIE_Y_INTERGAL vs the table sum
  - Random123              Philox4x32-10 known-answer vectors (the RNG both sides share)
"""
import ctypes as C
import math
import struct

import numpy as np
import pytest

import oracle_lib as O
from yart import abi


def _d3(*v):
    return (C.c_double * 3)(*v)


def test_sanitize_drops_non_finite_samples():  # main.rs:808-818
    for bad in (float("nan"), float("inf")):
        out = _d3(0, 0, 0)
        O.lib().oracle_sanitize_sample_xyz(_d3(bad, 1.0, 1.0), out)
        assert list(out) == [0.0, 0.0, 0.0]


def test_sanitize_clamps_luminance_preserving_chromaticity():  # main.rs:820-828
    out = _d3(0, 0, 0)
    O.lib().oracle_sanitize_sample_xyz(_d3(40.0, 80.0, 20.0), out)
    assert abs(out[1] - 20.0) < 1e-9
    assert abs(out[0] / out[1] - 40.0 / 80.0) < 1e-9
    assert abs(out[2] / out[1] - 20.0 / 80.0) < 1e-9
    # Y <= 0 passes through unchanged (main.rs:454)
    O.lib().oracle_sanitize_sample_xyz(_d3(5.0, -3.0, 7.0), out)
    assert list(out) == [5.0, -3.0, 7.0]


def test_gamma_clamps_negative_linear_channels():  # color.rs:1988-1997
    out = _d3(0, 0, 0)
    O.lib().oracle_gamma_corrected(_d3(-0.25, 0.18, -1.0), out)
    assert out[0] == 0.0 and out[2] == 0.0 and out[1] > 0.0
    assert all(math.isfinite(x) for x in out)


def test_gamma_linear_segment():  # color.rs:1999-2006
    out = _d3(0, 0, 0)
    O.lib().oracle_gamma_corrected(_d3(0.001, 0.002, 0.003), out)
    for got, want in zip(out, (0.01292, 0.02584, 0.03876)):
        assert abs(got - want) < 1e-6


def test_clamp_display_channel():  # main.rs:461-463
    f = O.lib().oracle_clamp_display_channel
    assert f(-1.0) == 0 and f(0.0) == 0 and f(0.5) == 128 and f(1.0) == 255 and f(0.999) == 255
    assert f(float("nan")) == 0


def test_push_hit_children_pushes_only_hit_lanes_in_order():  # qbvh.rs:801-817
    stack = (C.c_uint32 * 8)()
    children = (C.c_uint32 * 4)(10, 20, 30, 40)
    order = (C.c_uint32 * 4)(2, 0, 3, 1)
    hits = (C.c_int * 4)(1, 0, 1, 0)
    cursor = O.lib().oracle_push_hit_children(stack, 0, children, order, hits)
    assert cursor == 2 and stack[0] == 30 and stack[1] == 10


# qbvh.rs:1175-1235: the bench fixture's four triangles and ray.
FIXTURE_TRIS = [
    ([(-1.076726, -0.017016, 0.613202), (-1.117708, -0.041064, 0.593336), (-1.124824, -0.040218, 0.613324)],
     [(-0.578671, 0.815558, 0.00217971), (-0.439594, 0.864849, -0.242472), (-0.398821, 0.894699, -0.201137)]),
    ([(-1.076726, -0.017016, 0.613202), (-1.124824, -0.040218, 0.613324), (-1.07417, -0.017264, 0.633146)],
     [(-0.578671, 0.815558, 0.00217971), (-0.398821, 0.894699, -0.201137), (-0.540938, 0.840891, 0.0169749)]),
    ([(-1.074288, -0.017314, 0.593228), (-1.117708, -0.041064, 0.593336), (-1.076726, -0.017016, 0.613202)],
     [(-0.628594, 0.765563, -0.137049), (-0.439594, 0.864849, -0.242472), (-0.578671, 0.815558, 0.00217971)]),
    ([(-1.105662, -0.042332, 0.573312), (-1.117708, -0.041064, 0.593336), (-1.074288, -0.017314, 0.593228)],
     [(-0.471386, 0.817334, -0.331301), (-0.439594, 0.864849, -0.242472), (-0.628594, 0.765563, -0.137049)]),
]
FIXTURE_RAY = [-0.003898251, 2.0127985, 9.99872, -1.1280149, -2.129233, -9.836952]


def fixture_scene(reverse=False):
    b = O.DescBuilder()
    t = b.texture((0.5, 0.5, 0.5))
    m = b.material(abi.MAT_LAMBERTIAN, t)
    tris = list(reversed(FIXTURE_TRIS)) if reverse else FIXTURE_TRIS
    for v, n in tris:
        p = [c for vv in v for c in vv] + [c for nn in n for c in nn] + [0.0] * 6
        b.obj(abi.PRIM_TRIANGLE, m, p)
    return b


@pytest.mark.parametrize("reverse", [False, True])
def test_qbvh_fixture_known_answer(reverse):  # qbvh.rs:1168-1246, best and worst case order
    b = fixture_scene(reverse)
    s = O.OracleScene(b.desc())
    hits, obj = s.intersect(np.array(FIXTURE_RAY + [0.0, np.inf]))
    want_index = 2 if reverse else 1
    assert obj[0] == want_index
    assert abs(hits[0, 0] - 0.954084586) < 1e-9
    # every one of the four triangles is hit by this ray (the fixture's point)
    for i in range(4):
        one = O.DescBuilder()
        tx = one.texture((0.5, 0.5, 0.5))
        mm = one.material(abi.MAT_LAMBERTIAN, tx)
        v, n = FIXTURE_TRIS[i]
        one.obj(abi.PRIM_TRIANGLE, mm, [c for vv in v for c in vv] + [c for nn in n for c in nn] + [0.0] * 6)
        h, o = O.OracleScene(one.desc()).intersect(np.array(FIXTURE_RAY + [0.0, np.inf]))
        assert o[0] == 0
        assert abs(h[0, 0] - [0.954208725, 0.954084586, 0.954344529, 0.956675921][i]) < 1e-8


def test_qbvh_fixture_through_mesh_path():
    """The same four triangles inside a TriangleMesh (L4QBVH::hit) padded with far-away triangles
    (a mesh needs > 4 triangles: qbvh.rs:383-384)."""
    b = O.DescBuilder()
    m = b.material(abi.MAT_LAMBERTIAN, b.texture((0.5, 0.5, 0.5)))
    pos, nrm = [], []
    for v, n in FIXTURE_TRIS:
        pos.append([c for vv in v for c in vv])
        nrm.append([c for nn in n for c in nn])
    for k in range(5):  # padding far away
        pos.append([100 + k, 0, 0, 101 + k, 0, 0, 100 + k, 1, 0])
        nrm.append([0, 0, 1] * 3)
    # positions are f32 in a mesh (tobj); compare against f32-rounded triangles in a list
    mi = b.mesh(np.array(pos, dtype=np.float32), np.array(nrm))
    b.obj(abi.PRIM_MESH, m, mesh=mi)
    s = O.OracleScene(b.desc())
    hits, obj = s.intersect(np.array(FIXTURE_RAY + [0.0, np.inf]))
    ref = O.DescBuilder()
    rm = ref.material(abi.MAT_LAMBERTIAN, ref.texture((0.5, 0.5, 0.5)))
    for p, n in zip(pos[:4], nrm[:4]):
        ref.obj(abi.PRIM_TRIANGLE, rm, [float(np.float32(x)) for x in p] + list(n) + [0.0] * 6)
    h2, o2 = O.OracleScene(ref.desc()).intersect(np.array(FIXTURE_RAY + [0.0, np.inf]))
    assert obj[0] == 0 and o2[0] == 1
    assert hits[0, 0] == h2[0, 0]
    np.testing.assert_array_equal(hits[0, 1:4], h2[0, 1:4])


SF66_B = (2.0245976, 0.470187196, 2.59970433)
SF66_C = (0.0147053225 * 1e6, 0.0692998276 * 1e6, 161.817601 * 1e6)


@pytest.mark.parametrize("wl,n", [(360.0, 2.071760), (400.0, 2.014043), (486.13, 1.954587), (587.56, 1.922860),
                                  (656.27, 1.910387), (719.99, 1.902129)])
def test_sf66_sellmeier_index(wl, n):  # material.rs:178-185, 251-257 (N-SF66 nd = 1.92286)
    got = O.lib().oracle_sellmeier_index(_d3(*SF66_B), _d3(*SF66_C), wl)
    assert abs(got - n) < 5e-7


def test_cie_tables_and_integral(repo):  # color.rs:12, 286-1709
    raw = (repo / "tables" / "cie1931_xyz_1nm_360_830.f64").read_bytes()
    cie = np.frombuffer(raw, dtype="<f8").reshape(471, 3)
    assert abs(cie[:, 1].sum() - 106.856895) < 1e-3
    out = _d3(0, 0, 0)
    O.lib().oracle_xyz_from_wavelength(555.9, out)  # index (555.9 - 360) as isize = 195
    assert list(out) == list(cie[195])
    O.lib().oracle_xyz_from_wavelength(359.5, out)  # -0.5 as isize = 0 (truncation)
    assert list(out) == list(cie[0])
    O.lib().oracle_xyz_from_wavelength(831.0, out)  # index 471 -> out of table -> 0
    assert list(out) == [0.0, 0.0, 0.0]


def test_smits_spectrum_of_white_and_primaries(repo):  # color.rs:54-90
    raw = (repo / "tables" / "smits_basis_36bin.f64").read_bytes()
    smits = np.frombuffer(raw, dtype="<f8").reshape(7, 36)
    f = O.lib().oracle_rgb_reflect
    for i in range(36):
        wl = 360.0 + 10.0 * i + 5.0
        assert f(_d3(1.0, 1.0, 1.0), wl) == smits[0, i]          # white
        assert f(_d3(0.0, 0.0, 1.0), wl) == smits[6, i]          # blue (red<=green<=blue)
        assert f(_d3(1.0, 0.0, 0.0), wl) == smits[4, i]          # red
    assert f(_d3(0.5, 0.5, 0.5), 300.0) == 0.5 * smits[0, 0]     # clamped to bin 0
    assert f(_d3(0.5, 0.5, 0.5), 900.0) == 0.5 * smits[0, 35]    # clamped to bin 35


def test_philox_random123_known_answers():
    """Philox4x32-10 KAT vectors from Random123's kat_vectors."""
    f = O.lib().oracle_philox4x32_10
    cases = [
        ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
        ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
        ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
         (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
    ]
    for ctr, key, want in cases:
        out = (C.c_uint32 * 4)()
        f((C.c_uint32 * 4)(*ctr), (C.c_uint32 * 2)(*key), out)
        assert tuple(out) == want


def test_rng_stream_is_uniform_and_deterministic():
    a = O.rng_f64(7, 123, 4, 20000)
    b = O.rng_f64(7, 123, 4, 20000)
    np.testing.assert_array_equal(a, b)
    assert a.min() >= 0.0 and a.max() < 1.0
    assert abs(a.mean() - 0.5) < 0.01
    c = O.rng_f64(7, 123, 5, 16)
    assert not np.array_equal(a[:16], c)
    # gen::<f64>() keeps 53 bits: every value is a multiple of 2^-53
    assert np.all(np.floor(a * 2.0**53) == a * 2.0**53)


def test_gen_range_within_bounds():
    f = O.lib().oracle_gen_range_f64
    vals = [f(1, p, 0, 360.0, 720.0) for p in range(5000)]
    assert min(vals) >= 360.0 and max(vals) < 720.0
    assert abs(np.mean(vals) - 540.0) < 5.0


def test_sin_cos_within_one_ulp_of_libm():
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.uniform(0.0, 2 * math.pi, 20000), rng.uniform(-200.0, 200.0, 20000),
                         rng.uniform(-1e4, 1e4, 5000), [0.0, 1e-300, -0.0, math.pi, math.pi / 2, 2 * math.pi]])
    L = O.lib()
    worst = 0
    for x in xs:
        for mine, ref in ((L.oracle_sin(x), math.sin(x)), (L.oracle_cos(x), math.cos(x))):
            if mine == ref:
                continue
            ulp = abs(struct.unpack("<q", struct.pack("<d", mine))[0] - struct.unpack("<q", struct.pack("<d", ref))[0])
            worst = max(worst, ulp)
    assert worst <= 1


def _ulps(a, b):
    return abs(struct.unpack("<q", struct.pack("<d", a))[0] - struct.unpack("<q", struct.pack("<d", b))[0])


def test_libm_twins_against_this_hosts_glibc_on_the_draw_domains():
    """What the fdlibm twins (oracle.c = kernels.hip, bitwise) differ by from the libm the reference
    links on Linux (glibc; Rust's f64::sin / cos / ln / acos / atan2 call it), on the inputs the path
    feeds them: sin / cos of 2 pi r (cosine and sphere-light sampling), ln of a uniform draw
    (ConstantMedium's free path), acos / atan2 of unit-vector components (sphere uv). At most 1 ulp
    everywhere; the share of values that differ, measured with this container's glibc 2.35 (which is
    itself not correctly rounded on 0.24 % of the sin / cos inputs), is what DESIGN.md §2 states:
    sin / cos ~3 %, ln ~7 %, acos ~8 %, atan2 ~18 %. The reference's own generator is unseedable, so
    these last-ulp differences sit far inside the statistical comparison (test_statistical.py)."""
    rng = np.random.default_rng(11)
    L = O.lib()
    n = 40000
    r = rng.integers(0, 1 << 53, n, dtype=np.int64).astype(np.float64) * 2.0 ** -53
    shares = {}
    for name, cases in (
            ("sin", [(L.oracle_sin(2.0 * math.pi * x), math.sin(2.0 * math.pi * x)) for x in r]),
            ("cos", [(L.oracle_cos(2.0 * math.pi * x), math.cos(2.0 * math.pi * x)) for x in r]),
            ("ln", [(L.oracle_log(1.0 - x), math.log(1.0 - x)) for x in r]),
            ("acos", [(L.oracle_acos(2.0 * x - 1.0), math.acos(2.0 * x - 1.0)) for x in r])):
        ulps = [_ulps(a, b) for a, b in cases]
        assert max(ulps) <= 1, name
        shares[name] = sum(u != 0 for u in ulps) / n
    yx = rng.uniform(-1.0, 1.0, (n, 2))
    ulps = [_ulps(L.oracle_atan2(y, x), math.atan2(y, x)) for y, x in yx]
    assert max(ulps) <= 1
    shares["atan2"] = sum(u != 0 for u in ulps) / n
    assert 0.01 < shares["sin"] < 0.06 and 0.01 < shares["cos"] < 0.06, shares
    assert shares["ln"] < 0.12 and shares["acos"] < 0.12 and shares["atan2"] < 0.25, shares


def test_coverage_skips_row_224_of_a_225_row_image():  # main.rs:643-646
    m = O.coverage(400, 225)
    assert m[:224].all() and not m[224].any()
    m2 = O.coverage(1003, 16)  # W*col/8 vs col*(W/8) leaves interior columns unsampled
    assert not m2[:, 375].any() and m2[:, 374].all()
    assert O.coverage(800, 800).all()


@pytest.mark.parametrize("scene,w,h,spp", [("cornell-box", 24, 24, 8), ("random-scene", 24, 16, 4), ("david", 16, 9, 2)])
def test_recursive_and_iterative_integrators_agree(scene, w, h, spp):
    """ray_reflectance as the reference writes it (main.rs:537-588: recursion, att * R' * spdf / pdf
    on the way back) against the front-to-back loop the oracle and the kernel run
    (T <- ((T * att) * spdf) / pdf, terminal value last). Same draws, same hits: the two differ only
    by the association of the throughput product, a few ulps per bounce (<= 50 bounces), never
    more. Measured: <= 3.3e-15 relative per pixel sum; 62-94 % of the sums are bit-identical."""
    import yart
    p = yart.Preset(scene)
    cam, prm = p.camera(w, h), yart.render_params(w, h, spp, 50)
    o = O.OracleScene(p.desc)
    it = o.render(cam, prm, threads=8)
    rec = o.render(cam, prm, threads=8, recursive=True)
    nz = it != 0
    assert (rec[~nz] == 0).all()
    rel = np.abs(it - rec)[nz] / np.abs(it)[nz]
    assert rel.max() <= 50 * 2 * 2.0 ** -52, rel.max()
    assert (it == rec).mean() > 0.5
