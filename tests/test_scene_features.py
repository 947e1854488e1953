"""Known answers for the scene features of SURVEY §8f rank 1 that this build adds to the hot path:
NoiseTexture / Perlin (texture.rs:84-300), ConstantMedium + Isotropic (hittable.rs:258-326,
material.rs:357-381), and the deterministic natural log they need. CPU only (the oracle)."""
import math

import numpy as np
import pytest

import oracle_lib as O
import yart
from yart import abi


def test_log_within_one_ulp_of_libm_and_special_values():
    L = O.lib()
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.uniform(0, 1, 20000), 10.0 ** rng.uniform(-300, 300, 20000),
                         rng.uniform(0.999, 1.001, 2000), [2.0 ** -1074, 5e-324 * 3, 1.0, 2.0, 0.5]])
    for x in xs:
        got, want = L.oracle_log(float(x)), math.log(float(x))
        assert got == want or abs(got - want) <= abs(math.ulp(want)), (x, got, want)
    assert L.oracle_log(0.0) == -math.inf and L.oracle_log(1.0) == 0.0
    assert math.isnan(L.oracle_log(-1.0)) and L.oracle_log(math.inf) == math.inf


def _noise_scene(noise_type, scale):
    b = O.DescBuilder()
    t = b.noise_texture(noise_type, scale)
    m = b.material(abi.MAT_LAMBERTIAN, t)
    b.obj(abi.PRIM_SPHERE, m, (0.0, 0.0, 0.0, 1.0))
    d = b.desc()
    perlin = b.textures[t].perlin.contents
    return O.OracleScene(d), t, perlin


def _white(wl):
    return O.lib().oracle_rgb_reflect((O.C.c_double * 3)(1.0, 1.0, 1.0), wl)


def _perm(P, i, j, k):
    return P.perm_x[i & 255] ^ P.perm_y[j & 255] ^ P.perm_z[k & 255]


def test_noise_smooth_vanishes_on_the_lattice():
    """perlin_interp at integer points: u = v = w = 0, every weight vector is (0 - di, ...), so
    only the (0,0,0) corner has weight 1 and its dot product is with (0,0,0): noise = 0 and the
    texture is white * 0.5 exactly (texture.rs:209-228, 290-296)."""
    s, t, _ = _noise_scene(abi.NOISE_SMOOTH, 1.0)
    for p in [(0, 0, 0), (3, -7, 12), (-100, 5, 255)]:
        assert s.texture(t, 500.0, np.array(p, float)) == _white(500.0) * 0.5 * (1.0 + 0.0)


def test_noise_trilinear_reads_the_corner_value_on_the_lattice():
    s, t, P = _noise_scene(abi.NOISE_TRILINEAR, 1.0)
    for p in [(0, 0, 0), (4, 9, -3), (-1, -1, -1)]:
        c = P.ranfloat[_perm(P, p[0], p[1], p[2])]
        # (0*u + 1*(1-u)) products are exactly 1 at the corner; the others multiply by 0
        assert s.texture(t, 450.0, np.array(p, float)) == _white(450.0) * 0.5 * (1.0 + c)


def test_noise_square_hashes_four_times_the_point():
    s, t, P = _noise_scene(abi.NOISE_SQUARE, 2.0)
    p = np.array([0.3, -1.7, 12.9])
    q = p * 2.0
    i, j, k = (int(math.trunc(4.0 * q[0])) & 255, int(math.trunc(4.0 * q[1])) & 255, int(math.trunc(4.0 * q[2])) & 255)
    assert s.texture(t, 600.0, p) == _white(600.0) * 0.5 * (1.0 + P.ranfloat[P.perm_x[i] ^ P.perm_y[j] ^ P.perm_z[k]])


def test_noise_marble_matches_a_restatement():
    """Marble (texture.rs:280-288) = white * 0.5 * (1 + sin(scale * p.z + 10 * turb(p, 7))), with
    turb the 7-octave |sum| of the smooth noise; restated here in numpy for random points."""
    s, t, P = _noise_scene(abi.NOISE_MARBLE, 4.0)
    rv = np.array([[P.ranvec[i][k] for k in range(3)] for i in range(256)])

    def noise(p):
        f = np.floor(p)
        u, v, w = p - f
        i, j, k = (int(x) for x in f)
        uu, vv, ww = u * u * (3.0 - 2.0 * u), v * v * (3.0 - 2.0 * v), w * w * (3.0 - 2.0 * w)
        acc = 0.0
        for di in range(2):
            for dj in range(2):
                for dk in range(2):
                    c = rv[_perm(P, i + di, j + dj, k + dk)]
                    wv = (u - di, v - dj, w - dk)
                    acc += ((di * uu + (1.0 - di) * (1.0 - uu)) * (dj * vv + (1.0 - dj) * (1.0 - vv)) *
                            (dk * ww + (1.0 - dk) * (1.0 - ww)) * (wv[0] * c[0] + wv[1] * c[1] + wv[2] * c[2]))
        return acc

    def turb(p):
        acc, wgt = 0.0, 1.0
        for _ in range(7):
            acc += wgt * noise(p)
            wgt *= 0.5
            p = p * 2.0
        return abs(acc)

    rng = np.random.default_rng(3)
    for p in rng.uniform(-20, 20, (50, 3)):
        want = _white(520.0) * 0.5 * (1.0 + math.sin(4.0 * p[2] + 10.0 * turb(p)))
        assert abs(s.texture(t, 520.0, p) - want) <= 1e-12 * max(1.0, abs(want))  # sin: libm vs fdlibm


def _medium_scene(density):
    b = O.DescBuilder()
    m = b.material(abi.MAT_ISOTROPIC, b.texture((1.0, 1.0, 1.0)))
    b.obj(abi.PRIM_BOX, m, (0.0, 0.0, 0.0, 1.0, 1.0, 1.0), xforms=[(abi.XF_MEDIUM, (density, 0.0, 0.0))])
    return b.desc()


@pytest.mark.parametrize("density", [0.3, 0.7, 2.5])
def test_constant_medium_free_path_is_exponential(density):
    """Rays crossing a unit slab of the medium scatter with probability 1 - exp(-density · L)
    (hittable.rs:299-316), each query drawing its own exponential free path."""
    d = _medium_scene(density)
    n = 40000
    rays = np.zeros((n, 8))
    rays[:, 0] = -1.0
    rays[:, 1:3] = np.random.default_rng(2).uniform(0.1, 0.9, (n, 2))
    rays[:, 3] = 1.0  # +x through the box: inside length 1
    rays[:, 6], rays[:, 7] = 0.001, np.inf
    h, o = O.OracleScene(d).intersect(rays)
    frac = (o >= 0).mean()
    want = 1.0 - math.exp(-density)
    assert abs(frac - want) < 5 * math.sqrt(want * (1 - want) / n)
    hit = o >= 0
    np.testing.assert_array_equal(h[hit, 4:7], np.tile([1.0, 0.0, 0.0], (hit.sum(), 1)))  # normal (1,0,0)
    assert (h[hit, 7] == 1.0).all()  # front_face
    assert ((h[hit, 0] >= 1.0) & (h[hit, 0] <= 2.0)).all()  # inside the box


def test_smoke_preset_flattens_two_media():
    p = yart.Preset("cornell-box-smoke")
    d = p.desc.contents
    assert (p.defaults.width, p.defaults.height, p.defaults.samples_per_pixel) == (600, 600, 200)
    media = [d.objects[i] for i in range(d.n_objects) if d.objects[i].n_xforms and d.objects[i].xforms[0].kind == abi.XF_MEDIUM]
    assert len(media) == 2 and d.n_objects == 8 and d.n_lights == 0
    for m in media:
        assert m.kind == abi.PRIM_BOX and m.xforms[0].v[0] == 0.01
        assert [m.xforms[1].kind, m.xforms[2].kind] == [abi.XF_TRANSLATE, abi.XF_ROTATE_Y]
        assert d.materials[m.material].kind == abi.MAT_ISOTROPIC
    albedo = sorted(tuple(d.textures[d.materials[m.material].texture].rgb) for m in media)
    assert albedo == [(0.0, 0.0, 0.0), (1.0, 1.0, 1.0)]


def test_perlin_presets_draw_two_table_sets():
    p = yart.Preset("two-perlin-spheres")
    d = p.desc.contents
    texs = [d.textures[d.materials[d.objects[i].material].texture] for i in range(d.n_objects)]
    assert all(t.kind == abi.TEX_NOISE and t.noise_type == abi.NOISE_MARBLE and t.scale == 4.0 for t in texs)
    P0, P1 = texs[0].perlin.contents, texs[1].perlin.contents
    for P in (P0, P1):
        for name in ("perm_x", "perm_y", "perm_z"):
            assert sorted(getattr(P, name)) == list(range(256))
        assert all(0.0 <= P.ranfloat[i] < 1.0 for i in range(256))
        assert all(-1.0 <= P.ranvec[i][k] < 1.0 for i in range(256) for k in range(3))
    assert list(P0.perm_x) != list(P1.perm_x)  # each NoiseTexture::new draws its own tables
    sl = yart.Preset("simple-light").desc.contents
    assert sl.n_objects == 3 and sl.objects[2].kind == abi.PRIM_XY_RECT


# ---- ImageTexture (texture.rs:302-345) and get_sphere_uv's acos / atan2 (sphere.rs:213-220)
def test_acos_atan2_within_one_ulp_of_libm_and_exact_specials():
    L = O.lib()
    rng = np.random.default_rng(8)
    for x in np.concatenate([rng.uniform(-1, 1, 30000), [1.0, -1.0, 0.0, -0.0, 0.5, -0.5, 1e-300]]):
        got, want = L.oracle_acos(float(x)), math.acos(float(x))
        assert got == want or abs(got - want) <= math.ulp(want), (x, got, want)
    ys, xs = rng.normal(size=(2, 30000)) * 10.0 ** rng.uniform(-5, 5, (2, 30000))
    for y, x in zip(ys, xs):
        got, want = L.oracle_atan2(float(y), float(x)), math.atan2(float(y), float(x))
        assert got == want or abs(got - want) <= math.ulp(want), (y, x, got, want)
    for y, x in [(0.0, 1.0), (-0.0, 1.0), (0.0, -1.0), (-0.0, -1.0), (1.0, 0.0), (-1.0, 0.0), (math.inf, math.inf)]:
        got, want = L.oracle_atan2(y, x), math.atan2(y, x)
        assert got == want and math.copysign(1, got) == math.copysign(1, want)


def test_image_texture_texel_lookup():
    b = O.DescBuilder()
    img = np.random.default_rng(9).integers(0, 256, (8, 16, 3), dtype=np.uint8)
    t = b.image_texture(img)
    m = b.material(abi.MAT_LAMBERTIAN, t)
    b.obj(abi.PRIM_SPHERE, m, (0.0, 0.0, 0.0, 1.0))
    s = O.OracleScene(b.desc())
    L = O.lib()
    p0 = np.zeros(3)

    def want(i, j, wl):
        rgb = (O.C.c_double * 3)(*[(1.0 / 255.0) * float(c) for c in img[j, i]])
        return L.oracle_rgb_reflect(rgb, wl)

    # u -> column i = floor(u * W); v is flipped: row j = floor((1 - v) * H); both clamp
    for u, v, i, j in [(0.0, 1.0, 0, 0), (0.25, 0.75, 4, 2), (0.999, 0.001, 15, 7), (1.0, 0.0, 15, 7),
                       (1.5, -0.5, 15, 7), (-3.0, 2.0, 0, 0), (math.nan, math.nan, 0, 0)]:
        assert s.texture(t, 480.0, p0, u, v) == want(i, j, 480.0), (u, v)


def test_earth_preset_uses_the_decoded_map():
    p = yart.Preset("earth")
    d = p.desc.contents
    assert d.n_objects == 1 and list(d.objects[0].p[:4]) == [0.0, 0.0, 0.0, 2.0]
    t = d.textures[d.materials[d.objects[0].material].texture]
    assert (t.kind, t.width, t.height) == (abi.TEX_IMAGE, 1024, 512)
    assert list(p.defaults.lookfrom) == [13.0, 2.0, 3.0]


# ---- MovingSphere (sphere.rs:121-211)
def moving_scene(with_glass=True):
    b = O.DescBuilder(background=(0.7, 0.8, 1.0))
    red = b.material(abi.MAT_LAMBERTIAN, b.texture((0.7, 0.3, 0.1)))
    ground = b.material(abi.MAT_LAMBERTIAN, b.texture((0.5, 0.5, 0.5)))
    b.obj(abi.PRIM_SPHERE, ground, (0.0, -1000.0, 0.0, 1000.0))
    for k in range(5):  # centre0 -> centre1 over time 0..1, as the book's bouncing spheres
        c0 = (-4.0 + 2.0 * k, 0.5, 0.0)
        b.obj(abi.PRIM_MOVING_SPHERE, red, c0 + (c0[0], 0.5 + 0.4 * k, 0.0, 0.0, 1.0, 0.5))
    if with_glass:
        glass = b.material(abi.MAT_DIELECTRIC, 0, b=(1.03961212, 0.231792344, 1.01046945),
                           c=(6000.69867, 20017.9144, 103560653.0))
        b.obj(abi.PRIM_MOVING_SPHERE, glass, (0.0, 1.5, 2.0, 0.0, 1.5, 2.5, 0.0, 1.0, -0.8))
    return b


def test_moving_sphere_at_time0_hits_like_a_still_sphere():
    """Intersect rays carry time 0: a moving sphere is then its centre0 sphere; from outside its
    ray-facing normal is the outward one, as StillSphere's."""
    bm, bs = O.DescBuilder(), O.DescBuilder()
    mm = bm.material(abi.MAT_LAMBERTIAN, bm.texture((0.5, 0.5, 0.5)))
    ms = bs.material(abi.MAT_LAMBERTIAN, bs.texture((0.5, 0.5, 0.5)))
    bm.obj(abi.PRIM_MOVING_SPHERE, mm, (1.0, 2.0, 3.0, 9.0, 9.0, 9.0, 0.0, 1.0, 1.5))
    bs.obj(abi.PRIM_SPHERE, ms, (1.0, 2.0, 3.0, 1.5))
    rng = np.random.default_rng(10)
    n = 20000
    o = rng.uniform(-10, 10, (n, 3))
    o = o[np.linalg.norm(o - [1, 2, 3], axis=1) > 2.0][:5000]
    d = np.array([1.0, 2.0, 3.0]) + rng.uniform(-1.6, 1.6, (len(o), 3)) - o
    rays = np.concatenate([o, d, np.full((len(o), 1), 0.001), np.full((len(o), 1), np.inf)], axis=1)
    h1, o1 = O.OracleScene(bm.desc()).intersect(rays)
    h2, o2 = O.OracleScene(bs.desc()).intersect(rays)
    np.testing.assert_array_equal(o1, o2)
    assert (o1 >= 0).mean() > 0.5
    np.testing.assert_array_equal(h1[o1 >= 0], h2[o2 >= 0])


def test_moving_spheres_blur_along_their_path():
    """The shutter time is drawn per sample once a MovingSphere is present (camera.rs:91): a sphere
    moving in y smears over its path, so the render differs from the time-0 scene."""
    b = moving_scene(with_glass=False)
    d = b.desc()
    cam = yart.make_camera((0.0, 2.0, 12.0), (0.0, 1.0, 0.0), 40.0, 48 / 32, 0.0, 10.0)
    img = O.OracleScene(d).render(cam, yart.render_params(48, 32, 8, 8))
    assert np.isfinite(img).all() and img.mean() > 0
