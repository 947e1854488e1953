"""ctypes access to oracle/liboracle.so — TEST INFRASTRUCTURE (the checker, never the product)."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "yet-another-raytracer_amd"))
from yart import abi  # noqa: E402

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    path = REPO / "oracle" / "liboracle.so"
    if not path.exists():
        raise FileNotFoundError(f"{path} not built; run `make oracle`")
    L = C.CDLL(str(path))
    P, U32, U64, D, I = C.c_void_p, C.c_uint32, C.c_uint64, C.c_double, C.c_int
    sigs = {
        "oracle_scene_create": (I, [C.POINTER(abi.SceneDesc), C.POINTER(P)]),
        "oracle_scene_destroy": (None, [P]),
        "oracle_qbvh_stats": (I, [P, U32, C.POINTER(U32), C.POINTER(U32), C.POINTER(U32)]),
        "oracle_render": (I, [P, C.POINTER(abi.Camera), C.POINTER(abi.RenderParams), P, I, I]),
        "oracle_finalize_rgba8": (I, [P, U32, U32, U32, P]),
        "oracle_intersect": (I, [P, P, U32, P, P]),
        "oracle_coverage": (I, [U32, U32, P]),
        "oracle_sanitize_sample_xyz": (None, [P, P]),
        "oracle_clamp_display_channel": (C.c_uint8, [D]),
        "oracle_gamma_corrected": (None, [P, P]),
        "oracle_xyz_into_rgb": (None, [P, P]),
        "oracle_xyz_from_wavelength": (None, [D, P]),
        "oracle_rgb_reflect": (D, [P, D]),
        "oracle_sellmeier_index": (D, [P, P, D]),
        "oracle_schlick": (D, [D, D]),
        "oracle_push_hit_children": (I, [P, I, P, P, P]),
        "oracle_rng_f64": (None, [U64, U32, U32, U32, P]),
        "oracle_philox4x32_10": (None, [P, P, P]),
        "oracle_gen_range_f64": (D, [U64, U32, U32, D, D]),
        "oracle_sin": (D, [D]),
        "oracle_cos": (D, [D]),
        "oracle_log": (D, [D]),
        "oracle_texture_probe": (D, [P, U32, D, P, D, D]),
        "oracle_acos": (D, [D]),
        "oracle_atan2": (D, [D, D]),
        "oracle_display_bytes": (None, [P, C.c_size_t, P]),
        "oracle_obj_count": (I, [C.c_char_p, C.POINTER(U32)]),
        "oracle_obj_load": (I, [C.c_char_p, P, P, P, U32]),
    }
    for name, (res, args) in sigs.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _p(a):
    return C.c_void_p(a.ctypes.data)


class OracleScene:
    def __init__(self, desc):
        self._s = C.c_void_p()
        rc = lib().oracle_scene_create(desc, C.byref(self._s))
        if rc != 0:
            raise RuntimeError(f"oracle_scene_create failed: {rc}")

    def __del__(self):
        if getattr(self, "_s", None):
            lib().oracle_scene_destroy(self._s)

    def qbvh_stats(self, m=0):
        n, l, d = C.c_uint32(), C.c_uint32(), C.c_uint32()
        rc = lib().oracle_qbvh_stats(self._s, m, C.byref(n), C.byref(l), C.byref(d))
        assert rc == 0
        return n.value, l.value, d.value

    def render(self, cam, params, threads=0, recursive=False, chacha=False):
        out = np.zeros((params.height, params.width, 3), dtype=np.float64)
        rc = lib().oracle_render(self._s, C.byref(cam), C.byref(params), _p(out), threads,
                                  (1 if recursive else 0) | (2 if chacha else 0))
        assert rc == 0
        return out

    def texture(self, tex, wl, p, u=0.0, v=0.0):
        pt = np.ascontiguousarray(p, dtype=np.float64)
        return lib().oracle_texture_probe(self._s, tex, wl, _p(pt), u, v)

    def intersect(self, rays):
        rays = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 8)
        n = rays.shape[0]
        hits = np.empty((n, 8), dtype=np.float64)
        obj = np.empty(n, dtype=np.int32)
        assert lib().oracle_intersect(self._s, _p(rays), n, _p(hits), _p(obj)) == 0
        return hits, obj


def load_obj(path):
    """The oracle's own OBJ reader (oracle_obj.c): positions (n, 9) f32, normals (n, 9) and uvs
    (n, 6) f64."""
    L = lib()
    n = C.c_uint32()
    rc = L.oracle_obj_count(str(path).encode(), C.byref(n))
    assert rc == 0, rc
    pos = np.zeros((n.value, 9), np.float32)
    nrm = np.zeros((n.value, 9), np.float64)
    uv = np.zeros((n.value, 6), np.float64)
    rc = L.oracle_obj_load(str(path).encode(), _p(pos), _p(nrm), _p(uv), n.value)
    assert rc == 0, rc
    return pos, nrm, uv


def finalize(xyz_sum, spp):
    h, w, _ = xyz_sum.shape
    x = np.ascontiguousarray(xyz_sum, dtype=np.float64)
    out = np.zeros((h, w, 4), dtype=np.uint8)
    assert lib().oracle_finalize_rgba8(_p(x), w, h, spp, _p(out)) == 0
    return out


def display_bytes(linear):
    """The reference's 8-bit channel of each linear value (gamma_channel with glibc's pow, then
    clamp_display_channel)."""
    x = np.ascontiguousarray(linear, dtype=np.float64)
    out = np.empty(x.shape, dtype=np.uint8)
    lib().oracle_display_bytes(_p(x), x.size, _p(out))
    return out


def coverage(w, h):
    m = np.zeros((h, w), dtype=np.uint8)
    lib().oracle_coverage(w, h, _p(m))
    return m.astype(bool)


def rng_f64(seed, pixel, sample, n):
    out = np.empty(n, dtype=np.float64)
    lib().oracle_rng_f64(seed, pixel, sample, n, _p(out))
    return out


class DescBuilder:
    """Build a yart_scene_desc by hand (for primitive-level known-answer tests)."""

    def __init__(self, background=(0.0, 0.0, 0.0)):
        self.objects, self.lights, self.materials, self.textures, self.meshes = [], [], [], [], []
        self._keep = []
        self.background = background

    def texture(self, rgb, rgb_even=None):
        t = abi.Texture()
        t.kind = abi.TEX_SOLID if rgb_even is None else abi.TEX_CHECKER
        t.rgb = (C.c_double * 3)(*rgb)
        if rgb_even is not None:
            t.rgb_even = (C.c_double * 3)(*rgb_even)
        self.textures.append(t)
        return len(self.textures) - 1

    def noise_texture(self, noise_type, scale, seed=7):
        """A NoiseTexture with Perlin tables drawn from numpy (any tables are valid input)."""
        rng = np.random.default_rng(seed)
        P = abi.Perlin()
        for i, v in enumerate(rng.uniform(0, 1, 256)):
            P.ranfloat[i] = v
        for i, v in enumerate(rng.uniform(-1, 1, (256, 3))):
            for k in range(3):
                P.ranvec[i][k] = v[k]
        for name in ("perm_x", "perm_y", "perm_z"):
            arr = getattr(P, name)
            for i, v in enumerate(rng.permutation(256)):
                arr[i] = int(v)
        self._keep.append(P)
        t = abi.Texture()
        t.kind, t.noise_type, t.scale = abi.TEX_NOISE, noise_type, scale
        t.rgb = (C.c_double * 3)(1.0, 1.0, 1.0)
        t.perlin = C.pointer(P)
        self.textures.append(t)
        return len(self.textures) - 1

    def image_texture(self, rgb8):
        """An ImageTexture over an (h, w, 3) uint8 array (rows top first)."""
        px = np.ascontiguousarray(rgb8, dtype=np.uint8)
        self._keep.append(px)
        t = abi.Texture()
        t.kind, t.height, t.width = abi.TEX_IMAGE, px.shape[0], px.shape[1]
        t.pixels = px.ctypes.data_as(C.POINTER(C.c_uint8))
        self.textures.append(t)
        return len(self.textures) - 1

    def material(self, kind, texture=0, fuzz=0.0, b=(0, 0, 0), c=(0, 0, 0)):
        m = abi.Material()
        m.kind, m.texture, m.fuzz = kind, texture, fuzz
        m.b = (C.c_double * 3)(*b)
        m.c = (C.c_double * 3)(*c)
        self.materials.append(m)
        return len(self.materials) - 1

    def mesh(self, positions, normals):
        pos = np.ascontiguousarray(positions, dtype=np.float32).reshape(-1, 9)
        nrm = np.ascontiguousarray(normals, dtype=np.float64).reshape(-1, 9)
        self._keep += [pos, nrm]
        m = abi.Mesh()
        m.n_triangles = pos.shape[0]
        m.positions = pos.ctypes.data_as(C.POINTER(C.c_float))
        m.normals = nrm.ctypes.data_as(C.POINTER(C.c_double))
        self.meshes.append(m)
        return len(self.meshes) - 1

    def obj(self, kind, material, p=(), xforms=(), mesh=0, light=False):
        o = abi.Object()
        o.kind, o.material, o.mesh = kind, material, mesh
        o.n_xforms = len(xforms)
        for i, (k, v) in enumerate(xforms):
            o.xforms[i].kind = k
            for j, x in enumerate(v):
                o.xforms[i].v[j] = x
        for i, x in enumerate(p):
            o.p[i] = x
        (self.lights if light else self.objects).append(o)
        return o

    def desc(self):
        def arr(T, xs):
            a = (T * max(1, len(xs)))(*xs)
            self._keep.append(a)
            return a
        d = abi.SceneDesc()
        d.abi_version = abi.ABI_VERSION
        d.n_objects, d.n_lights = len(self.objects), len(self.lights)
        d.n_materials, d.n_textures, d.n_meshes = len(self.materials), len(self.textures), len(self.meshes)
        d.objects = arr(abi.Object, self.objects)
        d.lights = arr(abi.Object, self.lights)
        d.materials = arr(abi.Material, self.materials)
        d.textures = arr(abi.Texture, self.textures)
        d.meshes = arr(abi.Mesh, self.meshes)
        d.background = (C.c_double * 3)(*self.background)
        self._desc = d
        return C.pointer(d)


def mixed_list_desc(n, seed, spread=50.0, shaded=False):
    """A scene description of n mixed list entries (test infrastructure): plain and hollow
    translated spheres, XZ rects, translated + rotated boxes, triangles and flipped YZ rects at
    random places within +-spread, one Lambertian material. The world BVH's structural and parity
    tests run over these."""
    import numpy as np
    rng = np.random.default_rng(seed)
    b = DescBuilder()
    m = b.material(abi.MAT_LAMBERTIAN, b.texture((0.5, 0.5, 0.5)))
    mats = [m]
    if shaded:  # every material kind of the list kernels: checker, metal, glass, emitter
        mats += [b.material(abi.MAT_LAMBERTIAN, b.texture((0.9, 0.1, 0.1), (0.1, 0.1, 0.9))),
                 b.material(abi.MAT_METAL, b.texture((0.8, 0.8, 0.6)), fuzz=0.3),
                 b.material(abi.MAT_DIELECTRIC, b=(1.73759695, 0.313747346, 1.89878101),
                            c=(0.013188707, 0.0623068142, 155.23629)),
                 b.material(abi.MAT_DIFFUSE_LIGHT, b.texture((4.0, 4.0, 4.0)))]
    for k in range(n):
        c = tuple(float(x) for x in rng.uniform(-spread, spread, 3))
        kind = k % 6
        m = mats[int(rng.integers(0, len(mats)))]
        if kind == 0:
            b.obj(abi.PRIM_SPHERE, m, c + (float(rng.uniform(0.1, 3)),))
        elif kind == 1:
            b.obj(abi.PRIM_SPHERE, m, (0.0, 0.0, 0.0, -float(rng.uniform(0.1, 3))), xforms=[(abi.XF_TRANSLATE, c)])
        elif kind == 2:
            b.obj(abi.PRIM_XZ_RECT, m, (c[0], c[0] + 4.0, c[2], c[2] + 3.0, c[1]))
        elif kind == 3:
            b.obj(abi.PRIM_BOX, m, (0.0, 0.0, 0.0, 2.0, 5.0, 1.0),
                  xforms=[(abi.XF_TRANSLATE, c), (abi.XF_ROTATE_Y, (float(rng.uniform(-180, 180)), 0.0, 0.0))])
        elif kind == 4:
            v = rng.uniform(-2, 2, 9) + np.tile(c, 3)
            b.obj(abi.PRIM_TRIANGLE, m, tuple(float(x) for x in v) + (0.0, 1.0, 0.0) * 3 + (0.0,) * 6)
        else:
            b.obj(abi.PRIM_YZ_RECT, m, (c[1], c[1] + 2.0, c[2], c[2] + 2.0, c[0]), xforms=[(abi.XF_FLIP_FACE, (0.0, 0.0, 0.0))])
    if shaded:  # rotated spheres, rects and triangles too, and a light list (rect + sphere)
        for k in range(n // 4):
            c = tuple(float(x) for x in rng.uniform(-spread, spread, 3))
            rot = (abi.XF_ROTATE_Y, (float(rng.uniform(-180, 180)), 0.0, 0.0))
            m = mats[int(rng.integers(0, len(mats)))]
            if k % 3 == 0:
                b.obj(abi.PRIM_SPHERE, m, c + (float(rng.uniform(0.3, 2)),), xforms=[rot])
            elif k % 3 == 1:
                b.obj(abi.PRIM_XY_RECT, m, (c[0], c[0] + 3.0, c[1], c[1] + 2.0, c[2]), xforms=[rot])
            else:
                v = rng.uniform(-2, 2, 9) + np.tile(c, 3)
                b.obj(abi.PRIM_TRIANGLE, m, tuple(float(x) for x in v) + (0.0, 0.0, 1.0) * 3 + (0.0,) * 6,
                      xforms=[(abi.XF_TRANSLATE, (0.5, 0.0, -0.5)), rot])
        light = mats[-1]
        b.obj(abi.PRIM_XZ_RECT, light, (-3.0, 3.0, -3.0, 3.0, spread + 4.0), xforms=[(abi.XF_FLIP_FACE, (0.0, 0.0, 0.0))])
        b.obj(abi.PRIM_XZ_RECT, light, (-3.0, 3.0, -3.0, 3.0, spread + 4.0), light=True)
        b.obj(abi.PRIM_SPHERE, light, (0.0, -spread - 6.0, 0.0, 2.0))
        b.obj(abi.PRIM_SPHERE, light, (0.0, -spread - 6.0, 0.0, 2.0), light=True)
    return b


def big_sphere_desc(n, seed, clustered):
    """A list of n plain spheres built straight into the C arrays (test infrastructure; n up to
    millions): uniform in a 2000-unit cube, or clustered — 64 centres, each with its own spread
    from 1e-6 to 10 units, radii from 1e-7 to 1 — the kind of list whose SAH tree runs deep
    (the 4-wide collapse then exceeded the walk's stack and the BVH was dropped).
    Returns (POINTER(SceneDesc), keep-alive tuple)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    b = DescBuilder()
    m = b.material(abi.MAT_LAMBERTIAN, b.texture((0.5, 0.5, 0.5)))
    objs = (abi.Object * n)()
    raw = np.frombuffer(objs, dtype=np.uint8).reshape(n, C.sizeof(abi.Object))
    u32 = raw[:, :16].view(np.uint32)
    u32[:, 0] = abi.PRIM_SPHERE
    u32[:, 1] = m
    if clustered:
        centres = rng.uniform(-1000, 1000, (64, 3))
        spread = 10.0 ** rng.uniform(-6, 1, 64)
        k = rng.integers(0, 64, n)
        c = centres[k] + rng.normal(0, 1, (n, 3)) * spread[k][:, None]
        r = 10.0 ** rng.uniform(-7, 0, n)
    else:
        c = rng.uniform(-1000, 1000, (n, 3))
        r = rng.uniform(0.1, 1.0, n)
    off = abi.Object.p.offset
    p = np.zeros((n, 4))
    p[:, :3] = c
    p[:, 3] = r
    raw[:, off:off + 32] = p.view(np.uint8)
    d = abi.SceneDesc()
    d.abi_version = abi.ABI_VERSION
    d.n_objects, d.n_lights, d.n_materials, d.n_textures, d.n_meshes = n, 0, 1, 1, 0
    mats = (abi.Material * 1)(*b.materials)
    texs = (abi.Texture * 1)(*b.textures)
    d.objects = C.cast(objs, C.POINTER(abi.Object))
    d.materials = C.cast(mats, C.POINTER(abi.Material))
    d.textures = C.cast(texs, C.POINTER(abi.Texture))
    d.background = (C.c_double * 3)(0.5, 0.6, 0.7)
    keep = (objs, mats, texs, b, d)
    return C.pointer(d), keep
