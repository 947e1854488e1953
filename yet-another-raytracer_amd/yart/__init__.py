"""Python glue over the two C ABIs (include/yart.h, include/yart_host.h).

The product is the HIP library libyart.so (kernels + C ABI) and the C++ host layer
libyart_host.so (presets, OBJ loading, CLI resolution); this module only loads them with
ctypes for tests, bench.py and smoke(). If torch is going to be used in the same process,
import it BEFORE load_device() so libyart.so binds to the HIP runtime torch already loaded
(both carry the soname libamdhip64.so.7) and device pointers are shared.
"""
import ctypes as C
import os
from pathlib import Path

import numpy as np

from . import abi, buildid

PKG_DIR = Path(__file__).resolve().parent.parent
REPO_DIR = PKG_DIR.parent
LIB_DIR = PKG_DIR / "lib"
ASSET_DIR = REPO_DIR / "assets"
DEFAULT_SEED = 0x59415254  # counter RNG seed for every run

_host = None
_dev = None


class StaleLibraryError(RuntimeError):
    """libyart.so's yart_build_id() is not the sha256 of this tree's sources (yart/buildid.py)."""


def build_id():
    """(library build id, this tree's source hash)."""
    L = load_device()
    return L.yart_build_id().decode(), buildid.build_id()


class YartError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"yart error {code}: {msg}")
        self.code = code


def _sig(lib, name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)


def load_host():
    """libyart_host.so (C++, no GPU)."""
    global _host
    if _host is not None:
        return _host
    path = LIB_DIR / "libyart_host.so"
    if not path.exists():
        raise FileNotFoundError(f"{path} is not built; run `make` (or __graft_entry__.build())")
    L = C.CDLL(str(path))
    P, U32, U64, D, I = C.c_void_p, C.c_uint32, C.c_uint64, C.c_double, C.c_int
    _sig(L, "yart_preset_create", I, C.c_char_p, C.c_char_p, U64, C.POINTER(P))
    _sig(L, "yart_preset_destroy", None, P)
    _sig(L, "yart_preset_desc", C.POINTER(abi.SceneDesc), P)
    _sig(L, "yart_preset_defaults", I, P, C.POINTER(abi.RenderDefaults))
    _sig(L, "yart_preset_stand_in", C.c_char_p, P)
    _sig(L, "yart_scene_names", I, C.POINTER(C.c_char_p), I)
    _sig(L, "yart_resolve_dimensions", None, U32, U32, U32, U32, C.POINTER(U32), C.POINTER(U32))
    _sig(L, "yart_cli_parse", I, I, C.POINTER(C.c_char_p), C.POINTER(abi.Cli))
    _sig(L, "yart_resolve_render_options", I, C.c_char_p, C.POINTER(abi.RenderDefaults), C.POINTER(abi.Cli),
         C.POINTER(abi.RenderOptions))
    _sig(L, "yart_obj_triangle_count", I, C.c_char_p, C.POINTER(U32))
    _sig(L, "yart_obj_load", I, C.c_char_p, P, P, P, U32)
    _sig(L, "yart_write_png", I, C.c_char_p, P, U32, U32)
    _sig(L, "yart_host_camera_init", I, C.POINTER(abi.Camera), P, P, P, D, D, D, D, D, D)
    _sig(L, "yart_host_last_error", C.c_char_p)
    _host = L
    return L


def load_device():
    """libyart.so (HIP kernels for gfx950 + C ABI). Raises if it is not built."""
    global _dev
    if _dev is not None:
        return _dev
    variant = os.environ.get("YART_DEVICE_LIB")  # A/B builds (tools/ab.py): a patched tree, its own id
    path = Path(variant or LIB_DIR / "libyart.so")
    if not path.exists():
        raise FileNotFoundError(f"{path} is not built; the HIP path has no fallback")
    L = C.CDLL(str(path))
    P, U32, U64, D, I = C.c_void_p, C.c_uint32, C.c_uint64, C.c_double, C.c_int
    _sig(L, "yart_version", C.c_char_p)
    if not variant:
        # the shipped .so must be the one built from this tree's sources
        lib_id = "(none: a build without yart_build_id)"
        if hasattr(L, "yart_build_id"):
            _sig(L, "yart_build_id", C.c_char_p)
            lib_id = L.yart_build_id().decode()
        tree_id = buildid.build_id()
        if lib_id != tree_id:
            raise StaleLibraryError(f"{path} was built from other sources (build id {lib_id}) than this tree's "
                                    f"({tree_id}); run `make`")
    elif hasattr(L, "yart_build_id"):
        _sig(L, "yart_build_id", C.c_char_p)
    _sig(L, "yart_last_error", C.c_char_p)
    _sig(L, "yart_device_count", I, C.POINTER(I))
    _sig(L, "yart_scene_create", I, I, C.POINTER(abi.SceneDesc), C.POINTER(P))
    _sig(L, "yart_scene_destroy", None, P)
    _sig(L, "yart_scene_get_info", I, P, C.POINTER(abi.SceneInfo))
    _sig(L, "yart_camera_init", I, C.POINTER(abi.Camera), P, P, P, D, D, D, D, D, D)
    _sig(L, "yart_render_async", I, P, C.POINTER(abi.Camera), C.POINTER(abi.RenderParams), P, P)
    _sig(L, "yart_frame_timing", I, P, P, C.POINTER(D), C.POINTER(D), C.POINTER(U32))
    _sig(L, "yart_render", I, P, C.POINTER(abi.Camera), C.POINTER(abi.RenderParams), P, abi.PROGRESS_FN, P)
    _sig(L, "yart_render_with_stats", I, P, C.POINTER(abi.Camera), C.POINTER(abi.RenderParams), P,
         C.POINTER(abi.RenderStats))
    _sig(L, "yart_finalize_rgba8_async", I, I, P, U32, U32, U32, P, P)
    _sig(L, "yart_finalize_rgba8", I, I, P, U32, U32, U32, P)
    _sig(L, "yart_intersect", I, P, P, U32, P, P)
    _sig(L, "yart_probe_rng", I, I, U64, U32, U32, U32, P)
    _sig(L, "yart_probe_math", I, I, I, P, P, U32, P)
    _sig(L, "yart_debug_force_rewalk", I, I, I)
    _sig(L, "yart_shard_packed_len", U64, U32, U32, U32, U32)
    _sig(L, "yart_render_packed_async", I, P, C.POINTER(abi.Camera), C.POINTER(abi.RenderParams), P, P)
    _sig(L, "yart_comm_unique_id", I, P)
    _sig(L, "yart_comm_init_rank", I, P, I, I, I, C.POINTER(P))
    _sig(L, "yart_comm_init_all", I, I, P, P)
    _sig(L, "yart_comm_destroy", None, P)
    _sig(L, "yart_gather_frame_async", I, P, P, U32, U32, I, P, P)
    _sig(L, "yart_multi_create", I, I, P, C.POINTER(abi.SceneDesc), C.POINTER(P))
    _sig(L, "yart_render_multi", I, P, C.POINTER(abi.Camera), C.POINTER(abi.RenderParams), P, abi.PROGRESS_FN, P)
    _sig(L, "yart_render_multi_async", I, P, C.POINTER(abi.Camera), C.POINTER(abi.RenderParams), P, P)
    _sig(L, "yart_multi_frame_timing", I, P, C.POINTER(D), C.POINTER(D), C.POINTER(U32))
    _sig(L, "yart_unpack_shards_async", I, I, P, U32, U64, U32, U32, P, P)
    _sig(L, "yart_multi_last_timing", I, P, C.POINTER(D), C.POINTER(D))
    if hasattr(L, "yart_multi_device_timing"):  # absent from older A/B builds
        _sig(L, "yart_multi_device_timing", I, P, I, C.POINTER(D), C.POINTER(D), C.POINTER(U32))
    _sig(L, "yart_multi_destroy", None, P)
    if hasattr(L, "yart_multi_query"):  # diagnostics only (bench.py's watchdog); absent from older A/B builds
        _sig(L, "yart_multi_query", I, P, P, P)
    _sig(L, "yart_qbvh_build", I, P, P, U32, U32, C.POINTER(abi.QbvhBuildInfo))
    if hasattr(L, "yart_world_bvh_build"):  # host-side check only; absent from older A/B builds
        _sig(L, "yart_world_bvh_build", I, C.POINTER(abi.SceneDesc), C.POINTER(abi.WorldBvhInfo))
    _sig(L, "yart_debug_set_option", I, I, C.c_int64)
    _sig(L, "yart_debug_get_option", I, I, C.POINTER(C.c_int64))
    _dev = L
    # Tools and A/B scripts pass library options as YART_OPTIONS="world_bvh=1,mesh_wavefront=0" to
    # this glue (tools/ab.py children, bench_configs.py); the library itself reads no environment.
    for item in filter(None, os.environ.get("YART_OPTIONS", "").split(",")):
        k, v = item.split("=")
        set_option(k.strip(), int(v))
    return L


# yart_debug_set_option keys (include/yart.h YART_OPT_*)
OPTIONS = {"qbvh_ties_desc": 0, "qbvh_threads": 1, "walk_tree": 2, "mesh_walk_ref": 3, "world_bvh": 4,
           "mesh_wavefront": 5, "wf_pool": 6, "scratch_bytes": 7, "units_per_wave": 8,
           "mesh_park": 9}


def get_option(name):
    v = C.c_int64()
    _check_dev(load_device().yart_debug_get_option(OPTIONS[name], C.byref(v)))
    return v.value


def set_option(name, value):
    """Sets a library option (yart_debug_set_option); returns the previous value."""
    old = get_option(name)
    _check_dev(load_device().yart_debug_set_option(OPTIONS[name], int(value)))
    return old


class option:
    """with yart.option("world_bvh", 1): ... — sets a library option and restores it on exit."""

    def __init__(self, name, value):
        self.name, self.value, self.old = name, value, None

    def __enter__(self):
        self.old = set_option(self.name, self.value)
        return self

    def __exit__(self, *exc):
        set_option(self.name, self.old)
        return False


def _check_host(rc):
    if rc != 0:
        raise YartError(rc, load_host().yart_host_last_error().decode())


def _check_dev(rc):
    if rc != 0:
        raise YartError(rc, load_device().yart_last_error().decode())


def _ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


class Preset:
    """build_scene_preset (main.rs:211-432) through libyart_host; owns the flattened desc."""

    def __init__(self, name, asset_dir=None, scene_seed=42):
        H = load_host()
        self._h = C.c_void_p()
        _check_host(H.yart_preset_create(name.encode(), str(asset_dir or ASSET_DIR).encode(), scene_seed,
                                         C.byref(self._h)))
        self.name = name
        self.desc = H.yart_preset_desc(self._h)
        d = abi.RenderDefaults()
        _check_host(H.yart_preset_defaults(self._h, C.byref(d)))
        self.defaults = d
        self.stand_in = H.yart_preset_stand_in(self._h).decode()

    def close(self):
        if self._h:
            load_host().yart_preset_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def camera(self, width, height, vfov=None, aperture=None):
        """render()'s camera (main.rs:610-626): vup (0,1,0), focus 10, shutter [0, 1)."""
        return make_camera(self.defaults.lookfrom, self.defaults.lookat, vfov if vfov is not None else self.defaults.vfov,
                           width / height, aperture if aperture is not None else self.defaults.aperture)


def make_camera(lookfrom, lookat, vfov, aspect, aperture, focus_dist=10.0, vup=(0.0, 1.0, 0.0)):
    cam = abi.Camera()
    lf = (C.c_double * 3)(*lookfrom)
    la = (C.c_double * 3)(*lookat)
    up = (C.c_double * 3)(*vup)
    _check_host(load_host().yart_host_camera_init(C.byref(cam), lf, la, up, vfov, aspect, aperture, focus_dist, 0.0, 1.0))
    return cam


def render_params(width, height, spp, max_depth, seed=DEFAULT_SEED, shard_index=0, shard_count=1, samples_per_unit=0):
    return abi.RenderParams(width, height, spp, max_depth, seed, shard_index, shard_count, samples_per_unit, 0)


class DeviceScene:
    """A scene resident in one GPU's HBM (yart_scene_create)."""

    def __init__(self, desc, device=0):
        """desc: a POINTER(SceneDesc), or an object owning one (Preset) - kept alive until create
        returns, since yart_scene_create copies everything it needs."""
        L = load_device()
        owner = desc
        if hasattr(desc, "desc"):
            desc = desc.desc
        self._s = C.c_void_p()
        _check_dev(L.yart_scene_create(device, desc, C.byref(self._s)))
        del owner
        self.device = device

    def close(self):
        if self._s:
            load_device().yart_scene_destroy(self._s)
            self._s = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self):
        i = abi.SceneInfo()
        _check_dev(load_device().yart_scene_get_info(self._s, C.byref(i)))
        return i

    def render(self, cam, params, progress=None):
        """Host-output render (yart_render). progress: optional callable(pixels_done), called on
        this thread while the device works."""
        out = np.zeros((params.height, params.width, 3), dtype=np.float64)
        cb = abi.PROGRESS_FN((lambda px, user: progress(px)) if progress else 0)
        _check_dev(load_device().yart_render(self._s, C.byref(cam), C.byref(params), _ptr(out), cb, None))
        return out

    def render_packed_async(self, cam, params, d_packed_ptr, stream_ptr):
        _check_dev(load_device().yart_render_packed_async(self._s, C.byref(cam), C.byref(params),
                                                         C.c_void_p(d_packed_ptr), C.c_void_p(stream_ptr)))

    def render_with_stats(self, cam, params):
        out = np.zeros((params.height, params.width, 3), dtype=np.float64)
        st = abi.RenderStats()
        _check_dev(load_device().yart_render_with_stats(self._s, C.byref(cam), C.byref(params), _ptr(out), C.byref(st)))
        return out, st

    def render_async(self, cam, params, d_xyz_ptr, stream_ptr):
        _check_dev(load_device().yart_render_async(self._s, C.byref(cam), C.byref(params), C.c_void_p(d_xyz_ptr),
                                                  C.c_void_p(stream_ptr)))

    def frame_timing(self, stream_ptr):
        """(render_ms, accumulate_ms, frames): summed kernel times of the frames launched on that
        stream since the last call (HIP events on the stream)."""
        r, a, n = C.c_double(), C.c_double(), C.c_uint32()
        _check_dev(load_device().yart_frame_timing(self._s, C.c_void_p(stream_ptr), C.byref(r), C.byref(a), C.byref(n)))
        return r.value, a.value, n.value

    def intersect(self, rays):
        rays = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 8)
        n = rays.shape[0]
        hits = np.empty((n, 8), dtype=np.float64)
        obj = np.empty(n, dtype=np.int32)
        _check_dev(load_device().yart_intersect(self._s, _ptr(rays), n, _ptr(hits), _ptr(obj)))
        return hits, obj


QBVH_TIES_DESC, QBVH_SERIAL, QBVH_WALK = 1, 2, 4


def load_obj(path, with_uv=False):
    """TriangleMesh::from_obj's triangles (tobj semantics, libyart_host): f32 positions (n, 9) and
    f64 normals (n, 9) (and f64 uvs (n, 6) with with_uv)."""
    H = load_host()
    n = C.c_uint32()
    _check_host(H.yart_obj_triangle_count(str(path).encode(), C.byref(n)))
    pos = np.zeros((n.value, 9), np.float32)
    nrm = np.zeros((n.value, 9), np.float64)
    uv = np.zeros((n.value, 6), np.float64)
    _check_host(H.yart_obj_load(str(path).encode(), _ptr(pos), _ptr(nrm), _ptr(uv), n.value))
    return (pos, nrm, uv) if with_uv else (pos, nrm)


def qbvh_build(positions, normals, flags=0):
    """Host-only L4QBVH build (yart_qbvh_build): shape, tie exposure, digest and build time."""
    positions = np.ascontiguousarray(positions, np.float32)
    normals = np.ascontiguousarray(normals, np.float64)
    info = abi.QbvhBuildInfo()
    _check_dev(load_device().yart_qbvh_build(_ptr(positions), _ptr(normals), len(positions), flags, C.byref(info)))
    return {k: getattr(info, k) for k, _ in info._fields_ if "reserved" not in k}


def world_bvh_build(desc):
    """Host-only world BVH build of a scene description (yart_world_bvh_build): the binary and
    4-wide trees as scene creation builds them, and the 4-wide tree's structural check."""
    info = abi.WorldBvhInfo()
    _check_dev(load_device().yart_world_bvh_build(desc, C.byref(info)))
    return {k: getattr(info, k) for k, _ in info._fields_}


def finalize_rgba8(xyz_sum, spp, device=0):
    h, w, _ = xyz_sum.shape
    xyz = np.ascontiguousarray(xyz_sum, dtype=np.float64)
    out = np.zeros((h, w, 4), dtype=np.uint8)
    _check_dev(load_device().yart_finalize_rgba8(device, _ptr(xyz), w, h, spp, _ptr(out)))
    return out


def write_png(path, rgba):
    rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
    h, w, _ = rgba.shape
    _check_host(load_host().yart_write_png(str(path).encode(), _ptr(rgba), w, h))


def shard_packed_len(width, height, shard_index, shard_count):
    """Doubles in shard `shard_index`'s block-packed buffer (yart_shard_packed_len)."""
    return int(load_device().yart_shard_packed_len(width, height, shard_index, shard_count))


def unpack_shards_async(device, d_recv_ptr, shards, stride, width, height, d_frame_ptr, stream_ptr):
    """yart_unpack_shards_async: `shards` packed shards back to back (stride doubles apart) ->
    the W x H x 3 frame, on the device."""
    _check_dev(load_device().yart_unpack_shards_async(device, C.c_void_p(d_recv_ptr), shards, stride, width, height,
                                                      C.c_void_p(d_frame_ptr), C.c_void_p(stream_ptr)))


class Comm:
    """An RCCL communicator of libyart (yart_comm_init_rank): one rank per process/GPU. The root's
    128-byte id reaches the other ranks through the caller's own channel (e.g. torch.distributed)."""

    @staticmethod
    def unique_id():
        buf = (C.c_uint8 * abi.COMM_ID_BYTES)()
        _check_dev(load_device().yart_comm_unique_id(buf))
        return bytes(buf)

    def __init__(self, uid, n_ranks, rank, device):
        assert len(uid) == abi.COMM_ID_BYTES
        buf = (C.c_uint8 * abi.COMM_ID_BYTES).from_buffer_copy(uid)
        self._c = C.c_void_p()
        _check_dev(load_device().yart_comm_init_rank(buf, n_ranks, rank, device, C.byref(self._c)))
        self.n_ranks, self.rank, self.device = n_ranks, rank, device

    def gather_frame_async(self, d_packed_ptr, width, height, d_frame_ptr, stream_ptr, root=0):
        _check_dev(load_device().yart_gather_frame_async(self._c, C.c_void_p(d_packed_ptr), width, height, root,
                                                        C.c_void_p(d_frame_ptr), C.c_void_p(stream_ptr)))

    def close(self):
        if self._c:
            load_device().yart_comm_destroy(self._c)
            self._c = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MultiScene:
    """One process, N devices (yart_multi_create): a scene on each and an RCCL communicator."""

    def __init__(self, desc, devices):
        L = load_device()
        owner = desc
        if hasattr(desc, "desc"):
            desc = desc.desc
        devs = (C.c_int * len(devices))(*devices)
        self._m = C.c_void_p()
        _check_dev(L.yart_multi_create(len(devices), devs, desc, C.byref(self._m)))
        del owner
        self.devices = list(devices)

    def render(self, cam, params, progress=None):
        out = np.zeros((params.height, params.width, 3), dtype=np.float64)
        cb = abi.PROGRESS_FN((lambda px, user: progress(px)) if progress else 0)
        _check_dev(load_device().yart_render_multi(self._m, C.byref(cam), C.byref(params), _ptr(out), cb, None))
        return out

    def render_async(self, cam, params, d_frame_ptr, stream_ptr):
        """yart_render_multi_async: the frame lands in d_frame (on devices[0]) in the order of
        stream_ptr (a stream of devices[0]); no host wait."""
        _check_dev(load_device().yart_render_multi_async(self._m, C.byref(cam), C.byref(params), C.c_void_p(d_frame_ptr),
                                                         C.c_void_p(stream_ptr)))

    def frame_timing(self):
        """(render_ms, gather_ms, frames) summed over the async frames since the last call: the
        slowest device's render time and the root's gather + unpack time."""
        r, g, n = C.c_double(), C.c_double(), C.c_uint32()
        _check_dev(load_device().yart_multi_frame_timing(self._m, C.byref(r), C.byref(g), C.byref(n)))
        return r.value, g.value, n.value

    def query(self):
        """yart_multi_query: (per-device state of the latest frame: 0 rendering, 1 rendered,
        2 gathered, -1 unknown; unpacked 1 / 0 / -1). Never waits."""
        st = (C.c_int32 * len(self.devices))()
        up = C.c_int32()
        _check_dev(load_device().yart_multi_query(self._m, st, C.byref(up)))
        return list(st), up.value

    def device_timing(self):
        """yart_multi_device_timing: per device, summed over the frames of the latest frame_timing()
        read — (render_ms list, own-gather_ms list, frames)."""
        n = len(self.devices)
        r, g, f = (C.c_double * n)(), (C.c_double * n)(), C.c_uint32()
        _check_dev(load_device().yart_multi_device_timing(self._m, n, r, g, C.byref(f)))
        return list(r), list(g), f.value

    def last_timing(self):
        r, g = C.c_double(), C.c_double()
        _check_dev(load_device().yart_multi_last_timing(self._m, C.byref(r), C.byref(g)))
        return r.value, g.value

    def close(self):
        if self._m:
            load_device().yart_multi_destroy(self._m)
            self._m = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
