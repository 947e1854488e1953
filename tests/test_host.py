"""Host layer (libyart_host.so): the reference's CLI/option tests restated, presets, OBJ loading,
PNG output. No GPU."""
import ctypes as C
import struct
import zlib

import numpy as np
import pytest

import oracle_lib as O
import yart
from yart import abi


def H():
    return yart.load_host()


def parse(*args):
    argv = (C.c_char_p * (len(args) + 1))(b"yart", *[a.encode() for a in args])
    cli = abi.Cli()
    rc = H().yart_cli_parse(len(args) + 1, argv, C.byref(cli))
    return rc, cli, H().yart_host_last_error().decode()


def dims(dw, dh, wo, ho):
    w, h = C.c_uint32(), C.c_uint32()
    H().yart_resolve_dimensions(dw, dh, wo, ho, C.byref(w), C.byref(h))
    return w.value, h.value


# ---- main.rs:830-842
def test_cli_accepts_named_scene_values():
    rc, cli, _ = parse("--scene", "david")
    assert rc == 0 and cli.scene == b"david"


def test_cli_rejects_unknown_scene_values():
    rc, _, err = parse("--scene", "unknown-scene")
    assert rc == abi.ERR_INVALID and "invalid value 'unknown-scene'" in err


def test_cli_requires_scene_and_positive_values():
    assert parse()[0] == abi.ERR_INVALID
    rc, _, err = parse("--scene", "david", "--samples", "0")
    assert rc == abi.ERR_INVALID and "value must be greater than 0" in err  # parse_positive_usize main.rs:151-160
    rc, _, err = parse("--scene", "david", "--width", "0")
    assert rc == abi.ERR_INVALID
    rc, cli, _ = parse("--scene=cornell-box", "--width", "640", "--max-depth=12", "--vfov", "45.5", "--aperture", "0.25")
    assert rc == 0 and cli.width == 640 and cli.max_depth == 12 and cli.vfov == 45.5 and cli.aperture == 0.25


# ---- main.rs:844-865
def test_resolve_dimensions():
    assert dims(1200, 800, 0, 0) == (1200, 800)
    assert dims(1200, 800, 600, 0) == (600, 400)
    assert dims(1200, 800, 0, 400) == (600, 400)
    assert dims(1200, 800, 1024, 512) == (1024, 512)
    assert dims(1200, 800, 1, 0) == (1, 1)  # .round().max(1.0)


def _defaults():
    d = abi.RenderDefaults(1200, 800, 100, 50, 30, 20.0, 0.0)
    return d


# ---- main.rs:867-915
def test_resolve_render_options_uses_default_output_when_not_overridden():
    _, cli, _ = parse("--scene", "david")
    o = abi.RenderOptions()
    assert H().yart_resolve_render_options(b"david.png", C.byref(_defaults()), C.byref(cli), C.byref(o)) == 0
    assert o.output_path == b"output/david.png"


def test_resolve_render_options_respects_output_and_scalar_overrides():
    _, cli, _ = parse("--scene", "david", "--output", "custom/output.png", "--width", "600", "--samples", "32",
                      "--max-depth", "12", "--workers", "8", "--vfov", "45", "--aperture", "0.25")
    o = abi.RenderOptions()
    assert H().yart_resolve_render_options(b"david.png", C.byref(_defaults()), C.byref(cli), C.byref(o)) == 0
    assert o.output_path == b"custom/output.png"
    assert (o.width, o.height, o.samples_per_pixel, o.max_depth, o.workers) == (600, 400, 32, 12, 8)
    assert (o.vfov, o.aperture) == (45.0, 0.25)


# ---- presets (main.rs:211-432, scenes.rs)
def test_scene_names_are_the_reference_value_enum():
    arr = (C.c_char_p * 32)()
    n = H().yart_scene_names(arr, 32)
    assert [arr[i].decode() for i in range(n)] == [
        "random-scene", "two-spheres", "two-perlin-spheres", "earth", "simple-light", "cornell-box",
        "cornell-box-smoke", "next-week-final", "teapot", "bunny", "three-spheres", "sycee", "david"]


def test_cornell_preset_flattens_like_scenes_rs():
    p = yart.Preset("cornell-box")
    d = p.desc.contents
    assert (p.defaults.width, p.defaults.height, p.defaults.samples_per_pixel, p.defaults.vfov) == (600, 600, 100, 40.0)
    assert list(p.defaults.lookfrom) == [278.0, 278.0, -800.0]
    kinds = [d.objects[i].kind for i in range(d.n_objects)]
    assert kinds == [abi.PRIM_YZ_RECT, abi.PRIM_YZ_RECT, abi.PRIM_XZ_RECT, abi.PRIM_XZ_RECT, abi.PRIM_XZ_RECT,
                     abi.PRIM_XY_RECT, abi.PRIM_BOX, abi.PRIM_SPHERE]
    light = d.objects[2]
    assert light.n_xforms == 1 and light.xforms[0].kind == abi.XF_FLIP_FACE
    box = d.objects[6]
    assert box.n_xforms == 2 and box.xforms[0].kind == abi.XF_TRANSLATE and box.xforms[1].kind == abi.XF_ROTATE_Y
    assert list(box.xforms[0].v) == [265.0, 0.0, 295.0] and box.xforms[1].v[0] == 15.0
    assert list(box.p[:6]) == [0, 0, 0, 165, 330, 165]
    assert d.materials[d.objects[7].material].kind == abi.MAT_DIELECTRIC
    assert d.materials[light.material].kind == abi.MAT_DIFFUSE_LIGHT
    assert d.n_lights == 2 and d.lights[0].kind == abi.PRIM_XZ_RECT and d.lights[1].kind == abi.PRIM_SPHERE
    assert list(d.lights[0].p[:5]) == [213.0, 343.0, 227.0, 332.0, 554.0]
    assert list(d.background) == [0.0, 0.0, 0.0]


def test_bunny_uses_declared_stand_in_and_reference_lights():
    p = yart.Preset("bunny")
    assert "stand-in mesh: sycee.obj" in p.stand_in
    d = p.desc.contents
    assert d.meshes[0].n_triangles == 31642
    assert list(d.lights[0].p[:4]) == [0.0, 6.0, 2.0, 2.0]   # main.rs:335-339 (+2)
    assert list(d.objects[3].p[:4]) == [0.0, 6.0, -2.0, 2.0]  # scenes.rs:572-576 (-2)


def test_david_shares_one_mesh_between_instances():
    p = yart.Preset("david")
    d = p.desc.contents
    meshes = [d.objects[i] for i in range(d.n_objects) if d.objects[i].kind == abi.PRIM_MESH]
    assert len(meshes) == 2 and meshes[0].mesh == meshes[1].mesh == 0 and d.n_meshes == 1
    assert meshes[1].xforms[1].v[0] == 300.0 and list(meshes[1].xforms[0].v) == [50.0, 0.0, 50.0]
    assert d.n_lights == 5


def test_random_scene_is_deterministic_per_seed():
    pa_, pb_, pc_ = (yart.Preset("random-scene", scene_seed=s) for s in (42, 42, 43))  # keep the owners alive
    a, b, c = pa_.desc.contents, pb_.desc.contents, pc_.desc.contents
    pa = [tuple(a.objects[i].p[:4]) for i in range(a.n_objects)]
    assert pa == [tuple(b.objects[i].p[:4]) for i in range(b.n_objects)]
    assert pa != [tuple(c.objects[i].p[:4]) for i in range(c.n_objects)]
    assert pa[0] == (0.0, -1000.0, 0.0, 1000.0) and pa[-1] == (4.0, 1.0, 0.0, 1.0)
    for (x, y, z, r) in pa[1:-3]:
        assert r == 0.2 and y == 0.2 and np.hypot(x - 4.0, z) > 0.9
    # negative Lambertian albedos are kept (scenes.rs:44-48)
    assert any(min(a.textures[i].rgb) < 0 for i in range(a.n_textures))


@pytest.mark.parametrize("name,code", [("next-week-final", abi.ERR_UNSUPPORTED), ("nope", abi.ERR_INVALID)])
def test_out_of_scope_presets_fail_loudly(name, code):
    with pytest.raises(yart.YartError) as e:
        yart.Preset(name)
    assert e.value.code == code


# ---- OBJ loader (tobj 4.0.2 GPU_LOAD_OPTIONS semantics, triangle.rs:111-174)
@pytest.mark.parametrize("name,n", [("cube", 12), ("david", 46664), ("sycee", 31642)])
def test_obj_triangle_counts(repo, name, n):
    c = C.c_uint32()
    assert H().yart_obj_triangle_count(str(repo / "assets" / f"{name}.obj").encode(), C.byref(c)) == 0
    assert c.value == n


def test_obj_cube_fan_triangulation_and_f32_positions(repo):
    n = 12
    pos = np.zeros((n, 9), dtype=np.float32)
    nrm = np.zeros((n, 9))
    uv = np.zeros((n, 6))
    assert H().yart_obj_load(str(repo / "assets" / "cube.obj").encode(), C.c_void_p(pos.ctypes.data),
                             C.c_void_p(nrm.ctypes.data), C.c_void_p(uv.ctypes.data), n) == 0
    # first face "f 2/1/1 3/2/1 4/3/1" with v2 = (1,-1,1), v3 = (-1,-1,1), v4 = (-1,-1,-1)
    np.testing.assert_array_equal(pos[0], np.float32([1, -1, 1, -1, -1, 1, -1, -1, -1]))
    assert (np.abs(np.linalg.norm(nrm.reshape(-1, 3), axis=1) - 1) < 1e-3).all()
    # "v 1.000000 1.000000 -0.999999" parses to the nearest f32, as tobj does
    assert np.float32(-0.999999) in pos


def test_obj_missing_file_reports_io_error():
    c = C.c_uint32()
    assert H().yart_obj_triangle_count(b"/nonexistent.obj", C.byref(c)) == abi.ERR_IO
    assert "Failed to load OBJ file" in H().yart_host_last_error().decode()


def test_david_qbvh_shape_matches_reference_algorithm():
    p = yart.Preset("david")
    assert O.OracleScene(p.desc).qbvh_stats(0) == (5461, 16384, 7)


# ---- PNG (main.rs:774)
def test_png_roundtrip(tmp_path):
    rgba = (np.arange(7 * 5 * 4, dtype=np.uint32) % 251).astype(np.uint8).reshape(5, 7, 4)
    path = tmp_path / "x.png"
    yart.write_png(path, rgba)
    data = path.read_bytes()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    w, h, bd, ct = struct.unpack(">IIBB", data[16:26])
    assert (w, h, bd, ct) == (7, 5, 8, 6)
    i, idat = 8, b""
    while i < len(data):
        ln, typ = struct.unpack(">I4s", data[i:i + 8])
        chunk = data[i + 8:i + 8 + ln]
        assert zlib.crc32(typ + chunk) == struct.unpack(">I", data[i + 8 + ln:i + 12 + ln])[0]
        if typ == b"IDAT":
            idat += chunk
        i += 12 + ln
    raw = np.frombuffer(zlib.decompress(idat), dtype=np.uint8).reshape(5, 1 + 7 * 4)
    assert (raw[:, 0] == 0).all()
    np.testing.assert_array_equal(raw[:, 1:].reshape(5, 7, 4), rgba)


def test_host_camera_matches_camera_rs():
    cam = yart.make_camera((278.0, 278.0, -800.0), (278.0, 278.0, 0.0), 40.0, 1.0, 0.0)
    assert list(cam.w) == [0.0, 0.0, -1.0] and list(cam.u) == [-1.0, 0.0, 0.0]
    h = np.tan(np.radians(40.0) / 2.0) * 2.0
    assert abs(cam.horizontal[0] + 10.0 * h) < 1e-12 and cam.lens_radius == 0.0
    assert list(cam.origin) == [278.0, 278.0, -800.0]


@pytest.mark.parametrize("name", ["cube", "david", "sycee"])
def test_obj_loader_matches_the_oracles_independent_reader(repo, name):
    """The product's OBJ loader (host/scene.cpp) against the oracle's own reader (oracle_obj.c,
    written from triangle.rs:111-174 and tobj's GPU_LOAD_OPTIONS: f32 parse, fan triangulation,
    face normals for vertices without vn, (0, 0) without vt): the triangle arrays the renders use
    are the same bytes, so a loader bug cannot hide behind the oracle consuming the product's
    scene description (VERDICT r02 Missing #4)."""
    path = repo / "assets" / f"{name}.obj"
    pos, nrm, uv = yart.load_obj(path, with_uv=True)
    opos, onrm, ouv = O.load_obj(path)
    assert pos.tobytes() == opos.tobytes()
    assert nrm.tobytes() == onrm.tobytes()
    assert uv.tobytes() == ouv.tobytes()


def test_oracle_obj_reader_on_hand_made_faces(tmp_path):
    """Fan triangulation of an n-gon, negative (relative) indices, `v//vn` and `v/vt` forms, and the
    face normal of a vertex without vn - checked by hand, independent of both loaders."""
    f = tmp_path / "t.obj"
    f.write_text("v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nv 0.1 0.2 0.3\n"
                 "vt 0.25 0.75\nvt 0.5 0.5\nvt 1 1\nvt 0 1\n"
                 "f 1/1 2/2 3/3 4/4\n"      # quad -> (1,2,3), (1,3,4); uv from vt, face normal +z
                 "f -5/-4 -3/-2 -1/-1\n")   # relative: vertices 1, 3, 5
    pos, nrm, uv = O.load_obj(f)
    assert pos.shape == (3, 9)
    np.testing.assert_array_equal(pos[0], np.float32([0, 0, 0, 1, 0, 0, 1, 1, 0]))
    np.testing.assert_array_equal(pos[1], np.float32([0, 0, 0, 1, 1, 0, 0, 1, 0]))
    np.testing.assert_array_equal(pos[2], np.float32([0, 0, 0, 1, 1, 0, 0.1, 0.2, 0.3]))
    np.testing.assert_array_equal(nrm[0], [0, 0, 1] * 3)
    np.testing.assert_array_equal(uv[1], [0.25, 0.75, np.float32(1.0), 1.0, 0.0, 1.0])
    e1 = np.float64(pos[2, 3:6]) - np.float64(pos[2, :3])
    e2 = np.float64(pos[2, 6:9]) - np.float64(pos[2, :3])
    cr = np.cross(e1, e2)
    np.testing.assert_array_equal(nrm[2, :3], cr / np.sqrt((cr * cr).sum()))
    p2, n2, u2 = yart.load_obj(f, with_uv=True)  # and the product agrees
    assert p2.tobytes() == pos.tobytes() and n2.tobytes() == nrm.tobytes() and u2.tobytes() == uv.tobytes()


def test_rotated_plane_rays_are_in_plane_nan_hits_for_the_oracle():
    """tests/inplane_rays.py's construction (the data of test_rays_in_rotated_planes_match_oracle):
    no world direction component is zero, the local one is, and the oracle reports t = NaN hits
    on every rotated rect and box (aarect.rs:111-146 under hittable.rs:217-251)."""
    import time

    import inplane_rays as IR
    t0 = time.time()
    b, planes = IR.rotated_planes_scene()
    rays = IR.rotated_plane_rays(planes, 300)
    assert time.time() - t0 < 30
    assert (rays[:, 3:6] != 0).all()
    h, o = O.OracleScene(b.desc()).intersect(rays)
    nan = (o >= 0) & np.isnan(h[:, 0])
    assert nan.sum() > 500 and len(np.unique(o[nan])) == 6
