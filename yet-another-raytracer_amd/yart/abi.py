"""ctypes mirror of include/yart.h and include/yart_host.h (layout must match the C headers)."""
import ctypes as C

ABI_VERSION = 1

OK, ERR_INVALID, ERR_DEVICE, ERR_NO_MEMORY, ERR_UNSUPPORTED, ERR_IO = 0, -1, -2, -3, -4, -5

TEX_SOLID, TEX_CHECKER, TEX_NOISE, TEX_IMAGE = 0, 1, 2, 3
NOISE_SQUARE, NOISE_TRILINEAR, NOISE_SMOOTH, NOISE_MARBLE, NOISE_NET = range(5)
MAT_NONE, MAT_LAMBERTIAN, MAT_METAL, MAT_DIELECTRIC, MAT_DIFFUSE_LIGHT, MAT_ISOTROPIC = 0, 1, 2, 3, 4, 5
PRIM_SPHERE, PRIM_XY_RECT, PRIM_XZ_RECT, PRIM_YZ_RECT, PRIM_BOX, PRIM_TRIANGLE, PRIM_MESH, PRIM_MOVING_SPHERE = range(8)
XF_TRANSLATE, XF_ROTATE_Y, XF_FLIP_FACE, XF_MEDIUM = 1, 2, 3, 4
MAX_XFORMS = 4

D3 = C.c_double * 3


class Perlin(C.Structure):
    _fields_ = [("ranfloat", C.c_double * 256), ("ranvec", (C.c_double * 3) * 256), ("perm_x", C.c_int32 * 256),
                ("perm_y", C.c_int32 * 256), ("perm_z", C.c_int32 * 256)]


class Texture(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("noise_type", C.c_uint32), ("rgb", D3), ("rgb_even", D3), ("scale", C.c_double),
                ("perlin", C.POINTER(Perlin)), ("width", C.c_uint32), ("height", C.c_uint32),
                ("pixels", C.POINTER(C.c_uint8))]


class Material(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("texture", C.c_uint32), ("fuzz", C.c_double), ("b", D3), ("c", D3)]


class Xform(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("reserved", C.c_uint32), ("v", D3)]


class Object(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("material", C.c_uint32), ("mesh", C.c_uint32), ("n_xforms", C.c_uint32),
                ("xforms", Xform * MAX_XFORMS), ("p", C.c_double * 24)]


class Mesh(C.Structure):
    _fields_ = [("n_triangles", C.c_uint32), ("reserved", C.c_uint32), ("positions", C.POINTER(C.c_float)),
                ("normals", C.POINTER(C.c_double)), ("uvs", C.POINTER(C.c_double))]


class SceneDesc(C.Structure):
    _fields_ = [("abi_version", C.c_uint32), ("n_objects", C.c_uint32), ("n_lights", C.c_uint32),
                ("n_materials", C.c_uint32), ("n_textures", C.c_uint32), ("n_meshes", C.c_uint32),
                ("objects", C.POINTER(Object)), ("lights", C.POINTER(Object)),
                ("materials", C.POINTER(Material)), ("textures", C.POINTER(Texture)),
                ("meshes", C.POINTER(Mesh)), ("background", D3)]


class Camera(C.Structure):
    _fields_ = [("lower_left_corner", D3), ("horizontal", D3), ("vertical", D3), ("origin", D3),
                ("u", D3), ("v", D3), ("w", D3), ("lens_radius", C.c_double), ("time0", C.c_double),
                ("time1", C.c_double)]


class RenderParams(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("spp", C.c_uint32), ("max_depth", C.c_uint32),
                ("seed", C.c_uint64), ("shard_index", C.c_uint32), ("shard_count", C.c_uint32),
                ("samples_per_unit", C.c_uint32), ("reserved", C.c_uint32)]


class SceneInfo(C.Structure):
    _fields_ = [("device", C.c_int), ("n_objects", C.c_uint32), ("n_lights", C.c_uint32), ("n_meshes", C.c_uint32),
                ("bvh_nodes", C.c_uint32), ("bvh_leaves", C.c_uint32), ("bvh_max_depth", C.c_uint32),
                ("bvh_max_stack", C.c_uint32), ("device_bytes", C.c_uint64), ("world_nodes", C.c_uint32),
                ("world_depth", C.c_uint32), ("bvh_tied_cuts", C.c_uint32), ("bvh_tied_leaves", C.c_uint32),
                ("bvh_build_ms", C.c_double), ("upload_ms", C.c_double), ("walk_nodes", C.c_uint32),
                ("walk_depth", C.c_uint32)]


class QbvhBuildInfo(C.Structure):
    _fields_ = [("nodes", C.c_uint32), ("leaves", C.c_uint32), ("depth", C.c_uint32), ("tied_cuts", C.c_uint32),
                ("tied_leaves", C.c_uint32), ("reserved", C.c_uint32), ("digest", C.c_uint64),
                ("build_ms", C.c_double), ("walk_nodes", C.c_uint32), ("walk_depth", C.c_uint32),
                ("walk_valid", C.c_uint32), ("walk_reserved", C.c_uint32), ("walk_build_ms", C.c_double)]


class WorldBvhInfo(C.Structure):
    _fields_ = [("built", C.c_uint32), ("nodes", C.c_uint32), ("depth", C.c_uint32), ("nodes4", C.c_uint32),
                ("depth4", C.c_uint32), ("valid", C.c_uint32), ("digest", C.c_uint64)]


class RenderStats(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("segments", C.c_uint64), ("prim_tests", C.c_uint64),
                ("node_visits", C.c_uint64), ("leaf_visits", C.c_uint64), ("leaf_tris", C.c_uint64),
                ("light_tests", C.c_uint64), ("mesh_rewalks", C.c_uint64),
                ("coop_rounds", C.c_uint64), ("coop_leaf_rounds", C.c_uint64), ("coop_walks", C.c_uint64),
                ("coop_idle_slots", C.c_uint64), ("world_iters", C.c_uint64),
                ("world_leaf_iters", C.c_uint64), ("ovf_pushes", C.c_uint64),
                ("coop_node_rounds", C.c_uint64), ("coop_node_lanes", C.c_uint64), ("coop_leaf_lanes", C.c_uint64),
                ("coop_leaf_quad_lanes", C.c_uint64), ("iterations", C.c_uint64), ("camera_lanes", C.c_uint64),
                ("scatter_lanes", C.c_uint64), ("camera_iters", C.c_uint64), ("scatter_iters", C.c_uint64),
                ("parked_walks", C.c_uint64)]


class RenderDefaults(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("samples_per_pixel", C.c_uint64),
                ("max_depth", C.c_uint64), ("workers", C.c_uint64), ("vfov", C.c_double), ("aperture", C.c_double),
                ("lookfrom", D3), ("lookat", D3), ("background", D3), ("output_filename", C.c_char * 64)]


class Cli(C.Structure):
    _fields_ = [("scene", C.c_char * 64), ("output", C.c_char * 512), ("width", C.c_uint32), ("height", C.c_uint32),
                ("samples", C.c_uint64), ("max_depth", C.c_uint64), ("workers", C.c_uint64), ("vfov", C.c_double),
                ("aperture", C.c_double), ("seed", C.c_uint64), ("gpus", C.c_int32), ("assets", C.c_char * 512)]


class RenderOptions(C.Structure):
    _fields_ = [("output_path", C.c_char * 512), ("width", C.c_uint32), ("height", C.c_uint32),
                ("samples_per_pixel", C.c_uint64), ("max_depth", C.c_uint64), ("workers", C.c_uint64),
                ("vfov", C.c_double), ("aperture", C.c_double)]


PROGRESS_FN = C.CFUNCTYPE(None, C.c_uint64, C.c_void_p)

# Every symbol include/yart.h declares (checked by tests/test_abi.py without a GPU).
DEVICE_SYMBOLS = [
    "yart_version", "yart_build_id", "yart_multi_device_timing", "yart_last_error", "yart_device_count", "yart_scene_create", "yart_scene_destroy",
    "yart_scene_get_info", "yart_camera_init", "yart_render_async", "yart_frame_timing", "yart_render",
    "yart_render_with_stats",
    "yart_finalize_rgba8_async", "yart_finalize_rgba8", "yart_intersect", "yart_probe_rng", "yart_probe_math",
    "yart_debug_force_rewalk",
    "yart_debug_set_option",
    "yart_debug_get_option",
    "yart_multi_query",
    "yart_world_bvh_build",
    "yart_shard_packed_len", "yart_render_packed_async", "yart_comm_unique_id", "yart_comm_init_rank",
    "yart_comm_init_all", "yart_comm_destroy", "yart_gather_frame_async", "yart_multi_create", "yart_render_multi",
    "yart_multi_last_timing", "yart_multi_destroy", "yart_qbvh_build", "yart_render_multi_async",
    "yart_multi_frame_timing", "yart_unpack_shards_async",
]
COMM_ID_BYTES = 128
HOST_SYMBOLS = [
    "yart_preset_create", "yart_preset_destroy", "yart_preset_desc", "yart_preset_defaults", "yart_preset_stand_in",
    "yart_scene_names", "yart_resolve_dimensions", "yart_cli_parse", "yart_resolve_render_options",
    "yart_obj_triangle_count", "yart_obj_load", "yart_write_png", "yart_host_camera_init", "yart_host_last_error",
]
