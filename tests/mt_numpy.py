"""Moller-Trumbore in numpy, in the reference's operation order (qbvh.rs:420-450: h = d x e2,
a = e1 . h, f = 1 / a, u = f (s . h), q = s x e1, v = f (d . q), t = f (e2 . q); accept when
|a| >= f64::EPSILON, u in [0, 1], v >= 0, u + v <= 1, t in [t_min, t_max)), with the world ray
taken into a mesh instance's frame as the oracle does (oracle.c object_hit: the translate / rotate_y
wrappers, outermost first). numpy's elementwise float64 operations are single IEEE operations, so
every t is bitwise the reference's. Test infrastructure: the near-coplanar study of the mesh walk
(tests/test_gpu_parity.py, tools/coplanar_analyze.py)."""
import numpy as np

from yart import abi

EPS = np.finfo(np.float64).eps


def mesh_triangles(desc, k):
    m = desc.meshes[k]
    n = int(m.n_triangles)
    return np.ctypeslib.as_array(m.positions, shape=(n * 9,)).reshape(n, 3, 3).astype(np.float64)


def local_ray(obj, o, d):
    """World ray -> the mesh's frame through obj's wrappers (oracle.c:947-968)."""
    o, d = np.array(o, np.float64), np.array(d, np.float64)
    for level in range(int(obj.n_xforms)):
        x = obj.xforms[level]
        if x.kind == abi.XF_TRANSLATE:
            o = np.array([o[0] - x.v[0], o[1] - x.v[1], o[2] - x.v[2]])
        elif x.kind == abi.XF_ROTATE_Y:
            rad = x.v[0] * np.pi / 180.0
            sn, cs = np.sin(rad), np.cos(rad)
            o = np.array([cs * o[0] - sn * o[2], o[1], sn * o[0] + cs * o[2]])
            d = np.array([cs * d[0] - sn * d[2], d[1], sn * d[0] + cs * d[2]])
        else:
            raise ValueError(f"wrapper kind {x.kind}")
    return o, d


def mt_all(tris, o, d, tmin, tmax):
    """Every triangle's MT test on one ray: (indices of accepted triangles, t, a) for all."""
    v0 = tris[:, 0]
    e1 = tris[:, 1] - v0
    e2 = tris[:, 2] - v0
    h = np.stack([d[1] * e2[:, 2] - d[2] * e2[:, 1], d[2] * e2[:, 0] - d[0] * e2[:, 2],
                  d[0] * e2[:, 1] - d[1] * e2[:, 0]], 1)
    a = e1[:, 0] * h[:, 0] + e1[:, 1] * h[:, 1] + e1[:, 2] * h[:, 2]
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        f = 1.0 / a
        s = o[None, :] - v0
        u = f * (s[:, 0] * h[:, 0] + s[:, 1] * h[:, 1] + s[:, 2] * h[:, 2])
        q = np.stack([s[:, 1] * e1[:, 2] - s[:, 2] * e1[:, 1], s[:, 2] * e1[:, 0] - s[:, 0] * e1[:, 2],
                      s[:, 0] * e1[:, 1] - s[:, 1] * e1[:, 0]], 1)
        v = f * (d[0] * q[:, 0] + d[1] * q[:, 1] + d[2] * q[:, 2])
        t = f * (e2[:, 0] * q[:, 0] + e2[:, 1] * q[:, 1] + e2[:, 2] * q[:, 2])
    ok = ~((a > -EPS) & (a < EPS)) & (u >= 0) & (u <= 1) & (v >= 0) & (u + v <= 1) & (t >= tmin) & (t < tmax)
    return np.flatnonzero(ok), t, a


def own_box_interval(tris, idx, o, d, tmin):
    """[entry, exit] of each triangle's own bounding box along the ray (the reference's slab test)."""
    lo, hi = tris[idx].min(axis=1), tris[idx].max(axis=1)
    with np.errstate(divide="ignore", invalid="ignore"):
        iv = 1.0 / d
        t0, t1 = (lo - o) * iv, (hi - o) * iv
    return np.maximum(np.fmin(t0, t1).max(axis=1), tmin), np.fmax(t0, t1).min(axis=1)


def answer_outside_own_box(desc, ray, obj_index, t):
    """For a closest hit (object obj_index of the list, a mesh instance, at t): the triangles whose MT
    t is bitwise that t, each as (triangle, a, entry, exit) of its own box along the local ray."""
    obj = desc.objects[obj_index]
    tris = mesh_triangles(desc, int(obj.mesh))
    o, d = local_ray(obj, ray[0:3], ray[3:6])
    idx, tt, a = mt_all(tris, o, d, ray[6], ray[7])
    idx = idx[tt[idx] == t]
    ent, ext = own_box_interval(tris, idx, o, d, ray[6])
    return [(int(i), float(a[i]), float(e0), float(e1)) for i, e0, e1 in zip(idx, ent, ext)]
