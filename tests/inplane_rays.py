"""Rays lying EXACTLY in a rotated planar object's own plane (test data, CPU only).

A rect's test (aarect.rs:111-146) divides (k - o_a) by d_a in the object's local frame. When both
are exactly 0 the reference gets t = NaN, which passes its range and bounds tests: a "hit" wherever
the ray runs. Under RotateY (hittable.rs:217-251) the local frame's d_a = cos·d_x - sin·d_z (or
sin·d_x + cos·d_z) can cancel to exactly 0 while no world component is 0, so a world-space test
for zero components does not see it. This module builds such rays by searching the doubles next
to the analytic solution until the local component — evaluated with exactly the operations of
to_local (kernels.hip) / the oracle — is 0, and the local origin component is the plane's k.
"""
import math

import numpy as np

import oracle_lib as O
from yart import abi


def sincos_deg(angle):
    """RotateY::new (hittable.rs:173-176) as capi.cpp / oracle.c evaluate it."""
    rad = angle * 3.141592653589793 / 180.0
    return math.sin(rad), math.cos(rad)


def to_local(chain, o, d):
    """kernels.hip to_local over a chain of ('T', (x, y, z)) / ('R', sn, cs), outermost first."""
    o, d = list(o), list(d)
    for step in chain:
        if step[0] == "T":
            o = [o[k] - step[1][k] for k in range(3)]
        else:
            sn, cs = step[1], step[2]
            o = [cs * o[0] - sn * o[2], o[1], sn * o[0] + cs * o[2]]
            d = [cs * d[0] - sn * d[2], d[1], sn * d[0] + cs * d[2]]
    return o, d


def _solve(f, x0, free, target, reach=256):
    """A double x near x0 with f(x) == target exactly, searching outwards ulp by ulp (None: none)."""
    for base in (x0, free):
        if base is None or not math.isfinite(base):
            continue
        lo = hi = base
        for _ in range(reach):
            for x in (lo, hi):
                if f(x) == target:
                    return x
            lo, hi = math.nextafter(lo, -math.inf), math.nextafter(hi, math.inf)
    return None


def plane_rays(chain, axis, k, n, rng, span=30.0):
    """n rays whose local direction component `axis` (0 = x, 2 = z) is exactly 0; the first half
    also start exactly in the local plane x (or z) = k, the rest off it (their t is +-inf: a miss)."""
    rays = []
    tries = 0
    while len(rays) < n and tries < 20 * n:
        tries += 1
        d = list(rng.normal(size=3))
        o = list(rng.uniform(-span, span, 3))
        # the direction: solve d_x with d_z kept, else d_z with d_x kept, for a zero local component;
        # the guesses from the composite rotation's angle (RotateYs compose additively)
        ang = sum(math.atan2(s[1], s[2]) for s in chain if s[0] == "R")
        sa, ca = math.sin(ang), math.cos(ang)
        fx = lambda x: to_local(chain, o, [x, d[1], d[2]])[1][axis]
        fz = lambda z: to_local(chain, o, [d[0], d[1], z])[1][axis]
        if axis == 0:  # ca d_x - sa d_z = 0
            gx, gz = (sa * d[2] / ca if ca else None), (ca * d[0] / sa if sa else None)
        else:          # sa d_x + ca d_z = 0
            gx, gz = (-ca * d[2] / sa if sa else None), (-sa * d[0] / ca if ca else None)
        x = _solve(fx, gx, None, 0.0)
        if x is not None:
            d[0] = x
        else:
            z = _solve(fz, gz, None, 0.0)
            if z is None:
                continue
            d[2] = z
        if len(rays) < n // 2:  # the origin: o_x (else o_z) such that the local o_a is exactly k
            done = False
            for c in (0, 2):
                def fo(v, c=c):
                    oo = list(o)
                    oo[c] = v
                    return to_local(chain, oo, d)[0][axis]
                a0, a1 = fo(0.0), fo(1.0)  # local o_a is affine in each world component
                g = (k - a0) / (a1 - a0) if a1 != a0 else None
                v = _solve(fo, g, None, k)
                if v is not None:
                    o[c] = v
                    done = True
                    break
            if not done:
                continue
        lo, ld = to_local(chain, o, d)
        assert ld[axis] == 0.0 and all(c != 0.0 for c in d)
        rays.append(o + d + [0.001, math.inf])
    return np.array(rays, dtype=np.float64)


def rotated_planes_scene(seed=5):
    """A 26-object list (world BVH eligible): 16 spheres, and 8 rotated rects and boxes — RotateY
    by 90, 30, -18, 200 and 271.5 degrees, one under Translate, one under two RotateYs, one
    FlipFace. Returns (DescBuilder, [(chain, axis, k)]) with the local planes to aim at."""
    rng = np.random.default_rng(seed)
    b = O.DescBuilder()
    m = b.material(abi.MAT_LAMBERTIAN, b.texture((0.5, 0.6, 0.7)))
    for _ in range(16):
        b.obj(abi.PRIM_SPHERE, m, tuple(rng.uniform(-20, 20, 3)) + (float(rng.uniform(0.5, 2.0)),))
    planes = []

    def rot(angle):
        sn, cs = sincos_deg(angle)
        return ("R", sn, cs)

    # YZ rect (plane x = k) under RotateY(90): cos 90 . d_x == sin 90 . d_z cancels exactly
    b.obj(abi.PRIM_YZ_RECT, m, (-3.0, 4.0, -2.0, 5.0, 2.5), xforms=[(abi.XF_ROTATE_Y, (90.0,))])
    planes.append(([rot(90.0)], 0, 2.5))
    # XY rect (plane z = k) under RotateY(30)
    b.obj(abi.PRIM_XY_RECT, m, (-4.0, 3.0, -1.0, 6.0, -7.25), xforms=[(abi.XF_ROTATE_Y, (30.0,))])
    planes.append(([rot(30.0)], 2, -7.25))
    # the cornell box's tall box: Translate(RotateY(-18)(Box)) — faces x = 0, x = 165, z = 0, z = 165
    b.obj(abi.PRIM_BOX, m, (0.0, 0.0, 0.0, 16.5, 33.0, 16.5),
          xforms=[(abi.XF_TRANSLATE, (2.65, 0.0, 2.95)), (abi.XF_ROTATE_Y, (-18.0,))])
    tchain = [("T", (2.65, 0.0, 2.95)), rot(-18.0)]
    planes += [(tchain, 0, 0.0), (tchain, 0, 16.5), (tchain, 2, 0.0), (tchain, 2, 16.5)]
    # a box under RotateY(90)
    b.obj(abi.PRIM_BOX, m, (-2.0, -2.0, -2.0, 3.0, 1.0, 4.0), xforms=[(abi.XF_ROTATE_Y, (90.0,))])
    planes += [([rot(90.0)], 0, -2.0), ([rot(90.0)], 2, 4.0)]
    # two RotateYs (200 then 271.5) around a YZ rect
    b.obj(abi.PRIM_YZ_RECT, m, (-5.0, 5.0, -5.0, 5.0, 1.0),
          xforms=[(abi.XF_ROTATE_Y, (200.0,)), (abi.XF_ROTATE_Y, (271.5,))])
    planes.append(([rot(200.0), rot(271.5)], 0, 1.0))
    # FlipFace(RotateY(200)(XY rect))
    b.obj(abi.PRIM_XY_RECT, m, (-6.0, 6.0, -6.0, 6.0, 3.0),
          xforms=[(abi.XF_FLIP_FACE, (0.0,)), (abi.XF_ROTATE_Y, (200.0,))])
    planes.append(([rot(200.0)], 2, 3.0))
    # plain (unrotated) rect and box too
    b.obj(abi.PRIM_XZ_RECT, m, (-8.0, 8.0, -8.0, 8.0, -1.0))
    b.obj(abi.PRIM_BOX, m, (10.0, 10.0, 10.0, 12.0, 12.0, 12.0))
    return b, planes


def rotated_plane_rays(planes, per_plane, seed=6):
    """per_plane rays per plane; chains of two RotateYs rarely cancel exactly (the search gives up
    on most draws), so they get a tenth of that."""
    rng = np.random.default_rng(seed)
    return np.concatenate([plane_rays(c, a, k, per_plane if len([s for s in c if s[0] == "R"]) < 2 else per_plane // 10,
                                      rng) for c, a, k in planes])
