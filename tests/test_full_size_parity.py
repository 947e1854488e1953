"""Parity at the BASELINE.json configurations themselves, on the production work plan.

The GPU renders each config's FULL frame exactly as bench.py / tools/bench_configs.py do (one
yart_render call, samples_per_unit = 0: the library's own chunk/pass plan, so C2 runs the
8-10-spp units of its persistent-wave plan; C5 in one scratch pass, and in 12 under a 4 GiB budget). The oracle
(oracle/, the CPU restatement of main.rs:628-708) then renders either the same full frame (C1, C2:
cheap enough) or only a fixed, spread subset of 8x8 blocks (b % stride == 0, through the same
shard rule), and the two must be BITWISE equal on every pixel the oracle rendered.

Sizes: C1 two-spheres 400x225x16 d8, C2 cornell-box 800x800x256 d50, C3 random-scene
1200x800x500, C4 bunny (sycee stand-in) 800x800x512, C5 david 1920x1080x1024 d50.
"""
import os

import numpy as np
import pytest

import oracle_lib as O
import yart

pytestmark = pytest.mark.gpu

# oracle threads: the GPU box's CPU share is 16 (os.cpu_count() there reports the whole machine)
THREADS = min(16, os.cpu_count() or 1)

# config, scene, W, H, spp, depth, oracle block stride (1 = the whole frame)
CONFIGS = [
    ("C1", "two-spheres", 400, 225, 16, 8, 1),
    ("C2", "cornell-box", 800, 800, 256, 50, 1),
    ("C3", "random-scene", 1200, 800, 500, 50, 97),
    ("C4", "bunny", 800, 800, 512, 50, 61),
    ("C5", "david", 1920, 1080, 1024, 50, 997),
]


def block_mask(w, h, stride):
    bx = (w + 7) // 8
    ys, xs = np.mgrid[0:h, 0:w]
    return (((ys // 8) * bx + (xs // 8)) % stride) == 0


@pytest.mark.parametrize("cfg,scene,W,H,spp,depth,stride", CONFIGS, ids=[c[0] for c in CONFIGS])
def test_config_full_frame_bitwise(cfg, scene, W, H, spp, depth, stride):
    p = yart.Preset(scene)
    cam = p.camera(W, H)
    s = yart.DeviceScene(p)
    gpu = s.render(cam, yart.render_params(W, H, spp, depth))  # production plan (samples_per_unit = 0)
    assert np.isfinite(gpu).all()
    cov = O.coverage(W, H)
    assert (gpu[~cov] == 0).all()
    oracle = O.OracleScene(p.desc).render(cam, yart.render_params(W, H, spp, depth, shard_index=0, shard_count=stride),
                                          threads=THREADS)
    m = block_mask(W, H, stride) & cov
    assert m.sum() >= 64 * 8, "the subset must hold several blocks"
    bad = np.argwhere((gpu != oracle).any(axis=-1) & m)
    assert len(bad) == 0, f"{cfg}: {len(bad)} of {m.sum()} checked pixels differ, e.g. (y, x) {bad[:4].tolist()}"
    # the oracle rendered nothing outside its blocks; the GPU rendered everything covered
    assert (oracle[~m] == 0).all()
    assert (gpu[cov].sum(axis=-1) != 0).mean() > 0.5
    # the product's output, the RGBA8 image (main.rs:710-718): the device's k_finalize of the GPU
    # frame equals the oracle's finalize (glibc pow) of the oracle frame on every checked pixel, and
    # the oracle's finalize of the GPU frame on every pixel of the frame
    g8 = yart.finalize_rgba8(gpu, spp)
    o8 = O.finalize(oracle, spp)
    bad8 = np.argwhere((g8 != o8).any(axis=-1) & m)
    assert len(bad8) == 0, f"{cfg}: {len(bad8)} RGBA8 pixels differ, e.g. (y, x) {bad8[:4].tolist()}"
    np.testing.assert_array_equal(g8, O.finalize(gpu, spp))


def test_c5_in_one_pass_and_in_scratch_passes_agree():
    """C5's sample scratch is 49.8 MB per sample, 51 GB for the frame: the auto budget (min(16 GiB,
    device memory / 8), capi.cpp scratch_budget) renders it in 7 overlapped passes over two 8 GiB
    halves (r06), a 4 GiB budget in 25 over two 2 GiB halves, a 64 GiB budget in ONE pass; each pass
    with its own accumulate, the odd ones rendered on a helper stream. The plans must give the same
    frame bit for bit (k_accumulate adds samples in sample order whatever the split), so the
    oracle check of test_config_full_frame_bitwise[C5] (the auto plan) covers them all."""
    W, H, spp, depth = 1920, 1080, 1024, 50
    per_sample = ((W + 7) // 8) * ((H + 7) // 8) * 64 * 3 * 8
    assert yart.get_option("scratch_bytes") == 0  # auto
    assert per_sample * spp <= 64 << 30 and (16 << 30) // per_sample < spp
    p = yart.Preset("david")
    cam = p.camera(W, H)
    s = yart.DeviceScene(p)
    auto = s.render(cam, yart.render_params(W, H, spp, depth))
    with yart.option("scratch_bytes", 64 << 30):
        one = s.render(cam, yart.render_params(W, H, spp, depth))
    with yart.option("scratch_bytes", 4 << 30):
        split = s.render(cam, yart.render_params(W, H, spp, depth))
    assert np.array_equal(one, auto)
    assert np.array_equal(one, split)
