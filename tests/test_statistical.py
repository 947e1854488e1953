"""Statistical parity with the reference's own generator family.

The reference draws from rand 0.8.5's ThreadRng — ChaCha12 seeded from OS entropy — so no run of it
can be reproduced bit for bit; the build's GPU and oracle share one counter-based Philox stream
instead and agree bitwise (test_gpu_parity.py). What remains to show is that the Philox stream
changes nothing but the noise: renders drawn from independent ChaCha12 streams (the oracle's
independent-stream mode: one sequential stream per sample in the reference's draw order, rejection
loops included) must agree with the Philox renders in distribution. Per pixel-channel z-test over
K independent renders a side, plus an image-level z-test.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
import yart

K = 8  # independent renders per side (seeds): the variance of each side's mean comes from them


def test_chacha_block_known_answers():
    """oracle_chacha_block against the all-zero key / nonce / counter keystreams: ChaCha20
    (RFC 7539 A.1, test vector #1), ChaCha12 and ChaCha8 (Strombergson's ChaCha test vectors,
    TC1 256-bit key)."""
    L = O.lib()
    inp = (C.c_uint32 * 16)(*([0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + [0] * 12))
    out = (C.c_uint32 * 16)()
    want = {10: "76b8e0ada0f13d90405d6ae55386bd28", 6: "9bf49a6a0755f953811fce125f2683d5",
            4: "3e00ef2f895f40d67f5bb8e81f09a5a1"}
    L.oracle_chacha_block.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_int]
    for double_rounds, hexs in want.items():
        L.oracle_chacha_block(inp, out, double_rounds)
        assert np.array(list(out), dtype="<u4").tobytes()[:16].hex() == hexs


def _stack(render, seeds):
    return np.stack([render(s) for s in seeds])  # (K, H, W, 3) sums


def _z_tests(a, b, spp):
    """a, b: (K, H, W, 3) per-render sums of two independent sets. Returns per-channel z and the
    image-level z of the per-render image means."""
    ma, mb = a.mean(0) / spp, b.mean(0) / spp
    va, vb = a.var(0, ddof=1) / spp ** 2 / a.shape[0], b.var(0, ddof=1) / spp ** 2 / b.shape[0]
    den = np.sqrt(va + vb)
    ok = den > 0
    z = np.zeros_like(ma)
    z[ok] = (ma[ok] - mb[ok]) / den[ok]
    ia, ib = a.reshape(a.shape[0], -1).mean(1), b.reshape(b.shape[0], -1).mean(1)
    z_img = (ia.mean() - ib.mean()) / np.sqrt(ia.var(ddof=1) / len(ia) + ib.var(ddof=1) / len(ib))
    return z[ok], z_img


def _check(z, z_img):
    # K = 8 per side: each variance has 7 dof, |z| has t-like tails (P(|t_14| > 4.5) ~ 5e-4)
    assert np.mean(np.abs(z) > 4.5) <= 0.005, np.sort(np.abs(z))[-10:]
    assert 0.6 < np.mean(np.abs(z)) < 1.0   # E|Z| = 0.80 for a standard normal
    assert abs(z_img) < 4.5, z_img


@pytest.mark.parametrize("scene,W,H,spp,depth", [("cornell-box", 32, 32, 64, 50), ("random-scene", 32, 24, 32, 50)])
def test_philox_and_independent_chacha_streams_agree(scene, W, H, spp, depth):
    p = yart.Preset(scene)
    cam = p.camera(W, H)
    s = O.OracleScene(p.desc)
    philox = _stack(lambda seed: s.render(cam, yart.render_params(W, H, spp, depth, seed=seed)), range(1, K + 1))
    chacha = _stack(lambda seed: s.render(cam, yart.render_params(W, H, spp, depth, seed=seed), chacha=True),
                    range(101, 101 + K))
    assert not np.array_equal(philox[0], chacha[0])
    _check(*_z_tests(philox, chacha, spp))


@pytest.mark.gpu
@pytest.mark.parametrize("scene,W,H,spp", [("cornell-box", 32, 32, 64), ("random-scene", 32, 24, 32),
                                           ("bunny", 24, 24, 32), ("david", 32, 18, 32)])
def test_gpu_render_agrees_with_independent_chacha_streams(scene, W, H, spp):
    """The HIP path (Philox) against the oracle's ChaCha12 streams drawn in the reference's order
    (main.rs:692-697, camera.rs:25-33, material.rs:276,311, pdf.rs:16-17,92, hittable.rs:119):
    the cornell box, the random scene (metal fuzz, dispersive glass, negative albedos) and the two
    mesh scenes - the bunny stand-in's SF66 glass and the david pair, white and glass (the mesh
    scenes on the wavefront path)."""
    p = yart.Preset(scene)
    cam = p.camera(W, H)
    dev = yart.DeviceScene(p.desc)
    s = O.OracleScene(p.desc)
    gpu = _stack(lambda seed: dev.render(cam, yart.render_params(W, H, spp, 50, seed=seed)), range(1, K + 1))
    chacha = _stack(lambda seed: s.render(cam, yart.render_params(W, H, spp, 50, seed=seed), chacha=True),
                    range(101, 101 + K))
    assert not np.array_equal(gpu[0], chacha[0])
    _check(*_z_tests(gpu, chacha, spp))


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["bunny", "david"])
def test_gpu_mesh_render_agrees_with_chacha_streams_at_higher_power(scene):
    """the mesh scenes at 64x64 and 128 spp with K = 12 renders a side (the
    low-power test above runs them at 24x24 / 32x18 and 32 spp, K = 8): 12,288 pixel-channels, each
    a mean of 1,536 samples a side, so a per-channel bias of a few percent of a pixel's noise shows
    as a shift of the |z| distribution. Ties the Philox stream to the reference's draw semantics
    (main.rs:692-697, material.rs:276,311, pdf.rs:16-17,92) where the glass and the mesh walk are."""
    k, W, H, spp = 12, 64, 64, 128
    p = yart.Preset(scene)
    cam = p.camera(W, H)
    dev = yart.DeviceScene(p.desc)
    s = O.OracleScene(p.desc)
    gpu = _stack(lambda seed: dev.render(cam, yart.render_params(W, H, spp, 50, seed=seed)), range(1, k + 1))
    chacha = _stack(lambda seed: s.render(cam, yart.render_params(W, H, spp, 50, seed=seed), chacha=True),
                    range(201, 201 + k))
    z, z_img = _z_tests(gpu, chacha, spp)
    assert z.size > 5000
    _check(z, z_img)
