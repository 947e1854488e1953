"""Committed golden fixtures (tests/golden/make_golden.py): the CPU restatement must keep
reproducing them bitwise (CPU), and so must the device path (GPU)."""
from pathlib import Path

import numpy as np
import pytest

import oracle_lib as O
import yart

GOLDEN = sorted((Path(__file__).resolve().parent / "golden").glob("*.npz"))


def _load(path):
    g = np.load(path)
    return g, yart.Preset(str(g["scene"]))


@pytest.mark.parametrize("path", GOLDEN, ids=[p.stem for p in GOLDEN])
def test_oracle_reproduces_golden(path):
    g, p = _load(path)
    w, h, spp, depth = int(g["width"]), int(g["height"]), int(g["spp"]), int(g["depth"])
    xyz = O.OracleScene(p.desc).render(p.camera(w, h), yart.render_params(w, h, spp, depth, seed=int(g["seed"])))
    np.testing.assert_array_equal(xyz, g["xyz"])
    np.testing.assert_array_equal(O.finalize(xyz, spp), g["rgba"])


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN, ids=[p.stem for p in GOLDEN])
def test_device_reproduces_golden(path):
    g, p = _load(path)
    w, h, spp, depth = int(g["width"]), int(g["height"]), int(g["spp"]), int(g["depth"])
    xyz = yart.DeviceScene(p).render(p.camera(w, h), yart.render_params(w, h, spp, depth, seed=int(g["seed"])))
    np.testing.assert_array_equal(xyz, g["xyz"])
    rgba = yart.finalize_rgba8(xyz, spp)
    np.testing.assert_array_equal(rgba, g["rgba"])
