"""The experiment records kept under tools/ (VERDICT r04 item 8): every patch that DESIGN.md cites as
a measured-and-dropped experiment must still apply to this tree's kernels.hip and compile for gfx950
(device syntax check), or be removed — a record that no longer applies has silently rotted. CPU only."""
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
PATCHES = sorted((ROOT / "tools").glob("patch_*.py"))
DIFFS = sorted((ROOT / "tools").glob("exp_*.diff"))


def _syntax_check(src):
    hipcc = "/opt/rocm/bin/hipcc"
    if not Path(hipcc).exists():
        pytest.skip("no hipcc")
    r = subprocess.run([hipcc, "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                        f"-I{ROOT / 'build' / 'gen'}", f"-I{ROOT / 'yet-another-raytracer_amd' / 'csrc'}",
                        "--cuda-device-only", "-fsyntax-only", str(src)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.parametrize("patch", PATCHES, ids=lambda p: p.name)
def test_patch_applies_and_compiles(patch, tmp_path):
    if not (ROOT / "build" / "gen" / "cie_xyz.inc").exists():
        pytest.skip("tables not generated (make)")
    k = tmp_path / "kernels.hip"
    shutil.copy(ROOT / "yet-another-raytracer_amd" / "csrc" / "kernels.hip", k)
    r = subprocess.run([sys.executable, str(patch), str(k)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, f"{patch.name} no longer applies to kernels.hip: {r.stderr[-1500:]}"
    assert k.read_text() != (ROOT / "yet-another-raytracer_amd" / "csrc" / "kernels.hip").read_text()
    _syntax_check(k)


@pytest.mark.parametrize("diff", DIFFS, ids=lambda p: p.name)
def test_diff_applies(diff):
    r = subprocess.run(["git", "apply", "--check", str(diff)], capture_output=True, text=True, cwd=str(ROOT))
    assert r.returncode == 0, f"{diff.name} no longer applies: {r.stderr}"
