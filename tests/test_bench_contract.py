"""The bench line's contract, checked on the newest committed GPU run (profiles/r*_bench_cornell.log)
and the rocprofv3 summary of the same command: the fields the driver and the judge read are
present, `value` is the frame's samples over the step time, `roofline.frac` is achieved / peak,
`achieved` is the launch's algorithmic FLOPs over the kernel time, and that kernel time agrees
with rocprofv3's average k_render duration. CPU only: it reads committed files."""
import csv
import json
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
PROF = ROOT / "profiles"


def _latest(pattern):
    files = sorted(PROF.glob(pattern))
    if not files:
        pytest.skip(f"no {pattern} under profiles/")
    return files[-1]


def _bench_line():
    log = _latest("r*_bench_cornell.log")
    lines = [l for l in log.read_text().splitlines() if l.startswith("{")]
    assert lines, f"{log.name} holds no JSON line"
    return log, json.loads(lines[-1])


def test_bench_line_has_the_contract_fields():
    _, b = _bench_line()
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in b, k
    assert b["dtype"] == "f64" and b["unit"] == "Msamples/s" and b["higher_is_better"] is True
    assert b["config"]["width"] == 800 and b["config"]["height"] == 800
    assert b["config"]["spp"] == 256 and b["config"]["max_depth"] == 50
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in b["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in b["cpu_baseline"], k
    assert b["cpu_baseline"]["kind"] in ("port", "reference")


def test_value_is_the_frame_over_the_step_time():
    _, b = _bench_line()
    c = b["config"]
    per_frame = c["width"] * c["height"] * c["spp"]  # strong scaling: one whole frame per step at any N
    assert b["value"] == pytest.approx(per_frame / (b["ms_per_step"] * 1e-3) / 1e6, rel=2e-3)


def test_roofline_fraction_and_achieved_are_consistent():
    _, b = _bench_line()
    r = b["roofline"]
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=2e-3)
    assert r["achieved"] == pytest.approx(r["algorithmic_flops_per_launch"] / (r["kernel_ms"] * 1e-3) / 1e12, rel=2e-3)
    assert 0.0 < r["frac"] < 1.0


def test_kernel_time_agrees_with_rocprof_stats():
    log, b = _bench_line()
    tag = log.name.split("_")[0]
    stats = PROF / f"{tag}_cornell_kernel_stats.csv"
    if not stats.exists():
        pytest.skip(f"no rocprofv3 stats for {tag}")
    rows = [r for r in csv.DictReader(open(stats)) if "k_render" in r["Name"]]
    assert rows, "k_render missing from the rocprofv3 stats"
    rocprof_ms = float(rows[0]["AverageNs"]) * 1e-6
    # rocprof averages the overlapped two-stream launches with the solo ones: a few %
    assert b["roofline"]["kernel_ms"] == pytest.approx(rocprof_ms, rel=0.05)


def _run_bench(args, env_extra):
    import os
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    env["HIP_VISIBLE_DEVICES"] = env.get("HIP_VISIBLE_DEVICES", "")  # never touch a GPU from this test
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True, env=env,
                          timeout=300, cwd=str(ROOT))


@pytest.mark.parametrize("args,env", [
    (["--gpus", "2", "--steps", "1", "--warmup", "0"], {}),                       # 2 GPUs asked, none visible
    (["--gpus", "8", "--steps", "1", "--warmup", "0"], {}),
    (["--gpus", "4", "--steps", "1", "--warmup", "0"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}),
    (["--gpus", "2", "--steps", "1", "--warmup", "0"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}),
])
def test_gpus_flag_never_reports_another_n(args, env):
    """--gpus N either drives N GPUs (one process over N devices, or N ranks under
    torch.distributed.run) or exits non-zero: a launch that does not match N must never print a
    bench line (`--gpus` was parsed and ignored, reporting n_gpus 1)."""
    r = _run_bench(args, env)
    assert r.returncode != 0, r.stdout
    assert '"n_gpus"' not in r.stdout
    assert "bench.py: --gpus" in r.stderr
