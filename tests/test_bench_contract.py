"""The bench line's contract, checked on the newest committed GPU run (profiles/r*_bench_cornell.log)
and the rocprofv3 summary of the same command: the fields the driver and the judge read are
present, `value` is the frame's samples over the step time, `roofline.frac` is achieved / peak,
`achieved` is the launch's algorithmic FLOPs over the kernel time, and that kernel time agrees
with rocprofv3's average k_render duration. CPU only: it reads committed files."""
import csv
import subprocess
import sys
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


def test_watchdog_names_the_stalled_stage_and_exits_3():
    """yart/watchdog.py: a stage that overruns its deadline prints ONE JSON line naming the stage
    (and the watchdog's diagnosis of where the frame stands) and ends the process with exit 3."""
    code = ("import sys, time; sys.path.insert(0, 'yet-another-raytracer_amd');"
            "from yart.watchdog import Watchdog;"
            "wd = Watchdog('m', poll_s=0.05);"
            "ctx = wd.stage('gather', 0.5, lambda: {'frame': 'gather (device(s) [1] not through ncclGather)'});"
            "ctx.__enter__(); time.sleep(30); print('not reached')")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, cwd=str(ROOT))
    assert r.returncode == 3, (r.returncode, r.stdout, r.stderr)
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and "not reached" not in r.stdout
    e = lines[0]
    assert e["stage"] == "gather" and "gather" in e["error"] and e["value"] is None
    assert "device(s) [1]" in e["detail"]["frame"]


def test_bench_stalled_first_stage_exits_nonzero_naming_it():
    """bench.py's N > 1 per-rank path with its peer rank never arriving: the gloo control plane's
    setup stalls (a real stall, not an injected one), and with a 3 s deadline the run must end with
    exit 3 and one JSON line whose error names that stage — not a silent kill at the driver's limit.
    Runs on the CPU: the stage comes before any GPU call."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
           "YART_BENCH_DEADLINE_S": "3"}
    r = _run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0"], env)
    assert r.returncode == 3, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and lines[0]["value"] is None
    assert lines[0]["stage"].startswith("process group init") and "deadline" in lines[0]["error"]


def test_device_balance_fields():
    """an N-GPU line says which device was slowest and how long each waited in
    the gather, so a scaling shortfall can be told apart as imbalance or gather cost."""
    sys.path.insert(0, str(ROOT))
    import importlib
    bench = importlib.import_module("bench")
    b = bench.device_balance([4.10, 4.20, 4.00, 4.30], [0.40, 0.30, 0.50, 0.20])
    assert b["per_device_render_ms"] == [4.1, 4.2, 4.0, 4.3]
    assert b["per_device_gather_ms"] == [0.4, 0.3, 0.5, 0.2]
    assert b["render_max_over_mean"] == pytest.approx(4.30 / 4.15, rel=1e-3)
    assert b["slowest_device"] == 3


def test_rehearsal_line_carries_the_per_device_fields():
    """The committed N = 2 rehearsal of bench.py's per-rank path (profiles/r05_rehearse_n2.log,
    YART_BENCH_SAME_DEVICE=1: both ranks on one GPU, gloo gather) carries the per-device fields."""
    logs = sorted(PROF.glob("r0[5-9]*_rehearse_n2.log"))
    if not logs:
        pytest.skip("no r05+ rehearsal log")
    lines = [json.loads(l) for l in logs[-1].read_text().splitlines() if l.startswith("{")]
    assert lines, logs[-1]
    b = lines[-1]
    assert b["n_gpus"] == 2
    bal = b["device_balance"]
    assert len(bal["per_device_render_ms"]) == 2 and len(bal["per_device_gather_ms"]) == 2
    assert bal["render_max_over_mean"] >= 1.0
    assert b["roofline"]["per_device_render_ms"] == bal["per_device_render_ms"]
    assert len(b["config"]["build_id"]) == 64


def test_bench_line_build_id_matches_the_pmc_snapshot():
    """the newest bench line names the library build it timed, and the PMC
    snapshot it took traffic from belongs to the same build."""
    _, b = _bench_line()
    bid = b["config"].get("build_id")
    if bid is None:
        pytest.skip("bench line older than build ids")
    pmc = json.loads((PROF / "pmc_render_cornell.json").read_text())
    if b["roofline"]["traffic"] is not None:
        assert pmc.get("build_id") == bid


def _check_david(d, n):
    assert d["n_gpus"] == n and d["spp"] > 0 and d["frames"] >= 1 and d["warmup"] == 1
    assert d["workload"].startswith("david 1920x1080x")
    assert d["msamples_per_s"] == pytest.approx(1920 * 1080 * d["spp"] / (d["ms_per_frame"] * 1e-3) / 1e6, rel=2e-3)
    bal = d["device_balance"]
    assert len(bal["per_device_render_ms"]) == n and bal["render_max_over_mean"] >= 1.0
    if n > 1:
        assert len(bal["per_device_gather_ms"]) == n
        assert d["frame_check"] == "assembled frame bitwise equal to the one-device render"


def test_bench_line_carries_the_david_sub_record():
    """the bench line also times BASELINE configs[4] (david 1920x1080, the
    config BASELINE assigns to 8 GPUs) at reduced spp on the same N-GPU path, so the driver's
    first 8-GPU run says whether david scales; checked on the newest N = 1 line and the newest
    N = 2 rehearsal (r06+)."""
    log, b = _bench_line()
    if "david" not in b:
        pytest.skip(f"{log.name} predates the david sub-record")
    _check_david(b["david"], b["n_gpus"])
    logs = sorted(PROF.glob("r0[6-9]*_rehearse_n2.log"))
    if not logs:
        pytest.skip("no r06+ rehearsal log")
    r = [json.loads(l) for l in logs[-1].read_text().splitlines() if l.startswith("{")][-1]
    _check_david(r["david"], 2)
