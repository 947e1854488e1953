"""The C-ABI contract of include/yart.h on the device: concurrent renders on one scene handle,
progress reporting, the block-packed shard format, the RCCL gather and the one-process
multi-device render, and the CLI binary end to end.

References: SURVEY.md §8(b) threading (the reference runs 64 tile jobs concurrently on a shared
read-only scene, main.rs:633-649), RenderUpdate::Progress per rendered row (main.rs:720-721), the
fan-out + stitching of tile results (main.rs:633-660, 747-760), and `raytracer --scene ...`
(main.rs:777-781)."""
import os
import subprocess
import sys
import threading

import numpy as np
import pytest
import torch

import oracle_lib as O
import yart

pytestmark = pytest.mark.gpu


def test_concurrent_renders_on_one_handle():
    """4 host threads, 4 different cameras (and sample plans), ONE scene handle: each result must
    be bitwise its serial render, which itself equals the oracle."""
    p = yart.Preset("cornell-box")
    s = yart.DeviceScene(p)
    W, H, spp = 64, 48, 16
    jobs = []
    for k in range(4):
        cam = yart.make_camera((278.0 + 40 * k, 278.0, -800.0), (278.0, 278.0 - 10 * k, 0.0), 40.0, W / H, 0.0)
        prm = yart.render_params(W, H, spp, 50, samples_per_unit=(0, 3, spp, 5)[k])
        jobs.append((cam, prm))
    serial = [s.render(c, q) for c, q in jobs]
    results = [None] * 4
    errors = []

    def run(k):
        try:
            for _ in range(3):
                results[k] = s.render(*jobs[k])
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    th = [threading.Thread(target=run, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for k in range(4):
        np.testing.assert_array_equal(results[k], serial[k])
    np.testing.assert_array_equal(serial[0], O.OracleScene(p.desc).render(*jobs[0]))


def test_progress_is_monotone_and_complete():
    p = yart.Preset("cornell-box")
    s = yart.DeviceScene(p)
    W, H, spp = 400, 300, 256  # long enough (tens of ms) for several polls
    calls = []
    img = s.render(p.camera(W, H), yart.render_params(W, H, spp, 50), progress=calls.append)
    total = int(O.coverage(W, H).sum())
    assert len(calls) > 1, calls
    assert all(b > a for a, b in zip(calls, calls[1:])), calls
    assert calls[-1] == total
    np.testing.assert_array_equal(img, s.render(p.camera(W, H), yart.render_params(W, H, spp, 50)))


def test_progress_of_a_shard_counts_its_pixels():
    p = yart.Preset("cornell-box")
    s = yart.DeviceScene(p)
    W, H = 100, 60
    calls = []
    s.render(p.camera(W, H), yart.render_params(W, H, 8, 50, shard_index=1, shard_count=3, samples_per_unit=8),
             progress=calls.append)
    bx = (W + 7) // 8
    ys, xs = np.mgrid[0:H, 0:W]
    mine = (((ys // 8) * bx + xs // 8) % 3 == 1) & O.coverage(W, H)
    assert calls[-1] == int(mine.sum())


@pytest.mark.parametrize("spu", [0, 4, 1 << 20])
def test_packed_shard_layout(spu):
    """yart_render_packed_async writes a shard's pixels block by block (slot = (y%8)*8 + x%8)."""
    p = yart.Preset("cornell-box")
    s = yart.DeviceScene(p)
    W, H, spp, n = 52, 36, 4, 3
    cam = p.camera(W, H)
    full = s.render(cam, yart.render_params(W, H, spp, 50))
    cov = O.coverage(W, H)
    bx = (W + 7) // 8
    for k in range(n):
        m = yart.shard_packed_len(W, H, k, n)
        d = torch.zeros(m, dtype=torch.float64, device="cuda:0")
        st = torch.cuda.current_stream()
        s.render_packed_async(cam, yart.render_params(W, H, spp, 50, shard_index=k, shard_count=n, samples_per_unit=spu),
                              d.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        pk = d.cpu().numpy().reshape(-1, 64, 3)
        for j in range(pk.shape[0]):
            b = k + j * n
            for slot in range(64):
                x, y = (b % bx) * 8 + slot % 8, (b // bx) * 8 + slot // 8
                if x < W and y < H and cov[y, x]:
                    np.testing.assert_array_equal(pk[j, slot], full[y, x])


def test_rccl_gather_one_rank_is_the_render():
    """yart_comm_init_rank over one rank + yart_gather_frame_async: packed shard -> frame,
    bitwise the plain render (the N > 1 code path is the same ncclGather with more ranks)."""
    p = yart.Preset("cornell-box")
    s = yart.DeviceScene(p)
    W, H, spp = 80, 64, 8
    cam = p.camera(W, H)
    full = s.render(cam, yart.render_params(W, H, spp, 50))
    comm = yart.Comm(yart.Comm.unique_id(), 1, 0, 0)
    st = torch.cuda.current_stream()
    pk = torch.zeros(yart.shard_packed_len(W, H, 0, 1), dtype=torch.float64, device="cuda:0")
    frame = torch.full((H, W, 3), float("nan"), dtype=torch.float64, device="cuda:0")
    for _ in range(2):
        s.render_packed_async(cam, yart.render_params(W, H, spp, 50), pk.data_ptr(), st.cuda_stream)
        comm.gather_frame_async(pk.data_ptr(), W, H, frame.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(frame.cpu().numpy(), full)
    comm.close()


def test_render_multi_on_one_device_is_the_render():
    p = yart.Preset("cornell-box")
    W, H, spp = 64, 40, 8
    cam = p.camera(W, H)
    ref = yart.DeviceScene(p).render(cam, yart.render_params(W, H, spp, 50))
    m = yart.MultiScene(p, [0])
    calls = []
    for _ in range(2):
        out = m.render(cam, yart.render_params(W, H, spp, 50), progress=calls.append)
        np.testing.assert_array_equal(out, ref)
    r, g = m.last_timing()
    assert r > 0 and g >= 0
    assert calls[-1] == int(O.coverage(W, H).sum())
    m.close()


def test_render_multi_async_on_one_device_is_the_render():
    """yart_render_multi_async (bench.py's one-process N-GPU path) at n = 1: renders, grouped
    ncclGather and unpack enqueued without a host wait, frames alternating over two caller
    streams - every frame bitwise yart_render; the timing covers every frame."""
    p = yart.Preset("cornell-box")
    W, H, spp = 72, 40, 8
    cam = p.camera(W, H)
    prm = yart.render_params(W, H, spp, 50)
    ref = yart.DeviceScene(p).render(cam, prm)
    m = yart.MultiScene(p, [0])
    sts = [torch.cuda.current_stream(), torch.cuda.Stream()]
    frames = [torch.full((H, W, 3), float("nan"), dtype=torch.float64, device="cuda:0") for _ in range(2)]
    for i in range(5):
        with torch.cuda.stream(sts[i % 2]):
            m.render_async(cam, prm, frames[i % 2].data_ptr(), sts[i % 2].cuda_stream)
    torch.cuda.synchronize()
    for f in frames:
        np.testing.assert_array_equal(f.cpu().numpy(), ref)
    r, g, n = m.frame_timing()
    assert n == 5 and r > 0 and g > 0
    m.close()


def test_render_multi_async_evicts_slots_beyond_eight_caller_streams():
    """a multi handle keeps per-caller-stream slots for at most 8 streams; a 9th and 10th
    caller stream take over the least recently used slots (their frames drained first), and a reused
    stream afterwards gets a slot again. Every frame stays bitwise yart_render; yart_multi_query
    reports the latest frame gathered and unpacked once it is done; the per-device timing covers it."""
    p = yart.Preset("cornell-box")
    W, H, spp = 40, 24, 4
    cam = p.camera(W, H)
    prm = yart.render_params(W, H, spp, 50)
    ref = yart.DeviceScene(p).render(cam, prm)
    m = yart.MultiScene(p, [0])
    sts = [torch.cuda.Stream() for _ in range(10)]
    order = list(range(10)) + [0, 3, 9, 1]  # 10 streams (two evictions), then reuse of evicted ones
    frames = [torch.full((H, W, 3), float("nan"), dtype=torch.float64, device="cuda:0") for _ in order]
    for k, i in enumerate(order):
        with torch.cuda.stream(sts[i]):
            m.render_async(cam, prm, frames[k].data_ptr(), sts[i].cuda_stream)
    torch.cuda.synchronize()
    for f in frames:
        np.testing.assert_array_equal(f.cpu().numpy(), ref)
    state, unpacked = m.query()
    assert state == [2] and unpacked == 1
    r, g, n = m.frame_timing()
    assert n >= 8 and r > 0  # frames of evicted slots are dropped from the timing
    dr, dg, dn = m.device_timing()
    assert len(dr) == 1 and dn == n and dr[0] == pytest.approx(r) and dg[0] > 0
    m.close()


def test_wavefront_frames_back_to_back_on_one_stream():
    """ADVICE r03 (status-ring race): on the wavefront path a pass ends at a data-dependent
    iteration j while iterations j+1 .. j+6 are still queued; the next pass or frame on the same
    stream must not re-arm a status slot one of them has yet to write. Twelve frames of different
    spp (so the pass lengths, and the j at which each ends, differ), some split into one-sample
    scratch passes, enqueued back to back on ONE stream with no host wait between them and a small
    path pool (hundreds of iterations per pass): each must be bitwise its megakernel render."""
    p = yart.Preset("bunny")
    W, H = 24, 24
    cam = p.camera(W, H)
    spps = [1, 2, 3, 5, 4, 7, 6, 8, 2, 9, 3, 5]
    with yart.option("mesh_wavefront", 0):
        mega = yart.DeviceScene(p)
        refs = [mega.render(cam, yart.render_params(W, H, spp, 50)) for spp in spps]
    with yart.option("mesh_wavefront", 1), yart.option("wf_pool", 256):
        wf = yart.DeviceScene(p)
    st = torch.cuda.current_stream()
    outs = [torch.zeros((H, W, 3), dtype=torch.float64, device="cuda:0") for _ in spps]
    for k, (spp, out) in enumerate(zip(spps, outs)):
        budget = ((W + 7) // 8) * ((H + 7) // 8) * 64 * 24 * (1 if k % 3 == 1 else 64)  # every third: one sample per pass
        with yart.option("scratch_bytes", budget):
            wf.render_async(cam, yart.render_params(W, H, spp, 50), out.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    for k, (out, ref) in enumerate(zip(outs, refs)):
        np.testing.assert_array_equal(out.cpu().numpy(), ref, err_msg=f"frame {k} (spp {spps[k]})")


@pytest.mark.parametrize("n", [2, 3, 4])
def test_unpack_of_n_packed_shards_is_the_render(n):
    """The root side of the N-rank gather without the transport: shard k rendered by
    yart_render_packed_async into slot k of ONE buffer whose slots are shard 0's packet length
    apart (ncclGather's equal-sized packets), then yart_unpack_shards_async - bitwise the plain
    render. Ragged W and H, so shard 0 holds more blocks than the others; the tails of the smaller
    shards' slots are NaN and must never be read. (The multi-device RCCL transport itself runs only
    on the driver's 8-GPU node.)"""
    p = yart.Preset("cornell-box")
    s = yart.DeviceScene(p)
    W, H, spp = 52, 36, 4  # 7 x 5 = 35 blocks
    cam = p.camera(W, H)
    full = s.render(cam, yart.render_params(W, H, spp, 50))
    stride = yart.shard_packed_len(W, H, 0, n)
    assert stride > yart.shard_packed_len(W, H, n - 1, n)
    recv = torch.full((n * stride,), float("nan"), dtype=torch.float64, device="cuda:0")
    st = torch.cuda.current_stream()
    for k in range(n):
        s.render_packed_async(cam, yart.render_params(W, H, spp, 50, shard_index=k, shard_count=n),
                              recv.data_ptr() + 8 * k * stride, st.cuda_stream)
    frame = torch.full((H, W, 3), float("nan"), dtype=torch.float64, device="cuda:0")
    yart.unpack_shards_async(0, recv.data_ptr(), n, stride, W, H, frame.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(frame.cpu().numpy(), full)


def test_bench_gpus_beyond_the_box_exits_nonzero(repo):
    """On a 1-GPU box, `bench.py --gpus 2` (the driver's command form) refuses instead of
    reporting a 1-GPU number."""
    r = subprocess.run([sys.executable, str(repo / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--no-stats", "--cpu-spp", "0"], capture_output=True, text=True, timeout=300, cwd=str(repo))
    if torch.cuda.device_count() >= 2:
        assert r.returncode == 0 and '"n_gpus": 2' in r.stdout, r.stderr
    else:
        assert r.returncode != 0 and '"n_gpus"' not in r.stdout


def test_cli_end_to_end(tmp_path, repo):
    """bin/yart --scene cornell-box ... writes the PNG; its pixels are the oracle's finalize of the
    oracle's render, byte for byte."""
    out = tmp_path / "sub" / "cb.png"
    exe = repo / "yet-another-raytracer_amd" / "bin" / "yart"
    r = subprocess.run([str(exe), "--scene", "cornell-box", "--width", "64", "--height", "64", "--samples", "8",
                        "--output", str(out), "--assets", str(repo / "assets")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "rendered in" in r.stdout
    from PIL import Image  # noqa: PLC0415 - optional decoder, present in the image
    png = np.asarray(Image.open(out).convert("RGBA"))
    p = yart.Preset("cornell-box")
    want = O.finalize(O.OracleScene(p.desc).render(p.camera(64, 64), yart.render_params(64, 64, 8, 50)), 8)
    np.testing.assert_array_equal(png, want)


def test_cli_gpus_flag_uses_the_multi_device_path(tmp_path, repo):
    out = tmp_path / "cb1.png"
    exe = repo / "yet-another-raytracer_amd" / "bin" / "yart"
    r = subprocess.run([str(exe), "--scene", "cornell-box", "--width", "48", "--height", "32", "--samples", "4",
                        "--gpus", "1", "--output", str(out)], capture_output=True, text=True, timeout=120,
                       cwd=str(repo))
    assert r.returncode == 0, r.stderr
    assert out.exists() and out.stat().st_size > 100
