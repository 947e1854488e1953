"""World-size 2 and 3 gloo runs of the multi-GPU data path on CPU: each rank renders its pixel
blocks (the CPU restatement standing in for the device kernel, same (shard_index, shard_count)
rule) and the frame is assembled on rank 0 three ways — the packed-shard gather bench.py issues
(libyart's ncclGather wire format, restated by yart.shard.PackedGather), and the two test-only
reference forms (a full-frame reduce, a pixel-index gather). Each must equal the single-process
render bitwise."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O
import yart
from yart.shard import PackedGather, ShardGather, assemble_frame, block_owner, packed_pixels

W, H, SPP, DEPTH = 40, 24, 2, 50


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = yart.Preset("cornell-box")
    cam = p.camera(W, H)
    mine_np = O.OracleScene(p.desc).render(cam, yart.render_params(W, H, SPP, DEPTH, shard_index=rank, shard_count=world),
                                           threads=2)
    mine = torch.from_numpy(mine_np)
    frame = torch.zeros_like(mine)
    for _ in range(2):  # repeated steps must not double count (bench.py reuses the buffers)
        assemble_frame(mine, frame, dist, dst=0)
    if rank == 0:
        np.save(out_path, frame.numpy())
    # bench.py's path: each rank's own pixels, one gather; the non-owned part of `mine` is garbage
    # here to show it is never read
    mine2 = mine.clone()
    mine2[torch.from_numpy(block_owner(W, H, world) != rank)] = float("nan")
    g = ShardGather(W, H, 3, world, rank, torch.device("cpu"))
    frame2 = torch.full_like(mine, -1.0)
    for _ in range(2):
        g(mine2, frame2, dist)
    if rank == 0:
        np.save(out_path.replace(".npy", "_gather.npy"), frame2.numpy())
    # bench.py's N > 1 data path: the rank's block-packed shard (libyart's wire format) and the
    # packet gather libyart issues as one ncclGather; unused / uncovered slots hold garbage
    pix = packed_pixels(W, H, world, rank)
    packed = torch.full((len(pix), 3), float("nan"), dtype=torch.float64)
    keep = pix >= 0
    packed[torch.from_numpy(keep)] = mine.view(-1, 3)[torch.from_numpy(pix[keep])]
    pg = PackedGather(W, H, world, rank, torch.device("cpu"))
    frame3 = torch.zeros_like(mine)
    for _ in range(2):
        pg(packed, frame3, dist)
    if rank == 0:
        np.save(out_path.replace(".npy", "_packed.npy"), frame3.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_two_rank_gloo_frame_assembly(tmp_path, world):
    out = tmp_path / "frame.npy"
    mp.spawn(_worker, args=(world, _free_port(), str(out)), nprocs=world, join=True)
    p = yart.Preset("cornell-box")
    full = O.OracleScene(p.desc).render(p.camera(W, H), yart.render_params(W, H, SPP, DEPTH), threads=2)
    np.testing.assert_array_equal(np.load(out), full)
    np.testing.assert_array_equal(np.load(str(out).replace(".npy", "_gather.npy")), full)
    np.testing.assert_array_equal(np.load(str(out).replace(".npy", "_packed.npy")), full)


def test_packed_pixels_partition_the_covered_frame():
    for (w, h, n) in [(40, 24, 2), (37, 29, 3), (400, 225, 8), (1920, 1080, 8)]:
        seen = np.concatenate([packed_pixels(w, h, n, r) for r in range(n)])
        seen = seen[seen >= 0]
        assert len(seen) == len(np.unique(seen))
        cov = O.coverage(w, h).reshape(-1)
        assert set(seen.tolist()) == set(np.flatnonzero(cov).tolist())
        # shard 0 is the largest packet (ncclGather's equal-size packets)
        assert all(len(packed_pixels(w, h, n, r)) <= len(packed_pixels(w, h, n, 0)) for r in range(n))


def test_block_owner_matches_shard_renders():
    p = yart.Preset("cornell-box")
    cam = p.camera(W, H)
    s = O.OracleScene(p.desc)
    owner = block_owner(W, H, 3)
    full = s.render(cam, yart.render_params(W, H, SPP, DEPTH), threads=2)
    for r in range(3):
        part = s.render(cam, yart.render_params(W, H, SPP, DEPTH, shard_index=r, shard_count=3), threads=2)
        np.testing.assert_array_equal(part[owner == r], full[owner == r])
        assert (part[owner != r] == 0).all()
