"""Pixel-block sharding across ranks and the collectives that assemble the frame (Python side).

Block b (8x8 pixels, row-major over ceil(W/8) x ceil(H/8)) belongs to rank b % world — the rule
libyart.so's k_render applies to (shard_index, shard_count) and the oracle restates.

On the product path the frame is assembled inside libyart (yart_gather_frame_async: ONE
ncclGather of block-packed shards + k_unpack_shards; yart_render_multi_async for one process
driving N devices). What lives here:

* `PackedGather` — the same packets and unpack restated over torch.distributed, for backends
  libyart cannot drive: bench.py's gloo rehearsal on one device and its torch-RCCL fallback;
* `packed_pixels`, `block_owner`, `covered_axis` — the layout, for tests;
* `assemble_frame` (a full-frame reduce) and `ShardGather` (pixel-index gather) — TEST-ONLY
  reference forms the CPU tests (tests/test_distributed.py) check the packed gather against; no
  product path uses them.
"""
import numpy as np
import torch


def covered_axis(n):
    """main.rs:636-647: the 8 crops of width n // 8 start at n * col // 8."""
    m = np.zeros(n, dtype=bool)
    cw = n // 8
    for col in range(8):
        x0 = n * col // 8
        m[x0:x0 + cw] = True
    return m


def block_owner(width, height, world):
    """(H, W) int array: the rank that renders each pixel."""
    bx = (width + 7) // 8
    ys, xs = np.mgrid[0:height, 0:width]
    return ((ys // 8) * bx + (xs // 8)) % world


def assemble_frame(mine, frame, dist, dst=0):
    """Copy this rank's shard into `frame` and reduce-sum all ranks' shards into dst's `frame`.
    `mine` must keep only this rank's pixels (zeros elsewhere) across calls; `frame` is scratch on
    non-destination ranks."""
    frame.copy_(mine)
    dist.reduce(frame, dst=dst, op=dist.ReduceOp.SUM)
    return frame


class ShardGather:
    """Packs this rank's pixels of an (H, W, C) frame, gathers every rank's pack on `dst` and
    scatters them into dst's frame. The index tensors are built once; a step is one index_select,
    one gather and (on dst) one index_copy per rank."""

    def __init__(self, width, height, channels, world, rank, device, dtype=torch.float64, dst=0):
        owner = block_owner(width, height, world).reshape(-1)
        self.idx = [torch.from_numpy(np.flatnonzero(owner == r)).to(device) for r in range(world)]
        self.n = [int(i.numel()) for i in self.idx]
        self.n_max = max(self.n)
        self.rank, self.world, self.dst, self.channels = rank, world, dst, channels
        self.send = torch.zeros((self.n_max, channels), dtype=dtype, device=device)
        self.recv = ([torch.zeros_like(self.send) for _ in range(world)] if rank == dst else None)

    def __call__(self, mine, frame, dist):
        """`mine`: this rank's render (its pixels; the rest is not read). On dst, `frame` is
        overwritten with every rank's pixels; elsewhere it is not touched."""
        r = self.rank
        torch.index_select(mine.reshape(-1, self.channels), 0, self.idx[r], out=self.send[:self.n[r]])
        dist.gather(self.send, self.recv, dst=self.dst)
        if r == self.dst:
            flat = frame.view(-1, self.channels)
            for k in range(self.world):
                flat.index_copy_(0, self.idx[k], self.recv[k][:self.n[k]])
        return frame


def packed_pixels(width, height, world, rank):
    """For shard `rank` of `world` in libyart's block-packed layout (yart_shard_packed_len): the
    frame pixel index (y * W + x) of every slot, -1 for slots outside the frame or the crop grid.
    Slot s of local block j is pixel (x, y) of global block b = rank + j * world with
    x = (b % bx) * 8 + s % 8, y = (b // bx) * 8 + s // 8."""
    bx, by = (width + 7) // 8, (height + 7) // 8
    blocks = np.arange(rank, bx * by, world)
    s = np.arange(64)
    x = (blocks[:, None] % bx) * 8 + s[None, :] % 8
    y = (blocks[:, None] // bx) * 8 + s[None, :] // 8
    cx, cy = covered_axis(width), covered_axis(height)
    ok = (x < width) & (y < height)
    ok[ok] = cx[x[ok]] & cy[y[ok]]
    return np.where(ok, y * width + x, -1).reshape(-1)


class PackedGather:
    """The frame gather libyart does natively (yart_gather_frame_async: one ncclGather + unpack
    kernel), restated over torch.distributed for backends libyart cannot drive (gloo rehearsals
    on one device, CPU tests): every rank sends its packed shard (equal-sized packets of the
    largest shard's length), dst scatters them into the frame. Bitwise the native path."""

    def __init__(self, width, height, world, rank, device, dtype=torch.float64, dst=0):
        self.rank, self.world, self.dst = rank, world, dst
        self.n_max = len(packed_pixels(width, height, world, 0))  # shard 0 is the largest
        self.send = torch.zeros((self.n_max, 3), dtype=dtype, device=device)
        if rank == dst:
            self.recv = [torch.zeros_like(self.send) for _ in range(world)]
            self.idx, self.sel = [], []
            for r in range(world):
                pix = packed_pixels(width, height, world, r)
                keep = np.flatnonzero(pix >= 0)
                self.sel.append(torch.from_numpy(keep).to(device))
                self.idx.append(torch.from_numpy(pix[keep]).to(device))
        else:
            self.recv = None

    def __call__(self, packed, frame, dist, group=None):
        """`packed`: this rank's packed shard (n * 64 * 3 doubles); on dst `frame` (H, W, 3) gets
        every covered pixel (uncovered ones are left as they are: zero them once)."""
        n = min(packed.numel() // 3, self.n_max)
        self.send[:n].copy_(packed.view(-1, 3)[:n])
        dist.gather(self.send, self.recv, dst=self.dst, group=group)
        if self.rank == self.dst:
            flat = frame.view(-1, 3)
            for r in range(self.world):
                flat.index_copy_(0, self.idx[r], self.recv[r].index_select(0, self.sel[r]))
        return frame
