"""Pixel-block sharding across ranks and the one collective that assembles the frame.

Block b (8x8 pixels, row-major over ceil(W/8) x ceil(H/8)) belongs to rank b % world — the rule
libyart.so's k_render applies to (shard_index, shard_count) and the oracle restates. Every rank
renders only its own blocks into a zeroed full-frame buffer. Two ways to assemble rank dst's frame:

* `assemble_frame`: ONE reduce(SUM) of the full frames — exact, since each pixel has exactly one
  non-zero contributor; simple, but every rank ships W*H*24 bytes through the ring.
* `ShardGather`: each rank packs its own pixels (1/world of the frame) and ONE gather to dst
  collects them over the point-to-point xGMI links, where they are scattered back into place —
  the same bits, world x less data (the xGMI links are per peer, so the gather is one hop each).
"""
import numpy as np
import torch


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
