"""Pixel-block sharding across ranks and the one collective that assembles the frame.

Block b (8x8 pixels, row-major over ceil(W/8) x ceil(H/8)) belongs to rank b % world — the rule
libyart.so's k_render applies to (shard_index, shard_count) and the oracle restates. Every rank
writes only its own blocks into a zeroed full-frame buffer, so ONE reduce(SUM) to the destination
rank assembles the frame exactly (each pixel has exactly one non-zero contributor)."""
import numpy as np


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
