"""Edge sharding for multi-GPU update()/BA.

Keyframes are split into contiguous blocks balanced by out-degree; a rank owns
every edge whose source frame ii is in its block, plus those frames' disps,
damping, net/inp and correlation volumes.  poses and fmaps are replicated.
Every per-edge stage (reprojection, lookup, update operator, GraphAgg) and
every depth-frame Schur term is then local; the only exchange is one
all_reduce of the reduced camera system per Gauss-Newton iteration.
"""
import numpy as np


def frame_blocks(ii, num_frames, world):
    """contiguous [lo, hi) per rank with roughly equal out-degree."""
    deg = np.bincount(np.asarray(ii), minlength=num_frames).astype(np.float64)
    cum = np.cumsum(deg)
    total = cum[-1] if len(cum) else 0.0
    bounds = [0]
    for r in range(1, world):
        bounds.append(int(np.searchsorted(cum, total * r / world, side="left")) + 1)
    bounds.append(num_frames)
    bounds = np.maximum.accumulate(np.clip(bounds, 0, num_frames))
    return [(int(bounds[r]), int(bounds[r + 1])) for r in range(world)]


def shard_edges(ii, jj, num_frames, rank, world):
    ii = np.asarray(ii)
    jj = np.asarray(jj)
    lo, hi = frame_blocks(ii, num_frames, world)[rank]
    m = (ii >= lo) & (ii < hi)
    return ii[m], jj[m], (lo, hi)
