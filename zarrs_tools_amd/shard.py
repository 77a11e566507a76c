"""Per-GPU partition of the chunk work queue.

The reference processes output chunks independently on a rayon pool
(guided_filter.rs:260-316). Across GPUs the same independence gives a plain split with no
collective: rank g owns the contiguous chunk rows [g*n/G, (g+1)*n/G) along axis 0 and loads its
slab plus the 2r halo rows the reference's ArraySubsetOverlap would read
(array_subset_overlap.rs:11-35), clamped at the array edges.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class SlabAssignment:
    rank: int
    world: int
    chunk_row_begin: int   # first owned chunk row (axis 0)
    chunk_row_end: int     # one past the last owned chunk row
    out_z0: int            # first owned output row
    out_nz: int            # owned output rows
    in_z0: int             # first input row loaded (owned rows minus the halo, clamped)
    in_nz: int             # input rows loaded


def slab_assignment(rank: int, world: int, n_rows: int, chunk_rows: int, halo: int
                    ) -> SlabAssignment:
    """Contiguous split of the ceil(n_rows/chunk_rows) chunk rows over `world` ranks."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    n_chunk_rows = -(-n_rows // chunk_rows) if n_rows > 0 else 0
    c0 = rank * n_chunk_rows // world
    c1 = (rank + 1) * n_chunk_rows // world
    z0 = min(c0 * chunk_rows, n_rows)
    z1 = min(c1 * chunk_rows, n_rows)
    i0 = max(z0 - halo, 0)
    i1 = min(z1 + halo, n_rows)
    if z1 <= z0:
        i0 = i1 = z0
    return SlabAssignment(rank, world, c0, c1, z0, z1 - z0, i0, i1 - i0)
