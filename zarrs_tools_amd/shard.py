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


# ---- zarrs_ome pyramid: octant ownership ------------------------------------
#
# The reference computes level i from level i-1 chunk by chunk (zarrs_ome.rs:515-738). Across GPUs
# the level-0 array is split into boxes whose boundaries are multiples of factor^L (L = the number
# of levels), so every level's downsample windows (exact_chunks, downsample.rs:72-97) stay inside
# one box: each rank computes all L levels of its box locally, with no exchange, and the union of
# the ranks' levels is the global pyramid. Output chunks that span several boxes (the upper levels,
# smaller than a chunk per rank) are assembled on the host from the ranks' sub-blocks
# (assemble_chunk) before they are encoded.


def pyramid_level_shapes(shape, factor, max_levels: int) -> list:
    """Level shapes and stop rule of zarrs_ome.rs:515-560, :731-737 (output = max(n / f, 1))."""
    cur, out = list(shape), []
    for _ in range(max_levels):
        nxt = [max(s // f, 1) for s, f in zip(cur, factor)]
        out.append(tuple(nxt))
        cur = nxt
        if all(f == 1 or s == 1 for f, s in zip(factor, nxt)):
            break
    return out


@dataclass(frozen=True)
class OctantAssignment:
    rank: int
    world: int
    grid: tuple          # ranks per axis (their product may be < world: the rest own nothing)
    coord: tuple         # this rank's position in the rank grid (None: owns nothing)
    start: tuple         # level-0 box start (multiple of factor^local_levels per axis)
    shape: tuple         # level-0 box shape (zeros: owns nothing)
    local_levels: int    # levels every rank computes on its own box (1..L)
    level_boxes: tuple   # ((start, shape) of the owned box of level k) for k = 1..local_levels
    levels: int          # all levels of the pyramid; levels past local_levels are computed by
                         # rank 0 from the assembled level local_levels (small by construction)


def _rank_grid(world: int, units) -> tuple:
    """Factor `world` over the axes, each prime factor (largest first) to the axis with the
    most aligned units per rank, never below one unit per rank (ties: the slowest axis).
    Factors that fit no axis are dropped: the product may be less than `world`."""
    grid = [1] * len(units)
    n, p, primes = world, 2, []
    while n > 1:
        while n % p == 0:
            primes.append(p)
            n //= p
        p += 1
    for p in sorted(primes, reverse=True):
        fits = [d for d in range(len(units)) if units[d] // (grid[d] * p) >= 1]
        if not fits:
            continue
        best = max(fits, key=lambda d: (units[d] / grid[d], -d))
        grid[best] *= p
    return tuple(grid)


def octant_assignment(rank: int, world: int, shape, factor, max_levels: int) -> OctantAssignment:
    """The level-0 box rank `rank` of `world` owns and its box at every locally computed level:
    the most levels L whose factor^L-aligned split still uses all ranks (else the split using
    the most ranks)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    levels = pyramid_level_shapes(shape, factor, max_levels)
    nd = len(shape)
    best = None
    for L in range(len(levels), 0, -1):
        units = [s // (f ** L) for s, f in zip(shape, factor)]
        g = _rank_grid(world, units)
        n = 1
        for x in g:
            n *= x
        if best is None or n > best[0]:
            best = (n, L, g)
        if n == world:
            break
    if best is None:  # no levels at all
        return OctantAssignment(rank, world, (1,) * nd, None if rank else (0,) * nd,
                                (0,) * nd, tuple(shape) if rank == 0 else (0,) * nd, 0, (), 0)
    nranks, L, grid = best
    if rank >= nranks:
        return OctantAssignment(rank, world, grid, None, (0,) * nd, (0,) * nd, L, (),
                                len(levels))
    align = [f ** L for f in factor]
    units = [s // a for s, a in zip(shape, align)]
    coord, r = [], rank
    for g in reversed(grid):
        coord.append(r % g)
        r //= g
    coord = tuple(reversed(coord))
    start, end = [], []
    for d, (g, c) in enumerate(zip(grid, coord)):
        u0, u1 = c * units[d] // g, (c + 1) * units[d] // g
        start.append(u0 * align[d])
        end.append(shape[d] if c == g - 1 else u1 * align[d])
    boxes = []
    for k in range(1, L + 1):
        fk = [f ** k for f in factor]
        s_k = [a // f for a, f in zip(start, fk)]
        e_k = [levels[k - 1][d] if coord[d] == grid[d] - 1 else end[d] // fk[d]
               for d in range(nd)]
        boxes.append((tuple(s_k), tuple(b - a for a, b in zip(s_k, e_k))))
    return OctantAssignment(rank, world, grid, coord, tuple(start),
                            tuple(b - a for a, b in zip(start, end)), L, tuple(boxes),
                            len(levels))


def assemble_chunk(chunk_start, chunk_shape, pieces):
    """Host gather of one output chunk from the ranks' sub-blocks of a level: `pieces` is a list
    of (box_start, array) in the level's coordinates; each contributes its intersection."""
    import numpy as np
    out = None
    for bstart, arr in pieces:
        lo = [max(c, b) for c, b in zip(chunk_start, bstart)]
        hi = [min(c + s, b + n) for c, s, b, n in zip(chunk_start, chunk_shape, bstart, arr.shape)]
        if any(h <= l for l, h in zip(lo, hi)):
            continue
        if out is None:
            out = np.zeros(tuple(chunk_shape), dtype=arr.dtype)
        dst = tuple(slice(l - c, h - c) for l, h, c in zip(lo, hi, chunk_start))
        src = tuple(slice(l - b, h - b) for l, h, b in zip(lo, hi, bstart))
        out[dst] = arr[src]
    return out


@dataclass(frozen=True)
class BlockAssignment:
    """Rank `rank`'s box of whole output chunks over the two leading axes (all of the others),
    and the input box it reads: the output box plus the halo on axes 0 and 1, clamped."""
    rank: int
    world: int
    groups: tuple          # (g0, g1): ranks along axis 0 and axis 1
    out_start: tuple
    out_shape: tuple
    in_start: tuple
    in_shape: tuple


def _split(n_chunks: int, parts: int, k: int) -> tuple:
    return k * n_chunks // parts, (k + 1) * n_chunks // parts


def block_split(world: int, shape, chunk_shape, halo: int) -> tuple:
    """(g0, g1) with g0 * g1 == world that minimises the input the ranks read in all — the
    stage-1 work, since every rank recomputes its halo (config T, SURVEY.md §8(e): a t-only split
    of a (32, 1024^3) series in (4, 256^3) chunks reads 12 timepoints for 4 output ones, 3x; a
    (t, z) split of 4 x 2 reads 12 x 520 planes per 8 x 512 outputs, 1.5x). Ties: fewer groups
    along axis 1."""
    n0 = -(-shape[0] // chunk_shape[0])
    n1 = -(-shape[1] // chunk_shape[1]) if len(shape) > 1 else 1
    best = None
    for g0 in range(1, world + 1):
        if world % g0:
            continue
        g1 = world // g0
        if g0 > n0 or g1 > n1:
            continue
        total = 0
        for k0 in range(g0):
            c0, c1 = _split(n0, g0, k0)
            a0, b0 = c0 * chunk_shape[0], min(c1 * chunk_shape[0], shape[0])
            e0 = min(b0 + halo, shape[0]) - max(a0 - halo, 0)
            for k1 in range(g1):
                d0, d1 = _split(n1, g1, k1)
                a1, b1 = d0 * chunk_shape[1], min(d1 * chunk_shape[1], shape[1])
                e1 = min(b1 + halo, shape[1]) - max(a1 - halo, 0)
                total += e0 * e1
        key = (total, g1)
        if best is None or key < best[0]:
            best = (key, (g0, g1))
    return best[1] if best else (world, 1)


def block_assignment(rank: int, world: int, shape, chunk_shape, halo: int,
                     groups=None) -> BlockAssignment:
    """Rank `rank` of `world`: its (axis-0, axis-1) box of whole output chunks (groups from
    block_split unless given) and the halo'd input box (ArraySubsetOverlap,
    array_subset_overlap.rs:11-35, on the box instead of each chunk)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    g0, g1 = groups or block_split(world, shape, chunk_shape, halo)
    if g0 * g1 != world:
        raise ValueError("groups must multiply to world")
    nd = len(shape)
    n0 = -(-shape[0] // chunk_shape[0])
    n1 = -(-shape[1] // chunk_shape[1])
    k0, k1 = rank // g1, rank % g1
    c0, c1 = _split(n0, g0, k0)
    d0, d1 = _split(n1, g1, k1)
    a0, b0 = min(c0 * chunk_shape[0], shape[0]), min(c1 * chunk_shape[0], shape[0])
    a1, b1 = min(d0 * chunk_shape[1], shape[1]), min(d1 * chunk_shape[1], shape[1])
    out_start = (a0, a1) + (0,) * (nd - 2)
    out_shape = (b0 - a0, b1 - a1) + tuple(shape[2:])
    i0, i1 = max(a0 - halo, 0), max(a1 - halo, 0)
    in_start = (i0, i1) + (0,) * (nd - 2)
    in_shape = (min(b0 + halo, shape[0]) - i0, min(b1 + halo, shape[1]) - i1) + tuple(shape[2:])
    if b0 <= a0 or b1 <= a1:
        in_shape = (0,) * nd
    return BlockAssignment(rank, world, (g0, g1), out_start, out_shape, in_start, in_shape)
