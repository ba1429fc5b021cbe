"""Window sharding across GPUs: contiguous window ranges,
input slice = the range's samples plus an N - hop halo, no exchange step.

The same arithmetic runs in C++ inside libmtbridge.so (batch_start in
csrc/mtbridge.cpp) when a session spans several devices (gpu_init(-1, ...)).
"""
from __future__ import annotations


def shard_windows(n_windows: int, n_shards: int, shard: int) -> tuple[int, int]:
    """(first window, window count) of `shard`; ceil split, trailing shards may be short/empty."""
    per = -(-n_windows // n_shards)
    w0 = min(shard * per, n_windows)
    return w0, max(0, min(per, n_windows - w0))


def shard_series_slice(w0: int, nw: int, hop: int, window_len: int) -> tuple[int, int]:
    """[start, end) of the series samples shard windows [w0, w0+nw) read (halo included)."""
    if nw <= 0:
        return w0 * hop, w0 * hop
    return w0 * hop, (w0 + nw - 1) * hop + window_len


def split_symbols(window_costs: list[int], n_windows: list[int], n_shards: int, shard: int) -> list[tuple[int, int, int]]:
    """Pieces (symbol, first window, window count) that `shard` owns when whole symbols are not enough to
    balance (C5 at 8 ranks: 28 symbols of four sizes): McNaughton's wrap-around rule.  The symbols'
    windows are laid end to end on one cost line (window j of symbol i costs window_costs[i], integers),
    the line is cut into n_shards equal parts, and window j goes to the part its start falls in.  Every
    shard's cost is within one window of total / n_shards, and each symbol is cut at most n_shards - 1
    times, so the pieces stay long (a rank seeds few segments); hop = 1 pieces read their N - 1 halo."""
    total = sum(c * n for c, n in zip(window_costs, n_windows))
    lo_b, hi_b = total * shard // n_shards, total * (shard + 1) // n_shards
    out, start = [], 0
    for i, (c, n) in enumerate(zip(window_costs, n_windows)):
        if c <= 0:
            raise ValueError("window costs are positive integers")
        # windows j with lo_b <= start + j c < hi_b
        j0 = min(n, max(0, -(-(lo_b - start) // c)))
        j1 = min(n, max(0, -(-(hi_b - start) // c)))
        if j1 > j0:
            out.append((i, j0, j1 - j0))
        start += c * n
    return out


def shard_symbols(costs: list[float], n_shards: int, shard: int) -> list[int]:
    """Indices of the symbols (whole per-symbol batches, C5) that `shard` owns: greedy
    longest-first assignment to the least-loaded shard, balanced by `costs` (output bytes)."""
    load = [0.0] * n_shards
    owner = [0] * len(costs)
    for i in sorted(range(len(costs)), key=lambda i: (-costs[i], i)):
        g = min(range(n_shards), key=lambda g: (load[g], g))
        owner[i] = g
        load[g] += costs[i]
    return [i for i in range(len(costs)) if owner[i] == shard]
