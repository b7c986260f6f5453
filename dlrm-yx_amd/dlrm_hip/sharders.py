"""Table sharders — same registry, names and placements as the reference (sharders.py:1-62).

``shard(Es, ndevices, alg)`` returns device_indices[t] = the rank owning table t.
"""
from __future__ import annotations

import sys
from typing import Callable, Dict, List, Sequence

_sharders: Dict[str, Callable[[Sequence[int], int], List[int]]] = {}


def get_splits(T: int, ndevices: int) -> List[int]:
    """First T mod n ranks get one extra table (sharders.py:3-9)."""
    k, m = divmod(T, ndevices)
    if m == 0:
        return [k] * ndevices
    return [(k + 1) if i < m else k for i in range(ndevices)]


def register_sharder(name: str):
    def deco(fn):
        _sharders[name] = fn
        return fn
    return deco


def shard(Es: Sequence[int], ndevices: int, alg: str = "naive") -> List[int]:
    """sharders.py:23-27 (exits like the reference on an unknown algorithm)."""
    if alg not in _sharders:
        sys.exit("ERROR: sharder not found")
    return _sharders[alg](Es, ndevices)


@register_sharder("naive")
def naive_shard(Es, ndevices):
    """Round-robin (sharders.py:30-32)."""
    return [x % ndevices for x in range(len(Es))]


@register_sharder("naive_chunk")
def naive_chunk_shard(Es, ndevices):
    """Contiguous chunks (sharders.py:35-42)."""
    out: List[int] = []
    for idx, s in enumerate(get_splits(len(Es), ndevices)):
        out.extend([idx] * s)
    return out


@register_sharder("greedy")
def greedy_shard(Es, ndevices):
    """Row-balanced: each table in order goes to the rank with the fewest rows so far,
    ties to the lowest rank (sharders.py:45-54; the driver default, dlrm_s_pytorch.py:1172)."""
    buckets = [0] * ndevices
    out = [0] * len(Es)
    for k, E in enumerate(Es):
        d = buckets.index(min(buckets))
        buckets[d] += int(E)
        out[k] = d
    return out


@register_sharder("hardcode")
def hardcode_shard(Es, ndevices):
    """sharders.py:57-60."""
    return [0] + [1] * (len(Es) - 1)
