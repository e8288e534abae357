"""GOP sharding across processes (one per GPU).

A keyframe resets every context state (ffv1enc.c:1171-1172), so the packets
of a GOP depend only on that GOP's frames and the stream parameters: GOP k
can be encoded on rank k mod N with no communication, and the stream is the
in-order concatenation of the per-GOP packets.  The only exchange is the
final gather of packets to the muxing rank (here with torch.distributed
point-to-point send/recv; RCCL over xGMI on GPUs, gloo in the CPU tests).
"""
from __future__ import annotations

from typing import Callable, Dict, List, Sequence, Tuple


def gop_ranges(n_frames: int, gop: int) -> List[Tuple[int, int]]:
    """[start, end) frame ranges of the GOPs of an n-frame stream."""
    if gop <= 1:
        return [(i, i + 1) for i in range(n_frames)]
    return [(s, min(s + gop, n_frames)) for s in range(0, n_frames, gop)]


def shard_gops(n_frames: int, gop: int, world: int, rank: int) -> List[Tuple[int, int]]:
    """GOPs owned by `rank`: round-robin, GOP k -> rank k % world."""
    return [r for k, r in enumerate(gop_ranges(n_frames, gop)) if k % world == rank]


def encode_shard(encoder_factory: Callable[[], object], frames: Callable[[int], Sequence],
                 ranges: Sequence[Tuple[int, int]]) -> Dict[int, Tuple[bytes, bool]]:
    """Encode each owned GOP with a fresh encoder (picture_number 0 = GOP start,
    so keyframe placement matches the global stream).  The encoder object must
    have ``encode(list_of_frames) -> [(packet, key)]``."""
    out: Dict[int, Tuple[bytes, bool]] = {}
    for start, end in ranges:
        enc = encoder_factory()
        pk = enc.encode([frames(i) for i in range(start, end)])
        for i, p in zip(range(start, end), pk):
            out[i] = p
    return out


def gather_packets(local: Dict[int, Tuple[bytes, bool]], n_frames: int, dist, rank: int,
                   world: int, dst: int = 0):
    """Collect every rank's packets on `dst` in stream order (others get None)."""
    if world == 1:
        return [local[i] for i in range(n_frames)]
    objs = [None] * world if rank == dst else None
    dist.gather_object(local, objs, dst=dst)
    if rank != dst:
        return None
    merged: Dict[int, Tuple[bytes, bool]] = {}
    for o in objs:
        merged.update(o)
    return [merged[i] for i in range(n_frames)]
