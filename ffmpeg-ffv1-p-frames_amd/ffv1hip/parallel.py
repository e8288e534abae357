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

import numpy as np


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
        _close(enc)
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


# ---------------------------------------------------------------------------
# The within-GOP exchange step: when a stream has fewer GOPs than
# ranks (or GOPs too long to balance), frames are split into contiguous
# ranges and a range that starts inside a GOP continues the P-frame chain of
# the rank before it.  The only state crossing ranks is the per-slice
# context-state snapshot after the previous range's last frame
# (2 x contexts x 32 bytes per slice: 2.73 MB for 64 slices, context model
# 0), sent point-to-point (RCCL over xGMI on GPUs, gloo on CPU).

def contiguous_ranges(n_frames: int, world: int) -> List[Tuple[int, int]]:
    """[lo, hi) frame range of every rank: contiguous, sizes differ by <= 1."""
    base, extra = divmod(n_frames, world)
    out, lo = [], 0
    for r in range(world):
        hi = lo + base + (1 if r < extra else 0)
        out.append((lo, hi))
        lo = hi
    return out


def _is_key(i: int, gop: int) -> bool:
    return gop == 0 or i % gop == 0  # ffv1enc.c:1299


def encode_exchanged(encoder_factory: Callable[[], object], frames: Callable[[int], Sequence],
                     n_frames: int, gop: int, dist, rank: int, world: int,
                     to_tensor: Callable, from_tensor: Callable,
                     state_bytes: int, device=None) -> Dict[int, Tuple[bytes, bool]]:
    """Encode this rank's contiguous range.

    The part of the range from its first keyframe on (the body) is
    independent and is encoded first; its final states go to rank+1 when
    rank+1's range starts inside a GOP.  The head (the frames before the
    first keyframe) waits for rank-1's states, then continues that chain in
    a second encoder placed at the right picture number.  Encoders need
    ``encode``, ``get_slice_states`` and ``set_slice_states(buf, pn)``;
    ``to_tensor``/``from_tensor`` move a state blob to and from the
    communication device.  With ``device`` (a torch GPU device; RCCL) the
    blob never leaves HBM: the encoder's ``get_slice_states_device`` /
    ``set_slice_states_device`` copy it device to device, and the send and
    receive move the device tensor itself."""
    if n_frames < world:
        raise ValueError("the exchange step needs at least one frame per rank")
    ranges = contiguous_ranges(n_frames, world)
    lo, hi = ranges[rank]
    out: Dict[int, Tuple[bytes, bool]] = {}
    first_key = next((i for i in range(lo, hi) if _is_key(i, gop)), hi)
    send_next = rank + 1 < world and not _is_key(ranges[rank + 1][0], gop)

    def send(enc):
        if device is not None:
            import torch
            buf = torch.empty(state_bytes, dtype=torch.uint8, device=device)
            dist.send(enc.get_slice_states_device(buf), dst=rank + 1)
        else:
            dist.send(to_tensor(enc.get_slice_states()), dst=rank + 1)

    if first_key < hi:  # body: independent of the other ranks
        enc = encoder_factory()
        for i, p in zip(range(first_key, hi), enc.encode([frames(i) for i in range(first_key, hi)])):
            out[i] = p
        if send_next:
            send(enc)
        _close(enc)  # one encoder's device buffers at a time
        enc = None
    if lo < first_key:  # head: continue rank-1's chain
        if device is not None:
            import torch
            buf = torch.empty(state_bytes, dtype=torch.uint8, device=device)
        else:
            buf = to_tensor(np.zeros(state_bytes, np.uint8))
        dist.recv(buf, src=rank - 1)
        enc = encoder_factory()
        if device is not None:
            enc.set_slice_states_device(buf, lo)
        else:
            enc.set_slice_states(from_tensor(buf), lo)
        for i, p in zip(range(lo, first_key), enc.encode([frames(i) for i in range(lo, first_key)])):
            out[i] = p
        if first_key == hi and send_next:  # no keyframe in the range: pass the chain on
            send(enc)
        _close(enc)
    return out


def _close(enc):
    close = getattr(enc, "close", None)
    if close is not None:
        close()
