"""Test helpers: stream definitions shared by the CPU and GPU tests."""
from __future__ import annotations

import hashlib
import json
import os
from dataclasses import dataclass, field

import numpy as np

from oracle import oracle
from ffv1hip import synth

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_golden(name):
    with open(os.path.join(GOLDEN_DIR, name)) as f:
        return json.load(f)


@dataclass
class Stream:
    """One encoder configuration + input clip."""
    name: str
    width: int
    height: int
    pix_fmt: str
    nframes: int
    slices: int = 0
    level: int = -1
    coder: int = 1
    context: int = 0
    gop_size: int = 12
    bits_per_raw_sample: int = 0
    source: str = "videogen"       # videogen | d2 | random
    depth: int = 8                 # widening depth for videogen sources
    chroma444: bool = False
    allow_large_grid: bool = False
    experimental: bool = False     # -strict experimental (version 4)
    seed: int = 1
    # False where the reference itself leaves samples uncoded: odd slice x
    # offsets with chroma subsampling (cx = x >> hs, ffv1enc.c:1186-1188)
    lossless: bool = True
    extra: dict = field(default_factory=dict)

    def oracle_config(self):
        if self.allow_large_grid:
            # the reference encoder refuses >64 slices; build the extended
            # grid configuration directly (decoder limit: 256 slices)
            cfg = oracle.configure(self.width, self.height, self.pix_fmt, slices=0,
                                   level=self.level, coder=self.coder, context=self.context,
                                   gop_size=self.gop_size,
                                   bits_per_raw_sample=self.bits_per_raw_sample)
            nh, nv = self.extra["grid"]
            cfg.num_h_slices, cfg.num_v_slices = nh, nv
            return cfg
        return oracle.configure(self.width, self.height, self.pix_fmt, slices=self.slices,
                                level=self.level, coder=self.coder, context=self.context,
                                gop_size=self.gop_size,
                                bits_per_raw_sample=self.bits_per_raw_sample,
                                experimental=self.experimental)

    def frames(self):
        if self.source == "videogen":
            yield from synth.videogen_frames(self.width, self.height, self.nframes, self.depth,
                                             self.chroma444)
        elif self.source == "d2":
            yield from synth.d2_frames(self.width, self.height, self.nframes, self.depth,
                                       self.chroma444)
        else:
            cfg = self.oracle_config()
            rng = np.random.default_rng(self.seed)
            dt = np.uint8 if cfg.sample_bytes in (1, 4) else np.uint16
            hi = 1 << (cfg.bits_per_raw_sample if cfg.packed_at_lsb or cfg.sample_bytes != 2 else 16)
            for _ in range(self.nframes):
                fr = []
                for shp in oracle.plane_shapes(cfg):
                    a = rng.integers(0, hi, size=shp, dtype=np.int64)
                    # a smooth ramp plus noise keeps contexts varied
                    yy, xx = np.mgrid[0:shp[0], 0:shp[1]]
                    a = (a // 8 + (xx * 3 + yy * 5) * (hi // 512 or 1)) % hi
                    fr.append(np.ascontiguousarray(a.astype(dt)))
                yield fr


def oracle_encode(stream: Stream, frames=None):
    cfg = stream.oracle_config()
    enc = oracle.Encoder(cfg)
    ex = enc.extradata()
    pkts = []
    for f in (frames if frames is not None else stream.frames()):
        pkts.append(enc.encode(f))
    return cfg, ex, pkts


def md5(b: bytes) -> str:
    return hashlib.md5(b).hexdigest()


# Parity matrix: covers both coders' range paths, every bit depth, P-frames
# across batch boundaries, odd geometry, context model 1 and the 16x16 grid.
PARITY_STREAMS = [
    Stream("cif420_range_intra_v3", 352, 288, "yuv420p", 4, slices=4, gop_size=1),
    Stream("p10_gop4", 480, 270, "yuv420p10", 9, slices=4, gop_size=4, depth=10),
    Stream("p10_d2_gop5", 320, 180, "yuv420p10", 7, slices=6, gop_size=5, source="d2", depth=10),
    # an odd slice count (3x3): the states walk pairs slices per wave, the last alone
    Stream("p10_9slices", 360, 270, "yuv420p10", 5, slices=9, gop_size=3, source="d2", depth=10),
    Stream("p12_444", 256, 144, "yuv444p16", 5, slices=4, gop_size=3, bits_per_raw_sample=12,
           depth=16, chroma444=True),
    Stream("p16_444_wrap", 128, 96, "yuv444p16", 3, slices=4, gop_size=2, source="random"),
    Stream("vsynth3_34x34", 34, 34, "yuv420p", 14, level=3, gop_size=12),
    Stream("odd_422p10", 95, 61, "yuv422p10", 4, slices=6, gop_size=3, source="random",
           lossless=False),
    Stream("ctx1_p10", 352, 288, "yuv420p10", 4, slices=4, gop_size=3, context=1, depth=10),
    Stream("v1_inband_header", 176, 144, "yuv420p10", 4, gop_size=3, depth=10),
    Stream("range_default_tab", 176, 144, "yuv420p", 3, slices=4, coder=-2, gop_size=2),
    Stream("gray16", 96, 64, "gray16", 3, slices=4, gop_size=2, source="random"),
    Stream("grid16x16", 960, 544, "yuv420p10", 3, slices=256, gop_size=2, source="d2", depth=10,
           allow_large_grid=True, extra={"grid": (16, 16)}),
    # Golomb-Rice (coder=0): v0 single slice with in-band header, v3 P-frames,
    # context model 1, and the odd 34x34 geometry of FATE vsynth3
    Stream("golomb_v0_cif_intra", 352, 288, "yuv420p", 3, coder=0, gop_size=1),
    Stream("golomb_v3_pframes", 352, 288, "yuv420p", 7, slices=4, coder=0, gop_size=4),
    Stream("golomb_ctx1", 176, 144, "yuv422p", 4, slices=4, coder=0, context=1, gop_size=3,
           source="random"),
    Stream("golomb_vsynth3", 34, 34, "yuv420p", 13, slices=4, coder=0, gop_size=12),
]

# RGB through the reversible colour transform (chained coders on the GPU):
# bgr0 with both coders and context models, gbrp at 9..14 bits (range coder
# forced), odd geometry and a 3x3 grid.
RGB_STREAMS = [
    Stream("bgr0_v3", 176, 144, "bgr0", 4, slices=4, level=3, gop_size=3, source="random"),
    Stream("bgr0_golomb_v1", 96, 64, "bgr0", 3, level=1, coder=0, gop_size=2, source="random"),
    Stream("bgr0_range_ctx1", 120, 90, "bgr0", 4, slices=9, coder=1, context=1, gop_size=2,
           source="random"),
    Stream("gbrp9_odd", 75, 49, "gbrp9", 3, slices=4, gop_size=2, source="random"),
    Stream("gbrp10_v3", 128, 96, "gbrp10", 3, slices=4, level=3, gop_size=2, source="random"),
    Stream("gbrp12_v1", 64, 48, "gbrp12", 3, level=1, gop_size=3, source="random"),
    Stream("gbrp14_ctx1", 64, 48, "gbrp14", 3, slices=4, context=1, gop_size=3, source="random"),
]


def corrupt_slice(packet: bytes, ec: bool, nslices: int, slice_index: int) -> bytes:
    """Flip one byte in the middle of a slice's coded bytes (not its header
    or trailer): the slice then fails its CRC (ffv1dec.c:963-977)."""
    trailer = 3 + (5 if ec else 0)
    end, spans = len(packet), []
    for _ in range(nslices):
        size = int.from_bytes(packet[end - trailer:end - trailer + 3], "big")
        spans.append((end - trailer - size, end - trailer))
        end -= size + trailer
    a, b = spans[nslices - 1 - slice_index]
    k = (a + b) // 2 + 16
    assert a + 16 < k < b
    return packet[:k] + bytes([packet[k] ^ 0x5A]) + packet[k + 1:]


def slice_rect(cfg, i):
    nh, nv = cfg.num_h_slices, cfg.num_v_slices
    sx, sy = i % nh, i // nh
    x0, x1 = cfg.width * sx // nh, cfg.width * (sx + 1) // nh
    y0, y1 = cfg.height * sy // nv, cfg.height * (sy + 1) // nv
    return x0, y0, x1, y1
