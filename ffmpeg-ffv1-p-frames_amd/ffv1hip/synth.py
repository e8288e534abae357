"""Synthetic input streams for the FFV1 encode path.

* D1 -- the reference's own benchmark/FATE source clip (tests/videogen.c),
  re-derived in csrc/synth.c and widened to 10/12/16 bit the way the
  reference's swscale limited-range path does (``v << (depth - 8)``).
* D2 -- the seeded LSB-active stress clip of SURVEY.md 8d (numpy PCG64).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _paths

_lib = None


def _synth():
    global _lib
    if _lib is None:
        path = _paths.synth_lib()
        L = ctypes.CDLL(path)
        L.ffv1syn_clip_new.argtypes = [ctypes.c_int, ctypes.c_int]
        L.ffv1syn_clip_new.restype = ctypes.c_void_p
        L.ffv1syn_clip_free.argtypes = [ctypes.c_void_p]
        L.ffv1syn_clip_next.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8)]
        L.ffv1syn_clip_next.restype = ctypes.c_int
        L.ffv1syn_clip_skip.argtypes = [ctypes.c_void_p]
        L.ffv1syn_roto_new.argtypes = [ctypes.POINTER(ctypes.c_uint8), ctypes.c_int, ctypes.c_int]
        L.ffv1syn_roto_new.restype = ctypes.c_void_p
        L.ffv1syn_roto_free.argtypes = [ctypes.c_void_p]
        L.ffv1syn_roto_next.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8)]
        L.ffv1syn_roto_next.restype = ctypes.c_int
        _lib = L
    return _lib


class VideogenClip:
    """Frame iterator over the D1 clip at any even WxH (yuv420p, u8)."""

    def __init__(self, width: int, height: int):
        self.w, self.h = width, height
        self._h = _synth().ffv1syn_clip_new(width, height)
        if not self._h:
            raise ValueError("videogen needs even dimensions")

    def __del__(self):
        if getattr(self, "_h", None):
            _synth().ffv1syn_clip_free(self._h)
            self._h = None

    def next_yuv420p(self):
        n = self.w * self.h
        buf = np.empty(n * 3 // 2, np.uint8)
        _synth().ffv1syn_clip_next(self._h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
        y = buf[:n].reshape(self.h, self.w)
        u = buf[n:n + n // 4].reshape(self.h // 2, self.w // 2)
        v = buf[n + n // 4:].reshape(self.h // 2, self.w // 2)
        return [y, u, v]

    def skip(self, n: int = 1):
        """Advance past n frames without drawing them."""
        for _ in range(n):
            _synth().ffv1syn_clip_skip(self._h)


class RotozoomClip:
    """The reference's "vsynth2" clip (tests/rotozoom.c), yuv420p u8 frames.

    ``pnm`` is the 256x256 RGB24 source picture as a binary PPM (the
    reference keeps it as tests/reference.pnm; a copy is a test fixture under
    tests/golden/).
    """

    def __init__(self, pnm: bytes, width: int = 352, height: int = 288):
        if len(pnm) < 15 + 256 * 256 * 3:
            raise ValueError("rotozoom needs a 256x256 binary PPM")
        self.w, self.h = width, height
        self._src = np.frombuffer(pnm, np.uint8)[15:15 + 256 * 256 * 3].copy()
        self._h = _synth().ffv1syn_roto_new(
            self._src.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), width, height)
        if not self._h:
            raise ValueError("rotozoom needs even dimensions")

    def __del__(self):
        if getattr(self, "_h", None):
            _synth().ffv1syn_roto_free(self._h)
            self._h = None

    def next_yuv420p(self):
        n = self.w * self.h
        buf = np.empty(n * 3 // 2, np.uint8)
        _synth().ffv1syn_roto_next(self._h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
        return [buf[:n].reshape(self.h, self.w),
                buf[n:n + n // 4].reshape(self.h // 2, self.w // 2),
                buf[n + n // 4:].reshape(self.h // 2, self.w // 2)]


def widen(planes, depth: int):
    """u8 planes -> u16 planes holding v << (depth - 8) (swscale shiftonly)."""
    return [np.ascontiguousarray(p.astype(np.uint16) << (depth - 8)) for p in planes]


def upsample_444(planes):
    """yuv420p -> yuv444p by sample repetition (nearest neighbour)."""
    y, u, v = planes
    h, w = y.shape
    up = lambda c: np.ascontiguousarray(np.repeat(np.repeat(c, 2, 0), 2, 1)[:h, :w])
    return [y, up(u), up(v)]


def upsample_422(planes):
    """yuv420p -> yuv422p by row repetition (swscale SWS_POINT: chroma row y>>1)."""
    y, u, v = planes
    h = y.shape[0]
    return [y] + [np.ascontiguousarray(np.repeat(c, 2, 0)[:h]) for c in (u, v)]


def _trunc_div(a: int, b: int) -> int:
    q = abs(a) // abs(b)
    return q if (a < 0) == (b < 0) else -q


def _yuv2rgb_lut():
    """The 32-bpp tables of ff_yuv2rgb_c_init_tables (libswscale/yuv2rgb.c:
    765-842, 959-983) for limited-range input, the default BT.601 matrix
    (ff_yuv2rgb_coeffs[SWS_CS_DEFAULT], :49-61; vf_scale.c:227-248) and unit
    contrast / saturation: a luma curve ``ytab`` and the per-U / per-V index
    offsets of fill_table / fill_gv_table (:728-751)."""
    crv, cbu, cgu, cgv = 104597, 132201, -25675, -53279
    cy = (1 << 16) * 255 // 219
    oy = 16 << 16
    crv, cbu, cgu, cgv = [_trunc_div(c * (1 << 16) + 0x8000, cy) for c in (crv, cbu, cgu, cgv)]
    yb = -(384 << 16) - 512 * cy - oy
    i = np.arange(2048, dtype=np.int64)
    ytab = np.clip((yb + i * cy + 0x8000) >> 16, 0, 255).astype(np.uint8)
    v = np.arange(256, dtype=np.int64)
    return (ytab, 838 - (crv >> 9) + ((v * crv) >> 16), 838 - (cbu >> 9) + ((v * cbu) >> 16),
            838 - (cgu >> 9) + ((v * cgu) >> 16), -(cgv >> 9) + ((v * cgv) >> 16))


def yuv420p_to_bgr0(planes):
    """yuv420p u8 -> bgr0 as ``-sws_flags neighbor+bitexact`` converts it:
    BGR0 is scaled as BGRA (libswscale/utils.c:1031-1039); the even width
    keeps half-resolution chroma (:1275-1291, 1362-1363) so each chroma
    sample covers a 2x2 block (point filter, :344-358), and every output
    pixel is three table reads (output.c yuv2rgb_write / yuv2rgb.c
    yuv2rgb_c_32: R = r[Y], G = g[Y], B = b[Y]).  The padding byte is the
    tables' alpha, 255; FFV1 does not code it."""
    ytab, r_off, b_off, gu_off, gv_off = _yuv2rgb_lut()
    y, u, v = [np.asarray(p).astype(np.int64) for p in planes]
    h, w = y.shape
    u = u[np.arange(h) >> 1][:, np.arange(w) >> 1]
    v = v[np.arange(h) >> 1][:, np.arange(w) >> 1]
    out = np.empty((h, w, 4), np.uint8)
    out[..., 0] = ytab[y + b_off[u]]
    out[..., 1] = ytab[y + gu_off[u] + gv_off[v]]
    out[..., 2] = ytab[y + r_off[v]]
    out[..., 3] = 255
    return [out.reshape(h, 4 * w)]


def convert(planes, pix_fmt: str):
    """yuv420p u8 -> ``pix_fmt`` as the FATE vsynth tests convert their input
    (``-sws_flags neighbor+bitexact``, tests/fate/vcodec.mak:116-124):
    point-sampled chroma (libswscale/utils.c:344-359 with the default chroma
    positions of :284-291 gives source index i>>1) and the depth change of the
    15/19-bit intermediates (v << 7 >> 5, v << 11 >> 3: ``v << (depth - 8)``).
    """
    table = {"yuv420p": (None, 8), "yuv420p10": (None, 10), "yuv420p16": (None, 16),
             "yuv422p": (upsample_422, 8), "yuv422p10": (upsample_422, 10),
             "yuv422p16": (upsample_422, 16), "yuv444p": (upsample_444, 8),
             "yuv444p10": (upsample_444, 10), "yuv444p16": (upsample_444, 16)}
    if pix_fmt == "bgr0":
        return yuv420p_to_bgr0(planes)
    if pix_fmt not in table:
        raise ValueError(f"no FATE conversion to {pix_fmt}")
    up, depth = table[pix_fmt]
    f = up(planes) if up else list(planes)
    if depth > 8:
        f = widen(f, depth)
    return [np.ascontiguousarray(p) for p in f]


def videogen_frames(width: int, height: int, n: int, depth: int = 8, chroma444: bool = False,
                    keep=None):
    """n frames of the D1 clip; with ``keep`` (frame index -> bool) only the
    kept frames are drawn and yielded, the others skipped."""
    clip = VideogenClip(width, height)
    for i in range(n):
        if keep is not None and not keep(i):
            clip.skip()
            continue
        f = clip.next_yuv420p()
        if chroma444:
            f = upsample_444(f)
        if depth > 8:
            f = widen(f, depth)
        yield [np.ascontiguousarray(p) for p in f]


def d2_frames(width: int, height: int, n: int, depth: int = 10, chroma444: bool = False,
              seed: int = 20261015, keep=None):
    """SURVEY.md 8d "D2": smooth moving field + uniform noise, LSB-active.

    Y = clip(512 + 300 sin((x+8t)/97) cos((y-5t)/61) + U{-8..8}, 0, 1023)
    cb = 512 + 200 sin((x2+4t)/53); U = clip(cb + U{-4..4}); V = clip(1023-cb+U{-4..4})
    Amplitudes scale by 2^(depth-10); samples are u16 (LSB aligned).  With
    ``keep``, skipped frames still draw their noise (the RNG stream is shared).
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    scale = 2.0 ** (depth - 10)
    maxv = (1 << depth) - 1
    cw = width if chroma444 else (width + 1) // 2
    chh = height if chroma444 else (height + 1) // 2
    ys = np.arange(height, dtype=np.float64)[:, None]
    xs = np.arange(width, dtype=np.float64)[None, :]
    xc = np.arange(cw, dtype=np.float64)[None, :]
    for t in range(n):
        ny = rng.integers(-8, 9, size=(height, width))
        nu = rng.integers(-4, 5, size=(chh, cw))
        nv = rng.integers(-4, 5, size=(chh, cw))
        if keep is not None and not keep(t):
            continue
        base = 512 + 300 * np.sin((xs + 8 * t) / 97) * np.cos((ys - 5 * t) / 61)
        Y = np.rint(base * scale) + ny * scale
        cb = (512 + 200 * np.sin((xc + 4 * t) / 53)) * scale
        cb = np.broadcast_to(cb, (chh, cw))
        U = np.rint(cb) + nu * scale
        V = np.rint(maxv - cb) + nv * scale
        yield [np.ascontiguousarray(np.clip(p, 0, maxv).astype(np.uint16)) for p in (Y, U, V)]
