"""ctypes binding for the CPU oracle (oracle/ffv1_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, ``__graft_entry__.smoke()`` and
``bench.py``'s cpu_baseline leg, where it is the checker / the CPU baseline,
never the thing measured or shipped.  The product (ffmpeg-ffv1-p-frames_amd/)
never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# FFV1_ORACLE_LIB: another build of the same source (the sanitizer build,
# `make -C oracle sanitize`)
_LIB_PATH = os.environ.get("FFV1_ORACLE_LIB") or os.path.join(_HERE, "libffv1_oracle.so")


class Config(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "width", "height", "chroma_planes", "chroma_h_shift", "chroma_v_shift",
        "transparency", "bits_per_raw_sample", "packed_at_lsb", "sample_bytes",
        "version", "ac", "ec", "context_model", "num_h_slices", "num_v_slices",
        "gop_size", "sar_num", "sar_den", "colorspace")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.POINTER
        u8p = P(ctypes.c_uint8)
        L.ffv1o_configure.argtypes = [P(Config), ctypes.c_int, ctypes.c_int, ctypes.c_char_p] + [ctypes.c_int] * 7
        L.ffv1o_configure.restype = ctypes.c_int
        L.ffv1o_enc_new.argtypes = [P(Config)]
        L.ffv1o_enc_new.restype = ctypes.c_void_p
        L.ffv1o_enc_free.argtypes = [ctypes.c_void_p]
        L.ffv1o_enc_extradata.argtypes = [ctypes.c_void_p, u8p, ctypes.c_int]
        L.ffv1o_enc_extradata.restype = ctypes.c_int
        L.ffv1o_enc_frame.argtypes = [ctypes.c_void_p, P(u8p), P(ctypes.c_int), u8p, ctypes.c_int64, P(ctypes.c_int)]
        L.ffv1o_enc_frame.restype = ctypes.c_int64
        L.ffv1o_enc_frame_mt.argtypes = [ctypes.c_void_p, P(u8p), P(ctypes.c_int), u8p, ctypes.c_int64,
                                         P(ctypes.c_int), ctypes.c_int]
        L.ffv1o_enc_frame_mt.restype = ctypes.c_int64
        L.ffv1o_enc_last_slice_bytes.argtypes = [ctypes.c_void_p, P(ctypes.c_int), ctypes.c_int]
        L.ffv1o_enc_last_slice_pcm.argtypes = [ctypes.c_void_p, P(ctypes.c_int), ctypes.c_int]
        L.ffv1o_enc_get_states.argtypes = [ctypes.c_void_p, P(ctypes.c_uint8), ctypes.c_int64]
        L.ffv1o_enc_get_states.restype = ctypes.c_int64
        L.ffv1o_enc_set_states.argtypes = [ctypes.c_void_p, P(ctypes.c_uint8), ctypes.c_int64,
                                           ctypes.c_int64]
        L.ffv1o_enc_set_states.restype = ctypes.c_int
        L.ffv1o_slice_symbols.argtypes = [P(Config), P(u8p), P(ctypes.c_int), ctypes.c_int, P(ctypes.c_int32), ctypes.c_int64]
        L.ffv1o_slice_symbols.restype = ctypes.c_int64
        L.ffv1o_dec_new.argtypes = [P(Config), u8p, ctypes.c_int]
        L.ffv1o_dec_new.restype = ctypes.c_void_p
        L.ffv1o_dec_free.argtypes = [ctypes.c_void_p]
        L.ffv1o_dec_frame.argtypes = [ctypes.c_void_p, u8p, ctypes.c_int64, P(u8p), P(ctypes.c_int), P(ctypes.c_int)]
        L.ffv1o_dec_frame.restype = ctypes.c_int
        L.ffv1o_configure2.argtypes = [P(Config), ctypes.c_int, ctypes.c_int, ctypes.c_char_p] + \
            [ctypes.c_int] * 8
        L.ffv1o_configure2.restype = ctypes.c_int
        L.ffv1o_configure3.argtypes = [P(Config), ctypes.c_int, ctypes.c_int, ctypes.c_char_p] + \
            [ctypes.c_int] * 9
        L.ffv1o_configure3.restype = ctypes.c_int
        L.ffv1o_enc_new2.argtypes = [P(Config), ctypes.c_int, ctypes.c_char_p]
        L.ffv1o_enc_new2.restype = ctypes.c_void_p
        L.ffv1o_enc_stats_out.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64]
        L.ffv1o_enc_stats_out.restype = ctypes.c_int64
        L.ffv1o_crc32.argtypes = [ctypes.c_uint32, u8p, ctypes.c_int64]
        L.ffv1o_crc32.restype = ctypes.c_uint32
        _lib = L
    return _lib


def _u8p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def configure(width, height, pix_fmt, slices=0, level=-1, coder=-1, context=0,
              gop_size=12, bits_per_raw_sample=0, slicecrc=-1, pass_=0, experimental=False) -> Config:
    """encode_init's parameter derivation (ffv1enc.c:669-1029); pass_ 1 / 2
    are AV_CODEC_FLAG_PASS1 / PASS2; experimental = -strict experimental
    (version 4 at level 4, ffv1enc.c:703-706)."""
    cfg = Config()
    rc = lib().ffv1o_configure3(ctypes.byref(cfg), width, height, pix_fmt.encode(), slices,
                                level, coder, context, gop_size, bits_per_raw_sample, slicecrc,
                                pass_, int(experimental))
    if rc < 0:
        raise ValueError(f"ffv1o_configure rejected {pix_fmt} {width}x{height} slices={slices}: {rc}")
    return cfg


def plane_shapes(cfg: Config):
    """(rows, samples) of each input plane: Y, Cb, Cr, then A for YUVA; YA8
    one plane of interleaved Y, A bytes; bgr0 / RGB32 one of 4-byte pixels."""
    w, h = cfg.width, cfg.height
    if cfg.colorspace and cfg.sample_bytes == 4:  # bgr0 / RGB32: one packed plane
        return [(h, 4 * w)]
    if cfg.transparency and not cfg.chroma_planes:  # YA8
        return [(h, 2 * w)]
    cw = -((-w) >> cfg.chroma_h_shift)
    ch = -((-h) >> cfg.chroma_v_shift)
    shapes = [(h, w)]
    if cfg.chroma_planes:
        shapes += [(ch, cw), (ch, cw)]
    if cfg.transparency:
        shapes.append((h, w))
    return shapes


def _plane_ptrs(planes):
    arr = (ctypes.POINTER(ctypes.c_uint8) * 4)()
    strides = (ctypes.c_int * 4)()
    for i, p in enumerate(planes):
        assert p.flags["C_CONTIGUOUS"]
        arr[i] = _u8p(p.view(np.uint8))
        strides[i] = p.strides[0]
    for i in range(len(planes), 4):
        arr[i] = arr[0]
        strides[i] = strides[0]
    return arr, strides


class Encoder:
    """The oracle encoder: one instance = one stream (keeps P-frame state)."""

    def __init__(self, cfg: Config, pass_: int = 0, stats_in: str = None):
        self.cfg = cfg
        self._h = lib().ffv1o_enc_new2(ctypes.byref(cfg), pass_,
                                       stats_in.encode() if stats_in is not None else None)
        if not self._h:
            raise ValueError("ffv1o_enc_new failed")

    def stats_out(self) -> str:
        """Pass 1: the statistics text (avctx->stats_out at the flush)."""
        n = lib().ffv1o_enc_stats_out(self._h, None, 0)
        if n < 0:
            raise RuntimeError(n)
        buf = ctypes.create_string_buffer(int(n) + 1)
        lib().ffv1o_enc_stats_out(self._h, buf, n + 1)
        return buf.value.decode()

    def __del__(self):
        if getattr(self, "_h", None):
            lib().ffv1o_enc_free(self._h)
            self._h = None

    def extradata(self) -> bytes:
        buf = np.zeros(10000 + 4 + (7563 + 666) * 32 * 4, np.uint8)  # ffv1enc.c:556-557, generously
        n = lib().ffv1o_enc_extradata(self._h, _u8p(buf), buf.size)
        if n < 0:
            raise RuntimeError(n)
        return buf[:n].tobytes()

    def encode(self, planes, threads: int = 1):
        """One frame; threads > 1 codes its slices on that many threads (the
        reference's per-slice jobs, ffv1enc.c:1323): the same bytes."""
        for k, (rows, cols) in enumerate(plane_shapes(self.cfg)):
            a = planes[k]
            if a.shape[0] < rows or a.shape[1] < cols:
                raise ValueError(f"plane {k}: shape {a.shape}, the configuration needs {(rows, cols)}")
        arr, strides = _plane_ptrs(planes)
        cap = 1 << 20
        for p in planes:
            cap += p.nbytes * 20  # <= 33 decisions (bytes) per 16-bit sample
        out = np.empty(cap, np.uint8)
        key = ctypes.c_int()
        n = lib().ffv1o_enc_frame_mt(self._h, arr, strides, _u8p(out), cap, ctypes.byref(key), int(threads))
        if n < 0:
            raise RuntimeError(f"ffv1o_enc_frame: {n}")
        return out[:n].tobytes(), bool(key.value)

    def get_slice_states(self) -> np.ndarray:
        n = lib().ffv1o_enc_get_states(self._h, None, 0)
        buf = np.zeros(n, np.uint8)
        lib().ffv1o_enc_get_states(self._h, _u8p(buf), n)
        return buf

    def set_slice_states(self, buf: np.ndarray, picture_number: int):
        buf = np.ascontiguousarray(buf, np.uint8)
        if lib().ffv1o_enc_set_states(self._h, _u8p(buf), buf.size, picture_number) < 0:
            raise ValueError("state blob size")

    def last_slice_bytes(self):
        n = self.cfg.num_h_slices * self.cfg.num_v_slices
        arr = (ctypes.c_int * n)()
        lib().ffv1o_enc_last_slice_bytes(self._h, arr, n)
        return list(arr)

    def last_slice_pcm(self):
        """Per slice: the last frame coded it as PCM (v4 slice_coding_mode 1)."""
        n = self.cfg.num_h_slices * self.cfg.num_v_slices
        arr = (ctypes.c_int * n)()
        lib().ffv1o_enc_last_slice_pcm(self._h, arr, n)
        return list(arr)


def slice_symbols(cfg: Config, planes, slice_index: int) -> np.ndarray:
    arr, strides = _plane_ptrs(planes)
    cap = sum(p.shape[0] * p.shape[1] for p in planes) + 16
    out = np.empty(cap, np.int32)
    n = lib().ffv1o_slice_symbols(ctypes.byref(cfg), arr, strides, slice_index,
                                  out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), cap)
    return out[:n]


class Decoder:
    def __init__(self, cfg: Config, extradata: bytes = b""):
        self.cfg = cfg
        ex = np.frombuffer(extradata, np.uint8).copy() if extradata else np.zeros(1, np.uint8)
        self._h = lib().ffv1o_dec_new(ctypes.byref(cfg), _u8p(ex), len(extradata))
        if not self._h:
            raise ValueError("ffv1o_dec_new failed (extradata rejected)")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().ffv1o_dec_free(self._h)
            self._h = None

    def decode(self, packet: bytes):
        dt = np.uint8 if self.cfg.sample_bytes in (1, 4) else np.uint16
        planes = [np.zeros(s, dt) for s in plane_shapes(self.cfg)]
        arr, strides = _plane_ptrs(planes)
        pk = np.frombuffer(packet, np.uint8).copy()
        key = ctypes.c_int()
        rc = lib().ffv1o_dec_frame(self._h, _u8p(pk), len(packet), arr, strides, ctypes.byref(key))
        if rc < 0:
            raise RuntimeError(f"ffv1o_dec_frame: {rc}")
        return planes, bool(key.value)


def crc32(data: bytes, crc: int = 0) -> int:
    a = np.frombuffer(data, np.uint8).copy()
    return lib().ffv1o_crc32(crc, _u8p(a), len(data))
