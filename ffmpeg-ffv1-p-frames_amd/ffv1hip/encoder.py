"""Host-side mirror of the reference's FFV1 AVCodec, backed by the HIP C-ABI.

The reference plugs its encoder into FFmpeg as ``ff_ffv1_encoder``
(libavcodec/ffv1enc.c:1415-1444): ``init`` = encode_init (:669),
``encode2`` = encode_frame (:1222), ``close`` = encode_close (:1375), with
``AV_CODEC_CAP_DELAY`` so frames may be buffered and drained by a NULL frame.
:class:`FFV1Encoder` keeps those names, argument meanings and error
behaviour; every call goes through ``lib/libffv1hip.so``
(include/ffv1hip.h).  There is no CPU fallback: if the HIP library is
missing or no GPU is visible, construction raises.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _paths

AVERROR_INVALIDDATA = -1094995529


class Options(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int), ("pix_fmt", ctypes.c_char_p),
                ("slices", ctypes.c_int), ("level", ctypes.c_int), ("coder", ctypes.c_int),
                ("context", ctypes.c_int), ("gop_size", ctypes.c_int),
                ("bits_per_raw_sample", ctypes.c_int), ("slicecrc", ctypes.c_int),
                ("allow_large_grid", ctypes.c_int), ("pass_", ctypes.c_int), ("experimental", ctypes.c_int)]


class Params(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "width", "height", "chroma_planes", "chroma_h_shift", "chroma_v_shift",
        "bits_per_raw_sample", "packed_at_lsb", "sample_bytes", "version", "ac", "ec",
        "context_model", "num_h_slices", "num_v_slices", "gop_size", "sar_num", "sar_den",
        "colorspace", "transparency")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}

    @property
    def nslices(self):
        return self.num_h_slices * self.num_v_slices

    def plane_shapes(self):
        """(rows, samples) of each host plane: Y, Cb, Cr (+ A for YUVA); one
        packed plane for bgr0 / RGB32 (4 bytes a pixel) and YA8 (Y, A bytes)."""
        if self.sample_bytes == 4:  # bgr0 / RGB32: one packed B, G, R, X / A plane
            return [(self.height, 4 * self.width)]
        if self.transparency and not self.chroma_planes:  # YA8
            return [(self.height, 2 * self.width)]
        cw = -((-self.width) >> self.chroma_h_shift)
        ch = -((-self.height) >> self.chroma_v_shift)
        shapes = [(self.height, self.width)]
        if self.chroma_planes:
            shapes += [(ch, cw), (ch, cw)]
        if self.transparency:
            shapes.append((self.height, self.width))
        return shapes

    @property
    def planes_per_frame(self):
        """Plane pointers per frame in the C-ABI's arrays (FFV1HIP_PLANES[_YUVA])."""
        return 4 if len(self.plane_shapes()) == 4 else 3


EXPORTED_SYMBOLS = (
    "ffv1hip_configure", "ffv1hip_create", "ffv1hip_destroy", "ffv1hip_extradata",
    "ffv1hip_max_packet_size", "ffv1hip_encode", "ffv1hip_encode_device", "ffv1hip_fetch",
    "ffv1hip_device_packets", "ffv1hip_picture_number", "ffv1hip_reset",
    "ffv1hip_get_slice_states", "ffv1hip_set_slice_states", "ffv1hip_last_error",
    "ffv1hip_abi_version", "ffv1hip_debug_checks", "ffv1hip_host_register", "ffv1hip_host_unregister",
    "ffv1hip_get_slice_states_device", "ffv1hip_set_slice_states_device", "ffv1hip_set_profiling", "ffv1hip_last_kernel_ms",
    "ffv1hip_last_kernel_stats", "ffv1hip_synchronize",
    "ffv1hip_dec_create", "ffv1hip_dec_destroy", "ffv1hip_decode", "ffv1hip_dec_reset",
    "ffv1hip_set_picture_number", "ffv1hip_encode2", "ffv1hip_encode2_delay", "ffv1hip_encode2_last_packet",
    "ffv1hip_dec_damaged_slices",
    "ffv1hip_set_pass", "ffv1hip_stats_out", "ffv1hip_debug_counter",
)


class KernelStats(ctypes.Structure):
    _fields_ = [("symbols_ms", ctypes.c_float), ("code_ms", ctypes.c_float),
                ("assemble_ms", ctypes.c_float), ("symbols_launches", ctypes.c_int),
                ("code_launches", ctypes.c_int), ("assemble_launches", ctypes.c_int),
                ("frames_coded_per_launch_max", ctypes.c_int64), ("states_ms", ctypes.c_float),
                ("states_launches", ctypes.c_int), ("layout_ms", ctypes.c_float),
                ("bits_ms", ctypes.c_float), ("layout_launches", ctypes.c_int),
                ("bits_launches", ctypes.c_int), ("sink_ms", ctypes.c_float),
                ("sink_launches", ctypes.c_int), ("dseg_ms", ctypes.c_float),
                ("dfix_ms", ctypes.c_float), ("dseg_launches", ctypes.c_int),
                ("dfix_launches", ctypes.c_int)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}

_lib = None


def load_library():
    """Load lib/libffv1hip.so and declare the C-ABI.  Raises if missing."""
    global _lib
    if _lib is not None:
        return _lib
    L = ctypes.CDLL(_paths.hip_lib())
    P = ctypes.POINTER
    vp, i64, u8p = ctypes.c_void_p, ctypes.c_int64, P(ctypes.c_uint8)
    L.ffv1hip_configure.argtypes = [P(Params), P(Options)]
    L.ffv1hip_configure.restype = ctypes.c_int
    L.ffv1hip_create.argtypes = [P(Params), ctypes.c_int, ctypes.c_int, P(ctypes.c_int)]
    L.ffv1hip_create.restype = vp
    L.ffv1hip_destroy.argtypes = [vp]
    L.ffv1hip_destroy.restype = None
    L.ffv1hip_extradata.argtypes = [vp, u8p, ctypes.c_int]
    L.ffv1hip_extradata.restype = ctypes.c_int
    L.ffv1hip_max_packet_size.argtypes = [vp]
    L.ffv1hip_max_packet_size.restype = i64
    L.ffv1hip_encode.argtypes = [vp, P(vp), P(ctypes.c_int), ctypes.c_int, u8p, i64, P(i64), P(ctypes.c_int)]
    L.ffv1hip_encode.restype = ctypes.c_int
    L.ffv1hip_encode2.argtypes = [vp, P(vp), P(ctypes.c_int), i64, u8p, i64, P(i64), P(i64),
                                  P(ctypes.c_int), P(ctypes.c_int)]
    L.ffv1hip_encode2.restype = ctypes.c_int
    L.ffv1hip_encode2_delay.argtypes = [vp]
    L.ffv1hip_encode2_delay.restype = ctypes.c_int
    L.ffv1hip_encode2_last_packet.argtypes = [vp, u8p, i64]
    L.ffv1hip_encode2_last_packet.restype = i64
    L.ffv1hip_set_pass.argtypes = [vp, ctypes.c_int, ctypes.c_char_p]
    L.ffv1hip_set_pass.restype = ctypes.c_int
    L.ffv1hip_stats_out.argtypes = [vp, ctypes.c_char_p, i64]
    L.ffv1hip_stats_out.restype = i64
    L.ffv1hip_encode_device.argtypes = [vp, vp, i64, P(i64), P(ctypes.c_int), ctypes.c_int, vp]
    L.ffv1hip_encode_device.restype = ctypes.c_int
    L.ffv1hip_fetch.argtypes = [vp, u8p, i64, P(i64), P(ctypes.c_int)]
    L.ffv1hip_fetch.restype = ctypes.c_int
    L.ffv1hip_synchronize.argtypes = [vp]
    L.ffv1hip_synchronize.restype = ctypes.c_int
    L.ffv1hip_device_packets.argtypes = [vp, P(vp), P(i64), P(vp)]
    L.ffv1hip_device_packets.restype = ctypes.c_int
    L.ffv1hip_picture_number.argtypes = [vp]
    L.ffv1hip_picture_number.restype = i64
    L.ffv1hip_reset.argtypes = [vp]
    L.ffv1hip_reset.restype = None
    L.ffv1hip_get_slice_states.argtypes = [vp, u8p, i64]
    L.ffv1hip_get_slice_states.restype = i64
    L.ffv1hip_set_slice_states.argtypes = [vp, u8p, i64]
    L.ffv1hip_set_slice_states.restype = ctypes.c_int
    L.ffv1hip_set_picture_number.argtypes = [vp, i64]
    L.ffv1hip_set_picture_number.restype = ctypes.c_int
    L.ffv1hip_last_error.argtypes = []
    L.ffv1hip_last_error.restype = ctypes.c_char_p
    L.ffv1hip_set_profiling.argtypes = [vp, ctypes.c_int]
    L.ffv1hip_set_profiling.restype = ctypes.c_int
    L.ffv1hip_last_kernel_ms.argtypes = [vp, P(ctypes.c_float), P(ctypes.c_float)]
    L.ffv1hip_last_kernel_ms.restype = ctypes.c_int
    L.ffv1hip_last_kernel_stats.argtypes = [vp, P(KernelStats)]
    L.ffv1hip_last_kernel_stats.restype = ctypes.c_int
    L.ffv1hip_dec_create.argtypes = [P(Params), u8p, ctypes.c_int, ctypes.c_int, P(ctypes.c_int)]
    L.ffv1hip_dec_create.restype = vp
    L.ffv1hip_dec_destroy.argtypes = [vp]
    L.ffv1hip_dec_destroy.restype = None
    L.ffv1hip_decode.argtypes = [vp, u8p, P(i64), ctypes.c_int, P(vp), P(ctypes.c_int), P(ctypes.c_int)]
    L.ffv1hip_decode.restype = ctypes.c_int
    L.ffv1hip_dec_reset.argtypes = [vp]
    L.ffv1hip_dec_reset.restype = None
    L.ffv1hip_dec_damaged_slices.argtypes = [vp]
    L.ffv1hip_dec_damaged_slices.restype = ctypes.c_int
    L.ffv1hip_abi_version.argtypes = []
    L.ffv1hip_debug_counter.argtypes = [vp, ctypes.c_char_p]
    L.ffv1hip_debug_counter.restype = ctypes.c_int64
    L.ffv1hip_abi_version.restype = ctypes.c_int
    L.ffv1hip_get_slice_states_device.argtypes = [vp, vp, i64, vp]
    L.ffv1hip_get_slice_states_device.restype = i64
    L.ffv1hip_set_slice_states_device.argtypes = [vp, vp, i64, vp]
    L.ffv1hip_set_slice_states_device.restype = ctypes.c_int
    L.ffv1hip_host_register.argtypes = [vp, vp, i64]
    L.ffv1hip_host_register.restype = ctypes.c_int
    L.ffv1hip_host_unregister.argtypes = [vp, vp]
    L.ffv1hip_host_unregister.restype = ctypes.c_int
    L.ffv1hip_debug_checks.argtypes = []
    L.ffv1hip_debug_checks.restype = ctypes.c_int
    _lib = L
    return L


class FFV1Error(RuntimeError):
    def __init__(self, code: int, what: str):
        msg = load_library().ffv1hip_last_error().decode(errors="replace")
        super().__init__(f"{what}: error {code}: {msg}")
        self.code = code


def configure(width: int, height: int, pix_fmt: str, slices: int = 0, level: int = -1,
              coder: int = -1, context: int = 0, gop_size: int = 12,
              bits_per_raw_sample: int = 0, slicecrc: int = -1,
              allow_large_grid: bool = False, pass_: int = 0, experimental: bool = False) -> Params:
    """encode_init's option -> bitstream-parameter derivation (ffv1enc.c:669-1029);
    pass_ 1 / 2 are AV_CODEC_FLAG_PASS1 / PASS2; experimental is -strict
    experimental (versions 2 and 4 at levels 2 and 4, ffv1enc.c:703-706)."""
    L = load_library()
    o = Options(width, height, pix_fmt.encode(), slices, level, coder, context, gop_size,
                bits_per_raw_sample, slicecrc, int(allow_large_grid), pass_, int(experimental))
    p = Params()
    rc = L.ffv1hip_configure(ctypes.byref(p), ctypes.byref(o))
    if rc < 0:
        raise FFV1Error(rc, "ffv1hip_configure")
    return p


def check_planes(params: Params, planes: Sequence[np.ndarray]):
    """The library copies rows x row-bytes of every plane from host memory:
    a plane smaller than the parameters say would be read past its end."""
    shapes = params.plane_shapes()
    if len(planes) < len(shapes):
        raise ValueError(f"{len(planes)} planes, {params.width}x{params.height} needs {len(shapes)}")
    itemsize = 1 if params.sample_bytes in (1, 4) else 2
    for k, (rows, cols) in enumerate(shapes):
        a = np.asarray(planes[k])
        if a.ndim != 2 or a.shape[0] < rows or a.shape[1] * a.itemsize < cols * itemsize:
            raise ValueError(f"plane {k}: shape {a.shape} ({a.dtype}), need {rows} rows of {cols} "
                             f"{'bytes' if itemsize == 1 else 'u16 samples'}")


def _u8p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


class HipEncoder:
    """Thin owner of one ``ffv1hip_ctx`` (one stream, P-frame state on device)."""

    def __init__(self, params: Params, device: int = 0, max_batch: int = 16):
        L = load_library()
        self.params = params
        self.max_batch = max_batch
        err = ctypes.c_int(0)
        self._h = L.ffv1hip_create(ctypes.byref(params), device, max_batch, ctypes.byref(err))
        if not self._h:
            raise FFV1Error(err.value, "ffv1hip_create")

    def close(self):
        if getattr(self, "_h", None):
            load_library().ffv1hip_destroy(self._h)
            self._h = None

    __del__ = close

    def register_host(self, arr: np.ndarray):
        """Page-lock a (C-contiguous) array the caller keeps alive, so that
        frames in it go to HBM straight from it (ffv1hip_host_register)."""
        rc = load_library().ffv1hip_host_register(self._h, arr.ctypes.data, arr.nbytes)
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_host_register")

    def unregister_host(self, arr: np.ndarray):
        rc = load_library().ffv1hip_host_unregister(self._h, arr.ctypes.data)
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_host_unregister")

    def set_pass(self, pass_: int, stats_in: Optional[str] = None):
        """2-pass mode, before the first frame (ffv1hip_set_pass)."""
        rc = load_library().ffv1hip_set_pass(self._h, pass_,
                                             stats_in.encode() if stats_in is not None else None)
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_set_pass")

    def stats_out(self) -> str:
        """Pass 1: the statistics text (avctx->stats_out at the end of the stream)."""
        L = load_library()
        n = L.ffv1hip_stats_out(self._h, None, 0)
        if n < 0:
            raise FFV1Error(n, "ffv1hip_stats_out")
        buf = ctypes.create_string_buffer(n + 1)
        n = L.ffv1hip_stats_out(self._h, buf, n + 1)
        if n < 0:
            raise FFV1Error(n, "ffv1hip_stats_out")
        return buf.value.decode()

    def extradata(self) -> bytes:
        L = load_library()
        n = L.ffv1hip_extradata(self._h, None, 0)
        buf = np.zeros(max(n, 1), np.uint8)
        n = L.ffv1hip_extradata(self._h, _u8p(buf), buf.size)
        if n < 0:
            raise FFV1Error(n, "ffv1hip_extradata")
        return buf[:n].tobytes()

    @property
    def picture_number(self) -> int:
        return load_library().ffv1hip_picture_number(self._h)

    def max_packet_size(self) -> int:
        return load_library().ffv1hip_max_packet_size(self._h)

    def encode2_delay(self) -> int:
        """Frames ffv1hip_encode2 holds back (avctx->delay)."""
        rc = load_library().ffv1hip_encode2_delay(self._h)
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_encode2_delay")
        return rc

    def encode(self, frames: Sequence[Sequence[np.ndarray]]) -> List[Tuple[bytes, bool]]:
        """Encode host frames (each a list of 2-D uint8/uint16 planes) in order."""
        L = load_library()
        n = len(frames)
        np_planes = len(self.params.plane_shapes())
        for fr in frames:
            check_planes(self.params, fr)
        ppf = self.params.planes_per_frame
        ptrs = (ctypes.c_void_p * (ppf * n))()
        strides = (ctypes.c_int * (ppf * n))()
        keep = []
        for i, fr in enumerate(frames):
            for k in range(ppf):
                a = fr[min(k, np_planes - 1)]
                a = np.ascontiguousarray(a)
                keep.append(a)
                ptrs[ppf * i + k] = a.ctypes.data
                strides[ppf * i + k] = a.strides[0]
        total_in = sum(a.nbytes for a in keep)
        cap = total_in * 4 + 65536 * n
        out = np.empty(cap, np.uint8)
        sizes = (ctypes.c_int64 * n)()
        keys = (ctypes.c_int * n)()
        rc = L.ffv1hip_encode(self._h, ptrs, strides, n, _u8p(out), cap, sizes, keys)
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_encode")
        res, pos = [], 0
        for i in range(n):
            res.append((out[pos:pos + sizes[i]].tobytes(), bool(keys[i])))
            pos += sizes[i]
        return res

    def encode_device(self, d_frames: int, frame_bytes: int, plane_offset, plane_stride,
                      n_frames: int, stream: int = 0):
        L = load_library()
        off = (ctypes.c_int64 * 4)(*plane_offset)
        st = (ctypes.c_int * 4)(*plane_stride)
        rc = L.ffv1hip_encode_device(self._h, ctypes.c_void_p(d_frames), frame_bytes, off, st,
                                     n_frames, ctypes.c_void_p(stream) if stream else None)
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_encode_device")

    def fetch(self, n_frames: int) -> List[Tuple[bytes, bool]]:
        L = load_library()
        sizes = (ctypes.c_int64 * n_frames)()
        keys = (ctypes.c_int * n_frames)()
        rc = L.ffv1hip_fetch(self._h, None, 0, sizes, keys)
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_fetch")
        total = sum(sizes)
        out = np.empty(max(total, 1), np.uint8)
        rc = L.ffv1hip_fetch(self._h, _u8p(out), total, sizes, keys)
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_fetch")
        res, pos = [], 0
        for i in range(n_frames):
            res.append((out[pos:pos + sizes[i]].tobytes(), bool(keys[i])))
            pos += sizes[i]
        return res

    def synchronize(self) -> None:
        """Wait for all of the encoder's queued work (encode_device is asynchronous)."""
        rc = load_library().ffv1hip_synchronize(self._h)
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_synchronize")

    def device_packets(self):
        L = load_library()
        d_p, d_s = ctypes.c_void_p(), ctypes.c_void_p()
        stride = ctypes.c_int64()
        L.ffv1hip_device_packets(self._h, ctypes.byref(d_p), ctypes.byref(stride), ctypes.byref(d_s))
        return d_p.value, stride.value, d_s.value

    def get_slice_states(self) -> np.ndarray:
        """The P-frame carry after the last frame encoded: [slice][2][contexts][32]."""
        L = load_library()
        n = L.ffv1hip_get_slice_states(self._h, None, 0)
        if n < 0:
            raise FFV1Error(n, "ffv1hip_get_slice_states")
        buf = np.zeros(n, np.uint8)
        rc = L.ffv1hip_get_slice_states(self._h, _u8p(buf), n)
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_get_slice_states")
        return buf

    def set_slice_states(self, buf: np.ndarray, picture_number: int):
        """Continue another encoder's stream at `picture_number` from its states."""
        L = load_library()
        buf = np.ascontiguousarray(buf, np.uint8)
        rc = L.ffv1hip_set_slice_states(self._h, _u8p(buf), buf.size)
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_set_slice_states")
        rc = L.ffv1hip_set_picture_number(self._h, picture_number)
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_set_picture_number")

    def state_bytes(self) -> int:
        n = load_library().ffv1hip_get_slice_states(self._h, None, 0)
        if n < 0:
            raise FFV1Error(n, "ffv1hip_get_slice_states")
        return n

    def get_slice_states_device(self, out):
        """The carry into `out`, a uint8 torch tensor on this encoder's GPU,
        queued on torch's current stream (ffv1hip_get_slice_states_device):
        no host copy, ready for an RCCL send."""
        import torch
        assert out.is_cuda and out.dtype == torch.uint8 and out.is_contiguous()
        st = torch.cuda.current_stream(out.device).cuda_stream
        n = load_library().ffv1hip_get_slice_states_device(self._h, out.data_ptr(), out.numel(), st)
        if n < 0:
            raise FFV1Error(n, "ffv1hip_get_slice_states_device")
        return out

    def set_slice_states_device(self, buf, picture_number: int):
        """Continue another encoder's stream at `picture_number` from states in
        a device tensor (received over RCCL), ordered after torch's current
        stream (ffv1hip_set_slice_states_device)."""
        import torch
        assert buf.is_cuda and buf.dtype == torch.uint8 and buf.is_contiguous()
        L = load_library()
        st = torch.cuda.current_stream(buf.device).cuda_stream
        rc = L.ffv1hip_set_slice_states_device(self._h, buf.data_ptr(), buf.numel(), st)
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_set_slice_states_device")
        rc = L.ffv1hip_set_picture_number(self._h, picture_number)
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_set_picture_number")

    def set_profiling(self, on: bool = True):
        rc = load_library().ffv1hip_set_profiling(self._h, int(on))
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_set_profiling")

    def last_kernel_ms(self):
        e, a = ctypes.c_float(), ctypes.c_float()
        rc = load_library().ffv1hip_last_kernel_ms(self._h, ctypes.byref(e), ctypes.byref(a))
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_last_kernel_ms")
        return e.value, a.value

    def last_kernel_stats(self) -> dict:
        st = KernelStats()
        rc = load_library().ffv1hip_last_kernel_stats(self._h, ctypes.byref(st))
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_last_kernel_stats")
        return st.as_dict()

    def debug_counter(self, name: str) -> int:
        """A test counter of the context (ffv1hip_debug_counter): guard_skips, guard_reruns."""
        return int(load_library().ffv1hip_debug_counter(self._h, name.encode()))

    def slice_states(self) -> bytes:
        L = load_library()
        n = L.ffv1hip_get_slice_states(self._h, None, 0)
        buf = np.empty(n, np.uint8)
        rc = L.ffv1hip_get_slice_states(self._h, _u8p(buf), n)
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_get_slice_states")
        return buf.tobytes()


@dataclass
class AVPacket:
    data: bytes
    pts: int
    dts: int
    key: bool

    @property
    def flags(self) -> int:  # AV_PKT_FLAG_KEY
        return 1 if self.key else 0


@dataclass
class AVCodecContext:
    """The AVCodecContext fields encode_init/encode_frame read."""
    width: int
    height: int
    pix_fmt: str
    gop_size: int = 12
    slices: int = 0
    level: int = -1
    coder: int = -1
    context: int = 0
    bits_per_raw_sample: int = 0
    slicecrc: int = -1
    extradata: bytes = b""
    allow_large_grid: bool = False
    strict_std_compliance: int = 0   # FF_COMPLIANCE_EXPERIMENTAL (-2) admits versions 2 and 4
    flags: int = 0                   # AV_CODEC_FLAG_PASS1 / PASS2
    stats_in: Optional[str] = None   # pass 2: what pass 1 left in stats_out
    stats_out: str = ""              # pass 1: written at the flush (ffv1enc.c:1236-1277)
    delay: int = 0                   # frames encode2 holds back, set by init
    priv: dict = field(default_factory=dict)


AV_CODEC_FLAG_PASS1 = 1 << 9   # avcodec.h
FF_COMPLIANCE_EXPERIMENTAL = -2  # avcodec.h: -strict experimental (ffv1enc.c:703-706)
AV_CODEC_FLAG_PASS2 = 1 << 10


class FFV1Encoder:
    """Mirror of ff_ffv1_encoder (ffv1enc.c:1415-1444), name "ffv1_hip".

    ``encode2(frame, pts)`` is AVCodec.encode2 (avcodec.h:3642-3643) under
    AV_CODEC_CAP_DELAY, driven the way avcodec_encode_video2 drives it
    (utils.c:1922-1990): each call hands over one frame (``None`` = flush)
    and returns at most one packet (``got_packet``), or ``None``.  The
    queueing is the library's (``ffv1hip_encode2``, the entry point an
    AVCodec shim's encode2 forwards to): frames are encoded
    on the GPU ``batch`` at a time, one batch coding while the next queues,
    so the first packet comes out with frame ``avctx.delay`` + 1 (2 x batch
    - 1 frames of delay) and the encoder then returns one packet per call; a
    ``None`` frame encodes what is queued and the caller keeps flushing until
    ``None`` comes back (ffmpeg.c:1699-1776).  Every packet carries pts = dts
    = its frame's pts and the KEY flag (ffv1enc.c:1365-1370).
    """

    name = "ffv1_hip"
    long_name = "FFmpeg video codec #1 (MI355X HIP)"
    capabilities = ("SLICE_THREADS", "DELAY")
    pix_fmts = ("yuv420p", "yuv422p", "yuv444p", "yuv440p", "yuv411p", "yuv410p", "gray",
                "yuv420p9", "yuv422p9", "yuv444p9", "yuv420p10", "yuv422p10", "yuv444p10",
                "yuv420p16", "yuv422p16", "yuv444p16", "gray16", "bgr0", "0rgb32", "gbrp9",
                "gbrp10", "gbrp12", "gbrp14", "yuva420p", "yuva422p", "yuva444p", "yuva420p9",
                "yuva422p9", "yuva444p9", "yuva420p10", "yuva422p10", "yuva444p10", "yuva420p16",
                "yuva422p16", "yuva444p16", "ya8", "bgra", "rgb32")

    def __init__(self, batch: int = 12, device: int = 0):
        if batch < 1:
            raise ValueError("batch must be >= 1")
        self.batch = batch
        self.device = device
        self.avctx: Optional[AVCodecContext] = None
        self.params: Optional[Params] = None
        self._enc: Optional[HipEncoder] = None
        self._pass = 0
        self._frames_in = 0
        self._out = None

    def init(self, avctx: AVCodecContext) -> int:
        self.avctx = avctx
        pass_ = 1 if avctx.flags & AV_CODEC_FLAG_PASS1 else 2 if avctx.flags & AV_CODEC_FLAG_PASS2 else 0
        self.params = configure(avctx.width, avctx.height, avctx.pix_fmt, avctx.slices,
                                avctx.level, avctx.coder, avctx.context, avctx.gop_size,
                                avctx.bits_per_raw_sample, avctx.slicecrc,
                                avctx.allow_large_grid, pass_,
                                avctx.strict_std_compliance <= FF_COMPLIANCE_EXPERIMENTAL)
        self._enc = HipEncoder(self.params, self.device, self.batch)
        self._pass = pass_
        if pass_ == 1 or (pass_ == 2 and avctx.stats_in is not None):
            self._enc.set_pass(pass_, avctx.stats_in)
        avctx.extradata = self._enc.extradata()
        avctx.delay = self._enc.encode2_delay()
        return 0

    def encode2(self, frame: Optional[Sequence[np.ndarray]], pts: Optional[int] = None) -> Optional[AVPacket]:
        if self._enc is None:
            raise FFV1Error(-22, "encode2 before init")
        L = load_library()
        ptrs = (ctypes.c_void_p * 4)()
        strides = (ctypes.c_int * 4)()
        keep = []
        if frame is not None:
            check_planes(self.params, frame)
            np_planes = len(self.params.plane_shapes())
            for k in range(np_planes):
                a = np.ascontiguousarray(frame[min(k, np_planes - 1)])
                keep.append(a)
                ptrs[k] = a.ctypes.data
                strides[k] = a.strides[0]
            if pts is None:
                pts = self._frames_in
            self._frames_in += 1
        size, pts_out = ctypes.c_int64(), ctypes.c_int64()
        key, got = ctypes.c_int(), ctypes.c_int()
        # the shim flow (include/ffv1hip.h): the packet handed out without a
        # copy, then copied into a buffer of exactly its size (ff_alloc_packet2)
        rc = L.ffv1hip_encode2(self._enc._h, ptrs if frame is not None else None,
                               strides if frame is not None else None, pts or 0, None, 0,
                               ctypes.byref(size), ctypes.byref(pts_out), ctypes.byref(key), ctypes.byref(got))
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_encode2")
        if not got.value:
            if frame is None and self._pass == 1:  # the flush: stats_out (ffv1enc.c:1236-1277)
                self.avctx.stats_out = self._enc.stats_out()
            return None
        out = np.empty(max(1, size.value), np.uint8)
        n = L.ffv1hip_encode2_last_packet(self._enc._h, _u8p(out), out.size)
        if n < 0:
            raise FFV1Error(int(n), "ffv1hip_encode2_last_packet")
        return AVPacket(out[:n].tobytes(), pts_out.value, pts_out.value, bool(key.value))

    def close(self) -> int:
        if self._enc is not None:
            self._enc.close()
            self._enc = None
        return 0


class HipDecoder:
    """Owner of one ``ffv1hip_dec``: ff_ffv1_decoder's decode_frame on the GPU
    (ffv1dec.c:896-1005) for every stream the encoder writes (versions 0, 1,
    3 and 4, range or Golomb-Rice, context model 0 / 1, YCbCr / RGB, alpha).
    Context states carry across :meth:`decode` calls like the encoder's."""

    def __init__(self, params: Params, extradata: bytes, device: int = 0):
        L = load_library()
        self.params = params
        err = ctypes.c_int(0)
        ex = np.frombuffer(bytes(extradata) or b"\0", np.uint8).copy()
        self._h = L.ffv1hip_dec_create(ctypes.byref(params), _u8p(ex), len(extradata), device,
                                       ctypes.byref(err))
        if not self._h:
            raise FFV1Error(err.value, "ffv1hip_dec_create")

    def close(self):
        if getattr(self, "_h", None):
            load_library().ffv1hip_dec_destroy(self._h)
            self._h = None

    __del__ = close

    def reset(self):
        load_library().ffv1hip_dec_reset(self._h)

    @property
    def damaged_slices(self) -> int:
        """(frame, slice) pairs of the last decode call that were damaged
        (CRC, slice header or end mismatch) and concealed."""
        return load_library().ffv1hip_dec_damaged_slices(self._h)

    def decode(self, packets: Sequence[bytes]) -> List[Tuple[List[np.ndarray], bool]]:
        """Decode packets in order; returns (planes, key) per frame, planes as
        2-D uint8/uint16 arrays in the encoder's input layout."""
        L = load_library()
        n = len(packets)
        if n == 0:
            return []
        buf = np.frombuffer(b"".join(packets), np.uint8).copy()
        sizes = (ctypes.c_int64 * n)(*[len(pk) for pk in packets])
        dt = np.uint8 if self.params.sample_bytes in (1, 4) else np.uint16
        shapes = self.params.plane_shapes()
        frames = [[np.zeros(shp, dt) for shp in shapes] for _ in range(n)]
        npf = self.params.planes_per_frame
        ptrs = (ctypes.c_void_p * (npf * n))()
        strides = (ctypes.c_int * (npf * n))()
        for i, fr in enumerate(frames):
            for k in range(npf):
                a = fr[min(k, len(fr) - 1)]
                ptrs[npf * i + k] = a.ctypes.data
                strides[npf * i + k] = a.strides[0]
        keys = (ctypes.c_int * n)()
        rc = L.ffv1hip_decode(self._h, _u8p(buf), sizes, n, ptrs, strides, keys)
        if rc < 0:
            raise FFV1Error(rc, "ffv1hip_decode")
        return [(frames[i], bool(keys[i])) for i in range(n)]
