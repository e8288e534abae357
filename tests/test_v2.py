"""FFV1 version 2 (`-strict experimental`, level 2; ffv1enc.c:703-706): the
configuration in the extradata as at version 3, but without slice headers;
the slice layout and every plane's quant set index travel in-band, in the
keyframe header coded after the key bit (write_header, ffv1enc.c:523-541,
one state array for all of it).  Slice 0 has no size trailer
(ffv1enc.c:1334-1337), and the extradata carries no ec field, so slice CRCs
are refused at version 2 (the reference decoder could not find them).
The decoder side is read_header's v2 branch (ffv1dec.c:801-868).

Parity unpinned: the reference's FATE set has no version-2 vector, so the
oracle's restatement is checked by its own lossless round trip and by the
header's bytes decoded field by field; the HIP encoder is checked
byte-for-byte against the oracle, and the GPU decoder against the oracle
decoder.
"""
import numpy as np
import pytest

from helpers import Stream, oracle, oracle_encode

V2_STREAMS = [
    Stream("v2_yuv420p_range", 96, 64, "yuv420p", 5, level=2, slices=4, coder=1, gop_size=3, source="random",
           experimental=True, seed=21),
    Stream("v2_yuv420p_golomb", 80, 48, "yuv420p", 4, level=2, slices=6, coder=0, gop_size=2, source="random",
           experimental=True, seed=22),
    Stream("v2_yuv422p10_ctx1", 80, 48, "yuv422p10", 4, level=2, slices=6, coder=1, context=1, gop_size=4,
           source="random", experimental=True, seed=23),
    Stream("v2_yuva420p_default_tab", 64, 40, "yuva420p", 3, level=2, slices=4, coder=-2, gop_size=2,
           source="random", experimental=True, seed=24),
    Stream("v2_bgr0", 64, 48, "bgr0", 4, level=2, slices=4, coder=1, gop_size=2, source="random",
           experimental=True, seed=25),
    Stream("v2_gray16_s12", 96, 72, "gray16", 3, level=2, slices=12, coder=1, context=1, gop_size=3,
           source="random", experimental=True, seed=26),
]
IDS = [s.name for s in V2_STREAMS]


def _lossless(cfg, ex, pkts, frames):
    dec = oracle.Decoder(cfg, ex)
    for (pk, key), fr in zip(pkts, frames):
        planes, k = dec.decode(pk)
        assert k == key
        for a, b in zip(planes, fr):
            if cfg.colorspace and cfg.sample_bytes == 4 and not cfg.transparency:
                a, b = a.reshape(a.shape[0], -1, 4)[..., :3], b.reshape(b.shape[0], -1, 4)[..., :3]
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("stream", V2_STREAMS, ids=IDS)
def test_oracle_v2_roundtrip(stream):
    frames = list(stream.frames())
    cfg, ex, pkts = oracle_encode(stream, frames)
    assert cfg.version == 2
    _lossless(cfg, ex, pkts, frames)


def test_v2_needs_experimental_and_no_slice_crc():
    with pytest.raises(ValueError):  # AVERROR_INVALIDDATA without -strict experimental
        oracle.configure(64, 48, "yuv420p", level=2, slices=4)
    with pytest.raises(ValueError):  # no ec field in a v2 extradata
        oracle.configure(64, 48, "yuv420p", level=2, slices=4, slicecrc=1, experimental=True)
    assert oracle.configure(64, 48, "yuv420p", level=2, slices=4, experimental=True).version == 2


@pytest.mark.parametrize("fmt,slices,coder", [("yuv420p", 4, 1), ("yuv422p10", 6, 0), ("bgr0", 12, 1),
                                               ("yuva420p", 0, -2)])
def test_configure_v2_matches_oracle(fmt, slices, coder):
    """The library's configure (host only) takes level 2 with -strict
    experimental as the oracle does, and refuses it without, and with slice
    CRCs."""
    from ffv1hip import configure, FFV1Error
    from test_abi import FIELDS
    ref = oracle.configure(352, 288, fmt, slices=slices, level=2, coder=coder, experimental=True).as_dict()
    got = configure(352, 288, fmt, slices=slices, level=2, coder=coder, experimental=True).as_dict()
    assert got["version"] == 2
    for f in FIELDS:
        assert got[f] == ref[f], f
    with pytest.raises(FFV1Error):
        configure(352, 288, fmt, slices=slices, level=2, coder=coder)
    with pytest.raises(FFV1Error):
        configure(352, 288, fmt, slices=slices, level=2, coder=coder, slicecrc=1, experimental=True)


class _RangeDecoder:
    """get_rac / get_symbol (rangecoder.h:106-135, ffv1dec.c:42-70) with the
    default state table, for reading the keyframe header back here."""

    def __init__(self, buf):
        self.b, self.p = buf, 2
        self.low = (buf[0] << 8) | buf[1]
        self.range = 0xFF00
        one = [0] * 256
        # ff_build_rac_states(c, 0.05 * 2^32, 256 - 8) (rangecoder.c:62-108)
        factor, max_p = int(0.05 * (1 << 32)), 256 - 8
        last_p8, p = 0, (1 << 32) // 2
        for i in range(128):
            p8 = (256 * p + (1 << 31)) >> 32
            if p8 <= last_p8:
                p8 = last_p8 + 1
            if last_p8 and last_p8 < 256 and p8 <= max_p:
                one[last_p8] = p8
            p += ((1 << 32) - p) * factor + (1 << 31) >> 32
            last_p8 = p8
        for i in range(256 - max_p, max_p + 1):
            if one[i]:
                continue
            p = (i * (1 << 32) + 128) >> 8
            p += ((1 << 32) - p) * factor + (1 << 31) >> 32
            p8 = (256 * p + (1 << 31)) >> 32
            if p8 <= i:
                p8 = i + 1
            if p8 > max_p:
                p8 = max_p
            one[i] = p8
        self.one = one
        self.zero = [0] * 256
        for i in range(1, 255):
            self.zero[i] = 256 - one[256 - i]

    def _refill(self):
        if self.range < 0x100:
            self.range <<= 8
            self.low <<= 8
            if self.p < len(self.b):
                self.low += self.b[self.p]
            self.p += 1

    def rac(self, st, i):
        r1 = (self.range * st[i]) >> 8
        self.range -= r1
        if self.low < self.range:
            st[i] = self.zero[st[i]]
            self._refill()
            return 0
        self.low -= self.range
        st[i] = self.one[st[i]]
        self.range = r1
        self._refill()
        return 1

    def symbol(self, st):
        if self.rac(st, 0):
            return 0
        e = 0
        while self.rac(st, 1 + min(e, 9)):
            e += 1
        a = 1
        for i in range(e - 1, -1, -1):
            a += a + self.rac(st, 22 + min(i, 9))
        return a  # unsigned: no sign decision (is_signed 0)


@pytest.mark.parametrize("stream", [V2_STREAMS[0], V2_STREAMS[2], V2_STREAMS[3]], ids=lambda s: s.name)
def test_v2_keyframe_header_fields(stream):
    """The keyframe header read back field by field: slice count, each
    slice's grid position and size in grid units (row-major slice order,
    ffv1.c:125-128), then plane_count quant set indices, all the context
    model; P-frames carry only the key bit before the slice data."""
    frames = list(stream.frames())[:2]
    cfg, ex, pkts = oracle_encode(stream, frames)
    nh, nv = cfg.num_h_slices, cfg.num_v_slices
    d = _RangeDecoder(pkts[0][0])
    ks = [128]
    assert d.rac(ks, 0) == 1
    st = [128] * 32
    assert d.symbol(st) == nh * nv
    planes = 2 + (1 if cfg.transparency else 0)
    for i in range(nh * nv):
        sx, sy = i % nh, i // nh
        assert [d.symbol(st) for _ in range(4)] == [sx, sy, 0, 0]
        assert [d.symbol(st) for _ in range(planes)] == [stream.context] * planes
    assert pkts[1][1] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("stream", V2_STREAMS, ids=IDS)
def test_hip_v2_matches_oracle(stream):
    """HIP (the v2 keyframe header among slice 0's header decisions) against
    the oracle, batch of 3."""
    from test_gpu_parity import hip_encode
    frames = list(stream.frames())
    _, ex_ref, ref = oracle_encode(stream, frames)
    ex, got = hip_encode(stream, frames, batch=3)
    assert ex == ex_ref
    for i, (g, r) in enumerate(zip(got, ref)):
        assert g == r, f"frame {i}"


def _v2_params(s):
    from ffv1hip import configure
    return configure(s.width, s.height, s.pix_fmt, slices=s.slices, level=2, coder=s.coder, context=s.context,
                     gop_size=s.gop_size, experimental=True)


@pytest.mark.gpu
@pytest.mark.parametrize("stream", V2_STREAMS, ids=IDS)
def test_gpu_decoder_v2_matches_oracle_decoder(stream):
    """ffv1_decode_slices on version 2 (the slice layout and quant set from
    the keyframe header, ffv1dec.c:801-868; no slice headers): the oracle
    decoder's samples, losslessly the input."""
    from test_alpha import gpu_decode_vs_oracle
    frames = list(stream.frames())
    cfg, ex, pkts = oracle_encode(stream, frames)
    gpu_decode_vs_oracle(_v2_params(stream), cfg, ex, pkts, frames, pad_byte=stream.pix_fmt == "bgr0")
