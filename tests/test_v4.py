"""FFV1 version 4 (`-strict experimental`, level 4; ffv1enc.c:703-706):
micro_version 2 in the extradata (:566-570), per-slice RCT luma
coefficients from choose_rct_params (:1064-1144) used by the colour
transform (:450) and written in the slice header with slice_coding_mode
(:1052-1061), and the PCM re-code of a range-coded slice that runs out of
its buffer (:282-286, 294-304, 1207-1217; buffers :1281-1282, 1317-1322),
on the GPU too.
The decoder side is ffv1dec.c:344-356, 111-120, 252-269, 414-415.

Parity unpinned: the reference's FATE set has no version-4 vector, so the
oracle's restatement is checked by its own lossless round trip, and the HIP
encoder byte-for-byte against the oracle.  Version 4 is admitted where the
reference's choose_rct_params reads stay inside the frame: the RGB formats
and >8-bit 4:4:4 YCbCr (8-bit YCbCr is read as 32-bit RGB words, subsampled
chroma at luma positions, gray through null planes 1 and 2).
"""
import numpy as np
import pytest

from helpers import Stream, oracle, oracle_encode

V4_STREAMS = [
    Stream("v4_bgr0_range", 96, 64, "bgr0", 5, level=4, slices=4, coder=1, gop_size=3, source="random",
           experimental=True, seed=11),
    Stream("v4_bgra_golomb", 64, 48, "bgra", 4, level=4, slices=4, coder=0, gop_size=2, source="random",
           experimental=True, seed=12),
    Stream("v4_gbrp10_ctx1", 80, 48, "gbrp10", 4, level=4, slices=6, coder=1, context=1, gop_size=4,
           source="random", experimental=True, seed=13),
    Stream("v4_gbrp14_default_tab", 64, 40, "gbrp14", 3, level=4, slices=4, coder=-2, gop_size=2,
           source="random", experimental=True, seed=14),
    Stream("v4_yuv444p10", 64, 48, "yuv444p10", 4, level=4, slices=4, coder=1, gop_size=2, source="random",
           experimental=True, seed=15),
    Stream("v4_yuva444p16_ctx1", 48, 32, "yuva444p16", 3, level=4, slices=4, coder=1, context=1, gop_size=3,
           source="random", experimental=True, seed=16),
]
IDS = [s.name for s in V4_STREAMS]


def _lossless(cfg, ex, pkts, frames):
    dec = oracle.Decoder(cfg, ex)
    for (pk, key), fr in zip(pkts, frames):
        planes, k = dec.decode(pk)
        assert k == key
        for a, b in zip(planes, fr):
            if cfg.colorspace and cfg.sample_bytes == 4 and not cfg.transparency:
                a, b = a.reshape(a.shape[0], -1, 4)[..., :3], b.reshape(b.shape[0], -1, 4)[..., :3]
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("stream", V4_STREAMS, ids=IDS)
def test_oracle_v4_roundtrip(stream):
    frames = list(stream.frames())
    cfg, ex, pkts = oracle_encode(stream, frames)
    assert cfg.version == 4
    _lossless(cfg, ex, pkts, frames)


def test_v4_needs_experimental_and_a_readable_format():
    with pytest.raises(ValueError):  # AVERROR_INVALIDDATA without -strict experimental
        oracle.configure(64, 48, "bgr0", level=4)
    for fmt in ("yuv420p10", "yuv444p", "gray16", "ya8", "yuva420p10"):
        with pytest.raises(ValueError):
            oracle.configure(64, 48, fmt, level=4, experimental=True)
    assert oracle.configure(64, 48, "yuv444p16", level=4, experimental=True).version == 4


def test_v4_rct_coefficients_follow_the_content():
    """A slice whose R carries G's detail and B is flat picks a coefficient
    pair other than (1, 1); the stream still decodes losslessly, and differs
    from the same frame coded at version 3 beyond the header."""
    W, H = 64, 32
    rng = np.random.default_rng(3)
    g = rng.integers(0, 200, size=(H, W))
    px = np.zeros((H, W, 4), np.uint8)
    px[..., 1] = g
    px[..., 2] = np.clip(g + rng.integers(0, 2, size=(H, W)), 0, 255)
    px[..., 0] = 17
    frame = [np.ascontiguousarray(px.reshape(H, 4 * W))]
    cfg4 = oracle.configure(W, H, "bgr0", level=4, slices=4, coder=1, experimental=True)
    enc = oracle.Encoder(cfg4)
    pk4 = enc.encode(frame)
    _lossless(cfg4, enc.extradata(), [pk4], [frame])
    cfg3 = oracle.configure(W, H, "bgr0", level=3, slices=4, coder=1)
    pk3 = oracle.Encoder(cfg3).encode(frame)
    assert len(pk4[0]) < len(pk3[0])  # the better transform codes smaller


def test_v4_pcm_fallback():
    """Slices two rows high in a 370-400 wide gbrp14 frame of noise run out
    of their 1/6 of the 12-bytes-per-pixel packet partway (the 35 * w check)
    and are coded again as PCM; slice 0 owns the whole packet and never
    does.  The PCM stream decodes losslessly."""
    rng = np.random.default_rng(1)
    cfg = oracle.configure(376, 4, "gbrp14", level=4, slices=6, coder=1, gop_size=2, experimental=True)
    frames = [[np.ascontiguousarray(rng.integers(0, 1 << 14, size=s).astype(np.uint16))
               for s in oracle.plane_shapes(cfg)] for _ in range(3)]
    enc = oracle.Encoder(cfg)
    pkts, modes = [], []
    for f in frames:
        pkts.append(enc.encode(f))
        modes.append(enc.last_slice_pcm())
    assert all(m == [0, 1, 1, 1, 1, 1] for m in modes)
    _lossless(cfg, enc.extradata(), pkts, frames)


@pytest.mark.gpu
@pytest.mark.parametrize("stream", V4_STREAMS, ids=IDS)
def test_hip_v4_matches_oracle(stream):
    """HIP (RCT coefficients chosen on the device per frame and slice, the
    slice header taking them) against the oracle, batch of 3."""
    from test_gpu_parity import hip_encode
    frames = list(stream.frames())
    _, ex_ref, ref = oracle_encode(stream, frames)
    ex, got = hip_encode(stream, frames, batch=3)
    assert ex == ex_ref
    for i, (g, r) in enumerate(zip(got, ref)):
        assert g == r, f"frame {i}"


def _pcm_frames(pix_fmt, w, h, slices, mixed, n=5, seed=1):
    """Noise frames whose thin slices fail the 35 * w buffer check; with
    `mixed`, every other frame is a smooth ramp that codes normally, so the
    P-frame carry after a PCM slice (its states cleared by the PCM slice
    header, ffv1enc.c:1054-1055) is exercised."""
    cfg = oracle.configure(w, h, pix_fmt, level=4, slices=slices, coder=1, gop_size=3, experimental=True)
    rng = np.random.default_rng(seed)
    hi = 1 << (16 if cfg.sample_bytes == 2 and not cfg.packed_at_lsb else cfg.bits_per_raw_sample)
    frames = []
    for t in range(n):
        fr = []
        for s in oracle.plane_shapes(cfg):
            if mixed and t % 2:
                yy, xx = np.mgrid[0:s[0], 0:s[1]]
                a = (xx * 7 + yy * 3 + t) % hi
            else:
                a = rng.integers(0, hi, size=s)
            fr.append(np.ascontiguousarray(a.astype(np.uint16)))
        frames.append(fr)
    return cfg, frames


PCM_CASES = [("gbrp14", 376, 4, 6, False), ("yuv444p16", 376, 4, 6, False), ("gbrp14", 376, 12, 12, True),
             ("yuv444p16", 376, 12, 12, True)]


@pytest.mark.parametrize("case", PCM_CASES, ids=[f"{c[0]}_{c[1]}x{c[2]}_s{c[3]}{'_mixed' if c[4] else ''}"
                                                  for c in PCM_CASES])
def test_oracle_v4_pcm_cases_code_pcm_and_roundtrip(case):
    cfg, frames = _pcm_frames(*case, n=5)
    enc = oracle.Encoder(cfg)
    pkts, modes = [], []
    for f in frames:
        pkts.append(enc.encode(f))
        modes.append(enc.last_slice_pcm())
    assert any(any(m) for m in modes)
    _lossless(cfg, enc.extradata(), pkts, frames)


@pytest.mark.gpu
@pytest.mark.parametrize("case", PCM_CASES, ids=[f"{c[0]}_{c[1]}x{c[2]}_s{c[3]}{'_mixed' if c[4] else ''}"
                                                  for c in PCM_CASES])
def test_hip_v4_pcm_matches_oracle(case):
    """Where the reference re-codes slices as PCM (the per-line 35 * w check,
    ffv1enc.c:282-286, 1207-1217), the chained HIP coder does the same on the
    device: the packets equal the oracle's (parity unpinned: no reference
    vector for version 4)."""
    from ffv1hip import HipEncoder, configure
    pix_fmt, w, h, slices, mixed = case
    cfg, frames = _pcm_frames(*case, n=5)
    enc = oracle.Encoder(cfg)
    ref = [enc.encode(f) for f in frames]
    p = configure(w, h, pix_fmt, slices=slices, level=4, coder=1, gop_size=3, experimental=True)
    henc = HipEncoder(p, 0, 2)
    got = henc.encode(frames)
    henc.close()
    for i, (g, r) in enumerate(zip(got, ref)):
        assert g == r, f"frame {i}"


def _v4_params(s):
    from ffv1hip import configure
    return configure(s.width, s.height, s.pix_fmt, slices=s.slices, level=4, coder=s.coder, context=s.context,
                     gop_size=s.gop_size, experimental=True)


@pytest.mark.gpu
@pytest.mark.parametrize("stream", V4_STREAMS, ids=IDS)
def test_gpu_decoder_v4_matches_oracle_decoder(stream):
    """ffv1_decode_slices on version 4 (ffv1dec.c:344-356 the slice header's
    reset bit, slice_coding_mode and RCT coefficients, 252-269 the RCT with
    them): the oracle decoder's samples, losslessly the input."""
    from test_alpha import gpu_decode_vs_oracle
    frames = list(stream.frames())
    cfg, ex, pkts = oracle_encode(stream, frames)
    gpu_decode_vs_oracle(_v4_params(stream), cfg, ex, pkts, frames, pad_byte=stream.pix_fmt == "bgr0")


@pytest.mark.gpu
@pytest.mark.parametrize("case", PCM_CASES, ids=[f"{c[0]}_{c[1]}x{c[2]}_s{c[3]}{'_mixed' if c[4] else ''}"
                                                  for c in PCM_CASES])
def test_gpu_decoder_v4_pcm_slices(case):
    """PCM slices (ffv1dec.c:111-120, every bit on a fresh state 128, no
    RCT) and the states cleared after them (the reset bit): the oracle
    decoder's samples, losslessly the input."""
    from ffv1hip import configure
    from test_alpha import gpu_decode_vs_oracle
    pix_fmt, w, h, slices, mixed = case
    cfg, frames = _pcm_frames(*case, n=5)
    enc = oracle.Encoder(cfg)
    pkts = [enc.encode(f) for f in frames]
    p = configure(w, h, pix_fmt, slices=slices, level=4, coder=1, gop_size=3, experimental=True)
    gpu_decode_vs_oracle(p, cfg, enc.extradata(), pkts, frames)


# Slice 0 owns the whole v4 packet and never fails the 35 * w check at real
# sizes; a test hook lowers its buffer alone (oracle: FFV1_ORACLE_V4_CAP0,
# HIP: FFV1HIP_DEBUG=v4_cap0) so that slice 0 re-codes as PCM: the re-code
# restarts after the key bit with a fresh slice-header state (ffv1enc.c:1031,
# 1157, 1207-1217).  (case, slice 0's buffer bytes)
PCM0_CASES = [(("gbrp14", 376, 8, 4, False), 10250), (("yuv444p16", 340, 8, 4, True), 10000)]
PCM0_IDS = [f"{c[0][0]}_{c[0][1]}x{c[0][2]}{'_mixed' if c[0][4] else ''}" for c in PCM0_CASES]


@pytest.mark.parametrize("case,cap0", PCM0_CASES, ids=PCM0_IDS)
def test_oracle_v4_pcm_slice0_roundtrip(case, cap0, monkeypatch):
    monkeypatch.setenv("FFV1_ORACLE_V4_CAP0", str(cap0))
    cfg, frames = _pcm_frames(*case, n=4)
    enc = oracle.Encoder(cfg)
    pkts, modes = [], []
    for f in frames:
        pkts.append(enc.encode(f))
        modes.append(enc.last_slice_pcm())
    assert modes[0][0] == 1 and modes[2][0] == 1
    _lossless(cfg, enc.extradata(), pkts, frames)


@pytest.mark.gpu
@pytest.mark.parametrize("case,cap0", PCM0_CASES, ids=PCM0_IDS)
def test_hip_v4_pcm_slice0_matches_oracle(case, cap0, monkeypatch):
    """Slice 0 re-coded as PCM (its buffer lowered by the hooks): the HIP
    packets equal the oracle's (parity unpinned)."""
    from ffv1hip import HipEncoder, configure
    monkeypatch.setenv("FFV1_ORACLE_V4_CAP0", str(cap0))
    monkeypatch.setenv("FFV1HIP_DEBUG", f"v4_cap0={cap0}")
    pix_fmt, w, h, slices, mixed = case
    cfg, frames = _pcm_frames(*case, n=4)
    enc = oracle.Encoder(cfg)
    ref = [enc.encode(f) for f in frames]
    p = configure(w, h, pix_fmt, slices=slices, level=4, coder=1, gop_size=3, experimental=True)
    henc = HipEncoder(p, 0, 2)
    got = henc.encode(frames)
    henc.close()
    for i, (g, r) in enumerate(zip(got, ref)):
        assert g == r, f"frame {i}"
