"""Alpha formats: YUVA (the A plane after Cr, plane context 2, ffv1enc.c:
1197-1198), YA8 (Y and A bytes of one packed plane, A with plane context 1,
:1199-1201) and RGB32 (A as the fourth interleaved row of encode_rgb_frame,
plane context (3 + 1) / 2 = 2, coded at 9 bits like the others, :440-467);
plane_count = 3 in the slice header and the states (:720, 890-891); the
decoder side is ffv1dec.c:437-453, 226-280, 558-559.

Parity unpinned: the reference's FATE set holds no FFV1 alpha vector
(tests/fate/vcodec.mak:113-127, tests/ref/vsynth/*ffv1*), so the oracle's
restatement is checked by its own lossless round trip and against the
non-alpha path it extends (a YUVA stream's first planes code as the YUV
stream's), and the HIP encoder byte-for-byte against the oracle.
"""
import numpy as np
import pytest

from helpers import Stream, oracle, oracle_encode

ALPHA_STREAMS = [
    Stream("yuva420p_range_g3", 96, 64, "yuva420p", 7, slices=4, coder=1, gop_size=3, source="random"),
    Stream("yuva420p_golomb_v0", 64, 48, "yuva420p", 5, coder=0, gop_size=2, source="random"),
    Stream("yuva444p10_ctx1", 80, 48, "yuva444p10", 5, slices=4, coder=1, context=1, gop_size=4,
           source="random", seed=3),
    Stream("yuva422p16_range", 64, 36, "yuva422p16", 4, slices=6, coder=1, gop_size=3, source="random",
           seed=4),
    Stream("yuva420p9_default_tab", 64, 40, "yuva420p9", 4, level=3, coder=-2, gop_size=2, source="random",
           seed=5),
    Stream("ya8_range", 72, 40, "ya8", 6, slices=4, coder=1, gop_size=3, source="random", seed=6),
    Stream("ya8_golomb_v1", 48, 32, "ya8", 4, level=1, coder=0, gop_size=2, source="random", seed=7),
    Stream("bgra_range", 64, 48, "bgra", 5, slices=4, coder=1, gop_size=3, source="random", seed=8),
    Stream("bgra_golomb", 48, 40, "bgra", 4, slices=4, coder=0, gop_size=2, source="random", seed=9),
    Stream("rgb32_v1_ctx1", 40, 32, "rgb32", 4, level=1, coder=1, context=1, gop_size=2, source="random",
           seed=10),
]
IDS = [s.name for s in ALPHA_STREAMS]


@pytest.mark.parametrize("stream", ALPHA_STREAMS, ids=IDS)
def test_oracle_alpha_roundtrip(stream):
    """Oracle encoder -> oracle decoder is lossless, keys and all."""
    cfg, ex, pkts = oracle_encode(stream)
    assert cfg.transparency == 1
    dec = oracle.Decoder(cfg, ex)
    for (pk, key), fr in zip(pkts, stream.frames()):
        planes, k = dec.decode(pk)
        assert k == key
        for a, b in zip(planes, fr):
            np.testing.assert_array_equal(a, b)


def test_oracle_alpha_plane_is_coded_last():
    """A YUVA slice codes Y, Cb, Cr exactly as the YUV stream with the same
    options would, then A: with one slice and no CRC, the YUVA packet's
    bytes differ from the YUV packet's only from where A starts, and a
    different A changes the packet."""
    yuv = Stream("a", 64, 48, "yuv420p", 2, level=1, coder=1, gop_size=2, source="random", seed=2)
    frames = list(yuv.frames())
    rng = np.random.default_rng(5)
    alpha = [rng.integers(0, 256, size=(48, 64)).astype(np.uint8) for _ in frames]
    cfg_a = oracle.configure(64, 48, "yuva420p", level=1, coder=1, gop_size=2)
    enc_a = oracle.Encoder(cfg_a)
    pk_a = [enc_a.encode(f + [a])[0] for f, a in zip(frames, alpha)]
    _, _, pk = oracle_encode(yuv, frames)
    assert all(len(a) > len(p) for a, (p, _) in zip(pk_a, pk))
    enc_b = oracle.Encoder(cfg_a)
    pk_b = [enc_b.encode(f + [np.ascontiguousarray(255 - a)])[0] for f, a in zip(frames, alpha)]
    assert pk_b != pk_a


@pytest.mark.gpu
@pytest.mark.parametrize("stream", ALPHA_STREAMS, ids=IDS)
def test_hip_alpha_matches_oracle(stream):
    """The HIP encoder (chained coders, a third plane context) gives the
    oracle's bytes, with P-frame states crossing calls (batch of 3)."""
    from test_gpu_parity import hip_encode
    frames = list(stream.frames())
    _, ex_ref, ref = oracle_encode(stream, frames)
    ex, got = hip_encode(stream, frames, batch=3)
    assert ex == ex_ref
    assert len(got) == len(ref)
    for i, (g, r) in enumerate(zip(got, ref)):
        assert g == r, f"frame {i}"


@pytest.mark.gpu
def test_hip_alpha_encode2_and_states():
    """encode2 one frame per call on a YUVA stream, and the P-frame carry
    (three plane contexts) handed to a second encoder mid-GOP."""
    from ffv1hip import AVCodecContext, FFV1Encoder, HipEncoder
    from test_gpu_parity import hip_params
    s = ALPHA_STREAMS[0]
    frames = list(s.frames())
    _, ex_ref, ref = oracle_encode(s, frames)
    avctx = AVCodecContext(s.width, s.height, s.pix_fmt, gop_size=s.gop_size, slices=s.slices, coder=s.coder)
    enc = FFV1Encoder(batch=2)
    assert enc.init(avctx) == 0
    assert avctx.extradata == ex_ref
    pkts = [enc.encode2(f, pts=i) for i, f in enumerate(frames)]
    pkts = [p for p in pkts if p is not None]
    while (p := enc.encode2(None)) is not None:
        pkts.append(p)
    enc.close()
    assert [(p.data, p.key) for p in pkts] == ref
    a = HipEncoder(hip_params(s), 0, 4)
    head = a.encode(frames[:4])
    blob = a.get_slice_states()
    assert blob.size == 3 * 666 * 32 * s.slices  # plane_count 3
    b = HipEncoder(hip_params(s), 0, 4)
    b.set_slice_states(blob, 4)
    tail = b.encode(frames[4:])
    a.close()
    b.close()
    assert head + tail == ref


def gpu_decode_vs_oracle(params, cfg, ex, pkts, frames=None, pad_byte=False):
    """The GPU decoder's samples equal the oracle decoder's (and the input,
    when frames are given) for every packet; with pad_byte (bgr0) the
    input's unused fourth byte comes back 0."""
    from ffv1hip import HipDecoder
    odec = oracle.Decoder(cfg, ex)
    hdec = HipDecoder(params, ex, 0)
    got = hdec.decode([p for p, _ in pkts])
    hdec.close()
    for i, ((p, key), (planes, k)) in enumerate(zip(pkts, got)):
        ref, rk = odec.decode(p)
        assert k == key == rk, f"frame {i}: key flag"
        assert len(planes) == len(ref)
        for a, b in zip(planes, ref):
            np.testing.assert_array_equal(a, b, err_msg=f"frame {i}")
        if frames is not None:
            for a, b in zip(planes, frames[i]):
                if pad_byte:
                    b = b.copy()
                    b[:, 3::4] = 0
                np.testing.assert_array_equal(a, b, err_msg=f"frame {i}: not lossless")


@pytest.mark.gpu
@pytest.mark.parametrize("stream", ALPHA_STREAMS, ids=IDS)
def test_gpu_decoder_alpha_matches_oracle_decoder(stream):
    """ffv1_decode_slices on alpha streams (ffv1dec.c:437-453: YUVA's A
    plane with plane context 2, YA8's Y and A of one packed plane, RGB32's A
    row): the oracle decoder's samples, which are the input (lossless)."""
    from test_gpu_parity import hip_params
    frames = list(stream.frames())
    cfg, ex, pkts = oracle_encode(stream, frames)
    gpu_decode_vs_oracle(hip_params(stream), cfg, ex, pkts, frames)


@pytest.mark.gpu
def test_gpu_decoder_alpha_conceals_damaged_slices():
    """A flipped byte in a YUVA slice: CRC failure, decoded on, then
    concealed from the previous picture, all four planes, as the oracle."""
    from helpers import corrupt_slice
    from test_gpu_parity import hip_params
    s = Stream("yuva420p_ec", 96, 64, "yuva420p", 5, slices=4, coder=1, gop_size=5, source="random", seed=21)
    frames = list(s.frames())
    cfg, ex, pkts = oracle_encode(s, frames)
    assert cfg.ec
    n = cfg.num_h_slices * cfg.num_v_slices
    pkts = [(corrupt_slice(p, True, n, 1) if i == 2 else p, k) for i, (p, k) in enumerate(pkts)]
    gpu_decode_vs_oracle(hip_params(s), cfg, ex, pkts)
