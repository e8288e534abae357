"""GPU decoder (ffv1_decode_slices + ffv1_conceal, through the C-ABI)
against the CPU oracle.

The oracle's decoder (oracle/ffv1_oracle.c, following ffv1dec.c) is the
checker: for every stream of the parity matrix -- range coder and
Golomb-Rice, context models 0 and 1, versions 0, 1 and 3, YCbCr and RGB --
the HIP decoder must return exactly the oracle decoder's samples for the
oracle encoder's packets, and the input frames themselves where the stream
is lossless.  Damaged slices (a flipped byte: CRC mismatch) are decoded on
and concealed as ffv1dec.c:963-977, 998-1021 do; the HIP decoder must give
the oracle's pictures for them too.  At full size (4K 10-bit, BASELINE
configs[2]) the property is the lossless round trip HIP encode -> HIP
decode.  Error cases follow ffv1dec.c:931-989 (slice sizes, a stream that
starts with a P-frame).
"""
import numpy as np
import pytest

from helpers import PARITY_STREAMS, RGB_STREAMS, Stream, corrupt_slice, oracle_encode
from oracle import oracle

pytestmark = pytest.mark.gpu

DEC_STREAMS = PARITY_STREAMS + RGB_STREAMS


def hip_params(s: Stream):
    from ffv1hip import configure
    return configure(s.width, s.height, s.pix_fmt, slices=s.slices, level=s.level, coder=s.coder,
                     context=s.context, gop_size=s.gop_size,
                     bits_per_raw_sample=s.bits_per_raw_sample,
                     allow_large_grid=s.allow_large_grid)


@pytest.mark.parametrize("stream", DEC_STREAMS, ids=[s.name for s in DEC_STREAMS])
def test_hip_decoder_matches_oracle_decoder(stream):
    from ffv1hip import HipDecoder
    frames = list(stream.frames())
    cfg, ex, pkts = oracle_encode(stream, frames)
    odec = oracle.Decoder(cfg, ex)
    hdec = HipDecoder(hip_params(stream), ex, 0)
    got = hdec.decode([p for p, _ in pkts])
    for i, ((p, key), (planes, k)) in enumerate(zip(pkts, got)):
        ref, rk = odec.decode(p)
        assert k == key == rk, f"frame {i}: key flag"
        for a, b in zip(planes, ref):
            np.testing.assert_array_equal(a, b, err_msg=f"frame {i}")
        if stream.lossless:
            for a, b in zip(planes, frames[i]):
                if stream.pix_fmt == "bgr0":  # the padding byte comes back 0
                    b = b.copy()
                    b[:, 3::4] = 0
                np.testing.assert_array_equal(a, b, err_msg=f"frame {i}: not lossless")
    hdec.close()


def test_hip_decoder_state_carry_across_calls():
    """Split calls continue the P-frame chain like one call (ffv1dec.c keeps
    the slice contexts between decode_frame calls)."""
    from ffv1hip import HipDecoder
    s = Stream("p10_gop5", 320, 180, "yuv420p10", 8, slices=6, gop_size=5, source="d2", depth=10)
    frames = list(s.frames())
    _, ex, pkts = oracle_encode(s, frames)
    dec = HipDecoder(hip_params(s), ex, 0)
    got = []
    for lo, hi in ((0, 2), (2, 3), (3, 8)):
        got += dec.decode([p for p, _ in pkts[lo:hi]])
    for i, (planes, _) in enumerate(got):
        for a, b in zip(planes, frames[i]):
            np.testing.assert_array_equal(a, b, err_msg=f"frame {i}")


def test_hip_decoder_errors():
    from ffv1hip import AVERROR_INVALIDDATA, FFV1Error, HipDecoder
    s = Stream("err", 176, 144, "yuv420p10", 3, slices=4, gop_size=3, depth=10)
    _, ex, pkts = oracle_encode(s)
    # a stream may not start with a P-frame
    dec = HipDecoder(hip_params(s), ex, 0)
    with pytest.raises(FFV1Error) as e:
        dec.decode([pkts[1][0]])
    assert e.value.code == AVERROR_INVALIDDATA
    # a truncated packet breaks the slice chain
    with pytest.raises(FFV1Error):
        dec.decode([pkts[0][0][:-7]])
    # extradata of other parameters is refused
    with pytest.raises(FFV1Error):
        HipDecoder(hip_params(s), ex[:-1] + bytes([ex[-1] ^ 1]), 0)
    # after the errors the decoder still decodes a keyframe-led stream
    got = dec.decode([p for p, _ in pkts])
    assert [k for _, k in got] == [True, False, False]
    dec.close()


CONCEAL_STREAMS = [
    Stream("conceal_range", 176, 144, "yuv420p", 9, slices=4, gop_size=4),
    Stream("conceal_p10_ctx1", 160, 120, "yuv420p10", 7, slices=6, gop_size=3, context=1, depth=10),
    Stream("conceal_golomb", 176, 144, "yuv422p", 7, slices=4, coder=0, gop_size=4, source="random"),
    Stream("conceal_bgr0", 96, 64, "bgr0", 6, slices=4, level=3, gop_size=3, source="random"),
    Stream("conceal_gbrp10", 96, 64, "gbrp10", 6, slices=4, gop_size=3, source="random"),
]


@pytest.mark.parametrize("stream", CONCEAL_STREAMS, ids=[s.name for s in CONCEAL_STREAMS])
def test_hip_decoder_conceals_like_oracle(stream):
    """Flipped bytes in a keyframe slice and in P-frame slices: the slices
    fail their CRC, decode on (garbage and all) and are concealed from the
    previous picture until the next keyframe -- sample for sample what the
    oracle decoder (ffv1dec.c) gives, across two calls."""
    from ffv1hip import HipDecoder
    frames = list(stream.frames())
    cfg, ex, pkts = oracle_encode(stream, frames)
    ns = cfg.num_h_slices * cfg.num_v_slices
    bad = [p for p, _ in pkts]
    bad[0] = corrupt_slice(bad[0], True, ns, ns - 1)
    bad[1] = corrupt_slice(bad[1], True, ns, 1)
    bad[4] = corrupt_slice(bad[4], True, ns, 0)
    odec = oracle.Decoder(cfg, ex)
    want = [odec.decode(p)[0] for p in bad]
    hdec = HipDecoder(hip_params(stream), ex, 0)
    got = [pl for pl, _ in hdec.decode(bad[:3])]
    assert hdec.damaged_slices >= 2
    got += [pl for pl, _ in hdec.decode(bad[3:])]
    hdec.close()
    for i, (g, w) in enumerate(zip(got, want)):
        for a, b in zip(g, w):
            np.testing.assert_array_equal(a, b, err_msg=f"frame {i}")


def _swap_slices(packet: bytes, ec: bool, nslices: int, i: int, j: int) -> bytes:
    """The packet with the coded slices at positions i and j exchanged, each
    with its own trailer (size, and with ec its CRC, which stays valid)."""
    trailer = 3 + (5 if ec else 0)
    end, chunks = len(packet), []
    for _ in range(nslices):
        size = int.from_bytes(packet[end - trailer:end - trailer + 3], "big")
        chunks.append(packet[end - trailer - size:end])
        end -= size + trailer
    chunks.reverse()
    assert end == 0
    chunks[i], chunks[j] = chunks[j], chunks[i]
    return b"".join(chunks)


def test_hip_decoder_header_naming_another_slice_diverges():
    """The one documented divergence ("Known reference quirks"):
    a slice header that parses but names another slice's rectangle.  Slices
    1 and 2 of a keyframe exchanged (CRCs intact, no key bit in either):
    the reference decoder decodes each slice into the rectangle its header
    names with the states of the slice position (ffv1dec.c:282-359, 410-419),
    which a keyframe has just reset, so the oracle decoder returns the input
    picture exactly; the GPU decoder counts both headers as failed, leaves
    the two rectangles undecoded and reports them damaged, and decodes every
    other slice as the oracle does."""
    from ffv1hip import HipDecoder
    from helpers import slice_rect
    s = Stream("swap", 192, 96, "yuv420p10", 1, slices=6, gop_size=1, source="random", depth=10)
    frames = list(s.frames())
    cfg, ex, pkts = oracle_encode(s, frames)
    ns = cfg.num_h_slices * cfg.num_v_slices
    bad = _swap_slices(pkts[0][0], True, ns, 1, 2)
    assert bad != pkts[0][0] and len(bad) == len(pkts[0][0])
    want, key = oracle.Decoder(cfg, ex).decode(bad)
    assert key
    for a, b in zip(want, frames[0]):  # the reference's behaviour: decoded into the named rectangles
        np.testing.assert_array_equal(a, b)
    hdec = HipDecoder(hip_params(s), ex, 0)
    (got, k), = hdec.decode([bad])
    assert k and hdec.damaged_slices == 2
    hdec.close()
    mask = np.zeros((s.height, s.width), bool)
    for i in (1, 2):
        x0, y0, x1, y1 = slice_rect(cfg, i)
        mask[y0:y1, x0:x1] = True
    # luma: equal outside the two rectangles, different inside (left undecoded)
    np.testing.assert_array_equal(got[0][~mask], want[0][~mask])
    assert (got[0][mask] != want[0][mask]).mean() > 0.9


def test_hip_encode_decode_4k_p10_roundtrip():
    """BASELINE configs[2] at full size: HIP encoder -> HIP decoder is lossless."""
    from ffv1hip import HipDecoder, HipEncoder
    s = Stream("c3", 3840, 2160, "yuv420p10", 4, slices=64, gop_size=3, source="d2", depth=10)
    frames = list(s.frames())
    enc = HipEncoder(hip_params(s), 0, 4)
    ex = enc.extradata()
    pkts = enc.encode(frames)
    enc.close()
    dec = HipDecoder(hip_params(s), ex, 0)
    got = dec.decode([p for p, _ in pkts])
    for i, ((planes, k), (_, key)) in enumerate(zip(got, pkts)):
        assert k == key
        for a, b in zip(planes, frames[i]):
            np.testing.assert_array_equal(a, b, err_msg=f"frame {i}")
    dec.close()


@pytest.mark.parametrize("shape", ["8k_grid16", "1080p_intra_8bit", "4k_444p12"])
def test_hip_encode_decode_roundtrip_baseline_shapes(shape):
    """The other BASELINE configs at full frame size: HIP encode -> HIP decode
    returns the input (8K has no reference bitstream; this is its check)."""
    from ffv1hip import HipDecoder, HipEncoder
    s = {
        "8k_grid16": Stream("8k", 7680, 4320, "yuv420p10", 3, slices=256, gop_size=2, source="d2",
                            depth=10, allow_large_grid=True, extra={"grid": (16, 16)}),
        "1080p_intra_8bit": Stream("c2", 1920, 1080, "yuv420p", 3, slices=24, gop_size=1),
        "4k_444p12": Stream("c4", 3840, 2160, "yuv444p16", 3, slices=64, gop_size=12,
                            bits_per_raw_sample=12, depth=16, chroma444=True),
    }[shape]
    frames = list(s.frames())
    enc = HipEncoder(hip_params(s), 0, len(frames))
    ex = enc.extradata()
    pkts = enc.encode(frames)
    enc.close()
    dec = HipDecoder(hip_params(s), ex, 0)
    got = dec.decode([p for p, _ in pkts])
    dec.close()
    for i, ((planes, k), (_, key)) in enumerate(zip(got, pkts)):
        assert k == key
        for a, b in zip(planes, frames[i]):
            np.testing.assert_array_equal(a, b, err_msg=f"frame {i}")
