"""2-pass encoding on the GPU (ffv1enc.c:898-986, 1236-1277) against the oracle.

Pass 1: the statistics text (every plane decision counted by state value and
by (context, slot), the keyframe count) equals the oracle's for the same
clip.  Pass 2: from the same stats_in, the extradata (re-sorted custom table,
initial states) and every packet equal the oracle's; the GPU decoder reads
the stream back losslessly.  Parity here is against the oracle restatement:
the reference holds no 2-pass fixture ("parity unpinned").
"""
import numpy as np
import pytest

from helpers import Stream

pytestmark = pytest.mark.gpu

TWO_PASS = [
    Stream("p10_custom", 240, 160, "yuv420p10", 7, slices=4, coder=1, gop_size=3, depth=10),
    Stream("p8_default", 176, 144, "yuv420p", 5, slices=4, coder=-2, gop_size=2),
    Stream("ctx1_chained", 160, 120, "yuv420p10", 4, slices=4, coder=1, context=1, gop_size=2,
           source="d2", depth=10),
    Stream("bgr0_chained", 96, 64, "bgr0", 4, slices=4, coder=1, gop_size=2, source="random"),
    # version 2: the initial states in its extradata, read back at keyframes
    Stream("p8_v2", 176, 144, "yuv420p", 4, level=2, slices=4, coder=1, gop_size=2, experimental=True),
]
# pass 1 on the chained coder beyond TWO_PASS: alpha (a third plane context)
# and version 4 (RCT coefficients per slice); parity unpinned
PASS1_EXTRA = [
    Stream("yuva_chained", 128, 96, "yuva420p10", 3, slices=4, coder=1, gop_size=2, source="random", depth=10),
    Stream("gbrp12_v4", 96, 64, "gbrp12", 3, slices=4, coder=1, gop_size=2, source="random", experimental=True),
]


def _kw(s):
    kw = dict(slices=s.slices, coder=s.coder, context=s.context, gop_size=s.gop_size)
    if s.experimental:
        kw.update(level=s.level if s.level >= 0 else 4, experimental=True)
    return kw


def _oracle_pass1(s, frames):
    from oracle import oracle
    e = oracle.Encoder(oracle.configure(s.width, s.height, s.pix_fmt, pass_=1, **_kw(s)), 1)
    for f in frames:
        e.encode(f)
    return e.stats_out()


@pytest.mark.parametrize("stream", TWO_PASS + PASS1_EXTRA, ids=[s.name for s in TWO_PASS + PASS1_EXTRA])
def test_pass1_statistics_match_oracle(stream):
    """Frame-parallel (YCbCr, context model 0: from the decision stream and
    the walk records) and chained (context model 1, RGB, alpha, version 4:
    counted by ffv1_code as it codes) pass-1 statistics, equal to the
    oracle's text."""
    from ffv1hip import HipEncoder, configure
    frames = list(stream.frames())
    enc = HipEncoder(configure(stream.width, stream.height, stream.pix_fmt, pass_=1, **_kw(stream)), 0, 3)
    enc.set_pass(1)
    for i in range(0, len(frames), 3):
        enc.encode(frames[i:i + 3])
    got = enc.stats_out()
    enc.close()
    assert got == _oracle_pass1(stream, frames)


def test_pass1_golomb_counts_nothing():
    from ffv1hip import HipEncoder, configure
    s = Stream("g", 96, 64, "yuv420p", 4, slices=4, coder=0, gop_size=2)
    frames = list(s.frames())
    enc = HipEncoder(configure(s.width, s.height, s.pix_fmt, pass_=1, **_kw(s)), 0, 4)
    enc.set_pass(1)
    enc.encode(frames)
    assert enc.stats_out() == _oracle_pass1(s, frames)
    enc.close()


@pytest.mark.parametrize("stream", TWO_PASS, ids=[s.name for s in TWO_PASS])
def test_pass2_matches_oracle_and_decodes(stream):
    from ffv1hip import HipDecoder, HipEncoder, configure
    from oracle import oracle
    frames = list(stream.frames())
    stats = _oracle_pass1(stream, frames)
    cfg = oracle.configure(stream.width, stream.height, stream.pix_fmt, pass_=2, **_kw(stream))
    ref = oracle.Encoder(cfg, 2, stats)
    ref_ex = ref.extradata()
    ref_pk = [ref.encode(f) for f in frames]
    params = configure(stream.width, stream.height, stream.pix_fmt, pass_=2, **_kw(stream))
    enc = HipEncoder(params, 0, 2)
    enc.set_pass(2, stats)
    ex = enc.extradata()
    pk = []
    for i in range(0, len(frames), 2):
        pk += enc.encode(frames[i:i + 2])
    enc.close()
    assert ex == ref_ex
    assert pk == ref_pk
    dec = HipDecoder(params, ex, 0)
    for (planes, _), f in zip(dec.decode([p for p, _ in pk]), frames):
        for a, b in zip(planes, f):
            if stream.pix_fmt == "bgr0":
                b = b.copy()
                b[:, 3::4] = 0
            np.testing.assert_array_equal(a, b)
    dec.close()


def test_avcodec_flags_two_pass():
    """FFV1Encoder with AV_CODEC_FLAG_PASS1 leaves stats_out at the flush;
    a PASS2 run from it equals the HipEncoder's pass-2 packets."""
    from ffv1hip import AV_CODEC_FLAG_PASS1, AV_CODEC_FLAG_PASS2, AVCodecContext, FFV1Encoder
    s = TWO_PASS[0]
    frames = list(s.frames())

    def run(flags, stats_in=None):
        avctx = AVCodecContext(s.width, s.height, s.pix_fmt, gop_size=s.gop_size, slices=s.slices,
                               coder=s.coder, flags=flags, stats_in=stats_in)
        enc = FFV1Encoder(batch=3)
        enc.init(avctx)
        out = [enc.encode2(f, i) for i, f in enumerate(frames)]
        while (pkt := enc.encode2(None)) is not None:
            out.append(pkt)
        enc.close()
        return avctx, [p for p in out if p is not None]

    a1, _ = run(AV_CODEC_FLAG_PASS1)
    assert a1.stats_out == _oracle_pass1(s, frames)
    a2, pk = run(AV_CODEC_FLAG_PASS2, a1.stats_out)
    from oracle import oracle
    ref = oracle.Encoder(oracle.configure(s.width, s.height, s.pix_fmt, pass_=2, **_kw(s)), 2, a1.stats_out)
    assert a2.extradata == ref.extradata()
    assert [(p.data, p.key) for p in pk] == [ref.encode(f) for f in frames]
