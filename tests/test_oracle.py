"""CPU oracle checks: pinned against the reference's own known answers.

The oracle (oracle/ffv1_oracle.c) is the parity checker for the GPU path, so
it is pinned first: it must reproduce the reference encoder's recorded
packet MD5s (tests/golden/known_answers.json), and its decoder
must invert every stream of the parity matrix losslessly.
"""
import hashlib

import numpy as np
import pytest

from helpers import (PARITY_STREAMS, RGB_STREAMS, Stream, corrupt_slice, load_golden, md5, oracle_encode,
                     slice_rect)
from oracle import oracle

PINS = {p["name"]: p for p in load_golden("known_answers.json")["streams"]}


def _check_pin(pin, stream):
    cfg, ex, pkts = oracle_encode(stream)
    if "extradata_md5_prefix" in pin:
        assert len(ex) == pin["extradata_size"]
        assert md5(ex).startswith(pin["extradata_md5_prefix"])
    for i, size in pin.get("frame_sizes", {}).items():
        assert len(pkts[int(i)][0]) == size
    for i, pre in pin.get("frame_md5_prefix", {}).items():
        assert md5(pkts[int(i)][0]).startswith(pre)
    h = hashlib.md5()
    for p, _ in pkts:
        h.update(p)
    assert h.hexdigest() == pin["stream_md5"]
    return pkts


def test_pin_config1_cif_golomb_v0():
    pin = PINS["config1_cif_yuv420p_coder0_g1"]
    _check_pin(pin, Stream("c1", 352, 288, "yuv420p", pin["frames"], coder=0, gop_size=1))


@pytest.mark.slow
def test_pin_config2_1080p_range_intra():
    pin = PINS["config2_1080p_yuv420p_coder1_slices24_g1"]
    _check_pin(pin, Stream("c2", 1920, 1080, "yuv420p", pin["frames"], slices=24, gop_size=1))


@pytest.mark.slow
def test_pin_config3_4k_p10_pframes():
    pin = PINS["config3_4k_yuv420p10_coder1_slices64_g12"]
    pkts = _check_pin(pin, Stream("c3", 3840, 2160, "yuv420p10", pin["frames"], slices=64,
                                  gop_size=12, depth=10))
    assert [k for _, k in pkts] == [i % 12 == 0 for i in range(len(pkts))]


def test_config_derivation_matches_reference_contract():
    # CIF defaults => v0 Golomb, 1 slice; >8 bit forces the range coder (v1)
    c = oracle.configure(352, 288, "yuv420p")
    assert (c.version, c.ac, c.num_h_slices * c.num_v_slices, c.ec) == (0, 0, 1, 0)
    c = oracle.configure(352, 288, "yuv420p10")
    assert (c.version, c.ac) == (1, 2)
    c = oracle.configure(1920, 1080, "yuv420p", coder=1, slices=24)
    assert (c.version, c.num_h_slices, c.num_v_slices, c.ec) == (3, 6, 4, 1)
    c = oracle.configure(3840, 2160, "yuv420p10", coder=1, slices=64)
    assert (c.num_h_slices, c.num_v_slices, c.packed_at_lsb, c.bits_per_raw_sample) == (8, 8, 1, 10)
    c = oracle.configure(3840, 2160, "yuv444p16", coder=1, slices=64, bits_per_raw_sample=12)
    assert (c.packed_at_lsb, c.bits_per_raw_sample, c.chroma_h_shift) == (0, 12, 0)
    with pytest.raises(ValueError):  # slices > 64 are refused (ffv1enc.c:992)
        oracle.configure(7680, 4320, "yuv420p10", coder=1, slices=256)
    with pytest.raises(ValueError):  # 5 slices: no grid
        oracle.configure(1920, 1080, "yuv420p", slices=5)


@pytest.mark.parametrize("stream", PARITY_STREAMS[:-1], ids=[s.name for s in PARITY_STREAMS[:-1]])
def test_oracle_roundtrip_lossless(stream):
    if not stream.lossless:
        pytest.skip("reference leaves chroma columns uncoded for this geometry")
    frames = list(stream.frames())
    cfg, ex, pkts = oracle_encode(stream, frames)
    dec = oracle.Decoder(cfg, ex)
    for (p, key), f in zip(pkts, frames):
        planes, k = dec.decode(p)
        assert k == key
        for a, b in zip(planes, f):
            if cfg.sample_bytes == 2 and not cfg.packed_at_lsb:
                b = (b >> (16 - cfg.bits_per_raw_sample)) << (16 - cfg.bits_per_raw_sample)
            np.testing.assert_array_equal(a, b)


def test_oracle_golomb_roundtrip_and_pframes():
    s = Stream("golomb_v3", 176, 144, "yuv420p", 6, slices=4, coder=0, gop_size=3)
    frames = list(s.frames())
    cfg, ex, pkts = oracle_encode(s, frames)
    assert cfg.version == 3 and cfg.ac == 0
    dec = oracle.Decoder(cfg, ex)
    for (p, key), f in zip(pkts, frames):
        planes, _ = dec.decode(p)
        for a, b in zip(planes, f):
            np.testing.assert_array_equal(a, b)


def test_slice_crc_residue_is_zero():
    s = Stream("crc", 176, 144, "yuv420p", 2, slices=4, gop_size=2)
    cfg, ex, pkts = oracle_encode(s)
    assert oracle.crc32(ex) == 0  # extradata CRC (ffv1dec.c:619-626)
    data = pkts[1][0]
    end, n = len(data), 0
    while end > 0:  # walk the slice chain backwards (ffv1dec.c:948-989)
        size = int.from_bytes(data[end - 8:end - 5], "big")
        start = end - size - 8
        assert oracle.crc32(data[start:end]) == 0
        end, n = start, n + 1
    assert n == 4


def test_pframes_smaller_than_keyframes_and_state_carry_matters():
    s = Stream("carry", 352, 288, "yuv420p10", 4, slices=4, gop_size=4, depth=10)
    frames = list(s.frames())
    _, _, pk = oracle_encode(s, frames)
    intra = Stream("intra", 352, 288, "yuv420p10", 4, slices=4, gop_size=1, depth=10)
    _, _, pi = oracle_encode(intra, frames)
    assert pk[0][0] == pi[0][0]
    for i in range(1, 4):
        assert not pk[i][1] and pi[i][1]
        assert len(pk[i][0]) < len(pi[i][0])


@pytest.mark.parametrize("stream", RGB_STREAMS, ids=[s.name for s in RGB_STREAMS])
def test_oracle_rgb_roundtrip(stream):
    """RGB through the reversible colour transform (ffv1enc.c:413-473,
    ffv1dec.c:226-280): lossless, the bgr0 padding byte comes back 0."""
    frames = list(stream.frames())
    cfg, ex, pkts = oracle_encode(stream, frames)
    assert cfg.colorspace == 1
    if stream.pix_fmt.startswith("gbrp"):
        assert cfg.ac >= 1 and cfg.version >= 1  # coder forced (ffv1enc.c:810-814)
    dec = oracle.Decoder(cfg, ex)
    for (p, key), f in zip(pkts, frames):
        planes, k = dec.decode(p)
        assert k == key
        for a, b in zip(planes, f):
            if stream.pix_fmt == "bgr0":
                b = b.copy()
                b[:, 3::4] = 0
            np.testing.assert_array_equal(a, b)


def test_oracle_conceals_damaged_slices():
    """A P-frame slice failing its CRC is replaced by the previous picture's
    rectangle and stays so until the next keyframe (slice_damaged is only
    cleared by read_header; ffv1dec.c:820-825, 998-1021)."""
    s = Stream("conceal", 176, 144, "yuv420p", 8, slices=4, gop_size=4)
    frames = list(s.frames())
    cfg, ex, pkts = oracle_encode(s, frames)
    bad = [p for p, _ in pkts]
    bad[1] = corrupt_slice(bad[1], True, 4, 2)
    dec = oracle.Decoder(cfg, ex)
    out = [dec.decode(p)[0] for p in bad]
    x0, y0, x1, y1 = slice_rect(cfg, 2)
    for f in range(8):
        for k in range(3):
            sh = 1 if k else 0
            got, want = out[f][k], frames[f][k]
            r = (slice(y0 >> sh, -(-y1 >> sh)), slice(x0 >> sh, -(-x1 >> sh)))
            if f in (1, 2, 3):  # damaged from frame 1 to the end of the GOP
                np.testing.assert_array_equal(got[r], frames[0][k][r])
                m = np.ones(got.shape, bool)
                m[r] = False
                np.testing.assert_array_equal(got[m], want[m])
            else:
                np.testing.assert_array_equal(got, want)


def two_pass(stream: Stream, frames, coder):
    """Pass 1 then pass 2 through the oracle (ffv1enc.c:898-986)."""
    kw = dict(slices=stream.slices, coder=coder, context=stream.context, gop_size=stream.gop_size)
    cfg = oracle.configure(stream.width, stream.height, stream.pix_fmt, pass_=1, **kw)
    e1 = oracle.Encoder(cfg, 1)
    p1 = [e1.encode(f) for f in frames]
    stats = e1.stats_out()
    cfg2 = oracle.configure(stream.width, stream.height, stream.pix_fmt, pass_=2, **kw)
    e2 = oracle.Encoder(cfg2, 2, stats)
    return cfg2, stats, p1, e2.extradata(), [e2.encode(f) for f in frames]


@pytest.mark.parametrize("coder", [1, -2], ids=["custom_table", "default_table"])
def test_oracle_two_pass(coder):
    """Pass 1 writes the decision counts; pass 2's initial states and
    (custom) re-sorted table code the same clip smaller, the decoder reads
    them back from the extradata and the clip is lossless."""
    s = Stream("2pass", 176, 144, "yuv420p", 6, slices=4, gop_size=3)
    frames = list(s.frames())
    cfg, stats, p1, ex, p2 = two_pass(s, frames, coder)
    assert cfg.version == 3
    head, rest = stats.split("\n", 1)
    assert len(head.split()) == 512 and rest.split()[-1] == "2"  # two keyframes
    assert len(rest.split()) == (666 + 7563) * 64 + 1
    assert sum(len(p) for p, _ in p2) < sum(len(p) for p, _ in p1)
    dec = oracle.Decoder(cfg, ex)
    for (p, _), f in zip(p2, frames):
        for a, b in zip(dec.decode(p)[0], f):
            np.testing.assert_array_equal(a, b)
    # stats_in may hold several runs; the last one counts (ffv1enc.c:914-953)
    e = oracle.Encoder(cfg, 2, "0 " * 512 + "\n" + "0 " * ((666 + 7563) * 64) + "7\n" + stats)
    assert e.extradata() == ex
    with pytest.raises(ValueError):
        oracle.Encoder(cfg, 2, stats.rsplit(" ", 3)[0])


@pytest.mark.parametrize("name", ["p10_gop4", "p10_9slices", "golomb_v3_pframes", "grid16x16", "bgr0_v3"])
def test_slice_threaded_oracle_equals_serial(name):
    # the per-slice-threaded oracle (the reference's threading model, the
    # CPU baseline's slice-threaded figure) writes the same bytes
    streams = {s.name: s for s in PARITY_STREAMS + RGB_STREAMS}
    s = streams[name]
    cfg = s.oracle_config()
    frames = list(s.frames())
    serial, threaded = oracle.Encoder(cfg), oracle.Encoder(cfg)
    for f in frames:
        assert threaded.encode(f, threads=3) == serial.encode(f)
