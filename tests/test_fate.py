"""The reference's own FATE pins for FFV1 (tests/ref/vsynth/vsynth{1,2,3}-ffv1*).

CPU: the oracle encoder's AVI equals each pinned file (MD5 and size), and the
generated clips equal the reference's vsynth inputs (the decoded-output MD5
of a lossless test is the input's MD5).  GPU: the HIP encoder, through the
C-ABI, gives the same AVI files, and the GPU decoder returns the clip.

Covered by these pins: Golomb-Rice v0 (single slice, in-band header) and v3
(4 slices) P-frame streams at 8 bit, the range coder with the custom state
table at 8-bit 4:2:0, 10-bit 4:2:2 and 16-bit 4:4:4, and v3 bgr0 (the
reversible colour transform, Golomb-Rice), all with gop 12 P-frames, at
352x288 and the odd 34x34 geometry.
"""
import pytest

from fate import (PINS, avi_bytes, back_to_yuv420p, encoder_options, input_frames,
                  raw_clip, raw_md5)
from helpers import md5
from oracle import oracle

_raw_cache = {}


def _raw(pin):
    key = (pin["source"], pin["width"], pin["height"])
    if key not in _raw_cache:
        _raw_cache[key] = raw_clip(pin)
    return _raw_cache[key]


def _ids(pins):
    return [p["test"] for p in pins]


@pytest.mark.parametrize("source", ["vsynth1", "vsynth2", "vsynth3"])
def test_clip_generators_match_reference_inputs(source):
    """videogen / rotozoom restatements produce the reference's vsynth*.yuv:
    the lossless tests' decoded-output MD5 is the input clip's MD5."""
    pin = next(p for p in PINS if p["test"] == f"{source}-ffv1")
    assert "MAXDIFF:    0" in pin["psnr_line"]
    assert raw_md5(_raw(pin)) == pin["decoded_md5"]


def _check_decoded(pin, frames, decoded):
    """YUV pins: the clip decoded back to yuv420p has the pinned MD5.  bgr0
    pins (whose pinned MD5 is after an RGB -> yuv420p conversion): the
    decoded pictures equal the encoder's input, padding byte aside."""
    if pin["pix_fmt"] == "bgr0":
        for planes, f in zip(decoded, frames):
            a, b = planes[0].reshape(-1, 4), f[0].reshape(-1, 4)
            assert (a[:, :3] == b[:, :3]).all() and not a[:, 3].any()
        return
    out = [back_to_yuv420p(planes, pin) for planes in decoded]
    assert raw_md5(out) == pin["decoded_md5"]


@pytest.mark.parametrize("pin", PINS, ids=_ids(PINS))
def test_oracle_avi_matches_fate(pin):
    frames = input_frames(pin, _raw(pin))
    o = encoder_options(pin)
    cfg = oracle.configure(pin["width"], pin["height"], pin["pix_fmt"], **o)
    enc = oracle.Encoder(cfg)
    ex = enc.extradata()
    pkts = [enc.encode(f) for f in frames]
    avi = avi_bytes(pin, ex, pkts)
    assert len(avi) == pin["avi_size"]
    assert md5(avi) == pin["avi_md5"]
    # and the oracle decoder gives the clip back
    dec = oracle.Decoder(cfg, ex)
    _check_decoded(pin, frames, [dec.decode(p)[0] for p, _ in pkts])


@pytest.mark.gpu
@pytest.mark.parametrize("pin", PINS, ids=_ids(PINS))
@pytest.mark.parametrize("batch", [50, 7])
def test_hip_avi_matches_fate(pin, batch):
    from ffv1hip import HipDecoder, HipEncoder, configure
    frames = input_frames(pin, _raw(pin))
    params = configure(pin["width"], pin["height"], pin["pix_fmt"], **encoder_options(pin))
    enc = HipEncoder(params, 0, batch)
    ex = enc.extradata()
    pkts = []
    for i in range(0, len(frames), batch):
        pkts += enc.encode(frames[i:i + batch])
    enc.close()
    avi = avi_bytes(pin, ex, pkts)
    assert len(avi) == pin["avi_size"]
    assert md5(avi) == pin["avi_md5"]
    if batch != 50:
        return  # the decoded output is checked once per pin
    # every pin through the GPU decoder: Golomb-Rice and range, v0 and v3,
    # YCbCr and bgr0 (include/ffv1hip.h, ffv1hip_dec_create)
    dec = HipDecoder(params, ex, 0)
    out = [planes for planes, _ in dec.decode([p for p, _ in pkts])]
    dec.close()
    _check_decoded(pin, frames, out)
