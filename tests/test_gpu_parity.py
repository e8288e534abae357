"""GPU parity: the HIP encoder (through the C-ABI) against the CPU oracle.

Bit-exact on every byte of every packet and of the extradata.  Streams are
sized so the oracle finishes in seconds; the full-size BASELINE configs are
checked against the reference's own known-answer MD5s (tests/golden) and,
for 8K where no reference bitstream exists, by a lossless round trip
through the oracle decoder.
"""
import hashlib

import numpy as np
import pytest

from helpers import PARITY_STREAMS, Stream, load_golden, md5, oracle_encode
from oracle import oracle

pytestmark = pytest.mark.gpu


def hip_params(s: Stream):
    from ffv1hip import configure
    return configure(s.width, s.height, s.pix_fmt, slices=s.slices, level=s.level, coder=s.coder,
                     context=s.context, gop_size=s.gop_size,
                     bits_per_raw_sample=s.bits_per_raw_sample,
                     allow_large_grid=s.allow_large_grid)


def hip_encode(s: Stream, frames, batch):
    from ffv1hip import HipEncoder
    enc = HipEncoder(hip_params(s), 0, batch)
    ex = enc.extradata()
    pkts = []
    for i in range(0, len(frames), batch):
        pkts += enc.encode(frames[i:i + batch])
    enc.close()
    return ex, pkts


@pytest.mark.parametrize("stream", PARITY_STREAMS, ids=[s.name for s in PARITY_STREAMS])
def test_hip_matches_oracle(stream):
    frames = list(stream.frames())
    cfg, ex_ref, ref = oracle_encode(stream, frames)
    # batch of 3 frames: P-frame state crosses encode calls
    ex, got = hip_encode(stream, frames, batch=3)
    assert ex == ex_ref
    assert len(got) == len(ref)
    for i, ((g, gk), (r, rk)) in enumerate(zip(got, ref)):
        assert gk == rk, f"frame {i} key flag"
        if g != r:
            n = min(len(g), len(r))
            first = next((k for k in range(n) if g[k] != r[k]), n)
            pytest.fail(f"frame {i}: {len(g)} vs {len(r)} bytes, first diff at {first}")


@pytest.mark.parametrize("stream", [s for s in PARITY_STREAMS if s.coder != 0][:6],
                         ids=[s.name for s in PARITY_STREAMS if s.coder != 0][:6])
def test_chained_coder_matches_oracle(stream, monkeypatch):
    """The per-GOP chained range coder (FFV1HIP_CODER=chain) gives the same
    bytes as the frame-parallel default."""
    monkeypatch.setenv("FFV1HIP_CODER", "chain")
    frames = list(stream.frames())
    _, _, ref = oracle_encode(stream, frames)
    _, got = hip_encode(stream, frames, batch=4)
    assert got == ref


def test_whole_batch_equals_split_batches():
    s = PARITY_STREAMS[1]
    frames = list(s.frames())
    _, a = hip_encode(s, frames, batch=len(frames))
    _, b = hip_encode(s, frames, batch=2)
    assert a == b


def _pinned(name):
    return next(p for p in load_golden("known_answers.json")["streams"] if p["name"] == name)


def test_config1_cif_golomb_known_answer():
    pin = _pinned("config1_cif_yuv420p_coder0_g1")
    s = Stream("c1", 352, 288, "yuv420p", pin["frames"], coder=0, gop_size=1)
    ex, pkts = hip_encode(s, list(s.frames()), batch=30)
    assert ex == b""
    for i, size in pin["frame_sizes"].items():
        assert len(pkts[int(i)][0]) == size
    h = hashlib.md5()
    for p, _ in pkts:
        h.update(p)
    assert h.hexdigest() == pin["stream_md5"]


def test_config2_1080p_intra_known_answer():
    pin = _pinned("config2_1080p_yuv420p_coder1_slices24_g1")
    s = Stream("c2", 1920, 1080, "yuv420p", pin["frames"], slices=24, gop_size=1)
    ex, pkts = hip_encode(s, list(s.frames()), batch=25)
    assert md5(ex).startswith(pin["extradata_md5_prefix"])
    h = hashlib.md5()
    for p, _ in pkts:
        h.update(p)
    assert h.hexdigest() == pin["stream_md5"]


def test_config3_4k_p10_pframes_known_answer():
    pin = _pinned("config3_4k_yuv420p10_coder1_slices64_g12")
    s = Stream("c3", 3840, 2160, "yuv420p10", pin["frames"], slices=64, gop_size=12, depth=10)
    ex, pkts = hip_encode(s, list(s.frames()), batch=8)
    assert md5(ex).startswith(pin["extradata_md5_prefix"])
    for i, fp in pin["frame_md5_prefix"].items():
        assert md5(pkts[int(i)][0]).startswith(fp)
    h = hashlib.md5()
    for p, _ in pkts:
        h.update(p)
    assert h.hexdigest() == pin["stream_md5"]


def test_8k_grid16_lossless_roundtrip():
    s = Stream("8k", 7680, 4320, "yuv420p10", 2, slices=256, gop_size=12, source="d2", depth=10,
               allow_large_grid=True, extra={"grid": (16, 16)})
    frames = list(s.frames())
    ex, pkts = hip_encode(s, frames, batch=2)
    cfg = s.oracle_config()
    dec = oracle.Decoder(cfg, ex)
    for (p, key), f in zip(pkts, frames):
        planes, k = dec.decode(p)
        assert k == key
        for a, b in zip(planes, f):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("split", [2, 5])
def test_state_forwarding_between_contexts(split):
    """The multi-GPU exchange step through the C-ABI: a second context resumes
    the P-frame chain mid-GOP from the first's slice states
    (ffv1hip_get_slice_states -> ffv1hip_set_slice_states +
    ffv1hip_set_picture_number) and the packets equal one context's."""
    from ffv1hip import HipEncoder
    s = Stream("fwd", 320, 180, "yuv420p10", 9, slices=6, gop_size=12, source="d2", depth=10)
    frames = list(s.frames())
    _, ref = hip_encode(s, frames, batch=9)
    a = HipEncoder(hip_params(s), 0, 9)
    head = a.encode(frames[:split])
    st = a.get_slice_states()
    a.close()
    b = HipEncoder(hip_params(s), 0, 9)
    b.set_slice_states(st, split)
    tail = b.encode(frames[split:])
    b.close()
    assert head + tail == ref
    assert [k for _, k in head + tail] == [True] + [False] * 8
