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

from helpers import PARITY_STREAMS, RGB_STREAMS, Stream, load_golden, md5, oracle_encode
from oracle import oracle

pytestmark = pytest.mark.gpu


def hip_params(s: Stream):
    from ffv1hip import configure
    return configure(s.width, s.height, s.pix_fmt, slices=s.slices, level=s.level, coder=s.coder,
                     context=s.context, gop_size=s.gop_size,
                     bits_per_raw_sample=s.bits_per_raw_sample,
                     allow_large_grid=s.allow_large_grid, experimental=s.experimental)


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


@pytest.mark.parametrize("stream", RGB_STREAMS, ids=[s.name for s in RGB_STREAMS])
def test_hip_rgb_matches_oracle(stream):
    """bgr0 / gbrp: the colour transform and the row-interleaved planes of
    encode_rgb_frame (ffv1enc.c:413-473), bit-exact with the oracle."""
    frames = list(stream.frames())
    _, ex_ref, ref = oracle_encode(stream, frames)
    ex, got = hip_encode(stream, frames, batch=2)
    assert ex == ex_ref
    assert got == ref


@pytest.mark.parametrize("stream", [s for s in PARITY_STREAMS if s.coder != 0][:6],
                         ids=[s.name for s in PARITY_STREAMS if s.coder != 0][:6])
def test_chained_coder_matches_oracle(stream, monkeypatch):
    """The per-GOP chained range coder (FFV1HIP_DEBUG=coder=chain) gives the
    same bytes as the frame-parallel default."""
    monkeypatch.setenv("FFV1HIP_DEBUG", "coder=chain")
    frames = list(stream.frames())
    _, _, ref = oracle_encode(stream, frames)
    _, got = hip_encode(stream, frames, batch=4)
    assert got == ref


@pytest.mark.parametrize("cpw", [1, 3, 64])
def test_chained_chains_per_wave_match_oracle(cpw, monkeypatch):
    """ffv1_code / ffv1_code_golomb with cpw chains per wave (the code_cpw
    hook; by default launch_code spreads few chains over more waves, 64 is
    the one-chain-per-lane form): the idle lanes, which run on dummy tables
    in the range coder, leave every chain's bytes as the oracle's, with the
    P-frame states carried across encode calls in the chains' tables."""
    monkeypatch.setenv("FFV1HIP_DEBUG", f"coder=chain,code_cpw={cpw}")
    for s in [Stream("cpw_ctx1", 176, 144, "yuv420p10", 8, slices=6, coder=1, context=1, gop_size=4, depth=10),
              Stream("cpw_rgb", 128, 96, "bgr0", 6, slices=4, level=3, gop_size=3, source="random"),
              Stream("cpw_golomb", 176, 144, "yuv420p", 6, slices=6, level=3, coder=0, gop_size=3,
                     source="random")]:
        frames = list(s.frames())
        _, _, ref = oracle_encode(s, frames)
        _, got = hip_encode(s, frames, batch=4)
        assert got == ref, (cpw, s.name)


@pytest.mark.parametrize("debug", ["walk_blocks=0", "serial", "walk_blocks=0,serial"])
def test_schedule_variants_match_oracle(debug, monkeypatch):
    """The walk in 5-wave or one-wave blocks, overlapped or one kernel at a
    time: the same bytes, at a batch (two GOPs of 4:2:0
    10-bit and a 4:4:4 stream, whose chroma chains are the long ones) that
    puts every chain in one round."""
    monkeypatch.setenv("FFV1HIP_DEBUG", debug)
    for s in [Stream("sched420", 352, 288, "yuv420p10", 8, slices=4, coder=1, gop_size=4, depth=10),
              Stream("sched444", 176, 144, "yuv444p16", 6, slices=4, coder=1, gop_size=3,
                     bits_per_raw_sample=12, depth=16, chroma444=True)]:
        frames = list(s.frames())
        _, _, ref = oracle_encode(s, frames)
        _, got = hip_encode(s, frames, batch=len(frames))
        assert got == ref, (debug, s.name)


@pytest.mark.parametrize("debug", ["", "compact=0", "compact=0,walk_blocks=0"])
def test_compact_rows_at_8_bits_match_oracle(debug, monkeypatch):
    """8-bit context model 0 in the frame-parallel path: the walk's LDS rows
    hold the 24 slots a symbol can use at 8 bits (e <= 7), an unused slot's
    byte in the dummy row (the default), or all 32 (compact=0, a test hook):
    the oracle's bytes either way, on video, noise (every exponent and sign
    slot) and 4:4:4 / gray."""
    monkeypatch.setenv("FFV1HIP_DEBUG", debug)
    for s in [Stream("c8_420", 352, 288, "yuv420p", 8, slices=4, coder=1, gop_size=4),
              Stream("c8_noise", 176, 144, "yuv420p", 6, slices=4, coder=1, gop_size=3, source="random"),
              Stream("c8_444", 176, 144, "yuv444p", 5, slices=6, coder=-2, gop_size=5, chroma444=True),
              Stream("c8_gray", 128, 96, "gray", 4, slices=4, coder=1, gop_size=2, source="random")]:
        frames = list(s.frames())
        _, _, ref = oracle_encode(s, frames)
        _, got = hip_encode(s, frames, batch=len(frames))
        assert got == ref, (debug, s.name)


@pytest.mark.parametrize("debug", ["dsets=lazy", "dsets=lazy,rec2_drop=1", "dsets=lazy,rec2_drop=0",
                                   "dsets=eager,rec2_drop=0", "dsets=lazy,budget=4", "dsets=lazy,budget=8,rec2_drop=1"])
def test_lazy_decision_sets_match_oracle(debug, monkeypatch):
    """Decision sets sized from the first batches (dsets=lazy, the default
    for large batches), the second records set taken afterwards, and given
    back when a set has to grow (rec2_drop=k: as if set k did not fit beside
    it; the batch's own records set is kept); budget=q: the slice byte budget
    lowered to 1/q in the first batch (what happens when the second records
    set does not fit), the random batches then re-encoded with a larger one.
    A flat first batch makes the later random ones grow both sets."""
    monkeypatch.setenv("FFV1HIP_DEBUG", debug)
    s = Stream("lazy420", 176, 144, "yuv420p10", 9, slices=4, coder=1, gop_size=3, source="random", depth=10)
    frames = list(s.frames())
    frames[:3] = [[np.full_like(p, 200) for p in f] for f in frames[:3]]
    _, _, ref = oracle_encode(s, frames)
    _, got = hip_encode(s, frames, batch=3)
    assert got == ref


@pytest.mark.parametrize("pack", ["pack=1", "pack=0"])
def test_packed_10bit_host_frames(pack, monkeypatch):
    """10-bit host frames cross PCIe packed three samples to a word and are
    unpacked in HBM (ffv1_unpack10); a frame with a sample over 10 bits (the
    encoder codes the 16-bit value as it is) goes as it is, beside packed
    ones in the same batch; odd widths leave one or two samples in a row's
    last word.  The oracle's packets either way (pack=0: no packing)."""
    monkeypatch.setenv("FFV1HIP_DEBUG", pack)
    for s in [Stream("pk420", 190, 64, "yuv420p10", 7, slices=4, coder=1, gop_size=3, source="random", depth=10),
              Stream("pk422", 95, 61, "yuv422p10", 5, slices=4, coder=1, gop_size=5, source="random", depth=10)]:
        frames = [[p.copy() for p in f] for f in s.frames()]
        frames[1][0][3, 5] = 1500    # luma over 10 bits
        frames[4][2][0, 0] = 1024    # Cr, just over
        _, _, ref = oracle_encode(s, frames)
        _, got = hip_encode(s, frames, batch=3)
        assert got == ref, s.name


@pytest.mark.parametrize("recsets", [2, 1])
@pytest.mark.parametrize("stream", [s for s in PARITY_STREAMS if s.coder != 0 and s.gop_size != 1][:4],
                         ids=[s.name for s in PARITY_STREAMS if s.coder != 0 and s.gop_size != 1][:4])
def test_split_walk_matches_oracle(stream, recsets, monkeypatch):
    """The split schedule with a walk in two launches (first part 3 waves,
    forced by the test hooks) and the next batch's symbols beside its second
    part (two records sets), and one records set (symbols, walk, bits beside
    it): the same bytes as the oracle across batches."""
    monkeypatch.setenv("FFV1HIP_DEBUG", f"recsets={recsets},walk_part_a=3")
    frames = list(stream.frames())
    _, ex_ref, ref = oracle_encode(stream, frames)
    ex, got = hip_encode(stream, frames, batch=4)
    assert ex == ex_ref
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


def test_dense_rows_keep_packets_and_carried_states(monkeypatch):
    """Above 8 bits the walk numbers the 365 reachable contexts densely
    (ffv1_internal.h, dense_ctx / dense_row).  The packets, and the P-frame
    carry exported mid-GOP (ffv1hip_get_slice_states, context numbering, the
    contexts that cannot occur at their initial 128), equal those of the
    context-numbered walk (FFV1HIP_DEBUG=dense=0) and of the chained coder."""
    from ffv1hip import HipEncoder
    s = Stream("dense", 320, 180, "yuv420p10", 7, slices=6, gop_size=12, source="d2", depth=10)
    frames = list(s.frames())
    _, _, ref = oracle_encode(s, frames)
    states = {}
    for mode, dbg in [("dense", ""), ("contexts", "dense=0"), ("chain", "coder=chain")]:
        monkeypatch.setenv("FFV1HIP_DEBUG", dbg)
        enc = HipEncoder(hip_params(s), 0, 7)
        got = enc.encode(frames[:5])
        states[mode] = bytes(enc.get_slice_states())
        got += enc.encode(frames[5:])
        enc.close()
        assert got == ref, mode
    assert states["dense"] == states["contexts"] == states["chain"]


def test_batch_ending_in_one_frame_segment():
    """A batch that starts mid-GOP (its first segment loads the carried
    states) and ends with a one-frame segment (which saves them): load and
    save of one slice in one launch go to different buffers."""
    from ffv1hip import HipEncoder
    s = Stream("seg1", 320, 180, "yuv420p10", 11, slices=6, gop_size=4, source="d2", depth=10)
    frames = list(s.frames())
    _, _, ref = oracle_encode(s, frames)
    enc = HipEncoder(hip_params(s), 0, 5)
    got = []
    for a, b in [(0, 2), (2, 5), (5, 9), (9, 11)]:  # [2,3]+[4], [5,6,7]+[8], [9,10]
        got += enc.encode(frames[a:b])
    enc.close()
    assert got == ref


@pytest.mark.parametrize("coder", ["frames", "chain"])
def test_slice_budget_overflow_reencodes(coder, monkeypatch):
    """A slice over the byte budget is encoded again with a larger budget
    (the reference codes it: its buffer is ~w*h*140 bytes, ffv1enc.c:1232),
    with the P-frame carry rolled back: the stream equals the oracle's."""
    monkeypatch.setenv("FFV1HIP_DEBUG", "slice_cap=512" + (",coder=chain" if coder == "chain" else ""))
    s = PARITY_STREAMS[1]
    frames = list(s.frames())
    _, _, ref = oracle_encode(s, frames)
    _, got = hip_encode(s, frames, batch=3)
    assert got == ref


@pytest.mark.parametrize("pix_fmt,bpr,nframes", [("yuv444p16", 12, 2), ("yuv444p16", 0, 1)])
def test_full_entropy_noise_c4_shape(pix_fmt, bpr, nframes):
    """Full-entropy noise at the config-4 shape (4K 4:4:4, 64 slices): the
    most bytes per sample the path produces; equal to the oracle."""
    import numpy as np
    s = Stream("noise", 3840, 2160, pix_fmt, nframes, slices=64, gop_size=12, bits_per_raw_sample=bpr)
    rng = np.random.default_rng(7)
    shift = 16 - bpr if bpr else 0
    frames = [[np.ascontiguousarray((rng.integers(0, 1 << (16 - shift), size=(2160, 3840)) << shift)
                                    .astype(np.uint16)) for _ in range(3)] for _ in range(nframes)]
    _, _, ref = oracle_encode(s, frames)
    _, got = hip_encode(s, frames, batch=nframes)
    assert [len(p) for p, _ in got] == [len(p) for p, _ in ref]
    assert got == ref


@pytest.mark.parametrize("batch", [12, 5])
def test_avcodec_mirror_c3_known_answer(batch):
    """FFV1Encoder's init / encode2 / encode2(NULL) / close (the AVCodec
    callbacks of ff_ffv1_encoder, ffv1enc.c:1415-1444, driven the way
    avcodec_encode_video2 drives them, utils.c:1922-1990) with
    AV_CODEC_CAP_DELAY batching: the reference's config-3 stream, each
    packet's pts/dts the frame's, KEY on every 12th."""
    from ffv1hip import AVCodecContext, FFV1Encoder
    pin = _pinned("config3_4k_yuv420p10_coder1_slices64_g12")
    s = Stream("c3", 3840, 2160, "yuv420p10", pin["frames"], slices=64, gop_size=12, depth=10)
    avctx = AVCodecContext(3840, 2160, "yuv420p10", gop_size=12, slices=64, coder=1)
    enc = FFV1Encoder(batch=batch)
    assert enc.init(avctx) == 0
    assert md5(avctx.extradata).startswith(pin["extradata_md5_prefix"])
    pkts, got = [], []
    for i, f in enumerate(s.frames()):
        pk = enc.encode2(f, pts=1000 + i)  # at most one packet per call
        got.append(pk is not None)
        if pk is not None:
            pkts.append(pk)
    while True:  # flush: NULL frames until no packet comes back
        pk = enc.encode2(None)
        if pk is None:
            break
        pkts.append(pk)
    assert enc.close() == 0
    assert len(pkts) == pin["frames"]
    n = pin["frames"]
    # the delay: two batches (one codes while the next queues)
    assert avctx.delay == 2 * batch - 1
    assert got == [i >= avctx.delay for i in range(n)]
    assert [p.pts for p in pkts] == [1000 + i for i in range(len(pkts))]
    assert [p.dts for p in pkts] == [p.pts for p in pkts]
    assert [p.key for p in pkts] == [i % 12 == 0 for i in range(len(pkts))]
    h = hashlib.md5()
    for p in pkts:
        h.update(p.data)
    assert h.hexdigest() == pin["stream_md5"]


@pytest.mark.parametrize("batch", [3, 4])
def test_encode2_pipelined_budget_reencode(batch, monkeypatch):
    """encode2 one frame per call with a 512-byte starting slice budget: every
    batch goes over it while the next one is already coding, so the re-encode
    rolls back two batches in flight; packets, pts and keys equal the
    oracle's stream."""
    from ffv1hip import AVCodecContext, FFV1Encoder
    monkeypatch.setenv("FFV1HIP_DEBUG", "slice_cap=512")
    s = PARITY_STREAMS[1]
    frames = list(s.frames())
    _, ex_ref, ref = oracle_encode(s, frames)
    avctx = AVCodecContext(s.width, s.height, s.pix_fmt, gop_size=s.gop_size, slices=s.slices, coder=s.coder)
    enc = FFV1Encoder(batch=batch)
    assert enc.init(avctx) == 0
    assert avctx.extradata == ex_ref
    pkts = [enc.encode2(f, pts=i) for i, f in enumerate(frames)]
    pkts = [p for p in pkts if p is not None]
    while (p := enc.encode2(None)) is not None:
        pkts.append(p)
    enc.close()
    assert [p.pts for p in pkts] == list(range(len(frames)))
    assert [(p.data, p.key) for p in pkts] == ref


@pytest.mark.parametrize("fsets", [None, "2"])
@pytest.mark.parametrize("cap", [None, "512"])
def test_host_encode_many_batches(cap, fsets, monkeypatch):
    """ffv1hip_encode over several batches in one call (frames staged while
    the previous batch codes), with and without the budget re-encode, with
    three frame sets (the default: batch k+2 stages while batch k finishes)
    and with two (fsets=2)."""
    hooks = ([f"slice_cap={cap}"] if cap else []) + ([f"fsets={fsets}"] if fsets else [])
    if hooks:
        monkeypatch.setenv("FFV1HIP_DEBUG", ",".join(hooks))
    from ffv1hip import HipEncoder
    s = PARITY_STREAMS[1]
    frames = list(s.frames())
    _, _, ref = oracle_encode(s, frames)
    enc = HipEncoder(hip_params(s), 0, 3)
    got = enc.encode(frames)
    enc.close()
    assert got == ref


def _pool_views(pool, shapes_dtypes, nframes):
    """Frames as views into one flat uint8 buffer (a caller's frame pool)."""
    out, off = [], 0
    for _ in range(nframes):
        f = []
        for shp, dt in shapes_dtypes:
            nb = int(np.prod(shp)) * np.dtype(dt).itemsize
            f.append(pool[off:off + nb].view(dt).reshape(shp))
            off += nb
        out.append(f)
    return out


@pytest.mark.parametrize("cap", [None, "512"])
def test_registered_host_frames(cap, monkeypatch):
    """Frames in caller-pinned memory (ffv1hip_host_register) go to HBM by DMA
    straight from it: ffv1hip_encode over several batches from a registered
    pool, and ffv1hip_encode2 from ONE registered buffer the caller rewrites
    after every call (the frame's copy is done when the call returns), with
    and without the budget re-encode, which reads the batch's frames again:
    the oracle's packets."""
    if cap:
        monkeypatch.setenv("FFV1HIP_DEBUG", f"slice_cap={cap}")
    from ffv1hip import AVCodecContext, FFV1Encoder, HipEncoder
    s = PARITY_STREAMS[1]
    frames = list(s.frames())
    _, _, ref = oracle_encode(s, frames)
    sd = [(p.shape, p.dtype) for p in frames[0]]
    fbytes = sum(p.nbytes for p in frames[0])
    pool = np.empty(fbytes * len(frames), np.uint8)
    views = _pool_views(pool, sd, len(frames))
    for v, f in zip(views, frames):
        for a, b in zip(v, f):
            a[...] = b
    enc = HipEncoder(hip_params(s), 0, 3)
    enc.register_host(pool)
    assert enc.encode(views) == ref
    enc.unregister_host(pool)
    with pytest.raises(Exception, match="no range registered"):
        enc.unregister_host(pool)
    enc.close()

    avctx = AVCodecContext(s.width, s.height, s.pix_fmt, gop_size=s.gop_size, slices=s.slices, coder=s.coder)
    e2 = FFV1Encoder(batch=3)
    assert e2.init(avctx) == 0
    buf = np.empty(fbytes, np.uint8)
    e2._enc.register_host(buf)
    (one,) = _pool_views(buf, sd, 1)
    pkts = []
    for i, f in enumerate(frames):
        for a, b in zip(one, f):
            a[...] = b
        pk = e2.encode2(one, pts=i)
        for a in one:  # the caller reuses the buffer at once
            a[...] = 0
        if pk is not None:
            pkts.append(pk)
    while (pk := e2.encode2(None)) is not None:
        pkts.append(pk)
    assert e2.close() == 0
    assert [(p.data, p.key) for p in pkts] == ref


def _d2h(ptr, nbytes):
    """Device bytes at `ptr` through the HIP runtime the library links."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    out = np.empty(max(nbytes, 1), np.uint8)
    assert hip.hipMemcpy(out.ctypes.data, ctypes.c_void_p(ptr), nbytes, 2) == 0  # DeviceToHost
    return out[:nbytes]


def _device_batch(params, frames):
    """Frames packed planar into one HBM buffer the way bench.py stages them."""
    import torch
    shapes = params.plane_shapes()
    plane_bytes = [h * w * params.sample_bytes for h, w in shapes]
    frame_bytes = (sum(plane_bytes) + 255) // 256 * 256
    host = np.zeros((len(frames), frame_bytes), np.uint8)
    for i, f in enumerate(frames):
        flat = np.concatenate([p.reshape(-1).view(np.uint8) for p in f])
        host[i, :flat.size] = flat
    offs = [0, plane_bytes[0], plane_bytes[0] + plane_bytes[1]]
    strides = [shapes[k][1] * params.sample_bytes for k in range(3)]
    return torch.from_numpy(host).to("cuda:0"), frame_bytes, offs, strides


@pytest.mark.parametrize("sync", ["synchronize", "device_packets"])
def test_device_path_never_truncates(sync, monkeypatch):
    """encode_device twice back to back with a 512-byte starting slice budget
    (every slice over it), then the packets of the last call through
    ffv1hip_synchronize / ffv1hip_device_packets: the oracle's bytes (the
    budget re-encode runs there), never capped slices (VERDICT r2, weak 4;
    the reference fails a frame it cannot fit, ffv1enc.c:283-292)."""
    import torch
    from ffv1hip import HipEncoder
    monkeypatch.setenv("FFV1HIP_DEBUG", "slice_cap=512")
    s = PARITY_STREAMS[1]  # 480x270 10-bit, 4 slices, gop 4
    frames = list(s.frames())[:8]
    _, _, ref = oracle_encode(s, frames)
    params = hip_params(s)
    enc = HipEncoder(params, 0, 4)
    a = _device_batch(params, frames[:4])
    b = _device_batch(params, frames[4:])
    enc.encode_device(a[0].data_ptr(), a[1], a[2], a[3], 4)
    enc.encode_device(b[0].data_ptr(), b[1], b[2], b[3], 4)
    if sync == "synchronize":
        enc.synchronize()
    d_p, stride, d_s = enc.device_packets()
    sizes = _d2h(d_s, 8 * 4).view(np.int64)
    got = [_d2h(d_p + i * stride, int(sizes[i])).tobytes() for i in range(4)]
    torch.cuda.synchronize()
    enc.close()
    assert got == [p for p, _ in ref[4:]]


@pytest.mark.parametrize("path", ["encode", "encode_fsets2", "encode_batches", "device_fetch", "encode2"])
def test_guarded_launch_recovery_matches_oracle(path, monkeypatch):
    """The recovery path of a guarded launch: a batch launched
    before its decision count is read back, whose decisions then do not fit
    its decision set, is skipped by every kernel (ds_over), flagged by
    ffv1_range (status[3]) and encoded again at settle with the total read
    back.  The guard_skip hook forces it on every batch (including the next
    batch's re-run that a rolled-back batch drags along); the packets of every
    host path equal the oracle's and the re-runs are counted."""
    from ffv1hip import AVCodecContext, FFV1Encoder, HipEncoder
    monkeypatch.setenv("FFV1HIP_DEBUG", "guard_skip" + (",fsets=2" if path == "encode_fsets2" else ""))
    s = PARITY_STREAMS[1]  # 480x270 10-bit, 4 slices, gop 4
    frames = list(s.frames())
    _, ex_ref, ref = oracle_encode(s, frames)
    params = hip_params(s)
    if path == "encode2":
        avctx = AVCodecContext(s.width, s.height, s.pix_fmt, gop_size=s.gop_size, slices=s.slices, coder=s.coder)
        enc2 = FFV1Encoder(batch=3)
        assert enc2.init(avctx) == 0
        pkts = [enc2.encode2(f, pts=i) for i, f in enumerate(frames)]
        pkts = [p for p in pkts if p is not None]
        while (p := enc2.encode2(None)) is not None:
            pkts.append(p)
        skips, reruns = enc2._enc.debug_counter("guard_skips"), enc2._enc.debug_counter("guard_reruns")
        enc2.close()
        got = [(p.data, p.key) for p in pkts]
    else:
        enc = HipEncoder(params, 0, 3)
        if path in ("encode", "encode_fsets2"):
            got = enc.encode(frames)
        elif path == "encode_batches":
            got = []
            for i in range(0, len(frames), 3):
                got += enc.encode(frames[i:i + 3])
        else:
            import torch
            got = []
            for i in range(0, len(frames), 3):
                part = frames[i:i + 3]
                d = _device_batch(params, part)
                enc.encode_device(d[0].data_ptr(), d[1], d[2], d[3], len(part))
                got += enc.fetch(len(part))
                torch.cuda.synchronize()
        skips, reruns = enc.debug_counter("guard_skips"), enc.debug_counter("guard_reruns")
        enc.close()
    assert got == ref
    # every batch's first launch was skipped; each skipped run is either run
    # again at its settle (counted) or replaced by the re-run that a rolled-back
    # earlier batch drags along (which may be skipped in turn)
    assert skips >= (len(frames) + 2) // 3, (skips, reruns)
    assert 1 <= reruns <= skips, (skips, reruns)


FULL_SIZE = {
    # BASELINE configs[3]: 4K yuv444p16 at 12 bit (u16 >> 4), videogen content
    "c4_4k_444p12": Stream("c4", 3840, 2160, "yuv444p16", 3, slices=64, gop_size=12,
                           bits_per_raw_sample=12, depth=16, chroma444=True),
    # BASELINE configs[4]: 8K yuv420p10, the 16x16 grid (no reference bitstream)
    "c5_8k_p10_grid16": Stream("c5", 7680, 4320, "yuv420p10", 3, slices=256, gop_size=12, depth=10,
                               allow_large_grid=True, extra={"grid": (16, 16)}),
}


@pytest.mark.parametrize("name", sorted(FULL_SIZE))
def test_full_size_configs_match_oracle(name):
    """The bench's c4 and c5 workloads at full size on the D1 clip (a
    keyframe and two P-frames), every byte against the oracle encoder
    (8K parity is the CPU restatement, bit-exact)."""
    s = FULL_SIZE[name]
    frames = list(s.frames())
    _, ex_ref, ref = oracle_encode(s, frames)
    ex, got = hip_encode(s, frames, batch=3)
    assert ex == ex_ref
    assert [len(p) for p, _ in got] == [len(p) for p, _ in ref]
    assert got == ref


def test_batch_too_large_for_hbm_is_enomem():
    """A batch that cannot fit in HBM is refused with -ENOMEM and the
    largest batch that fits (not a HIP out-of-memory -EIO half way through
    the allocations), and that batch can then be created."""
    import re
    from ffv1hip import FFV1Error, HipEncoder, configure
    params = configure(3840, 2160, "yuv444p16", slices=64, coder=1, gop_size=12, bits_per_raw_sample=12)
    with pytest.raises(FFV1Error) as e:
        HipEncoder(params, 0, 5000)
    assert e.value.code == -12
    fit = int(re.search(r"at most (\d+) frames", str(e.value)).group(1))
    assert 12 <= fit < 5000
    enc = HipEncoder(params, 0, min(fit, 48))
    enc.close()
