"""The AVI container (ffv1hip.avi) and the command line (python -m ffv1hip).

CPU: the muxer's file for a FATE pin reads back to the same extradata,
packets and key flags.  GPU: ``python -m ffv1hip encode`` over the FATE raw
clip writes the reference's pinned AVI file (the ffmpeg command of
tests/fate-run.sh:171-193, drop-in), and ``decode`` gives the clip back.
"""
import numpy as np
import pytest

from fate import PINS, avi_bytes, encoder_options, input_frames, raw_clip
from helpers import md5
from oracle import oracle
from ffv1hip.avi import read_avi


def _pin(name):
    return next(p for p in PINS if p["test"] == name)


def test_avi_reads_back_what_it_writes():
    pin = _pin("vsynth3-ffv1-v3-yuv420p")
    frames = input_frames(pin, raw_clip(pin))
    enc = oracle.Encoder(oracle.configure(pin["width"], pin["height"], pin["pix_fmt"],
                                          **encoder_options(pin)))
    ex = enc.extradata()
    pkts = [enc.encode(f) for f in frames]
    data = avi_bytes(pin, ex, pkts)
    assert md5(data) == pin["avi_md5"]
    w, h, fourcc, ex2, pk2 = read_avi(data)
    assert (w, h, fourcc, ex2) == (pin["width"], pin["height"], b"FFV1", ex)
    assert pk2 == pkts
    assert sum(k for _, k in pk2) == 5  # gop 12 over 50 frames


def test_cli_info(tmp_path, capsys):
    from ffv1hip.__main__ import main
    pin = _pin("vsynth3-ffv1")
    frames = input_frames(pin, raw_clip(pin))
    enc = oracle.Encoder(oracle.configure(pin["width"], pin["height"], pin["pix_fmt"],
                                          **encoder_options(pin)))
    path = tmp_path / "a.avi"
    path.write_bytes(avi_bytes(pin, enc.extradata(), [enc.encode(f) for f in frames]))
    assert main(["info", str(path)]) == 0
    assert "FFV1 34x34, 50 packets (5 key)" in capsys.readouterr().out


def _write_raw(path, frames):
    with open(path, "wb") as f:
        for fr in frames:
            for p in fr:
                f.write(np.ascontiguousarray(p).astype(p.dtype.newbyteorder("<")).tobytes())


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["vsynth1-ffv1", "vsynth1-ffv1-v3-yuv422p10",
                                  "vsynth2-ffv1-v3-bgr0"])
def test_cli_encode_writes_the_fate_file(tmp_path, name):
    from ffv1hip.__main__ import main
    pin = _pin(name)
    frames = input_frames(pin, raw_clip(pin))
    raw = tmp_path / "in.raw"
    _write_raw(raw, frames)
    out = tmp_path / "out.avi"
    opts = pin["options"]
    argv = ["encode", "-s", f"{pin['width']}x{pin['height']}", "-pix_fmt", pin["pix_fmt"],
            "-g", str(pin["gop_size"]), "-batch", "7"]
    for k in ("slices", "level"):
        if k in opts:
            argv += [f"-{k}", str(opts[k])]
    assert main(argv + [str(raw), str(out)]) == 0
    data = out.read_bytes()
    assert len(data) == pin["avi_size"] and md5(data) == pin["avi_md5"]
    if pin["pix_fmt"] != "bgr0" and "level" in opts:  # the GPU decoder reads v3 YCbCr
        back = tmp_path / "back.raw"
        assert main(["decode", "-pix_fmt", pin["pix_fmt"], "-slices", str(opts.get("slices", 0)),
                     "-level", str(opts["level"]), str(out), str(back)]) == 0
        assert back.read_bytes() == raw.read_bytes()


def test_cli_strict_names():
    from ffv1hip.__main__ import _strict
    assert _strict("experimental") == -2 and _strict("normal") == 0 and _strict("-2") == -2


@pytest.mark.gpu
def test_cli_level2_strict_experimental_roundtrip(tmp_path):
    """`-level 2 -strict experimental` (ffv1enc.c:703-706) through the CLI:
    the AVI's packets equal the oracle's version-2 packets, and the GPU
    decoder gives the raw frames back; without -strict the level is refused."""
    from ffv1hip.__main__ import main
    from ffv1hip.avi import read_avi
    from ffv1hip.encoder import FFV1Error
    from helpers import Stream
    s = Stream("cli_v2", 96, 64, "yuv420p", 5, level=2, slices=4, coder=1, gop_size=3, source="random",
               experimental=True, seed=31)
    frames = list(s.frames())
    raw = tmp_path / "in.raw"
    _write_raw(raw, frames)
    out = tmp_path / "out.avi"
    argv = ["encode", "-s", "96x64", "-pix_fmt", "yuv420p", "-g", "3", "-slices", "4", "-level", "2",
            "-coder", "1", "-batch", "2"]
    with pytest.raises(FFV1Error):
        main(argv + [str(raw), str(out)])
    assert main(argv + ["-strict", "experimental", str(raw), str(out)]) == 0
    _, _, _, ex, pk = read_avi(out.read_bytes())
    cfg = oracle.configure(96, 64, "yuv420p", slices=4, level=2, coder=1, gop_size=3, experimental=True)
    enc = oracle.Encoder(cfg)
    assert ex == enc.extradata()
    assert [p for p, _ in pk] == [enc.encode(f)[0] for f in frames]
    back = tmp_path / "back.raw"
    assert main(["decode", "-pix_fmt", "yuv420p", "-slices", "4", "-level", "2", "-coder", "1", "-g", "3",
                 "-strict", "experimental", str(out), str(back)]) == 0
    assert back.read_bytes() == raw.read_bytes()
