"""CPU checks of the product's C-ABI (no GPU compute is called here).

* lib/libffv1hip.so loads and exports every function include/ffv1hip.h declares;
* ffv1hip_configure (encode_init's parameter contract, host-only) agrees with
  the oracle's restatement over a grid of options;
* without a GPU, creating an encoder fails loudly (no CPU fallback).
"""
import ctypes
import os
import re

import pytest

from helpers import PARITY_STREAMS
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ffv1hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ffv1hip_\w+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from ffv1hip import load_library, EXPORTED_SYMBOLS
    lib = load_library()
    names = declared_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/ffv1hip.h but not exported"
    assert set(names) == set(EXPORTED_SYMBOLS)
    assert lib.ffv1hip_abi_version() == 6


FIELDS = ["width", "height", "chroma_planes", "chroma_h_shift", "chroma_v_shift",
          "bits_per_raw_sample", "packed_at_lsb", "sample_bytes", "version", "ac", "ec",
          "context_model", "num_h_slices", "num_v_slices", "gop_size", "colorspace", "transparency"]

OPTION_GRID = [
    (352, 288, "yuv420p", 0, -1, -1, 0, 12, 0),
    (352, 288, "yuv420p", 4, -1, -1, 0, 12, 0),
    (352, 288, "yuv420p", 0, 3, 1, 0, 12, 0),
    (352, 288, "yuv422p10", 0, 3, -1, 0, 12, 0),
    (352, 288, "yuv444p16", 0, 3, -1, 0, 12, 0),
    (1920, 1080, "yuv420p", 24, -1, 1, 0, 1, 0),
    (1920, 1080, "yuv420p", 0, -1, 1, 1, 12, 0),
    (3840, 2160, "yuv420p10", 64, -1, 1, 0, 12, 0),
    (3840, 2160, "yuv444p16", 64, -1, 1, 0, 12, 12),
    (176, 144, "yuv420p10", 0, -1, 1, 0, 3, 0),
    (176, 144, "gray", 0, -1, 0, 0, 12, 0),
    (176, 144, "yuv410p", 9, -1, -2, 0, 12, 0),
    (720, 576, "yuv420p9", 0, -1, 0, 0, 12, 0),
    (352, 288, "bgr0", 0, 3, -1, 0, 12, 0),
    (352, 288, "bgr0", 0, -1, 1, 1, 12, 0),
    (176, 144, "0rgb32", 0, 1, 0, 0, 12, 0),
    (352, 288, "gbrp9", 4, -1, 0, 0, 12, 0),
    (352, 288, "yuva420p", 4, -1, 1, 0, 12, 0),
    (352, 288, "yuva420p", 0, -1, 0, 0, 12, 0),
    (352, 288, "yuva444p10", 0, 3, 1, 1, 12, 0),
    (720, 576, "yuva422p16", 0, -1, -1, 0, 12, 0),
    (176, 144, "ya8", 0, 1, 1, 0, 12, 0),
    (352, 288, "bgra", 0, 3, 0, 0, 12, 0),
    (352, 288, "rgb32", 4, -1, 1, 0, 12, 0),
    (1920, 1080, "gbrp10", 0, -1, -1, 0, 12, 0),
    (352, 288, "gbrp12", 0, 3, 1, 0, 12, 0),
    (352, 288, "gbrp14", 0, 3, 1, 0, 12, 13),
]


@pytest.mark.parametrize("opt", OPTION_GRID)
def test_configure_matches_oracle_contract(opt):
    from ffv1hip import configure
    w, h, fmt, slices, level, coder, context, gop, bpr = opt
    ref = oracle.configure(w, h, fmt, slices=slices, level=level, coder=coder, context=context,
                           gop_size=gop, bits_per_raw_sample=bpr).as_dict()
    got = configure(w, h, fmt, slices=slices, level=level, coder=coder, context=context,
                    gop_size=gop, bits_per_raw_sample=bpr).as_dict()
    for f in FIELDS:
        assert got[f] == ref[f], f


def test_configure_rejections_match():
    from ffv1hip import configure, FFV1Error
    for args in [(1920, 1080, "yuv420p", 5), (7680, 4320, "yuv420p10", 256),
                 (352, 288, "rgb48", 0)]:
        with pytest.raises(FFV1Error):
            configure(*args)
        with pytest.raises((ValueError, Exception)):
            oracle.configure(*args)
    p = configure(7680, 4320, "yuv420p10", slices=256, coder=1, allow_large_grid=True)
    assert (p.num_h_slices, p.num_v_slices, p.version) == (16, 16, 3)


def test_no_silent_cpu_fallback_without_gpu():
    import torch
    from ffv1hip import configure, HipEncoder, FFV1Error
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(FFV1Error):
        HipEncoder(configure(352, 288, "yuv420p", coder=1, slices=4), 0, 2)


def test_unsupported_parameters_are_refused():
    from ffv1hip import configure, HipEncoder, FFV1Error
    p = configure(352, 288, "yuv420p", coder=1, slices=4)
    p.version = 2  # experimental in the reference (ffv1enc.c:703-706)
    with pytest.raises(FFV1Error) as e:
        HipEncoder(p, 0, 1)
    assert e.value.code == -38


@pytest.mark.parametrize("var,val,msg", [("FFV1HIP_DENSE", "0", "FFV1HIP_DENSE is not read"),
                                          ("FFV1HIP_DEBUG", "serial,no_such_hook", "unknown hook")])
def test_hooks_misspelt_or_legacy_are_refused(var, val, msg, monkeypatch):
    """Measurement hooks go through FFV1HIP_DEBUG=name[=value],... only: an
    unknown name there, or one of the per-hook variables of earlier rounds,
    fails create (before any GPU work) instead of silently measuring the
    default."""
    from ffv1hip import configure, HipEncoder, FFV1Error
    monkeypatch.setenv(var, val)
    with pytest.raises(FFV1Error) as e:
        HipEncoder(configure(352, 288, "yuv420p", coder=1, slices=4), 0, 1)
    assert e.value.code == -22 and msg in str(e.value)


def test_other_ffv1hip_variables_are_not_hooks(monkeypatch):
    """Only the legacy per-hook names are refused: FFV1HIP_TWOPASS_LIB (the
    sanitizer run's), FFV1HIP_LIB and the like belong to other tools, and a
    process carrying them still creates its encoder (here, without a GPU, it
    gets as far as the device check)."""
    from ffv1hip import configure, HipEncoder, FFV1Error
    monkeypatch.setenv("FFV1HIP_TWOPASS_LIB", "/nonexistent/libffv1twopass.so")
    monkeypatch.setenv("FFV1HIP_SOMETHING_ELSE", "1")
    try:
        HipEncoder(configure(352, 288, "yuv420p", coder=1, slices=4), 0, 1).close()
    except FFV1Error as e:
        assert "is not read" not in str(e) and "unknown hook" not in str(e)


def test_decoder_contract_checks_before_the_gpu():
    """ffv1hip_dec_create refuses what the GPU decoder does not decode
    (-ENOSYS) and extradata the parameters would not produce
    (AVERROR_INVALIDDATA) on the host, before any HIP call."""
    from ffv1hip import AVERROR_INVALIDDATA, FFV1Error, HipDecoder, configure
    from oracle import oracle
    p = configure(352, 288, "yuv420p10", coder=1, slices=4)
    ex = oracle.Encoder(oracle.configure(352, 288, "yuv420p10", coder=1, slices=4)).extradata()
    for field, value in (("version", 2), ("version", 1), ("context_model", 2), ("colorspace", 2),
                         ("ac", 3)):
        q = configure(352, 288, "yuv420p10", coder=1, slices=4)
        setattr(q, field, value)  # version 1 has a single slice
        with pytest.raises(FFV1Error) as e:
            HipDecoder(q, ex, 0)
        assert e.value.code == -38, field
    with pytest.raises(FFV1Error) as e:
        HipDecoder(p, ex[:-1] + bytes([ex[-1] ^ 0x5A]), 0)
    assert e.value.code == AVERROR_INVALIDDATA


def test_decoder_no_silent_cpu_fallback_without_gpu():
    import torch
    from ffv1hip import FFV1Error, HipDecoder, configure
    from oracle import oracle
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    p = configure(352, 288, "yuv420p10", coder=1, slices=4)
    ex = oracle.Encoder(oracle.configure(352, 288, "yuv420p10", coder=1, slices=4)).extradata()
    with pytest.raises(FFV1Error) as e:
        HipDecoder(p, ex, 0)
    assert e.value.code == -5


def test_configure_pass_flags_select_version_3():
    """AV_CODEC_FLAG_PASS1/2 force version >= 2 (ffv1enc.c:680-682), v3 at the default level."""
    from ffv1hip import configure
    for pass_ in (1, 2):
        got = configure(352, 288, "yuv420p", pass_=pass_).as_dict()
        ref = oracle.configure(352, 288, "yuv420p", pass_=pass_).as_dict()
        assert got["version"] == ref["version"] == 3
        assert {f: got[f] for f in FIELDS} == {f: ref[f] for f in FIELDS}


def test_host_planes_are_checked_before_the_copy():
    """A plane smaller than the parameters say is refused before the library
    would read past its end (4:2:2 needs full-height chroma)."""
    import numpy as np
    from ffv1hip import configure
    from ffv1hip.encoder import check_planes
    p = configure(160, 120, "yuv422p10", slices=4)
    good = [np.zeros((120, 160), np.uint16), np.zeros((120, 80), np.uint16), np.zeros((120, 80), np.uint16)]
    check_planes(p, good)
    with pytest.raises(ValueError):
        check_planes(p, [good[0], good[1][:60], good[2][:60]])
    with pytest.raises(ValueError):
        check_planes(p, [g.astype(np.uint8) for g in good])
    q = configure(64, 32, "bgr0")
    check_planes(q, [np.zeros((32, 256), np.uint8)])
    with pytest.raises(ValueError):
        check_planes(q, [np.zeros((32, 64), np.uint8)])


@pytest.mark.parametrize("fmt,slices,coder", [("bgr0", 4, 1), ("bgra", 0, 0), ("gbrp12", 6, -2),
                                              ("yuv444p10", 4, 1), ("yuva444p16", 0, 1)])
def test_configure_v4_matches_oracle(fmt, slices, coder):
    """-strict experimental admits level 4 (ffv1enc.c:703-706); the same
    formats are refused on both sides without it and for 8-bit / subsampled
    YCbCr (choose_rct_params reads outside the frame there)."""
    from ffv1hip import configure, FFV1Error
    ref = oracle.configure(352, 288, fmt, slices=slices, level=4, coder=coder, experimental=True).as_dict()
    got = configure(352, 288, fmt, slices=slices, level=4, coder=coder, experimental=True).as_dict()
    assert got["version"] == 4
    for f in FIELDS:
        assert got[f] == ref[f], f
    with pytest.raises(FFV1Error):
        configure(352, 288, fmt, slices=slices, level=4, coder=coder)
    for bad in ("yuv420p10", "yuv444p", "gray16"):
        with pytest.raises(FFV1Error):
            configure(352, 288, bad, level=4, experimental=True)
