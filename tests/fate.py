"""The reference's FATE vsynth FFV1 tests, rebuilt as test inputs (TEST INFRA).

Each pin in tests/golden/fate_vsynth.json is one reference FATE test
(tests/fate/vcodec.mak:113-127): a 50-frame yuv420p clip (vsynth1 =
tests/videogen.c at 352x288, vsynth2 = tests/rotozoom.c over
tests/reference.pnm, vsynth3 = videogen at 34x34), converted to the test's
pixel format the way ``-sws_flags neighbor+bitexact`` does, encoded with the
test's options (ffmpeg defaults otherwise: gop 12, coder from the private
option's default), muxed to AVI.  The pins are the AVI's MD5 and size and
the MD5 of the clip decoded back to yuv420p.
"""
from __future__ import annotations

import hashlib
import os

import numpy as np

from helpers import GOLDEN_DIR, load_golden
from ffv1hip import synth
from ffv1hip.avi import write_avi

PINS = load_golden("fate_vsynth.json")["pins"]


def raw_clip(pin):
    """The FATE source clip: 50 yuv420p u8 frames."""
    if pin["source"] == "videogen":
        clip = synth.VideogenClip(pin["width"], pin["height"])
    else:
        with open(os.path.join(GOLDEN_DIR, "reference.pnm"), "rb") as f:
            clip = synth.RotozoomClip(f.read(), pin["width"], pin["height"])
    return [[np.ascontiguousarray(p) for p in clip.next_yuv420p()] for _ in range(pin["frames"])]


def input_frames(pin, raw):
    return [synth.convert(f, pin["pix_fmt"]) for f in raw]


def encoder_options(pin):
    o = dict(pin["options"])
    return dict(slices=o.get("slices", 0), level=o.get("level", -1), coder=-1,
                gop_size=pin["gop_size"])


def avi_bytes(pin, extradata, packets):
    return write_avi(pin["width"], pin["height"], extradata, packets)


def raw_md5(raw):
    h = hashlib.md5()
    for f in raw:
        for p in f:
            h.update(p.tobytes())
    return h.hexdigest()


def back_to_yuv420p(planes, pin):
    """Decoded planes -> yuv420p u8 (the inverse of synth.convert on the
    samples it produced: drop the depth shift, take every other chroma row /
    column)."""
    fmt = pin["pix_fmt"]
    depth = 16 if fmt.endswith("16") else 10 if fmt.endswith("10") else 8
    y, u, v = [np.asarray(p) for p in planes]
    if fmt.startswith("yuv444"):
        u, v = u[::2, ::2], v[::2, ::2]
    elif fmt.startswith("yuv422"):
        u, v = u[::2], v[::2]
    return [np.ascontiguousarray((p >> (depth - 8)).astype(np.uint8)) for p in (y, u, v)]
