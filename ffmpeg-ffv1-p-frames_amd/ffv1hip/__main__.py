"""Command line: raw video <-> FFV1 in AVI on the GPU.

    python -m ffv1hip encode -s 352x288 -pix_fmt yuv420p [-slices 4] [-level 3]
                             [-coder 1] [-context 0] [-g 12] [-slicecrc 1]
                             [-strict experimental] [-batch 12] in.yuv out.avi
    python -m ffv1hip decode in.avi out.yuv
    python -m ffv1hip info in.avi

``encode`` is what ``ffmpeg -f rawvideo -pix_fmt F -s WxH -i in.yuv -c:v ffv1
<options> -flags +bitexact -fflags +bitexact out.avi`` does with the
reference (tests/fate-run.sh:171-193): the raw frames (planes back to back,
little-endian 16-bit samples above 8 bit, rawvideo's layout) go through
AVCodec.encode2 one frame per call (FFV1Encoder, AV_CODEC_CAP_DELAY) and the
packets into the bit-exact AVI muxer (ffv1hip.avi).  Option names and
defaults are ffmpeg's (ffv1enc.c:1383-1413, options_table.h).  ``decode``
runs the GPU decoder (the streams it reads: include/ffv1hip.h) and writes
the raw frames back.
"""
from __future__ import annotations

import argparse
import sys

import numpy as np

from . import AVCodecContext, FFV1Encoder, HipDecoder, configure
from .encoder import FF_COMPLIANCE_EXPERIMENTAL


def _strict(v: str) -> int:
    """ffmpeg's -strict: a number or one of its names (options_table.h)."""
    names = {"very": 2, "strict": 1, "normal": 0, "unofficial": -1, "experimental": -2}
    return names[v] if v in names else int(v)
from .avi import read_avi, write_avi


def _frame_planes(params):
    dt = np.uint8 if params.sample_bytes in (1, 4) else np.dtype("<u2")
    return params.plane_shapes(), dt


def _read_frames(path, params):
    shapes, dt = _frame_planes(params)
    n = sum(h * w for h, w in shapes)
    itemsize = np.dtype(dt).itemsize
    with open(path, "rb") as f:
        while True:
            buf = f.read(n * itemsize)
            if len(buf) < n * itemsize:
                return
            flat = np.frombuffer(buf, dt)
            planes, off = [], 0
            for h, w in shapes:
                planes.append(flat[off:off + h * w].reshape(h, w))
                off += h * w
            yield planes


def encode(a) -> int:
    w, h = (int(v) for v in a.s.lower().split("x"))
    avctx = AVCodecContext(w, h, a.pix_fmt, gop_size=a.g, slices=a.slices, level=a.level,
                           coder=a.coder, context=a.context, slicecrc=a.slicecrc,
                           strict_std_compliance=_strict(a.strict))
    enc = FFV1Encoder(batch=a.batch)
    enc.init(avctx)
    params = enc.params
    packets = []
    for pts, frame in enumerate(_read_frames(a.input, params)):
        pkt = enc.encode2(frame, pts)
        if pkt is not None:
            packets.append((pkt.data, pkt.key))
    while (pkt := enc.encode2(None)) is not None:
        packets.append((pkt.data, pkt.key))
    enc.close()
    with open(a.output, "wb") as f:
        f.write(write_avi(w, h, avctx.extradata, packets))
    print(f"{len(packets)} frames, {sum(len(p) for p, _ in packets)} bytes of packets -> {a.output}",
          file=sys.stderr)
    return 0


def decode(a) -> int:
    with open(a.input, "rb") as f:
        w, h, fourcc, extradata, packets = read_avi(f.read())
    if fourcc != b"FFV1":
        raise SystemExit(f"{a.input}: not an FFV1 stream ({fourcc!r})")
    params = configure(w, h, a.pix_fmt, slices=a.slices, coder=a.coder, context=a.context,
                       gop_size=a.g, level=a.level, slicecrc=a.slicecrc,
                       experimental=_strict(a.strict) <= FF_COMPLIANCE_EXPERIMENTAL)
    dec = HipDecoder(params, extradata, 0)
    with open(a.output, "wb") as f:
        for i in range(0, len(packets), a.batch):
            for planes, _ in dec.decode([p for p, _ in packets[i:i + a.batch]]):
                for p in planes:
                    f.write(np.ascontiguousarray(p).astype(p.dtype.newbyteorder("<")).tobytes())
    dec.close()
    return 0


def info(a) -> int:
    with open(a.input, "rb") as f:
        w, h, fourcc, extradata, packets = read_avi(f.read())
    keys = sum(k for _, k in packets)
    print(f"{a.input}: {fourcc.decode(errors='replace')} {w}x{h}, {len(packets)} packets "
          f"({keys} key), {sum(len(p) for p, _ in packets)} bytes, extradata {len(extradata)} bytes")
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m ffv1hip")
    sub = ap.add_subparsers(dest="cmd", required=True)
    for name in ("encode", "decode"):
        p = sub.add_parser(name)
        p.add_argument("-s", required=(name == "encode"), help="WxH (encode)")
        p.add_argument("-pix_fmt", default="yuv420p")
        p.add_argument("-slices", type=int, default=0)
        p.add_argument("-level", type=int, default=-1)
        p.add_argument("-coder", type=int, default=-1)
        p.add_argument("-context", type=int, default=0)
        p.add_argument("-g", type=int, default=12)
        p.add_argument("-slicecrc", type=int, default=-1)
        p.add_argument("-strict", default="normal", help="-strict experimental: levels 2 and 4")
        p.add_argument("-batch", type=int, default=12, help="frames per GPU call")
        p.add_argument("input")
        p.add_argument("output")
    p = sub.add_parser("info")
    p.add_argument("input")
    a = ap.parse_args(argv)
    return {"encode": encode, "decode": decode, "info": info}[a.cmd](a)


if __name__ == "__main__":
    sys.exit(main())
