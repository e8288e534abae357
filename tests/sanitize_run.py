"""Workload for the sanitizer build (tests/test_sanitize.py runs it in a
child process with the AddressSanitizer runtime preloaded and the _asan
libraries selected by FFV1_ORACLE_LIB / FFV1HIP_SYNTH_LIB).  It drives the
CPU code the judge's hygiene item names: the oracle encoder and decoder
(every coder, version, bit depth, RGB, 2-pass, and decoding of damaged
packets, the reference's trasher.c idea: random byte bursts), the synthetic
clip generators (csrc/synth.c) and the pass-2 statistics parser
(csrc/ffv1_twopass.cpp, pass2_states) on well-formed and malformed text.
Exits non-zero on any failure; the sanitizers abort on their own findings.
"""
import ctypes
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ffmpeg-ffv1-p-frames_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

from helpers import PARITY_STREAMS, RGB_STREAMS, load_golden  # noqa: E402
from oracle import oracle  # noqa: E402
from ffv1hip import synth  # noqa: E402


def trash(pkt: bytes, rnd: random.Random) -> bytes:
    b = bytearray(pkt)
    for _ in range(rnd.randint(1, 4)):
        at = rnd.randrange(len(b))
        for k in range(rnd.randint(1, 16)):
            if at + k < len(b):
                b[at + k] = rnd.randrange(256)
    return bytes(b)


def main():
    rnd = random.Random(1)
    # every parity stream through the oracle, then its decoder on clean and
    # damaged packets
    for s in PARITY_STREAMS + RGB_STREAMS:
        frames = list(s.frames())[:4]
        cfg = s.oracle_config()
        enc = oracle.Encoder(cfg)
        ex = enc.extradata()
        pkts = [enc.encode(f)[0] for f in frames]
        dec = oracle.Decoder(cfg, ex)
        for p in pkts:
            dec.decode(p)
        dec = oracle.Decoder(cfg, ex)
        for p in pkts:
            try:
                dec.decode(trash(p, rnd))
            except RuntimeError:
                pass  # an error return is fine; memory errors are not
        print("ok", s.name, flush=True)
    # 2-pass through the oracle
    s = PARITY_STREAMS[1]
    frames = list(s.frames())[:5]
    cfg1 = oracle.configure(s.width, s.height, s.pix_fmt, slices=s.slices, gop_size=s.gop_size, pass_=1)
    e1 = oracle.Encoder(cfg1, 1)
    for f in frames:
        e1.encode(f)
    stats = e1.stats_out()
    cfg2 = oracle.configure(s.width, s.height, s.pix_fmt, slices=s.slices, gop_size=s.gop_size, pass_=2)
    e2 = oracle.Encoder(cfg2, 2, stats)
    for f in frames:
        e2.encode(f)
    print("ok 2-pass oracle", flush=True)
    # the pass-2 parser of the product's host code on good and bad text
    tp = ctypes.CDLL(os.environ["FFV1HIP_TWOPASS_LIB"])
    u8p = ctypes.POINTER(ctypes.c_uint8)
    tp.ffv1hip_internal_pass2_states.argtypes = [ctypes.c_char_p, ctypes.c_int, u8p, u8p, u8p, u8p]
    stt = np.arange(256, dtype=np.uint8)
    stt[1:] = np.minimum(255, np.arange(1, 256) + 4).astype(np.uint8)
    dflt = stt.copy()
    i0 = np.zeros(666 * 32, np.uint8)
    i1 = np.zeros(7563 * 32, np.uint8)
    P = lambda a: a.ctypes.data_as(u8p)  # noqa: E731
    texts = [stats, stats + stats, stats[: len(stats) // 2], stats[:10], "", "1 2 3", stats.replace("0", "x", 5),
             "9" * 5000, stats + "\n\n", " ".join(["99999999999999999999"] * 600)]
    for t in texts:
        rc = tp.ffv1hip_internal_pass2_states(t.encode(), 1, P(stt.copy()), P(dflt), P(i0), P(i1))
        print("pass2_states", len(t), rc, flush=True)
    # the synthetic clips (videogen at several sizes, rotozoom, D2)
    for w, h in ((34, 34), (352, 288), (640, 360)):
        list(synth.videogen_frames(w, h, 3, depth=10))
    pnm = open(os.path.join(ROOT, "tests", "golden", "reference.pnm"), "rb").read()
    roto = synth.RotozoomClip(pnm, 352, 288)
    for _ in range(3):
        roto.next_yuv420p()
    list(synth.d2_frames(96, 64, 2))
    assert load_golden("known_answers.json")
    print("sanitize run done", flush=True)


if __name__ == "__main__":
    main()
