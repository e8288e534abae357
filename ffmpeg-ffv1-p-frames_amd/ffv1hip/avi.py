"""AVI container for FFV1 streams: the bit-exact muxer the reference's
FATE tests write, and a reader for what it writes.

The reference's FATE tests (tests/fate/vcodec.mak:113-127, enc_dec in
tests/fate-run.sh:171-193) encode a raw clip to ``<test>.avi`` with
``-flags +bitexact -fflags +bitexact`` and record the MD5 and size of that
file (tests/ref/vsynth/vsynth*-ffv1*).  ``write_avi`` writes the same
single-video-stream AVI the reference muxer writes for a seekable output,
so a stream from this encoder lands in the same file bytes.  It restates:

* libavformat/avienc.c:237-525  avi_write_header (avih, strl/strh/strf,
  the OpenDML master-index JUNK placeholder :210-235, the odml JUNK list
  :491-500, the 1016-byte JUNK padding :507-517, LIST movi);
* libavformat/avienc.c:794-843  avi_write_packet_internal (``00dc`` chunk,
  idx1 entry, odd-size pad byte);
* libavformat/avienc.c:618-671, 845-905  idx1 and the trailer's counters
  (frame counts, dwSuggestedBufferSize = largest chunk);
* libavformat/riffenc.c:30-48  ff_start_tag / ff_end_tag, and :207-250
  ff_put_bmp_header (BITMAPINFOHEADER + extradata, padded to even).

What the ffmpeg CLI feeds the muxer in those runs (ffmpeg 3.x defaults):
time base 1/25 (rawvideo demuxer default rate), ``bit_rate`` 200000
(AV_CODEC_DEFAULT_BITRATE, libavcodec/options_table.h:42-45),
``bits_per_coded_sample`` 0 (so the BMP depth is 24), codec tag 'FFV1'
(libavformat/riff.c:316), SAR 0/1 (no vprp), no INFO list under bitexact
(libavformat/mux.c:411-415).

``read_avi`` is the matching demuxer subset (avidec.c: strf extradata,
``00dc`` chunks in movi order, key flags from idx1).
"""
from __future__ import annotations

import io
import math
import struct
from typing import Iterable, List, Tuple

AVIF_HASINDEX = 0x10
AVIF_ISINTERLEAVED = 0x100
AVIF_TRUSTCKTYPE = 0x800
AVIIF_KEYFRAME = 0x10
AVI_MASTER_INDEX_SIZE = 256


class _Riff:
    def __init__(self):
        self.b = io.BytesIO()

    def tell(self):
        return self.b.tell()

    def w(self, data: bytes):
        self.b.write(data)

    def wl32(self, v):
        self.w(struct.pack("<I", v & 0xFFFFFFFF))

    def wl16(self, v):
        self.w(struct.pack("<H", v & 0xFFFF))

    def start_tag(self, tag: bytes) -> int:
        self.w(tag)
        self.wl32(0xFFFFFFFF)
        return self.tell()

    def end_tag(self, start: int):
        pos = self.tell()
        if pos & 1:
            self.w(b"\0")
        self.b.seek(start - 4)
        self.wl32(pos - start)
        self.b.seek((pos + 1) & ~1)

    def patch32(self, at: int, v: int):
        cur = self.tell()
        self.b.seek(at)
        self.wl32(v)
        self.b.seek(cur)


def write_avi(width: int, height: int, extradata: bytes,
              packets: Iterable[Tuple[bytes, bool]], tb=(1, 25), bit_rate=200000,
              fourcc=b"FFV1") -> bytes:
    """One video stream of FFV1 packets ``(data, key)`` -> the AVI file bytes."""
    r = _Riff()
    # avi_start_new_riff (avienc.c:137-156)
    riff_start = r.start_tag(b"RIFF")
    r.w(b"AVI ")
    list1 = r.start_tag(b"LIST")
    r.w(b"hdrl")
    # avih (avienc.c:265-308)
    r.w(b"avih")
    r.wl32(14 * 4)
    r.wl32(1000000 * tb[0] // tb[1])
    r.wl32(bit_rate // 8)
    r.wl32(0)
    r.wl32(AVIF_TRUSTCKTYPE | AVIF_HASINDEX | AVIF_ISINTERLEAVED)
    frames_hdr_all = r.tell()
    r.wl32(0)
    r.wl32(0)
    r.wl32(1)
    r.wl32(1024 * 1024)
    r.wl32(width)
    r.wl32(height)
    for _ in range(4):
        r.wl32(0)
    # strl (avienc.c:311-489)
    list2 = r.start_tag(b"LIST")
    r.w(b"strl")
    strh = r.start_tag(b"strh")
    r.w(b"vids")
    r.w(fourcc)
    r.wl32(0)          # flags
    r.wl16(0)          # priority
    r.wl16(0)          # language
    r.wl32(0)          # initial frame
    g = math.gcd(tb[0], tb[1])
    r.wl32(tb[0] // g)  # scale
    r.wl32(tb[1] // g)  # rate
    r.wl32(0)          # start
    frames_hdr_strm = r.tell()
    r.wl32(0)          # length, filled by the trailer
    r.wl32(1024 * 1024)  # suggested buffer size, replaced by max chunk size
    r.wl32(0xFFFFFFFF)  # quality
    r.wl32(0)          # sample size (block_align)
    r.wl32(0)
    r.wl16(width)
    r.wl16(height)
    r.end_tag(strh)
    strf = r.start_tag(b"strf")
    # ff_put_bmp_header (riffenc.c:207-250)
    r.wl32(40 + len(extradata))
    r.wl32(width)
    r.wl32(height)      # codec_tag != 0: stored as is
    r.wl16(1)
    r.wl16(24)
    r.w(fourcc)
    r.wl32((width * height * 24 + 7) // 8)
    for _ in range(4):
        r.wl32(0)
    if extradata:
        r.w(extradata)
        if len(extradata) & 1:
            r.w(b"\0")
    r.end_tag(strf)
    # write_odml_master (avienc.c:210-235)
    indx = r.start_tag(b"JUNK")
    r.wl16(4)
    r.w(b"\0\0")
    r.wl32(0)
    r.w(b"00dc")
    r.w(b"\0" * 12)
    r.w(b"\0" * (8 * AVI_MASTER_INDEX_SIZE * 2))
    r.end_tag(indx)
    r.end_tag(list2)
    # odml placeholder (avienc.c:491-500)
    odml = r.start_tag(b"JUNK")
    r.w(b"odml")
    r.w(b"dmlh")
    r.wl32(248)
    r.w(b"\0" * 248)
    r.end_tag(odml)
    r.end_tag(list1)
    # padding (avienc.c:507-517)
    junk = r.start_tag(b"JUNK")
    r.w(b"\0" * 1016)
    r.end_tag(junk)
    movi = r.start_tag(b"LIST")
    r.w(b"movi")
    # packets (avienc.c:794-843)
    index = []
    count = 0
    max_size = 0
    for data, key in packets:
        count += 1
        index.append((AVIIF_KEYFRAME if key else 0, r.tell() - movi, len(data)))
        max_size = max(max_size, len(data))
        r.w(b"00dc")
        r.wl32(len(data))
        r.w(data)
        if len(data) & 1:
            r.w(b"\0")
    # trailer (avienc.c:858-862, 618-671)
    r.end_tag(movi)
    idx = r.start_tag(b"idx1")
    for flags, pos, size in index:
        r.w(b"00dc")
        r.wl32(flags)
        r.wl32(pos)
        r.wl32(size)
    r.end_tag(idx)
    r.patch32(frames_hdr_strm, count)
    r.patch32(frames_hdr_all, count)
    r.end_tag(riff_start)
    r.patch32(frames_hdr_strm + 4, max_size)
    return r.b.getvalue()


def read_avi(data: bytes):
    """The first video stream of an AVI: ``(width, height, fourcc, extradata,
    [(packet, key), ...])``.  Keyframe flags come from idx1 when present."""
    if data[:4] != b"RIFF" or data[8:12] != b"AVI ":
        raise ValueError("not an AVI file")
    width = height = 0
    fourcc, extradata = b"", b""
    packets: List[bytes] = []
    flags: List[int] = []

    def walk(pos, end):
        nonlocal width, height, fourcc, extradata
        while pos + 8 <= end:
            tag = data[pos:pos + 4]
            size = struct.unpack_from("<I", data, pos + 4)[0]
            body = pos + 8
            if tag == b"LIST":
                walk(body + 4, min(end, body + size))
            elif tag == b"strf" and not fourcc:
                hdr = struct.unpack_from("<IiiHH4s", data, body)
                width, height, fourcc = hdr[1], abs(hdr[2]), hdr[5]
                extradata = data[body + 40:body + hdr[0]]
            elif tag[2:] in (b"dc", b"db") and tag[:2] == b"00":
                packets.append(data[body:body + size])
            elif tag == b"idx1":
                for k in range(size // 16):
                    ck, fl = struct.unpack_from("<4sI", data, body + 16 * k)
                    if ck[:2] == b"00" and ck[2:] in (b"dc", b"db"):
                        flags.append(fl)
            pos = body + size + (size & 1)

    walk(12, len(data))
    keys = [bool(f & AVIIF_KEYFRAME) for f in flags] if len(flags) == len(packets) else \
        [True] * len(packets)
    return width, height, fourcc, extradata, list(zip(packets, keys))
