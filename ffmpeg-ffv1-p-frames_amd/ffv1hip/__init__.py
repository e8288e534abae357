"""MI355X-native FFV1 encoder (host side).

The per-slice hot path (prediction, context quantisation, binarisation,
range coding with P-frame context-state carry, slice CRC and packet
assembly) runs as HIP kernels in ``lib/libffv1hip.so``; this package is the
host mirror of the reference's AVCodec interface over that C-ABI.
"""
from .encoder import (AV_CODEC_FLAG_PASS1, AV_CODEC_FLAG_PASS2, AVCodecContext, AVPacket, FFV1Encoder, FFV1Error, HipEncoder, Options,
                      Params, configure, load_library, EXPORTED_SYMBOLS, AVERROR_INVALIDDATA,
                      HipDecoder)

__all__ = ["AV_CODEC_FLAG_PASS1", "AV_CODEC_FLAG_PASS2", "AVCodecContext", "AVPacket", "FFV1Encoder", "FFV1Error", "HipEncoder", "Options",
           "Params", "configure", "load_library", "EXPORTED_SYMBOLS", "AVERROR_INVALIDDATA",
           "HipDecoder"]
