"""Locations of the native libraries built in-tree by build.py."""
from __future__ import annotations

import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT_DIR = os.path.dirname(PKG_DIR)               # ffmpeg-ffv1-p-frames_amd/
CSRC_DIR = os.path.join(ROOT_DIR, "csrc")
LIB_DIR = os.path.join(ROOT_DIR, "lib")
REPO_DIR = os.path.dirname(ROOT_DIR)
INCLUDE_DIR = os.path.join(REPO_DIR, "include")


def synth_lib() -> str:
    # FFV1HIP_SYNTH_LIB: another build of the same source (the sanitizer
    # build, oracle/Makefile `sanitize`)
    p = os.environ.get("FFV1HIP_SYNTH_LIB") or os.path.join(LIB_DIR, "libffv1synth.so")
    if not os.path.exists(p):
        raise FileNotFoundError(f"{p} missing: run `python ffmpeg-ffv1-p-frames_amd/build.py`")
    return p


def hip_lib() -> str:
    p = os.environ.get("FFV1HIP_LIB") or os.path.join(LIB_DIR, "libffv1hip.so")
    if not os.path.exists(p):
        raise FileNotFoundError(
            f"{p} missing: the HIP encoder is not built (run `python ffmpeg-ffv1-p-frames_amd/build.py`)")
    return p
