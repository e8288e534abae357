#!/usr/bin/env python3
"""Builds the in-tree native libraries of the MI355X FFV1 encoder.

  lib/libffv1hip.so    HIP kernels (gfx950) + the C-ABI of include/ffv1hip.h
  lib/libffv1hip_check.so  the same with the device bounds checks (-DFFV1HIP_BOUNDS:
                       the walk's and the coder's writes checked against their
                       extents, ffv1_internal.h Bounds); select it with
                       FFV1HIP_LIB (ffv1hip/_paths.py)
  lib/libffv1synth.so  synthetic input clips (host C)

Everything is built in-tree so the .so files travel with the repo snapshot to
the GPU box (they are git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
ARCH = os.environ.get("FFV1HIP_ARCH", "gfx950")


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def build_synth(force=False):
    os.makedirs(LIB, exist_ok=True)
    out = os.path.join(LIB, "libffv1synth.so")
    src = [os.path.join(CSRC, "synth.c")]
    if force or _stale(out, src):
        _run(["gcc", "-O2", "-std=c11", "-Wall", "-fPIC", "-shared", "-o", out] + src)
    return out


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def build_hip(force=False, extra=(), check=False):
    os.makedirs(LIB, exist_ok=True)
    out = os.path.join(LIB, "libffv1hip_check.so" if check else "libffv1hip.so")
    if check:
        extra = ("-DFFV1HIP_BOUNDS", *extra)
    srcs = [os.path.join(CSRC, "ffv1_kernels.hip"), os.path.join(CSRC, "ffv1_decode.hip"),
            os.path.join(CSRC, "ffv1_host.cpp"), os.path.join(CSRC, "ffv1_twopass.cpp")]
    deps = srcs + [os.path.join(CSRC, "ffv1_internal.h"), os.path.join(INCLUDE, "ffv1hip.h")]
    if force or _stale(out, deps):
        _run([hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
              "-Wall", "-Wno-unused-function", "-I", INCLUDE, "-o", out, *extra] + srcs)
    return out


def build_all(force=False, check=True):
    # the release and the checked library compile side by side (~70 s each)
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(2) as ex:
        jobs = [ex.submit(build_hip, force)] + ([ex.submit(build_hip, force, (), True)] if check else [])
        return [build_synth(force)] + [j.result() for j in jobs]


if __name__ == "__main__":
    force = "--force" in sys.argv
    for p in build_all(force, check="--no-check" not in sys.argv):
        print(p)
