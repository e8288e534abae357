"""Collect the reference's FATE pins for the FFV1 vsynth tests into a fixture.

Reads /root/reference/tests/ref/vsynth/vsynth{1,2,3}-ffv1* (data: the MD5 and
size of each encoded AVI, and the MD5 of the decoded raw video) and the
options each test passes (tests/fate/vcodec.mak:113-127), and writes
tests/golden/fate_vsynth.json.  Run here only; the GPU box reads the JSON.
"""
import json
import os
import re

REF = "/root/reference/tests/ref/vsynth"
OUT = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "fate_vsynth.json")

# vcodec.mak:116-127 -> (pix_fmt, encoder options)
VARIANTS = {
    "ffv1": ("yuv420p", {"slices": 4}),
    "ffv1-v0": ("yuv420p", {}),
    "ffv1-v3-yuv420p": ("yuv420p", {"level": 3}),
    "ffv1-v3-yuv422p10": ("yuv422p10", {"level": 3}),
    "ffv1-v3-yuv444p16": ("yuv444p16", {"level": 3}),
    "ffv1-v3-bgr0": ("bgr0", {"level": 3}),
}
SOURCES = {"vsynth1": ("videogen", 352, 288), "vsynth2": ("rotozoom", 352, 288),
           "vsynth3": ("videogen", 34, 34)}

pins = []
for src, (gen, w, h) in SOURCES.items():
    for var, (fmt, opts) in VARIANTS.items():
        text = open(os.path.join(REF, f"{src}-{var}")).read().split("\n")
        avi_md5 = re.match(r"([0-9a-f]{32}) ", text[0]).group(1)
        avi_size = int(text[1].split()[0])
        raw_md5 = re.match(r"([0-9a-f]{32}) ", text[2]).group(1)
        pins.append({"test": f"{src}-{var}", "source": gen, "width": w, "height": h,
                     "frames": 50, "pix_fmt": fmt, "options": opts, "gop_size": 12,
                     "avi_md5": avi_md5, "avi_size": avi_size, "decoded_md5": raw_md5,
                     "psnr_line": text[3]})
with open(OUT, "w") as f:
    json.dump({"origin": "reference tests/ref/vsynth (FATE), tests/fate/vcodec.mak:1-10,113-127",
               "pins": pins}, f, indent=1)
print(len(pins), "pins ->", OUT)
