#!/usr/bin/env python3
"""One ffv1_code configuration for PMC profiling (argv: width height slices frames gop)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ffmpeg-ffv1-p-frames_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
w, h, sl, n, g = (int(x) for x in sys.argv[1:6])
import diag
diag.run(w, h, sl, n, g, f"{w}x{h}_s{sl}_n{n}", reps=1)
