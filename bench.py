#!/usr/bin/env python3
"""Benchmark: Mpixels/s of bit-exact FFV1 P-frame encoding on MI355X.

Workload (BASELINE.json configs[2], the metric's config): 3840x2160
yuv420p10le, coder=1 (range coder, custom state table), slices=64 (8x8),
keyint=12, i.e. FFV1 v3 with P-frames whose context states carry across the
GOP.  Input is the reference's own synthetic clip (tests/videogen, widened
to 10 bit) or the LSB-active D2 clip (--data d2), generated on the host and
made resident in HBM before timing.

A "step" = one pass of the encoder over a batch of --gops GOPs (12 frames
each) already in HBM: slice coding + packet assembly, packets left in HBM.
Multi-GPU: one process per GPU over ONE clip of N x gops GOPs: rank r encodes
GOPs r, r+N, r+2N, ... (GOPs are independent: keyframes reset every context
state, ffv1enc.c:1171-1172), no data-path collective; value = all frames of
all ranks / max-over-ranks time.  After the timed steps the per-GOP packet
digests are gathered on rank 0 (a digest of the first config-default count
of GOPs that does not depend on N), the packets of the pinned frames are gathered from the ranks
that own them and checked against the reference's MD5, and every rank
decodes its own packets with the GPU decoder.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ffmpeg-ffv1-p-frames_amd"))

W, H, PIX_FMT, SLICES, GOP = 3840, 2160, "yuv420p10", 64, 12
# --config: c3 is the metric's workload (BASELINE configs[2]); the others are
# the remaining BASELINE configs on one GPU, checked by the GPU decoder's
# lossless round trip (and c2 also by the reference's MD5 pin).
CONFIGS = {
    "c3": dict(W=3840, H=2160, PIX_FMT="yuv420p10", SLICES=64, GOP=12, BPR=0, DEPTH=10, C444=False,
               GRID=False, GOPS=24, PIN=("08e3975d4d0f5f2e5c82cd4037764789", 24),  # 24 GOPs: 1280 walk waves in 5-wave blocks, one round
               metric="Mpixels/s encoded (bit-exact) 4K yuv420p10 FFV1 P-frames",
               workload="4K 3840x2160 yuv420p10le, coder=1 (range, custom table), slices=64, keyint=12 P-frames"),
    "c2": dict(W=1920, H=1080, PIX_FMT="yuv420p", SLICES=24, GOP=1, BPR=0, DEPTH=8, C444=False,
               GRID=False, GOPS=480, PIN=("58e800634d515e024a515ba618f24dc3", 50),
               metric="Mpixels/s encoded (bit-exact) 1080p yuv420p FFV1 intra",
               workload="1080p 1920x1080 yuv420p, coder=1 (range, custom table), slices=24, intra-only"),
    "c4": dict(W=3840, H=2160, PIX_FMT="yuv444p16", SLICES=64, GOP=12, BPR=12, DEPTH=16, C444=True,
               GRID=False, GOPS=21, PIN=None,  # 21: 1024 walk waves in 4-wave blocks, both records sets (8.59 vs 8.21 Gpix/s at 20); 22: one set, 6.55
               metric="Mpixels/s encoded (lossless) 4K yuv444p12 FFV1 P-frames",
               workload="4K 3840x2160 yuv444p16le + bits_per_raw_sample=12, coder=1, slices=64, keyint=12 P-frames"),
    "c5": dict(W=7680, H=4320, PIX_FMT="yuv420p10", SLICES=256, GOP=12, BPR=0, DEPTH=10, C444=False,
               GRID=True, GOPS=6, PIN=None,  # 6 GOPs: 1280 walk waves in 5-wave blocks, one round (5: 14.1 vs 15.5 Gpix/s)
               metric="Mpixels/s encoded (lossless) 8K yuv420p10 FFV1 P-frames",
               workload="8K 7680x4320 yuv420p10le, coder=1, slices=256 (16x16 grid), keyint=12 P-frames"),
}
CFG = CONFIGS["c3"]
BPR, DEPTH, C444, GRID = 0, 10, False, False


def select_config(name):
    global W, H, PIX_FMT, SLICES, GOP, BPR, DEPTH, C444, GRID, CFG
    CFG = CONFIGS[name]
    W, H, PIX_FMT, SLICES, GOP = CFG["W"], CFG["H"], CFG["PIX_FMT"], CFG["SLICES"], CFG["GOP"]
    BPR, DEPTH, C444, GRID = CFG["BPR"], CFG["DEPTH"], CFG["C444"], CFG["GRID"]


def hip_configure():
    from ffv1hip import configure
    return configure(W, H, PIX_FMT, slices=SLICES, coder=1, gop_size=GOP, bits_per_raw_sample=BPR,
                     allow_large_grid=GRID)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
KERNEL = {"symbols": "ffv1_symbols", "layout": "ffv1_layout", "bits": "ffv1_bits", "states": "ffv1_walk",
          "code": "ffv1_range", "dseg": "ffv1_dseg", "dfix": "ffv1_dfix", "sink": "ffv1_sink",
          "assemble": "ffv1_assemble_packets"}
PIN_MD5_24 = "08e3975d4d0f5f2e5c82cd4037764789"  # tests/golden/known_answers.json (config 3)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def clip_frames(n_total, data, keep):
    """The frames i < n_total of the clip with keep(i), one at a time; the
    others are skipped (D1: the objects move, nothing is drawn; D2: the
    frame's noise is still drawn, the RNG stream being shared)."""
    from ffv1hip import synth
    if data == "d1":
        return synth.videogen_frames(W, H, n_total, depth=DEPTH, chroma444=C444, keep=keep)
    return synth.d2_frames(W, H, n_total, depth=DEPTH, chroma444=C444, keep=keep)


def pack_clip(gen, n, frame_bytes):
    """This rank's n frames packed as they are generated into one host batch
    [frame][frame_bytes] (what goes to HBM), and the frames as plane views
    into it: a rank holds one batch of host memory, never a frame list beside it."""
    buf = np.zeros((n, frame_bytes), np.uint8)
    frames = []
    for i, f in enumerate(gen):
        off, views = 0, []
        for p in f:
            nb = p.size * p.itemsize
            buf[i, off:off + nb] = p.reshape(-1).view(np.uint8)
            views.append(buf[i, off:off + nb].view(p.dtype).reshape(p.shape))
            off += nb
        frames.append(views)
    assert len(frames) == n
    return buf, frames


def make_frames(n_total, data, keep):
    """The kept frames of the clip as a list (tools and tests)."""
    return [f for f in clip_frames(n_total, data, keep)]


def cpu_threads():
    """The host cores this process may use: the affinity mask, capped at the
    box's CPU share for one GPU (OMP_NUM_THREADS, 16 on the GPU boxes)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(avail, share) if share > 0 else avail)


def cpu_baseline(frames, threads):
    """The CPU oracle (a port of the reference encoder, oracle/) on host cores.

    `value`: GOP-sharded, the strongest CPU configuration:
    each worker thread encodes whole GOPs (1 key + 11 P frames) with its own
    encoder; ctypes drops the GIL, so the threads run in parallel.  When the
    batch has fewer GOPs than threads (c5: 6 GOPs), each GOP's slices are
    coded on threads // GOPs threads, so every core works.  Plus the
    reference's own threading model, one job per slice on min(cores, slices)
    threads over one GOP (`slice_threaded`, ffv1enc.c:1323), and a one-thread
    run of one GOP.  Bounded sample: one GOP per GOP worker.
    """
    sys.path.insert(0, ROOT)
    from oracle import oracle
    if GRID:
        cfg = oracle.configure(W, H, PIX_FMT, slices=0, coder=1, gop_size=GOP)
        cfg.num_h_slices, cfg.num_v_slices = 16, 16
    else:
        cfg = oracle.configure(W, H, PIX_FMT, slices=SLICES, coder=1, gop_size=GOP,
                               bits_per_raw_sample=BPR)
    nslices = cfg.num_h_slices * cfg.num_v_slices
    per = max(GOP, 1)
    ngops = len(frames) // per
    workers = max(1, min(threads, ngops))
    # slice threads per GOP worker: the cores shared out, the first
    # threads % workers workers one more (c5: 6 GOPs on 16 cores = 4 x 3 + 2 x 2)
    inner = [max(1, threads // workers + (1 if g < threads % workers else 0)) for g in range(workers)]

    def one(g, th=1):
        enc = oracle.Encoder(cfg)
        for f in frames[g * per:(g + 1) * per]:
            enc.encode(f, threads=th)

    t0 = time.perf_counter()
    one(0)
    single = per * W * H / (time.perf_counter() - t0) / 1e6
    sl_threads = max(1, min(threads, nslices))
    t0 = time.perf_counter()
    one(0, sl_threads)
    slice_mt = per * W * H / (time.perf_counter() - t0) / 1e6
    ths = [threading.Thread(target=one, args=(g, inner[g])) for g in range(workers)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    multi = workers * per * W * H / (time.perf_counter() - t0) / 1e6
    return {
        "value": round(multi, 3), "unit": "Mpixels/s", "cores": sum(inner), "kind": "port",
        "sample": f"{workers} GOP workers with {'/'.join(map(str, sorted(set(inner), reverse=True)))} slice "
                  f"thread(s) each ({sum(inner)} in all), 1 GOP ({per} frames) each of the same "
                  f"{W}x{H} {PIX_FMT} clip, oracle/ffv1_oracle.c, GOP-sharded",
        "host_cpus": os.cpu_count(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
        "slice_threaded": {"value": round(slice_mt, 3), "cores": sl_threads,
                           "sample": f"1 GOP ({per} frames), one job per slice on {sl_threads} threads "
                                     f"(the reference's threading, ffv1enc.c:1323)"},
        "single_thread": {"value": round(single, 3), "cores": 1, "sample": f"1 GOP ({per} frames)"},
        "port_vs_reference": "the port runs at ~0.6x the reference ffmpeg single-threaded on the "
                             "same 8-core host (12 vs 20.1 Mpix/s, BASELINE.md / DESIGN.md)",
    }


def load_traffic(frames_per_step, kernel, data="d1"):
    """HBM bytes per launch of `kernel` from the committed PMC profile of the
    same configuration, batch and clip (profiles/pmc_traffic*.json; a file
    without a "data" key was profiled on the D1 clip), else None."""
    import glob
    import re

    def newest_first(path):  # pmc_traffic_rNN*.json: the latest round's profile wins
        m = re.search(r"_r(\d+)", os.path.basename(path))
        return (-int(m.group(1)) if m else 0, path)

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic*.json")), key=newest_first):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if (d.get("frames_per_launch") == frames_per_step and d.get("config") == f"{W}x{H} {PIX_FMT}"
                and d.get("data", "d1") == data):
            k = d.get("kernels", {}).get(kernel)
            if k:
                return k.get("hbm_bytes")
    return None


def spawn_ranks(n: int, script: str = "", argv=None) -> int:
    """`--gpus N` without a launcher: start N copies of this script, one per
    GPU, with the torch.distributed environment a launcher would set
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*, rendezvous on 127.0.0.1), and
    return the worst exit code.  Runs before anything touches a GPU: this
    process only waits for its children (started as new processes, never
    exec'd over this one)."""
    import signal
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        cmd = [sys.executable, script or os.path.abspath(__file__)] + list(sys.argv[1:] if argv is None else argv)
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0:
                    rc = rc or code
                    for q in live:  # a failed rank leaves the others waiting at a barrier
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


def load_bench_golden(name):
    """Per-GOP oracle digests of a config's clip (tests/golden/bench_gops.json,
    tools/make_bench_golden.py; key <config> for D1, <config>_d2 for D2), or None."""
    path = os.path.join(ROOT, "tests", "golden", "bench_gops.json")
    try:
        return json.load(open(path)).get(name)
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)  # the pipelines fill and drain once per run
    ap.add_argument("--warmup", type=int, default=1)
    # c3: 20 GOPs = 240 frames per batch: 1280 walk waves, all resident at
    # once (5 per CU with the dense context rows), one walk round per batch
    ap.add_argument("--gops", type=int, default=0,
                    help="GOPs per rank per step (default: 20 for c3, see CONFIGS)")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c3",
                    help="BASELINE config: c3 (the metric's, default), c2, c4, c5")
    ap.add_argument("--data", choices=("d1", "d2"), default="d1")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (default: this process's cores, capped at OMP_NUM_THREADS)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-decode-check", action="store_true",
                    help="skip decoding the last step's packets with the GPU decoder")
    args = ap.parse_args()
    select_config(args.config)
    if args.gops <= 0:
        args.gops = CFG["GOPS"]

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: one rank per GPU expected")

    import torch
    from ffv1hip import HipEncoder, configure

    # FFV1_BENCH_ONE_DEVICE=1 (rehearsal on a one-GPU box): every rank on
    # device 0, gloo instead of RCCL for the barrier / max / gather
    one_dev = os.environ.get("FFV1_BENCH_ONE_DEVICE") == "1"
    if one_dev:
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if one_dev:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    B = args.gops * GOP
    params = hip_configure()
    shapes = params.plane_shapes()
    plane_bytes = [h * w * params.sample_bytes for h, w in shapes]
    frame_bytes = (sum(plane_bytes) + 255) // 256 * 256
    offs = [0, plane_bytes[0], plane_bytes[0] + plane_bytes[1]]
    strides = [shapes[k][1] * params.sample_bytes for k in range(3)]

    # one clip of world x gops GOPs; this rank's are GOPs rank, rank+world, ...
    my_gops = [rank + world * j for j in range(args.gops)]
    t0 = time.perf_counter()
    host, frames = pack_clip(clip_frames(world * B, args.data, keep=lambda i: (i // GOP) % world == rank),
                             B, frame_bytes)
    d_frames = torch.from_numpy(host).to(f"cuda:{local_rank}")
    torch.cuda.synchronize()
    log(f"[rank {rank}] {B} frames (GOPs {my_gops[0]}, {my_gops[0] + world}, ...) generated and "
        f"resident in HBM in {time.perf_counter() - t0:.1f}s")

    enc = HipEncoder(params, device=local_rank, max_batch=B)

    def step():
        enc.encode_device(d_frames.data_ptr(), frame_bytes, offs, strides, B)

    for _ in range(args.warmup):
        step()
    enc.synchronize()
    torch.cuda.synchronize()

    # Kernel durations: HIP events recorded around every launch on the stream
    # it runs on, accumulated by the encoder over the timed steps and read
    # after them (reading per step would serialise the states walk of step
    # k+1 with the coding of step k, which the encoder overlaps).
    enc.set_profiling(True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    enc.synchronize()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    stats = enc.last_kernel_stats()
    if dist:
        dist.barrier()
        t = torch.tensor([elapsed], device="cpu" if one_dev else f"cuda:{local_rank}", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # packets of the last step (outside the timed region): this rank's GOPs
    pkts = enc.fetch(B)
    out_bytes = sum(len(p) for p, _ in pkts)
    gop_digest = {}
    for j, g in enumerate(my_gops):
        h = hashlib.md5()
        for p, _ in pkts[j * GOP:(j + 1) * GOP]:
            h.update(p)
        gop_digest[g] = (h.hexdigest(), sum(len(p) for p, _ in pkts[j * GOP:(j + 1) * GOP]))
    pin = CFG["PIN"]
    pin_gops = set(range((pin[1] + GOP - 1) // GOP)) if (pin and args.data == "d1") else set()
    pin_pkts = {g: [p for p, _ in pkts[j * GOP:(j + 1) * GOP]] for j, g in enumerate(my_gops)
                if g in pin_gops}
    if dist:
        # the exchange after the encode: per-GOP digests from every rank, and
        # the packets of the pinned frames from the ranks that own them
        gathered = [None] * world
        dist.all_gather_object(gathered, (gop_digest, out_bytes, pin_pkts))
    else:
        gathered = [(gop_digest, out_bytes, pin_pkts)]
    all_digest, all_pins, total_out = {}, {}, 0
    for d, ob, pp in gathered:
        all_digest.update(d)
        all_pins.update(pp)
        total_out += ob
    bitexact = None
    if pin_gops and all(g in all_pins for g in pin_gops):
        h = hashlib.md5()
        stream = [p for g in sorted(pin_gops) for p in all_pins[g]][:pin[1]]
        for p in stream:
            h.update(p)
        bitexact = h.hexdigest() == pin[0]
    n_all = len(all_digest)
    first = min(n_all, CFG["GOPS"])
    digest_first = hashlib.md5("".join(all_digest[g][0] for g in range(first)).encode()).hexdigest()
    # every timed GOP against the oracle's digest of the same GOP (the last
    # step's packets: every step re-encodes the same batch)
    vs_oracle = None
    golden = load_bench_golden(args.config if args.data == "d1" else f"{args.config}_d2")
    if golden:
        ref = golden["gops"]
        checked = [g for g in sorted(all_digest) if g < len(ref)]
        bad = [g for g in checked if (all_digest[g][0], all_digest[g][1]) != (ref[g]["md5"], ref[g]["bytes"])]
        vs_oracle = {"gops_checked": len(checked), "gops_encoded": n_all,
                     "frames_checked": len(checked) * max(GOP, 1), "equal": not bad,
                     "first_mismatch_gop": bad[0] if bad else None,
                     "fixture": "tests/golden/bench_gops.json (oracle, tools/make_bench_golden.py)"}

    # on-device lossless self-check (outside the timed region, every rank on
    # its own packets): the GPU decoder (ffv1_decode_slices)
    decode = None
    if not args.no_decode_check:
        from ffv1hip import HipDecoder
        dec = HipDecoder(params, enc.extradata(), local_rank)
        td = time.perf_counter()
        got = dec.decode([p for p, _ in pkts])
        td = time.perf_counter() - td
        dec.close()
        lossless = all(k == key and all(np.array_equal(a, b) for a, b in zip(planes, f))
                       for (planes, k), (_, key), f in zip(got, pkts, frames))
        del got
        if dist:
            t = torch.tensor([1 if lossless else 0], device="cpu" if one_dev else f"cuda:{local_rank}",
                             dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            lossless = bool(t.item())
        decode = {"frames": B * world, "lossless": lossless, "seconds": round(td, 3),
                  "mpix_s_per_gpu": round(B * W * H / td / 1e6, 2),
                  "note": "ffv1hip_decode on every rank of its own packets, incl. H2D of the "
                          "packets and D2H of the frames"}
        log(f"[rank {rank}] GPU decode self-check: {B} frames in {td:.2f}s, lossless={lossless}")

    names = ("symbols", "layout", "bits", "states", "code", "dseg", "dfix", "sink", "assemble")
    per_step = {k: stats[k + "_ms"] / args.steps for k in names}
    launches = {k: stats[k + "_launches"] // args.steps for k in names}
    # Dominant kernel: the longest per step of the two serial chains, the
    # states walk (ffv1_walk) and the range coder's serial pass (ffv1_range): each is ONE
    # launch per step over every frame of the batch.  Algorithmic bytes per
    # launch: the input planes of the batch (3.0 B per luma
    # pixel at 4:2:0 10 bit) + the packet bytes it produces.
    dom = max(("states", "code"), key=lambda k: per_step[k] / max(launches[k], 1))
    n_dom = max(launches[dom], 1)
    in_bytes = B * sum(plane_bytes)
    algo_per_launch = (in_bytes + out_bytes) / n_dom
    ms_per_launch = per_step[dom] / n_dom
    achieved = algo_per_launch / (ms_per_launch * 1e-3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(frames, args.cpu_threads or cpu_threads())

    mpix = args.steps * B * W * H * world / elapsed / 1e6
    if rank == 0:
        res = {
            "metric": CFG["metric"],
            "value": round(mpix, 2),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8" if params.sample_bytes == 1 else "u16",
            "data": f"synthetic ({f'tests/videogen clip at {DEPTH} bit' if args.data == 'd1' else 'D2 seeded noisy clip'}), HBM-resident",
            "config": {
                "workload": CFG["workload"],
                "frames_per_step_per_gpu": B,
                "gops_per_step_per_gpu": args.gops,
                "parallelism": f"gop-sharded x{world} (rank r: GOPs r, r+{world}, ... of one clip)",
            },
            "bits_per_pixel": round(total_out * 8 / (B * world * W * H), 4),
            "bitexact_vs_reference_pin": bitexact,
            "bitexact_vs_oracle": vs_oracle,
            "gop_digest": {"gops": n_all, f"first_{first}_gops_md5": digest_first,
                           "note": "md5 over the per-GOP packet md5s in GOP order: the same for "
                                   "every --gpus N (GOP bytes do not depend on the rank)"},
            # kernels of the overlapped pipelines: symbols -> layout -> walk
            # (batch k+1), bits beside the walk, range -> dseg -> dfix -> sink -> assemble (batch k)
            "kernel_ms_per_step": dict(
                **{KERNEL[k]: round(per_step[k], 3) for k in names},
                launches={KERNEL[k]: launches[k] for k in names}),
            "roofline": {
                "bound": "hbm",
                "kernel": KERNEL[dom],
                "achieved": round(achieved, 3),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6),
                "traffic": load_traffic(B, KERNEL[dom], args.data),
                "algorithmic_bytes_per_launch": int(algo_per_launch),
                "avg_launch_ms": round(ms_per_launch, 3),
            },
            "cpu_baseline": cpu,
            "decode_selfcheck": decode,
        }
        # on a line of its own: a process group's connection chatter on stdout
        # (gloo) may have left a partial line
        print("\n" + json.dumps(res), flush=True)
    enc.close()
    if dist:
        dist.destroy_process_group()
    if (vs_oracle and not vs_oracle["equal"]) or bitexact is False:
        log("bench.py: packets differ from the oracle / reference pin")
        sys.exit(3)


if __name__ == "__main__":
    main()
