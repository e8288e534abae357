"""The decision-stream coder's segment join (ffv1_range / ffv1_dseg /
ffv1_dfix, csrc/ffv1_kernels.hip), restated in Python and checked against
the serial range coder (rangecoder.h:85-102 put_rac with renorm_encoder's
shifts, rangecoder.c:104-116 terminate): the values of low at every shift
(the digits ffv1_sink turns into bytes) are the same.  Host-only: this pins
the method (range alone per stream, segments coded from checkpoints with
low = 0, the carry-in fixed in each segment's first two digits), including
segments with no or one shift (near-certain decisions), on random decision
streams.  The GPU parity tests pin the kernels themselves.
"""
import random

import pytest


def serial_digits(states, bits):
    low, rng, digs = 0, 0xFF00, []

    def put(s, b):
        nonlocal low, rng
        r1 = (rng * s) >> 8
        if b:
            low += rng - r1
            rng = r1
        else:
            rng -= r1
        while rng < 0x100:
            digs.append(low)
            low = (low & 0xFF) << 8
            rng <<= 8

    for s, b in zip(states, bits):
        put(s, b)
    put(129, 0)  # the slice trailer decision, then ff_rac_terminate
    low += 0xFF
    for _ in range(2):
        digs.append(low)
        low = (low & 0xFF) << 8
    return digs


def segmented_digits(states, bits, K):
    n = len(states)
    # pass 1 (ffv1_range): range alone, a checkpoint every K decisions
    ck, rng, J = [], 0xFF00, 0
    for i in range(n):
        if i % K == 0:
            ck.append((rng, J))
        r1 = (rng * states[i]) >> 8
        rng = r1 if bits[i] else rng - r1
        if rng < 0x100:
            rng <<= 8
            J += 1
    # pass 2 (ffv1_dseg): every segment from its checkpoint with low = 0
    out, rec = {}, []
    for si, (r, j0) in enumerate(ck):
        low, rng, k = 0, r, j0
        seq = list(zip(states[si * K:(si + 1) * K], bits[si * K:(si + 1) * K]))
        if si == len(ck) - 1:
            seq.append((129, 0))
        for s, b in seq:
            r1 = (rng * s) >> 8
            if b:
                low += rng - r1
                rng = r1
            else:
                rng -= r1
            if rng < 0x100:
                out[k] = low
                k += 1
                low = (low & 0xFF) << 8
                rng <<= 8
        if si == len(ck) - 1:
            low += 0xFF
            for _ in range(2):
                out[k] = low
                k += 1
                low = (low & 0xFF) << 8
        rec.append((low, k - j0))
    # pass 3 (ffv1_dfix): join
    L, total = 0, 0
    for si, (r, j) in enumerate(ck):
        e, nn = rec[si]
        total = j + nn
        if nn == 0:
            L += e
            continue
        v = out[j]
        x = L + v
        out[j] = x
        delta = ((x & 0xFF) - (v & 0xFF)) << 8
        if nn == 1:
            L = e + delta
        else:
            out[j + 1] += delta
            L = e
    return [out[i] for i in range(total)]


@pytest.mark.parametrize("seed", range(40))
def test_segments_join_to_the_serial_digits(seed):
    rnd = random.Random(seed)
    n = rnd.randint(1, 2500)
    K = rnd.choice([32, 64, 96, 256, 1024])
    p1 = rnd.random()
    kind = rnd.choice(["mixed", "certain", "uncertain"])
    states = []
    for _ in range(n):
        if kind == "certain":  # long runs without a shift
            states.append(rnd.randint(245, 255) if rnd.random() < 0.9 else rnd.randint(1, 255))
        elif kind == "uncertain":
            states.append(rnd.randint(100, 156))
        else:
            states.append(rnd.choice([rnd.randint(1, 255), rnd.randint(240, 255), rnd.randint(1, 20)]))
    bits = [1 if rnd.random() < p1 else 0 for _ in range(n)]
    if kind == "certain":
        bits = [1 if s > 128 else 0 for s in states]
    assert segmented_digits(states, bits, K) == serial_digits(states, bits)
