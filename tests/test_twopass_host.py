"""Host-only check of sort_stt (ffv1enc.c:621-667), the pass-2 re-ordering of
the custom state-transition table, on pass-1 counts of 2^31 and more.

The reference swaps its 64-bit counters with FFSWAP(int, a, b), which is
{ int tmp = b; b = a; a = tmp; } (libavutil/common.h:99): b takes a whole, a
takes b truncated to 32 bits and sign-extended.  Once a count passes 2^31 (a
few hundred 4K frames of statistics) that truncation changes the later swap
decisions, the sorted table, the extradata and every pass-2 packet.  The
restatement below is written from the reference's text (its macros expand
size0 / sizeX into one left-to-right sum of eight products); the oracle's
sort_stt and the HIP library's host copy must both equal it.  No GPU.
"""
import ctypes
import math
import random

import numpy as np
import pytest

from oracle import oracle

M64 = (1 << 64) - 1


def _int32(v):
    """(int) of a uint64_t: the low 32 bits, two's complement."""
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


def sort_stt_ref(st, stt, buggy=False):
    """ffv1enc.c:621-667 with C semantics.  st: 256 x [c0, c1] uint64 as ints.
    buggy=True swaps in the opposite direction (the round-2 mistake)."""
    st = [list(x) for x in st]
    stt = list(stt)

    def cost_terms(o, n):
        return [float(st[o][0]) * -math.log2((256 - n) / 256.0),
                float(st[o][1]) * -math.log2(n / 256.0)]

    def size(i, a, i2, b):
        terms = cost_terms(i, a) + cost_terms(256 - i, 256 - a) + cost_terms(i2, b) + \
            cost_terms(256 - i2, 256 - b)
        s = terms[0]
        for t in terms[1:]:
            s = s + t
        return s

    def ffswap_int(x, y, k):  # FFSWAP(int, st[x][k], st[y][k])
        if buggy:
            t = _int32(st[x][k])
            st[x][k] = st[y][k]
            st[y][k] = t & M64
        else:
            t = _int32(st[y][k])
            st[y][k] = st[x][k]
            st[x][k] = t & M64

    changed = True
    while changed:
        changed = False
        for i in range(12, 244):
            for i2 in range(i + 1, min(245, i + 4)):
                size0 = size(i, i, i2, i2)
                sizex = size(i, i2, i2, i)
                if size0 - sizex > size0 * 1e-14 and i != 128 and i2 != 128:
                    stt[i], stt[i2] = stt[i2], stt[i]
                    ffswap_int(i, i2, 0)
                    ffswap_int(i, i2, 1)
                    if i != 256 - i2:
                        stt[256 - i], stt[256 - i2] = stt[256 - i2], stt[256 - i]
                        ffswap_int(256 - i, 256 - i2, 0)
                        ffswap_int(256 - i, 256 - i2, 1)
                    for j in range(1, 256):
                        if stt[j] == i:
                            stt[j] = i2
                        elif stt[j] == i2:
                            stt[j] = i
                        if i != 256 - i2:
                            if stt[256 - j] == 256 - i:
                                stt[256 - j] = 256 - i2
                            elif stt[256 - j] == 256 - i2:
                                stt[256 - j] = 256 - i
                    changed = True
    return stt


def _table():
    """A custom-table shape: a one-decision moves the state up by a step that
    shrinks towards the ends (what ver2_state looks like, ffv1enc.c:120-137)."""
    t = [0] * 256
    for i in range(1, 256):
        t[i] = min(255, i + max(1, (256 - i) // 12))
    return t


def _counts(seed, big):
    rnd = random.Random(seed)
    st = []
    for i in range(256):
        # counts shaped like real statistics: ones more likely at high states
        tot = rnd.randrange(1 << 20, 1 << 34) if big else rnd.randrange(1 << 8, 1 << 24)
        p1 = min(0.999, max(0.001, i / 256.0 + rnd.uniform(-0.08, 0.08)))
        c1 = int(tot * p1)
        st.append([tot - c1, c1])
    return st


def _via_oracle(st, stt):
    a = np.array([v for pair in st for v in pair], np.uint64)
    t = np.array(stt, np.uint8)
    oracle.lib().ffv1o_sort_stt.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint8)]
    oracle.lib().ffv1o_sort_stt(a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                t.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    return t.tolist()


def _via_hip(st, stt):
    from ffv1hip import _paths
    L = ctypes.CDLL(_paths.hip_lib())
    f = L.ffv1hip_internal_sort_stt
    f.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint8)]
    a = np.array([v for pair in st for v in pair], np.uint64)
    t = np.array(stt, np.uint8)
    f(a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), t.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    return t.tolist()


@pytest.mark.parametrize("seed,big", [(1, False), (2, False), (3, True), (4, True), (5, True)])
def test_sort_stt_matches_reference_semantics(seed, big):
    st, stt = _counts(seed, big), _table()
    want = sort_stt_ref(st, stt)
    assert _via_oracle(st, stt) == want
    assert _via_hip(st, stt) == want


def test_large_counts_exercise_the_truncation():
    """Counts past 2^31 make the swap direction visible: the round-2
    (reversed) swap gives a different table on these inputs."""
    differs = 0
    for seed in (3, 4, 5):
        st, stt = _counts(seed, True), _table()
        differs += sort_stt_ref(st, stt) != sort_stt_ref(st, stt, buggy=True)
    assert differs >= 1
