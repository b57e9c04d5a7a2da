"""The register-only pairwise sum of a constant run (wf_device.h pw_const_sum: spine + one
(Q(B_d), Q(B_d + 1)) pair per depth, no leaf table) restated line by line in Python and
checked against numpy's pairwise tree (the leaf-table walk the oracle follows,
numpy/_core/src/umath/loops_utils.h.src pairwise_sum) for every buffer length."""
import random

import numpy as np


def seqsum(v, k):
    r = 0.0
    for _ in range(k):
        r += v
    return r


def pairwise(n, v):
    """numpy pairwise_sum over n copies of v (n <= 8192)."""
    if n < 8:
        return seqsum(v, n)
    if n <= 128:
        res = 8.0 * seqsum(v, n >> 3)        # eight equal accumulators, tree = exact doublings
        for _ in range(n & 7):
            res += v
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return pairwise(n2, v) + pairwise(n - n2, v)


def pw_const_sum(n, v):
    """Line-by-line restatement of wf_device.h pw_const_sum."""
    a0, K, m, sel = n >> 4, 0, n, 0
    while m > 128:
        a = m >> 4
        sel |= (1 if a != (a0 >> K) else 0) << K
        m -= 8 * a
        K += 1
    Db, Dmax, xB, xC, need16 = 0, -1, 0, 0, False
    if K > 0:
        Db = max(0, a0.bit_length() - 4)
        Dmax = max(K - 1, Db)
        xB = a0 >> Db
        xC = a0 >> (Db + 1) if Dmax == Db + 1 else 0
        need16 = Db >= 1 and (a0 >> (Db - 1)) == 16
    mL = m if m < 8 else m >> 3
    imax = max(xB, mL, 16 if need16 else 0)
    t = sB = sC = sL = 0.0
    for i in range(1, imax + 1):
        t += v
        sB = t if i == xB else sB
        sC = t if i == xC else sC
        sL = t if i == mL else sL
    if m < 8:
        R = sL
    else:
        R = 8.0 * sL
        for _ in range(m & 7):
            R += v
    q0 = q1 = 0.0
    for d in range(Dmax, -1, -1):
        B = a0 >> d
        if d >= Db:
            sd = sB if d == Db else sC
            q0, q1 = 8.0 * sd, 8.0 * (sd + v)
        else:
            c0, c1 = q0, q1
            q0, q1 = (c0 + c1, c1 + c1) if B & 1 else (c0 + c0, c0 + c1)
            if B == 16:
                q0 = 8.0 * t
        if d < K:
            R = (q1 if (sel >> d) & 1 else q0) + R
    return R


def test_pw_const_sum_matches_pairwise_every_length():
    rng = random.Random(7)
    values = [rng.uniform(0.05, 1.0) for _ in range(3)] + [1.0 / 3.0, 0.987654321]
    for v in values:
        for n in range(1, 8192):
            assert pw_const_sum(n, v) == pairwise(n, v), (n, v)


def test_pairwise_model_is_numpy():
    rng = np.random.default_rng(3)
    for n in list(range(1, 300)) + [1000, 1031, 4103, 8191]:
        v = float(rng.uniform(0.1, 1.0))
        assert float(np.add.reduce(np.full(n, v))) == 0.0 + pairwise(n, v), n
