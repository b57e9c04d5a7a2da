"""The register-only pairwise sums of one-run segments (wf_device.h): pw_const_sum (a run
over the whole locus: spine + one (Q(B_d), Q(B_d + 1)) pair per depth, no leaf table) and
pw_run_sum (any run [lo, hi): the split node, a suffix and a prefix path, whole siblings
from the same pair chain, run_leaf at the path ends), restated line by line in Python and
checked against numpy's pairwise tree (numpy/_core/src/umath/loops_utils.h.src
pairwise_sum) -- for every buffer length, and on explicit arrays for partial runs."""
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


def pairwise_arr(a):
    n = len(a)
    if n < 8:
        r = 0.0
        for x in a: r += x
        return r
    if n <= 128:
        r = list(a[:8])
        i = 8
        m = n - (n % 8)
        while i < m:
            for j in range(8): r[j] += a[i + j]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res += a[i]; i += 1
        return res
    n2 = n // 2; n2 -= n2 % 8
    return pairwise_arr(a[:n2]) + pairwise_arr(a[n2:])


def run_leaf(lo, hi, v, st, ln):
    # device run_leaf restated: leaf [st, st+ln) over sites v on [lo, hi)
    m = ln >> 3; be = st + (m << 3)
    hi = max(hi, lo)
    res = 0.0
    def below(base, bound, m):
        d = bound - base
        return 0 if d <= 0 else min(m, (d + 7) >> 3)
    if m > 0:
        k = [below(st + c, hi, m) - below(st + c, lo, m) for c in range(8)]
        kmin = min(k)
        s0 = seqsum(v, kmin); s1 = s0 + v; s2 = s1 + v
        r = [s0 if kc == kmin else (s1 if kc == kmin + 1 else s2) for kc in k]
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
    for x in range(be, st + ln):
        res += v if (lo <= x < hi) else 0.0
    return res


def run_leaf_code(lo, hi, st, ln):
    """wf_device.h run_leaf_code: (kmin, 2 bits per accumulator | tail << 16 | (m > 0) << 20)"""
    m = ln >> 3; be = st + (m << 3)
    hi = max(hi, lo)
    def below(base, bound, m):
        d = bound - base
        return 0 if d <= 0 else min(m, (d + 7) >> 3)
    k = [below(st + c, hi, m) - below(st + c, lo, m) for c in range(8)]
    kmin = min([m] + k)
    code = 0
    for c in range(8):
        code |= min(k[c] - kmin, 2) << (2 * c)
    tail = max(0, min(st + ln, hi) - max(be, lo))
    return kmin, code | (tail << 16) | ((1 << 20) if m > 0 else 0)


def run_leaf_value(v, lc, s0):
    kmin, code = lc
    res = 0.0
    if (code >> 20) & 1:
        s1 = s0 + v; s2 = s1 + v
        r = [(s0, s1, s2)[(code >> (2 * c)) & 3] for c in range(8)]
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
    for _ in range((code >> 16) & 15):
        res += v
    return res


def pw_run_sum(n, lo, hi, v):
    """Line-by-line restatement of wf_device.h pw_run_sum (integer walks, one seqsum chain
    feeding the pair chain and the two boundary leaves, bitmask bookkeeping, one ascent)."""
    lo = max(lo, 0); hi = min(hi, n)
    if hi <= lo: return 0.0
    a0 = n >> 4; K = 0; m = n; sel = 0
    while m > 128:
        a = m >> 4
        sel |= (1 if a != (a0 >> K) else 0) << K
        m -= 8 * a; K += 1
    Db, Dmax, xB, xC, need16 = 0, -1, 0, 0, False
    if K > 0:
        Db = max(0, a0.bit_length() - 4); Dmax = max(K - 1, Db)
        xB = a0 >> Db; xC = (a0 >> (Db + 1)) if Dmax == Db + 1 else 0
        need16 = Db >= 1 and (a0 >> (Db - 1)) == 16
    # node = (s, size, kind(1 pair), cls, t)
    def child(s, size, kind, cls, t, right):
        if kind == 0:
            nl = 8 * (size >> 4)
            return (s + nl, size - nl, 0, 0, t + 1) if right else (s, nl, 1, (sel >> t) & 1, t + 1)
        x = size >> 3; xl = x >> 1; Bt = a0 >> t
        return (s + 8 * xl, 8 * (x - xl), 1, (x - xl) - Bt, t + 1) if right else (s, 8 * xl, 1, xl - Bt, t + 1)
    s, size, kind, cls, t = 0, n, 0, 0, 0
    mode = 0   # 0 two paths, 1 whole node, 2 one leaf
    while True:
        if lo <= s and hi >= s + size: mode = 1; break
        if size <= 128: mode = 2; break
        nl = 8 * (size >> 4) if kind == 0 else 8 * ((size >> 3) >> 1)
        if hi <= s + nl: s, size, kind, cls, t = child(s, size, kind, cls, t, False)
        elif lo >= s + nl: s, size, kind, cls, t = child(s, size, kind, cls, t, True)
        else: break
    ts = t
    W_t = t; W_kind = kind; W_cls = cls
    # paths: [term depth, term type (0 full spine, 1 full pair, 2 leaf), cls, ev, evk, evc, leaf]
    P = [[0, 0, 0, 0, 0, 0, None], [0, 0, 0, 0, 0, 0, None]]
    if mode == 0:
        for i, suffix in enumerate((True, False)):
            s2, sz2, k2, c2, t2 = child(s, size, kind, cls, t, not suffix)
            ev = evk = evc = 0
            while True:
                if (suffix and lo <= s2) or ((not suffix) and hi >= s2 + sz2):
                    P[i] = [t2, 0 if k2 == 0 else 1, c2, ev, evk, evc, None]; break
                if sz2 <= 128:
                    lc = run_leaf_code(lo, s2 + sz2, s2, sz2) if suffix else run_leaf_code(s2, hi, s2, sz2)
                    P[i] = [t2, 2, 0, ev, evk, evc, lc]; break
                L = child(s2, sz2, k2, c2, t2, False); R = child(s2, sz2, k2, c2, t2, True)
                if suffix:
                    if lo < R[0]:
                        ev |= 1 << (t2 + 1); evk |= (1 if R[2] == 0 else 0) << (t2 + 1); evc |= R[3] << (t2 + 1)
                        s2, sz2, k2, c2, t2 = L
                    else: s2, sz2, k2, c2, t2 = R
                else:
                    if hi > R[0]:
                        ev |= 1 << (t2 + 1); evc |= L[3] << (t2 + 1)
                        s2, sz2, k2, c2, t2 = R
                    else: s2, sz2, k2, c2, t2 = L
    elif mode == 2:
        P[0] = [0, 2, 0, 0, 0, 0, run_leaf_code(lo, hi, s, size)]
    k0 = P[0][6][0] if P[0][1] == 2 else 0
    k1 = P[1][6][0] if P[1][1] == 2 else 0
    mL = m if m < 8 else m >> 3
    imax = k0 if mode == 2 else max(xB, mL, 16 if need16 else 0, k0, k1)
    tt = 0.0; sB = sC = sL = s0a = s0b = 0.0
    for i in range(1, imax + 1):
        tt += v
        if i == xB: sB = tt
        if i == xC: sC = tt
        if i == mL: sL = tt
        if i == k0: s0a = tt
        if i == k1: s0b = tt
    lv = [0.0, 0.0]
    if P[0][1] == 2:
        lv[0] = run_leaf_value(v, P[0][6], s0a)
    if mode == 2: return lv[0]
    if P[1][1] == 2:
        lv[1] = run_leaf_value(v, P[1][6], s0b)
    if m < 8: Rv = sL
    else:
        Rv = 8.0 * sL
        for _ in range(m & 7): Rv += v
    q0 = q1 = 0.0
    acc = [0.0, 0.0]
    for d in range(Dmax, -2, -1):
        u = d + 1
        if d >= 0:
            B = a0 >> d
            if d >= Db:
                sd = sB if d == Db else sC
                q0, q1 = 8.0 * sd, 8.0 * (sd + v)
            else:
                c0, c1 = q0, q1
                q0, q1 = (c0 + c1, c1 + c1) if B & 1 else (c0 + c0, c0 + c1)
                if B == 16: q0 = 8.0 * tt
        # (Rv is R_u here)
        if mode == 1 and u == W_t:
            return Rv if W_kind == 0 else (q1 if W_cls else q0)
        if mode == 0:
            for i in (0, 1):
                tu, ty, tc, ev, evk, evc, _ = P[i]
                if u == tu:
                    acc[i] = lv[i] if ty == 2 else (Rv if ty == 0 else (q1 if tc else q0))
                if u <= tu and (ev >> u) & 1:
                    sib = Rv if (evk >> u) & 1 else (q1 if (evc >> u) & 1 else q0)
                    acc[i] = acc[i] + sib if i == 0 else sib + acc[i]
            if u == ts + 1:
                return acc[0] + acc[1]
        if 0 <= d < K:
            Rv = (q1 if (sel >> d) & 1 else q0) + Rv
    raise Exception("unreachable")


def test_pw_run_sum_matches_pairwise_on_arrays():
    rng = random.Random(11)
    lengths = list(range(1, 260)) + rng.sample(range(260, 8192), 250) + [1000, 1031, 2048, 4096,
                                                                          4103, 8190, 8191]
    for n in lengths:
        for trial in range(6):
            v = rng.uniform(0.05, 1.0)
            if trial == 0:
                lo, hi = 0, n
            elif trial == 1:
                lo, hi = rng.randrange(n), n
            elif trial == 2:
                lo, hi = 0, rng.randrange(1, n + 1)
            elif trial == 3:
                lo = rng.randrange(n)
                hi = min(n, lo + rng.randrange(1, 10))
            else:
                lo = rng.randrange(n)
                hi = rng.randrange(lo + 1, n + 1)
            a = [v if lo <= i < hi else 0.0 for i in range(n)]
            assert pw_run_sum(n, lo, hi, v) == pairwise_arr(a), (n, lo, hi, v)


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


def test_pw_run_sum_whole_run_equals_pw_const_sum():
    """The level-0 triage (wf_triage.hip) evaluates every one-run segment by pw_run_sum, whole
    runs included: over [0, n) it must equal pw_const_sum bit for bit at every buffer length."""
    rng = random.Random(5)
    for v in [rng.uniform(0.05, 1.0) for _ in range(2)] + [0.987654321]:
        for n in range(1, 8192):
            assert pw_run_sum(n, 0, n, v) == pw_const_sum(n, v), (n, v)
