"""Test helper: a vectorised numpy restatement of StereoSGBM (MODE_SGBM).

Independent of oracle/sgbm_oracle.c in structure: the cost volume is built
whole, every aggregation direction is its own recurrence (dirs 1-3 row by
row over all columns, dirs 0/4 column by column over all rows), as the GPU
kernels organise it but written from the published formulas. Used by
tests/test_sgbm_cpu.py to cross-check the C oracle's loop on small images.
"""
import numpy as np

MAX_COST = 32767


def _t16(a):
    return ((np.asarray(a, np.int64) + 32768) % 65536) - 32768


def _sat16(a):
    return np.clip(a, -32768, 32767)


def _channels(img, ftzero):
    v = img.astype(np.int64)
    up = np.vstack([v[:1], v[:-1]])
    dn = np.vstack([v[1:], v[-1:]])
    g = np.zeros_like(v)
    g[:, 1:-1] = (v[:, 2:] - v[:, :-2]) * 2 + up[:, 2:] - up[:, :-2] + dn[:, 2:] - dn[:, :-2]
    pref = np.clip(g, -ftzero, ftzero) + ftzero
    raw = v.copy()
    pref[:, 0] = pref[:, -1] = raw[:, 0] = raw[:, -1] = ftzero
    out = []
    for c in (pref, raw):
        left = (c + np.concatenate([c[:, :1], c[:, :-1]], axis=1)) // 2
        right = (c + np.concatenate([c[:, 1:], c[:, -1:]], axis=1)) // 2
        out.append((c, np.minimum(np.minimum(left, right), c), np.maximum(np.maximum(left, right), c)))
    return out


def cost_volume(L, R, D=128, ftzero=15, SW2=10, SH2=10):
    H, W = L.shape
    w1 = W - D
    cl, cr = _channels(L, ftzero), _channels(R, ftzero)
    xs = np.arange(D, W)
    pix = np.zeros((H, w1, D), np.int64)
    for ch, shift in ((0, 0), (1, 2)):
        u, u0, u1 = (a[:, xs][:, :, None] for a in cl[ch])
        xr = xs[:, None] - np.arange(D)[None, :]
        v, v0, v1 = (a[:, xr] for a in cr[ch])
        c0 = np.maximum(np.maximum(0, u - v1), v0 - u)
        c1 = np.maximum(np.maximum(0, v - u1), u0 - v)
        pix += np.minimum(c0, c1) >> shift
    idx = np.clip(np.arange(w1)[:, None] + np.arange(-SW2, SW2 + 1)[None, :], 0, w1 - 1)
    hsum = pix[:, idx, :].sum(axis=2)
    C = np.zeros((H, w1, D), np.int64)
    cur = sum(hsum[min(k, H - 1)] * (SH2 + 1 if k == 0 else 1) for k in range(SH2 + 1))
    C[0] = cur
    for y in range(1, H):
        if y + SH2 < H:
            cur = cur.copy()
            cur[1:] += hsum[y + SH2, 1:] - hsum[max(y - SH2 - 1, 0), 1:]
        C[y] = cur
    return _t16(C)


def _step(c, prev, pmin, P1, P2):
    delta = (pmin + P2)[:, None]
    n = prev.shape[0]
    big = np.full((n, 1), MAX_COST)
    left = np.concatenate([big, prev[:, :-1]], axis=1)
    right = np.concatenate([prev[:, 1:], big], axis=1)
    m = np.minimum(np.minimum(prev, delta), np.minimum(left, right) + P1)
    Lv = c + m - delta
    return Lv, _t16(Lv), _t16(Lv.min(axis=1))


def sgbm(L, R, block=21, P1=0, P2=0, disp12_max_diff=0, prefilter_cap=0, uniqueness=0):
    H, W = L.shape
    D = 128
    SW2 = block // 2
    P1 = P1 if P1 > 0 else 2
    P2 = max(P2 if P2 > 0 else 5, P1 + 1)
    ftzero = max(prefilter_cap, 15) | 1
    d12 = disp12_max_diff if disp12_max_diff > 0 else 1
    C = cost_volume(L, R, D, ftzero, SW2, SW2)
    w1 = W - D
    Ls = []
    # dirs 1, 2, 3: row by row over all columns (predecessor column x-1, x, x+1 of the previous row)
    for sh in (1, 0, -1):
        out = np.zeros((H, w1, D), np.int64)
        prev = np.zeros((w1, D), np.int64)
        pmin = np.zeros(w1, np.int64)
        for y in range(H):
            if sh == 1:
                p = np.vstack([np.zeros((1, D), np.int64), prev[:-1]])
                pm = np.concatenate([[0], pmin[:-1]])
            elif sh == -1:
                p = np.vstack([prev[1:], np.zeros((1, D), np.int64)])
                pm = np.concatenate([pmin[1:], [0]])
            else:
                p, pm = prev, pmin
            if y == 0:
                p, pm = np.zeros_like(p), np.zeros_like(pm)
            Lv, prev, pmin = _step(C[y], p, pm, P1, P2)
            out[y] = Lv
        Ls.append(out)
    # dirs 0 and 4: column by column over all rows
    for order in (range(w1), range(w1 - 1, -1, -1)):
        out = np.zeros((H, w1, D), np.int64)
        prev = np.zeros((H, D), np.int64)
        pmin = np.zeros(H, np.int64)
        for x in order:
            Lv, prev, pmin = _step(C[:, x], prev, pmin, P1, P2)
            out[:, x] = Lv
        Ls.append(out)
    S = _sat16(_sat16(Ls[0] + Ls[1] + Ls[2] + Ls[3]) + Ls[4])
    disp = np.full((H, W), -16, np.int64)
    for y in range(H):
        d1 = np.full(W, -16, np.int64)
        d2 = np.full(W, -16, np.int64)
        d2c = np.full(W, MAX_COST, np.int64)
        for x in range(w1 - 1, -1, -1):
            s = S[y, x]
            best = int(np.argmin(s))
            minS = int(s[best])
            if minS == MAX_COST:
                continue        # strict "<" from MAX_COST never fires: bestDisp = -1 -> INVALID
            if uniqueness > 0 and np.any((s * (100 - uniqueness) < minS * 100) & (np.abs(best - np.arange(D)) > 1)):
                continue
            x2 = x + D - best
            if d2c[x2] > minS:
                d2c[x2] = minS
                d2[x2] = best
            if 0 < best < D - 1:
                den = max(int(s[best - 1]) + int(s[best + 1]) - 2 * minS, 1)
                num = (int(s[best - 1]) - int(s[best + 1])) * 16 + den
                q = abs(num) // (2 * den)
                dd = best * 16 + (q if num >= 0 else -q)     # C division truncates toward zero
            else:
                dd = best * 16
            d1[x + D] = dd
        for x in range(D, W):
            v = d1[x]
            if v == -16:
                continue
            _d, d_ = v >> 4, (v + 15) >> 4
            _x, x_ = x - _d, x - d_
            if 0 <= _x < W and d2[_x] >= 0 and abs(d2[_x] - _d) > d12 and 0 <= x_ < W and d2[x_] >= 0 and \
                    abs(d2[x_] - d_) > d12:
                d1[x] = -16
        disp[y] = d1
    return disp.astype(np.int16)
