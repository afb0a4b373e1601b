"""The SGBM walks' packed path step (csrc/kernels/sgbm.hip: pk_l / pk_commit, round 4) against OpenCV's 32-bit
step (oracle/sgbm_oracle.c, the formula of DESIGN §7.4), as integer algebra on the CPU.

The kernel computes both disparities of a lane with v_pk_* 16-bit operations: the terms of the min that can
exceed 32767 are saturated, q = delta - m and L = C - q wrap modulo 2^16, and the range error (an L below -32768)
is detected as sat16(L_stored - C) > 0. This emulates those operations with numpy int16 / int32 arithmetic on
random and extreme operands (stored L values, the previous step's min, the d +- 1 neighbours with MAX_COST at
the ends, costs C over the whole int16 range, 0 <= P1 <= P2 <= 15) and checks, element by element, that

  * q, the stored (int16-truncated) L and the lane's min equal the 32-bit step's whenever no L leaves int16;
  * the range flag is raised exactly when the 32-bit L is below -32768.

The GPU tests (tests/test_gpu_sgbm.py) check the kernels themselves bit for bit against the oracle; this pins
the algebra on operands (C near -32768) that synthetic images do not reach.
"""
import numpy as np

MAXC = 32767


def sat16(x):
    return np.clip(x, -32768, 32767)


def wrap16(x):
    return ((np.asarray(x, np.int64) + 32768) % 65536 - 32768).astype(np.int64)


def ref_step(p, lft, rgt, pmin, C, P1, P2):
    """OpenCV's step in 32-bit: (L untruncated, q = C - L)"""
    delta = pmin + P2
    m = np.minimum(np.minimum(p, delta), np.minimum(lft, rgt) + P1)
    L = C + m - delta
    return L, C - L


def packed_step(p, lft, rgt, pmin, C, P1, P2):
    """the kernel's v_pk_* arithmetic: (q, L stored, range flag)"""
    delta = pmin + P2
    ds = min(delta, MAXC)                       # (short)min(delta, kMaxCost)
    dw = wrap16(delta)                          # (short)delta
    n1 = sat16(np.minimum(lft, rgt) + P1)       # v_pk_min_i16, v_pk_add_i16 clamp
    m = np.minimum(np.minimum(p, ds), n1)       # two v_pk_min_i16
    q = wrap16(dw - m)                          # v_pk_sub (wrapping)
    L = wrap16(C - q)                           # v_pk_sub (wrapping)
    flag = sat16(L - C) > 0                     # v_pk_sub_i16 clamp, running v_pk_max_i16
    return q, L, flag


def draw(rng, n):
    """operands as one walk step sees them: stored L values >= pmin, C anywhere in int16 (extremes weighted)"""
    pmin = rng.choice(np.r_[rng.integers(-32768, 32768, 6), -32768, -32767, 32767, 32760, 0])
    hi = 32767
    p = rng.integers(pmin, hi + 1, n)
    lft = rng.integers(pmin, hi + 1, n)
    rgt = rng.integers(pmin, hi + 1, n)
    ends = rng.random(n) < 0.05                 # lane 0 / lane 63: the missing neighbour reads MAX_COST
    lft[ends] = MAXC
    rgt[rng.random(n) < 0.05] = MAXC
    C = rng.integers(-32768, 32768, n)
    low = rng.random(n) < 0.3                   # costs at the bottom of int16, where an L can leave it
    C[low] = rng.integers(-32768, -32768 + 40, low.sum())
    return int(pmin), p, lft, rgt, C


def test_packed_step_equals_the_32bit_step():
    rng = np.random.default_rng(20261017)
    seen_flag = seen_ok = 0
    for it in range(4000):
        P1 = int(rng.integers(0, 16))
        P2 = int(rng.integers(P1, 16))
        pmin, p, lft, rgt, C = draw(rng, 256)
        L_ref, q_ref = ref_step(p, lft, rgt, pmin, C, P1, P2)
        q, L, flag = packed_step(p, lft, rgt, pmin, C, P1, P2)
        out = L_ref < -32768
        assert np.array_equal(flag, out), (it, P1, P2, pmin)
        ok = ~out
        assert np.all((q_ref[ok] >= 0) & (q_ref[ok] <= P2))
        assert np.array_equal(q[ok], q_ref[ok]), (it, P1, P2, pmin)
        assert np.array_equal(L[ok], wrap16(L_ref[ok])), (it, P1, P2, pmin)
        if ok.all():   # the wave's min (the next step's pmin) from the stored pairs
            assert int(L.min()) == int(wrap16(L_ref.min()))
        seen_flag += int(out.sum())
        seen_ok += int(ok.sum())
    assert seen_flag > 1000 and seen_ok > 100000   # both outcomes exercised


def test_q_byte_packs_both_nibbles():
    # q_byte_pk: (q | q >> 12) & 0xFF with d0's q in bits 0-3 and d1's in bits 16-19
    for q0 in range(16):
        for q1 in range(16):
            q = q0 | (q1 << 16)
            assert (q | (q >> 12)) & 0xFF == q0 | (q1 << 4)


def test_right_view_key_order():
    """the row walk's right-view update as a minimum of (cost + 32768) << 16 | (0xFFFF - x): visiting pixels in
    decreasing x and keeping the first strictly smaller cost (OpenCV's disp2cost test) selects the same pixel"""
    rng = np.random.default_rng(7)
    for _ in range(2000):
        n = int(rng.integers(1, 40))
        xs = np.sort(rng.choice(2048, n, replace=False))[::-1]   # visiting order: decreasing x
        costs = rng.integers(-32768, 32767, n)                  # minS < MAX_COST (saturated pixels never update)
        costs[rng.random(n) < 0.3] = costs[0]                   # ties
        best_cost, best_x = MAXC, None
        for x, c in zip(xs, costs):
            if best_cost > c:
                best_cost, best_x = c, x
        keys = ((costs + 32768).astype(np.uint64) << 16) | (0xFFFF - xs).astype(np.uint64)
        k = int(keys.min())
        assert 0xFFFF - (k & 0xFFFF) == best_x and (k >> 16) - 32768 == best_cost
