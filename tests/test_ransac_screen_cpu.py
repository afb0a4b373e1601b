"""The RANSAC evaluation's fp32 screen bound, checked numerically on the CPU.

ransac_eval_kernel (stereo.vision_amd/csrc/kernels/ransac_batch.hip) screens every trial in fp32: per sample point
the term |rcp(d) * (cx*Ba + cy*Bb + Cc) - 1| with cx = x - cw_hi, cy = y - ch_hi, Ba = B a, Bb = B b,
Cc = fB c - cw_lo B a - ch_lo B b (fp64, rounded to fp32), summed per lane in fp32 (<= 10 terms a lane), the lanes'
sums in fp64; and the bound (sum of rcp(d) (|cx Ba| + |cy Bb| + |Cc|) + k) * 2^-18 on the difference to the
reference's fp64 sum of |X a + Y b + Z c - 1| (functions.py:275, the distance before the division by |abc|).
The kernel's note derives a 4x margin; this test replays the fp32 arithmetic in numpy (fma emulated in fp64, rcp
as the correctly rounded reciprocal, which v_rcp_f32 is within 1 ulp of) on random and adversarial planes and
checks the derived bound holds. Parity of the winner itself is pinned on the GPU (tests/test_gpu_ransac_batch.py).
"""
import numpy as np

F_PX, B_M, CW, CH = 399.9745178222656, 0.2090607502, 474.5, 262.0
f32 = np.float32


def fma32(a, b, c):
    # fp32 fused multiply-add: the product of two fp32 values is exact in fp64; one rounding of the sum to fp32
    # (the double rounding through fp64 differs from a true fma by at most an ulp in rare ties: inside the margin)
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(f32)


def screen(x, y, d, a, b, c):
    """fp32 screen of one trial as the kernel computes it: (sum over lanes of the lane's fp32 sum, bound)."""
    fB = F_PX * B_M
    cw_hi = f32(CW); cw_lo = f32(CW - float(cw_hi))
    ch_hi = f32(CH); ch_lo = f32(CH - float(ch_hi))
    Ba64, Bb64 = B_M * a, B_M * b
    Ba, Bb = f32(Ba64), f32(Bb64)
    Cc = f32(fB * c - float(cw_lo) * Ba64 - float(ch_lo) * Bb64)
    cx = (x.astype(f32) - cw_hi).astype(f32)
    cy = (y.astype(f32) - ch_hi).astype(f32)
    rr = (f32(1.0) / d.astype(f32)).astype(f32)
    inner = fma32(cy, np.full_like(cy, Bb), np.full_like(cy, Cc))
    s = fma32(cx, np.full_like(cx, Ba), inner)
    t = fma32(rr, s, np.full_like(s, f32(-1.0)))
    q = fma32(np.abs(cx), np.full_like(cx, abs(Ba)), fma32(np.abs(cy), np.full_like(cy, abs(Bb)), np.full_like(cy, abs(Cc))))
    # lanes: terms j, j + 64, ... summed in fp32 in that order, then the lanes in fp64
    k = x.size
    tot = 0.0
    bnd = 0.0
    for lane in range(64):
        ls = f32(0.0)
        lb = f32(0.0)
        for j in range(lane, k, 64):
            ls = f32(ls + np.abs(t[j]))
            lb = fma32(np.array([rr[j]]), np.array([q[j]]), np.array([lb]))[0]
        tot += float(ls)
        bnd += float(lb)
    return tot, (bnd + k) * 2.0 ** -18


def reference(x, y, d, a, b, c):
    """the reference's fp64 sum of |X a + Y b + Z c - 1| (functions.py:191-193, 275; the kernel's fp64 path uses
    numpy's rounding of the dot, immaterial at this precision)"""
    Z = (F_PX * B_M) / d
    X = ((x - CW) * Z) / F_PX
    Y = ((y - CH) * Z) / F_PX
    return float(np.abs(X * a + Y * b + Z * c - 1.0).sum())


def _trial(rng, k, plane):
    x = rng.integers(0, 512, k) * 2
    y = rng.integers(0, 272, k) * 2
    d = rng.integers(1, 256, k)
    return x.astype(np.float64), y.astype(np.float64), d.astype(np.float64), plane


def test_screen_bound_holds_on_random_and_adversarial_planes():
    rng = np.random.default_rng(7)
    planes = [(0.0, 2.86997918, 0.44487511)]   # the synthetic road plane (oracle.synthetic_plane)
    planes += [tuple(rng.normal(0, s, 3)) for s in (0.1, 1.0, 10.0, 1000.0) for _ in range(4)]
    # near-singular fits: huge coefficients that cancel (the sum's terms large, their sum small)
    planes += [(1e4, -1e4 * 0.5, 3.0), (-3e5, 1e5, 7e4), (1e-6, 1e-6, 1.0 / (F_PX * B_M) * 10)]
    worst = 0.0
    for plane in planes:
        for k in (1, 7, 600):
            x, y, d, (a, b, c) = _trial(rng, k, plane)
            e32, bound = screen(x, y, d, a, b, c)
            e64 = reference(x, y, d, a, b, c)
            err = abs(e32 - e64)
            assert err <= bound, (plane, k, e32, e64, bound)
            if bound > 0:
                worst = max(worst, err / bound)
    assert worst < 0.25, worst   # a worst-case derivation with a ~4x margin; random cases sit far below (~0.01)
