/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.
 *
 * Plain-C, scalar, fp64 restatement of the thien/stereo.vision hot path, used
 * exclusively as the CHECKER by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg. The product path (stereo.vision_amd/svx + libsvx.so) never
 * links, loads or calls this file.
 *
 * Parity: pinned against tests/golden/ — fixtures produced by running the
 * reference's own Python functions (tests/golden/make_golden.py, container
 * only) — and against the SURVEY.md §8c digests.
 *
 * Every function cites the reference line it restates (paths relative to the
 * reference repo root). Build: oracle/Makefile → oracle/_build/libsvx_oracle.so
 * with -O2 -ffp-contract=off so no operation is fused behind our back.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { double f, B, cw, ch; } svo_camera;

/* ------------------------------------------------------------------------
 * Synthetic frame generator. Counter based: the value of a
 * pixel depends only on (frame id, y, x), so host and device agree.
 * --------------------------------------------------------------------- */
static inline uint64_t svo_mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline int64_t floordiv(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) q -= 1;
    return q;
}

void svo_synth_frame(int64_t frame_id, int H, int W, uint8_t* disp, uint8_t* bgr) {
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            uint64_t idx = ((uint64_t)frame_id * (uint64_t)H + (uint64_t)y) * (uint64_t)W + (uint64_t)x;
            uint64_t r = svo_mix64(idx + 0x5EED000000000001ull);
            uint64_t r2 = svo_mix64(idx + 0x5EED000000000002ull);
            int64_t t = floordiv(3 * (int64_t)(y - 200), 5) + (int64_t)((r >> 8) & 7) - 3;
            if (t < 0) t = 0;
            if (t > 254) t = 254;
            int d = (int)(t & ~1ll);
            if ((r & 0xFF) < 38) d = 0;
            disp[(size_t)y * W + x] = (uint8_t)d;
            if (bgr) {
                uint8_t* px = bgr + ((size_t)y * W + x) * 3;
                if (y >= 262) {
                    px[0] = (uint8_t)(110 + (r2 & 3));
                    px[1] = (uint8_t)(100 + ((r2 >> 2) & 3));
                    px[2] = (uint8_t)(90 + ((r2 >> 4) & 3));
                } else {
                    px[0] = (uint8_t)(r2 & 255);
                    px[1] = (uint8_t)((r2 >> 8) & 255);
                    px[2] = (uint8_t)((r2 >> 16) & 255);
                }
            }
        }
    }
}

/* ------------------------------------------------------------------------
 * a1: projectDisparityTo3d — functions.py:178-198.
 * Grid: y in range(0, H-1, step), x in range(0, W-1, step) (:185-186; the
 * reference hard-codes step 2). d == 0 skipped (:188). fp64:
 *   Z = (f*B)/d ; X = ((x-cw)*Z)/f ; Y = ((y-ch)*Z)/f      (:191-193)
 * rgb row = (bgr[..,2], bgr[..,1], bgr[..,0])             (:195)
 * Returns N; xyz is N x 3, rgb (optional) N x 3, src (optional) N x 2 (y, x).
 * --------------------------------------------------------------------- */
int64_t svo_project(const uint8_t* disp, int H, int W, int64_t ld_disp,
                    const uint8_t* bgr, int64_t ld_bgr, int step, const svo_camera* cam,
                    double* xyz, uint8_t* rgb, int32_t* src) {
    const double f = cam->f, B = cam->B;
    const double fB = f * B;
    int64_t n = 0;
    for (int y = 0; y < H - 1; y += step) {
        for (int x = 0; x < W - 1; x += step) {
            const uint8_t d = disp[(int64_t)y * ld_disp + x];
            if (d == 0) continue;
            const double Z = fB / (double)d;
            const double X = (((double)x - cam->cw) * Z) / f;
            const double Y = (((double)y - cam->ch) * Z) / f;
            xyz[3 * n + 0] = X;
            xyz[3 * n + 1] = Y;
            xyz[3 * n + 2] = Z;
            if (rgb && bgr) {
                const uint8_t* px = bgr + (int64_t)y * ld_bgr + 3 * (int64_t)x;
                rgb[3 * n + 0] = px[2];
                rgb[3 * n + 1] = px[1];
                rgb[3 * n + 2] = px[0];
            }
            if (src) { src[2 * n] = y; src[2 * n + 1] = x; }
            ++n;
        }
    }
    return n;
}

/* Dense variant: every grid point, (0,0,0) where d == 0. Output planes are
 * Hg x pitch (row-major); columns >= Wg are written as 0. Used to check the
 * dense K1 output of the batched API. */
void svo_project_dense(const uint8_t* disp, int H, int W, int step, const svo_camera* cam,
                       int pitch, double* X, double* Y, double* Z) {
    const double f = cam->f, fB = cam->f * cam->B;
    const int Hg = (H - 1 + step - 1) / step, Wg = (W - 1 + step - 1) / step;
    for (int gy = 0; gy < Hg; ++gy) {
        for (int gx = 0; gx < pitch; ++gx) {
            double vx = 0, vy = 0, vz = 0;
            if (gx < Wg) {
                const int y = gy * step, x = gx * step;
                const uint8_t d = disp[(int64_t)y * W + x];
                if (d) {
                    vz = fB / (double)d;
                    vx = (((double)x - cam->cw) * vz) / f;
                    vy = (((double)y - cam->ch) * vz) / f;
                }
            }
            X[(int64_t)gy * pitch + gx] = vx;
            Y[(int64_t)gy * pitch + gx] = vy;
            Z[(int64_t)gy * pitch + gx] = vz;
        }
    }
}

/* Checker of one frame of the device's dense fp32 planes (Hg rows at a stride of pitch)
 * against the fp64 values of svo_project_dense on the synthetic frame
 * `frame_id` (generated here): returns the number of grid points whose zero
 * pattern differs or whose relative error exceeds rtol, and the worst
 * relative error in *max_rel. Used by the GPU tests for EVERY frame of the
 * headline batch (the device's own digest kernel is not the checker there). */
int64_t svo_check_dense_f32(int64_t frame_id, int H, int W, int step, const svo_camera* cam, int pitch,
                            const float* X, const float* Y, const float* Z, double rtol, double* max_rel) {
    uint8_t* disp = (uint8_t*)malloc((size_t)H * W);
    if (!disp) return -1;
    svo_synth_frame(frame_id, H, W, disp, NULL);
    const double f = cam->f, fB = cam->f * cam->B;
    const int Hg = (H - 1 + step - 1) / step, Wg = (W - 1 + step - 1) / step;
    int64_t bad = 0;
    double worst = 0.0;
    for (int gy = 0; gy < Hg; ++gy) {
        for (int gx = 0; gx < Wg; ++gx) {   /* the reference's grid; pad columns up to pitch are not points */
            double v[3] = {0, 0, 0};
            {
                const int y = gy * step, x = gx * step;
                const uint8_t d = disp[(int64_t)y * W + x];
                if (d) {
                    v[2] = fB / (double)d;
                    v[0] = (((double)x - cam->cw) * v[2]) / f;
                    v[1] = (((double)y - cam->ch) * v[2]) / f;
                }
            }
            const int64_t o = (int64_t)gy * pitch + gx;
            const float g[3] = {X[o], Y[o], Z[o]};
            for (int k = 0; k < 3; ++k) {
                if ((v[k] == 0.0) != (g[k] == 0.0f)) {
                    ++bad;
                    continue;
                }
                if (v[k] == 0.0) continue;
                const double rel = fabs((double)g[k] - v[k]) / fabs(v[k]);
                if (rel > worst) worst = rel;
                if (!(rel <= rtol)) ++bad;
            }
        }
    }
    free(disp);
    *max_rel = worst;
    return bad;
}

/* ------------------------------------------------------------------------
 * a7: project3DPointsTo2DImagePoints — functions.py:201-209 (fp64):
 *   x = ((X*f)/Z) + cw ; y = ((Y*f)/Z) + ch
 * --------------------------------------------------------------------- */
void svo_backproject(const double* xyz, int64_t n, int64_t ld, const svo_camera* cam, double* xy) {
    for (int64_t i = 0; i < n; ++i) {
        const double X = xyz[i * ld], Y = xyz[i * ld + 1], Z = xyz[i * ld + 2];
        xy[2 * i] = ((X * cam->f) / Z) + cam->cw;
        xy[2 * i + 1] = ((Y * cam->f) / Z) + cam->ch;
    }
}

/* a8: np.array(planePoints, np.int32) — stereovision.py:112: C truncation. */
static inline int32_t trunc_i32(double v) { return (int32_t)v; }

/* ------------------------------------------------------------------------
 * a2: calculatePointErrors — functions.py:300-312.
 *   nrm = sqrt(a*a + b*b + c*c)         (:307, left-to-right)
 *   dist = |(P . abc) - 1| / nrm         (:310)
 * The dot goes through BLAS in the reference; the order below is the one
 * OpenBLAS produces bit-for-bit (checked by tests against the golden dist
 * values). Only the keep mask (a3) is a parity claim.
 * --------------------------------------------------------------------- */
static inline double plane_norm(const double* abc) {
    return sqrt(abc[0] * abc[0] + abc[1] * abc[1] + abc[2] * abc[2]);
}
static inline double plane_dist(double X, double Y, double Z, const double* abc, double nrm) {
    const double dot = fma(Z, abc[2], fma(X, abc[0], Y * abc[1]));
    return fabs((dot - 1.0) / nrm);
}
void svo_point_errors(const double* xyz, int64_t n, int64_t ld, const double* abc, double* dist) {
    const double nrm = plane_norm(abc);
    for (int64_t i = 0; i < n; ++i)
        dist[i] = plane_dist(xyz[i * ld], xyz[i * ld + 1], xyz[i * ld + 2], abc, nrm);
}

/* ------------------------------------------------------------------------
 * RANSAC's plane and error with numpy's rounding — functions.py:267-275, :289.
 *   abc = np.dot(np.linalg.inv([P1; P2; P3]), np.ones([3, 1]))
 * numpy's inv is LAPACK dgesv(A, I) of its bundled OpenBLAS (0.3.29 here):
 * dgetf2 (left-looking LU: pivot = the first largest |a|, the column below the
 * pivot scaled by the pivot's reciprocal, update products rounded before they
 * are subtracted, column 2's two-term update as one fma chain), then dgetrs
 * (the permuted identity through trsm: unit-lower forward with fused
 * multiply-subtracts; upper backward with the diagonal applied as a multiply by
 * its reciprocal, row 2's update of rows 0 and 1 a rounded product); the dot
 * with ones adds each row left to right. Returns 1 when a pivot is exactly 0
 * (dgesv info > 0: numpy raises LinAlgError). The device's rb_solve_record is
 * the same sequence. Pinned to numpy by tests/test_ransac_cpu.py.
 * --------------------------------------------------------------------- */
int svo_plane_lapack(const double* P1, const double* P2, const double* P3, double* abc) {
    double m[3][3] = {{P1[0], P1[1], P1[2]}, {P2[0], P2[1], P2[2]}, {P3[0], P3[1], P3[2]}};
    int perm[3] = {0, 1, 2};
    int piv = 0;
    for (int i = 1; i < 3; ++i)
        if (fabs(m[i][0]) > fabs(m[piv][0])) piv = i;
    if (piv) {
        for (int c = 0; c < 3; ++c) { double t = m[0][c]; m[0][c] = m[piv][c]; m[piv][c] = t; }
        int t = perm[0]; perm[0] = perm[piv]; perm[piv] = t;
    }
    const double u00 = m[0][0];
    double l10 = m[1][0], l20 = m[2][0];
    if (u00 != 0.0) { const double r = 1.0 / u00; l10 *= r; l20 *= r; }
    double b1 = m[1][1] - l10 * m[0][1], b2 = m[2][1] - l20 * m[0][1];
    double c1 = m[1][2], c2 = m[2][2];
    if (fabs(b2) > fabs(b1)) {
        double t = b1; b1 = b2; b2 = t;
        t = l10; l10 = l20; l20 = t;
        t = c1; c1 = c2; c2 = t;
        int q = perm[1]; perm[1] = perm[2]; perm[2] = q;
    }
    const double u11 = b1;
    double l21 = b2;
    if (u11 != 0.0) l21 *= 1.0 / u11;
    const double u01 = m[0][1], u02 = m[0][2];
    const double u12 = c1 - l10 * u02;
    const double u22 = c2 - fma(l21, u12, l20 * u02);
    const double i00 = 1.0 / u00, i11 = 1.0 / u11, i22 = 1.0 / u22;
    for (int c = 0; c < 3; ++c) {
        double x0 = perm[0] == c, x1 = perm[1] == c, x2 = perm[2] == c;
        x1 = fma(-x0, l10, x1);
        x2 = fma(-x0, l20, x2);
        x2 = fma(-x1, l21, x2);
        x2 = x2 * i22;
        x0 = x0 - u02 * x2;
        x1 = x1 - u12 * x2;
        x1 = x1 * i11;
        x0 = fma(-x1, u01, x0);
        x0 = x0 * i00;
        if (c == 0) { abc[0] = x0; abc[1] = x1; abc[2] = x2; }
        else { abc[0] += x0; abc[1] += x1; abc[2] += x2; }
    }
    return u00 == 0.0 || u11 == 0.0 || u22 == 0.0;
}

/* numpy's pairwise summation (numpy/_core/src/umath/loops_utils.h.src), as
 * add.reduce runs it from the initial 0.0. */
static double np_pairwise(const double* a, int64_t n) {
    if (n < 8) {
        double r = 0.0;
        for (int64_t i = 0; i < n; ++i) r += a[i];
        return r;
    }
    if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise(a, n2) + np_pairwise(a + n2, n - n2);
}

/* error = np.mean(abs((np.dot(T, abc) - 1) / d)), d = math.sqrt(a a + b b + c c)
 * (functions.py:269-275, :289) over the n rows of T (stride ld): the gemv's dot as
 * plane_dist's fma chain (one row is a (1, 3) x (3, 1) product, which numpy sends
 * to ddot instead: x a first, then y b and z c fused in order), then numpy's
 * pairwise sum / n. */
double svo_ransac_err(const double* T, int64_t n, int64_t ld, const double* abc) {
    const double nrm = plane_norm(abc);
    double* t = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) t[i] = plane_dist(T[i * ld], T[i * ld + 1], T[i * ld + 2], abc, nrm);
    if (n == 1) t[0] = fabs((fma(T[2], abc[2], fma(T[1], abc[1], T[0] * abc[0])) - 1.0) / nrm);
    const double s = np_pairwise(t, n);
    free(t);
    return s / (double)n;
}

/* ------------------------------------------------------------------------
 * a4: BGRtoHSVHue + colorsys.rgb_to_hsv — functions.py:73-78 (inputs are
 * numpy uint8 scalars). Key str(round(h,3)) <-> integer bin rint(h*1000):
 *   rc,gc,bc = (mx-c)/(mx-mn)   (fp64 true division of exact integers)
 *   h = bc-gc | (2+rc)-bc | (4+gc)-rc   ; h = (h/6) mod 1 (numpy floor-mod)
 *   bin = rint(h*1000) (numpy round = multiply, rint half-even, divide)
 * Grey (mx == mn) returns hue 0.0 -> bin 0.
 * --------------------------------------------------------------------- */
int svo_hue_bin(int r, int g, int b) {
    int mx = r, mn = r;
    if (g > mx) mx = g;
    if (b > mx) mx = b;
    if (g < mn) mn = g;
    if (b < mn) mn = b;
    if (mx == mn) return 0;
    const double rng = (double)(mx - mn);
    const double rc = (double)(mx - r) / rng;
    const double gc = (double)(mx - g) / rng;
    const double bc = (double)(mx - b) / rng;
    double h;
    if (r == mx) h = bc - gc;
    else if (g == mx) h = (2.0 + rc) - bc;
    else h = (4.0 + gc) - rc;
    h = h / 6.0;
    double m = fmod(h, 1.0);
    if (m != 0.0) {
        if (m < 0.0) m += 1.0;
    } else {
        m = 0.0;
    }
    return (int)nearbyint(m * 1000.0);
}

/* Full 2^24 LUT, index R<<16 | G<<8 | B (SURVEY.md §8c digest). */
void svo_hue_lut(int16_t* lut) {
    for (int r = 0; r < 256; ++r)
        for (int g = 0; g < 256; ++g)
            for (int b = 0; b < 256; ++b)
                lut[(r << 16) | (g << 8) | b] = (int16_t)svo_hue_bin(r, g, b);
}

/* ------------------------------------------------------------------------
 * Back-projection delta tables: the int32 of the fp64 round trip
 * x -> X -> x' depends only on (x, d) (resp. (y, d)), so
 *   dx[d][x] = trunc(((X(x,d)*f)/Z(d)) + cw) - x     in {-1, 0}
 * d = 0 column is 0. Layout [d][coord] (256 x W, 256 x H).
 * --------------------------------------------------------------------- */
void svo_delta_tables(int H, int W, const svo_camera* cam, int8_t* dx, int8_t* dy) {
    const double f = cam->f, fB = cam->f * cam->B;
    for (int d = 0; d < 256; ++d) {
        const double Z = d ? fB / (double)d : 0.0;
        for (int x = 0; x < W; ++x) {
            int8_t v = 0;
            if (d) {
                const double X = (((double)x - cam->cw) * Z) / f;
                v = (int8_t)(trunc_i32(((X * f) / Z) + cam->cw) - x);
            }
            dx[d * W + x] = v;
        }
        for (int y = 0; y < H; ++y) {
            int8_t v = 0;
            if (d) {
                const double Y = (((double)y - cam->ch) * Z) / f;
                v = (int8_t)(trunc_i32(((Y * f) / Z) + cam->ch) - y);
            }
            dy[d * H + y] = v;
        }
    }
}

/* ------------------------------------------------------------------------
 * The whole per-frame chain (stereovision.py:84,97-113):
 *   project (a1) -> errors (a2) -> keep dist < point_thr (a3, order kept)
 *   -> hue histogram of kept (a5) -> keep hist[bin] > hist_thr (a6)
 *   -> back-project (a7) -> int32 trunc (a8)
 * Outputs (caller sized to the grid count):
 *   counts[3]   = N_valid, N_kept, N_kept2
 *   hist[1024]  = per-bin count over the plane-kept points (bins 0..999)
 *   xyz2 (N_kept2 x 3, fp64), pts (N_kept2 x 2 int32), src2 (N_kept2 x 2: y,x)
 * --------------------------------------------------------------------- */
int svo_pipeline_frame(const uint8_t* disp, const uint8_t* bgr, int H, int W, int step,
                       const svo_camera* cam, const double* abc, double point_thr, int hist_thr,
                       int64_t* counts, uint32_t* hist, double* xyz2, int32_t* pts, int32_t* src2,
                       double* scratch_xyz, uint8_t* scratch_rgb, int32_t* scratch_src,
                       uint8_t* scratch_keep, int16_t* scratch_bin) {
    const int64_t n = svo_project(disp, H, W, W, bgr, (int64_t)W * 3, step, cam,
                                  scratch_xyz, scratch_rgb, scratch_src);
    const double nrm = plane_norm(abc);
    int64_t n1 = 0;
    memset(hist, 0, 1024 * sizeof(uint32_t));
    for (int64_t i = 0; i < n; ++i) {
        const double dd = plane_dist(scratch_xyz[3 * i], scratch_xyz[3 * i + 1],
                                     scratch_xyz[3 * i + 2], abc, nrm);
        scratch_keep[i] = dd < point_thr;
        if (scratch_keep[i]) {
            const int bin = svo_hue_bin(scratch_rgb[3 * i], scratch_rgb[3 * i + 1], scratch_rgb[3 * i + 2]);
            scratch_bin[i] = (int16_t)bin;
            hist[bin] += 1;
            ++n1;
        }
    }
    int64_t n2 = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (!scratch_keep[i]) continue;
        if (!((int64_t)hist[scratch_bin[i]] > (int64_t)hist_thr)) continue;
        const double X = scratch_xyz[3 * i], Y = scratch_xyz[3 * i + 1], Z = scratch_xyz[3 * i + 2];
        if (xyz2) { xyz2[3 * n2] = X; xyz2[3 * n2 + 1] = Y; xyz2[3 * n2 + 2] = Z; }
        pts[2 * n2] = trunc_i32(((X * cam->f) / Z) + cam->cw);
        pts[2 * n2 + 1] = trunc_i32(((Y * cam->f) / Z) + cam->ch);
        if (src2) { src2[2 * n2] = scratch_src[2 * i]; src2[2 * n2 + 1] = scratch_src[2 * i + 1]; }
        ++n2;
    }
    counts[0] = n;
    counts[1] = n1;
    counts[2] = n2;
    return 0;
}

/* ------------------------------------------------------------------------
 * Per-frame digests: the checker's summary of one full-size synthetic frame.
 * The device computes the same summary of its own outputs (digest kernels,
 * sv_batch_digest), so EVERY frame of a batch is checked at full size without
 * moving the outputs off the GPU. Definitions (the spec shared with
 * stereo.vision_amd/csrc/kernels/digest.hip; sums mod 2^64):
 *   disp_hash = sum_j mix64(j << 32 | word_j), word_j = little-endian u32 j of
 *               the frame's disparity (H*W % 4 == 0)
 *   hist_hash = sum_{k<1000} mix64((k + 65536) << 32 | hist[k])
 *   pts_hash  = sum_i mix64(A_i ^ mix64(i)) over the surviving points in
 *               order, A_i = (x | y << 12 | d << 24) << 32 | (px & 0xFFFF) |
 *               (py & 0xFFFF) << 16: source pixel (x, y), its disparity d and
 *               its int32 back-projection (px, py) (functions.py:201-209,
 *               stereovision.py:112)
 * counts = svo_pipeline_frame's (N_valid, N_kept, N_kept2).
 * --------------------------------------------------------------------- */
uint64_t svo_digest_mix(uint64_t z) { return svo_mix64(z); }

/* The same digest of a given frame (disparity H x W, BGR H x W x 3): frames
 * that are not the generator's, e.g. the pre-pass-cleaned ones of the
 * per-frame-plane loop (tests/golden/make_plane_digests.py). */
int svo_digest_frame(const uint8_t* disp, const uint8_t* bgr, int H, int W, int step, const svo_camera* cam,
                     const double* abc, double point_thr, int hist_thr, int64_t* counts, uint64_t* hashes) {
    const int Hg = (H - 1 + step - 1) / step, Wg = (W - 1 + step - 1) / step;
    const size_t cap = (size_t)(Hg > 0 && Wg > 0 ? Hg * Wg : 1);
    const size_t px = (size_t)H * W;
    int32_t* pts = malloc(cap * 2 * sizeof(int32_t));
    int32_t* src2 = malloc(cap * 2 * sizeof(int32_t));
    double* s_xyz = malloc(cap * 3 * sizeof(double));
    uint8_t* s_rgb = malloc(cap * 3);
    int32_t* s_src = malloc(cap * 2 * sizeof(int32_t));
    uint8_t* s_keep = malloc(cap);
    int16_t* s_bin = malloc(cap * sizeof(int16_t));
    uint32_t hist[1024];
    int rc = -1;
    if (!pts || !src2 || !s_xyz || !s_rgb || !s_src || !s_keep || !s_bin || (px % 4) || W > 4096 || H > 4096)
        goto out;
    svo_pipeline_frame(disp, bgr, H, W, step, cam, abc, point_thr, hist_thr, counts, hist, NULL, pts, src2,
                       s_xyz, s_rgb, s_src, s_keep, s_bin);
    uint64_t hd = 0, hh = 0, hp = 0;
    for (size_t j = 0; j < px / 4; ++j) {
        uint32_t w = (uint32_t)disp[4 * j] | ((uint32_t)disp[4 * j + 1] << 8) | ((uint32_t)disp[4 * j + 2] << 16) |
                     ((uint32_t)disp[4 * j + 3] << 24);
        hd += svo_mix64(((uint64_t)j << 32) | w);
    }
    for (uint64_t k = 0; k < 1000; ++k) hh += svo_mix64(((k + 65536) << 32) | hist[k]);
    for (int64_t i = 0; i < counts[2]; ++i) {
        const uint32_t y = (uint32_t)src2[2 * i], x = (uint32_t)src2[2 * i + 1];
        const uint32_t d = disp[(size_t)y * W + x];
        const uint64_t a = ((uint64_t)(x | (y << 12) | (d << 24)) << 32) |
                           (uint64_t)(((uint32_t)pts[2 * i] & 0xFFFFu) | (((uint32_t)pts[2 * i + 1] & 0xFFFFu) << 16));
        hp += svo_mix64(a ^ svo_mix64((uint64_t)i));
    }
    hashes[0] = hd;
    hashes[1] = hh;
    hashes[2] = hp;
    rc = 0;
out:
    free(pts); free(src2);
    free(s_xyz); free(s_rgb); free(s_src); free(s_keep); free(s_bin);
    return rc;
}

int svo_frame_digest(int64_t frame_id, int H, int W, int step, const svo_camera* cam, const double* abc,
                     double point_thr, int hist_thr, int64_t* counts, uint64_t* hashes) {
    const size_t px = (size_t)H * W;
    uint8_t* disp = malloc(px ? px : 1);
    uint8_t* bgr = malloc(px ? px * 3 : 1);
    int rc = -1;
    if (disp && bgr) {
        svo_synth_frame(frame_id, H, W, disp, bgr);
        rc = svo_digest_frame(disp, bgr, H, W, step, cam, abc, point_thr, hist_thr, counts, hashes);
    }
    free(disp);
    free(bgr);
    return rc;
}
