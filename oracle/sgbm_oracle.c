/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.
 *
 * Plain-C restatement of the disparity stage upstream of the hot path
 * (functions.py:81-128):
 *
 *   preProcessImages / gammaChange (functions.py:61-67, :81-87)  — numpy table, see oracle/sgbm.py
 *   greyscale (functions.py:89-97)  = cv2.cvtColor(BGR2GRAY) + cv2.equalizeHist
 *   disparity (functions.py:104-128) = StereoSGBM(0, 128, 21).compute
 *                                        (computeDisparitySGBM + medianBlur 3)
 *                                      + cv2.filterSpeckles(d, 0, 4000, 123)
 *                                      + cv2.threshold(TOZERO at 0) + /16 -> u8
 *                                      + optional crop + x(256/128) -> u8
 *
 * The reference delegates all of it to OpenCV, which is a third-party
 * dependency absent from /root/reference and from this image (no cv2 module,
 * no OpenCV sources). The reference pins no version (no requirements file;
 * readme.md asks for "opencv"), so this file restates the algorithm OpenCV
 * 4.x publishes for these calls (modules/calib3d/src/stereosgbm.cpp:
 * StereoSGBMImpl::compute, computeDisparitySGBM with mode MODE_SGBM,
 * calcPixelCostBT, filterSpecklesImpl; imgproc/median_blur medianBlur_SortNet;
 * modules/imgproc: RGB2Gray<uchar> fixed point, equalizeHist), structure for
 * structure: the same row-by-row loop, the same cyclic horizontal-sum buffer,
 * the same int16 (CostType) truncations and saturations, the same MAX_COST
 * sentinels and border rules. PARITY UNPINNED: the reference holds no
 * disparity fixtures (its dataset is absent) and cv2 cannot run here.
 * tests/test_sgbm_cv2.py compares this file with cv2 wherever cv2 imports.
 *
 * The GPU kernels (stereo.vision_amd/csrc/kernels/sgbm.hip) reorganise the
 * computation completely (per-path waves instead of one row loop); this file
 * keeps OpenCV's loop so that agreement between the two checks the
 * reorganisation.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef int16_t cost_t;                /* OpenCV's CostType (short)  */
#define MAX_COST 32767                 /* SHRT_MAX                    */
#define DISP_SHIFT 4                   /* StereoMatcher::DISP_SHIFT   */
#define DISP_SCALE (1 << DISP_SHIFT)

typedef struct {
    int min_disp, num_disp, block, P1, P2, disp12_max_diff, prefilter_cap, uniqueness;
} svo_sgbm_params;

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline cost_t sat16(int v) { return (cost_t)(v < -32768 ? -32768 : v > 32767 ? 32767 : v); }

/* ------------------------------------------------------------------------
 * cv2.cvtColor(img, COLOR_BGR2GRAY) for 8-bit: fixed point with 14 fraction
 * bits, Y = (B*1868 + G*9617 + R*4899 + 2^13) >> 14 (R2Y/G2Y/B2Y of
 * color.hpp, yuv_shift = 14); then cv2.equalizeHist: hist, first non-empty
 * bin i0, scale = 255.f / (total - hist[i0]) in fp32, lut[i0] = 0,
 * lut[i] = saturate_cast<uchar>((float)cumsum * scale) (round half to even).
 * A constant image maps to its own value (functions.py:89-97).
 * --------------------------------------------------------------------- */
void svo_grey_equalize(const uint8_t* bgr, int H, int W, uint8_t* out) {
    const int64_t n = (int64_t)H * W;
    int64_t hist[256] = {0};
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t* p = bgr + 3 * i;
        int y = (p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + (1 << 13)) >> 14;
        out[i] = (uint8_t)y;
        hist[y]++;
    }
    if (n == 0) return;
    int i = 0;
    while (!hist[i]) ++i;
    if (hist[i] == n) {
        memset(out, i, (size_t)n);
        return;
    }
    uint8_t lut[256] = {0};
    float scale = 255.f / (float)(n - hist[i]);
    int64_t sum = 0;
    for (lut[i++] = 0; i < 256; ++i) {
        sum += hist[i];
        float v = (float)sum * scale;
        /* cvRound: nearest, ties to even (lrintf under the default mode) */
        float r = __builtin_rintf(v);
        int iv = (int)r;
        lut[i] = (uint8_t)(iv < 0 ? 0 : iv > 255 ? 255 : iv);
    }
    for (int64_t k = 0; k < n; ++k) out[k] = lut[out[k]];
}

/* ------------------------------------------------------------------------
 * calcPixelCostBT for one row y: the Birchfield-Tomasi dissimilarity of the
 * x-derivative prefilter (Sobel-like, clipped to [-ftzero, ftzero] and
 * offset by ftzero) and of the raw intensity (>> 2), summed. Columns 0 and
 * W-1 of BOTH channels are set to ftzero (tab[0]), as OpenCV does.
 * cost[(x - minX1) * D + (d - minD)], x in [minX1, maxX1), d in [minD, maxD).
 * --------------------------------------------------------------------- */
static void row_channels(const uint8_t* img, int H, int W, int y, int ftzero, uint8_t* pref, uint8_t* raw) {
    const uint8_t* r = img + (size_t)y * W;
    const uint8_t* up = img + (size_t)(y > 0 ? y - 1 : y) * W;
    const uint8_t* dn = img + (size_t)(y < H - 1 ? y + 1 : y) * W;
    for (int x = 1; x < W - 1; ++x) {
        int v = (r[x + 1] - r[x - 1]) * 2 + up[x + 1] - up[x - 1] + dn[x + 1] - dn[x - 1];
        pref[x] = (uint8_t)(imin(imax(v, -ftzero), ftzero) + ftzero);
        raw[x] = r[x];
    }
    pref[0] = pref[W - 1] = raw[0] = raw[W - 1] = (uint8_t)ftzero;
}

static void half_minmax(const uint8_t* v, int W, uint8_t* lo, uint8_t* hi) {
    for (int x = 0; x < W; ++x) {
        int c = v[x];
        int l = x > 0 ? (c + v[x - 1]) / 2 : c;
        int r = x < W - 1 ? (c + v[x + 1]) / 2 : c;
        lo[x] = (uint8_t)imin(imin(l, r), c);
        hi[x] = (uint8_t)imax(imax(l, r), c);
    }
}

typedef struct {
    uint8_t *ch[2][2], *lo[2][2], *hi[2][2]; /* [image][channel] */
} bt_rows;

static void pixel_cost_bt(const uint8_t* L, const uint8_t* R, int H, int W, int y, int minD, int maxD, int ftzero,
                          bt_rows* t, cost_t* cost) {
    const int D = maxD - minD, minX1 = imax(maxD, 0), maxX1 = W + imin(minD, 0);
    row_channels(L, H, W, y, ftzero, t->ch[0][0], t->ch[0][1]);
    row_channels(R, H, W, y, ftzero, t->ch[1][0], t->ch[1][1]);
    for (int i = 0; i < 2; ++i)
        for (int c = 0; c < 2; ++c) half_minmax(t->ch[i][c], W, t->lo[i][c], t->hi[i][c]);
    for (int x = minX1; x < maxX1; ++x) {
        cost_t* cx = cost + (size_t)(x - minX1) * D;
        for (int d = minD; d < maxD; ++d) {
            int xr = x - d, acc = 0;
            for (int c = 0; c < 2; ++c) {
                int u = t->ch[0][c][x], u0 = t->lo[0][c][x], u1 = t->hi[0][c][x];
                int v = t->ch[1][c][xr], v0 = t->lo[1][c][xr], v1 = t->hi[1][c][xr];
                int c0 = imax(imax(0, u - v1), v0 - u);
                int c1 = imax(imax(0, v - u1), u0 - v);
                acc += imin(c0, c1) >> (c == 0 ? 0 : 2);
            }
            cx[d - minD] = (cost_t)acc;
        }
    }
}

/* ------------------------------------------------------------------------
 * computeDisparitySGBM, MODE_SGBM (single pass, 5 directions: the 4 of the
 * forward row loop — (-1,0), (-1,-1), (0,-1), (+1,-1) — and the (+1,0) pass
 * of the final right-to-left loop). OpenCV's defaults for zero parameters:
 * P1 -> 2, P2 -> max(5, P1 + 1), preFilterCap -> max(cap, 15) | 1,
 * disp12MaxDiff <= 0 -> 1, uniquenessRatio < 0 -> 10; speckleWindowSize 0
 * (no internal speckle filter). disp: H x W int16, scaled by 16.
 * Returns 0, or -1 for an unsupported geometry (D % 16, tiny width).
 *
 * Behaviour restated literally, including:
 *  - C (the block-summed cost) is int16 and wraps; for rows y > 0 it is
 *    updated only while y + SH2 < H, and never for the first pixel column of
 *    the cost domain (OpenCV's update loop starts at x = D);
 *  - a path start (outside the image) has L = 0 for every d and min L = 0;
 *  - S = sat16(sat16(L0 + L1 + L2 + L3) + L4), the L values untruncated;
 *  - subpixel: d*16 + ((S[d-1] - S[d+1])*16 + den) / (2 den), C division;
 *  - left-right check against disp2 filled in decreasing x, first minimum
 *    kept (strict >).
 * --------------------------------------------------------------------- */
int svo_sgbm(const uint8_t* img1, const uint8_t* img2, int H, int W, const svo_sgbm_params* prm, int16_t* disp1) {
    const int minD = prm->min_disp, maxD = minD + prm->num_disp;
    const int SW = prm->block > 0 ? prm->block : 5;
    const int ftzero = imax(prm->prefilter_cap, 15) | 1;
    const int uniq = prm->uniqueness >= 0 ? prm->uniqueness : 10;
    const int d12 = prm->disp12_max_diff > 0 ? prm->disp12_max_diff : 1;
    const int P1 = prm->P1 > 0 ? prm->P1 : 2;
    const int P2 = imax(prm->P2 > 0 ? prm->P2 : 5, P1 + 1);
    const int minX1 = imax(maxD, 0), maxX1 = W + imin(minD, 0);
    const int D = maxD - minD, width1 = maxX1 - minX1;
    const int INVALID = (minD - 1) * DISP_SCALE;
    const int SW2 = SW / 2, SH2 = SW / 2;
    if (minX1 >= maxX1) {
        for (int64_t i = 0; i < (int64_t)H * W; ++i) disp1[i] = (int16_t)INVALID;
        return 0;
    }
    if (D % 16 != 0 || width1 <= SW2) return -1;

    const int NR2 = 4, NLR = 2;
    const size_t rowc = (size_t)width1 * D;
    const int nhsum = SH2 * 2 + 2;
    cost_t* pixDiff = calloc(rowc, sizeof(cost_t));
    cost_t* hsumBuf = calloc(rowc * nhsum, sizeof(cost_t));
    cost_t* C = calloc(rowc, sizeof(cost_t));
    cost_t* S = calloc(rowc, sizeof(cost_t));
    /* Lr[k]: (width1 + 2) cells (x = -1 .. width1) x NR2 directions x (D + 2)
     * (d = -1 .. D, the ends holding the MAX_COST sentinels) */
    const int LD = D + 2;
    const size_t lrcell = (size_t)NR2 * LD;
    cost_t* LrBuf[NLR];
    cost_t* minLrBuf[NLR];
    for (int k = 0; k < NLR; ++k) {
        LrBuf[k] = calloc((width1 + 2) * lrcell, sizeof(cost_t));
        minLrBuf[k] = calloc((size_t)(width1 + 2) * NR2, sizeof(cost_t));
    }
    /* one slot of slack: with every S saturated bestDisp stays -1 and x2 = x + minX1 + 1 can be W
     * (OpenCV reads past its row there too; a short cost can never exceed minS = MAX_COST, so it
     * never writes) */
    int16_t* disp2 = malloc(sizeof(int16_t) * (W + 1));
    cost_t* disp2cost = malloc(sizeof(cost_t) * (W + 1));
    bt_rows t;
    uint8_t* rows = malloc((size_t)W * 12);
    for (int i = 0, k = 0; i < 2; ++i)
        for (int c = 0; c < 2; ++c, k += 3) {
            t.ch[i][c] = rows + (size_t)W * k;
            t.lo[i][c] = rows + (size_t)W * (k + 1);
            t.hi[i][c] = rows + (size_t)W * (k + 2);
        }
    if (!pixDiff || !hsumBuf || !C || !S || !LrBuf[0] || !LrBuf[1] || !minLrBuf[0] || !minLrBuf[1] || !disp2 ||
        !disp2cost || !rows)
        return -2;

/* Lr(k, x, r, d): x in [-1, width1], d in [-1, D] */
#define LR(k, x, r, d) LrBuf[k][((size_t)((x) + 1) * NR2 + (r)) * LD + ((d) + 1)]
#define MINLR(k, x, r) minLrBuf[k][(size_t)((x) + 1) * NR2 + (r)]
    int cur = 0, prv = 1; /* Lr[0] / Lr[1] of OpenCV (swapped after each row) */

    for (int y = 0; y < H; ++y) {
        int16_t* d1row = disp1 + (size_t)y * W;
        /* ---- C for row y (pass 1 of computeDisparitySGBM) ---- */
        int dy1 = y == 0 ? 0 : y + SH2, dy2 = y == 0 ? SH2 : dy1;
        for (int k = dy1; k <= dy2; ++k) {
            cost_t* hsumAdd = hsumBuf + (size_t)(imin(k, H - 1) % nhsum) * rowc;
            if (k < H) {
                pixel_cost_bt(img1, img2, H, W, k, minD, maxD, ftzero, &t, pixDiff);
                for (int d = 0; d < D; ++d) hsumAdd[d] = 0;
                for (int x = 0; x <= SW2; ++x) {
                    int scale = x == 0 ? SW2 + 1 : 1;
                    for (int d = 0; d < D; ++d)
                        hsumAdd[d] = (cost_t)(hsumAdd[d] + pixDiff[(size_t)x * D + d] * scale);
                }
                const cost_t* hsumSub = hsumBuf + (size_t)(imax(y - SH2 - 1, 0) % nhsum) * rowc;
                for (int x = 1; x < width1; ++x) {
                    const cost_t* pixAdd = pixDiff + (size_t)imin(x + SW2, width1 - 1) * D;
                    const cost_t* pixSub = pixDiff + (size_t)imax(x - SW2 - 1, 0) * D;
                    for (int d = 0; d < D; ++d) {
                        int hv = hsumAdd[(size_t)x * D + d] =
                            (cost_t)(hsumAdd[(size_t)(x - 1) * D + d] + pixAdd[d] - pixSub[d]);
                        if (y > 0) C[(size_t)x * D + d] = (cost_t)(C[(size_t)x * D + d] + hv - hsumSub[(size_t)x * D + d]);
                    }
                }
            }
            if (y == 0) {
                int scale = k == 0 ? SH2 + 1 : 1;
                for (size_t i = 0; i < rowc; ++i) C[i] = (cost_t)(C[i] + hsumAdd[i] * scale);
            }
        }
        memset(S, 0, rowc * sizeof(cost_t));

        /* clear the left and right borders of the current Lr / minLr */
        for (int r = 0; r < NR2; ++r) {
            for (int d = -1; d <= D; ++d) LR(cur, -1, r, d) = LR(cur, width1, r, d) = 0;
            MINLR(cur, -1, r) = MINLR(cur, width1, r) = 0;
        }

        /* ---- forward loop: directions 0..3 ---- */
        for (int x = 0; x < width1; ++x) {
            const int px[4] = {x - 1, x - 1, x, x + 1}; /* predecessor column per direction  */
            const int pk[4] = {cur, prv, prv, prv};     /* predecessor row buffer per direction */
            const cost_t* Cp = C + (size_t)x * D;
            cost_t* Sp = S + (size_t)x * D;
            int delta[4], minL[4];
            for (int r = 0; r < 4; ++r) {
                delta[r] = MINLR(pk[r], px[r], r) + P2;
                LR(pk[r], px[r], r, -1) = LR(pk[r], px[r], r, D) = MAX_COST;
                minL[r] = MAX_COST;
            }
            for (int d = 0; d < D; ++d) {
                int Cpd = Cp[d], sum = 0;
                for (int r = 0; r < 4; ++r) {
                    int a = LR(pk[r], px[r], r, d);
                    int b = LR(pk[r], px[r], r, d - 1) + P1;
                    int c = LR(pk[r], px[r], r, d + 1) + P1;
                    int L = Cpd + imin(a, imin(b, imin(c, delta[r]))) - delta[r];
                    LR(cur, x, r, d) = (cost_t)L;
                    minL[r] = imin(minL[r], L);
                    sum += L;
                }
                Sp[d] = sat16(Sp[d] + sum);
            }
            for (int r = 0; r < 4; ++r) MINLR(cur, x, r) = (cost_t)minL[r];
        }

        /* ---- final loop: direction (+1, 0), selection, disp2 ---- */
        for (int x = 0; x <= W; ++x) {
            if (x < W) d1row[x] = (int16_t)INVALID;
            disp2[x] = (int16_t)INVALID;
            disp2cost[x] = MAX_COST;
        }
        for (int x = width1 - 1; x >= 0; --x) {
            cost_t* Sp = S + (size_t)x * D;
            const cost_t* Cp = C + (size_t)x * D;
            int minS = MAX_COST, bestDisp = -1, minL0 = MAX_COST;
            int delta0 = MINLR(cur, x + 1, 0) + P2;
            LR(cur, x + 1, 0, -1) = LR(cur, x + 1, 0, D) = MAX_COST;
            for (int d = 0; d < D; ++d) {
                int L0 = Cp[d] + imin(LR(cur, x + 1, 0, d),
                                      imin(LR(cur, x + 1, 0, d - 1) + P1, imin(LR(cur, x + 1, 0, d + 1) + P1, delta0))) -
                         delta0;
                LR(cur, x, 0, d) = (cost_t)L0;
                minL0 = imin(minL0, L0);
                int Sval = Sp[d] = sat16(Sp[d] + L0);
                if (Sval < minS) {
                    minS = Sval;
                    bestDisp = d;
                }
            }
            MINLR(cur, x, 0) = (cost_t)minL0;

            int d;
            for (d = 0; d < D; ++d)
                if (Sp[d] * (100 - uniq) < minS * 100 && abs(bestDisp - d) > 1) break;
            if (d < D) continue;
            d = bestDisp;
            int x2 = x + minX1 - d - minD;
            if (disp2cost[x2] > minS) {
                disp2cost[x2] = (cost_t)minS;
                disp2[x2] = (int16_t)(d + minD);
            }
            if (0 < d && d < D - 1) {
                int denom2 = imax(Sp[d - 1] + Sp[d + 1] - 2 * Sp[d], 1);
                d = d * DISP_SCALE + ((Sp[d - 1] - Sp[d + 1]) * DISP_SCALE + denom2) / (denom2 * 2);
            } else {
                d *= DISP_SCALE;
            }
            d1row[x + minX1] = (int16_t)(d + minD * DISP_SCALE);
        }
        /* left-right consistency */
        for (int x = minX1; x < maxX1; ++x) {
            int dd = d1row[x];
            if (dd == INVALID) continue;
            int _d = dd >> DISP_SHIFT, d_ = (dd + DISP_SCALE - 1) >> DISP_SHIFT;
            int _x = x - _d, x_ = x - d_;
            if (0 <= _x && _x < W && disp2[_x] >= minD && abs(disp2[_x] - _d) > d12 && 0 <= x_ && x_ < W &&
                disp2[x_] >= minD && abs(disp2[x_] - d_) > d12)
                d1row[x] = (int16_t)INVALID;
        }
        cur ^= 1;
        prv ^= 1;
    }
#undef LR
#undef MINLR
    free(pixDiff);
    free(hsumBuf);
    free(C);
    free(S);
    for (int k = 0; k < NLR; ++k) {
        free(LrBuf[k]);
        free(minLrBuf[k]);
    }
    free(disp2);
    free(disp2cost);
    free(rows);
    return 0;
}

/* ------------------------------------------------------------------------
 * cv2.medianBlur(disp, disp, 3) on the int16 disparity, the step
 * StereoSGBM::compute runs right after computeDisparitySGBM (OpenCV 2.4's
 * StereoSGBM::operator(), 3.x and 4.x StereoSGBMImpl::compute) and before its
 * internal speckle filter (off here: speckleWindowSize 0). OpenCV's 3 x 3
 * sorting network (medianBlur_SortNet) yields the exact median of the 9
 * values; the border replicates (rows max(y-1, 0) / min(y+1, H-1), columns
 * likewise); a 1-row or 1-column image takes the median of 3 along its length.
 * In-place calls work on a copy (cv::medianBlur copies src when dst aliases it).
 * --------------------------------------------------------------------- */
static int med3i(int a, int b, int c) { return imax(imin(a, b), imin(imax(a, b), c)); }

void svo_median3_s16(const int16_t* src, int H, int W, int16_t* dst) {
    if (H <= 0 || W <= 0) return;
    if (H == 1 || W == 1) {
        const int n = H * W;
        for (int i = 0; i < n; ++i)
            dst[i] = (int16_t)med3i(src[i > 0 ? i - 1 : 0], src[i], src[i < n - 1 ? i + 1 : n - 1]);
        return;
    }
    for (int y = 0; y < H; ++y) {
        const int16_t* r[3] = {src + (size_t)imax(y - 1, 0) * W, src + (size_t)y * W, src + (size_t)imin(y + 1, H - 1) * W};
        for (int x = 0; x < W; ++x) {
            const int xs[3] = {imax(x - 1, 0), x, imin(x + 1, W - 1)};
            int v[9], k = 0;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) v[k++] = r[i][xs[j]];
            /* insertion sort of 9: the 5th smallest is the median */
            for (int i = 1; i < 9; ++i) {
                int t = v[i], j = i - 1;
                while (j >= 0 && v[j] > t) {
                    v[j + 1] = v[j];
                    --j;
                }
                v[j + 1] = t;
            }
            dst[(size_t)y * W + x] = (int16_t)v[4];
        }
    }
}

/* StereoSGBM::compute (MODE_SGBM, speckleWindowSize 0) = computeDisparitySGBM + medianBlur 3 */
int svo_sgbm_compute(const uint8_t* img1, const uint8_t* img2, int H, int W, const svo_sgbm_params* prm,
                     int16_t* disp1) {
    int16_t* raw = malloc(sizeof(int16_t) * (size_t)(H * W > 0 ? H * W : 1));
    if (!raw) return -2;
    int rc = svo_sgbm(img1, img2, H, W, prm, raw);
    if (rc == 0) svo_median3_s16(raw, H, W, disp1);
    free(raw);
    return rc;
}

/* ------------------------------------------------------------------------
 * cv2.filterSpeckles(img, newVal, maxSpeckleSize, maxDiff) on int16, in
 * place (filterSpecklesImpl<short>): 4-connected regions of pixels != newVal
 * whose neighbours differ by <= maxDiff; a region of <= maxSpeckleSize pixels
 * is set to newVal. Raster scan + depth-first flood fill, as OpenCV.
 * --------------------------------------------------------------------- */
int svo_filter_speckles(int16_t* img, int H, int W, int newVal, int maxSpeckleSize, int maxDiff) {
    const int64_t n = (int64_t)H * W;
    int32_t* labels = calloc((size_t)n, sizeof(int32_t));
    int32_t* stack = malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    uint8_t* rtype = calloc((size_t)n + 1, 1);
    if (!labels || !stack || !rtype) return -2;
    int32_t cur = 0;
    for (int i = 0; i < H; ++i) {
        for (int j = 0; j < W; ++j) {
            int64_t p0 = (int64_t)i * W + j;
            if (img[p0] == newVal) continue;
            if (labels[p0]) {
                if (rtype[labels[p0]]) img[p0] = (int16_t)newVal;
                continue;
            }
            int32_t sp = 0;
            int64_t count = 0;
            labels[p0] = ++cur;
            stack[sp++] = (int32_t)p0;
            while (sp > 0) {
                int64_t p = stack[--sp];
                ++count;
                int y = (int)(p / W), x = (int)(p % W);
                int dp = img[p];
                const int64_t nb[4] = {y < H - 1 ? p + W : -1, y > 0 ? p - W : -1, x < W - 1 ? p + 1 : -1,
                                       x > 0 ? p - 1 : -1};
                for (int k = 0; k < 4; ++k) {
                    int64_t q = nb[k];
                    if (q < 0 || labels[q] || img[q] == newVal || abs(dp - img[q]) > maxDiff) continue;
                    labels[q] = cur;
                    stack[sp++] = (int32_t)q;
                }
            }
            if (count <= maxSpeckleSize) {
                rtype[cur] = 1;
                img[p0] = (int16_t)newVal;
            } else {
                rtype[cur] = 0;
            }
        }
    }
    free(labels);
    free(stack);
    free(rtype);
    return 0;
}

/* ------------------------------------------------------------------------
 * The tail of functions.py:104-128 after filterSpeckles:
 * threshold(d, 0, max_disparity*16, THRESH_TOZERO) -> (d / 16.).astype(u8)
 * -> optional crop [0:390, 135:W] -> (x * (256. / max_disparity)).astype(u8).
 * out: rows x cols with rows = crop ? min(390, H) : H, cols = crop ? W - 135 : W.
 * --------------------------------------------------------------------- */
void svo_disparity_scale(const int16_t* d16, int H, int W, int max_disparity, int crop, uint8_t* out) {
    const int r0 = 0, c0 = crop ? 135 : 0;
    const int rows = crop ? imin(390, H) : H, cols = crop ? imax(W - 135, 0) : W;
    const double s = 256. / max_disparity;
    for (int y = 0; y < rows; ++y)
        for (int x = 0; x < cols; ++x) {
            int v = d16[(size_t)(y + r0) * W + x + c0];
            if (v < 0) v = 0;
            uint8_t q = (uint8_t)((double)v / 16.);
            out[(size_t)y * cols + x] = (uint8_t)((double)q * s);
        }
}

/* functions.py:104-128 disparity(grayL, grayR, max_disparity, crop_disparity) */
int svo_disparity(const uint8_t* L, const uint8_t* R, int H, int W, const svo_sgbm_params* prm, int max_disparity,
                  int crop, int16_t* work16, uint8_t* out) {
    int rc = svo_sgbm_compute(L, R, H, W, prm, work16);
    if (rc) return rc;
    rc = svo_filter_speckles(work16, H, W, 0, 4000, max_disparity - 5);
    if (rc) return rc;
    svo_disparity_scale(work16, H, W, max_disparity, crop, out);
    return 0;
}
