// Device-side building blocks shared by the svx kernels (gfx950 / CDNA4).
//
// Exactness contract ("three bit-exactness traps"):
//   * keep1 (dist < thr, functions.py:300-323): fp32 fast path with a rigorous
//     per-point error bound; points inside the band are decided by the exact
//     fp64 reference arithmetic. The mask is therefore bit-exact.
//   * hue bin (functions.py:73-78 + colorsys): exact integer rational path;
//     only exact rational ties (2q == den) run the fp64 colorsys emulation.
//   * int32 back-projection (functions.py:201-209, stereovision.py:112): the
//     fp64 round trip depends on (x,d) / (y,d) only -> 1-bit delta tables
//     built once per camera in fp64 on the device.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

// Measurement knobs (A/B selectors, placement probes, ablations
// whose results are invalid) exist only in the diagnostic build, libsvx_diag.so
// (`make diag`, -DSVX_DIAG; tools/prof.py selects it through SVX_LIB). The
// release libsvx.so reads no SVX_* environment variable: the argument is not
// even compiled, so no knob name is in its string table (tests/test_abi_cpu.py).
#ifdef SVX_DIAG
#define svx_knob(name) std::getenv(name)
#else
#define svx_knob(name) ((const char*)nullptr)
#endif

namespace svx {

constexpr int kWave = 64;
constexpr int kBins = 1024;   // hue bins 0..999 used; padded to 1024

// Everything a kernel needs, passed by value (kernarg segment, scalar loads).
struct KParams {
    int H, W, step, Hg, Wg, pitch, Q;   // Q = quads per grid row = pitch/4
    int frame_quads;                    // Hg * Q
    uint64_t Q_m40;                     // ceil(2^40 / Q): n / Q = (n * Q_m40) >> 40, exact for n < 2^28
    int64_t frame_px;                   // H * W
    // camera (functions.py:15-22)
    double f, B, cw, ch, fB;
    float fB32, B32;
    float cw_hi, cw_lo, ch_hi, ch_lo;   // cw = cw_hi + cw_lo (fp32 split): x - cw in fp32 to 2^-23 rel
    // plane (a*X+b*Y+c*Z = 1) and thresholds
    double a, b, c, nrm, thr;
    float a32, b32, c32, thr32, inv_nrm32, guard32;   // guard32 = 2^-18 / nrm
    float abs_a32, abs_b32, abs_cf32;      // |a|, |b|, |c|*f (bound of |aX|+|bY|+|cZ| per unit K)
    // keep1 in the division-free form |u - d| < t*d with u = B*(a*xc + b*yc + c*f)
    // (real-equivalent to dist < thr after multiplying by d/B > 0):
    // u = fma(al32, x, fma(bb32, y, b032)); decided in fp32 unless |e| <= g32.
    float al32, bb32, b032, tn32, g32;
    int hist_thr;
    int dx_words, dy_words;                // words per d-row of the delta bit tables
    int ablate;                            // DIAGNOSTIC ONLY (env SVX_ABLATE): skip work, results invalid
};

// The plane-dependent fields of KParams used by keep1, for one plane: the
// per-call plane of sv_batch_pipeline, one frame's plane of the per-frame-plane
// pipeline (planes from the batched RANSAC) or a plane broadcast into device
// memory. plane_fields is the single definition, shared by the host's
// set_plane and the device's plane kernels, so both give the same bits.
struct FramePlane {
    double a, b, c, nrm;
    // u = ual*x + ubb*y + ub0 (fp64) and t = thr*|abc|: keep1 <=> |u - d| < t*d
    // (chunk/tile bounds; the fp32 copies below decide single points)
    double ual, ubb, ub0, ut;
    double f, fB, cw, ch, thr;   // camera and point threshold: the exact fp64 path reads them with the plane
    float a32, b32, c32, inv_nrm32, guard32, abs_a32, abs_b32, abs_cf32;
    float al32, bb32, b032, tn32, g32;   // keep1_lean (see KParams)
    uint32_t valid;   // 0: RANSAC found no plane (the reference's plane step raises: no points)
};

// thr = point_thr (functions.py:314-323); W, H = the frame's size in pixels
// (bound of |x|, |y| in the keep1_lean error analysis).
__host__ __device__ inline void plane_fields(FramePlane& o, double a, double b, double c, double f, double B,
                                             double cw, double ch, double thr, int W, int H) {
    o.a = a;
    o.b = b;
    o.c = c;
    o.nrm = __builtin_sqrt(a * a + b * b + c * c);   // functions.py:307 (correctly rounded, host and device)
    o.f = f;
    o.fB = f * B;   // functions.py:191 evaluates f*B in fp64 (as KParams::fB)
    o.cw = cw;
    o.ch = ch;
    o.thr = thr;
    o.a32 = (float)a;
    o.b32 = (float)b;
    o.c32 = (float)c;
    o.inv_nrm32 = (float)(1.0 / o.nrm);
    o.guard32 = (float)(0x1p-18 / o.nrm);
    if (!__builtin_isfinite(o.guard32)) o.guard32 = __builtin_inff();   // degenerate plane: always the exact path
    o.abs_a32 = (float)__builtin_fabs(a);
    o.abs_b32 = (float)__builtin_fabs(b);
    o.abs_cf32 = (float)(__builtin_fabs(c) * f);
    // keep1_lean constants. u = B*(a*(x-cw) + b*(y-ch) + c*f) = al*x + bb*y + b0.
    // fp32 error of e = |u - d| - t*d is <= 2^-21 * M with
    // M = 2*U + 255*(1+t) + 255, U = |al|*W + |bb|*H + |b0| (derivation in
    // DESIGN.md §2.3); the reference's own fp64 error is <= 2^-48 * M. The guard
    // 2^-16 * M leaves a 32x margin; non-finite constants force the exact path.
    const double al = B * a, bb = B * b;
    const double b0 = B * c * f - bb * ch - al * cw;
    const double t = thr * o.nrm;
    const double U = __builtin_fabs(al) * W + __builtin_fabs(bb) * H + __builtin_fabs(b0);
    const double M = 2.0 * U + 255.0 * (1.0 + __builtin_fabs(t)) + 255.0;
    o.ual = al;
    o.ubb = bb;
    o.ub0 = b0;
    o.ut = t;
    o.al32 = (float)al;
    o.bb32 = (float)bb;
    o.b032 = (float)b0;
    o.tn32 = (float)t;
    const double g = M * 0x1p-16;
    const bool finite = __builtin_isfinite(g) && __builtin_isfinite((double)o.al32) &&
                        __builtin_isfinite((double)o.bb32) && __builtin_isfinite((double)o.b032) &&
                        __builtin_isfinite((double)o.tn32);
    o.g32 = finite ? (float)g : __builtin_inff();
    o.valid = 1;
}

__host__ __device__ inline void apply_plane(KParams& p, const FramePlane& o) {
    p.a = o.a;
    p.b = o.b;
    p.c = o.c;
    p.nrm = o.nrm;
    p.a32 = o.a32;
    p.b32 = o.b32;
    p.c32 = o.c32;
    p.inv_nrm32 = o.inv_nrm32;
    p.guard32 = o.guard32;
    p.abs_a32 = o.abs_a32;
    p.abs_b32 = o.abs_b32;
    p.abs_cf32 = o.abs_cf32;
    p.al32 = o.al32;
    p.bb32 = o.bb32;
    p.b032 = o.b032;
    p.tn32 = o.tn32;
    p.g32 = o.g32;
}

// Can some grid point with u in [umin, umax] be kept for some d in 1..255?
// keep1 <=> |u - d| < t*d (u affine in (x, y), so over a rectangle of grid
// points its extremes are at the corners). For t < 0.99 no d in [1, 255] is
// kept when u_max < 1 - t or u_min > 255 (1 + t). The margins (1e-9 relative,
// plus 1e-12 of mag = the largest |term| summed into u) dwarf both the
// reference's fp64 rounding and this bound's own (~1e-15 of mag). NaN:
// keepable (no skipping).
__host__ __device__ inline bool urange_keepable(double umin, double umax, double t, double mag) {
    if (!(t < 0.99)) return true;
    const double slack = 1e-12 + 1e-12 * mag;
    if (umax < (1.0 - t) * (1.0 - 1e-9) - slack) return false;
    if (umin > 255.0 * (1.0 + t) * (1.0 + 1e-9) + 1e-9 + slack) return false;
    return true;
}

// The grid rows gy0..gy1 (all columns 0..Wg-1) of a frame under plane o: keepable?
__host__ __device__ inline bool rows_keepable(const FramePlane& o, int gy0, int gy1, int Wg, int step) {
    const double ax0 = 0.0, ax1 = o.ual * (double)((Wg - 1) * step);
    const double by0 = __builtin_fma(o.ubb, (double)(gy0 * step), o.ub0);
    const double by1 = __builtin_fma(o.ubb, (double)(gy1 * step), o.ub0);
    const double umax = __builtin_fmax(ax0, ax1) + __builtin_fmax(by0, by1);
    const double umin = __builtin_fmin(ax0, ax1) + __builtin_fmin(by0, by1);
    const double mag = __builtin_fabs(ax1) + __builtin_fabs(o.ubb * (double)(gy1 * step)) + __builtin_fabs(o.ub0);
    return urange_keepable(umin, umax, o.ut, mag);
}

// ---------------------------------------------------------------------------
// Hue bin: integer bin k <-> reference key str(round(colorsys hue, 3)).
// exact rational t = 1000*n/(6*rng) (n in [0, 6 rng)); fp64 only on exact ties.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int hue_bin_tie_f64(int r, int g, int b, int mx, int mn) {
    // colorsys.rgb_to_hsv on numpy uint8 scalars, then numpy round(h, 3).
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
    return (int)rint(m * 1000.0);
}

__device__ __forceinline__ int hue_bin(int r, int g, int b) {
    const int mx = max(r, max(g, b));
    const int mn = min(r, min(g, b));
    const int rng = mx - mn;
    int n = (r == mx) ? (g - b) : ((g == mx) ? (2 * rng + b - r) : (4 * rng + r - g));
    n += (n < 0) ? 6 * rng : 0;
    // t = 1000 n / (6 rng) = num / den exactly (num < 2^20, den <= 765).
    // fp32: one rcp (<= 1 ulp) + one mul (0.5 ulp): |t - t_exact| < 1e-4.
    // A non-tie rational is >= 1/(2 den) >= 6.5e-4 from a half-integer, so
    // outside the +-2e-4 band around .5 the fp32 rounding is the exact one.
    const int num = 500 * n, den = 3 * rng;
    const float t = (float)num * __builtin_amdgcn_rcpf((float)den);
    const float fl = __builtin_floorf(t);
    const float fr = t - fl;
    const int m = (int)fl;
    int bin = m + (fr > 0.5f ? 1 : 0);
    if (__builtin_fabsf(fr - 0.5f) < 2e-4f) {   // rare: decide in exact integers
        const int two_rem = 2 * (num - m * den);
        bin = two_rem > den ? m + 1 : (two_rem < den ? m : hue_bin_tie_f64(r, g, b, mx, mn));
    }
    return rng == 0 ? 0 : bin;   // grey: colorsys returns hue 0.0
}

// n / d for 0 <= n < 2^28 with m40 = ceil(2^40 / d), d <= 2^12: with
// m40 = (2^40 + e)/d, 0 <= e < d, the error term n*e/(d*2^40) < 1/d, so the
// floor is exact. One 64-bit multiply instead of a ~20-instruction division.
__device__ __forceinline__ int fastdiv40(int n, uint64_t m40) {
    return (int)(((uint64_t)(uint32_t)n * m40) >> 40);
}

// x - c in fp32 with relative error <= 2^-23 for any fp64 centre c: the first
// subtraction is exact whenever x and c_hi are within 2x of each other
// (Sterbenz), and otherwise |x - c| is large so one rounding costs 2^-24.
__device__ __forceinline__ float centred(int x, float c_hi, float c_lo) {
    return ((float)x - c_hi) - c_lo;
}

// ---------------------------------------------------------------------------
// Plane keep test (functions.py:300-323) for grid pixel (x, y) with d > 0.
// K = B/d (fp32), xc = x - cw, yc = y - ch (fp32, rel err <= 2^-23).
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool keep1_f64(int x, int y, uint32_t d, const KParams& p) {
    const double Z = p.fB / (double)d;
    const double X = (((double)x - p.cw) * Z) / p.f;
    const double Y = (((double)y - p.ch) * Z) / p.f;
    const double dot = __builtin_fma(Z, p.c, __builtin_fma(X, p.a, Y * p.b));
    return __builtin_fabs((dot - 1.0) / p.nrm) < p.thr;
}

__device__ __forceinline__ bool keep1(int x, int y, uint32_t d, float xc, float yc, float K,
                                      float X, float Y, float Z, const KParams& p) {
    const float dot = __builtin_fmaf(Z, p.c32, __builtin_fmaf(X, p.a32, Y * p.b32));
    const float dist = __builtin_fabsf(dot - 1.0f) * p.inv_nrm32;
    const float S = __builtin_fmaf(p.abs_a32, __builtin_fabsf(xc),
                                   __builtin_fmaf(p.abs_b32, __builtin_fabsf(yc), p.abs_cf32)) * K;
    const float G = (S + 1.0f) * p.guard32;
    const float e = dist - p.thr32;
    if (__builtin_fabsf(e) > G) return e < 0.0f;
    return keep1_f64(x, y, d, p);
}

// Division-free keep1 for one grid point (see KParams): returns the fp32
// decision and flags *unc when the exact fp64 reference arithmetic must decide
// (|e| within the rigorous error guard g32, or e not finite). d == 0 never
// keeps and is never uncertain.
__device__ __forceinline__ bool keep1_lean(float xf, float beta, float df, const KParams& p, bool& unc) {
    const float u = __builtin_fmaf(p.al32, xf, beta);
    const float s = u - df;
    const float e = __builtin_fmaf(-p.tn32, df, __builtin_fabsf(s));
    unc = !(__builtin_fabsf(e) > p.g32) && df != 0.0f;
    return e < 0.0f && df != 0.0f;
}

// Hue bin in fp32 with one rcp (the resident pipeline's binning): |t - t_exact| <= 2.5 * 2^-23 * |t| < 3e-4,
// while a non-tie t is >= 1/(2*3*rng) >= 6.5e-4 from a half-integer, so outside the +-4e-4 band around .5 the
// fp32 rounding is the exact one; inside it (and at exact ties) the exact integer/fp64 path hue_bin() decides.
// The sector select is written as value selects. col = B | G << 8 | R << 16 (bits 24..31 ignored). Checked
// against the reference over all 2^24 colours (sv_hue_lut_variant 1, tests/test_gpu_parity.py).
__device__ __forceinline__ uint32_t hue_bin_sel(uint32_t col) {
    const int b = (int)(col & 0xFF), g = (int)((col >> 8) & 0xFF), r = (int)((col >> 16) & 0xFF);
    const int mx = max(r, max(g, b)), mn = min(r, min(g, b));
    const int rng = mx - mn;
    const int nr = g - b, ng = 2 * rng + b - r, nb = 4 * rng + r - g;
    const int n = (r == mx) ? nr : ((g == mx) ? ng : nb);
    const float t = ((float)n * __builtin_amdgcn_rcpf((float)rng)) * (500.0f / 3.0f);
    const float rt = __builtin_rintf(t);
    const bool near = __builtin_fabsf(t - rt) > 0.5f - 4e-4f;   // NaN (grey) -> false
    int bin = (int)rt + (n < 0 ? 1000 : 0);                     // (h mod 1): rint(t + 1000) = rint(t) + 1000
    bin = rng == 0 ? 0 : bin;
    if (__builtin_expect(near, 0)) bin = hue_bin(r, g, b);
    return (uint32_t)bin;
}

// ---------------------------------------------------------------------------
// Wave / block helpers (wave64).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }
// The wave's index in its workgroup, as a value the compiler knows is wave-uniform: addresses built from it stay
// in SGPRs, so a per-lane access is one scalar base + the lane's VGPR offset (no 64-bit VALU address arithmetic).
__device__ __forceinline__ int wave_uniform_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }
// A planePoints entry (functions.py:201-209 + stereovision.py:112's int32 cast) as one word: x and y as int16
// halves (-1 <= x < W, -1 <= y < H, both < 32768), widened back to the reference's int32 pair on read-back.
__host__ __device__ __forceinline__ uint32_t pp_pack(int x, int y) { return (uint32_t)(uint16_t)x | ((uint32_t)(uint16_t)y << 16); }
__host__ __device__ __forceinline__ int pp_x(uint32_t w) { return (int)(int16_t)(uint16_t)(w & 0xFFFFu); }
__host__ __device__ __forceinline__ int pp_y(uint32_t w) { return (int)(int16_t)(uint16_t)(w >> 16); }

// Inclusive wave64 scan of an operation with identity 0 (add, unsigned max, ...)
// in six DPP steps: row_shr 1/2/4/8 (Hillis-Steele inside each 16-lane row),
// then row_bcast 15 (rows 1, 3) and row_bcast 31 (rows 2, 3). A lane whose
// source is outside its row (or a row the mask leaves out) reads the identity.
// One VALU op a step instead of a ds_bpermute + compare + select (shfl_up).
// All 64 lanes must be active.
template <class Op>
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t v, Op op) {
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));   // row_shr:1
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));   // row_shr:2
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));   // row_shr:4
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));   // row_shr:8
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));   // row_bcast:15
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));   // row_bcast:31
    return v;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    return wave_scan_dpp(v, [](uint32_t a, uint32_t b) { return a + b; });
}

// Wave64 sum, uniform: the DPP scan's total (lane 63) read back — six VALU steps instead of the xor butterfly's six
// dependent ds_bpermute round trips. Integer addition, so any order gives the same sum. All 64 lanes must be active.
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(v), 63);
}

// ---------------------------------------------------------------------------
// Decoupled look-back (single-pass ordered compaction across workgroups).
// Status word: [63:62] flag (0 not ready, 1 aggregate, 2 inclusive), [31:0] value.
// One 8-byte granule per tile, written by ONE relaxed agent-scope (sc1) store
// and read by relaxed agent-scope loads: the data is the flag (MI355X guide
// §6 G16, form R2) — no separate payload, no fence needed.
// Forward progress: tile ids come from an atomic ticket, so every tile a wave
// waits on belongs to a workgroup that is already running.
// ---------------------------------------------------------------------------
constexpr uint64_t kFlagAgg = 1ull << 62;
constexpr uint64_t kFlagInc = 2ull << 62;

__device__ __forceinline__ void publish(uint64_t* st, uint64_t flag, uint32_t v) {
    __hip_atomic_store(st, flag | (uint64_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Called by ALL lanes of ONE wave. st points at this frame's tile 0.
// Returns the exclusive prefix of `tile`. Sets *err on (impossible) timeout.
__device__ uint32_t lookback(const uint64_t* st, int tile, uint32_t* err) {
    const int lane = lane_id();
    uint32_t excl = 0;
    int j = tile - 1;
    uint32_t spins = 0;
    while (true) {
        const int idx = j - lane;
        uint64_t w = kFlagInc;  // before the frame start: inclusive 0
        if (idx >= 0)
            w = __hip_atomic_load(st + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t flag = (uint32_t)(w >> 62);
        const uint64_t not_ready = __ballot(flag == 0);
        const uint64_t incl = __ballot(flag == 2);
        const int first_incl = incl ? __builtin_ctzll(incl) : 64;
        const int first_nr = not_ready ? __builtin_ctzll(not_ready) : 64;
        if (first_nr < first_incl) {
            if (++spins > (1u << 24)) {  // bounded: never hang the device
                if (lane == 0) atomicExch(err, 1u);
                return excl;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        const uint32_t v = (lane <= first_incl) ? (uint32_t)w : 0u;
        excl += wave_sum(v);
        if (first_incl < 64) return excl;
        j -= 64;
    }
}

}  // namespace svx
