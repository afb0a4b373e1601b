// SGBM disparity stage: functions.py:104-128
//   StereoSGBM(0, 128, 21).compute -> filterSpeckles(0, 4000, 123) -> TOZERO
//   -> /16 -> u8 -> optional crop -> x(256/128) -> u8
// plus the grey front end of functions.py:61-97 (gamma LUT, BGR2GRAY,
// equalizeHist) and a synthetic rectified-pair generator for the batch.
//
// OpenCV computes SGBM as one sequential row loop carrying the path costs of
// four directions in row buffers. Here every aggregation direction is a set of
// independent 1-D paths, one wave per path, 128 disparities as 64 lanes x 2:
//   hsum_kernel     one workgroup per row: BT pixel costs (LDS-staged row
//                   features) and the 21-wide horizontal box sum -> Hvol
//   vertical_kernel one wave per column: the vertical box sum (OpenCV's
//                   update rules, int16 wrap) -> Cvol, and the (0,-1) path -> L2
//   diag_kernel     one wave per diagonal: the (-1,-1) and (+1,-1) paths -> L1, L3
//   row_kernel      one wave per row: the (-1,0) path summed with L1..L3
//                   (P = sat16), then the (+1,0) path, S = sat16(P + L),
//                   winner, subpixel, disp2 and the left-right check -> int16
//   cc_* kernels    filterSpeckles as union-find connected components
//   out_rows_kernel speckle decision + TOZERO + scaling -> u8 (and int16), one wave a row
// Volumes are [frame][y][x][d] int16 (one 256-byte line per cell, lane l
// holding d = 2l, 2l+1), so every path step is one coalesced 4-byte load or
// store per lane. Exactness rules: see oracle/sgbm_oracle.c (same semantics).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "../svx_device.h"
#include "../svx_sgbm.h"

namespace svx {
namespace {

constexpr int kMaxCost = 32767;
constexpr int kInt16Min = -32768;

__device__ __forceinline__ int lo16(uint32_t v) { return (int)(int16_t)(v & 0xFFFF); }
__device__ __forceinline__ int hi16(uint32_t v) { return (int)(int16_t)(v >> 16); }
__device__ __forceinline__ uint32_t pack16(int a, int b) { return (uint32_t)(uint16_t)a | ((uint32_t)(uint16_t)b << 16); }
__device__ __forceinline__ int sat16(int v) { return v < kInt16Min ? kInt16Min : (v > kMaxCost ? kMaxCost : v); }
__device__ __forceinline__ bool out16(int v) { return v < kInt16Min || v > kMaxCost; }
// Lane hand-offs through LDS inside one wave: the hardware keeps a wave's LDS
// operations in order; this keeps the compiler from moving loads above them.
__device__ __forceinline__ void wave_lds_sync() { __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// min over the wave (signed), every lane active: inclusive DPP min-scan, lane 63.
__device__ __forceinline__ int wave_min_i32(int v) {
    v = min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, 0x111, 0xf, 0xf, false));   // row_shr:1
    v = min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, 0x112, 0xf, 0xf, false));   // row_shr:2
    v = min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, 0x114, 0xf, 0xf, false));   // row_shr:4
    v = min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, 0x118, 0xf, 0xf, false));   // row_shr:8
    v = min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, 0x142, 0xa, 0xf, false));   // row_bcast:15
    v = min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, 0x143, 0xc, 0xf, false));   // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}

// One step of a path (OpenCV formula 13): lane l holds d0 = 2l, d1 = 2l + 1.
// p0/p1: the predecessor's stored (int16) L; pmin: its stored min. A path
// start has p0 = p1 = pmin = 0; d = -1 and d = 128 read MAX_COST. Returns the
// untruncated L values (for the sums) and updates the state with the int16
// truncations OpenCV stores.
// Range: min(...) <= delta, so L <= C <= 32767 always; an L leaves int16 only below -32768, and the walk keeps
// the running minimum of its untruncated L (one v_min3 a step) and tests it once at the path's end.
struct PathState {
    int p0 = 0, p1 = 0, pmin = 0;
    int lmin = 0;
    __device__ bool ovf() const { return lmin < kInt16Min; }
};

// A step in two halves, so that a caller with a second wave minimum to take (the row walk's winner) can run
// both DPP scans interleaved: path_l gives L and min(L0, L1) of the lane, path_commit takes the wave's min.
__device__ __forceinline__ int path_l(int c0, int c1, const PathState& s, int P1, int P2, int& L0, int& L1) {
    const int delta = s.pmin + P2;
    const int left = __builtin_amdgcn_update_dpp(kMaxCost, s.p1, 0x138, 0xf, 0xf, false);   // wave_shr:1, d0 - 1
    const int right = __builtin_amdgcn_update_dpp(kMaxCost, s.p0, 0x130, 0xf, 0xf, false);  // wave_shl:1, d1 + 1
    const int m0 = min(min(s.p0, delta), min(left, s.p1) + P1);
    const int m1 = min(min(s.p1, delta), min(s.p0, right) + P1);
    L0 = c0 + m0 - delta;
    L1 = c1 + m1 - delta;
    return min(L0, L1);
}
__device__ __forceinline__ void path_commit(PathState& s, int L0, int L1, int lm, int wm) {
    s.lmin = min(s.lmin, lm);
    s.p0 = (int)(int16_t)L0;
    s.p1 = (int)(int16_t)L1;
    s.pmin = (int)(int16_t)wm;
}
__device__ __forceinline__ void path_step(int c0, int c1, PathState& s, int P1, int P2, int& L0, int& L1) {
    const int lm = path_l(c0, c1, s, P1, P2, L0, L1);
    path_commit(s, L0, L1, lm, wave_min_i32(lm));
}

// The same step on both disparities at once (v_pk_* 16-bit pairs), for the q-volume walks (0 <= P1, P2 <= 15).
// p holds the stored (int16) L pair. Every term of min(...) that the 32-bit form can take above 32767 (delta,
// N + P1) only meets min() beside p <= 32767, so saturating it changes nothing; q = delta - m is in [0, P2] and
// so exact in 16-bit wrapping arithmetic, and L = C - q wraps exactly as OpenCV's int16 store truncates. An L
// below -32768 is the one range error: then its truncation is C - q + 65536 > C, and sat(L - C) = 32767 > 0,
// where a good step gives -q <= 0 — the walk keeps the running max of that difference.
typedef short pk16 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pk16 as_pk(uint32_t v) { return __builtin_bit_cast(pk16, v); }
__device__ __forceinline__ uint32_t pk_bits(pk16 v) { return __builtin_bit_cast(uint32_t, v); }
struct PathPk {
    uint32_t p = 0;
    int pmin = 0;
    pk16 acc = {-32768, -32768};
    __device__ bool ovf() const { return max((int)acc.x, (int)acc.y) > 0; }
};
__device__ __forceinline__ uint32_t pk_l(uint32_t c, const PathPk& s, int P1, int P2, uint32_t& q, int& lm) {
    const int delta = s.pmin + P2;
    const short ds = (short)min(delta, kMaxCost), dw = (short)delta;
    const uint32_t sh = (uint32_t)__builtin_amdgcn_update_dpp(0x7FFF7FFF, (int)s.p, 0x138, 0xf, 0xf, false);  // lane - 1
    const uint32_t sl = (uint32_t)__builtin_amdgcn_update_dpp(0x7FFF7FFF, (int)s.p, 0x130, 0xf, 0xf, false);  // lane + 1
    const pk16 lft = as_pk(__builtin_amdgcn_alignbit(s.p, sh, 16));   // (d0 - 1, d1 - 1) = (sh.hi, p.lo)
    const pk16 rgt = as_pk(__builtin_amdgcn_alignbit(sl, s.p, 16));   // (d0 + 1, d1 + 1) = (p.hi, sl.lo)
    const pk16 n1 = __builtin_elementwise_add_sat(__builtin_elementwise_min(lft, rgt), (pk16){(short)P1, (short)P1});
    const pk16 m = __builtin_elementwise_min(__builtin_elementwise_min(as_pk(s.p), (pk16){ds, ds}), n1);
    const pk16 qq = (pk16){dw, dw} - m;
    const pk16 L = as_pk(c) - qq;
    q = pk_bits(qq);
    lm = min((int)L.x, (int)L.y);
    return pk_bits(L);
}
__device__ __forceinline__ void pk_commit(PathPk& s, uint32_t c, uint32_t L, int wm) {
    s.acc = __builtin_elementwise_max(s.acc, __builtin_elementwise_sub_sat(as_pk(L), as_pk(c)));
    s.p = L;
    s.pmin = wm;
}
__device__ __forceinline__ uint32_t pk_step(uint32_t c, PathPk& s, int P1, int P2, uint32_t& q) {
    int lm;
    const uint32_t L = pk_l(c, s, P1, P2, q, lm);
    pk_commit(s, c, L, wave_min_i32(lm));
    return L;
}
// both q of a lane (each 0 .. 15, in bits 0-3 and 16-19) as one byte, d0 in the low nibble
__device__ __forceinline__ uint8_t q_byte_pk(uint32_t q) { return (uint8_t)(q | (q >> 12)); }

// A wave-uniform buffer resource over a path's cells: an access is then the lane's byte offset (a loop-invariant
// VGPR) + the step's 32-bit SGPR offset, with no per-access VALU address arithmetic (a global access with a
// 64-bit per-lane address costs a v_lshl_add_u64 each). aux 2: non-temporal.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void* base, size_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)min(bytes, (size_t)0x7FFFFFFF),
                                             0x00020000);
}
__device__ __forceinline__ uint32_t bld32(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, bool nt = false) {
    return nt ? __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 2) : __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
}
__device__ __forceinline__ uint32_t bld8(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, bool nt = false) {
    return nt ? __builtin_amdgcn_raw_buffer_load_b8(r, voff, soff, 2) : __builtin_amdgcn_raw_buffer_load_b8(r, voff, soff, 0);
}
__device__ __forceinline__ void bst32(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, voff, soff, 0);
}
__device__ __forceinline__ void bst8(uint8_t v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_buffer_store_b8(v, r, voff, soff, 0);
}

// two wave minimums, their DPP steps interleaved (each step's input was written two instructions earlier)
__device__ __forceinline__ void wave_min2_i32(int a, int b, int& ra, int& rb) {
#define SVX_MIN2_STEP(ctl, rm)                                                                 \
    a = min(a, __builtin_amdgcn_update_dpp(0x7fffffff, a, ctl, rm, 0xf, false));               \
    b = min(b, __builtin_amdgcn_update_dpp(0x7fffffff, b, ctl, rm, 0xf, false))
    SVX_MIN2_STEP(0x111, 0xf);
    SVX_MIN2_STEP(0x112, 0xf);
    SVX_MIN2_STEP(0x114, 0xf);
    SVX_MIN2_STEP(0x118, 0xf);
    SVX_MIN2_STEP(0x142, 0xa);
    SVX_MIN2_STEP(0x143, 0xc);
#undef SVX_MIN2_STEP
    ra = __builtin_amdgcn_readlane(a, 63);
    rb = __builtin_amdgcn_readlane(b, 63);
}

// A path's L minus the cost it adds, as OpenCV computes it, is min(...) - delta
// in [-P2, 0] (the min includes delta = pmin + P2 and no term is below pmin), so
// for P2 <= 15 (the reference's default P2 is 5) the directions the row walk only
// sums — (-1,-1), (0,-1), (+1,-1) — are stored as q = C - L in a nibble, both of
// a lane's disparities in one byte (64 B per cell instead of 256): the row walk
// adds 3 C - (q1 + q2 + q3). Exact whenever no L leaves int16 (the frame's range
// flag is raised otherwise, and the call fails).
__device__ __forceinline__ uint8_t q_byte(int c0, int c1, int L0, int L1) {
    return (uint8_t)((c0 - L0) | ((c1 - L1) << 4));
}

// ---------------------------------------------------------------------------
// Row features: for each image and channel (0: clipped x-derivative, 1: raw
// intensity) value | half-neighbour min << 8 | max << 16 (calcPixelCostBT).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bt_pair(uint32_t fu, uint32_t fv) {
    const int u = fu & 0xFF, u0 = (fu >> 8) & 0xFF, u1 = fu >> 16;
    const int v = fv & 0xFF, v0 = (fv >> 8) & 0xFF, v1 = fv >> 16;
    const int c0 = max(max(0, u - v1), v0 - u);
    const int c1 = max(max(0, v - u1), u0 - v);
    return (uint32_t)min(c0, c1);
}

__global__ __launch_bounds__(256) void sgbm_hsum_kernel(SgbmK k, const uint8_t* __restrict__ left,
                                                          const uint8_t* __restrict__ right, uint32_t* __restrict__ hvol,
                                                          int frames) {
    extern __shared__ uint32_t smem[];
    const int W = k.W, H = k.H;
    const int f = blockIdx.x / H, y = blockIdx.x - f * H;
    if (f >= frames) return;
    uint32_t* feat = smem;                                   // [img][ch][W]
    uint8_t* tmp = reinterpret_cast<uint8_t*>(smem + 4 * W);  // [img][ch][W] values
    uint32_t* ring = smem + 5 * W;                           // per wave: RS x 64
    const int tid = threadIdx.x;
    const int yu = y > 0 ? y - 1 : y, yd = y < H - 1 ? y + 1 : y;
    for (int i = tid; i < 2 * W; i += blockDim.x) {
        const int img = i >= W, x = i - img * W;
        const uint8_t* src = (img ? right : left) + (size_t)f * k.frame_px;
        int pv = k.ftzero, rv = k.ftzero;
        if (x > 0 && x < W - 1) {
            const uint8_t* r = src + (size_t)y * W;
            const uint8_t* u = src + (size_t)yu * W;
            const uint8_t* d = src + (size_t)yd * W;
            const int g = (r[x + 1] - r[x - 1]) * 2 + u[x + 1] - u[x - 1] + d[x + 1] - d[x - 1];
            pv = min(max(g, -k.ftzero), k.ftzero) + k.ftzero;
            rv = r[x];
        }
        tmp[(img * 2 + 0) * W + x] = (uint8_t)pv;
        tmp[(img * 2 + 1) * W + x] = (uint8_t)rv;
    }
    __syncthreads();
    for (int i = tid; i < 4 * W; i += blockDim.x) {
        const int row = i / W, x = i - row * W;
        const uint8_t* v = tmp + row * W;
        const int c = v[x];
        const int l = x > 0 ? (c + v[x - 1]) >> 1 : c;
        const int r = x < W - 1 ? (c + v[x + 1]) >> 1 : c;
        feat[i] = (uint32_t)c | (uint32_t)min(min(l, r), c) << 8 | (uint32_t)max(max(l, r), c) << 16;
    }
    __syncthreads();

    const int lane = lane_id(), wave = tid >> 6, nwaves = blockDim.x >> 6;
    const int RS = 2 * k.SW2 + 1;
    uint32_t* myring = ring + wave * RS * 64 + lane;
    const int seg = (k.width1 + nwaves - 1) / nwaves;
    const int xs = wave * seg, xe = min(k.width1, xs + seg);
    if (xs >= xe) return;
    const uint32_t* fLp = feat;
    const uint32_t* fLr = feat + W;
    const uint32_t* fRp = feat + 2 * W;
    const uint32_t* fRr = feat + 3 * W;
    const int d0 = 2 * lane;
    // pixel cost pair (d0, d0 + 1) at cost column j (image column j + D)
    auto pix = [&](int j) -> uint32_t {
        j = min(max(j, 0), k.width1 - 1);
        const int x = j + kSgD;
        const uint32_t lp = fLp[x], lr = fLr[x];
        const int xr0 = x - d0, xr1 = xr0 - 1;
        const uint32_t a = bt_pair(lp, fRp[xr0]) + (bt_pair(lr, fRr[xr0]) >> 2);
        const uint32_t b = bt_pair(lp, fRp[xr1]) + (bt_pair(lr, fRr[xr1]) >> 2);
        return a | b << 16;
    };
    uint32_t sum = 0;
    for (int j = xs - k.SW2, s = 0; j <= xs + k.SW2; ++j, ++s) {
        const uint32_t v = pix(j);
        myring[s * 64] = v;
        sum += v;
    }
    uint32_t* out = hvol + ((size_t)f * H + y) * k.width1 * 64 + lane;
    int slot = 0;   // ring slot of column xi - SW2
    for (int xi = xs; xi < xe; ++xi) {
        out[(size_t)xi * 64] = sum;
        const uint32_t vn = pix(xi + 1 + k.SW2);
        const uint32_t vo = myring[slot * 64];
        myring[slot * 64] = vn;
        sum = (sum + vn) - vo;   // both halves stay >= 0: no borrow between them
        slot = slot + 1 == RS ? 0 : slot + 1;
    }
}

// The same horizontal sums for a compile-time half window (the reference's block 21: SW2 = 10), with less work
// per column. (1) Both BT channels in one packed 16-bit operation: a pixel's features are three words, value,
// half-neighbour min and max, each holding channel 0 (x-derivative) in the low and channel 1 (raw) in the high
// half, so a cost is 9 v_pk_* operations plus its channel sum. (2) Lane l's cost pair at column j reads the right
// features A_j(l) = R[j + D - 2l] and A_{j-1}(l) (= R[j + D - 2l - 1]); since A_{j+1}(l) = A_{j-1}(l - 1), the
// next column's right features are the previous-but-one's moved up a lane (DPP), lane 0 taking the new
// R[j + 1 + D], so the main loop reads LDS only at one address for the whole wave. (3) The window's RS columns
// are a register ring indexed by the unrolled step.
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s16x2 as_s16x2(uint32_t v) { return __builtin_bit_cast(s16x2, v); }
struct BtFeat {
    uint32_t v, lo, hi;   // value, half-neighbour min, max: channel 0 | channel 1 << 16
};
// max(u - v1, v0 - u, 0) = max(sat(u - v1), sat(v0 - u)) with unsigned saturating subtractions (the features
// are 0 .. 255): v_pk_sub_u16 clamp twice and a v_pk_max_u16 per direction.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
// both channels' costs (channel 0 in the low half, channel 1 in the high)
__device__ __forceinline__ uint32_t bt_cost_ch(const BtFeat& a, const BtFeat& b) {
    const u16x2 u = as_u16x2(a.v), u0 = as_u16x2(a.lo), u1 = as_u16x2(a.hi);
    const u16x2 v = as_u16x2(b.v), v0 = as_u16x2(b.lo), v1 = as_u16x2(b.hi);
    const u16x2 c0 = __builtin_elementwise_max(__builtin_elementwise_sub_sat(u, v1), __builtin_elementwise_sub_sat(v0, u));
    const u16x2 c1 = __builtin_elementwise_max(__builtin_elementwise_sub_sat(v, u1), __builtin_elementwise_sub_sat(u0, v));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(c0, c1));
}
// two pixels' costs as a pair: (c0(a) + c1(a) >> 2) | (c0(b) + c1(b) >> 2) << 16, with the channels regrouped
// by two v_perm so that the shift and the sum are one packed operation each for both
__device__ __forceinline__ uint32_t bt_cost_pair(const BtFeat& l, const BtFeat& a, const BtFeat& b) {
    const uint32_t ca = bt_cost_ch(l, a), cb = bt_cost_ch(l, b);
    const u16x2 ch0 = as_u16x2(__builtin_amdgcn_perm(cb, ca, 0x05040100u));   // (ca.lo, cb.lo)
    const u16x2 ch1 = as_u16x2(__builtin_amdgcn_perm(cb, ca, 0x07060302u));   // (ca.hi, cb.hi)
    return __builtin_bit_cast(uint32_t, ch0 + (ch1 >> (u16x2){2, 2}));
}

// ABL (diagnostic build only, results invalid): the same stores with no arithmetic, to find what bounds the
// kernel — 1 the staging and then each wave's quarter of the row written with constants, 2 the staging and then
// the four waves' stores interleaved by column (the workgroup writes 1 KB contiguous a step), 3 the stores of 1
// without the staging
template <int SW2C, int ABL = 0>
__global__ __launch_bounds__(256) void sgbm_hsum_ring_kernel(SgbmK k, const uint8_t* __restrict__ left,
                                                               const uint8_t* __restrict__ right,
                                                               uint32_t* __restrict__ hvol, int frames) {
    constexpr int RS = 2 * SW2C + 1;
    extern __shared__ uint32_t smem[];
    const int W = k.W, H = k.H;
    const int f = blockIdx.x / H, y = blockIdx.x - f * H;
    if (f >= frames) return;
    if constexpr (ABL != 0) {
        if (ABL == 3) {
            const int n = k.width1, seg = (n + 3) / 4, lane = lane_id(), wave = wave_uniform_id();
            uint32_t* out = hvol + ((size_t)f * H + y) * n * 64;
            for (int xi = wave * seg; xi < min(n, wave * seg + seg); ++xi) (out + (size_t)xi * 64)[(uint32_t)lane] = lane;
            return;
        }
    }
    uint2* featA = reinterpret_cast<uint2*>(smem);             // [img][W] (value, min)
    uint32_t* featB = reinterpret_cast<uint32_t*>(featA + 2 * W);   // [img][W] max
    uint8_t* raw = reinterpret_cast<uint8_t*>(smem);           // [img][row above, row, row below][W], dead before
                                                               // the features are written over it
    uint8_t* tmp = reinterpret_cast<uint8_t*>(featB + 2 * W);  // [img][ch][W] values
    const int tid = threadIdx.x;
    const int yu = y > 0 ? y - 1 : y, yd = y < H - 1 ? y + 1 : y;
    if (((W | (int)((uintptr_t)left | (uintptr_t)right)) & 3) == 0) {
        // 4-byte words, every load of the thread issued before the first is waited for (W <= 2048: <= 12 each)
        constexpr int kPer = 12;
        const int wpr = W >> 2, nw = 6 * wpr;
        uint32_t v[kPer];
#pragma unroll
        for (int t = 0; t < kPer; ++t) {
            const int i = tid + t * 256;
            if (i < nw) {
                const int r = i / wpr, xw = i - r * wpr;
                const int img = r >= 3, row = r - 3 * img;
                const int yy = row == 0 ? yu : (row == 1 ? y : yd);
                v[t] = reinterpret_cast<const uint32_t*>((img ? right : left) + (size_t)f * k.frame_px +
                                                         (size_t)yy * W)[xw];
            }
        }
#pragma unroll
        for (int t = 0; t < kPer; ++t) {
            const int i = tid + t * 256;
            if (i < nw) reinterpret_cast<uint32_t*>(raw)[i] = v[t];
        }
    } else {
        for (int i = tid; i < 6 * W; i += 256) {
            const int r = i / W, x = i - r * W;
            const int img = r >= 3, row = r - 3 * img;
            const int yy = row == 0 ? yu : (row == 1 ? y : yd);
            raw[i] = (img ? right : left)[(size_t)f * k.frame_px + (size_t)yy * W + x];
        }
    }
    __syncthreads();
    for (int i = tid; i < 2 * W; i += 256) {
        const int img = i >= W, x = i - img * W;
        const uint8_t* u = raw + img * 3 * W;
        const uint8_t* r = u + W;
        const uint8_t* d = r + W;
        int pv = k.ftzero, rv = k.ftzero;
        if (x > 0 && x < W - 1) {
            const int g = (r[x + 1] - r[x - 1]) * 2 + u[x + 1] - u[x - 1] + d[x + 1] - d[x - 1];
            pv = min(max(g, -k.ftzero), k.ftzero) + k.ftzero;
            rv = r[x];
        }
        tmp[(img * 2 + 0) * W + x] = (uint8_t)pv;
        tmp[(img * 2 + 1) * W + x] = (uint8_t)rv;
    }
    __syncthreads();
    for (int i = tid; i < 2 * W; i += 256) {
        const int img = i >= W, x = i - img * W;
        uint32_t fv = 0, flo = 0, fhi = 0;
#pragma unroll
        for (int ch = 0; ch < 2; ++ch) {
            const uint8_t* v = tmp + (img * 2 + ch) * W;
            const int c = v[x];
            const int l = x > 0 ? (c + v[x - 1]) >> 1 : c;
            const int r = x < W - 1 ? (c + v[x + 1]) >> 1 : c;
            fv |= (uint32_t)c << (16 * ch);
            flo |= (uint32_t)min(min(l, r), c) << (16 * ch);
            fhi |= (uint32_t)max(max(l, r), c) << (16 * ch);
        }
        featA[i] = make_uint2(fv, flo);
        featB[i] = fhi;
    }
    __syncthreads();

    const int lane = lane_id(), wave = wave_uniform_id();
    const int n = k.width1;
    const int seg = (n + 3) / 4;
    const int xs = wave * seg, xe = min(n, xs + seg);
    if constexpr (ABL == 1 || ABL == 2) {
        uint32_t* out = hvol + ((size_t)f * H + y) * n * 64;
        const uint32_t v = featB[lane];   // keeps the staging live
        if (ABL == 1)
            for (int xi = xs; xi < xe; ++xi) (out + (size_t)xi * 64)[(uint32_t)lane] = v;
        else
            for (int xi = wave; xi < n; xi += 4) (out + (size_t)xi * 64)[(uint32_t)lane] = v;
        return;
    }
    if (xs >= xe) return;
    const int d0 = 2 * lane;
    const auto feat = [&](int i) -> BtFeat {
        const uint2 a = featA[i];
        return BtFeat{a.x, a.y, featB[i]};
    };
    // cost pair (d0, d0 + 1) from the left features at x and the right ones at x - d0 (a) and x - d0 - 1 (b)
    const auto cost = [](const BtFeat& l, const BtFeat& a, const BtFeat& b) -> uint32_t {
        return bt_cost_pair(l, a, b);
    };
    const auto pix = [&](int j) -> uint32_t {
        j = min(max(j, 0), n - 1);
        const int x = j + kSgD;
        return cost(feat(x), feat(W + x - d0), feat(W + x - d0 - 1));
    };
    uint32_t ring[RS];
    uint32_t sum = 0;
#pragma unroll
    for (int s = 0; s < RS; ++s) {
        ring[s] = pix(xs - SW2C + s);
        sum += ring[s];
    }
    int jn = min(xs + SW2C, n - 1);   // the last column computed; ring[RS - 1] holds its cost
    uint32_t vlast = ring[RS - 1];
    BtFeat acur = feat(W + jn + kSgD - d0), aprev = feat(W + jn + kSgD - d0 - 1);   // A_jn, A_{jn - 1}
    uint32_t* out = hvol + ((size_t)f * H + y) * n * 64;   // wave-uniform row; + the lane per store
    // The main loop's feature reads at column x are the same for every lane; with x wave-uniform the compiler
    // copies the SGPR address into a VGPR for each of the four reads. An opaque zero added once keeps x in a
    // VGPR, stepped by one add per column.
    int vzero;
    __asm__("v_mov_b32 %0, 0" : "=v"(vzero));
    int xv = jn + kSgD + vzero;
    const auto step = [&]() {   // adds column jn + 1 (jn < n - 1)
        ++jn;
        const int x = ++xv;   // jn + kSgD
        const BtFeat rn = feat(W + x);   // lane 0's A_jn
        BtFeat anew;                     // wave_shr:1 of A_{jn - 2}
        anew.v = __builtin_amdgcn_update_dpp((int)rn.v, (int)aprev.v, 0x138, 0xf, 0xf, false);
        anew.lo = __builtin_amdgcn_update_dpp((int)rn.lo, (int)aprev.lo, 0x138, 0xf, 0xf, false);
        anew.hi = __builtin_amdgcn_update_dpp((int)rn.hi, (int)aprev.hi, 0x138, 0xf, 0xf, false);
        vlast = cost(feat(x), anew, acur);
        aprev = acur;
        acur = anew;
    };
    int x0 = xs;
    // whole blocks of RS columns that each store and each add a column: no condition in the unrolled block, so
    // the ring index is a compile-time register and the next columns' LDS reads can be issued early
    for (; x0 + RS <= xe && jn + RS <= n - 1; x0 += RS) {
        uint32_t* ob = out + (size_t)x0 * 64 + lane;   // the block's first cell: immediate offsets per step
#pragma unroll
        for (int u = 0; u < RS; ++u) {
            ob[u * 64] = sum;
            step();
            sum = (sum + vlast) - ring[u];
            ring[u] = vlast;
        }
    }
    // the rest (the row's last columns), the ring's phase unchanged
    for (; x0 < xe; x0 += RS) {
#pragma unroll
        for (int u = 0; u < RS; ++u) {
            const int xi = x0 + u;
            if (xi < xe) {
                (out + (size_t)xi * 64)[(uint32_t)lane] = sum;   // (non-temporal stores: no faster)
                // step xi adds column xi + 1 + SW2 (clamped: past the last column it is the last column again)
                if (jn < n - 1) step();
                sum = (sum + vlast) - ring[u];
                ring[u] = vlast;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Vertical box sum with OpenCV's row rules, and the (0,-1) path.
// ---------------------------------------------------------------------------
// The operands of a path step never depend on the recurrence, so every walk
// below keeps the next U steps' loads in flight (registers, clamped addresses:
// the loads past a path's end are redundant) while it runs the current U steps.
template <int U, bool DQ>
__global__ __launch_bounds__(256) void sgbm_vertical_kernel(SgbmK k, const uint32_t* __restrict__ hvol,
                                                              uint32_t* __restrict__ cvol, uint32_t* __restrict__ l2vol,
                                                              uint8_t* __restrict__ q2vol, uint32_t* __restrict__ flags,
                                                              int frames) {
    const int wpb = blockDim.x >> 6;
    const int cols_blocks = (k.width1 + wpb - 1) / wpb;
    const int f = blockIdx.x / cols_blocks;
    const int xi = (blockIdx.x - f * cols_blocks) * wpb + wave_uniform_id();
    if (f >= frames || xi >= k.width1) return;
    const uint32_t lane = lane_id();
    const int H = k.H, SH2 = k.SH2;
    const size_t rs = (size_t)k.width1 * 64;
    const size_t base = (size_t)f * H * rs + (size_t)xi * 64;   // wave-uniform: the column's cell at row 0
    const uint32_t* hb = hvol + base;
    int c0 = 0, c1 = 0;
    for (int kk = 0; kk <= SH2; ++kk) {
        const uint32_t h = (hb + (size_t)min(kk, H - 1) * rs)[lane];
        const int sc = kk == 0 ? SH2 + 1 : 1;
        c0 += lo16(h) * sc;
        c1 += hi16(h) * sc;
    }
    std::conditional_t<DQ, PathPk, PathState> st;
    const bool upd_col = xi > 0;
    // step y adds row y + SH2 and drops row y - SH2 - 1 (OpenCV's rules, below)
    const auto load = [&](int y, uint32_t& a, uint32_t& r) {
        a = (hb + (size_t)min(y + SH2, H - 1) * rs)[lane];
        r = (hb + (size_t)min(max(y - SH2 - 1, 0), H - 1) * rs)[lane];
    };
    uint32_t ca[U], cr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) load(u, ca[u], cr[u]);
    for (int y0 = 0; y0 < H; y0 += U) {
        uint32_t na[U], nr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) load(y0 + U + u, na[u], nr[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int y = y0 + u;
            if (y >= H) break;
            if (y > 0 && upd_col && y + SH2 < H) {
                c0 += lo16(ca[u]) - lo16(cr[u]);
                c1 += hi16(ca[u]) - hi16(cr[u]);
            }
            const int cw0 = (int)(int16_t)c0, cw1 = (int)(int16_t)c1;
            const size_t o = base + (size_t)y * rs;
            const uint32_t cw = pack16(cw0, cw1);
            (cvol + o)[lane] = cw;
            if constexpr (DQ) {
                uint32_t q;
                pk_step(cw, st, k.P1, k.P2, q);
                (q2vol + o)[lane] = q_byte_pk(q);
            } else {
                int L0, L1;
                path_step(cw0, cw1, st, k.P1, k.P2, L0, L1);
                (l2vol + o)[lane] = pack16(L0, L1);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ca[u] = na[u];
            cr[u] = nr[u];
        }
    }
    if (__any(st.ovf()) && lane == 0) atomicOr(flags + f, 1u);
}

// The same walk for a compile-time half window (the reference's block 21: SH2 = 10) with each horizontal sum
// read once: the row a step drops (max(y - SH2 - 1, 0)) is the row added RS = 2 SH2 + 1 steps before it, or
// one of rows 0 .. SH2 read for the first window, so the walk keeps the next RS drops in registers (a ring
// indexed by the unrolled step) and loads only the added rows, the next block's in flight.
#ifndef SVX_VRING_ABLATE
#define SVX_VRING_ABLATE 0
#endif
template <int SH2C, bool DQ>
__global__ __launch_bounds__(256) void sgbm_vertical_ring_kernel(SgbmK k, const uint32_t* __restrict__ hvol,
                                                                   uint32_t* __restrict__ cvol,
                                                                   uint32_t* __restrict__ l2vol,
                                                                   uint8_t* __restrict__ q2vol,
                                                                   uint32_t* __restrict__ flags, int frames) {
    constexpr int RS = 2 * SH2C + 1;
    const int wpb = blockDim.x >> 6;
    const int cols_blocks = (k.width1 + wpb - 1) / wpb;
    const int f = blockIdx.x / cols_blocks;
    const int xi = (blockIdx.x - f * cols_blocks) * wpb + wave_uniform_id();
    if (f >= frames || xi >= k.width1) return;
    const uint32_t lane = lane_id();
    const int H = k.H;
    const size_t rs = (size_t)k.width1 * 64;
    const size_t base = (size_t)f * H * rs + (size_t)xi * 64;   // wave-uniform: the column's cell at row 0
    const uint32_t rs32 = (uint32_t)rs;   // the column's cells are y * rs on: < 2^31 bytes a frame
    const __amdgpu_buffer_rsrc_t rh = wave_rsrc(hvol + base, (size_t)H * rs * 4),
                                 rcv = wave_rsrc(cvol + base, (size_t)H * rs * 4), rq2 = wave_rsrc(q2vol + base, (size_t)H * rs);
    const auto hrow = [&](int r) { return bld32(rh, lane * 4, (uint32_t)min(r, H - 1) * rs32 * 4); };
    // drop[u]: the row step y0 + u subtracts (block y0 = 0: rows max(u - SH2 - 1, 0), read with the first window)
    uint32_t drop[RS];
    int c0 = 0, c1 = 0;
#pragma unroll
    for (int kk = 0; kk <= SH2C; ++kk) {
        const uint32_t h = hrow(kk);
        const int sc = kk == 0 ? SH2C + 1 : 1;
        c0 += lo16(h) * sc;
        c1 += hi16(h) * sc;
        if (kk == 0) {
#pragma unroll
            for (int u = 0; u <= SH2C + 1; ++u) drop[u] = h;   // steps 1 .. SH2 + 1 drop row 0
        } else if (kk < SH2C) {
            drop[kk + SH2C + 1] = h;                           // step kk + SH2 + 1 drops row kk
        }   // row SH2 is step RS's drop: step 0 stores it (drop[0] = its added row, SH2)
    }
    std::conditional_t<DQ, PathPk, PathState> st;
    const bool upd_col = xi > 0;
    uint32_t add[RS];   // the rows steps y0 .. y0 + RS - 1 add (y + SH2, clamped)
#pragma unroll
    for (int u = 0; u < RS; ++u) add[u] = hrow(u + SH2C);
    const auto vstep = [&](int u, int y) {
        if (y > 0 && upd_col && y + SH2C < H) {
            c0 += lo16(add[u]) - lo16(drop[u]);
            c1 += hi16(add[u]) - hi16(drop[u]);
        }
        drop[u] = add[u];   // step y + RS drops row y + SH2
        const int cw0 = (int)(int16_t)c0, cw1 = (int)(int16_t)c1;
        const uint32_t cw = pack16(cw0, cw1);
        bst32(cw, rcv, lane * 4, (uint32_t)y * rs32 * 4);
        if constexpr (DQ) {
#if SVX_VRING_ABLATE   // A/B builds only (results invalid): the loads and stores without the path step
            bst8(cw, rq2, lane, (uint32_t)y * rs32);
#else
            uint32_t q;
            pk_step(cw, st, k.P1, k.P2, q);
            bst8(q_byte_pk(q), rq2, lane, (uint32_t)y * rs32);
#endif
        } else {
            int L0, L1;
            path_step(cw0, cw1, st, k.P1, k.P2, L0, L1);
            (l2vol + base + (size_t)y * rs)[lane] = pack16(L0, L1);
        }
    };
    // whole blocks (no exit inside the unrolled block, so both rings stay compile-time registers), the next
    // block's rows in flight; then the last, partial block
    int y0 = 0;
    for (; y0 + RS <= H; y0 += RS) {
        uint32_t nadd[RS];
#pragma unroll
        for (int u = 0; u < RS; ++u) nadd[u] = hrow(y0 + RS + u + SH2C);
#pragma unroll
        for (int u = 0; u < RS; ++u) vstep(u, y0 + u);
#pragma unroll
        for (int u = 0; u < RS; ++u) add[u] = nadd[u];
    }
#pragma unroll
    for (int u = 0; u < RS; ++u)
        if (y0 + u < H) vstep(u, y0 + u);
    if (__any(st.ovf()) && lane == 0) atomicOr(flags + f, 1u);
}

// ---------------------------------------------------------------------------
// Diagonal paths: dir 1 from (x-1, y-1), dir 3 from (x+1, y-1).
// ---------------------------------------------------------------------------
template <int U, bool DQ>
__global__ __launch_bounds__(256) void sgbm_diag_kernel(SgbmK k, const uint32_t* __restrict__ cvol,
                                                          uint32_t* __restrict__ l1vol, uint32_t* __restrict__ l3vol,
                                                          uint8_t* __restrict__ q1vol, uint8_t* __restrict__ q3vol,
                                                          uint32_t* __restrict__ flags, int frames) {
    const int wpb = blockDim.x >> 6;
    const int npaths = k.width1 + k.H - 1;   // per direction
    const int per_frame = 2 * npaths;
    const int gw = blockIdx.x * wpb + wave_uniform_id();
    const int f = gw / per_frame;
    if (f >= frames) return;
    int p = gw - f * per_frame;
    const int dir = p >= npaths;   // 0: from x-1 (L1), 1: from x+1 (L3)
    p -= dir * npaths;
    int xi, y;
    if (p < k.width1) {
        xi = p;
        y = 0;
    } else {
        xi = dir ? k.width1 - 1 : 0;
        y = p - k.width1 + 1;
    }
    // the path: cells (xi + t * dx, y + t), t < len; every address below is a wave-uniform cell + the lane
    const int len = min(k.H - y, dir ? xi + 1 : k.width1 - xi);
    const uint32_t lane = lane_id();
    const size_t rs = (size_t)k.width1 * 64;
    const size_t a0 = (size_t)f * k.H * rs + (size_t)y * rs + (size_t)xi * 64;
    const size_t step = dir ? rs - 64 : rs + 64;
    uint32_t* out = dir ? l3vol : l1vol;
    uint8_t* qout = dir ? q3vol : q1vol;
    // the path's cells from its first: t * step cells on, at most a frame's volume (< 2^31 bytes)
    const size_t span = (size_t)(len - 1) * step + 64;
    const __amdgpu_buffer_rsrc_t rc = wave_rsrc(cvol + a0, span * 4), rq = wave_rsrc(qout + a0, span);
    const uint32_t st32 = (uint32_t)step;
    const auto cell = [&](int t) { return bld32(rc, lane * 4, (uint32_t)min(t, len - 1) * st32 * 4); };
    std::conditional_t<DQ, PathPk, PathState> st;
    uint32_t cc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) cc[u] = cell(u);
    for (int t0 = 0; t0 < len; t0 += U) {
        uint32_t nc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) nc[u] = cell(t0 + U + u);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = t0 + u;
            if (t >= len) break;
            const size_t o = a0 + (size_t)t * step;
            if constexpr (DQ) {
                uint32_t q;
                pk_step(cc[u], st, k.P1, k.P2, q);
                bst8(q_byte_pk(q), rq, lane, (uint32_t)t * st32);
            } else {
                int L0, L1;
                path_step(lo16(cc[u]), hi16(cc[u]), st, k.P1, k.P2, L0, L1);
                (out + o)[lane] = pack16(L0, L1);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) cc[u] = nc[u];
    }
    if (__any(st.ovf()) && lane == 0) atomicOr(flags + f, 1u);
}

// ---------------------------------------------------------------------------
// Row kernel: (-1,0) path + sum, (+1,0) path + selection, left-right check.
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T ld_nt(const T* p, bool nt) { return nt ? __builtin_nontemporal_load(p) : *p; }

// LDS per wave: the right view's best cost per column as one word, (minS + 32768) << 16 | (0xFFFF - xi) — the
// reference's "if (disp2cost[x2] > minS)" in decreasing x is the minimum of that key (the smaller cost, then
// the larger xi, i.e. the pixel visited first), so the updates need no order and no read — then disp1 (int16).
__host__ __device__ constexpr size_t sgbm_row_lds_per_wave(int W) { return ((size_t)6 * W + 3) & ~(size_t)3; }

// steps in flight in each pass (A/B builds only: -DSVX_ROW_UA=16 / -DSVX_ROW_UB=16)
#ifndef SVX_ROW_UA
#define SVX_ROW_UA 0
#endif
#ifndef SVX_ROW_UB
#define SVX_ROW_UB 0
#endif
#ifndef SVX_ROW_ABLATE
#define SVX_ROW_ABLATE 0
#endif
template <int U0, bool NT, bool DQ>
__global__ __launch_bounds__(256) void sgbm_row_kernel(SgbmK k, const uint32_t* __restrict__ cvol,
                                                         uint32_t* __restrict__ l1p, const uint32_t* __restrict__ l2vol,
                                                         const uint32_t* __restrict__ l3vol,
                                                         uint8_t* __restrict__ q0vol, const uint8_t* __restrict__ q1vol,
                                                         const uint8_t* __restrict__ q2vol,
                                                         const uint8_t* __restrict__ q3vol, int16_t* __restrict__ d16,
                                                         uint32_t* __restrict__ flags, int frames) {
    constexpr int UA = SVX_ROW_UA > 0 && DQ ? SVX_ROW_UA : U0, UB = SVX_ROW_UB > 0 && DQ ? SVX_ROW_UB : U0;
    extern __shared__ uint32_t rsm32[];
    const int wpb = blockDim.x >> 6, wave = wave_uniform_id();
    const int gw = blockIdx.x * wpb + wave;
    const int f = gw / k.H, y = gw - f * k.H;
    if (f >= frames) return;
    const int W = k.W;
    const uint32_t lane = lane_id();
    uint32_t* d2key = rsm32 + wave * (sgbm_row_lds_per_wave(W) / 4);
    int16_t* disp1 = reinterpret_cast<int16_t*>(d2key + W);
    const int INVALID = -kSgScale;   // (minD - 1) * 16, minD = 0
    for (int x = lane; x < W; x += 64) {
        disp1[x] = (int16_t)INVALID;
        d2key[x] = ~0u;
    }
    wave_lds_sync();
    const size_t rs = (size_t)k.width1 * 64;
    const size_t rb = ((size_t)f * k.H + y) * rs;   // wave-uniform: the row's first cell
    const int n = k.width1;
    // the cell of column xi in a volume: a wave-uniform address + the lane (DQ: buffer resources over the row)
    const auto at = [&](auto* vol, int xi) { return vol + rb + (size_t)xi * 64; };
    const __amdgpu_buffer_rsrc_t rc = wave_rsrc(cvol + rb, rs * 4), rq0 = wave_rsrc(q0vol + rb, rs),
                                 rq1 = wave_rsrc(q1vol + rb, rs), rq2 = wave_rsrc(q2vol + rb, rs),
                                 rq3 = wave_rsrc(q3vol + rb, rs);
    std::conditional_t<DQ, PathPk, PathState> sa, sb;
    // pass A: x ascending, direction (-1, 0); P = sat16(L0 + L1 + L2 + L3) replaces L1.
    // DQ: pass A stores only its own q (q0 = C - L0) and pass B forms P = sat16(4 C - (q0 + q1 + q2 + q3))
    // from the four q bytes: C is read twice, the other directions once, as 64 B a cell.
    {
        constexpr int U = UA;
        uint32_t cc[U], ca[U], cb[U], ce[U];
        const auto load = [&](int xi, uint32_t& c, uint32_t& a, uint32_t& b, uint32_t& e) {
            xi = min(xi, n - 1);
            if constexpr (DQ) {
                c = bld32(rc, lane * 4, (uint32_t)xi * 256);
            } else {
                c = at(cvol, xi)[lane];
                a = ld_nt(at(l1p, xi) + lane, NT);
                b = ld_nt(at(l2vol, xi) + lane, NT);
                e = ld_nt(at(l3vol, xi) + lane, NT);
            }
        };
#pragma unroll
        for (int u = 0; u < U; ++u) load(u, cc[u], ca[u], cb[u], ce[u]);
        for (int x0 = 0; x0 < n; x0 += U) {
            uint32_t nc[U], na[U], nb[U], ne[U];
#pragma unroll
            for (int u = 0; u < U; ++u) load(x0 + U + u, nc[u], na[u], nb[u], ne[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int xi = x0 + u;
                if (xi >= n) break;
                if constexpr (DQ) {
#if SVX_ROW_ABLATE & 1   // A/B builds only (results invalid): the loads and stores without the path step (bit 0
                     // pass A, bit 1 pass B)
                    bst8(cc[u], rq0, lane, (uint32_t)xi * 64);
#else
                    uint32_t q;
                    pk_step(cc[u], sa, k.P1, k.P2, q);
                    bst8(q_byte_pk(q), rq0, lane, (uint32_t)xi * 64);
#endif
                } else {
                    int L0, L1;
                    path_step(lo16(cc[u]), hi16(cc[u]), sa, k.P1, k.P2, L0, L1);
                    const uint32_t pv = pack16(sat16(L0 + lo16(ca[u]) + lo16(cb[u]) + lo16(ce[u])),
                                               sat16(L1 + hi16(ca[u]) + hi16(cb[u]) + hi16(ce[u])));
                    if (NT)
                        __builtin_nontemporal_store(pv, at(l1p, xi) + lane);
                    else
                        at(l1p, xi)[lane] = pv;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                cc[u] = nc[u];
                ca[u] = na[u];
                cb[u] = nb[u];
                ce[u] = ne[u];
            }
        }
    }
    // pass B: x descending, direction (+1, 0), S = sat16(P + L), winner per pixel. The winner and its
    // neighbours' costs are wave-uniform; step u of a group of U parks them in lane u and the
    // group's subpixel divisions and LDS updates run once, lanes 0 .. U-1 side by side, after its U steps.
    {
        constexpr int U = UB;
        const int d0 = 2 * lane;
        uint32_t cc[U], cp[U];
        // step j visits xi = n - 1 - j (pass A's P of every cell is stored before these loads;
        // DQ: pp = the four q bytes, q0 | q1 << 8 | q2 << 16 | q3 << 24)
        const auto load = [&](int j, uint32_t& c, uint32_t& pp) {
            const int xi = max(n - 1 - j, 0);
            if constexpr (DQ) {
                const uint32_t so = (uint32_t)xi * 64;
                c = bld32(rc, lane * 4, so * 4, NT);
                pp = bld8(rq0, lane, so, NT) | bld8(rq1, lane, so, NT) << 8 | bld8(rq2, lane, so, NT) << 16 |
                     bld8(rq3, lane, so, NT) << 24;
            } else {
                c = ld_nt(at(cvol, xi) + lane, NT);
                pp = ld_nt(at(l1p, xi) + lane, NT);
            }
        };
#pragma unroll
        for (int u = 0; u < U; ++u) load(u, cc[u], cp[u]);
        for (int j0 = 0; j0 < n; j0 += U) {
            uint32_t nc[U], np[U];
#pragma unroll
            for (int u = 0; u < U; ++u) load(j0 + U + u, nc[u], np[u]);
            int gkey = -1, gnum = 0, gdv = 1;   // lane u: step u's kmin (-1: no pixel written), subpixel terms
#if SVX_ROW_ABLATE & 2
            if constexpr (DQ) {
                uint32_t acc = 0;
#pragma unroll
                for (int u = 0; u < U; ++u) acc ^= cc[u] ^ cp[u];
                if (acc == 0x9E3779B9u) gkey = 0;   // keeps the loads
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    cc[u] = nc[u];
                    cp[u] = np[u];
                }
                if (gkey >= 0) disp1[lane & 63] = 0;
                continue;
            }
#endif
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int xi = n - 1 - (j0 + u);
                if (xi < 0) break;
                int L0, L1, lm;
                uint32_t Lpk = 0;
                int P0, P1;
                if constexpr (DQ) {   // the byte sums of the low and the high nibbles (v_sad_u8 against 0)
                    uint32_t q;
                    Lpk = pk_l(cc[u], sb, k.P1, k.P2, q, lm);
                    L0 = lo16(Lpk);
                    L1 = hi16(Lpk);
                    P0 = sat16(4 * lo16(cc[u]) - (int)__builtin_amdgcn_sad_u8(cp[u] & 0x0F0F0F0Fu, 0u, 0u));
                    P1 = sat16(4 * hi16(cc[u]) - (int)__builtin_amdgcn_sad_u8((cp[u] >> 4) & 0x0F0F0F0Fu, 0u, 0u));
                } else {
                    lm = path_l(lo16(cc[u]), hi16(cc[u]), sb, k.P1, k.P2, L0, L1);
                    P0 = lo16(cp[u]);
                    P1 = hi16(cp[u]);
                }
                const int S0 = sat16(P0 + L0), S1 = sat16(P1 + L1);
                const int key = min(((S0 + 32768) << 7) | d0, ((S1 + 32768) << 7) | (d0 + 1));
                int wm, kmin;
                wave_min2_i32(lm, key, wm, kmin);
                if constexpr (DQ)
                    pk_commit(sb, cc[u], Lpk, wm);
                else
                    path_commit(sb, L0, L1, lm, wm);
                const int minS = (kmin >> 7) - 32768, best = kmin & 127;
                // a flag rather than `continue`: an exit from the unrolled step makes the compiler dispatch
                // each step's end through a state register (several scalar instructions and branches a step)
                // every S saturated: OpenCV's strict "<" never fires, bestDisp stays -1 and the pixel gets
                // (-1) * 16 = INVALID; disp2 is not touched (its cost test is strict too)
                bool write = minS != kMaxCost;
                if (k.uniq > 0) {
                    const bool bad = (S0 * (100 - k.uniq) < minS * 100 && abs(best - d0) > 1) ||
                                     (S1 * (100 - k.uniq) < minS * 100 && abs(best - d0 - 1) > 1);
                    if (__any(bad)) write = false;
                }
                int num = 0, dv = 1;   // dd = best * 16 + num / dv (C division)
                if (write && best > 0 && best < kSgD - 1) {
                    const uint32_t spk = pack16(S0, S1);
                    const uint32_t wm = (uint32_t)__builtin_amdgcn_readlane((int)spk, (best - 1) >> 1);
                    const uint32_t wp = (uint32_t)__builtin_amdgcn_readlane((int)spk, (best + 1) >> 1);
                    const int Sm = (best - 1) & 1 ? hi16(wm) : lo16(wm);
                    const int Sp = (best + 1) & 1 ? hi16(wp) : lo16(wp);
                    const int den = max(Sm + Sp - 2 * minS, 1);
                    num = (Sm - Sp) * kSgScale + den;
                    dv = den * 2;
                }
                if (write && lane == (uint32_t)u) {   // one v_cndmask each: the lane masks are loop invariants
                    gkey = kmin;
                    gnum = num;
                    gdv = dv;
                }
            }
            if (gkey >= 0) {   // lanes 0 .. U-1 whose step wrote a pixel
                const int xi = n - 1 - (j0 + (int)lane);
                const int best = gkey & 127, minS = (gkey >> 7) - 32768;
                disp1[xi + k.minX1] = (int16_t)(best * kSgScale + gnum / gdv);
                atomicMin(d2key + (xi + k.minX1 - best), (uint32_t)(minS + 32768) << 16 | (0xFFFFu - (uint32_t)xi));
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                cc[u] = nc[u];
                cp[u] = np[u];
            }
        }
    }
    wave_lds_sync();   // the group updates before the check reads them
    // left-right check -> the int16 result row; disp2 of column x from its key: -1 when never set, else
    // the best of the pixel xi that set it, xi + minX1 - x
    const auto disp2 = [&](int x) {
        const uint32_t kk = d2key[x];
        return kk == ~0u ? -1 : (int)(0xFFFFu - (kk & 0xFFFFu)) + k.minX1 - x;
    };
    int16_t* orow = d16 + (size_t)f * k.frame_px + (size_t)y * W;
    for (int x = lane; x < W; x += 64) {
        int v = disp1[x];
        if (v != INVALID) {
            const int _d = v >> 4, d_ = (v + kSgScale - 1) >> 4;
            const int _x = x - _d, x_ = x - d_;
            if (0 <= _x && _x < W && 0 <= x_ && x_ < W) {
                const int a = disp2(_x), b = disp2(x_);
                if (a >= 0 && abs(a - _d) > k.d12 && b >= 0 && abs(b - d_) > k.d12) v = INVALID;
            }
        }
        orow[x] = (int16_t)v;
    }
    if (__any(sa.ovf() || sb.ovf()) && lane == 0) atomicOr(flags + f, 1u);
}

// ---------------------------------------------------------------------------
// filterSpeckles: 4-connected components of pixels != newVal joined where
// |difference| <= maxDiff (union-find, hooking the larger root under the
// smaller), component sizes, then the speckle decision.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int cc_find(int32_t* par, int x) {
    int p = __atomic_load_n(par + x, __ATOMIC_RELAXED);
    while (p != x) {
        const int gp = __atomic_load_n(par + p, __ATOMIC_RELAXED);
        if (gp != p) __atomic_store_n(par + x, gp, __ATOMIC_RELAXED);   // path halving
        x = p;
        p = gp;
    }
    return x;
}

// Read-only find for the counting pass: once every union is done no path needs halving, and the counting
// pass's only writes are final roots into run starts (an earlier version stored every pixel's root while other
// threads' halving finds ran: a halving write could replace such a root with a mere ancestor).
__device__ __forceinline__ int cc_root(const int32_t* par, int x) {
    int p = __atomic_load_n(par + x, __ATOMIC_RELAXED);
    while (p != x) {
        x = p;
        p = __atomic_load_n(par + x, __ATOMIC_RELAXED);
    }
    return x;
}

__device__ __forceinline__ void cc_unite(int32_t* par, int a, int b) {
    a = cc_find(par, a);
    b = cc_find(par, b);
    while (a != b) {
        if (a > b) {
            const int t = a;
            a = b;
            b = t;
        }
        const int old = atomicCAS(par + b, b, a);
        if (old == b) break;
        b = old;   // b was hooked meanwhile: climb from its new parent
        a = cc_find(par, a);
        b = cc_find(par, b);
    }
}

// cv2.medianBlur(disp, disp, 3), which StereoSGBM::compute runs on the int16
// disparity right after computeDisparitySGBM (OpenCV 2.4 operator(), 3.x / 4.x
// StereoSGBMImpl::compute). OpenCV's sorting network gives the exact median of
// the 3 x 3 window with replicated borders; here each of the three columns is
// sorted (3 compare-exchanges) and median9 = med3(max of the column minima,
// med3 of the column medians, min of the column maxima), which is exact. A
// 1-row or 1-column image degenerates to OpenCV's 1-D median of 3 by itself
// (replicated columns / rows make the three columns equal / constant).
__device__ __forceinline__ int med3_i(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }

__global__ __launch_bounds__(256) void sgbm_median3_kernel(int H, int W, int64_t frame_px,
                                                             const int16_t* __restrict__ raw,
                                                             int16_t* __restrict__ out, int frames) {
    const int64_t f = blockIdx.y;   // grid (pixels of a frame, frames): no 64-bit division per pixel
    const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (f >= frames || p >= frame_px) return;
    const int64_t i = f * frame_px + p;
    const int y = p / W, x = p - y * W;
    const int16_t* d = raw + f * frame_px;
    const int16_t* r0 = d + (size_t)max(y - 1, 0) * W;
    const int16_t* r1 = d + (size_t)y * W;
    const int16_t* r2 = d + (size_t)min(y + 1, H - 1) * W;
    const int xs[3] = {max(x - 1, 0), x, min(x + 1, W - 1)};
    int lo[3], md[3], hi[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int a = r0[xs[j]], b = r1[xs[j]], c = r2[xs[j]];
        lo[j] = min(a, min(b, c));
        hi[j] = max(a, max(b, c));
        md[j] = med3_i(a, b, c);
    }
    const int v = med3_i(max(lo[0], max(lo[1], lo[2])), med3_i(md[0], md[1], md[2]), min(hi[0], min(hi[1], hi[2])));
    out[i] = (int16_t)v;
}

// Row runs: maximal horizontal runs of pixels != newVal whose neighbours differ
// by <= maxDiff. A run never needs a union inside it: every pixel's parent is
// its run's first pixel (one wave per row, a segmented max-scan of run starts).
__device__ __forceinline__ bool cc_link(int a, int b, const SgbmK& k) {
    return a != k.new_val && b != k.new_val && abs(a - b) <= k.max_diff;
}

// run start of lane's pixel x (x < W) given carry = start of the previous chunk's last pixel
__device__ __forceinline__ int cc_run_start(bool start, int x, int carry) {
    int v = start ? x + 1 : 0;   // 0 = "no start here"
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false));
    return v > 0 ? v - 1 : carry;
}

__global__ __launch_bounds__(256) void sgbm_cc_rows_kernel(SgbmK k, const int16_t* __restrict__ d16,
                                                             int32_t* __restrict__ parent, int frames) {
    const int gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int f = gw / k.H, y = gw - f * k.H;
    if (f >= frames) return;
    const int lane = lane_id(), W = k.W;
    const int16_t* d = d16 + (size_t)f * k.frame_px + (size_t)y * W;
    int32_t* par = parent + (size_t)f * k.frame_px + (size_t)y * W;
    int carry = 0;
    for (int x0 = 0; x0 < W; x0 += 64) {
        const int x = x0 + lane;
        const bool in = x < W;
        const int v = in ? d[x] : k.new_val;
        const int vl = in && x > 0 ? d[x - 1] : k.new_val;
        const int s = cc_run_start(in && !(x > 0 && cc_link(v, vl, k)), x, carry);
        if (in) par[x] = y * W + s;
        carry = __builtin_amdgcn_readlane(s, 63);
    }
}

// Vertical unions: pixel p with its lower neighbour q, skipped when p-1 / q-1
// are in the same runs as p / q and linked themselves (that union covered it).
__global__ __launch_bounds__(256) void sgbm_cc_union_kernel(SgbmK k, const int16_t* __restrict__ d16,
                                                              int32_t* __restrict__ parent, int frames) {
    const int64_t f = blockIdx.y;   // grid (pixels of a frame, frames): no 64-bit division per pixel
    const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (f >= frames || p >= k.frame_px) return;
    const int y = p / k.W, x = p - y * k.W;
    if (y + 1 >= k.H) return;
    const int16_t* d = d16 + f * k.frame_px;
    const int v = d[p], w = d[p + k.W];
    if (!cc_link(v, w, k)) return;
    if (x > 0) {
        const int vl = d[p - 1], wl = d[p + k.W - 1];
        if (cc_link(v, vl, k) && cc_link(w, wl, k) && cc_link(vl, wl, k)) return;
    }
    cc_unite(parent + f * k.frame_px, p, p + k.W);
}

// Component sizes: one wave per row; each run adds its length at its root,
// lanes sharing the wave's running root are summed first (large regions touch
// one address once per row, not once per run).
// Each run's end lane also points the run's first pixel straight at the root (a final value: every union is
// done, and readers following par see an ancestor or the root either way), so sgbm_out's finds take ~2 hops.
__global__ __launch_bounds__(256) void sgbm_cc_count_kernel(SgbmK k, const int16_t* __restrict__ d16,
                                                              int32_t* __restrict__ parent,
                                                              int32_t* __restrict__ size, int frames) {
    const int gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int f = gw / k.H, y = gw - f * k.H;
    if (f >= frames) return;
    const int lane = lane_id(), W = k.W;
    const int16_t* d = d16 + (size_t)f * k.frame_px + (size_t)y * W;
    int32_t* par = parent + (size_t)f * k.frame_px;
    int32_t* sz = size + (size_t)f * k.frame_px;
    int carry = 0, acc_root = -1, acc = 0;
    for (int x0 = 0; x0 < W; x0 += 64) {
        const int x = x0 + lane;
        const bool in = x < W;
        const int v = in ? d[x] : k.new_val;
        const int vl = in && x > 0 ? d[x - 1] : k.new_val;
        const int vr = x + 1 < W ? d[x + 1] : k.new_val;
        const int s = cc_run_start(in && !(x > 0 && cc_link(v, vl, k)), x, carry);
        carry = __builtin_amdgcn_readlane(s, 63);
        const bool end = in && v != k.new_val && !cc_link(v, vr, k);
        const int root = end ? cc_root(par, y * W + s) : -1;
        if (end && root != y * W + s) __hip_atomic_store(par + y * W + s, root, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int len = x - s + 1;
        const bool mine = end && root == acc_root;
        acc += (int)wave_sum(mine ? (uint32_t)len : 0u);   // (uniform loop: every lane active)
        const uint64_t rest = __ballot(end && !mine);
        if (rest) {
            // the first remaining run's root becomes the running root (flush the old one)
            const int r1 = __shfl(root, (int)__builtin_ctzll(rest), 64);
            const bool take = end && !mine && root == r1;
            const int add1 = (int)wave_sum(take ? (uint32_t)len : 0u);   // (`rest` is uniform: every lane active)
            if (lane == 0 && acc_root >= 0 && acc) atomicAdd(sz + acc_root, acc);
            acc_root = r1;
            acc = add1;
            if (end && !mine && !take) atomicAdd(sz + root, len);
        }
    }
    if (lane == 0 && acc_root >= 0 && acc) atomicAdd(sz + acc_root, acc);
}

// The speckle decision row by row (one wave a row, as the counting pass): a pixel's run start comes from the
// same segmented scan, its root is par[run start] (the counting pass pointed every run start at its root) and
// the root's size decides — two loads per run (the same address across the run's lanes), no per-pixel find.
__global__ __launch_bounds__(256) void sgbm_out_rows_kernel(SgbmK k, const int16_t* __restrict__ d16,
                                                            const int32_t* __restrict__ parent,
                                                            const int32_t* __restrict__ size,
                                                            uint8_t* __restrict__ out, int16_t* __restrict__ filt,
                                                            int frames) {
    const int gw = blockIdx.x * (blockDim.x >> 6) + wave_uniform_id();
    const int f = gw / k.H, y = gw - f * k.H;
    if (f >= frames) return;
    const int lane = lane_id(), W = k.W;
    const int16_t* d = d16 + (size_t)f * k.frame_px + (size_t)y * W;
    const int32_t* par = parent + (size_t)f * k.frame_px;
    const int32_t* sz = size + (size_t)f * k.frame_px;
    int carry = 0;
    for (int x0 = 0; x0 < W; x0 += 64) {
        const int x = x0 + lane;
        const bool in = x < W;
        int v = in ? d[x] : k.new_val;
        const int vl = in && x > 0 ? d[x - 1] : k.new_val;
        const int s = cc_run_start(in && !(x > 0 && cc_link(v, vl, k)), x, carry);
        carry = __builtin_amdgcn_readlane(s, 63);
        if (!in) continue;
        if (v != k.new_val) {
            const int root = __atomic_load_n(par + y * W + s, __ATOMIC_RELAXED);
            if (sz[root] <= k.max_size) v = k.new_val;
        }
        const int p = y * W + x;
        if (filt) filt[(size_t)f * k.frame_px + p] = (int16_t)v;
        if (!out) continue;
        const int ox = x - k.out_c0;
        if (y >= k.out_rows || ox < 0 || ox >= k.out_cols) continue;
        const int q = v > 0 ? v >> 4 : 0;   // TOZERO, then (d / 16.).astype(uint8)
        out[f * (int64_t)k.out_rows * k.out_stride + (int64_t)y * k.out_stride + ox] = (uint8_t)(int)((double)q * k.scale);
    }
}

// ---------------------------------------------------------------------------
// Front end: cv2.LUT, BGR2GRAY + equalizeHist, synthetic pairs.
// ---------------------------------------------------------------------------
__global__ void lut_kernel(const uint8_t* __restrict__ in, int64_t n, const uint8_t* __restrict__ lut,
                           uint8_t* __restrict__ out) {
    __shared__ uint8_t t[256];
    if (threadIdx.x < 256) t[threadIdx.x] = lut[threadIdx.x];
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = t[in[i]];
}

// lut (nullable): preProcessImages' gamma table (functions.py:81-87) applied to each channel as it is read, so
// the BGR pairs themselves are never rewritten (cv2.LUT returns a new image)
__global__ __launch_bounds__(256) void grey_hist_kernel(const uint8_t* __restrict__ bgr, int64_t px, int frames,
                                                          uint8_t* __restrict__ grey, uint32_t* __restrict__ hist,
                                                          const uint8_t* __restrict__ lut) {
    __shared__ uint32_t h[256];
    __shared__ uint8_t t[256];
    h[threadIdx.x] = 0;
    t[threadIdx.x] = lut ? lut[threadIdx.x] : (uint8_t)threadIdx.x;
    __syncthreads();
    const int64_t per = (px + gridDim.x - 1) / gridDim.x;   // gridDim.x blocks per frame in y
    const int f = blockIdx.y;
    const int64_t p0 = blockIdx.x * per, p1 = min(px, p0 + per);
    const uint8_t* src = bgr + (size_t)f * px * 3;
    for (int64_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
        const uint8_t* c = src + 3 * p;
        const int g = (t[c[0]] * 1868 + t[c[1]] * 9617 + t[c[2]] * 4899 + (1 << 13)) >> 14;
        grey[(size_t)f * px + p] = (uint8_t)g;
        atomicAdd(&h[g], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(hist + f * 256 + threadIdx.x, h[threadIdx.x]);
}

__global__ __launch_bounds__(256) void equalize_kernel(uint8_t* __restrict__ grey, int64_t px,
                                                         const uint32_t* __restrict__ hist) {
    __shared__ uint8_t lut[256];
    const int f = blockIdx.y;
    const uint32_t* h = hist + f * 256;
    if (threadIdx.x == 0) {
        int i = 0;
        while (i < 255 && !h[i]) ++i;
        if ((int64_t)h[i] == px) {
            for (int j = 0; j < 256; ++j) lut[j] = (uint8_t)i;   // a constant image keeps its value
        } else {
            const float scale = 255.f / (float)(px - (int64_t)h[i]);
            int64_t sum = 0;
            lut[i] = 0;
            for (int j = i + 1; j < 256; ++j) {
                sum += h[j];
                const float v = __fmul_rn((float)sum, scale);
                const int r = (int)rintf(v);
                lut[j] = (uint8_t)(r < 0 ? 0 : r > 255 ? 255 : r);
            }
            for (int j = 0; j < i; ++j) lut[j] = 0;
        }
    }
    __syncthreads();
    uint8_t* g = grey + (size_t)f * px;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < px; p += (int64_t)gridDim.x * blockDim.x)
        g[p] = lut[g[p]];
}

__global__ void synth_pair_kernel(uint8_t* __restrict__ left, uint8_t* __restrict__ right, int H, int W, int frames,
                                  int64_t first) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t px = (int64_t)H * W;
    const int64_t f = i / px;
    if (f >= frames) return;
    const int p = (int)(i - f * px);
    const int y = p / W, x = p - y * W;
    const int D = sgbm_pair_disparity(y);
    left[i] = sgbm_pair_texture(first + f, H, y, x);
    right[i] = sgbm_pair_texture(first + f, H, y, x + D);
}

__global__ void synth_bgr_pair_kernel(uint8_t* __restrict__ left, uint8_t* __restrict__ right, int H, int W,
                                      int frames, int64_t first) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t px = (int64_t)H * W;
    const int64_t f = i / px;
    if (f >= frames) return;
    const int p = (int)(i - f * px);
    const int y = p / W, x = p - y * W;
    const int D = sgbm_pair_disparity(y);
#pragma unroll
    for (int side = 0; side < 2; ++side) {
        const int u = side ? x + D : x;   // the scene column this pixel sees
        const int t = sgbm_pair_texture(first + f, H, y, u);
        // channel jitter of the scene point (a second texture draw), same in both views
        const int j = sgbm_pair_texture(first + f + 0x4000000000ll, H, y, u);
        uint8_t* o = (side ? right : left) + 3 * i;
        o[0] = (uint8_t)t;
        o[1] = (uint8_t)min(255, t + (j & 31));
        o[2] = (uint8_t)max(0, t - ((j >> 3) & 31));
    }
}

__global__ __launch_bounds__(256) void copy_bgr_region_kernel(const uint8_t* __restrict__ src, int Hp, int Wp,
                                                              uint8_t* __restrict__ dst, int H, int W, int Wu,
                                                              const uint8_t* __restrict__ lut) {
    __shared__ uint8_t t[256];
    t[threadIdx.x] = lut ? lut[threadIdx.x] : (uint8_t)threadIdx.x;
    __syncthreads();
    const int row = blockIdx.x, f = blockIdx.y;   // row < H <= Hp
    const uint8_t* s = src + ((int64_t)f * Hp + row) * Wp * 3;
    uint8_t* d = dst + ((int64_t)f * H + row) * W * 3;
    for (int b = threadIdx.x; b < 3 * Wu; b += blockDim.x) d[b] = t[s[b]];
}

}  // namespace

hipError_t launch_synth_bgr_pair(uint8_t* left, uint8_t* right, int H, int W, int frames, int64_t first,
                                 hipStream_t s) {
    const int64_t n = (int64_t)frames * H * W;
    hipLaunchKernelGGL(synth_bgr_pair_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, left, right, H, W,
                       frames, first);
    return hipGetLastError();
}

hipError_t launch_copy_bgr_region(const uint8_t* src, int Hp, int Wp, uint8_t* dst, int H, int W, int Wu, int frames,
                                  hipStream_t s, const uint8_t* lut) {
    if (frames <= 0 || H <= 0) return hipSuccess;
    if (H > Hp || Wu > Wp || Wu > W) return hipErrorInvalidValue;
    hipLaunchKernelGGL(copy_bgr_region_kernel, dim3((unsigned)H, (unsigned)frames), dim3(256), 0, s, src, Hp, Wp, dst,
                       H, W, Wu, lut);
    return hipGetLastError();
}

// steps each path walk keeps in flight (SVX_SGBM_PF: 1, 4 or 8; A/B only; 16 measured no faster)
static int sgbm_prefetch() {
    const char* e = svx_knob("SVX_SGBM_PF");
    return e && *e ? std::atoi(e) : 8;
}

bool sgbm_supported(const SgbmK& k) {
    // the walks address a frame's volume through buffer resources with 32-bit byte offsets (wave_rsrc): a frame's
    // int16 volume, diagonal stride included, stays below 2^31 bytes
    const size_t frame_vol = (size_t)(k.H + 1) * ((size_t)k.width1 * 64 + 64) * sizeof(uint32_t);
    return k.width1 > k.SW2 && k.W <= 2048 && k.H >= 1 && k.SW2 >= 0 && k.SW2 <= 31 && frame_vol < 0x7FFFFFFFu;
}

size_t sgbm_volume_bytes(const SgbmK& k) { return (size_t)k.H * k.width1 * kSgD * sizeof(int16_t); }

hipError_t launch_sgbm_compute(const SgbmK& k, const uint8_t* left, const uint8_t* right, int frames,
                               const SgbmScratch& s, hipStream_t st) {
    const int H = k.H;
    hipError_t e = hipMemsetAsync(s.flags, 0, sizeof(uint32_t) * frames, st);
    if (e != hipSuccess) return e;
    // hsum: features (4 W words) + byte values (W words) + 4 waves' rings
    // (the register-ring walk for the reference's block 21: features (24 W bytes, the staged rows (6 W) under
    // them) + byte values (4 W); SVX_SGBM_HRING=0: the generic kernel)
    const char* hr = svx_knob("SVX_SGBM_HRING");
#ifdef SVX_DIAG
    const char* ha = svx_knob("SVX_SGBM_HSUM_ABLATE");
    const int habl = ha && *ha ? std::atoi(ha) : 0;
#else
    constexpr int habl = 0;
#endif
    if (k.SW2 == 10 && !(hr && hr[0] == '0')) {
        if (habl == 0)
            hipLaunchKernelGGL(sgbm_hsum_ring_kernel<10>, dim3(frames * H), dim3(256), 28 * (size_t)k.W, st, k, left,
                               right, s.hl1, frames);
#ifdef SVX_DIAG
        else if (habl == 1)
            hipLaunchKernelGGL((sgbm_hsum_ring_kernel<10, 1>), dim3(frames * H), dim3(256), 28 * (size_t)k.W, st, k,
                               left, right, s.hl1, frames);
        else if (habl == 2)
            hipLaunchKernelGGL((sgbm_hsum_ring_kernel<10, 2>), dim3(frames * H), dim3(256), 28 * (size_t)k.W, st, k,
                               left, right, s.hl1, frames);
        else
            hipLaunchKernelGGL((sgbm_hsum_ring_kernel<10, 3>), dim3(frames * H), dim3(256), 28 * (size_t)k.W, st, k,
                               left, right, s.hl1, frames);
#endif
    } else {
        const size_t lds1 = sizeof(uint32_t) * (5 * (size_t)k.W + 4 * (2 * k.SW2 + 1) * 64);
        hipLaunchKernelGGL(sgbm_hsum_kernel, dim3(frames * H), dim3(256), lds1, st, k, left, right, s.hl1, frames);
    }
    const int cb = (k.width1 + 3) / 4;
    const int paths = 2 * (k.width1 + H - 1) * frames;
    const size_t lds4 = sgbm_row_lds_per_wave(k.W) * 4;
    const int pf = sgbm_prefetch();
    // the register-ring vertical walk for the reference's block 21 (SVX_SGBM_VRING=0: the generic walk)
    const char* vr = svx_knob("SVX_SGBM_VRING");
    const bool vring = k.SH2 == 10 && !(vr && vr[0] == '0');
    // non-temporal loads of the volumes the row walk reads for the last time, and of its P: 26.40 vs 26.48 ms per
    // 64 frames, faster in 4 of 5 alternations (SVX_SGBM_NT=0: plain accesses; A/B)
    const char* ntv = svx_knob("SVX_SGBM_NT");
    const bool nt = !(ntv && ntv[0] == '0');
    // the q-byte volumes of the four directions the row walk sums (P2 <= 15; SVX_SGBM_DQ=0: int16 L volumes and
    // P, A/B): four volumes of 64 B a cell in the space of the fourth int16 volume
    const char* dqv = svx_knob("SVX_SGBM_DQ");
    const bool dq = k.P1 >= 0 && k.P2 <= 15 && !(dqv && dqv[0] == '0');
    const size_t qb = (size_t)frames * H * k.width1 * 64;
    uint8_t* q0 = reinterpret_cast<uint8_t*>(s.l3);
    uint8_t* q1 = q0 + qb;
    uint8_t* q2 = q1 + qb;
    uint8_t* q3 = q2 + qb;
#define SVX_SGBM_WALKS(U, DQ)                                                                                     \
    if (vring)                                                                                                    \
        hipLaunchKernelGGL((sgbm_vertical_ring_kernel<10, DQ>), dim3(frames * cb), dim3(256), 0, st, k, s.hl1,   \
                           s.c, s.l2, q2, s.flags, frames);                                                       \
    else                                                                                                          \
        hipLaunchKernelGGL((sgbm_vertical_kernel<U, DQ>), dim3(frames * cb), dim3(256), 0, st, k, s.hl1, s.c,    \
                           s.l2, q2, s.flags, frames);                                                            \
    hipLaunchKernelGGL((sgbm_diag_kernel<U, DQ>), dim3((paths + 3) / 4), dim3(256), 0, st, k, s.c, s.hl1, s.l3,  \
                       q1, q3, s.flags, frames);                                                                  \
    if (nt)                                                                                                       \
        hipLaunchKernelGGL((sgbm_row_kernel<U, true, DQ>), dim3((frames * H + 3) / 4), dim3(256), lds4, st, k,   \
                           s.c, s.hl1, s.l2, s.l3, q0, q1, q2, q3, s.raw, s.flags, frames);                           \
    else                                                                                                          \
        hipLaunchKernelGGL((sgbm_row_kernel<U, false, DQ>), dim3((frames * H + 3) / 4), dim3(256), lds4, st, k,  \
                           s.c, s.hl1, s.l2, s.l3, q0, q1, q2, q3, s.raw, s.flags, frames)
    if (dq) {
        SVX_SGBM_WALKS(8, true);
    } else if (pf == 1) {
        SVX_SGBM_WALKS(1, false);
    } else if (pf == 4) {
        SVX_SGBM_WALKS(4, false);
    } else {
        SVX_SGBM_WALKS(8, false);
    }
#undef SVX_SGBM_WALKS
    // StereoSGBM::compute's medianBlur(disp, disp, 3): raw -> d16 (grid: a frame's pixels x frames)
    if (frames > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(sgbm_median3_kernel, dim3((unsigned)((k.frame_px + 255) / 256), (unsigned)frames), dim3(256), 0,
                       st, k.H, k.W, k.frame_px, s.raw, s.d16, frames);
    return hipGetLastError();
}

hipError_t launch_speckle_scale(const SgbmK& k, int frames, const SgbmScratch& s, uint8_t* out, int16_t* filt,
                                hipStream_t st) {
    const int64_t n = (int64_t)frames * k.frame_px;
    if (frames > 65535) return hipErrorInvalidValue;   // the pixel kernels' grid: a frame's pixels x frames
    const unsigned rows = (unsigned)((frames * k.H + 3) / 4);   // one wave per row
    hipLaunchKernelGGL(sgbm_cc_rows_kernel, dim3(rows), dim3(256), 0, st, k, s.d16, s.parent, frames);
    hipLaunchKernelGGL(sgbm_cc_union_kernel, dim3((unsigned)((k.frame_px + 255) / 256), (unsigned)frames), dim3(256), 0,
                       st, k, s.d16, s.parent, frames);
    hipError_t e = hipMemsetAsync(s.size, 0, sizeof(int32_t) * n, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(sgbm_cc_count_kernel, dim3(rows), dim3(256), 0, st, k, s.d16, s.parent, s.size, frames);
    hipLaunchKernelGGL(sgbm_out_rows_kernel, dim3(rows), dim3(256), 0, st, k, s.d16, s.parent, s.size, out, filt,
                       frames);
    return hipGetLastError();
}

hipError_t launch_lut(const uint8_t* in, int64_t n, const uint8_t* lut, uint8_t* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n + 1023) / 1024, 8192);
    hipLaunchKernelGGL(lut_kernel, dim3((unsigned)blocks), dim3(256), 0, s, in, n, lut, out);
    return hipGetLastError();
}

hipError_t launch_grey_equalize(const uint8_t* bgr, int64_t px, int frames, uint8_t* grey, uint32_t* hist,
                                hipStream_t s, const uint8_t* lut) {
    hipError_t e = hipMemsetAsync(hist, 0, sizeof(uint32_t) * 256 * frames, s);
    if (e != hipSuccess) return e;
    const unsigned bx = (unsigned)std::min<int64_t>((px + 4095) / 4096, 256);
    hipLaunchKernelGGL(grey_hist_kernel, dim3(bx, frames), dim3(256), 0, s, bgr, px, frames, grey, hist, lut);
    hipLaunchKernelGGL(equalize_kernel, dim3(bx, frames), dim3(256), 0, s, grey, px, hist);
    return hipGetLastError();
}

hipError_t launch_synth_pair(uint8_t* left, uint8_t* right, int H, int W, int frames, int64_t first, hipStream_t s) {
    const int64_t n = (int64_t)frames * H * W;
    hipLaunchKernelGGL(synth_pair_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, left, right, H, W,
                       frames, first);
    return hipGetLastError();
}

}  // namespace svx
