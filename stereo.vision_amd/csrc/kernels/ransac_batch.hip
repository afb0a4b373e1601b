// Batched RANSAC on the device ("batched-friendly").
//
//  * maskpoints_kernel — stereovision.py:85 for every frame of a batch:
//      projectDisparityTo3d(maskDisparity(disparity), 128) = the fp64 X, Y, Z of
//      every d > 0 grid point of the masked disparity on the reference's step-2
//      grid (functions.py:185-193), in raster order, same arithmetic as the
//      drop-in (bit-identical). One workgroup per frame, running offset,
//      LDS-staged coalesced output.
//  * ransac_draw_kernel — the draws of functions.py:278-298 for every frame,
//      with the batch RNG contract: frame F draws CPython's stream after
//      random.seed(seed_base + F). One wave per frame replays the stream:
//      init_by_array seeding (one lane), the MT19937 state advanced one
//      dependency level of the next twist at a time as the stream moves
//      (no copy of the outputs: tempered on read), _randbelow /
//      random.sample consumed 64 draws at a time (a ballot finds the
//      accepted draws, an LDS bitmap the already-selected indices, draws
//      repeated inside one round resolved in lane = stream order), then the
//      three sample(points, 1) draws and numpy's cross-product test
//      (functions.py:240-260), redrawn while collinear. Writes every trial's
//      sample and triple to memory.
//  * ransac_eval_kernel — one workgroup per frame: the frame's packed points
//      staged in LDS; every trial's plane solved from its triple with numpy's
//      rounding (the LAPACK dgesv + dot of functions.py:267 restated, round 3),
//      every trial screened in fp32 from LDS (one wave per trial, a rigorous
//      bound to the fp64 mean), then the trials the screen cannot rule out
//      evaluated in fp64 exactly as numpy does (the gemv's fmas, the pairwise
//      sum of np.mean) and the first strict minimum kept (functions.py:289-293):
//      the plane, its error and the winning trial are numpy's, bit for bit.
//   (One kernel doing both, wave 0 drawing beside wave 1 evaluating, was
//   bound by the screen's random 4-byte gathers: ~94 GB of sector traffic per
//   4096 frames, the points of the ~4096 frames in flight not fitting L2.)
#include "../svx_launch.h"

namespace svx {

// A maskpoint as (x, y, d) pixel coordinates in one word: x | y << 12 | d << 24
// (W, H <= 4096). Its fp64 X, Y, Z are a function of these (functions.py:191-193).
__device__ __forceinline__ uint32_t rb_pack(int x, int y, uint32_t d) {
    return (uint32_t)x | ((uint32_t)y << 12) | (d << 24);
}

// A packed maskpoint's fp64 X, Y, Z with the reference's arithmetic
// (functions.py:191-193): Z = fB / d, X = ((x - cw) * Z) / f, Y = ((y - ch) *
// Z) / f. On the step-2 grid X depends on (x / 2, d) only and Y on (y / 2, d),
// so the three are gathered from tables the batch builds once per call
// (ransac_tables_kernel, the same fp64 operations, -ffp-contract=off): a point
// costs three independent gathers (L2-resident: (W/2 + H/2 + 1) x 256 doubles)
// and no division on the RANSAC kernels' chains. Bit-identical to the
// reference's values (tests/test_gpu_ransac_batch.py reads them back).
struct RbTables {
    const double* X;   // [(W/2) x 256]: X of column x = 2 i at disparity d
    const double* Y;   // [(H/2) x 256]
    const double* Z;   // [256]
};

__device__ __forceinline__ void rb_point(uint32_t pk, const RbTables& t, double& X, double& Y, double& Z) {
    const uint32_t x2 = (pk & 0xFFF) >> 1, y2 = ((pk >> 12) & 0xFFF) >> 1, d = pk >> 24;
    X = t.X[x2 * 256 + d];
    Y = t.Y[y2 * 256 + d];
    Z = t.Z[d];
}

// the tables for a frame of H x W (step 2): X rows 0..W/2-1, then Y rows 0..H/2-1, then Z
__global__ void ransac_tables_kernel(int H, int W, KParams p, double* __restrict__ tab) {
    const int nx = (W + 1) / 2, ny = (H + 1) / 2;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (nx + ny + 1) * 256; i += gridDim.x * blockDim.x) {
        const int row = i >> 8, d = i & 255;
        const double Z = d ? p.fB / (double)d : 0.0;   // functions.py:191
        double v;
        if (row < nx) v = (((double)(2 * row) - p.cw) * Z) / p.f;             // :192
        else if (row < nx + ny) v = (((double)(2 * (row - nx)) - p.ch) * Z) / p.f;   // :193
        else v = Z;
        tab[i] = v;
    }
}

size_t ransac_tables_bytes(int H, int W) { return sizeof(double) * 256 * (size_t)((W + 1) / 2 + (H + 1) / 2 + 1); }

static RbTables rb_tables(const double* tab, int H, int W) {
    const int nx = (W + 1) / 2, ny = (H + 1) / 2;
    return RbTables{tab, tab + 256 * (size_t)nx, tab + 256 * (size_t)(nx + ny)};
}

// ---------------------------------------------------------------------------
// maskpoints: step-2 grid of the (optionally masked) disparity -> packed points
// (the fp64 X, Y, Z of a point are a function of its packed word: rb_point)
// ---------------------------------------------------------------------------
// One lane = one quad (4 consecutive grid points of a row): an 8-byte load of
// the row's pixels 8q..8q+7 holds the quad's 4 step-2 disparities (and one of
// the mask). The chunk's packed points go to LDS in output order, then out as
// contiguous words (coalesced). (Until round 3 the fp64 X, Y, Z were written
// too: 24 B per point, 2.6 GB per 4096 carmask frames, read back only by a few
// gathers; they are now computed where used, rb_point.)
struct MaskpointsShared {
    uint32_t wtot[4];
    uint32_t pk[1024];
};

__global__ __launch_bounds__(256) void maskpoints_kernel(const uint8_t* __restrict__ disp,
                                                         const uint8_t* __restrict__ mask_ff, int64_t frame_px,
                                                         int H, int W, KParams p,
                                                         uint32_t* __restrict__ packed, int64_t cap,
                                                         int64_t* __restrict__ counts) {
    __shared__ MaskpointsShared sh;
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.x;
    const uint8_t* fd = disp + (int64_t)frame * frame_px;
    uint32_t* fpk = packed + (int64_t)frame * cap;
    const int Hg = p.Hg, Wg = p.Wg;   // range(0, H-1, 2) x range(0, Wu-1, 2); W is the row stride
    const int Wq = (Wg + 3) / 4;
    const int64_t nq = (int64_t)Hg * Wq;
    const bool wide = (W % 4) == 0 && (reinterpret_cast<uintptr_t>(fd) & 7) == 0 &&
                      (!mask_ff || (reinterpret_cast<uintptr_t>(mask_ff) & 7) == 0);   // uniform
    uint32_t running = 0;
    for (int64_t base = 0; base < nq; base += 256) {
        const int64_t qi = base + tid;
        uint32_t dv[4] = {0, 0, 0, 0};
        int gy = 0, gx0 = 0;
        if (qi < nq) {
            gy = (int)(qi / Wq);
            gx0 = 4 * (int)(qi - (int64_t)gy * Wq);
            const int64_t px = (int64_t)(2 * gy) * W + 2 * gx0;
            if (wide && gx0 + 3 < Wg) {
                uint2 d8 = *reinterpret_cast<const uint2*>(fd + px);
                if (mask_ff) {
                    const uint2 m8 = *reinterpret_cast<const uint2*>(mask_ff + px);
                    d8.x &= m8.x;
                    d8.y &= m8.y;
                }
                dv[0] = d8.x & 0xFF;
                dv[1] = (d8.x >> 16) & 0xFF;
                dv[2] = d8.y & 0xFF;
                dv[3] = (d8.y >> 16) & 0xFF;
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (gx0 + k >= Wg) break;
                    uint32_t d = fd[px + 2 * k];
                    if (mask_ff) d &= mask_ff[px + 2 * k];
                    dv[k] = d;
                }
            }
        }
        uint32_t m = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) m |= (dv[k] != 0) << k;
        const uint32_t cnt = __builtin_popcount(m);
        const uint32_t inc = wave_incl_scan(cnt);
        if (lane == 63) sh.wtot[wave] = inc;
        __syncthreads();   // also: the previous chunk's writes have read sh.stage
        uint32_t wbase = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            wbase += w < wave ? sh.wtot[w] : 0u;
            tot += sh.wtot[w];
        }
        uint32_t o = wbase + inc - cnt;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (!(m & (1u << k))) continue;
            sh.pk[o++] = rb_pack(2 * (gx0 + k), 2 * gy, dv[k]);   // functions.py:191-193: rb_point
        }
        __syncthreads();   // sh.pk complete; sh.wtot free
        for (uint32_t j = tid; j < tot; j += 256) fpk[running + j] = sh.pk[j];
        running += tot;
    }
    if (tid == 0) counts[frame] = running;
}

hipError_t launch_maskpoints(const uint8_t* disp, const uint8_t* mask_ff, int frames, int H, int W, const KParams& p,
                             uint32_t* packed, int64_t cap, int64_t* counts, hipStream_t s) {
    if (frames <= 0) return hipSuccess;
    if (H > 4096 || W > 4096) return hipErrorInvalidValue;   // rb_pack's 12-bit coordinates
    hipLaunchKernelGGL(maskpoints_kernel, dim3(frames), dim3(256), 0, s, disp, mask_ff, (int64_t)H * W, H, W, p,
                       packed, cap, counts);
    return hipGetLastError();
}

// n packed points -> n x 3 fp64 (rb_point): the read-back of one frame's maskpoints
__global__ void maskpoints_xyz_kernel(const uint32_t* __restrict__ packed, int64_t n, RbTables t,
                                      double* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        double X, Y, Z;
        rb_point(packed[i], t, X, Y, Z);
        out[3 * i] = X;
        out[3 * i + 1] = Y;
        out[3 * i + 2] = Z;
    }
}

hipError_t launch_ransac_tables(int H, int W, const KParams& p, double* tab, hipStream_t s) {
    const int n = 256 * ((W + 1) / 2 + (H + 1) / 2 + 1);
    hipLaunchKernelGGL(ransac_tables_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, H, W, p, tab);
    return hipGetLastError();
}

hipError_t launch_maskpoints_xyz(const uint32_t* packed, int64_t n, const double* tab, int H, int W, double* out,
                                 hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(maskpoints_xyz_kernel, dim3(g), dim3(256), 0, s, packed, n, rb_tables(tab, H, W), out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// RANSAC, one workgroup per frame
// ---------------------------------------------------------------------------
constexpr int kRBMaxK = 1024;          // sample size limit
constexpr int kRBMaxTrials = 4096;     // the eval kernel keeps two doubles per trial in LDS
constexpr int kRBBitmapWords = 5120;   // 20 KB: the set branch for n <= 163,840 points
// randomNonCollinearPoints loops for ever on degenerate input (every triple
// collinear); the kernel gives up after this many attempts in one trial and
// flags the frame (8) instead of hanging the device
constexpr int kRBMaxAttempts = 1 << 16;
// every loop of the replay advances the stream; past this many draws in one
// frame (240k trials of 600) the frame stops with flag 16, so no input can keep
// a wave spinning
constexpr uint32_t kRBMaxDraws = 1u << 28;
// the pool branch's list (<= k words) shares the bitmap's words

// LDS of one frame: a fixed part (static) and, in dynamic LDS sized by the
// launch for the batch's largest frame, the sample bitmap (set branch) or the
// pool list (pool branch) and the two trial samples. RansacShared is the view
// (pointers into LDS, kept in registers) the device functions take.
template <class IdxT>
struct RansacShared {
    uint32_t* mt;
    uint32_t* bitmap;                         // set branch: selected indices of the current sample
    uint32_t* pool_list;                      // pool branch: the virtual pool's entries (same words, <= k)
    int k;
    uint32_t spread;                          // (a power of two, <= the bitmap's words) - 1: rejected claims' words
    int ablate;                               // DIAGNOSTIC (SVX_RANSAC_ABLATE, diag build)
};

// CPython's init_genrand + init_by_array (Modules/_randommodule.c) for a
// non-negative seed < 2^64: key = its 32-bit words, little-endian, at least one.
__device__ void rb_seed(uint32_t* mt, uint64_t seed) {
    mt[0] = 19650218u;
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    const int klen = (seed >> 32) ? 2 : 1;
    int i = 1, j = 0;
    for (int k = 624; k; --k) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        ++i;
        ++j;
        if (i >= 624) {
            mt[0] = mt[623];
            i = 1;
        }
        if (j >= klen) j = 0;
    }
    for (int k = 623; k; --k) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        ++i;
        if (i >= 624) {
            mt[0] = mt[623];
            i = 1;
        }
    }
    mt[0] = 0x80000000u;
}

// Wave 0's lanes hand data to each other through LDS with no workgroup
// barrier. The hardware keeps one wave's LDS operations in order, but the
// compiler reasons per lane (lane i's store to mt[j] never aliases lane i's
// load of mt[j - 35]) and may move loads above earlier stores: every hand-off
// between lanes goes through this point (a compiler memory barrier + LDS wait).
__device__ __forceinline__ void rb_wave_lds_sync() { __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ double rb_readlane_f64(double v, int l) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
}
// the wave's lane mask of a condition, straight from the compare (no 0/1 register in between)
__device__ __forceinline__ uint64_t rb_ballot(bool c) { return __builtin_amdgcn_ballot_w64(c); }

// MT19937 tempering; each masked step is a shift and one 3-input v_bitop3
// ((a & b) ^ c: truth table 0x6a)
__device__ __forceinline__ uint32_t rb_temper(uint32_t y) {
    y ^= (y >> 11);
#ifndef SVX_RB_NO_BITOP3
    y = __builtin_amdgcn_bitop3_b32(y << 7, 0x9d2c5680u, y, 0x6a);
    y = __builtin_amdgcn_bitop3_b32(y << 15, 0xefc60000u, y, 0x6a);
#else
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
#endif
    y ^= (y >> 18);
    return y;
}

// One dependency level of an MT19937 twist of mt (in place, one wave). The
// sequential in-place recurrence new[kk] = f(old[kk], old[kk+1], src) reads src
// = old[kk+397] for kk < 227 and new[kk-227] above, so it has three levels: [0,
// 227) from old words only, [227, 454) from level 1, [454, 624) from level 2
// (word 623 also reads new[0]). Within a level every lane reads all its inputs
// (up to 4 words a lane) before any lane writes, so no read sees a word of its
// own level already replaced. Branch-free: a lane's slot past the level's end
// computes from the clamped word hi - 1 and stores that word's new value again (the same value its owner stores:
// no LDS word is spent on a dump).
template <int LEV>
__device__ __forceinline__ void rb_twist_level(uint32_t* mt) {
    constexpr uint32_t UPPER = 0x80000000u, LOWER = 0x7fffffffu, A = 0x9908b0dfu;
    constexpr int lo = LEV == 0 ? 0 : LEV == 1 ? 227 : 454;
    constexpr int hi = LEV == 0 ? 227 : LEV == 1 ? 454 : 624;
    constexpr int NJ = (hi - lo + 63) / 64;
    const int lane = lane_id();
    uint32_t nv[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        int kk = lo + lane + 64 * j;
        if (lo + 64 * j + 63 >= hi) kk = min(kk, hi - 1);   // (compile-time: the level's last, partial slot)
        const uint32_t nxt = mt[LEV == 2 && kk == 623 ? 0 : kk + 1];
        const uint32_t y = (mt[kk] & UPPER) | (nxt & LOWER);
        const uint32_t src = LEV == 0 ? mt[kk + 397] : mt[kk - 227];
        nv[j] = src ^ (y >> 1) ^ ((y & 1u) ? A : 0u);
    }
    rb_wave_lds_sync();   // every read of this level before any write of it
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        int kk = lo + lane + 64 * j;
        if (lo + 64 * j + 63 >= hi) kk = min(kk, hi - 1);
        mt[kk] = nv[j];
    }
    rb_wave_lds_sync();   // the next level reads this one's words
}

// The stream without a copy of the outputs: the state words are advanced one
// dependency level of the next twist at a time, as the stream moves. With T
// whole twists and `lev` levels of twist T + 1 done, word w holds twist T + 1
// for w below the level boundary B[lev] (0, 227, 454) and twist T above, i.e.
// the state is exactly stream positions [G - 624, G), G = 624 T + B[lev]
// (position q = 624 (twist - 1) + word), and output q = temper(mt[q % 624]).
// A request [pos, pos + span) with span <= 192 advances levels while
// pos + span > G; a level moves G by at most 227, so the positions it drops
// (below the new G - 624 < pos + span - 397) were consumed already.
struct RbStream {   // wave 0's view of the frame's output stream (uniform)
    uint32_t pos = 0;   // next unconsumed output
    uint32_t pm = 0;    // pos % 624, kept as pos moves (a step is < 624)
    uint32_t G = 0;     // 624 x (whole twists done) + the level boundary (0, 227, 454) of the next one
    int lev = 0;        // levels of the next twist done (0..2)
    __device__ void step(uint32_t d) {
        pos += d;
        pm += d;
        pm -= pm >= 624u ? 624u : 0u;
    }
};

template <class IdxT>
__device__ __forceinline__ void rb_advance(RansacShared<IdxT>& sh, RbStream& st, uint32_t span) {
    while (st.pos + span > st.G) {
        if (st.lev == 0) rb_twist_level<0>(sh.mt);
        else if (st.lev == 1) rb_twist_level<1>(sh.mt);
        else rb_twist_level<2>(sh.mt);
        st.G += st.lev == 2 ? 170u : 227u;
        st.lev = st.lev == 2 ? 0 : st.lev + 1;
    }
}

// output pos + lane (lane < 64): state word (pm + lane) mod 624
template <class IdxT>
__device__ __forceinline__ uint32_t rb_word_at(const RansacShared<IdxT>& sh, const RbStream& st, uint32_t lane) {
    uint32_t i = st.pm + lane;
    i -= i >= 624u ? 624u : 0u;
    return rb_temper(sh.mt[i]);
}

// numpy.cross(P1 - P2, P2 - P3) all zero (functions.py:255-258); products rounded first
__device__ __forceinline__ bool rb_collinear(const double* p1, const double* p2, const double* p3) {
    const double a0 = p1[0] - p2[0], a1 = p1[1] - p2[1], a2 = p1[2] - p2[2];
    const double b0 = p2[0] - p3[0], b1 = p2[1] - p3[1], b2 = p2[2] - p3[2];
    const double c0 = a1 * b2 - a2 * b1, c1 = a2 * b0 - a0 * b2, c2 = a0 * b1 - a1 * b0;
    return c0 == 0.0 && c1 == 0.0 && c2 == 0.0;
}

// wave 0: k accepted draws of randbelow(n) in stream order -> out[0..m) (m <= 3)
template <class IdxT>
__device__ void rb_draw_below(RansacShared<IdxT>& sh, RbStream& st, uint32_t n, int kb, int m, uint32_t* out) {
    const int lane = lane_id();
    int got = 0;
    while (got < m && st.pos < kRBMaxDraws) {
        rb_advance(sh, st, 64u);
        const uint32_t r = rb_word_at(sh, st, (uint32_t)lane) >> (32 - kb);
        uint64_t acc = rb_ballot(r < n);
        int last = 63;
        while (acc && got < m) {
            const int l = __builtin_ctzll(acc);
            acc &= acc - 1;
            out[got++] = __builtin_amdgcn_readlane(r, l);   // l is wave-uniform: a scalar read
            last = l;
        }
        st.step((got == m) ? (uint32_t)(last + 1) : 64u);
    }
}

// wave 0: random.sample(range(n), k) into idx (set branch), then clear the bits.
// A round takes kRBWin windows of 64 draws (stream positions pos + 64 w + lane):
// every accepted draw claims its index bit with atomicOr, whose return says
// whether the bit was already set. LDS executes one wave's operations in
// order, so a window sees the claims of every earlier window; a set bit means
// an index selected earlier (rejected) or a value drawn twice in the same
// window, resolved by ballots: if some lane saw the bit clear, the value is new
// and its lowest lane (earliest draw) wins, otherwise every lane drawing it is
// rejected. The k-th selection in stream order ends the sample and the stream
// resumes right after it (bits claimed past it stay: the bitmap is cleared).
// 192 draws a round; a round must fit the state's 624 positions (RbStream): span <= 397, i.e. up to 6 windows
#ifndef SVX_RB_WIN
#define SVX_RB_WIN 3
#endif
constexpr int kRBWin = SVX_RB_WIN;
static_assert(kRBWin >= 1 && 64 * kRBWin <= 397, "a round's draws must fit the MT state (RbStream)");

template <class IdxT, bool TR>
__device__ void rb_sample_set(RansacShared<IdxT>& sh, RbStream& st, uint32_t n, int kb, int k, IdxT* idx,
                              int32_t* tr) {
    const int lane = lane_id();
    int have = 0;
    uint32_t r[kRBWin];
    while (have < k && st.pos < kRBMaxDraws) {
        rb_advance(sh, st, 64u * kRBWin);
        const uint32_t base = st.pm;
        uint32_t old[kRBWin];
#pragma unroll
        for (int w = 0; w < kRBWin; ++w) {
            uint32_t i = base + 64 * w + lane;
            i -= i >= 624 ? 624 : 0;
            r[w] = rb_temper(sh.mt[i]) >> (32 - kb);
        }
        uint64_t accm[kRBWin];   // the accepted draws of each window (ballot of the compare the claim selects on)
#pragma unroll
        for (int w = 0; w < kRBWin; ++w) {   // claims issued in window order; a rejected draw ORs 0 into a word of
            // the bitmap (spread by lane: no bank conflict), which changes nothing and whose return is not used
            const bool acc = r[w] < n;
            accm[w] = rb_ballot(acc);
            uint32_t* a = acc ? &sh.bitmap[r[w] >> 5] : &sh.bitmap[lane & sh.spread];
            old[w] = atomicOr(a, acc ? 1u << (r[w] & 31) : 0u);
        }
        // Selections are numbered in stream order from `have`; number q < k is the
        // sample's q-th pick, q >= k was drawn past the sample's end. The pick
        // numbered k - 1 fixes where the stream resumes.
        uint32_t consumed = 64u * kRBWin;
        int q0 = have;
#pragma unroll
        for (int w = 0; w < kRBWin; ++w) {
            // lane masks from single compares, combined in scalar registers (a ballot of a compound condition
            // costs a select and a compare more): accepted draws, draws whose bit was already set
            const uint64_t setm = rb_ballot((old[w] & (1u << (r[w] & 31))) != 0u);
            uint64_t hm = accm[w] & setm;
            uint64_t rej = hm;
            while (hm) {   // rare
                const int l = __builtin_ctzll(hm);
                const uint32_t v = __builtin_amdgcn_readlane(r[w], l);   // uniform lane: no LDS round trip
                const uint64_t eq = accm[w] & rb_ballot(r[w] == v);
                const uint64_t fresh = eq & ~setm;
                hm &= ~eq;
                rej = fresh ? ((rej & ~eq) | (eq & (eq - 1))) : (rej | eq);
            }
            const uint64_t sm = accm[w] & ~rej;   // the window's selections (rej is inside accm)
            const bool sel = __builtin_amdgcn_inverse_ballot_w64(sm);   // this lane's bit, as an exec-style mask
            const uint32_t q = (uint32_t)q0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u));
            // picks numbered >= k keep their claims: no later draw of this sample can see them (they are
            // past its end in stream order) and the whole bitmap is cleared after the sample
            if (sel && q < (uint32_t)k) {
                idx[q] = (IdxT)r[w];
                if (TR && tr) tr[q] = (int32_t)r[w];
            }
            const int nsel = (int)__builtin_popcountll(sm);
            // (uniform) the sample's last pick is in this window: q0 < k <= q0 + nsel as one unsigned compare (a
            // q0 past k wraps high): ransac alone 6.80 vs 6.97-7.01 ms (profiles/r06/ab_draw_lastpick_s11.txt)
            if ((uint32_t)(k - 1 - q0) < (uint32_t)nsel) {
                const uint64_t lastm = sm & rb_ballot(q == (uint32_t)(k - 1));
                consumed = 64u * w + (uint32_t)__builtin_ctzll(lastm) + 1u;
            }
            q0 += nsel;
        }
        have = q0 < k ? q0 : k;
        st.step(consumed);
        rb_wave_lds_sync();   // the next round reads bits set/cleared by other lanes
    }
    // clear the sample's bits (the whole bitmap, 16 bytes a store: the launch rounds it to 4 words)
    uint4* b4 = reinterpret_cast<uint4*>(sh.bitmap);
    for (uint32_t q = lane; q < (n + 127) / 128; q += kWave) b4[q] = make_uint4(0u, 0u, 0u, 0u);
    rb_wave_lds_sync();
}

// wave 0: random.sample(range(n), k), pool branch (n <= setsize), over a virtual pool. CPython keeps
// pool = list(range(n)) and per pick i takes j = randbelow(n - i), selects pool[j] and moves pool[n - i - 1] into
// slot j. Here the pool is V(x) = x unless the frame's LDS list holds an entry x | V(x) << 16 (n <= 4117 < 2^16):
// a pick reads V(j) and V(n - i - 1) from one scan of the list by the whole wave (four entries a lane per 16-byte
// read) and adds or replaces the entry of j, so the list holds at most k entries — k words of LDS instead of n,
// which is what lets the launch size the LDS without the frames' counts (positions >= n - i are never read again:
// the entry of n - i - 1 may stay).
template <class IdxT, bool TR>
__device__ void rb_sample_pool(RansacShared<IdxT>& sh, RbStream& st, uint32_t n, int k, IdxT* idx, int32_t* tr) {
    const int lane = lane_id();
    uint32_t* ml = sh.pool_list;
    uint32_t cnt = 0;   // list entries (uniform)
    for (int i = 0; i < k && st.pos < kRBMaxDraws; ++i) {
        const uint32_t bound = n - (uint32_t)i;
        const int kb = 32 - __builtin_clz(bound);
        uint32_t j = 0;
        rb_draw_below(sh, st, bound, kb, 1, &j);
        const uint32_t lk = bound - 1u;   // the last live position
        int pj = -1;                      // this lane's entry position of j, of lk (at most one lane each)
        uint32_t vj = 0u, vl = 0u;
        bool hl = false;
        for (uint32_t b = 0; b < cnt; b += 4u * kWave) {   // uniform
            const uint32_t e0 = b + 4u * (uint32_t)lane;
            if (e0 < cnt) {
                const uint4 w = *reinterpret_cast<const uint4*>(ml + e0);
                const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const bool live = e0 + (uint32_t)t < cnt;
                    const uint32_t key = ww[t] & 0xFFFFu;
                    if (live && key == j) {
                        pj = (int)(e0 + (uint32_t)t);
                        vj = ww[t] >> 16;
                    }
                    if (live && key == lk) {
                        hl = true;
                        vl = ww[t] >> 16;
                    }
                }
            }
        }
        const uint64_t mj = rb_ballot(pj >= 0), ml_ = rb_ballot(hl);
        const int posj = mj ? __builtin_amdgcn_readlane(pj, (int)__builtin_ctzll(mj)) : -1;
        const uint32_t valj = mj ? (uint32_t)__builtin_amdgcn_readlane((int)vj, (int)__builtin_ctzll(mj)) : j;
        const uint32_t vall = ml_ ? (uint32_t)__builtin_amdgcn_readlane((int)vl, (int)__builtin_ctzll(ml_)) : lk;
        if (lane == 0) {
            idx[i] = (IdxT)valj;
            if (TR && tr) tr[i] = (int32_t)valj;
            ml[posj >= 0 ? (uint32_t)posj : cnt] = j | (vall << 16);
        }
        cnt += posj >= 0 ? 0u : 1u;
        rb_wave_lds_sync();   // the next pick's scan reads lane 0's entry
    }
    rb_wave_lds_sync();   // idx (and the trace) read by every lane next
}

[[maybe_unused]] constexpr int kRBGather = 10;     // screen gathers a lane keeps in flight
constexpr int kRBEvalThreads = 1024;   // eval: 16 waves screen 16 trials at a time

// One trial's record: the draw kernel writes the triple's three indices into
// its first words, the eval kernel replaces them by a, b, c, |abc|, flag
// (0 ok, 1 singular: numpy's LinAlgError, skipped).
constexpr int kRBTri = 5;

// The trial's plane and its record (one lane): abc = np.dot(np.linalg.inv([P1;P2;P3]),
// np.ones([3, 1])) (functions.py:267) rounded exactly as numpy computes it, |abc| as
// math.sqrt does (:269), and the flag (1: singular, numpy raises LinAlgError and the
// trial is skipped). numpy's inv is LAPACK dgesv(A, I) from its bundled OpenBLAS
// 0.3.29: dgetf2's left-looking LU (partial pivoting on the first largest |a|, the
// column below a pivot scaled by its reciprocal, the update products rounded before
// they are subtracted, column 2's two-term update as fma(l21, u12, l20 u02)), then
// dgetrs's two triangular solves of the permuted identity (trsm: the diagonal
// applied as a multiply by its reciprocal, fused multiply-subtracts, except the
// backward solve's row-2 update of rows 0 and 1, a rounded product subtracted); then
// the dot with ones adds each row's three entries left to right. The restatement
// is oracle/svx_oracle.c svo_plane_lapack, which tests/test_ransac_cpu.py pins to
// numpy bit for bit on random and near-collinear systems.
__device__ __forceinline__ void rb_solve_record(const double* r1, const double* r2, const double* r3, double* o) {
    // the rows, pivoted in place (a row swap at step j equals dgetf2's swap of the
    // columns <= j plus its later re-application to the columns > j)
    double m0[3] = {r1[0], r1[1], r1[2]}, m1[3] = {r2[0], r2[1], r2[2]}, m2[3] = {r3[0], r3[1], r3[2]};
    int p0 = 0, p1 = 1, p2 = 2;   // original row of each position (the permutation dgetrs applies to I)
    const auto swap_rows = [](double (&x)[3], double (&y)[3], int& px, int& py) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double t = x[c];
            x[c] = y[c];
            y[c] = t;
        }
        const int t = px;
        px = py;
        py = t;
    };
    // column 0: pivot = the first largest |a| (idamax)
    int piv = 0;
    double amax = fabs(m0[0]);
    if (fabs(m1[0]) > amax) {
        piv = 1;
        amax = fabs(m1[0]);
    }
    if (fabs(m2[0]) > amax) piv = 2;
    if (piv == 1) swap_rows(m0, m1, p0, p1);
    else if (piv == 2) swap_rows(m0, m2, p0, p2);
    const double u00 = m0[0];
    double l10 = m1[0], l20 = m2[0];
    if (u00 != 0.0) {
        const double r = 1.0 / u00;
        l10 *= r;
        l20 *= r;
    }
    // column 1: the gemv update (rounded product, then subtracted), pivot among rows 1, 2
    double b1 = m1[1] - l10 * m0[1], b2 = m2[1] - l20 * m0[1];
    double c1 = m1[2], c2 = m2[2];
    if (fabs(b2) > fabs(b1)) {
        double t = b1;
        b1 = b2;
        b2 = t;
        t = l10;
        l10 = l20;
        l20 = t;
        t = c1;
        c1 = c2;
        c2 = t;
        const int q = p1;
        p1 = p2;
        p2 = q;
    }
    const double u11 = b1;
    double l21 = b2;
    if (u11 != 0.0) l21 *= 1.0 / u11;
    // column 2: u12 by the dot (rounded product), u22 by the two-term gemv
    const double u01 = m0[1], u02 = m0[2];
    const double u12 = c1 - l10 * u02;
    const double u22 = c2 - fma(l21, u12, l20 * u02);
    const bool singular = u00 == 0.0 || u11 == 0.0 || u22 == 0.0;   // dgesv info > 0
    const double i00 = 1.0 / u00, i11 = 1.0 / u11, i22 = 1.0 / u22;
    double abc[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int c = 0; c < 3; ++c) {   // column c of the inverse: L U x = P e_c
        double x0 = p0 == c ? 1.0 : 0.0, x1 = p1 == c ? 1.0 : 0.0, x2 = p2 == c ? 1.0 : 0.0;
        x1 = fma(-x0, l10, x1);   // forward, unit lower
        x2 = fma(-x0, l20, x2);
        x2 = fma(-x1, l21, x2);
        x2 = x2 * i22;            // backward, upper
        x0 = x0 - u02 * x2;
        x1 = x1 - u12 * x2;
        x1 = x1 * i11;
        x0 = fma(-x1, u01, x0);
        x0 = x0 * i00;
        if (c == 0) {   // np.dot(inv, ones): ((inv[r][0] + inv[r][1]) + inv[r][2])
            abc[0] = x0;
            abc[1] = x1;
            abc[2] = x2;
        } else {
            abc[0] += x0;
            abc[1] += x1;
            abc[2] += x2;
        }
    }
    o[0] = abc[0];
    o[1] = abc[1];
    o[2] = abc[2];
    o[3] = sqrt(abc[0] * abc[0] + abc[1] * abc[1] + abc[2] * abc[2]);   // ((a a + b b) + c c), no fma
    o[4] = singular ? 1.0 : 0.0;
}

template <class IdxT, bool TR, int WPG = 1>
__global__ __launch_bounds__(64 * WPG) void ransac_draw_kernel(const uint32_t* __restrict__ packed, RbTables tb, int64_t cap,
                                                         const int64_t* __restrict__ counts, uint64_t seed_base,
                                                         int64_t first_frame, int trials, int k,
                                                         IdxT* __restrict__ sidx, double* __restrict__ tri,
                                                         int32_t* __restrict__ fstat, int32_t* __restrict__ trace,
                                                         int trace_trials, int bitmap_words, int ablate,
                                                         uint64_t* __restrict__ started, uint64_t epoch, int nframes) {
    // the frame loop's dispatch signal: the last workgroup of the grid is placed after every other one, so once it
    // runs, every frame's wave is resident and another stream's kernel may take the rest of the CUs (loop_gate)
    if (started && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0)
        __hip_atomic_store(started, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // WPG waves a workgroup, each its own frame with its own LDS (no barrier between them): fewer workgroups
    // for the same waves (SVX_DRAW_WPG, diagnostic A/B)
    const int wave = (int)(threadIdx.x >> 6);
    __shared__ uint32_t mt_w[WPG][624];
    extern __shared__ uint4 rb_dyn4[];   // WPG x [bitmap_words] bitmap / pool list (16-byte aligned, 4-word multiple)
    uint32_t* rb_dyn = reinterpret_cast<uint32_t*>(rb_dyn4) + (size_t)wave * bitmap_words;
    RansacShared<IdxT> sh;
    sh.mt = mt_w[wave];
    sh.bitmap = rb_dyn;
    sh.pool_list = rb_dyn;
    sh.k = k;
    sh.spread = bitmap_words >= 64 ? 63u : bitmap_words >= 32 ? 31u : bitmap_words >= 16 ? 15u : bitmap_words >= 8 ? 7u : 3u;
    sh.ablate = ablate;
    const int lane = lane_id();
    // one frame a wave, or (the frame loop, gridDim.x < nframes) a wave's frames one after the other: fewer
    // waves resident at once hold less LDS beside the other batch's pipeline
    for (int frame = blockIdx.x * WPG + wave; frame < nframes; frame += gridDim.x * WPG) {
    const int64_t n64 = counts[frame];
    const uint32_t* fpk = packed + (int64_t)frame * cap;
    if (n64 < k || trials <= 0) {   // every trial's random.sample raises: (None, None)
        if (lane == 0) {
            fstat[2 * frame] = 0;
            fstat[2 * frame + 1] = 0;
        }
        continue;
    }
#ifdef SVX_DIAG
    // DIAGNOSTIC (diagnostic build, SVX_RANSAC_ABLATE bit 128; results invalid): the wave holds its resources for
    // 4 ms of wall clock and draws nothing (the evaluation then reads stale indices, clamped) — does the pipeline
    // beside the draw slow down for the draw's resources or for its work?
    if (ablate & 128) {
        const uint64_t t0 = wall_clock64();
        while (wall_clock64() - t0 < 400000u) __builtin_amdgcn_s_sleep(64);
        if (lane == 0) {
            fstat[2 * frame] = 0;
            fstat[2 * frame + 1] = trials;
        }
        continue;
    }
#endif
    const uint32_t n = (uint32_t)n64;
    const int kb = 32 - __builtin_clz(n);
    const bool pool = (int64_t)n <= ransac_setsize(k);
    // the launch sized the sample LDS from an upper bound of the counts; a frame above it (only if the bound's
    // premise broke) stops with status 3 rather than write past its LDS
    if (pool ? k > bitmap_words : (int64_t)(n + 31) / 32 > bitmap_words) {
        if (lane == 0) {
            fstat[2 * frame] = 3;
            fstat[2 * frame + 1] = 0;
        }
        continue;
    }
    for (int q = lane; q < bitmap_words; q += 64) sh.bitmap[q] = 0;
    if (lane == 0) rb_seed(sh.mt, seed_base + (uint64_t)(first_frame + frame));
    rb_wave_lds_sync();   // the wave's own LDS: lane 0's seeding (and the clears) before every lane's reads
    RbStream st;
    const int g_pt = lane % 3, g_co = min(lane / 3, 2);   // the triple gather: point, coordinate (rb_point's tables)
    const uint32_t tg_y = (uint32_t)((tb.Y - tb.X) / 256), tg_z = (uint32_t)((tb.Z - tb.X) / 256);   // table rows
    int status = 0, s = 0;
    for (; s < trials; ++s) {
        IdxT* idx = sidx + ((int64_t)frame * trials + s) * k;
        int32_t* tr = TR && s < trace_trials ? trace + ((int64_t)frame * trace_trials + s) * (k + 3) : nullptr;
        if (ablate & 16) {   // DIAGNOSTIC: no sample
        } else if (pool) {
            rb_sample_pool<IdxT, TR>(sh, st, n, k, idx, tr);
        } else {
            rb_sample_set<IdxT, TR>(sh, st, n, kb, k, idx, tr);
        }
        uint32_t t3[3] = {0, 0, 0};
        double p1[3], p2[3], p3[3];   // the triple's fp64 points (rb_point: the reference's X, Y, Z)
        int attempts = 0;
        bool degenerate = false;
        do {   // randomNonCollinearPoints
            if (++attempts > kRBMaxAttempts) {
                degenerate = true;
                break;
            }
            rb_draw_below(sh, st, n, kb, 3, t3);
            // lane 3 c + i (< 9) gathers coordinate c of point i: one load of the packed words, one of the
            // tables (two memory round trips); every lane then takes the nine values from lanes 0..8
            const uint32_t pk = fpk[g_pt == 0 ? t3[0] : g_pt == 1 ? t3[1] : t3[2]];
            // while the packed words are in flight: the next twist level, once the stream has consumed the
            // state words it replaces (a level drops positions below G - 397; pos >= G - 397 has read them all)
            if (st.pos + 397u >= st.G) rb_advance(sh, st, st.G + 1u - st.pos);
            const uint32_t x2 = (pk & 0xFFF) >> 1, y2 = ((pk >> 12) & 0xFFF) >> 1, dd = pk >> 24;
            // one load: the three tables are one allocation (X rows, then Y rows, then Z), so the lane's coordinate
            // picks a row, not a pointer (no exec branches): ransac alone 6.75-6.78 vs 6.82-6.83 ms, loop 14.34-14.37
            // vs 14.38-14.50 (profiles/r06/ab_draw_triple_gather_s12.txt)
            const uint32_t row = g_co == 0 ? x2 : g_co == 1 ? tg_y + y2 : tg_z;
            const double v = tb.X[row * 256 + dd];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                p1[c] = rb_readlane_f64(v, 3 * c + 0);
                p2[c] = rb_readlane_f64(v, 3 * c + 1);
                p3[c] = rb_readlane_f64(v, 3 * c + 2);
            }
        } while (st.pos < kRBMaxDraws && !(ablate & 8) && rb_collinear(p1, p2, p3));
        if (st.pos >= kRBMaxDraws) {
            status = 2;
            break;
        }
        if (degenerate) {
            status = 1;
            break;
        }
        if (TR && tr && lane < 3) tr[k + lane] = (int32_t)(lane == 0 ? t3[0] : lane == 1 ? t3[1] : t3[2]);
        if (lane < 3) {   // the triple (the eval kernel solves its plane, off this chain)
            uint32_t* trip = reinterpret_cast<uint32_t*>(tri + ((int64_t)frame * trials + s) * kRBTri);
            trip[lane] = lane == 0 ? t3[0] : lane == 1 ? t3[1] : t3[2];
        }
    }
    if (lane == 0) {
        fstat[2 * frame] = status;   // 1: the reference would never return; 2: draw budget
        fstat[2 * frame + 1] = s;    // trials drawn (the failing one excluded)
    }
    rb_wave_lds_sync();   // (the wave's own LDS) the next frame re-seeds mt and clears the bitmap
    }
}

// A lane's value read by every lane (src uniform across the wave).
__device__ __forceinline__ int rb_readlane(int v, int src) { return __builtin_amdgcn_readlane(v, src); }
__device__ __forceinline__ double rb_readlane(double v, int src) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, src);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), src);
    return __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
}

// np.mean's sum of a trial's k distance terms (functions.py:289), by one wave, in
// numpy's pairwise order (numpy/_core/src/umath/loops_utils.h.src pairwise_sum,
// reached from add.reduce with the initial 0.0): n < 8 terms summed in order from
// 0.0; n <= 128 in eight accumulators r[j] (terms j, j + 8, ... below n - n % 8,
// in order), combined ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)), then the
// last n % 8 added in order; n > 128 split at n2 = n/2 - (n/2) % 8 and the halves'
// sums added. So every leaf starts at a multiple of 8, and k <= 1024 has at most
// 16 leaves. The leaves are listed by a uniform walk of the split tree (a task
// stack held one entry a lane), their sums computed eight leaves at a time (lane
// 8g + j runs accumulator j of leaf g), and the tree walked again to add them.
// load(i) -> the packed point of sample entry i, term(u) -> its distance term.
template <class LoadF, class TermF>
__device__ double rb_np_pairwise(int k, LoadF load, TermF term) {
    const int lane = lane_id();
    int st_lo = 0, st_n = k;   // task stack, slot s in lane s; st_n < 0 marks an addition
    int sp = 1;
    int leaf_lo = 0, leaf_n = 0, nleaf = 0;   // leaf l in lane l
    while (sp > 0) {
        const int lo = rb_readlane(st_lo, sp - 1), n = rb_readlane(st_n, sp - 1);
        --sp;
        if (n <= 128) {
            if (lane == nleaf) {
                leaf_lo = lo;
                leaf_n = n;
            }
            ++nleaf;
        } else {
            const int n2 = n / 2 - (n / 2) % 8;
            if (lane == sp) {   // the right half, summed after the left
                st_lo = lo + n2;
                st_n = n - n2;
            }
            if (lane == sp + 1) {
                st_lo = lo;
                st_n = n2;
            }
            sp += 2;
        }
    }
    double leafsum = 0.0;   // leaf l's sum in lane l
    const int g = lane >> 3, j = lane & 7;
    for (int q = 0; q < nleaf; q += 8) {
        const int l = q + g;
        const bool live = l < nleaf;
        const int lo = __shfl(leaf_lo, live ? l : 0, kWave), n = live ? __shfl(leaf_n, l, kWave) : 0;
        const int mm = n >= 8 ? n - (n & 7) : 0;
        double r = 0.0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {   // accumulator j: terms j, j + 8, ... < mm (at most 16), eight loads in flight
            uint32_t u[8];
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                const int i = j + 8 * (8 * h + v);
                u[v] = i < mm ? load(lo + i) : 0u;
            }
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                const int i = j + 8 * (8 * h + v);
                if (i < mm) {
                    const double t = term(u[v]);
                    r = (h == 0 && v == 0) ? t : r + t;
                }
            }
        }
        double s = r + __shfl_xor(r, 1, kWave);
        s = s + __shfl_xor(s, 2, kWave);
        s = s + __shfl_xor(s, 4, kWave);
        if (live && j == 0)
            for (int i = mm; i < n; ++i) s += term(load(lo + i));   // n < 8: s = 0.0 + the n terms in order
        const double v = __shfl(s, ((lane - q) & 7) << 3, kWave);
        if (lane >= q && lane < q + 8) leafsum = v;
    }
    double vst = 0.0;   // value stack, slot s in lane s
    int vsp = 0, li = 0;
    st_lo = 0;
    st_n = k;
    sp = 1;
    while (sp > 0) {
        const int lo = rb_readlane(st_lo, sp - 1), n = rb_readlane(st_n, sp - 1);
        --sp;
        double push;
        if (n < 0) {   // both halves done: left + right
            const double b = rb_readlane(vst, vsp - 1), a = rb_readlane(vst, vsp - 2);
            vsp -= 2;
            push = a + b;
        } else if (n <= 128) {
            push = rb_readlane(leafsum, li++);
        } else {
            const int n2 = n / 2 - (n / 2) % 8;
            if (lane == sp) st_n = -1;
            if (lane == sp + 1) {
                st_lo = lo + n2;
                st_n = n - n2;
            }
            if (lane == sp + 2) {
                st_lo = lo;
                st_n = n2;
            }
            sp += 3;
            continue;
        }
        if (lane == vsp) vst = push;
        ++vsp;
    }
    return rb_readlane(vst, 0);
}

// One DPP step of an fp64 wave scan (both 32-bit halves moved with the same control; a lane whose source is
// outside its row or row mask reads 0.0) and the two-value wave sum built from six of them — the wave_scan_dpp
// pattern of svx_device.h (row_shr 1/2/4/8, then row_bcast 15 and 31; lane 63 ends with the total), the two
// chains interleaved. One VALU op a move instead of a ds_bpermute round trip: the xor butterfly of __shfl_xor had
// put six dependent LDS round trips on every trial's chain. All 64 lanes must be active. The additions run in
// another order than the butterfly's; the screen's sums are bounded approximations (64 fp64 lane sums round by
// ~2^-47 of their magnitude, far inside the screen's 4x margin) and the decision is taken on exact fp64 errors.
template <int CTL, int RM>
__device__ __forceinline__ double rb_dpp_f64(double v) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTL, RM, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTL, RM, 0xf, false);
    return __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
}
// The DPP move of an fp64 value where a lane with no source (or outside the row mask) reads +inf, and the min-scan
// step built from it.
template <int CTL, int RM = 0xf>
__device__ __forceinline__ double rb_dpp_inf_f64(double v) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    constexpr uint64_t kInf = 0x7FF0000000000000ull;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)kInf, (int)(uint32_t)u, CTL, RM, 0xf, false);
    const uint32_t hi =
        (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(kInf >> 32), (int)(uint32_t)(u >> 32), CTL, RM, 0xf, false);
    return __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
}
template <int CTL, int RM>
__device__ __forceinline__ double rb_dpp_min_f64(double v) { return fmin(v, rb_dpp_inf_f64<CTL, RM>(v)); }

__device__ __forceinline__ void rb_wave_sum2_f64(double& a, double& b) {
#define SVX_RB_SUM2_STEP(ctl, rm)        \
    a += rb_dpp_f64<ctl, rm>(a);         \
    b += rb_dpp_f64<ctl, rm>(b)
    SVX_RB_SUM2_STEP(0x111, 0xf);   // row_shr:1
    SVX_RB_SUM2_STEP(0x112, 0xf);   // row_shr:2
    SVX_RB_SUM2_STEP(0x114, 0xf);   // row_shr:4
    SVX_RB_SUM2_STEP(0x118, 0xf);   // row_shr:8
    SVX_RB_SUM2_STEP(0x142, 0xa);   // row_bcast:15
    SVX_RB_SUM2_STEP(0x143, 0xc);   // row_bcast:31
#undef SVX_RB_SUM2_STEP
    a = rb_readlane_f64(a, 63);
    b = rb_readlane_f64(b, 63);
}

#ifdef SVX_DIAG
// DIAGNOSTIC (diagnostic build, SVX_RANSAC_ABLATE bit 32; results valid): the evaluation's phases timed by each
// workgroup's thread 0 at the barriers that end them (wall clock, 10 ns ticks), summed over the workgroups:
// [0] the points' LDS fill, [1] the plane solves, [2] the screen, [3] the candidate compaction, [4] the candidates'
// fp64 errors, [5] the decision, [6] workgroups stamped. Read by sv_diag_eval_phases.
__device__ unsigned long long g_eval_phase[8];
#define SVX_EVAL_STAMP(i)                                                                       \
    do {                                                                                        \
        if ((ablate & 32) && tid == 0) {                                                        \
            const uint64_t now_ = wall_clock64();                                               \
            atomicAdd(&g_eval_phase[i], (unsigned long long)(now_ - stamp_));                   \
            stamp_ = now_;                                                                      \
        }                                                                                       \
    } while (0)
#else
#define SVX_EVAL_STAMP(i) \
    do {                  \
    } while (0)
#endif

// Screen + decision. LDS: the frame's packed points (LDS_PTS) or none, then
// per trial the screened mean and its bound (2 doubles).
template <class IdxT, bool LDS_PTS>
// 96 VGPRs (five waves' worth a SIMD, no spills) instead of the 123 the kernel takes unconstrained: its 1024-lane
// workgroup is four waves a SIMD, and at 123 they filled the register file, so nothing else ran on a CU beside an
// evaluation workgroup — in the frame loop the next batch's pre-pass waited for whole CUs (loop 15.30 -> 15.01 ms,
// four alternations, profiles/r05/ab_eval_vgpr_s19.txt).
#ifndef SVX_EVAL_WPE
#define SVX_EVAL_WPE 5
#endif
#ifndef SVX_SCREEN_RUN   // index vectors a lane loads before gathering (the grouped screen)
#define SVX_SCREEN_RUN 5
#endif
#ifndef SVX_SCREEN_GROUPED   // 0: the one-wave-a-trial screen (A/B build)
#define SVX_SCREEN_GROUPED 1
#endif
__global__ __launch_bounds__(kRBEvalThreads) __attribute__((amdgpu_waves_per_eu(SVX_EVAL_WPE))) void ransac_eval_kernel(
    const uint32_t* __restrict__ packed, RbTables tb, int64_t cap, KParams cp,
    const int64_t* __restrict__ counts, int trials, int k, const IdxT* __restrict__ sidx,
    double* __restrict__ tri, const int32_t* __restrict__ fstat, double* __restrict__ out_abc,
    double* __restrict__ out_err, int32_t* __restrict__ out_trial, uint32_t* __restrict__ out_flags, int ablate,
    int lds_pts_words) {
    extern __shared__ uint4 ev_dyn4[];   // 16-byte aligned: the points' fill stores 16 bytes a lane
    uint32_t* ev_dyn = reinterpret_cast<uint32_t*>(ev_dyn4);
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.x;
    const int64_t n64 = counts[frame];
    if (n64 < k || trials <= 0) {
        if (tid == 0) {
            out_trial[frame] = -1;
            out_flags[frame] = 0;
            out_err[frame] = 0.0;
            out_abc[3 * frame] = out_abc[3 * frame + 1] = out_abc[3 * frame + 2] = 0.0;
        }
        return;
    }
    const int status = fstat[2 * frame], T = fstat[2 * frame + 1];
#ifdef SVX_DIAG
    uint64_t stamp_ = (ablate & 32) ? wall_clock64() : 0;
    if ((ablate & 32) && tid == 0) atomicAdd(&g_eval_phase[6], 1ull);
#endif
    const uint32_t* fpk = packed + (int64_t)frame * cap;
    const uint32_t* P = fpk;
    if (LDS_PTS && n64 > lds_pts_words) {   // above the launch's LDS bound (only if its premise broke): flag 32
        if (tid == 0) {
            out_trial[frame] = -1;
            out_flags[frame] = 32;
            out_err[frame] = 0.0;
            out_abc[3 * frame] = out_abc[3 * frame + 1] = out_abc[3 * frame + 2] = 0.0;
        }
        return;
    }
    if constexpr (LDS_PTS) {
        // 16-byte loads, four in flight a thread (the frame's words start 16-byte aligned when cap % 4 == 0)
        int64_t done = 0;
        if ((reinterpret_cast<uintptr_t>(fpk) & 15) == 0) {
            const uint4* f4 = reinterpret_cast<const uint4*>(fpk);
            uint4* l4 = reinterpret_cast<uint4*>(ev_dyn);
            const int64_t n4 = n64 >> 2;
            for (int64_t b = 0; b < n4; b += 4 * kRBEvalThreads) {
                uint4 v[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int64_t q = b + i * kRBEvalThreads + tid;
                    v[i] = f4[q < n4 ? q : 0];
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int64_t q = b + i * kRBEvalThreads + tid;
                    if (q < n4) l4[q] = v[i];
                }
            }
            done = n4 << 2;
        }
        for (int64_t q = done + tid; q < n64; q += kRBEvalThreads) ev_dyn[q] = fpk[q];
        P = ev_dyn;
    }
    double* scr = reinterpret_cast<double*>(ev_dyn + (LDS_PTS ? lds_pts_words : 0));   // [T][2]
    double* ftri = tri + (int64_t)frame * trials * kRBTri;
    const IdxT* fidx = sidx + (int64_t)frame * trials * k;
    __syncthreads();
    SVX_EVAL_STAMP(0);
    // every trial's plane from its triple (the draw kernel wrote the three indices
    // into the record's first words), one lane a trial: the record in place
    if (!(ablate & 1)) {
        const uint32_t nm1 = (uint32_t)n64 - 1;
        for (int t = tid; t < T; t += kRBEvalThreads) {
            double* rec = ftri + (int64_t)t * kRBTri;
            const uint32_t* trip = reinterpret_cast<const uint32_t*>(rec);
            const uint32_t i1 = min(trip[0], nm1), i2 = min(trip[1], nm1), i3 = min(trip[2], nm1);
            double r1[3], r2[3], r3[3];
            rb_point(P[i1], tb, r1[0], r1[1], r1[2]);
            rb_point(P[i2], tb, r2[0], r2[1], r2[2]);
            rb_point(P[i3], tb, r3[0], r3[1], r3[2]);
            rb_solve_record(r1, r2, r3, rec);
        }
        __syncthreads();   // the records are read by other waves below (same workgroup: same L1)
    }
    SVX_EVAL_STAMP(1);
    // screen every trial in fp32 (one wave a trial): the mean distance from the
    // packed points and, per point, the bound (T' + 1) 2^-18 / |abc| on its
    // difference to the fp64 distance, T' = rcp(d) (|cx Ba| + |cy Bb| + |Cc|) (the
    // term's magnitudes, ~ |Xa| + |Yb| + |Zc|; `point` below). A term's error:
    // cx, cy (x - cw_hi: exact, or one rounding), Ba, Bb, Cc rounded to fp32 and
    // the two inner fmas, each <= 2^-24 of the magnitudes: <= 4 x 2^-24 T' d in
    // the sum; rcp(d) within 1 ulp (2^-23 T'); the last fma 2^-24 (T' + 1):
    // together <= 7 x 2^-24 (T' + 1). A lane's fp32 sum of <= 10 terms adds
    // <= 9 x 2^-24 of them: in all <= 16 x 2^-24 (T' + 1) = 2^-20 (T' + 1), under
    // the bound's 2^-18 (its sum in fp32, low by at most ~2^-20 relative) with a
    // margin of ~4x. (The reference's own fp64 roundings are ~2^-50 (T + 1).) The
    // lanes' sums are added in fp64.
    if (!(ablate & 1)) {
        // software-pipelined over the wave's trials: the next trial's indices and
        // record are loaded (global, just written by the draw kernel) while this
        // trial's points are gathered from LDS
        constexpr int NW = kRBEvalThreads / 64;
        // one point's fp32 distance term and bound term, summed per lane in fp32 (at most 10 terms a lane per
        // batch; the batches and the lanes in fp64): the sum's rounding, <= 9 x 2^-24 of the summed terms, stays
        // inside the bound's margin (see the note at the eval kernel). Per trial: Ba = B a, Bb = B b and
        // Cc = fB c - cw_lo B a - ch_lo B b (fp64, rounded to fp32), so with cx = x - cw_hi, cy = y - ch_hi the term
        // is |rcp(d) (cx Ba + cy Bb + Cc) - 1| (three fmas) and its bound term rcp(d) (|cx Ba| + |cy Bb| + |Cc|)
        // (the +1 of every term is added as k at the end). `live` masks the lanes past the sample (no branch).
        const auto point = [&](uint32_t u, bool live, float Ba, float Bb, float Cc, float& sum, float& bnd) {
            const float cx = (float)(u & 0xFFF) - cp.cw_hi, cy = (float)((u >> 12) & 0xFFF) - cp.ch_hi;
            const float rr = __builtin_amdgcn_rcpf((float)(u >> 24));
            const float t = __builtin_fmaf(rr, __builtin_fmaf(cx, Ba, __builtin_fmaf(cy, Bb, Cc)), -1.0f);
            const float q = __builtin_fmaf(__builtin_fabsf(cx), __builtin_fabsf(Ba),
                                           __builtin_fmaf(__builtin_fabsf(cy), __builtin_fabsf(Bb), __builtin_fabsf(Cc)));
            sum += live ? __builtin_fabsf(t) : 0.0f;
            bnd = __builtin_fmaf(rr, live ? q : 0.0f, bnd);
        };
        [[maybe_unused]] const auto finish = [&](int t, const double (&rec)[kRBTri], double sum, double bnd) {
            rb_wave_sum2_f64(sum, bnd);
            if (lane == 0) {   // the screened mean and its bound; bound -1 marks a singular trial
                const double inv = 1.0 / (rec[3] * k);   // (one more rounding each: inside the margin)
                scr[2 * t] = sum * inv;
                scr[2 * t + 1] = rec[4] == 1.0 ? -1.0 : (bnd + (double)k) * 0x1p-18 * inv;
            }
        };
#if SVX_SCREEN_GROUPED
        // Eight lanes a trial, eight trials a wave pass: lane gl of a trial's group takes the trial's indices in
        // vectors of VEC (one 16-byte load each; the group's eight loads are one 128-byte line), RUN vectors a lane
        // loaded before any is used (two runs for k = 600 at 16-bit indices), then its VEC-point fp32 batches
        // (<= 10 terms each, as the bound requires) added in fp64; the group's sums meet in three DPP steps, eight
        // trials at once, and the group's lane 0 stores the screened mean and bound. Against one wave a trial —
        // ten 2-byte index loads a lane waited for once a trial and a 64-lane fp64 reduction and division on every
        // trial's chain — the screen took 91 us a frame of the evaluation's 118, now 57 (RUN = 5: more spills
        // VGPRs at the kernel's 96; RUN = 3: 70 us) (profiles/r06/probe_eval_phases_s18.txt,
        // ab_eval_screen_grouped_s20.txt).
        {
            constexpr int GL = 8, TPW = kWave / GL;     // lanes a trial, trials a wave pass
            constexpr int VEC = 16 / (int)sizeof(IdxT);  // indices a 16-byte load holds
            constexpr int RUN = SVX_SCREEN_RUN;          // loads a lane holds (k <= 8 x RUN x VEC in one run)
            const int grp = lane / GL, gl = lane % GL;
            const uint32_t nm1 = (uint32_t)n64 - 1;
            // 16-byte loads need every trial's row 16-byte aligned (k x sizeof(IdxT) a multiple of 16); a lane past
            // the row's end loads the row's last whole vector (k % VEC == 0 then) and its points are masked
            const bool vec_ok = ((int64_t)k * (int64_t)sizeof(IdxT)) % 16 == 0 &&
                                (reinterpret_cast<uintptr_t>(fidx) & 15) == 0;
            for (int t0 = wave * TPW; t0 < T; t0 += NW * TPW) {   // uniform per wave
                const int t = min(t0 + grp, T - 1);   // a group past T repeats the last trial (not stored)
                double rec[kRBTri];
#pragma unroll
                for (int q = 0; q < kRBTri; ++q) rec[q] = ftri[(int64_t)t * kRBTri + q];
                const IdxT* idx = fidx + (int64_t)t * k;
                double sum = 0.0, bnd = 0.0;
                for (int r0 = 0; r0 < k; r0 += RUN * GL * VEC) {   // uniform: one run for k <= 640 (u16)
                    uint4 w[RUN];   // the run's index vectors, unpacked where used
#pragma unroll
                    for (int j = 0; j < RUN; ++j) {
                        const int i = r0 + j * GL * VEC + gl * VEC;
                        if (vec_ok) {
                            w[j] = *reinterpret_cast<const uint4*>(idx + min(i, k - VEC));
                        } else {   // element loads packed the same way
                            uint32_t ww[4] = {0u, 0u, 0u, 0u};
#pragma unroll
                            for (int e = 0; e < VEC; ++e) {
                                const uint32_t v = (uint32_t)idx[min(i + e, k - 1)];
                                if (sizeof(IdxT) == 2) ww[e / 2] |= v << (16 * (e % 2));
                                else ww[e] = v;
                            }
                            w[j] = make_uint4(ww[0], ww[1], ww[2], ww[3]);
                        }
                    }
                    const double Ba64 = cp.B * rec[0], Bb64 = cp.B * rec[1];
                    const float Ba = (float)Ba64, Bb = (float)Bb64;
                    const float Cc = (float)(cp.fB * rec[2] - (double)cp.cw_lo * Ba64 - (double)cp.ch_lo * Bb64);
#pragma unroll
                    for (int j = 0; j < RUN; ++j) {
                        const int i = r0 + j * GL * VEC + gl * VEC;
                        const uint32_t ww[4] = {w[j].x, w[j].y, w[j].z, w[j].w};
                        uint32_t u[VEC];
#pragma unroll
                        for (int e = 0; e < VEC; ++e) {
                            const uint32_t ix = sizeof(IdxT) == 2 ? (ww[e / 2] >> (16 * (e % 2))) & 0xFFFFu : ww[e];
#if defined(SVX_SCREEN_AB) && SVX_SCREEN_AB == 2   // DIAGNOSTIC A/B build (results invalid): no LDS gathers
                            u[e] = min(ix, nm1) * 0x9E3779B1u | 0x01000000u;
#else
                            u[e] = P[min(ix, nm1)];
#endif
                        }
                        float s32 = 0.0f, b32 = 0.0f;
#if defined(SVX_SCREEN_AB) && SVX_SCREEN_AB == 4   // DIAGNOSTIC A/B build (results invalid): no point arithmetic
#pragma unroll
                        for (int e = 0; e < VEC; ++e) s32 += (float)u[e];
#else
#pragma unroll
                        for (int e = 0; e < VEC; ++e) point(u[e], i + e < k, Ba, Bb, Cc, s32, b32);
#endif
                        sum += (double)s32;
                        bnd += (double)b32;
                    }
                }
                // the group's eight lane sums: quad_perm [1,0,3,2] and [2,3,0,1], then the other quad of the
                // half row (row_half_mirror); every lane of the group ends with the same total
                sum += rb_dpp_f64<0xB1, 0xf>(sum);
                bnd += rb_dpp_f64<0xB1, 0xf>(bnd);
                sum += rb_dpp_f64<0x4E, 0xf>(sum);
                bnd += rb_dpp_f64<0x4E, 0xf>(bnd);
                sum += rb_dpp_f64<0x141, 0xf>(sum);
                bnd += rb_dpp_f64<0x141, 0xf>(bnd);
                if (gl == 0 && t0 + grp < T) {   // the screened mean and its bound; bound -1 marks a singular trial
                    const double inv = 1.0 / (rec[3] * k);
                    scr[2 * t] = sum * inv;
                    scr[2 * t + 1] = rec[4] == 1.0 ? -1.0 : (bnd + (double)k) * 0x1p-18 * inv;
                }
            }
        }
#else
        {
            // every sample index is clamped to the frame's points before it addresses anything: the indices come
            // from memory another kernel wrote, and a word past the frame's n points (a stale LDS word or another
            // frame's) would send rb_point's table gathers (12-bit x, y fields) past the tables
            const uint32_t nm1 = (uint32_t)n64 - 1;
            auto load = [&](int t, uint32_t (&ix)[kRBGather], double (&rec)[kRBTri]) {
                const IdxT* idx = fidx + (int64_t)t * k;
#if defined(SVX_SCREEN_AB) && SVX_SCREEN_AB == 1   // DIAGNOSTIC A/B build (results invalid): the first trial's indices only
                if (t < NW)
#endif
#pragma unroll
                for (int v = 0; v < kRBGather; ++v)
                    ix[v] = min((uint32_t)idx[min(lane + kWave * v, k - 1)], nm1);   // no branch
#pragma unroll
                for (int q = 0; q < kRBTri; ++q) rec[q] = ftri[(int64_t)t * kRBTri + q];
            };
            uint32_t nix[kRBGather];
            double nrec[kRBTri];
            if (wave < T) load(wave, nix, nrec);
            for (int t = wave; t < T; t += NW) {
                uint32_t ix[kRBGather];
                double rec[kRBTri];
#pragma unroll
                for (int v = 0; v < kRBGather; ++v) ix[v] = nix[v];
#pragma unroll
                for (int q = 0; q < kRBTri; ++q) rec[q] = nrec[q];
                if (t + NW < T) load(t + NW, nix, nrec);
                double sum = 0.0, bnd = 0.0;
                if (rec[4] != 1.0) {
                    const double Ba64 = cp.B * rec[0], Bb64 = cp.B * rec[1];
                    const float Ba = (float)Ba64, Bb = (float)Bb64;
                    const float Cc = (float)(cp.fB * rec[2] - (double)cp.cw_lo * Ba64 - (double)cp.ch_lo * Bb64);
                    for (int j0 = lane, g = 0; j0 < k + lane; j0 += kRBGather * kWave, ++g) {   // uniform
                        uint32_t u[kRBGather];
                        float s32 = 0.0f, b32 = 0.0f;
                        if (g > 0) {   // k > 640: the rest of the sample (same order as the first batch)
#pragma unroll
                            for (int v = 0; v < kRBGather; ++v)
                                ix[v] = min((uint32_t)fidx[(int64_t)t * k + min(j0 + kWave * v, k - 1)], nm1);
                        }
#if defined(SVX_SCREEN_AB) && SVX_SCREEN_AB == 2   // DIAGNOSTIC A/B build (results invalid): no LDS gathers
#pragma unroll
                        for (int v = 0; v < kRBGather; ++v) u[v] = ix[v] * 0x9E3779B1u;
#else
#pragma unroll
                        for (int v = 0; v < kRBGather; ++v) u[v] = P[ix[v]];
#endif
#pragma unroll
                        for (int v = 0; v < kRBGather; ++v) point(u[v], j0 + kWave * v < k, Ba, Bb, Cc, s32, b32);
                        sum += (double)s32;
                        bnd += (double)b32;
                    }
                }
#if defined(SVX_SCREEN_AB) && SVX_SCREEN_AB == 3   // DIAGNOSTIC A/B build (results invalid): no wave sums
                if (lane == 0) scr[2 * t] = sum, scr[2 * t + 1] = bnd;
#else
                finish(t, rec, sum, bnd);
#endif
            }
        }
#endif
    } else {
        for (int t = tid; t < T; t += kRBEvalThreads) scr[2 * t + 1] = ftri[(int64_t)t * kRBTri + 4] == 1.0 ? -1.0 : 0.0;
    }
    __syncthreads();
    SVX_EVAL_STAMP(2);
    // Which trials can matter? The running best before trial t is exactly
    // min_{j<t} e_j (a trial the sequential screen skips has e_j >= LB_j >
    // best_{j-1}), and e_j <= UB_j = e32_j + eb_j, so every trial the
    // sequential procedure evaluates has LB_t <= min_{j<t} UB_j (1 + 1e-9): the
    // candidates below are a superset. Evaluating a superset cannot change the
    // winner (the first strict minimum), the error or the near-tie flag (a
    // trial the sequential procedure skips has e > best (1 + 1e-9)).
    // Wave 0: exclusive prefix-min of UB in trial order, the candidates
    // compacted in order into cand[]; then every wave evaluates candidates in
    // fp64 (the same per-lane order as before: bit-identical errors), and one
    // lane decides over them in trial order.
    int32_t* cand = reinterpret_cast<int32_t*>(scr + 2 * (int64_t)T);
    double* ce = reinterpret_cast<double*>(cand + ((T + 1) & ~1));
    __shared__ uint32_t ncand_s, any_singular_s;
    if (wave == 0) {
        double carry = __builtin_huge_val();
        uint32_t nc = 0, sing = 0;
        for (int t0 = 0; t0 < T; t0 += kWave) {
            const int t = t0 + lane;
            const bool in = t < T;
            const double e32 = in ? scr[2 * t] : 0.0, eb = in ? scr[2 * t + 1] : -1.0;
            const bool singular = in && eb < 0.0;
            const double ub = (in && !singular) ? e32 + eb : __builtin_huge_val();
            // inclusive min-scan over the wave by DPP (row_shr 1/2/4/8, row_bcast 15/31; a lane with no source keeps
            // +inf), then the exclusive one by wave_shr:1 — six VALU moves instead of six ds_bpermute round trips
            double inc = ub;
            inc = rb_dpp_min_f64<0x111, 0xf>(inc);
            inc = rb_dpp_min_f64<0x112, 0xf>(inc);
            inc = rb_dpp_min_f64<0x114, 0xf>(inc);
            inc = rb_dpp_min_f64<0x118, 0xf>(inc);
            inc = rb_dpp_min_f64<0x142, 0xa>(inc);
            inc = rb_dpp_min_f64<0x143, 0xc>(inc);
            double ex = rb_dpp_inf_f64<0x138>(inc);
            ex = lane == 0 ? carry : fmin(ex, carry);   // min over j < t
            bool c = in && !singular && !(e32 - eb > ex * (1.0 + 2e-9));   // NaN / inf: a candidate
            if (ablate & 4) c = in && !singular;
            if (ablate & 1) c = false;                                     // DIAGNOSTIC 1: no evaluation
            const uint64_t m = rb_ballot(c);
            if (c) cand[nc + __builtin_popcountll(m & ((1ull << lane) - 1))] = t;
            nc += (uint32_t)__builtin_popcountll(m);
            sing |= rb_ballot(singular) != 0 ? 1u : 0u;
            carry = fmin(carry, rb_readlane_f64(inc, kWave - 1));
        }
        if (lane == 0) {
            ncand_s = nc;
            any_singular_s = sing;
        }
    }
    __syncthreads();
    SVX_EVAL_STAMP(3);
    const uint32_t nc = ncand_s, nm1 = (uint32_t)n64 - 1;
    for (uint32_t ci = wave; ci < nc; ci += kRBEvalThreads / 64) {
        const int t = cand[ci];
        const double* tr = ftri + (int64_t)t * kRBTri;
        const double a = tr[0], b = tr[1], c = tr[2], d = tr[3];
        const IdxT* idx = fidx + (int64_t)t * k;
        // abs((np.dot(T, abc) - 1) / d) per sample point (functions.py:275): numpy's
        // gemv rounds each row's dot as fma(z, c, fma(x, a, y b)) (k = 1 is a (1, 3) x
        // (3, 1) product, numpy's ddot: fma(z, c, fma(y, b, x a))); np.mean (:289) =
        // the pairwise sum / k. Bit-identical to numpy (tests/test_ransac_cpu.py).
        const double sum = rb_np_pairwise(
            k, [&](int i) { return P[min((uint32_t)idx[i], nm1)]; },   // the packed point (LDS, or memory), clamped
            [&](uint32_t u) {
                double qx, qy, qz;
                rb_point(u, tb, qx, qy, qz);
                const double dot = k == 1 ? fma(qz, c, fma(qy, b, qx * a)) : fma(qz, c, fma(qx, a, qy * b));
                return fabs((dot - 1.0) / d);
            });
        if (lane == 0) ce[ci] = sum / k;
    }
    __syncthreads();
    SVX_EVAL_STAMP(4);
    double best = __builtin_huge_val(), second = __builtin_huge_val();
    int best_t = -1;
    uint32_t flags = any_singular_s ? 1u : 0u;
    double babc[3] = {0, 0, 0};
    if (tid == 0) {
        for (uint32_t ci = 0; ci < nc; ++ci) {   // trial order, strict <
            const double e = ce[ci];
            if (e < best) {
                const int t = cand[ci];
                const double* tr = ftri + (int64_t)t * kRBTri;
                second = best;
                best = e;
                best_t = t;
                babc[0] = tr[0];
                babc[1] = tr[1];
                babc[2] = tr[2];
            } else if (e < second) {
                second = e;
            }
        }
    }
    if (tid == 0) {
        if (status) {   // 1: the reference would never return; 2: draw budget; 3: above the launch's LDS bound
            best_t = -1;
            flags |= status == 1 ? 8u : status == 2 ? 16u : 32u;
        }
        if (best_t >= 0 && second <= best * (1.0 + 1e-9)) flags |= 4u;   // near-tie
        out_trial[frame] = best_t;
        out_err[frame] = best;
        out_flags[frame] = flags;
        out_abc[3 * frame + 0] = babc[0];
        out_abc[3 * frame + 1] = babc[1];
        out_abc[3 * frame + 2] = babc[2];
    }
    SVX_EVAL_STAMP(5);
}
#undef SVX_EVAL_STAMP

#ifdef SVX_DIAG
hipError_t diag_eval_phases(unsigned long long* out, bool reset) {   // (diagnostic build)
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_eval_phase), sizeof(unsigned long long) * 8);
    if (e == hipSuccess && reset) {
        static const unsigned long long zero[8] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_eval_phase), zero, sizeof(zero));
    }
    return e;
}
#endif

template <class IdxT>
static hipError_t launch_ransac_typed(const uint32_t* packed, const RbTables& tb, int64_t cap, const KParams& cp,
                                      const int64_t* counts, int64_t max_n, int64_t words, uint64_t seed_base,
                                      int64_t first_frame, int frames, int trials, int k, const RansacScratch& rs,
                                      double* abc, double* err, int32_t* trial, uint32_t* flags, int32_t* trace,
                                      int trace_trials, int ablate, int phases, uint64_t* started, uint64_t epoch,
                                      hipStream_t s) {
    IdxT* sidx = reinterpret_cast<IdxT*>(rs.sidx);
    // frames a draw wave walks: 1, or in the frame loop (started: the draw runs beside another batch's pipeline)
    // SVX_DRAW_FPW (diagnostic build, A/B)
    // eight frames' waves a workgroup (two a SIMD as the dispatcher places a workgroup's waves), each wave its own
    // frame and LDS: the batched RANSAC 6.35 vs 6.93 ms with four against one a workgroup, the frame loop
    // 14.48-14.68 vs 14.72-14.79 ms (profiles/r06/ab_draw_wpg_s16.txt); eight against four: RANSAC equal, the loop
    // 14.54-14.66 vs 14.65-14.83 ms in five alternations on two boxes (ab_draw_wpg_s17.txt, _s18.txt);
    // SVX_DRAW_WPG (diagnostic build) 1, 2, 4, 8 or 16
    int fpw = 1, wpg = 8;
    if (started)
        if (const char* e = svx_knob("SVX_DRAW_FPW")) fpw = std::max(1, std::atoi(e));
    if (const char* e = svx_knob("SVX_DRAW_WPG")) {
        const int v = std::atoi(e);
        wpg = v == 1 || v == 2 || v == 8 || v == 16 ? v : 4;
    }
    while (wpg > 1 && (trace || words * wpg > 16384)) wpg /= 2;   // traced: one wave a workgroup; dynamic LDS <= 64 KiB
    const int waves = (frames + fpw - 1) / fpw, grid = (waves + wpg - 1) / wpg;
    const size_t ddyn = sizeof(uint32_t) * (size_t)words * (size_t)wpg;
#define SVX_DRAW(TRv, WPGv, TRP, TRN)                                                                            \
    hipLaunchKernelGGL((ransac_draw_kernel<IdxT, TRv, WPGv>), dim3(grid), dim3(64 * WPGv), ddyn, s, packed, tb, cap, \
                       counts, seed_base, first_frame, trials, k, sidx, rs.tri, rs.fstat, TRP, TRN, (int)words,     \
                       ablate, started, epoch, frames)
    if (!(phases & 1)) {
    } else if (trace) {
        SVX_DRAW(true, 1, trace, trace_trials);
    } else if (wpg == 2) {
        SVX_DRAW(false, 2, nullptr, 0);
    } else if (wpg == 4) {
        SVX_DRAW(false, 4, nullptr, 0);
    } else if (wpg == 8) {
        SVX_DRAW(false, 8, nullptr, 0);
    } else if (wpg == 16) {
        SVX_DRAW(false, 16, nullptr, 0);
    } else {
        SVX_DRAW(false, 1, nullptr, 0);
    }
#undef SVX_DRAW
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !(phases & 2)) return e;
    if (ablate & (8 | 16)) ablate |= 1;   // DIAGNOSTIC: no samples / planes drawn -> no evaluation of them
    // eval LDS: the points when they fit beside the screen results (160 KiB per workgroup)
    // per trial: screened mean + bound (2 doubles), candidate index and its fp64 error
    const size_t scr = sizeof(double) * 2 * (size_t)trials + sizeof(int32_t) * ((size_t)trials + 1) +
                       sizeof(double) * ((size_t)trials + 1);
    const int64_t pts_words = (max_n + 1) & ~1ll;   // the doubles after the points stay 8-byte aligned
    const size_t pts_b = sizeof(uint32_t) * (size_t)pts_words;
    bool lds_pts = pts_b + scr <= 150 * 1024;
    // SVX_EVAL_LDS_PTS=0 (diagnostic build, A/B): the points gathered from memory (L2) instead of LDS
    if (const char* e = svx_knob("SVX_EVAL_LDS_PTS"); e && e[0] == '0') lds_pts = false;
    const size_t dyn = (lds_pts ? pts_b : 0) + scr;
    if (lds_pts) {
        // dynamic LDS above 64 KiB needs the per-kernel opt-in (on the current device)
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&ransac_eval_kernel<IdxT, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((ransac_eval_kernel<IdxT, true>), dim3(frames), dim3(kRBEvalThreads), dyn, s, packed,
                           tb, cap, cp, counts, trials, k, sidx, rs.tri, rs.fstat, abc, err, trial, flags, ablate,
                           (int)pts_words);
    } else {
        hipLaunchKernelGGL((ransac_eval_kernel<IdxT, false>), dim3(frames), dim3(kRBEvalThreads), dyn, s, packed,
                           tb, cap, cp, counts, trials, k, sidx, rs.tri, rs.fstat, abc, err, trial, flags, ablate, 0);
    }
    return hipGetLastError();
}

size_t ransac_sidx_bytes(int64_t max_n, int frames, int trials, int k) {
    return (max_n <= 65535 ? 2 : 4) * (size_t)frames * (size_t)trials * (size_t)k;
}

hipError_t launch_ransac_batch(const uint32_t* packed, const double* tab, int H, int W, int64_t cap, const KParams& cp,
                               const int64_t* counts, int64_t max_n, int64_t max_pool_n, uint64_t seed_base,
                               int64_t first_frame, int frames, int trials, int k, const RansacScratch& rs, double* abc,
                               double* err, int32_t* trial, uint32_t* flags, int32_t* trace, int trace_trials,
                               int ablate, int phases, uint64_t* started, uint64_t epoch, hipStream_t s) {
    if (frames <= 0) return hipSuccess;
    if (k < 1 || k > kRBMaxK || trials > kRBMaxTrials || cap > (int64_t)kRBBitmapWords * 32 || max_n > cap)
        return hipErrorInvalidValue;
    // draw-kernel LDS: the set branch's bitmap (n bits) for the largest frame, or the pool branch's list (k words)
    int64_t words = (max_n + 31) / 32;
    if (max_pool_n > 0 && k > words) words = k;
    if (words < 1) words = 1;
    words = (words + 3) & ~3ll;   // the bitmap is cleared 4 words a store
    // the samples as u16 indices when every frame has < 65536 points
    if (max_n <= 65535)
        return launch_ransac_typed<uint16_t>(packed, rb_tables(tab, H, W), cap, cp, counts, max_n, words, seed_base,
                                             first_frame,
                                             frames, trials, k, rs, abc, err, trial, flags, trace, trace_trials, ablate,
                                             phases, started, epoch, s);
    return launch_ransac_typed<int32_t>(packed, rb_tables(tab, H, W), cap, cp, counts, max_n, words, seed_base,
                                        first_frame, frames,
                                        trials, k, rs, abc, err, trial, flags, trace, trace_trials, ablate, phases,
                                        started, epoch, s);
}

// The frame loop's dispatch gate (one wave): returns once *flag >= epoch — the RANSAC draw kernel's last
// workgroup has been placed, so all its waves are resident — or after max_ns of wall clock (ordering is a
// performance heuristic only: nothing computed depends on it, so the gate never waits unboundedly). The kernel
// enqueued after it on the same stream then takes the CU resources the draw left.
__global__ __launch_bounds__(64) void loop_gate_kernel(const uint64_t* __restrict__ flag, uint64_t epoch,
                                                       uint64_t max_ticks) {
    if (lane_id() != 0) return;
    const uint64_t t0 = wall_clock64();   // constant 100 MHz counter
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch &&
           wall_clock64() - t0 < max_ticks)
        __builtin_amdgcn_s_sleep(8);
}

hipError_t launch_loop_gate(const uint64_t* flag, uint64_t epoch, double max_ms, hipStream_t s) {
    const uint64_t ticks = (uint64_t)(max_ms * 1e5);   // wall_clock64 ticks at 100 MHz
    hipLaunchKernelGGL(loop_gate_kernel, dim3(1), dim3(64), 0, s, flag, epoch, ticks);
    return hipGetLastError();
}

// keep1 plane fields of every frame (plane_fields, as the host's set_plane)
__global__ void frame_planes_kernel(const double* __restrict__ abc, const int32_t* __restrict__ trial, int frames,
                                    KParams p, double thr, FramePlane* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= frames) return;
    FramePlane o;
    if (!trial || trial[i] >= 0) {
        plane_fields(o, abc[3 * i], abc[3 * i + 1], abc[3 * i + 2], p.f, p.B, p.cw, p.ch, thr, p.W, p.H);
    } else {
        plane_fields(o, 0.0, 0.0, 0.0, p.f, p.B, p.cw, p.ch, thr, p.W, p.H);
        o.valid = 0;
    }
    out[i] = o;
}

hipError_t launch_frame_planes(const double* abc, const int32_t* trial, int frames, const KParams& p, double thr,
                               FramePlane* out, hipStream_t s) {
    if (frames <= 0) return hipSuccess;
    hipLaunchKernelGGL(frame_planes_kernel, dim3((frames + 255) / 256), dim3(256), 0, s, abc, trial, frames, p, thr,
                       out);
    return hipGetLastError();
}

}  // namespace svx
