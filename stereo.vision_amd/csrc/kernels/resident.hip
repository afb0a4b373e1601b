// Frame-resident pipeline (gfx950), config 4: one workgroup owns one frame.
//
// Same chain as pipeline.hip (stereovision.py:97-113): keep1 = dist(P, plane)
// < point_thr (functions.py:300-323); hist = hue-bin counts over keep1
// (functions.py:215-226); keep2 = keep1 & hist[bin] > hist_thr
// (functions.py:228-230); the keep2 points in raster order as fp32 X, Y, Z +
// int32 (x, y) back-projection (functions.py:201-209, stereovision.py:112).
//
// Because one workgroup walks its frame chunk by chunk (chunk = 256 lanes x
// QPL quads x 4 grid points, raster order), nothing crosses workgroups: the
// histogram lives in LDS, the output offset is a running register, and there
// are no tickets, look-back, global atomics or hand-off buffers.
//
//   pass 1  per chunk: disparity + BGR in (4 B/pt); division-free keep1
//           (|u - d| < t*d, fp32 with a rigorous guard, fp64 reference
//           arithmetic inside it); the colours of kept points are packed
//           densely into the wave's LDS region and binned there (fp32 hue,
//           exact integer/fp64 path in the tie band) with LDS atomics whose
//           return value marks "candidate" chunks: a point whose bin had fewer
//           than hist_thr points before it. A bin that ends <= hist_thr has
//           ALL its points candidates, so only candidate ("dirty") chunks can
//           lose keep1 points in pass 2.
//   pass 2  per chunk: disparity in (1 B/pt), keep1 again (same code, same
//           bits); dirty chunks re-read BGR and drop points whose bin ends
//           <= hist_thr; block scan; 4-byte descriptors (d | gy | gx) scattered
//           into LDS; lane j then produces outputs 4j..4j+3 with 16-byte
//           non-temporal stores to the SoA planes, so stores are contiguous.
// Frames <= kRMaxChunks chunks; the launcher falls back to the tiled pipeline
// otherwise (and for batches too small to fill the chip).
#include "../svx_launch.h"

namespace svx {

constexpr int kRMaxChunks = 256;
constexpr int kRStage = 4096;   // LDS staging slots; a power of two (wrap-around below)
constexpr int kRBins = 1000;    // bins 0..999: t < 1000 - 1000/(6*255) so rint(t) <= 999

struct ResidentShared {
    uint32_t hist[kRBins];
    uint32_t dirty[kRMaxChunks / 32];
    uint64_t wtot[4];
    uint32_t red[8];
    uint32_t stage[kRStage];
};
static_assert(sizeof(ResidentShared) <= 20480, "8 workgroups per CU (160 KiB LDS)");

template <int STEP>
struct RCfg {
    static constexpr int QPL = STEP == 1 ? 4 : 2;   // quads per lane per chunk
    static constexpr int CW = 3 * STEP;            // BGR dwords per quad
    static constexpr int PTS = 256 * QPL * 4;      // grid points per chunk
};

int resident_chunks_per_frame(const KParams& p, int step) {
    const int per = 256 * (step == 1 ? 4 : 2);
    return (p.frame_quads + per - 1) / per;
}

template <int STEP>
struct RQuads {   // this lane's quads of one chunk
    int gy[RCfg<STEP>::QPL];   // grid row, -1 past the frame end
    int q[RCfg<STEP>::QPL];    // quad within the row
};

template <int STEP>
__device__ __forceinline__ void r_geometry(int c, int tid, const KParams& p, RQuads<STEP>& g) {
    constexpr int QPL = RCfg<STEP>::QPL;
#pragma unroll
    for (int i = 0; i < QPL; ++i) {
        const int qi = (c * QPL + i) * 256 + tid;
        const bool ok = qi < p.frame_quads;
        const int qc = ok ? qi : p.frame_quads - 1;
        const int gy = fastdiv40(qc, p.Q_m40);
        g.q[i] = qc - gy * p.Q;
        g.gy[i] = ok ? gy : -1;
    }
}

template <int STEP>
__device__ __forceinline__ const uint8_t* r_row(const uint8_t* frame_base, int gy, int bpp, const KParams& p) {
    return frame_base + (int64_t)((gy < 0 ? 0 : gy) * STEP) * p.W * bpp;
}

template <int STEP>
__device__ __forceinline__ void r_load_disp(const uint8_t* fdisp, const RQuads<STEP>& g, const KParams& p,
                                            uint32_t (&dw)[RCfg<STEP>::QPL][STEP]) {
#pragma unroll
    for (int i = 0; i < RCfg<STEP>::QPL; ++i) {
        const uint8_t* row = r_row<STEP>(fdisp, g.gy[i], 1, p);
        if constexpr (STEP == 1) {
            dw[i][0] = *reinterpret_cast<const uint32_t*>(row + 4 * g.q[i]);
        } else {
            const uint2 w = *reinterpret_cast<const uint2*>(row + 8 * g.q[i]);
            dw[i][0] = w.x;
            dw[i][1] = w.y;
        }
    }
}

template <int STEP>
__device__ __forceinline__ void r_load_bgr(const uint8_t* fbgr, const RQuads<STEP>& g, const KParams& p,
                                           uint32_t (&cw)[RCfg<STEP>::QPL][RCfg<STEP>::CW]) {
#pragma unroll
    for (int i = 0; i < RCfg<STEP>::QPL; ++i) {
        const uint8_t* row = r_row<STEP>(fbgr, g.gy[i], 3, p);
        if constexpr (STEP == 1) {
            const uint32_t* cp = reinterpret_cast<const uint32_t*>(row + 12 * g.q[i]);
            cw[i][0] = cp[0];
            cw[i][1] = cp[1];
            cw[i][2] = cp[2];
        } else {
            const uint2* cp = reinterpret_cast<const uint2*>(row + 24 * g.q[i]);
            const uint2 a = cp[0], b = cp[1], c = cp[2];
            cw[i][0] = a.x; cw[i][1] = a.y; cw[i][2] = b.x; cw[i][3] = b.y; cw[i][4] = c.x; cw[i][5] = c.y;
        }
    }
}

// disparity byte of point k of a quad
template <int STEP>
__device__ __forceinline__ uint32_t r_d(const uint32_t (&w)[STEP], int k) {
    if constexpr (STEP == 1) return (w[0] >> (8 * k)) & 0xFF;
    else return (w[k >> 1] >> (16 * (k & 1))) & 0xFF;
}

// colour (B | G<<8 | R<<16, top byte junk) of point k of a quad
template <int STEP>
__device__ __forceinline__ uint32_t r_col(const uint32_t (&c)[RCfg<STEP>::CW], int k) {
    const int o = 3 * STEP * k, w = o >> 2, sh = o & 3;
    const uint32_t hi = (w + 1 < RCfg<STEP>::CW) ? c[w + 1] : 0u;
    return sh == 0 ? c[w] : __builtin_amdgcn_alignbyte(hi, c[w], sh);
}

__device__ __forceinline__ int r_bin(uint32_t col) {
    bool near;
    int bin = hue_bin_fast(col, near);
    if (__builtin_expect(near, 0))
        bin = hue_bin((int)((col >> 16) & 0xFF), (int)((col >> 8) & 0xFF), (int)(col & 0xFF));
    return bin;
}

// keep1 bits of this lane's chunk (bit 4i+k = point k of quad i) + valid count.
template <int STEP>
__device__ __forceinline__ uint32_t r_keep1(const uint32_t (&dw)[RCfg<STEP>::QPL][STEP], const RQuads<STEP>& g,
                                            const KParams& p, uint32_t* nvalid) {
    constexpr int QPL = RCfg<STEP>::QPL;
    uint32_t keep = 0, unc = 0, nv = 0;
#pragma unroll
    for (int i = 0; i < QPL; ++i) {
        const int y = g.gy[i] * STEP;
        const float beta = __builtin_fmaf(p.bb32, (float)y, p.b032);
        const bool rowok = g.gy[i] >= 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int gx = 4 * g.q[i] + k;
            const bool in = rowok && gx < p.Wg;
            const uint32_t d = r_d<STEP>(dw[i], k);
            bool u;
            const bool kp = keep1_lean((float)(gx * STEP), beta, (float)d, p, u);
            keep |= (uint32_t)(kp && in) << (4 * i + k);
            unc |= (uint32_t)(u && in) << (4 * i + k);
            nv += (d != 0 && in) ? 1u : 0u;
        }
    }
    if (__builtin_expect(unc != 0, 0)) {   // rare: the guard band -> exact fp64 reference arithmetic
#pragma unroll
        for (int i = 0; i < QPL; ++i) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t bit = 1u << (4 * i + k);
                if (unc & bit) {
                    const bool kk = keep1_f64((4 * g.q[i] + k) * STEP, g.gy[i] * STEP, r_d<STEP>(dw[i], k), p);
                    keep = kk ? (keep | bit) : (keep & ~bit);
                }
            }
        }
    }
    if (nvalid) *nvalid += nv;
    return keep;
}

typedef float v4f __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));

template <int STEP>
__global__ __launch_bounds__(256) void resident_kernel(PipeBuffers bf, int frame0, int nchunks, KParams p) {
    constexpr int QPL = RCfg<STEP>::QPL;
    constexpr int WREGION = 64 * QPL * 4;   // staging slots per wave in pass 1
    __shared__ ResidentShared sh;
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = frame0 + blockIdx.x;
    const uint8_t* fdisp = bf.disp + (int64_t)frame * p.frame_px;
    const uint8_t* fbgr = bf.bgr + (int64_t)frame * p.frame_px * 3;
    for (int i = tid; i < kRBins; i += 256) sh.hist[i] = 0;
    if (tid < kRMaxChunks / 32) sh.dirty[tid] = 0;
    __syncthreads();

    // ---------------- pass 1: histogram + candidate chunks ----------------
    uint32_t nvalid = 0, nkept = 0;
    uint32_t* wstage = sh.stage + wave * WREGION;
    for (int c = 0; c < ((p.ablate & 128) ? 0 : nchunks); ++c) {   // ablate: DIAGNOSTIC ONLY
        RQuads<STEP> g;
        r_geometry<STEP>(c, tid, p, g);
        uint32_t dw[QPL][STEP], cw[QPL][RCfg<STEP>::CW];
        r_load_disp<STEP>(fdisp, g, p, dw);
        r_load_bgr<STEP>(fbgr, g, p, cw);
        uint32_t keep = r_keep1<STEP>(dw, g, p, &nvalid);
        if (p.ablate & 1024) keep = (cw[0][0] == 12345u) ? keep : 0u;
        const uint32_t cnt = __builtin_popcount(keep);
        nkept += cnt;
        const uint32_t inc = wave_incl_scan(cnt);
        const uint32_t wtotal = __shfl(inc, 63, kWave);
        uint32_t pos = inc - cnt;
#pragma unroll
        for (int i = 0; i < QPL; ++i) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (keep & (1u << (4 * i + k))) wstage[pos++] = r_col<STEP>(cw[i], k);
            }
        }
        bool cand = false;
        for (uint32_t j = lane; j < ((p.ablate & 512) ? 0u : wtotal); j += kWave) {   // dense: kept colours only
            const int bin = r_bin(wstage[j]);
            const uint32_t old = atomicAdd(&sh.hist[bin], 1u);
            cand |= (int64_t)old < (int64_t)p.hist_thr;
        }
        if (__ballot(cand) && lane == 0) atomicOr(&sh.dirty[c >> 5], 1u << (c & 31));
    }
    __syncthreads();   // histogram complete

    {   // the frame's histogram (read back by the API; bins >= 1000 are never produced)
        uint32_t* gh = bf.hist + (int64_t)frame * kBins;
        for (int b = tid; b < kBins; b += 256) gh[b] = b < kRBins ? sh.hist[b] : 0u;
    }

    // ---------------- pass 2: keep2 + ordered compaction + outputs ----------
    float* oX = bf.xyz + (int64_t)frame * 3 * bf.cap;
    float* oY = oX + bf.cap;
    float* oZ = oY + bf.cap;
    int32_t* oP = bf.pts + (int64_t)frame * bf.cap * 2;
    uint32_t running = 0;
    for (int c = 0; c < ((p.ablate & 256) ? 0 : nchunks); ++c) {
        RQuads<STEP> g;
        r_geometry<STEP>(c, tid, p, g);
        uint32_t dw[QPL][STEP];
        r_load_disp<STEP>(fdisp, g, p, dw);
        uint32_t keep = r_keep1<STEP>(dw, g, p, nullptr);
        if ((sh.dirty[c >> 5] >> (c & 31)) & 1) {   // uniform: rare candidate chunk
            uint32_t cw[QPL][RCfg<STEP>::CW];
            r_load_bgr<STEP>(fbgr, g, p, cw);
#pragma unroll
            for (int i = 0; i < QPL; ++i) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t bit = 1u << (4 * i + k);
                    if (keep & bit) {
                        const int bin = r_bin(r_col<STEP>(cw[i], k));
                        if (!((int64_t)sh.hist[bin] > (int64_t)p.hist_thr)) keep &= ~bit;
                    }
                }
            }
        }
        uint64_t cnt = 0;
#pragma unroll
        for (int i = 0; i < QPL; ++i) cnt += (uint64_t)__builtin_popcount((keep >> (4 * i)) & 0xF) << (16 * i);
        uint64_t inc = cnt;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
            const uint64_t t = __shfl_up(inc, o, kWave);
            if (lane >= o) inc += t;
        }
        if (lane == 63) sh.wtot[wave] = inc;
        __syncthreads();
        uint64_t wbase = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint64_t v = sh.wtot[w];
            wbase += (w < wave) ? v : 0ull;
            tot += v;
        }
        const uint64_t excl = wbase + inc - cnt;
        // LDS slot s <-> output running - lead + s, so groups of 4 are 16-byte aligned
        const uint32_t lead = running & 3;
        uint32_t rowbase = lead;
#pragma unroll
        for (int i = 0; i < QPL; ++i) {
            uint32_t o = rowbase + (uint32_t)((excl >> (16 * i)) & 0xFFFF);
            rowbase += (uint32_t)((tot >> (16 * i)) & 0xFFFF);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (keep & (1u << (4 * i + k))) {
                    const uint32_t d = r_d<STEP>(dw[i], k);
                    sh.stage[(o++) & (kRStage - 1)] = (d << 24) | ((uint32_t)g.gy[i] << 12) | (uint32_t)(4 * g.q[i] + k);
                }
            }
        }
        const uint32_t end = rowbase;   // one past the last valid slot
        __syncthreads();
        const uint32_t g0 = running - lead;
        const uint32_t groups = (end + 3) >> 2;
        for (uint32_t m = tid; m < groups; m += 256) {
            const uint4 u4 = *reinterpret_cast<const uint4*>(&sh.stage[(4 * m) & (kRStage - 1)]);
            const uint32_t u[4] = {u4.x, u4.y, u4.z, u4.w};
            float X[4], Y[4], Z[4];
            int PX[4], PY[4];
            bool ok[4];
            uint32_t wx[4], wy[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t s_ = 4 * m + e;
                ok[e] = s_ >= lead && s_ < end;
                const uint32_t uu = ok[e] ? u[e] : (1u << 24);
                const uint32_t d = uu >> 24;
                const int y = (int)((uu >> 12) & 0xFFF) * STEP;
                const int x = (int)(uu & 0xFFF) * STEP;
                wx[e] = bf.dxbits[d * p.dx_words + (x >> 5)];
                wy[e] = bf.dybits[d * p.dy_words + (y >> 5)];
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t uu = ok[e] ? u[e] : (1u << 24);
                const uint32_t d = uu >> 24;
                const int y = (int)((uu >> 12) & 0xFFF) * STEP;
                const int x = (int)(uu & 0xFFF) * STEP;
                const float r = __builtin_amdgcn_rcpf((float)d);
                const float K = p.B32 * r;
                X[e] = centred(x, p.cw_hi, p.cw_lo) * K;
                Y[e] = centred(y, p.ch_hi, p.ch_lo) * K;
                Z[e] = p.fB32 * r;
                PX[e] = x - (int)((wx[e] >> (x & 31)) & 1);
                PY[e] = y - (int)((wy[e] >> (y & 31)) & 1);
            }
            const int64_t go = (int64_t)g0 + 4 * m;
            if (ok[0] && ok[3]) {   // full group: 16-byte non-temporal stores
                __builtin_nontemporal_store((v4f){X[0], X[1], X[2], X[3]}, reinterpret_cast<v4f*>(oX + go));
                __builtin_nontemporal_store((v4f){Y[0], Y[1], Y[2], Y[3]}, reinterpret_cast<v4f*>(oY + go));
                __builtin_nontemporal_store((v4f){Z[0], Z[1], Z[2], Z[3]}, reinterpret_cast<v4f*>(oZ + go));
                __builtin_nontemporal_store((v4i){PX[0], PY[0], PX[1], PY[1]}, reinterpret_cast<v4i*>(oP + 2 * go));
                __builtin_nontemporal_store((v4i){PX[2], PY[2], PX[3], PY[3]}, reinterpret_cast<v4i*>(oP + 2 * go + 4));
            } else {                // the chunk's first / last group
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (!ok[e]) continue;
                    oX[go + e] = X[e];
                    oY[go + e] = Y[e];
                    oZ[go + e] = Z[e];
                    *reinterpret_cast<int2*>(oP + 2 * (go + e)) = make_int2(PX[e], PY[e]);
                }
            }
        }
        running += end - lead;
    }

    // ---------------- frame counts ----------------
    nvalid = wave_sum(nvalid);
    nkept = wave_sum(nkept);
    if (lane == 0) {
        sh.red[wave] = nvalid;
        sh.red[4 + wave] = nkept;
    }
    __syncthreads();
    if (tid == 0) {
        int64_t* cn = bf.counts + 4 * (int64_t)frame;
        cn[0] = (int64_t)sh.red[0] + sh.red[1] + sh.red[2] + sh.red[3];
        cn[1] = (int64_t)sh.red[4] + sh.red[5] + sh.red[6] + sh.red[7];
        cn[2] = running;
    }
}

bool resident_supported(const KParams& p) {
    return (p.step == 1 || p.step == 2) && p.Wg <= 4096 && p.Hg <= 4096 &&
           resident_chunks_per_frame(p, p.step) <= kRMaxChunks;
}

hipError_t launch_pipeline_resident(const KParams& p, const PipeBuffers& b, int frames, hipStream_t s) {
    if (frames <= 0) return hipSuccess;
    if (!resident_supported(p)) return hipErrorInvalidValue;
    const int nch = resident_chunks_per_frame(p, p.step);
    if (p.step == 1)
        hipLaunchKernelGGL(resident_kernel<1>, dim3(frames), dim3(256), 0, s, b, 0, nch, p);
    else
        hipLaunchKernelGGL(resident_kernel<2>, dim3(frames), dim3(256), 0, s, b, 0, nch, p);
    return hipGetLastError();
}

}  // namespace svx
