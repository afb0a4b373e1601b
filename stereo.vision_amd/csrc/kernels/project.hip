// Projection kernels (gfx950).
//
//  * synth_kernel            — counter-based synthetic frames, on device
//  * project_dense_kernel    — K1: every grid pixel -> fp32 X,Y,Z planes (configs 2/3)
//  * project_compact_f64     — drop-in projectDisparityTo3d (functions.py:178-198):
//                              fp64, raster-ordered compaction of the d>0 pixels
//  * backproject_f64_kernel  — drop-in project3DPointsTo2DImagePoints (functions.py:201-209)
//
// K1 is a pure HBM stream: 1 B of disparity in, 12 B of fp32 XYZ out per grid
// point. One lane owns one "quad" (4 consecutive grid points of a row): a
// 4-byte (step 1) or 8-byte (step 2) disparity load and three 16-byte stores,
// one per plane, so every wave-instruction writes 1 KiB contiguous.
#include "../svx_launch.h"

namespace svx {

// ---------------------------------------------------------------------------
// Synthetic frames: one lane per 4 pixels (dword of disparity, 3 dwords BGR).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// grid (blocks over a frame's quads, frames): a quad's row and column from one 32-bit multiply-shift (fastdiv40,
// exact below 2^28 quads a frame), its pixels' counter from one 64-bit base; the row's disparity trend once a quad
__global__ __launch_bounds__(256) void synth_kernel(uint8_t* __restrict__ disp, uint8_t* __restrict__ bgr,
                                                    int H, int W, int frames, int64_t first_frame, uint64_t Wq_m40) {
    const int Wq = W / 4;
    const int qf = H * Wq;   // quads a frame
    for (int f = blockIdx.y; f < frames; f += gridDim.y) {
        const int64_t fq = (int64_t)f * qf;
        for (int qi = blockIdx.x * 256 + threadIdx.x; qi < qf; qi += gridDim.x * 256) {
            const int y = fastdiv40(qi, Wq_m40);
            const int x0 = 4 * (qi - y * Wq);
            const uint64_t base = ((uint64_t)(first_frame + f) * H + y) * W + x0;
            // floor((3*(y-200))/5) with Python floor semantics
            const int num = 3 * (y - 200);
            const int trend = (num >= 0) ? num / 5 : -((-num + 4) / 5);
            uint32_t dw = 0;
            uint32_t c[3] = {0, 0, 0};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t idx = base + k;
                const uint64_t r = mix64(idx + 0x5EED000000000001ull);
                const uint64_t r2 = mix64(idx + 0x5EED000000000002ull);
                int t = trend + (int)((r >> 8) & 7) - 3;
                t = t < 0 ? 0 : (t > 254 ? 254 : t);
                uint32_t d = (uint32_t)(t & ~1);
                if ((r & 0xFF) < 38) d = 0;
                dw |= d << (8 * k);
                uint32_t B, G, R;
                if (y >= 262) {
                    B = 110 + (uint32_t)(r2 & 3);
                    G = 100 + (uint32_t)((r2 >> 2) & 3);
                    R = 90 + (uint32_t)((r2 >> 4) & 3);
                } else {
                    B = (uint32_t)(r2 & 255);
                    G = (uint32_t)((r2 >> 8) & 255);
                    R = (uint32_t)((r2 >> 16) & 255);
                }
                const int o = 3 * k;
                c[(o + 0) >> 2] |= B << (8 * ((o + 0) & 3));
                c[(o + 1) >> 2] |= G << (8 * ((o + 1) & 3));
                c[(o + 2) >> 2] |= R << (8 * ((o + 2) & 3));
            }
            reinterpret_cast<uint32_t*>(disp)[fq + qi] = dw;
            if (bgr) {
                uint32_t* cb = reinterpret_cast<uint32_t*>(bgr) + 3 * (fq + qi);
                cb[0] = c[0];
                cb[1] = c[1];
                cb[2] = c[2];
            }
        }
    }
}

hipError_t launch_synth(const KParams& p, uint8_t* disp, uint8_t* bgr, int frames,
                        int64_t first_frame, hipStream_t s) {
    if (frames <= 0) return hipSuccess;
    const int64_t qf = (int64_t)p.H * (p.W / 4);
    if (qf <= 0) return hipSuccess;
    if (qf >= (1ll << 28) || p.W % 4) return hipErrorInvalidValue;   // fastdiv40's range; whole quads a row
    const unsigned bx = (unsigned)std::min<int64_t>((qf + 255) / 256, 1024);
    const unsigned by = (unsigned)std::min(frames, 65535);
    const uint64_t wq_m40 = ((1ull << 40) + (uint64_t)(p.W / 4) - 1) / (uint64_t)(p.W / 4);
    hipLaunchKernelGGL(synth_kernel, dim3(bx, by), dim3(256), 0, s, disp, bgr, p.H, p.W, frames, first_frame, wq_m40);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K1: dense projection. Z = fB/d, X = (x-cw)*B/d, Y = (y-ch)*B/d in fp32
// (B/d = Z/f; rcp has <= 1 ulp error: |rel err| < 2^-21 vs the fp64 reference,
// far inside the 1e-5 contract). d == 0 and pad columns (gx >= Wg) -> 0.
// ---------------------------------------------------------------------------
template <int STEP>
__device__ __forceinline__ void load_disp_quad(const uint8_t* row, int q, uint32_t (&d)[4]) {
    if constexpr (STEP == 1) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(row + 4 * q);
        d[0] = w & 0xFF; d[1] = (w >> 8) & 0xFF; d[2] = (w >> 16) & 0xFF; d[3] = w >> 24;
    } else {
        const uint2 w = *reinterpret_cast<const uint2*>(row + 8 * q);
        d[0] = w.x & 0xFF; d[1] = (w.x >> 16) & 0xFF; d[2] = w.y & 0xFF; d[3] = (w.y >> 16) & 0xFF;
    }
}

typedef float v4f __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void store4(float* p, float a, float b, float c, float d) {
    const v4f v = {a, b, c, d};
    if constexpr (NT) {
        __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(p));
    } else {
        *reinterpret_cast<v4f*>(p) = v;
    }
}

template <int STEP, bool NT>
__device__ __forceinline__ void project_quad(const uint32_t (&d)[4], int q, int y, float* __restrict__ X,
                                             float* __restrict__ Y, float* __restrict__ Z, size_t o,
                                             const KParams& p) {
    const float yc = centred(y, p.ch_hi, p.ch_lo);
    float ox[4], oy[4], oz[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int gx = 4 * q + k;
        const float xc = centred(gx * STEP, p.cw_hi, p.cw_lo);
        const float r = __builtin_amdgcn_rcpf((float)d[k]);
        const float K = p.B32 * r;
        const bool ok = (d[k] != 0) && (gx < p.Wg);
        ox[k] = ok ? xc * K : 0.0f;
        oy[k] = ok ? yc * K : 0.0f;
        oz[k] = ok ? p.fB32 * r : 0.0f;
    }
    store4<NT>(X + o, ox[0], ox[1], ox[2], ox[3]);
    store4<NT>(Y + o, oy[0], oy[1], oy[2], oy[3]);
    store4<NT>(Z + o, oz[0], oz[1], oz[2], oz[3]);
}

// One block = QPL consecutive 256-quad slabs of the flattened (frame, row,
// quad) space; every lane issues its QPL disparity loads before any store.
// TAG only names a second, identical instance (bench.py's 1-frame latency
// probe), so that profiler statistics keep its launches apart.
template <int STEP, bool NT, int QPL, int TAG = 0>
__global__ __launch_bounds__(256) void project_dense_kernel(const uint8_t* __restrict__ disp,
                                                            float* __restrict__ X, float* __restrict__ Y,
                                                            float* __restrict__ Z, uint32_t total_quads,
                                                            KParams p) {
    const uint32_t base = blockIdx.x * (256u * QPL) + threadIdx.x;
    uint32_t d[QPL][4];
    int qv[QPL], yv[QPL];
#pragma unroll
    for (int j = 0; j < QPL; ++j) {
        uint32_t g = base + 256u * j;
        g = g < total_quads ? g : total_quads - 1;   // branch-free; stores are masked below
        const uint32_t row = g / (uint32_t)p.Q;
        qv[j] = (int)(g - row * (uint32_t)p.Q);
        const uint32_t fl = row / (uint32_t)p.Hg;
        const int gy = (int)(row - fl * (uint32_t)p.Hg);
        yv[j] = gy * STEP;
        load_disp_quad<STEP>(disp + (int64_t)fl * p.frame_px + (int64_t)yv[j] * p.W, qv[j], d[j]);
    }
#pragma unroll
    for (int j = 0; j < QPL; ++j) {
        const uint32_t g = base + 256u * j;
        if (g < total_quads) project_quad<STEP, NT>(d[j], qv[j], yv[j], X, Y, Z, (size_t)g * 4, p);
    }
}

// the instance's name as rocprofv3 prints it (kname of launch_project_dense)
template <int STEP, bool NT, int QPL, int TAG>
static const char* dense_name() {
    static const char* const n[2][2][5][2] = {
        {{{}, {"svx::project_dense_kernel<1, false, 1, 0>", "svx::project_dense_kernel<1, false, 1, 1>"},
          {"svx::project_dense_kernel<1, false, 2, 0>"}, {}, {"svx::project_dense_kernel<1, false, 4, 0>"}},
         {{}, {"svx::project_dense_kernel<1, true, 1, 0>", "svx::project_dense_kernel<1, true, 1, 1>"},
          {"svx::project_dense_kernel<1, true, 2, 0>"}, {}, {"svx::project_dense_kernel<1, true, 4, 0>"}}},
        {{{}, {"svx::project_dense_kernel<2, false, 1, 0>", "svx::project_dense_kernel<2, false, 1, 1>"},
          {"svx::project_dense_kernel<2, false, 2, 0>"}, {}, {"svx::project_dense_kernel<2, false, 4, 0>"}},
         {{}, {"svx::project_dense_kernel<2, true, 1, 0>", "svx::project_dense_kernel<2, true, 1, 1>"},
          {"svx::project_dense_kernel<2, true, 2, 0>"}, {}, {"svx::project_dense_kernel<2, true, 4, 0>"}}}};
    return n[STEP - 1][NT ? 1 : 0][QPL][TAG];
}

template <int STEP, bool NT>
static const char* launch_dense_qpl(int qpl, dim3 block, const uint8_t* disp, float* X, float* Y, float* Z,
                                    uint32_t t, const KParams& p, hipStream_t s) {
    const uint32_t per = 256u * (uint32_t)qpl;
    const dim3 grid((t + per - 1) / per);
    switch (qpl) {
        case 2:
            hipLaunchKernelGGL((project_dense_kernel<STEP, NT, 2>), grid, block, 0, s, disp, X, Y, Z, t, p);
            return dense_name<STEP, NT, 2, 0>();
        case 4:
            hipLaunchKernelGGL((project_dense_kernel<STEP, NT, 4>), grid, block, 0, s, disp, X, Y, Z, t, p);
            return dense_name<STEP, NT, 4, 0>();
        default:
            hipLaunchKernelGGL((project_dense_kernel<STEP, NT, 1>), grid, block, 0, s, disp, X, Y, Z, t, p);
            return dense_name<STEP, NT, 1, 0>();
    }
}

hipError_t launch_project_dense(const KParams& p, const uint8_t* disp, float* X, float* Y, float* Z,
                                int frames, int qpl, int nontemporal, hipStream_t s, const char** kname) {
    const uint64_t total = (uint64_t)frames * (uint64_t)p.frame_quads;
    if (total >= (1ull << 32)) return hipErrorInvalidValue;
    const dim3 block(256);
    const uint32_t t = (uint32_t)total;
    const char* name = nullptr;
    if (nontemporal == 2) {   // the same K1, one quad per lane, as a separately named instance
        const dim3 grid((t + 255) / 256);
        if (p.step == 1) {
            hipLaunchKernelGGL((project_dense_kernel<1, true, 1, 1>), grid, block, 0, s, disp, X, Y, Z, t, p);
            name = dense_name<1, true, 1, 1>();
        } else if (p.step == 2) {
            hipLaunchKernelGGL((project_dense_kernel<2, true, 1, 1>), grid, block, 0, s, disp, X, Y, Z, t, p);
            name = dense_name<2, true, 1, 1>();
        } else {
            return hipErrorInvalidValue;
        }
    } else if (p.step == 1) {
        name = nontemporal ? launch_dense_qpl<1, true>(qpl, block, disp, X, Y, Z, t, p, s)
                           : launch_dense_qpl<1, false>(qpl, block, disp, X, Y, Z, t, p, s);
    } else if (p.step == 2) {
        name = nontemporal ? launch_dense_qpl<2, true>(qpl, block, disp, X, Y, Z, t, p, s)
                           : launch_dense_qpl<2, false>(qpl, block, disp, X, Y, Z, t, p, s);
    } else {
        return hipErrorInvalidValue;
    }
    if (kname) *kname = name;
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Drop-in projection (functions.py:178-198): fp64, bit-identical arithmetic,
// raster-ordered compaction of d > 0 across workgroups (decoupled look-back).
// Tile = 1024 consecutive grid points (256 lanes x 4). Any H, W, step.
// ---------------------------------------------------------------------------
constexpr int kCompactTile = 1024;

int project_compact_tiles(const KParams& p) {
    const int64_t ng = (int64_t)p.Hg * p.Wg;
    return (int)((ng + kCompactTile - 1) / kCompactTile);
}

__global__ __launch_bounds__(256) void project_compact_f64_kernel(
    const uint8_t* __restrict__ disp, int64_t ld_disp, const uint8_t* __restrict__ bgr, int64_t ld_bgr,
    double* __restrict__ xyz, uint8_t* __restrict__ rgb, uint64_t* status, uint32_t* ticket,
    uint32_t* count, uint32_t* err, int tiles, KParams p) {
    __shared__ uint32_t sh_tile, sh_excl;
    __shared__ uint32_t sh_wave[4];
    const int tid = threadIdx.x;
    if (tid == 0) sh_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const int tile = (int)sh_tile;
    const int64_t ng = (int64_t)p.Hg * p.Wg;
    const int64_t i0 = (int64_t)tile * kCompactTile + 4 * tid;
    uint32_t dv[4];
    int gyv[4], gxv[4];
    uint32_t mask = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t i = i0 + k;
        dv[k] = 0;
        gyv[k] = gxv[k] = 0;
        if (i < ng) {
            const int gy = (int)(i / p.Wg);
            const int gx = (int)(i - (int64_t)gy * p.Wg);
            gyv[k] = gy;
            gxv[k] = gx;
            dv[k] = disp[(int64_t)gy * p.step * ld_disp + (int64_t)gx * p.step];
            if (dv[k]) mask |= 1u << k;
        }
    }
    const uint32_t cnt = __builtin_popcount(mask);
    const uint32_t inc = wave_incl_scan(cnt);
    const int wave = tid >> 6;
    if (lane_id() == 63) sh_wave[wave] = inc;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t t = sh_wave[w];
        wbase += (w < wave) ? t : 0u;
        total += t;
    }
    if (wave == 0) {
        uint32_t excl = 0;
        if (tile == 0) {
            if (tid == 0) publish(status, kFlagInc, total);
        } else {
            if (tid == 0) publish(status + tile, kFlagAgg, total);
            excl = lookback(status, tile, err);
            if (tid == 0) publish(status + tile, kFlagInc, excl + total);
        }
        if (tid == 0) {
            sh_excl = excl;
            if (tile == tiles - 1) *count = excl + total;
        }
    }
    __syncthreads();
    uint32_t o = sh_excl + wbase + inc - cnt;
    const double fB = p.fB;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (!(mask & (1u << k))) continue;
        const int y = gyv[k] * p.step, x = gxv[k] * p.step;
        const double Zv = fB / (double)dv[k];
        const double Xv = (((double)x - p.cw) * Zv) / p.f;
        const double Yv = (((double)y - p.ch) * Zv) / p.f;
        xyz[3 * (size_t)o + 0] = Xv;
        xyz[3 * (size_t)o + 1] = Yv;
        xyz[3 * (size_t)o + 2] = Zv;
        if (rgb) {
            const uint8_t* px = bgr + (int64_t)y * ld_bgr + 3 * (int64_t)x;
            rgb[3 * (size_t)o + 0] = px[2];
            rgb[3 * (size_t)o + 1] = px[1];
            rgb[3 * (size_t)o + 2] = px[0];
        }
        ++o;
    }
}

hipError_t launch_project_compact_f64(const KParams& p, const uint8_t* disp, int64_t ld_disp,
                                      const uint8_t* bgr, int64_t ld_bgr, double* xyz, uint8_t* rgb,
                                      uint64_t* status, uint32_t* ticket, uint32_t* count,
                                      uint32_t* err, hipStream_t s) {
    const int tiles = project_compact_tiles(p);
    if (tiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(project_compact_f64_kernel, dim3(tiles), dim3(256), 0, s, disp, ld_disp, bgr,
                       ld_bgr, xyz, rgb, status, ticket, count, err, tiles, p);
    return hipGetLastError();
}

// The drop-in's rows (sv_project_rows): X, Y, Z and the colour bytes as doubles, 6 a row, so the host receives
// the array it returns in one copy (no numpy assembly of two arrays).
__global__ __launch_bounds__(256) void rows6_kernel(const double* __restrict__ xyz, const uint8_t* __restrict__ rgb,
                                                    int64_t n, double* __restrict__ rows) {
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        double* r = rows + 6 * i;
        r[0] = xyz[3 * i];
        r[1] = xyz[3 * i + 1];
        r[2] = xyz[3 * i + 2];
        r[3] = (double)rgb[3 * i];
        r[4] = (double)rgb[3 * i + 1];
        r[5] = (double)rgb[3 * i + 2];
    }
}

hipError_t launch_rows6(const double* xyz, const uint8_t* rgb, int64_t n, double* rows, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(rows6_kernel, dim3(g), dim3(256), 0, s, xyz, rgb, n, rows);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Drop-in back-projection (functions.py:201-209), fp64, bit-identical.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void backproject_f64_kernel(const double* __restrict__ xyz, int64_t n,
                                                              int64_t ld, double f, double cw, double ch,
                                                              double* __restrict__ xy) {
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const double X = xyz[i * ld], Y = xyz[i * ld + 1], Z = xyz[i * ld + 2];
        xy[2 * i] = ((X * f) / Z) + cw;
        xy[2 * i + 1] = ((Y * f) / Z) + ch;
    }
}

hipError_t launch_backproject_f64(const double* xyz, int64_t n, int64_t ld, double f, double cw,
                                  double ch, double* xy, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(backproject_f64_kernel, dim3((unsigned)blocks), dim3(256), 0, s, xyz, n, ld, f,
                       cw, ch, xy);
    return hipGetLastError();
}

}  // namespace svx
