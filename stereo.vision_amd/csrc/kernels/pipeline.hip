// Plane-threshold + hue-histogram + compaction pipeline (gfx950), config 4.
//
// Per frame (stereovision.py:97-113): keep1 = dist(P, plane) < point_thr
// (functions.py:300-323); hist = hue-bin counts over keep1 (functions.py:215-226);
// keep2 = keep1 & hist[bin] > hist_thr (functions.py:228-230); output the keep2
// points in reference (raster) order as fp32 XYZ + int32 (x,y) back-projection
// (functions.py:201-209 + stereovision.py:112).
//
// The histogram must be complete before any point can be filtered, so each
// chunk of frames takes two launches:
//   pass 1  hist_kernel     frames x slices workgroups; LDS histogram (4 KB),
//                           flushed with one global atomic per non-zero bin.
//   pass 2  compact_kernel  one 4096-point tile per workgroup; wave ballot/scan
//                           + LDS block scan inside the tile, decoupled
//                           look-back across the tiles of a frame (tile ids
//                           from an atomic ticket => forward progress).
// A chunk is small enough (default 16 frames = 36 MB of input) that pass 2
// re-reads its inputs from the 256 MB Infinity Cache rather than HBM.
#include "../svx_launch.h"

namespace svx {

constexpr int kHistQuadsPerThread = 16;   // pass-1 slice = 256 x 16 quads
constexpr int kQPT = 4;                   // pass-2 tile  = 256 x 4 quads = 4096 points

template <int STEP>
struct QuadIn {
    uint32_t d[4];
    uint32_t c[3 * STEP];  // BGR bytes of the quad's source pixels
};

template <int STEP>
__device__ __forceinline__ void load_quad(const uint8_t* drow, const uint8_t* crow, int q, QuadIn<STEP>& o) {
    if constexpr (STEP == 1) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(drow + 4 * q);
        o.d[0] = w & 0xFF; o.d[1] = (w >> 8) & 0xFF; o.d[2] = (w >> 16) & 0xFF; o.d[3] = w >> 24;
        const uint32_t* cp = reinterpret_cast<const uint32_t*>(crow + 12 * q);
        o.c[0] = cp[0]; o.c[1] = cp[1]; o.c[2] = cp[2];
    } else {
        const uint2 w = *reinterpret_cast<const uint2*>(drow + 8 * q);
        o.d[0] = w.x & 0xFF; o.d[1] = (w.x >> 16) & 0xFF; o.d[2] = w.y & 0xFF; o.d[3] = (w.y >> 16) & 0xFF;
        const uint2* cp = reinterpret_cast<const uint2*>(crow + 24 * q);
        const uint2 a = cp[0], b = cp[1], c = cp[2];
        o.c[0] = a.x; o.c[1] = a.y; o.c[2] = b.x; o.c[3] = b.y; o.c[4] = c.x; o.c[5] = c.y;
    }
}

template <int STEP>
__device__ __forceinline__ uint32_t quad_byte(const QuadIn<STEP>& o, int i) {
    return (o.c[i >> 2] >> (8 * (i & 3))) & 0xFF;
}

// Evaluate point k of a quad: returns 0 = not kept, 1 + bin = plane-kept.
template <int STEP>
__device__ __forceinline__ int eval_point(const QuadIn<STEP>& in, int k, int gx, int y, float yc,
                                          const KParams& p) {
    const uint32_t d = in.d[k];
    if (d == 0 || gx >= p.Wg) return 0;
    const int x = gx * STEP;
    const float xc = (float)((double)x - p.cw);
    const float r = __builtin_amdgcn_rcpf((float)d);
    const float K = p.B32 * r;
    const float X = xc * K, Y = yc * K, Z = p.fB32 * r;
    if (!keep1(x, y, d, xc, yc, K, X, Y, Z, p)) return 0;
    const int o = 3 * STEP * k;  // byte offset of the pixel inside the quad's BGR
    const int B = (int)quad_byte<STEP>(in, o), G = (int)quad_byte<STEP>(in, o + 1),
              R = (int)quad_byte<STEP>(in, o + 2);
    return 1 + hue_bin(R, G, B);
}

int pipeline_slices_per_frame(const KParams& p) {
    const int per = 256 * kHistQuadsPerThread;
    return (p.frame_quads + per - 1) / per;
}

int pipeline_tiles_per_frame(const KParams& p) {
    const int per = 256 * kQPT;
    return (p.frame_quads + per - 1) / per;
}

// ---------------------------------------------------------------------------
// pass 1: histogram + N_valid / N_kept. Also zeroes pass 2's look-back state.
// ---------------------------------------------------------------------------
template <int STEP>
__global__ __launch_bounds__(256) void hist_kernel(PipeBuffers bf, int frame0, int slices,
                                                   int status_words, KParams p) {
    __shared__ uint32_t sh_hist[kBins];
    __shared__ uint32_t sh_cnt[2];
    const int tid = threadIdx.x;
    for (int i = tid; i < kBins; i += 256) sh_hist[i] = 0;
    if (tid < 2) sh_cnt[tid] = 0;
    // zero this chunk's look-back granules and ticket (pass 2 runs after us)
    {
        const int per = (status_words + gridDim.x - 1) / gridDim.x;
        const int s0 = blockIdx.x * per;
        for (int i = s0 + tid; i < s0 + per && i < status_words; i += 256) bf.status[i] = 0;
        if (blockIdx.x == 0 && tid == 0) *bf.ticket = 0;
    }
    __syncthreads();

    const int fl = blockIdx.x / slices;
    const int slice = blockIdx.x - fl * slices;
    const int frame = frame0 + fl;
    const uint8_t* disp = bf.disp + (int64_t)frame * p.frame_px;
    const uint8_t* bgr = bf.bgr + (int64_t)frame * p.frame_px * 3;
    const int q0 = slice * 256 * kHistQuadsPerThread;
    const int q1 = min(q0 + 256 * kHistQuadsPerThread, p.frame_quads);
    uint32_t nv = 0, nk = 0;
    for (int qi = q0 + tid; qi < q1; qi += 256) {
        const int gy = qi / p.Q;
        const int q = qi - gy * p.Q;
        const int y = gy * STEP;
        QuadIn<STEP> in;
        load_quad<STEP>(disp + (int64_t)y * p.W, bgr + (int64_t)y * p.W * 3, q, in);
        const float yc = (float)((double)y - p.ch);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int gx = 4 * q + k;
            nv += (in.d[k] != 0 && gx < p.Wg) ? 1u : 0u;
            const int e = eval_point<STEP>(in, k, gx, y, yc, p);
            if (e) {
                ++nk;
                atomicAdd(&sh_hist[e - 1], 1u);
            }
        }
    }
    nv = wave_sum(nv);
    nk = wave_sum(nk);
    if (lane_id() == 0) {
        atomicAdd(&sh_cnt[0], nv);
        atomicAdd(&sh_cnt[1], nk);
    }
    __syncthreads();
    if (tid == 0) {
        atomicAdd(reinterpret_cast<unsigned long long*>(bf.counts + 4 * frame + 0), (unsigned long long)sh_cnt[0]);
        atomicAdd(reinterpret_cast<unsigned long long*>(bf.counts + 4 * frame + 1), (unsigned long long)sh_cnt[1]);
    }
    uint32_t* gh = bf.hist + (int64_t)frame * kBins;
    for (int i = tid; i < kBins; i += 256) {
        const uint32_t v = sh_hist[i];
        if (v) atomicAdd(gh + i, v);
    }
}

// ---------------------------------------------------------------------------
// pass 2: keep2 filter, ordered compaction, fp32 XYZ + int32 (x, y).
// Tile = 256 lanes x kQPT quads; quad (i, lane) = tile_base + i*256 + lane, so
// each load/store wave-instruction is contiguous; the raster order inside the
// tile is (i, lane), scanned with 4 x 16-bit fields packed in one u64.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v) {
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const uint64_t t = __shfl_up(v, o, kWave);
        if (lane >= o) v += t;
    }
    return v;
}

template <int STEP>
__global__ __launch_bounds__(256) void compact_kernel(PipeBuffers bf, int frame0, int tiles, KParams p) {
    __shared__ uint32_t sh_okbits[kBins / 32];
    __shared__ uint64_t sh_wave[4];
    __shared__ uint32_t sh_tile, sh_excl;
    const int tid = threadIdx.x;
    if (tid == 0) sh_tile = atomicAdd(bf.ticket, 1u);
    __syncthreads();
    const int g = (int)sh_tile;
    const int fl = g / tiles;
    const int tile = g - fl * tiles;
    const int frame = frame0 + fl;
    {   // hist[bin] > hist_thr as a 1024-bit mask
        const uint32_t* gh = bf.hist + (int64_t)frame * kBins;
        const int wave = tid >> 6;
#pragma unroll
        for (int r = 0; r < kBins / 256; ++r) {
            const int bin = r * 256 + tid;
            const uint64_t m = __ballot((int64_t)gh[bin] > (int64_t)p.hist_thr);
            if (lane_id() == 0) {
                sh_okbits[(r * 256 + wave * 64) / 32] = (uint32_t)m;
                sh_okbits[(r * 256 + wave * 64) / 32 + 1] = (uint32_t)(m >> 32);
            }
        }
    }
    __syncthreads();

    const uint8_t* disp = bf.disp + (int64_t)frame * p.frame_px;
    const uint8_t* bgr = bf.bgr + (int64_t)frame * p.frame_px * 3;
    const int qbase = tile * 256 * kQPT;
    uint32_t dpack[kQPT];
    uint32_t keep = 0;  // bit 4*i + k
    uint64_t cnt = 0;
#pragma unroll
    for (int i = 0; i < kQPT; ++i) {
        const int qi = qbase + i * 256 + tid;
        dpack[i] = 0;
        if (qi < p.frame_quads) {
            const int gy = qi / p.Q;
            const int q = qi - gy * p.Q;
            const int y = gy * STEP;
            QuadIn<STEP> in;
            load_quad<STEP>(disp + (int64_t)y * p.W, bgr + (int64_t)y * p.W * 3, q, in);
            dpack[i] = in.d[0] | (in.d[1] << 8) | (in.d[2] << 16) | (in.d[3] << 24);
            const float yc = (float)((double)y - p.ch);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int e = eval_point<STEP>(in, k, 4 * q + k, y, yc, p);
                if (e && ((sh_okbits[(e - 1) >> 5] >> ((e - 1) & 31)) & 1)) {
                    keep |= 1u << (4 * i + k);
                    cnt += 1ull << (16 * i);
                }
            }
        }
    }
    // block scan of the packed per-quad-row counts
    const uint64_t inc = wave_incl_scan64(cnt);
    const int wave = tid >> 6;
    if (lane_id() == 63) sh_wave[wave] = inc;
    __syncthreads();
    uint64_t wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint64_t t = sh_wave[w];
        wbase += (w < wave) ? t : 0ull;
        tot += t;
    }
    const uint64_t excl_packed = wbase + inc - cnt;
    uint32_t total = 0;
#pragma unroll
    for (int i = 0; i < kQPT; ++i) total += (uint32_t)((tot >> (16 * i)) & 0xFFFF);

    if (wave == 0) {
        uint64_t* st = bf.status + (int64_t)fl * tiles;
        uint32_t excl = 0;
        if (tile == 0) {
            if (tid == 0) publish(st, kFlagInc, total);
        } else {
            if (tid == 0) publish(st + tile, kFlagAgg, total);
            excl = lookback(st, tile, bf.err);
            if (tid == 0) publish(st + tile, kFlagInc, excl + total);
        }
        if (tid == 0) {
            sh_excl = excl;
            if (tile == tiles - 1) bf.counts[4 * frame + 2] = excl + total;
        }
    }
    __syncthreads();
    if (!keep) return;

    const int64_t fbase = (int64_t)frame * bf.cap + sh_excl;
    float* oxyz = bf.xyz;
    int32_t* opts = bf.pts;
    uint32_t rowbase = 0;
#pragma unroll
    for (int i = 0; i < kQPT; ++i) {
        uint32_t o = rowbase + (uint32_t)((excl_packed >> (16 * i)) & 0xFFFF);
        rowbase += (uint32_t)((tot >> (16 * i)) & 0xFFFF);
        const uint32_t km = (keep >> (4 * i)) & 0xF;
        if (!km) continue;
        const int qi = qbase + i * 256 + tid;
        const int gy = qi / p.Q;
        const int q = qi - gy * p.Q;
        const int y = gy * STEP;
        const float yc = (float)((double)y - p.ch);
        const int dyw = y >> 5, dyb = y & 31;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (!(km & (1u << k))) continue;
            const uint32_t d = (dpack[i] >> (8 * k)) & 0xFF;
            const int x = (4 * q + k) * STEP;
            const float xc = (float)((double)x - p.cw);
            const float r = __builtin_amdgcn_rcpf((float)d);
            const float K = p.B32 * r;
            const int64_t at = fbase + o;
            oxyz[3 * at + 0] = xc * K;
            oxyz[3 * at + 1] = yc * K;
            oxyz[3 * at + 2] = p.fB32 * r;
            const int ddx = (bf.dxbits[d * p.dx_words + (x >> 5)] >> (x & 31)) & 1;
            const int ddy = (bf.dybits[d * p.dy_words + dyw] >> dyb) & 1;
            *reinterpret_cast<int2*>(opts + 2 * at) = make_int2(x - ddx, y - ddy);
            ++o;
        }
    }
}

hipError_t launch_pipeline_chunk(const KParams& p, const PipeBuffers& b, int frame0, int frames,
                                 hipStream_t s) {
    const int slices = pipeline_slices_per_frame(p);
    const int tiles = pipeline_tiles_per_frame(p);
    const int status_words = frames * tiles;
    const dim3 g1(frames * slices), g2(frames * tiles), blk(256);
    if (p.step == 1) {
        hipLaunchKernelGGL(hist_kernel<1>, g1, blk, 0, s, b, frame0, slices, status_words, p);
        hipLaunchKernelGGL(compact_kernel<1>, g2, blk, 0, s, b, frame0, tiles, p);
    } else if (p.step == 2) {
        hipLaunchKernelGGL(hist_kernel<2>, g1, blk, 0, s, b, frame0, slices, status_words, p);
        hipLaunchKernelGGL(compact_kernel<2>, g2, blk, 0, s, b, frame0, tiles, p);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace svx
