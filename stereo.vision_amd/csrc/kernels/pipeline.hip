// Plane-threshold + hue-histogram + compaction pipeline (gfx950), config 4.
//
// Per frame (stereovision.py:97-113): keep1 = dist(P, plane) < point_thr
// (functions.py:300-323); hist = hue-bin counts over keep1 (functions.py:215-226);
// keep2 = keep1 & hist[bin] > hist_thr (functions.py:228-230); output the keep2
// points in reference (raster) order as fp32 XYZ + int32 (x,y) back-projection
// (functions.py:201-209 + stereovision.py:112).
//
// The histogram must be complete before any point of a frame can be filtered,
// so every frame is visited twice:
//   pass 1  hist_tile     LDS histogram (4 KB) per 4096-point tile, flushed with
//                         one global atomic per non-zero bin; N_valid, N_kept.
//   pass 2  compact_tile  wave ballot/scan + LDS block scan inside the tile,
//                         decoupled look-back across the tiles of a frame,
//                         then fp32 XYZ + int32 (x,y) stores.
// Frames go in chunks; launch c runs pass 2 of chunk c-1 together with pass 1
// of chunk c (one ticketed grid), so a chunk's second read comes from the
// 256 MB Infinity Cache shortly after its first, and there are chunks+1
// launches per call. All control words (histograms, counts, look-back
// granules, per-launch tickets) are zeroed by one memset per call.
#include "../svx_launch.h"

namespace svx {

constexpr int kQPT = 4;   // tile = 256 lanes x 4 quads = 4096 grid points (both passes)

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
    const float xc = centred(x, p.cw_hi, p.cw_lo);
    const float r = __builtin_amdgcn_rcpf((float)d);
    const float K = p.B32 * r;
    const float X = xc * K, Y = yc * K, Z = p.fB32 * r;
    if (!keep1(x, y, d, xc, yc, K, X, Y, Z, p)) return 0;
    const int o = 3 * STEP * k;  // byte offset of the pixel inside the quad's BGR
    const int B = (int)quad_byte<STEP>(in, o), G = (int)quad_byte<STEP>(in, o + 1),
              R = (int)quad_byte<STEP>(in, o + 2);
    return 1 + hue_bin(R, G, B);
}

int pipeline_tiles_per_frame(const KParams& p) {
    const int per = 256 * kQPT;
    return (p.frame_quads + per - 1) / per;
}


// Issue every load of the lane's kQPT quads before any use (memory-level
// parallelism: 4 x 16 B per lane in flight).
template <int STEP>
__device__ __forceinline__ void load_tile(const uint8_t* disp, const uint8_t* bgr, int qbase, int tid,
                                          const KParams& p, QuadIn<STEP> (&in)[kQPT], int (&gy)[kQPT],
                                          int (&q)[kQPT]) {
#pragma unroll
    for (int i = 0; i < kQPT; ++i) {
        // branch-free: out-of-range lanes re-load the last quad and are masked
        // (keeps the arrays in registers and every load in flight together)
        const int qi = qbase + i * 256 + tid;
        const bool ok = qi < p.frame_quads;
        const int qc = ok ? qi : p.frame_quads - 1;
        const int g = qc / p.Q;
        q[i] = qc - g * p.Q;
        gy[i] = ok ? g : -1;
        const int y = g * STEP;
        load_quad<STEP>(disp + (int64_t)y * p.W, bgr + (int64_t)y * p.W * 3, q[i], in[i]);
    }
#pragma unroll
    for (int i = 0; i < kQPT; ++i) {
#pragma unroll
        for (int k = 0; k < 4; ++k) in[i].d[k] = gy[i] < 0 ? 0u : in[i].d[k];
    }
}

// ---------------------------------------------------------------------------
// pass 1 tile: LDS histogram of the plane-kept points + N_valid / N_kept.
// ---------------------------------------------------------------------------
struct PipeShared {
    uint32_t hist[kBins];         // pass 1
    uint32_t okbits[kBins / 32];  // pass 2: hist[bin] > hist_thr
    uint64_t wave[4];             // pass 2 block scan
    uint32_t cnt[2];
    uint32_t tile, excl;
};
static_assert(sizeof(PipeShared) < 8192, "LDS budget");

template <int STEP>
__device__ __forceinline__ void hist_tile(const PipeBuffers& bf, int frame, int tile, const KParams& p,
                                          PipeShared& sh) {
    const int tid = threadIdx.x;
    for (int i = tid; i < kBins; i += 256) sh.hist[i] = 0;
    if (tid < 2) sh.cnt[tid] = 0;
    const uint8_t* disp = bf.disp + (int64_t)frame * p.frame_px;
    const uint8_t* bgr = bf.bgr + (int64_t)frame * p.frame_px * 3;
    QuadIn<STEP> in[kQPT];
    int gy[kQPT], q[kQPT];
    load_tile<STEP>(disp, bgr, tile * 256 * kQPT, tid, p, in, gy, q);
    __syncthreads();
    uint32_t nv = 0, nk = 0;
#pragma unroll
    for (int i = 0; i < kQPT; ++i) {
        if (gy[i] < 0) continue;
        const int y = gy[i] * STEP;
        const float yc = centred(y, p.ch_hi, p.ch_lo);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int gx = 4 * q[i] + k;
            nv += (in[i].d[k] != 0 && gx < p.Wg) ? 1u : 0u;
            const int e = eval_point<STEP>(in[i], k, gx, y, yc, p);
            if (e) {
                ++nk;
                atomicAdd(&sh.hist[e - 1], 1u);
            }
        }
    }
    nv = wave_sum(nv);
    nk = wave_sum(nk);
    if (lane_id() == 0) {
        atomicAdd(&sh.cnt[0], nv);
        atomicAdd(&sh.cnt[1], nk);
    }
    __syncthreads();
    if (tid == 0) {
        atomicAdd(reinterpret_cast<unsigned long long*>(bf.counts + 4 * frame + 0), (unsigned long long)sh.cnt[0]);
        atomicAdd(reinterpret_cast<unsigned long long*>(bf.counts + 4 * frame + 1), (unsigned long long)sh.cnt[1]);
    }
    uint32_t* gh = bf.hist + (int64_t)frame * kBins;
    for (int i = tid; i < kBins; i += 256) {
        const uint32_t v = sh.hist[i];
        if (v) atomicAdd(gh + i, v);
    }
}

// ---------------------------------------------------------------------------
// pass 2 tile: keep2 filter, ordered compaction, fp32 XYZ + int32 (x, y).
// Tile = 256 lanes x kQPT quads; quad (i, lane) = tile_base + i*256 + lane, so
// each load wave-instruction is contiguous; the raster order inside the tile
// is (i, lane), scanned with 4 x 16-bit fields packed in one u64.
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
__device__ __forceinline__ void compact_tile(const PipeBuffers& bf, int frame, int tile, int tiles,
                                             const KParams& p, PipeShared& sh) {
    const int tid = threadIdx.x;
    const uint8_t* disp = bf.disp + (int64_t)frame * p.frame_px;
    const uint8_t* bgr = bf.bgr + (int64_t)frame * p.frame_px * 3;
    const int qbase = tile * 256 * kQPT;
    QuadIn<STEP> in[kQPT];
    int gyv[kQPT], qv[kQPT];
    load_tile<STEP>(disp, bgr, qbase, tid, p, in, gyv, qv);
    {   // hist[bin] > hist_thr as a 1024-bit mask
        const uint32_t* gh = bf.hist + (int64_t)frame * kBins;
        const int wave = tid >> 6;
#pragma unroll
        for (int r = 0; r < kBins / 256; ++r) {
            const uint64_t m = __ballot((int64_t)gh[r * 256 + tid] > (int64_t)p.hist_thr);
            if (lane_id() == 0) {
                sh.okbits[(r * 256 + wave * 64) / 32] = (uint32_t)m;
                sh.okbits[(r * 256 + wave * 64) / 32 + 1] = (uint32_t)(m >> 32);
            }
        }
    }
    __syncthreads();
    uint32_t dpack[kQPT];
    uint32_t keep = 0;  // bit 4*i + k
    uint64_t cnt = 0;
#pragma unroll
    for (int i = 0; i < kQPT; ++i) {
        dpack[i] = in[i].d[0] | (in[i].d[1] << 8) | (in[i].d[2] << 16) | (in[i].d[3] << 24);
        if (gyv[i] < 0) continue;
        const int y = gyv[i] * STEP;
        const float yc = centred(y, p.ch_hi, p.ch_lo);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int e = eval_point<STEP>(in[i], k, 4 * qv[i] + k, y, yc, p);
            if (e && ((sh.okbits[(e - 1) >> 5] >> ((e - 1) & 31)) & 1)) {
                keep |= 1u << (4 * i + k);
                cnt += 1ull << (16 * i);
            }
        }
    }
    // block scan of the packed per-quad-row counts
    const uint64_t inc = wave_incl_scan64(cnt);
    const int wave = tid >> 6;
    if (lane_id() == 63) sh.wave[wave] = inc;
    __syncthreads();
    uint64_t wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint64_t t = sh.wave[w];
        wbase += (w < wave) ? t : 0ull;
        tot += t;
    }
    const uint64_t excl_packed = wbase + inc - cnt;
    uint32_t total = 0;
#pragma unroll
    for (int i = 0; i < kQPT; ++i) total += (uint32_t)((tot >> (16 * i)) & 0xFFFF);

    if (wave == 0) {
        uint64_t* st = bf.status + (int64_t)frame * tiles;
        uint32_t excl = 0;
        if (tile == 0) {
            if (tid == 0) publish(st, kFlagInc, total);
        } else {
            if (tid == 0) publish(st + tile, kFlagAgg, total);
            excl = lookback(st, tile, bf.err);
            if (tid == 0) publish(st + tile, kFlagInc, excl + total);
        }
        if (tid == 0) {
            sh.excl = excl;
            if (tile == tiles - 1) bf.counts[4 * frame + 2] = excl + total;
        }
    }
    __syncthreads();
    if (!keep) return;

    const int64_t fbase = (int64_t)frame * bf.cap + sh.excl;
    float* oxyz = bf.xyz;
    int32_t* opts = bf.pts;
    uint32_t rowbase = 0;
#pragma unroll
    for (int i = 0; i < kQPT; ++i) {
        uint32_t o = rowbase + (uint32_t)((excl_packed >> (16 * i)) & 0xFFFF);
        rowbase += (uint32_t)((tot >> (16 * i)) & 0xFFFF);
        const uint32_t km = (keep >> (4 * i)) & 0xF;
        if (!km) continue;
        const int q = qv[i];
        const int y = gyv[i] * STEP;
        const float yc = centred(y, p.ch_hi, p.ch_lo);
        const int dyw = y >> 5, dyb = y & 31;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (!(km & (1u << k))) continue;
            const uint32_t d = (dpack[i] >> (8 * k)) & 0xFF;
            const int x = (4 * q + k) * STEP;
            const float xc = centred(x, p.cw_hi, p.cw_lo);
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

// ---------------------------------------------------------------------------
// One launch = pass 2 of chunk c-1 (blocks [0, n2*tiles)) + pass 1 of chunk c
// (the rest). A pass-2 block is bound to a frame by blockIdx and takes its
// tile id from that frame's ticket (one counter per frame, each on its own
// 64-byte line: ~136 atomics per word instead of ~9K on one global word, which
// saturates at ~88/us). A tile waits only on lower tiles of its own frame,
// whose blocks took their tickets earlier and are therefore running: forward
// progress does not depend on dispatch order. Pass-1 blocks wait on nothing.
// ---------------------------------------------------------------------------
constexpr int kTicketStride = 16;  // u32 words per frame ticket (64 B)

template <int STEP>
__global__ __launch_bounds__(256) void pipeline_kernel(PipeBuffers bf, int p2_frame0, int p2_frames,
                                                       int p1_frame0, int tiles, uint32_t* tickets,
                                                       KParams p) {
    __shared__ PipeShared sh;
    const int n2 = p2_frames * tiles;
    const int bid = blockIdx.x;
    if (bid < n2) {
        const int frame = p2_frame0 + bid / tiles;
        if (threadIdx.x == 0) sh.tile = atomicAdd(tickets + (int64_t)frame * kTicketStride, 1u);
        __syncthreads();
        compact_tile<STEP>(bf, frame, (int)sh.tile, tiles, p, sh);
    } else {
        const int h = bid - n2;
        const int fl = h / tiles;
        hist_tile<STEP>(bf, p1_frame0 + fl, h - fl * tiles, p, sh);
    }
}

size_t pipeline_ticket_words(int frames) { return (size_t)frames * kTicketStride; }

hipError_t launch_pipeline(const KParams& p, const PipeBuffers& b, int frames, int chunk,
                           uint32_t* tickets, hipStream_t s) {
    const int tiles = pipeline_tiles_per_frame(p);
    const int nchunks = (frames + chunk - 1) / chunk;
    for (int c = 0; c <= nchunks; ++c) {
        const int f2 = (c - 1) * chunk, n2 = c >= 1 ? min(chunk, frames - f2) : 0;
        const int f1 = c * chunk, n1 = c < nchunks ? min(chunk, frames - f1) : 0;
        const dim3 grid((n2 + n1) * tiles), blk(256);
        if (p.step == 1)
            hipLaunchKernelGGL(pipeline_kernel<1>, grid, blk, 0, s, b, f2, n2, f1, tiles, tickets, p);
        else if (p.step == 2)
            hipLaunchKernelGGL(pipeline_kernel<2>, grid, blk, 0, s, b, f2, n2, f1, tiles, tickets, p);
        else
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace svx
