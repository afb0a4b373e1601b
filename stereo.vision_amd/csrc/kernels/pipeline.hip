// Plane-threshold + hue-histogram + compaction pipeline (gfx950), config 4.
//
// Per frame (stereovision.py:97-113): keep1 = dist(P, plane) < point_thr
// (functions.py:300-323); hist = hue-bin counts over keep1 (functions.py:215-226);
// keep2 = keep1 & hist[bin] > hist_thr (functions.py:228-230); output the keep2
// points in reference (raster) order as fp32 XYZ + int32 (x,y) back-projection
// (functions.py:201-209 + stereovision.py:112).
//
// The histogram must be complete before any point of a frame can be filtered,
// so every frame is visited twice, tile by tile (tile = 256 lanes x 4 quads =
// 4096 grid points):
//   pass 1  hist_tile     reads disparity + BGR (4 B/pt), evaluates keep1 and
//                         the hue bin of every point; LDS histogram flushed
//                         with one global atomic per non-zero bin; writes the
//                         tile's keep1 bitmask (2 B per lane = 1 bit/pt) and
//                         its bin-presence mask (1024 bits).
//   pass 2  compact_tile  reads the keep1 bits + disparity (~1.1 B/pt); a tile
//                         whose present bins are all above hist_thr ("clean",
//                         nearly all of them) needs no hue at all; a "dirty"
//                         tile re-reads its BGR and recomputes the bins of its
//                         keep1 points. Wave scan + LDS block scan inside the
//                         tile, decoupled look-back across the frame's tiles,
//                         then fp32 XYZ + int32 (x,y) stores.
// Frames go in chunks; launch c runs pass 2 of chunk c-1 together with pass 1
// of chunk c, so a chunk's second visit comes from the 256 MB Infinity Cache
// shortly after its first; there are chunks+1 launches per call. All control
// words (histograms, counts, look-back granules, tickets) are zeroed by one
// memset per call; the keep/presence masks are fully rewritten by pass 1.
#include "../svx_launch.h"

namespace svx {

constexpr int kQPT = 4;   // quads per lane: tile = 256 x 4 quads = 4096 grid points

template <int STEP>
struct QuadIn {
    uint32_t d[4];
    uint32_t c[3 * STEP];  // BGR bytes of the quad's source pixels
};

template <int STEP>
__device__ __forceinline__ void load_disp(const uint8_t* drow, int q, uint32_t (&d)[4]) {
    if constexpr (STEP == 1) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(drow + 4 * q);
        d[0] = w & 0xFF; d[1] = (w >> 8) & 0xFF; d[2] = (w >> 16) & 0xFF; d[3] = w >> 24;
    } else {
        const uint2 w = *reinterpret_cast<const uint2*>(drow + 8 * q);
        d[0] = w.x & 0xFF; d[1] = (w.x >> 16) & 0xFF; d[2] = w.y & 0xFF; d[3] = (w.y >> 16) & 0xFF;
    }
}

template <int STEP>
__device__ __forceinline__ void load_bgr(const uint8_t* crow, int q, QuadIn<STEP>& o) {
    if constexpr (STEP == 1) {
        const uint32_t* cp = reinterpret_cast<const uint32_t*>(crow + 12 * q);
        o.c[0] = cp[0]; o.c[1] = cp[1]; o.c[2] = cp[2];
    } else {
        const uint2* cp = reinterpret_cast<const uint2*>(crow + 24 * q);
        const uint2 a = cp[0], b = cp[1], c = cp[2];
        o.c[0] = a.x; o.c[1] = a.y; o.c[2] = b.x; o.c[3] = b.y; o.c[4] = c.x; o.c[5] = c.y;
    }
}

template <int STEP>
__device__ __forceinline__ int point_bin(const QuadIn<STEP>& in, int k) {
    const int o = 3 * STEP * k;  // byte offset of pixel k inside the quad's BGR
    const auto byte = [&](int i) { return (int)((in.c[i >> 2] >> (8 * (i & 3))) & 0xFF); };
    return hue_bin(byte(o + 2), byte(o + 1), byte(o));   // (R, G, B) from BGR
}

// keep1 for one grid point (functions.py:300-323).
template <int STEP>
__device__ __forceinline__ bool point_keep1(uint32_t d, int gx, int y, float yc, const KParams& p) {
    if (d == 0 || gx >= p.Wg) return false;
    const int x = gx * STEP;
    const float xc = centred(x, p.cw_hi, p.cw_lo);
    const float r = __builtin_amdgcn_rcpf((float)d);
    const float K = p.B32 * r;
    return keep1(x, y, d, xc, yc, K, xc * K, yc * K, p.fB32 * r, p);
}

int pipeline_tiles_per_frame(const KParams& p) {
    const int per = 256 * kQPT;
    return (p.frame_quads + per - 1) / per;
}

// Lane geometry of a tile: quad i of this lane = qbase + i*256 + lane (so each
// wave-instruction touches contiguous memory). Out-of-range quads re-address
// the last valid quad (branch-free loads) and are flagged gy = -1.
__device__ __forceinline__ void tile_geometry(int qbase, int tid, const KParams& p, int (&gy)[kQPT],
                                              int (&q)[kQPT]) {
#pragma unroll
    for (int i = 0; i < kQPT; ++i) {
        const int qi = qbase + i * 256 + tid;
        const bool ok = qi < p.frame_quads;
        const int qc = ok ? qi : p.frame_quads - 1;
        const int g = qc / p.Q;
        q[i] = qc - g * p.Q;
        gy[i] = ok ? g : -1;
    }
}

template <int STEP>
__device__ __forceinline__ const uint8_t* row_ptr(const uint8_t* base, int gy, int bpp, const KParams& p) {
    const int g = gy < 0 ? 0 : gy;
    return base + (int64_t)(g * STEP) * p.W * bpp;
}

struct PipeShared {
    uint32_t hist[kBins];         // pass 1
    uint32_t okbits[kBins / 32];  // pass 2: hist[bin] > hist_thr
    uint64_t wave[4];             // pass 2 block scan
    uint32_t cnt[2];
    uint32_t tile, excl, dirty;
};
static_assert(sizeof(PipeShared) < 8192, "LDS budget");

// ---------------------------------------------------------------------------
// pass 1 tile
// ---------------------------------------------------------------------------
template <int STEP>
__device__ __forceinline__ void hist_tile(const PipeBuffers& bf, int frame, int tile, int tiles,
                                          const KParams& p, PipeShared& sh) {
    const int tid = threadIdx.x;
    const uint8_t* disp = bf.disp + (int64_t)frame * p.frame_px;
    const uint8_t* bgr = bf.bgr + (int64_t)frame * p.frame_px * 3;
    int gy[kQPT], q[kQPT];
    tile_geometry(tile * 256 * kQPT, tid, p, gy, q);
    QuadIn<STEP> in[kQPT];
#pragma unroll
    for (int i = 0; i < kQPT; ++i) {   // all loads in flight before any use
        load_disp<STEP>(row_ptr<STEP>(disp, gy[i], 1, p), q[i], in[i].d);
        load_bgr<STEP>(row_ptr<STEP>(bgr, gy[i], 3, p), q[i], in[i]);
    }
    for (int i = tid; i < kBins; i += 256) sh.hist[i] = 0;
    if (tid < 2) sh.cnt[tid] = 0;
    __syncthreads();
    uint32_t nv = 0, keep = 0;
#pragma unroll
    for (int i = 0; i < kQPT; ++i) {
        if (gy[i] < 0) continue;
        const int y = gy[i] * STEP;
        const float yc = centred(y, p.ch_hi, p.ch_lo);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int gx = 4 * q[i] + k;
            nv += (in[i].d[k] != 0 && gx < p.Wg) ? 1u : 0u;
            if (point_keep1<STEP>(in[i].d[k], gx, y, yc, p)) {
                keep |= 1u << (4 * i + k);
                atomicAdd(&sh.hist[point_bin<STEP>(in[i], k)], 1u);
            }
        }
    }
    uint32_t nk = __builtin_popcount(keep);
    const int64_t slot = (int64_t)frame * tiles + tile;
    bf.kbits[slot * 256 + tid] = (uint16_t)keep;
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
    uint32_t* pres = bf.pres + slot * (kBins / 32);
    const int wave = tid >> 6;
#pragma unroll
    for (int r = 0; r < kBins / 256; ++r) {
        const int b = r * 256 + tid;
        const uint32_t v = sh.hist[b];
        if (v) atomicAdd(gh + b, v);
        const uint64_t m = __ballot(v != 0);
        if (lane_id() == 0) {
            pres[(r * 256 + wave * 64) / 32] = (uint32_t)m;
            pres[(r * 256 + wave * 64) / 32 + 1] = (uint32_t)(m >> 32);
        }
    }
}

// ---------------------------------------------------------------------------
// pass 2 tile
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
    int gyv[kQPT], qv[kQPT];
    tile_geometry(tile * 256 * kQPT, tid, p, gyv, qv);
    const int64_t slot = (int64_t)frame * tiles + tile;
    uint32_t keep = bf.kbits[slot * 256 + tid];
    uint32_t dv[kQPT][4];
#pragma unroll
    for (int i = 0; i < kQPT; ++i) load_disp<STEP>(row_ptr<STEP>(disp, gyv[i], 1, p), qv[i], dv[i]);
    {   // hist[bin] > hist_thr as a 1024-bit mask; the tile is dirty if a present bin fails it
        const uint32_t* gh = bf.hist + (int64_t)frame * kBins;
        const int wave = tid >> 6;
        if (tid == 0) sh.dirty = 0;
#pragma unroll
        for (int r = 0; r < kBins / 256; ++r) {
            const uint64_t m = __ballot((int64_t)gh[r * 256 + tid] > (int64_t)p.hist_thr);
            if (lane_id() == 0) {
                sh.okbits[(r * 256 + wave * 64) / 32] = (uint32_t)m;
                sh.okbits[(r * 256 + wave * 64) / 32 + 1] = (uint32_t)(m >> 32);
            }
        }
        __syncthreads();
        if (tid < kBins / 32) {
            const uint32_t bad = bf.pres[slot * (kBins / 32) + tid] & ~sh.okbits[tid];
            if (bad) atomicOr(&sh.dirty, 1u);
        }
        __syncthreads();
    }
    if (sh.dirty) {   // block-uniform and rare: recompute the bins of the keep1 points
        const uint8_t* bgr = bf.bgr + (int64_t)frame * p.frame_px * 3;
#pragma unroll
        for (int i = 0; i < kQPT; ++i) {
            if (!((keep >> (4 * i)) & 0xF)) continue;
            QuadIn<STEP> in;
            load_bgr<STEP>(row_ptr<STEP>(bgr, gyv[i], 3, p), qv[i], in);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (!(keep & (1u << (4 * i + k)))) continue;
                const int bin = point_bin<STEP>(in, k);
                if (!((sh.okbits[bin >> 5] >> (bin & 31)) & 1)) keep &= ~(1u << (4 * i + k));
            }
        }
    }
    uint64_t cnt = 0;
#pragma unroll
    for (int i = 0; i < kQPT; ++i) cnt += (uint64_t)__builtin_popcount((keep >> (4 * i)) & 0xF) << (16 * i);

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
            const uint32_t d = dv[i][k];
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
        hist_tile<STEP>(bf, p1_frame0 + fl, h - fl * tiles, tiles, p, sh);
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
