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
//   offsets               one small workgroup per frame: a tile whose present
//                         bins all pass hist_thr ("clean", nearly all) keeps
//                         its keep1 bits as keep2; a "dirty" tile re-reads its
//                         BGR and rewrites its bits to keep2; the per-tile
//                         counts are scanned into output offsets.
//   pass 2  compact       one workgroup per tile: keep2 bits + disparity
//                         (~1.1 B/pt) + offset in; block scan, LDS descriptor
//                         scatter, then contiguous non-temporal SoA stores.
// Frames go in chunks: launch c = pass 2 of chunk c-2 + pass 1 of chunk c in
// one grid with interleaved roles (pass 1 is VALU-heavy, pass 2 store-bound,
// so they share every CU); offsets(c-1) runs beside it on a second stream. The control words
// (histograms, counts) are zeroed by one memset per call; the keep /
// presence masks are fully rewritten by pass 1.
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
        const int g = fastdiv40(qc, p.Q_m40);
        q[i] = qc - g * p.Q;
        gy[i] = ok ? g : -1;
    }
}

template <int STEP>
__device__ __forceinline__ const uint8_t* row_ptr(const uint8_t* base, int gy, int bpp, const KParams& p) {
    const int g = gy < 0 ? 0 : gy;
    return base + (int64_t)(g * STEP) * p.W * bpp;
}

// Can any grid point of the tile be kept by the plane (keep1)? P.abc = u / d with
// u = B (a (x - cw) + b (y - ch) + c f), so keep1 <=> |u / d - 1| < t, t = thr |abc|
// (functions.py:300-323). u is affine in (x, y): over the tile's rows and the whole
// width its extremes are at the corners (urange_keepable, svx_device.h).
// Uniform per tile; false -> skip its colours.
__device__ __forceinline__ bool tile_keepable(int tile, const KParams& p) {
    const int q0 = tile * 256 * kQPT, q1 = min(q0 + 256 * kQPT, p.frame_quads) - 1;
    const double y0 = (double)(fastdiv40(q0, p.Q_m40) * p.step), y1 = (double)(fastdiv40(q1, p.Q_m40) * p.step);
    const double ax0 = p.a * (0.0 - p.cw), ax1 = p.a * ((double)((p.Wg - 1) * p.step) - p.cw);
    const double by0 = p.b * (y0 - p.ch), by1 = p.b * (y1 - p.ch);
    const double cf = p.c * p.f;
    const double umax = p.B * (fmax(ax0, ax1) + fmax(by0, by1) + cf);
    const double umin = p.B * (fmin(ax0, ax1) + fmin(by0, by1) + cf);
    const double mag = p.B * (fmax(fabs(ax0), fabs(ax1)) + fmax(fabs(by0), fabs(by1)) + fabs(cf));
    return urange_keepable(umin, umax, p.thr * p.nrm, mag);
}

struct PipeShared {   // pass 1
    uint32_t hist[kBins];
    uint32_t cnt[2];
};
static_assert(sizeof(PipeShared) < 8192, "LDS budget");

// ---------------------------------------------------------------------------
// pass 1 tile
// ---------------------------------------------------------------------------
template <int STEP, bool PF>
__device__ __forceinline__ void hist_tile(const PipeBuffers& bf, int frame, int tile, int tiles,
                                          const KParams& p0, PipeShared& sh) {
    const int tid = threadIdx.x;
    KParams p = p0;
    bool live = true;
    if constexpr (PF) {   // this frame's plane (uniform: scalar loads)
        const FramePlane fpl = bf.planes[(int64_t)frame * bf.plane_stride];
        apply_plane(p, fpl);
        live = fpl.valid != 0;
    }
    const uint8_t* disp = bf.disp + (int64_t)frame * p.frame_px;
    const uint8_t* bgr = bf.bgr + (int64_t)frame * p.frame_px * 3;
    int gy[kQPT], q[kQPT];
    tile_geometry(tile * 256 * kQPT, tid, p, gy, q);
    live = live && tile_keepable(tile, p);   // uniform: a tile the plane rules out needs only its valid count
    QuadIn<STEP> in[kQPT];
#pragma unroll
    for (int i = 0; i < kQPT; ++i) {   // all loads in flight before any use
        load_disp<STEP>(row_ptr<STEP>(disp, gy[i], 1, p), q[i], in[i].d);
        if (live) load_bgr<STEP>(row_ptr<STEP>(bgr, gy[i], 3, p), q[i], in[i]);
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
            if (live && point_keep1<STEP>(in[i].d[k], gx, y, yc, p)) {
                keep |= 1u << (4 * i + k);
                const int bin = (p.ablate & 1) ? 0 : point_bin<STEP>(in[i], k);
                if (!(p.ablate & 2)) atomicAdd(&sh.hist[bin], 1u);
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
        bf.tcount[slot] = sh.cnt[1];
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
// offsets: one workgroup per frame (tiny). Decides which tiles are dirty (a
// keep1 point whose bin fails hist_thr, from the presence masks), rewrites
// those tiles' bits from keep1 to keep2 (re-reading their BGR), and scans the
// per-tile keep2 counts into per-tile output offsets + N_kept2. After it, pass
// 2 is embarrassingly parallel: no tickets, no look-back, no BGR.
// ---------------------------------------------------------------------------
constexpr int kMaxTiles = 2048;   // tiles per frame supported by one offsets workgroup

struct OffsetsShared {
    uint32_t okbits[kBins / 32];
    uint32_t dirty[kMaxTiles / 32];
    uint32_t cnt[kMaxTiles];
    uint32_t wsum[4];
};

template <int STEP>
__global__ __launch_bounds__(256) void offsets_kernel(PipeBuffers bf, int frame0, int tiles, KParams p) {
    __shared__ OffsetsShared sh;
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = frame0 + blockIdx.x;
    const int64_t slot0 = (int64_t)frame * tiles;
    const uint32_t* gh = bf.hist + (int64_t)frame * kBins;
#pragma unroll
    for (int r = 0; r < kBins / 256; ++r) {   // hist[bin] > hist_thr as a 1024-bit mask
        const uint64_t m = __ballot((int64_t)gh[r * 256 + tid] > (int64_t)p.hist_thr);
        if (lane == 0) {
            sh.okbits[(r * 256 + wave * 64) / 32] = (uint32_t)m;
            sh.okbits[(r * 256 + wave * 64) / 32 + 1] = (uint32_t)(m >> 32);
        }
    }
    for (int w = tid; w < kMaxTiles / 32; w += 256) sh.dirty[w] = 0;
    for (int t = tid; t < tiles; t += 256) sh.cnt[t] = bf.tcount[slot0 + t];
    __syncthreads();
    for (int i = tid; i < tiles * (kBins / 32); i += 256) {
        const int t = i / (kBins / 32), w = i - t * (kBins / 32);
        if (bf.pres[(slot0 + t) * (kBins / 32) + w] & ~sh.okbits[w]) atomicOr(&sh.dirty[t >> 5], 1u << (t & 31));
    }
    __syncthreads();
    const uint8_t* bgr = bf.bgr + (int64_t)frame * p.frame_px * 3;
    for (int t = 0; t < tiles; ++t) {   // uniform loop; work only on (rare) dirty tiles
        if (!((sh.dirty[t >> 5] >> (t & 31)) & 1)) continue;
        uint16_t* kbp = bf.kbits + (slot0 + t) * 256 + tid;
        uint32_t keep = *kbp;
        int gy[kQPT], q[kQPT];
        tile_geometry(t * 256 * kQPT, tid, p, gy, q);
#pragma unroll
        for (int i = 0; i < kQPT; ++i) {
            if (!((keep >> (4 * i)) & 0xF)) continue;
            QuadIn<STEP> in;
            load_bgr<STEP>(row_ptr<STEP>(bgr, gy[i], 3, p), q[i], in);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (!(keep & (1u << (4 * i + k)))) continue;
                const int bin = point_bin<STEP>(in, k);
                if (!((sh.okbits[bin >> 5] >> (bin & 31)) & 1)) keep &= ~(1u << (4 * i + k));
            }
        }
        *kbp = (uint16_t)keep;
        const uint32_t c = wave_sum(__builtin_popcount(keep));
        if (lane == 0) sh.wsum[wave] = c;
        __syncthreads();
        if (tid == 0) sh.cnt[t] = sh.wsum[0] + sh.wsum[1] + sh.wsum[2] + sh.wsum[3];
        __syncthreads();
    }
    // exclusive scan of the tile counts (<= 8 per lane, lane-major)
    constexpr int PER = kMaxTiles / 256;
    uint32_t v[PER], run = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int t = tid * PER + j;
        v[j] = t < tiles ? sh.cnt[t] : 0u;
        run += v[j];
    }
    const uint32_t inc = wave_incl_scan(run);
    if (lane == 63) sh.wsum[wave] = inc;
    __syncthreads();
    uint32_t base = inc - run;
    for (int w = 0; w < wave; ++w) base += sh.wsum[w];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int t = tid * PER + j;
        if (t < tiles) bf.toff[slot0 + t] = base;
        base += v[j];
    }
    if (tid == 255) bf.counts[4 * frame + 2] = base;
}

// ---------------------------------------------------------------------------
// pass 2: one workgroup per tile. keep2 bits + disparity + the tile's output
// offset in; a block scan gives each keep2 point its slot; lanes scatter a
// 4-byte descriptor (d | gy | gx) into LDS at that slot, then lane j of the
// block produces output j — every store instruction writes contiguous lanes of
// the SoA outputs (X, Y, Z, (x,y)) with non-temporal stores, no partial lines.
// The delta-table words of 8 outputs per lane are loaded before any is used.
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

struct CompactShared {
    uint64_t wave[4];
    uint32_t desc[256 * kQPT * 4 + 4];   // one descriptor per keep2 point (+ alignment slack)
};

typedef float v4f __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));

template <int STEP>
__device__ __forceinline__ void compact_tile(const PipeBuffers& bf, int frame, int t, int tiles,
                                             const KParams& p, CompactShared& sh) {
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int64_t slot = (int64_t)frame * tiles + t;
    if (bf.tcount[slot] == 0) return;   // uniform: no keep1 point, so no output (no barrier skipped by part of the block)
    const uint8_t* disp = bf.disp + (int64_t)frame * p.frame_px;
    const uint32_t keep = bf.kbits[slot * 256 + tid];
    const uint32_t toff = bf.toff[slot];
    int gy[kQPT], q[kQPT];
    tile_geometry(t * 256 * kQPT, tid, p, gy, q);
    uint32_t dw[kQPT][STEP];
#pragma unroll
    for (int i = 0; i < kQPT; ++i) {
        const uint8_t* row = row_ptr<STEP>(disp, gy[i], 1, p);
        if constexpr (STEP == 1) {
            dw[i][0] = *reinterpret_cast<const uint32_t*>(row + 4 * q[i]);
        } else {
            const uint2 w = *reinterpret_cast<const uint2*>(row + 8 * q[i]);
            dw[i][0] = w.x;
            dw[i][1] = w.y;
        }
    }
    uint64_t cnt = 0;
#pragma unroll
    for (int i = 0; i < kQPT; ++i) cnt += (uint64_t)__builtin_popcount((keep >> (4 * i)) & 0xF) << (16 * i);
    const uint64_t inc = wave_incl_scan64(cnt);
    if (lane == 63) sh.wave[wave] = inc;
    __syncthreads();
    uint64_t wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint64_t v = sh.wave[w];
        wbase += (w < wave) ? v : 0ull;
        tot += v;
    }
    const uint64_t excl = wbase + inc - cnt;
    // descriptors land at LDS slot (toff & 3) + o, so that LDS slot s <-> global
    // element g0 + s with g0 = toff & ~3: output groups of 4 are 16-byte aligned
    const uint32_t lead = toff & 3;
    uint32_t rowbase = lead;
#pragma unroll
    for (int i = 0; i < kQPT; ++i) {
        uint32_t o = rowbase + (uint32_t)((excl >> (16 * i)) & 0xFFFF);
        rowbase += (uint32_t)((tot >> (16 * i)) & 0xFFFF);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (!(keep & (1u << (4 * i + k)))) continue;
            uint32_t d;
            if constexpr (STEP == 1) d = (dw[i][0] >> (8 * k)) & 0xFF;
            else d = (dw[i][k >> 1] >> (16 * (k & 1))) & 0xFF;
            sh.desc[o++] = (d << 24) | ((uint32_t)gy[i] << 12) | (uint32_t)(4 * q[i] + k);
        }
    }
    const uint32_t end = rowbase;            // one past the last valid LDS slot
    __syncthreads();
    const uint32_t g0 = toff - lead;
    float* oX = bf.ox + (int64_t)frame * bf.ofs + g0;
    float* oY = bf.oy + (int64_t)frame * bf.ofs + g0;
    float* oZ = bf.oz + (int64_t)frame * bf.ofs + g0;
    uint32_t* oPxy = bf.pxy + (int64_t)frame * bf.cap + g0;
    // Groups of 4 outputs at 16-byte-aligned slots: lane l of a wave stores the
    // X, Y, Z, (x, y) of group m0 + l, so every store instruction covers 1 KiB
    // contiguous of its plane.
    const uint32_t groups = (end + 3) >> 2;
    for (uint32_t m0 = tid & ~63u; m0 < groups; m0 += 256) {   // uniform per wave
        const uint32_t m = m0 + lane;
        if (m >= groups) continue;
        const uint4 u4 = *reinterpret_cast<const uint4*>(&sh.desc[4 * m]);
        uint32_t u[4] = {u4.x, u4.y, u4.z, u4.w}, wx[4], wy[4];
        bool ok[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {   // all table loads in flight together
            const uint32_t s_ = 4 * m + e;
            ok[e] = s_ >= lead && s_ < end;
            u[e] = ok[e] ? u[e] : (1u << 24);
            const uint32_t d = u[e] >> 24;
            const int y = (int)((u[e] >> 12) & 0xFFF) * STEP;
            const int x = (int)(u[e] & 0xFFF) * STEP;
            wx[e] = bf.dxbits[d * p.dx_words + (x >> 5)];
            wy[e] = bf.dybits[d * p.dy_words + (y >> 5)];
        }
        float X[4], Y[4], Z[4];
        int PX[4], PY[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint32_t d = u[e] >> 24;
            const int y = (int)((u[e] >> 12) & 0xFFF) * STEP;
            const int x = (int)(u[e] & 0xFFF) * STEP;
            const float r = __builtin_amdgcn_rcpf((float)d);
            const float K = p.B32 * r;
            X[e] = centred(x, p.cw_hi, p.cw_lo) * K;
            Y[e] = centred(y, p.ch_hi, p.ch_lo) * K;
            Z[e] = p.fB32 * r;
            PX[e] = x - (int)((wx[e] >> (x & 31)) & 1);
            PY[e] = y - (int)((wy[e] >> (y & 31)) & 1);
        }
        if (ok[0] && ok[3]) {   // full group: 16-byte non-temporal stores
            __builtin_nontemporal_store((v4f){X[0], X[1], X[2], X[3]}, reinterpret_cast<v4f*>(oX + 4 * m));
            __builtin_nontemporal_store((v4f){Y[0], Y[1], Y[2], Y[3]}, reinterpret_cast<v4f*>(oY + 4 * m));
            __builtin_nontemporal_store((v4f){Z[0], Z[1], Z[2], Z[3]}, reinterpret_cast<v4f*>(oZ + 4 * m));
            __builtin_nontemporal_store((v4i){(int)pp_pack(PX[0], PY[0]), (int)pp_pack(PX[1], PY[1]),
                                         (int)pp_pack(PX[2], PY[2]), (int)pp_pack(PX[3], PY[3])},
                                        reinterpret_cast<v4i*>(oPxy + 4 * m));
        } else {                // the tile's first / last group
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (!ok[e]) continue;
                oX[4 * m + e] = X[e];
                oY[4 * m + e] = Y[e];
                oZ[4 * m + e] = Z[e];
                oPxy[4 * m + e] = pp_pack(PX[e], PY[e]);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// One launch = pass 2 of one chunk + pass 1 of a later chunk. The two have no
// dependency on each other, and the workgroup roles are interleaved (even
// blockIdx: pass 2, odd: pass 1, while both last) so every CU runs VALU-heavy
// pass-1 waves beside store-bound pass-2 waves.
// ---------------------------------------------------------------------------
union StageShared {
    PipeShared p1;
    CompactShared p2;
};

template <int STEP, bool PF>
__global__ __launch_bounds__(256) void stage_kernel(PipeBuffers bf, int p2_frame0, int n2, int p1_frame0,
                                                    int n1, int tiles, KParams p) {
    __shared__ StageShared sh;
    const int b = blockIdx.x;
    const int both = 2 * min(n1, n2);
    int role, idx;   // role 2 = pass 2, 1 = pass 1
    if (p.ablate & 64) {   // diagnostic: no interleave (all pass-2 blocks first)
        role = b < n2 ? 2 : 1;
        idx = b < n2 ? b : b - n2;
    } else if (b < both) {
        role = (b & 1) ? 1 : 2;
        idx = b >> 1;
    } else {
        role = n2 > n1 ? 2 : 1;
        idx = (b - both) + both / 2;
    }
    const int fl = idx / tiles, t = idx - fl * tiles;
    if (role == 2) {
        if (!(p.ablate & 256)) compact_tile<STEP>(bf, p2_frame0 + fl, t, tiles, p, sh.p2);
    } else {
        if (!(p.ablate & 128)) hist_tile<STEP, PF>(bf, p1_frame0 + fl, t, tiles, p, sh.p1);
    }
}

// Schedule (lag 2, two streams): stream A runs stage(c) = pass 2 of chunk
// c-2 + pass 1 of chunk c; stream B runs offsets(c) as soon as stage(c) is
// done, concurrently with stage(c+1); stage(c+2) waits for offsets(c). So the
// small, latency-bound offsets kernel never sits on the critical path.
// ev must hold 2 * chunks events: ev[2c] = pass 1 of c done, ev[2c+1] = offsets(c) done.
hipError_t launch_pipeline(const KParams& p, const PipeBuffers& b, int frames, int chunk, hipStream_t sa,
                           hipStream_t sb, hipEvent_t* ev) {
    const int tiles = pipeline_tiles_per_frame(p);
    if (frames <= 0) return hipSuccess;
    if (tiles > kMaxTiles || p.Wg > 4096 || p.Hg > 4096 || (p.step != 1 && p.step != 2))
        return hipErrorInvalidValue;
    const int nchunks = (frames + chunk - 1) / chunk;
    const dim3 blk(256);
    hipError_t e = hipSuccess;
    for (int c = 0; c < nchunks + 2 && e == hipSuccess; ++c) {
        const int c2 = c - 2;
        const bool has2 = c2 >= 0 && c2 < nchunks, has1 = c < nchunks;
        const int f2 = c2 * chunk, n2 = has2 ? min(chunk, frames - f2) : 0;
        const int f1 = c * chunk, n1 = has1 ? min(chunk, frames - f1) : 0;
        if (!has1 && !has2) continue;   // the gap launch when there is a single chunk
        if (has2) e = hipStreamWaitEvent(sa, ev[2 * c2 + 1], 0);
        if (e != hipSuccess) break;
        const dim3 grid((n2 + n1) * tiles);
        const auto kern = b.planes ? (p.step == 1 ? stage_kernel<1, true> : stage_kernel<2, true>)
                                   : (p.step == 1 ? stage_kernel<1, false> : stage_kernel<2, false>);
        hipLaunchKernelGGL(kern, grid, blk, 0, sa, b, f2, n2 * tiles, f1, n1 * tiles, tiles, p);
        if (!has1) continue;
        e = hipEventRecord(ev[2 * c], sa);
        if (e == hipSuccess) e = hipStreamWaitEvent(sb, ev[2 * c], 0);
        if (e != hipSuccess) break;
        if (p.step == 1)
            hipLaunchKernelGGL(offsets_kernel<1>, dim3(n1), blk, 0, sb, b, f1, tiles, p);
        else
            hipLaunchKernelGGL(offsets_kernel<2>, dim3(n1), blk, 0, sb, b, f1, tiles, p);
        e = hipEventRecord(ev[2 * c + 1], sb);
    }
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

}  // namespace svx
