// Road raster + non-zero walk (gfx950), SURVEY §8f rank 2.
//
//  * raster_kernel   — generatePointsAsImage (functions.py:339-344): a black
//                      grey image with 255 at every [x, y] of the int32
//                      planePoints (stereovision.py:112-113, :136). Python's
//                      negative indices wrap (img[-1] is the last row); the
//                      host checks the range first, as numpy would raise.
//  * nonzero_kernel  — the pixel walk that ends sanitiseRoadImage
//                      (functions.py:359-365): [j, i] of every non-zero pixel
//                      in raster order. One workgroup per image; chunks of
//                      256 lanes x 16 pixels; a block scan orders the lanes,
//                      LDS holds the chunk's pixels in output order and a
//                      running offset orders the chunks, so the list is
//                      written once, in order, coalesced, with no
//                      cross-workgroup sync.
#include "../svx_launch.h"

namespace svx {

typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));

// point i of frame f: x = px[(f cap + i) * ps], y = py[(f cap + i) * ps] (ps = 2: interleaved (x, y) pairs); ps = 0:
// px holds the batch's pp_pack words (x and y as int16 halves); counts[frame * cstride + cidx] = points of the frame
__global__ __launch_bounds__(256) void raster_kernel(const int32_t* __restrict__ px, const int32_t* __restrict__ py,
                                                     int ps, const int64_t* __restrict__ counts, int cstride, int cidx,
                                                     int64_t cap, uint8_t* __restrict__ img, int H, int W, int Wu) {
    const int frame = blockIdx.y;
    const int64_t n = counts ? counts[(int64_t)frame * cstride + cidx] : cap;
    const int64_t f0 = (int64_t)frame * cap;
    uint8_t* fi = img + (int64_t)frame * H * W;
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        int qx, qy;
        if (ps == 0) {   // pp_pack words (a batch's planePoints)
            const uint32_t w = (uint32_t)px[f0 + i];
            qx = pp_x(w);
            qy = pp_y(w);
        } else {
            qx = px[(f0 + i) * ps];
            qy = py[(f0 + i) * ps];
        }
        const int x = qx < 0 ? qx + Wu : qx, y = qy < 0 ? qy + H : qy;
        fi[(int64_t)y * W + x] = 255;
    }
}

hipError_t launch_raster(const int32_t* px, const int32_t* py, int ps, const int64_t* counts, int cstride, int cidx,
                         int64_t cap, uint8_t* img, int frames, int H, int W, int Wu, hipStream_t s) {
    if (frames <= 0 || (int64_t)H * W <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(img, 0, (size_t)frames * H * W, s);
    if (e != hipSuccess) return e;
    if (cap <= 0) return hipSuccess;
    int64_t bx = (cap + 256 * 8 - 1) / (256 * 8);
    if (bx > 1024) bx = 1024;
    hipLaunchKernelGGL(raster_kernel, dim3((unsigned)bx, (unsigned)frames), dim3(256), 0, s, px, py, ps, counts,
                       cstride, cidx, cap, img, H, W, Wu);
    return hipGetLastError();
}

struct NonzeroShared {
    uint32_t wtot[4];
    uint32_t stage[256 * 16];   // the chunk's non-zero pixel indices, in output order
};

// img: frames x frame_px u8 (frame_px % 4 == 0); out: frames x cap x 2 int32 ([j, i]); counts[frame].
// Per chunk of 4096 pixels: each lane finds its 16 pixels' non-zero bits, a
// block scan orders them, lanes put the pixel indices into LDS in output order,
// then the whole chunk's [j, i] pairs are written contiguously (coalesced,
// non-temporal: written once, read by the caller later).
// A batch's walk entry (PK): x | y << 16 in one word (x < 4096, y < 65536), widened to the reference's [x, y]
// int32 pair when read back (sv_batch_read_road): the walk is written once and only the host reads it, so it
// moves 4 B per non-zero pixel instead of 8. The drop-in (sv_nonzero_points, any height) writes int32 pairs.
__device__ __forceinline__ uint32_t walk_pk(int x, int y) { return (uint32_t)x | ((uint32_t)y << 16); }

template <bool PK>
__global__ __launch_bounds__(256) void nonzero_kernel(const uint8_t* __restrict__ img, int64_t frame_px, int W,
                                                      uint64_t W_m40, int32_t* __restrict__ out, int64_t cap,
                                                      int64_t* __restrict__ counts) {
    __shared__ NonzeroShared sh;
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.x;
    const uint8_t* fb = img + (int64_t)frame * frame_px;
    const uint32_t* fi = reinterpret_cast<const uint32_t*>(fb);
    int2* fo = reinterpret_cast<int2*>(out) + (int64_t)frame * cap;
    const int64_t words = frame_px / 4, vecs = (words + 3) / 4;   // lane = 4 words = 16 pixels
    const bool vec16 = (reinterpret_cast<uintptr_t>(fb) & 15) == 0;   // uniform
    uint32_t running = 0;
    for (int64_t base = 0; base < vecs; base += 256) {
        const int64_t v = base + tid;
        uint32_t w[4];
        if (vec16 && 4 * v + 3 < words) {
            const uint4 q = *reinterpret_cast<const uint4*>(fi + 4 * v);
            w[0] = q.x; w[1] = q.y; w[2] = q.z; w[3] = q.w;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) w[k] = 4 * v + k < words ? fi[4 * v + k] : 0u;
        }
        uint32_t bits = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t nz = (((w[k] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w[k]) & 0x80808080u;   // bit 7 of each non-zero byte
            bits |= ((nz >> 7) & 1u) << (4 * k) | ((nz >> 15) & 1u) << (4 * k + 1) |
                    ((nz >> 23) & 1u) << (4 * k + 2) | ((nz >> 31) & 1u) << (4 * k + 3);
        }
        const uint32_t cnt = __builtin_popcount(bits);
        const uint32_t inc = wave_incl_scan(cnt);
        if (lane == 63) sh.wtot[wave] = inc;
        __syncthreads();   // also: the previous chunk's writes have read sh.stage
        uint32_t wbase = 0, tot = 0;
#pragma unroll
        for (int w4 = 0; w4 < 4; ++w4) {
            const uint32_t t = sh.wtot[w4];
            wbase += w4 < wave ? t : 0u;
            tot += t;
        }
        uint32_t o = wbase + inc - cnt;
        const uint32_t p0 = (uint32_t)(v * 16);
        while (bits) {
            const int b = __builtin_ctz(bits);
            bits &= bits - 1;
            sh.stage[o++] = p0 + (uint32_t)b;
        }
        __syncthreads();   // sh.wtot is rewritten next chunk; sh.stage is complete
        if (PK) {
            uint32_t* dst = reinterpret_cast<uint32_t*>(out) + (int64_t)frame * cap + running;
            for (uint32_t j = tid; j < tot; j += 256) {
                const uint32_t p = sh.stage[j];
                const int y = fastdiv40((int)p, W_m40);
                dst[j] = walk_pk((int)(p - (uint32_t)y * (uint32_t)W), y);
            }
        } else {
            v2i* dst = reinterpret_cast<v2i*>(fo + running);
            for (uint32_t j = tid; j < tot; j += 256) {
                const uint32_t p = sh.stage[j];
                const int y = fastdiv40((int)p, W_m40);
                __builtin_nontemporal_store((v2i){(int)(p - (uint32_t)y * (uint32_t)W), y}, dst + j);
            }
        }
        running += tot;
    }
    if (tid == 0) counts[frame] = running;
}

// ---------------------------------------------------------------------------
// The batch's road images and their walks in one pass (road_kernel). The
// pipeline's points come in raster order of their grid points, (x, y) = (gx -
// dx, gy - dy) with deltas 0 or 1, so y never drops by more than one along the
// list (y_j >= y_i - 1 for j > i). One workgroup per frame builds its image a
// band of rows at a time in LDS: it zeroes the band, marks the points whose
// row is in the band (scanning the list from a cursor; a chunk holding a row
// >= r1 + 1 ends the band, the first chunk holding a row >= r1 starts the next
// band's scan), writes the band's rows once (no memset, no read-modify-write
// of scattered bytes) and walks the band's non-zero pixels from LDS with the
// nonzero_kernel's scan and staging (no re-read of the image). A point with y
// = -1 (numpy's img[-1], the last row) is kept in a bit row until the band
// holding row H - 1. Bytes per frame: the points (8 B each) + the image once +
// the walk (8 B per non-zero pixel), against + the image three more times
// (zeroing, the scattered bytes' read-modify-write, the walk's read) before.
// ---------------------------------------------------------------------------
constexpr int kRoadPts = 4, kRoadChunk = 256 * kRoadPts;   // points per lane / chunk of the scan (8: 4.35 vs 4.13 ms)
constexpr int kRoadBandBytes = 12288;   // LDS of one band (W = 1024: 12 rows): 29 KB in all, 5 workgroups per CU

struct RoadShared {
    uint32_t wtot[4];
    uint32_t wrap[128];                   // bit x: row H - 1 has a point with y = -1 at x (W <= 4096)
    uint32_t stage[256 * 16];             // a walk chunk's pixel indices, in output order
};

// With paint != nullptr the same pass also writes stereovision.py:131-133's
// imageRoadMap: a copy of the frame's BGR (the gamma-corrected imgL, frames x H
// x W x 3 at a row stride of 3 W) with [0, 255, 0] wherever the band's image is
// marked — generatePointsAsImage and the paint index the same [y][x] with the
// same wrap, so the band in LDS is exactly the paint mask (3 B read + 3 B
// written per pixel, 8 bytes a lane).
__global__ __launch_bounds__(256) void road_kernel(const uint32_t* __restrict__ pxy,
                                                   const int64_t* __restrict__ counts, int64_t cap,
                                                   uint8_t* __restrict__ img, int H, int W, int Wu, int R,
                                                   uint64_t W_m40, int32_t* __restrict__ nzout,
                                                   int64_t* __restrict__ nzcount, const uint8_t* __restrict__ bgr,
                                                   uint8_t* __restrict__ paint, bool vec) {
    __shared__ RoadShared sh;
    extern __shared__ uint4 road_band[];   // the band: R rows of W bytes (dynamic LDS)
    uint8_t* const band = reinterpret_cast<uint8_t*>(road_band);
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.x;
    int64_t n = counts[4 * (int64_t)frame + 2];
    n = n < 0 ? 0 : (n > cap ? cap : n);
    const uint32_t* fxy = pxy + (int64_t)frame * cap;
    uint8_t* fimg = img + (int64_t)frame * H * W;
    uint32_t* fo = reinterpret_cast<uint32_t*>(nzout) + (int64_t)frame * cap;
    if (tid < 128) sh.wrap[tid] = 0;
    // this lane's kRoadPts consecutive points of the 256 * kRoadPts-point chunk at i0 (qy = -2: past the
    // list): one 16-byte load of pp_pack words when the plane is 16-byte aligned (vec), 4-byte loads at the end
    static_assert(kRoadPts == 4, "one uint4 of packed points per lane");
    const auto load = [&](int64_t i0, int (&qx)[kRoadPts], int (&qy)[kRoadPts]) {
        const int64_t i = i0 + kRoadPts * tid;
        if (vec && i + kRoadPts <= n) {
            const uint4 v = *reinterpret_cast<const uint4*>(fxy + i);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int t = 0; t < kRoadPts; ++t) {
                qx[t] = pp_x(w[t]);
                qy[t] = pp_y(w[t]);
            }
        } else {
#pragma unroll
            for (int t = 0; t < kRoadPts; ++t) {
                const bool ok = i + t < n;
                const uint32_t w = ok ? fxy[i + t] : 0u;
                qx[t] = ok ? pp_x(w) : 0;
                qy[t] = ok ? pp_y(w) : -2;
            }
        }
    };
    int64_t cur = 0;
    uint32_t running = 0;
    for (int r0 = 0; r0 < H; r0 += R) {
        const int r1 = min(r0 + R, H);
        const int bpx = (r1 - r0) * W, bz = (bpx + 15) & ~15;
        for (int o = 16 * tid; o < bz; o += 16 * 256) *reinterpret_cast<uint4*>(band + o) = make_uint4(0, 0, 0, 0);
        __syncthreads();   // band zeroed (and the previous band's walk is done with sh.stage)
        int64_t i = cur, next = -1;
        int qx[kRoadPts], qy[kRoadPts], nx[kRoadPts], ny[kRoadPts];
        if (i < n) load(i, qx, qy);
        while (i < n) {
            if (i + kRoadChunk < n) load(i + kRoadChunk, nx, ny);   // in flight while this chunk is marked
            bool ge1 = false, ge2 = false;
#pragma unroll
            for (int t = 0; t < kRoadPts; ++t) {
                const int y = qy[t];
                if (y == -2) continue;
                const int x = qx[t] < 0 ? qx[t] + Wu : qx[t];
                if (y < 0) atomicOr(&sh.wrap[x >> 5], 1u << (x & 31));
                else if (y >= r0 && y < r1) band[(y - r0) * W + x] = 255;
                ge1 |= y >= r1;
                ge2 |= y >= r1 + 1;
            }
            // (one barrier with the flags in LDS instead of two: 4.08-4.12 vs 4.06 ms, not kept)
            const bool any1 = __syncthreads_or(ge1) != 0;
            const bool any2 = __syncthreads_or(ge2) != 0;
            if (next < 0 && any1) next = i;   // the next band's rows start in this chunk at the earliest
            i += kRoadChunk;
            if (any2) break;                  // every later point lies at row r1 or below
#pragma unroll
            for (int t = 0; t < kRoadPts; ++t) {
                qx[t] = nx[t];
                qy[t] = ny[t];
            }
        }
        cur = next >= 0 ? next : i;
        if (r1 == H) {   // the wrapped points' marks on the last row
            for (int x = tid; x < W; x += 256)
                if ((sh.wrap[x >> 5] >> (x & 31)) & 1u) band[(H - 1 - r0) * W + x] = 255;
        }
        __syncthreads();   // the band is complete
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        typedef unsigned v2u __attribute__((ext_vector_type(2)));
        if ((W & 15) == 0) {   // uniform: 16-byte non-temporal row stores (the images are read back later, if at all)
            for (int o = 16 * tid; o < bpx; o += 16 * 256)
                __builtin_nontemporal_store(*reinterpret_cast<const v4u*>(band + o),
                                            reinterpret_cast<v4u*>(fimg + (int64_t)r0 * W + o));
        } else {
            for (int o = 8 * tid; o < bpx; o += 8 * 256)
                __builtin_nontemporal_store(*reinterpret_cast<const v2u*>(band + o),
                                            reinterpret_cast<v2u*>(fimg + (int64_t)r0 * W + o));
        }
        if (paint) {   // uniform: imageRoadMap rows r0..r1 (byte j of the band's rows is pixel j / 3, channel j % 3)
            const int64_t fo3 = ((int64_t)frame * H + r0) * W * 3;
            const uint2* src = reinterpret_cast<const uint2*>(bgr + fo3);
            v2u* dst = reinterpret_cast<v2u*>(paint + fo3);
            const int nb8 = bpx * 3 / 8;   // W % 8 == 0: whole 8-byte units
            for (int u = tid; u < nb8; u += 256) {
                const uint2 q = src[u];
                uint32_t w[2] = {q.x, q.y};
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint32_t j = (uint32_t)(8 * u + k);
                    const uint32_t pix = (j * 43691u) >> 17;   // j / 3 for j < 98304 (R W <= 16384)
                    const uint32_t ch = j - 3 * pix;
                    if (band[pix]) {
                        const uint32_t sh8 = 8 * (k & 3);
                        w[k >> 2] = (w[k >> 2] & ~(0xFFu << sh8)) | ((ch == 1 ? 0xFFu : 0u) << sh8);
                    }
                }
                __builtin_nontemporal_store((v2u){w[0], w[1]}, dst + u);
            }
        }
        // the band's non-zero pixels in raster order (nonzero_kernel's chunk logic, from LDS)
        const uint32_t* bw = reinterpret_cast<const uint32_t*>(band);
        const int vecs = bz / 16;
        for (int base = 0; base < vecs; base += 256) {
            const int v = base + tid;
            uint4 q = make_uint4(0, 0, 0, 0);
            if (v < vecs) q = *reinterpret_cast<const uint4*>(bw + 4 * v);
            const uint32_t w[4] = {q.x, q.y, q.z, q.w};
            uint32_t bits = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t nz = (((w[k] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w[k]) & 0x80808080u;
                bits |= ((nz >> 7) & 1u) << (4 * k) | ((nz >> 15) & 1u) << (4 * k + 1) |
                        ((nz >> 23) & 1u) << (4 * k + 2) | ((nz >> 31) & 1u) << (4 * k + 3);
            }
            const uint32_t cnt = __builtin_popcount(bits);
            const uint32_t inc = wave_incl_scan(cnt);
            if (lane == 63) sh.wtot[wave] = inc;
            __syncthreads();   // also: the previous chunk's writes have read sh.stage
            uint32_t wbase = 0, tot = 0;
#pragma unroll
            for (int w4 = 0; w4 < 4; ++w4) {
                const uint32_t t = sh.wtot[w4];
                wbase += w4 < wave ? t : 0u;
                tot += t;
            }
            uint32_t o = wbase + inc - cnt;
            const uint32_t p0 = (uint32_t)r0 * (uint32_t)W + (uint32_t)(v * 16);
            while (bits) {
                const int b = __builtin_ctz(bits);
                bits &= bits - 1;
                sh.stage[o++] = p0 + (uint32_t)b;
            }
            __syncthreads();   // sh.wtot is rewritten next chunk; sh.stage is complete
            uint32_t* dst = fo + running;   // packed entries (walk_pk), ordinary stores (partial lines merge in L2)
            for (uint32_t j = tid; j < tot; j += 256) {
                const uint32_t p = sh.stage[j];
                const int y = fastdiv40((int)p, W_m40);
                dst[j] = walk_pk((int)(p - (uint32_t)y * (uint32_t)W), y);
            }
            running += tot;
        }
    }
    if (tid == 0) nzcount[frame] = running;
}

// ---------------------------------------------------------------------------
// The road pass from the pipeline's bitmap (PipeBuffers::rbits: the resident pipeline marks every int32 point's
// pixel, numpy's -1 wrap included, as it makes the points; 1024-wide frames). The image, the walk and the paint
// are then functions of 68 KB a frame instead of the 8 B a point the road_kernel reads, and the rows are
// independent: one wave a row.
//  * road_rowscan_kernel — one workgroup a frame: each row's non-zero count (popcount of its 32 words), an
//                          exclusive scan over the rows -> the walk index of the row's first pixel; the frame's
//                          total -> nzcount.
//  * road_rows_kernel    — one wave a row: the row's bytes (0 / 255, 16 pixels a lane, one 16-byte store), its
//                          walk entries [x, y] in raster order (64 pixels a pass, ranked by v_mbcnt, each pass
//                          one coalesced run of 8-byte pairs), and on request the imageRoadMap row (the BGR row
//                          with [0, 255, 0] at every marked pixel).
// ---------------------------------------------------------------------------
constexpr int kRbWords = 32;   // words a row: 1024 pixels

__global__ __launch_bounds__(256) void road_rowscan_kernel(const uint32_t* __restrict__ bits, int H,
                                                           int32_t* __restrict__ roff, int64_t* __restrict__ nzcount) {
    __shared__ uint32_t wtot[4];
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.x;
    const uint4* fb = reinterpret_cast<const uint4*>(bits + (int64_t)frame * H * kRbWords);
    int32_t* fo = roff + (int64_t)frame * H;
    constexpr int R = 4;   // rows a thread (H <= 1024)
    uint32_t cnt[R], tot = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int row = tid * R + r;
        uint32_t c = 0;
        if (row < H) {
#pragma unroll
            for (int q = 0; q < kRbWords / 4; ++q) {
                const uint4 w = fb[row * (kRbWords / 4) + q];
                c += __builtin_popcount(w.x) + __builtin_popcount(w.y) + __builtin_popcount(w.z) +
                     __builtin_popcount(w.w);
            }
        }
        cnt[r] = c;
        tot += c;
    }
    const uint32_t inc = wave_incl_scan(tot);
    if (lane == 63) wtot[wave] = inc;
    __syncthreads();
    uint32_t wbase = 0, all = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        wbase += w < wave ? wtot[w] : 0u;
        all += wtot[w];
    }
    uint32_t run = wbase + inc - tot;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int row = tid * R + r;
        if (row < H) fo[row] = (int32_t)run;
        run += cnt[r];
    }
    if (tid == 0) nzcount[frame] = all;
}

// RPW rows a wave (rows y0, y0 + 4, ...: the workgroup's four waves interleave): the next row's 32 words are
// loaded (scalar) before this row's stores
template <bool NT, bool NTI>
__device__ __forceinline__ void road_row(const uint32_t (&ws)[kRbWords], uint32_t word, int32_t first, int frame,
                                         int y, int H,
                                         int64_t cap, uint8_t* __restrict__ img, int32_t* __restrict__ nzout,
                                         const uint8_t* __restrict__ bgr, uint8_t* __restrict__ paint) {
    const int lane = lane_id();
    const int64_t row = (int64_t)frame * H + y;
    const uint32_t b16 = (lane & 1) ? word >> 16 : word & 0xFFFFu;   // pixels 16 lane .. 16 lane + 15
    uint32_t q[4];   // bit k of a nibble -> byte k = 0xFF (v_perm selector 0x0D; 0x0C gives 0x00)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t nib = (b16 >> (4 * i)) & 0xFu;
        q[i] = __builtin_amdgcn_perm(0u, 0u, ((__umul24(nib, 0x00204081u) & 0x01010101u) + 0x0C0C0C0Cu));
    }
    v4i* irow = reinterpret_cast<v4i*>(img + row * (kRbWords * 32) + 16 * lane);
    if (NTI)
        __builtin_nontemporal_store((v4i){(int)q[0], (int)q[1], (int)q[2], (int)q[3]}, irow);
    else
        *irow = (v4i){(int)q[0], (int)q[1], (int)q[2], (int)q[3]};
    // the walk: [x, y] of the row's marked pixels in x order, from the row's first index. Pass i covers pixels
    // 64 i .. 64 i + 63, lane l pixel 64 i + l: its bit is bit l of words 2i, 2i+1 (scalar loads, the same for
    // the whole wave), its rank among the pass's marked pixels one v_mbcnt pair, and the pass's entries one
    // contiguous run after the previous passes' (s_bcnt1): sixteen coalesced stores, no loop, no LDS.
    uint32_t* dst = reinterpret_cast<uint32_t*>(nzout) + (int64_t)frame * cap + first;   // packed (walk_pk)
    uint32_t base = 0;
#pragma unroll
    for (int i = 0; i < kRbWords / 2; ++i) {
        const uint32_t lo = ws[2 * i], hi = ws[2 * i + 1];
        const uint32_t mine = lane < 32 ? lo >> lane : hi >> (lane - 32);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi(hi, __builtin_amdgcn_mbcnt_lo(lo, 0u));
        if (mine & 1u) {
            if (NT)
                __builtin_nontemporal_store(walk_pk(64 * i + lane, y), dst + base + rank);
            else
                dst[base + rank] = walk_pk(64 * i + lane, y);
        }
        base += __builtin_popcount(lo) + __builtin_popcount(hi);
    }
    if (paint) {   // imageRoadMap (stereovision.py:131-133): the lane's 16 pixels, 48 bytes
        const uint4* src = reinterpret_cast<const uint4*>(bgr + row * (kRbWords * 32) * 3 + 48 * lane);
        uint4 v[3] = {src[0], src[1], src[2]};
        uint8_t* px = reinterpret_cast<uint8_t*>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if ((b16 >> k) & 1u) {
                px[3 * k] = 0;
                px[3 * k + 1] = 255;
                px[3 * k + 2] = 0;
            }
        uint4* out = reinterpret_cast<uint4*>(paint + row * (kRbWords * 32) * 3 + 48 * lane);
        out[0] = v[0];
        out[1] = v[1];
        out[2] = v[2];
    }
}

template <bool NT, bool NTI, int RPW>
__global__ __launch_bounds__(256) void road_rows_kernel(const uint32_t* __restrict__ bits, int H,
                                                        const int32_t* __restrict__ roff, int64_t cap,
                                                        uint8_t* __restrict__ img, int32_t* __restrict__ nzout,
                                                        const uint8_t* __restrict__ bgr, uint8_t* __restrict__ paint) {
    const int frame = blockIdx.y;
    int y = blockIdx.x * 4 * RPW + wave_uniform_id();
    if (y >= H) return;
    const uint32_t* fb = bits + (int64_t)frame * H * kRbWords;   // wave-uniform addresses: scalar loads
    const int32_t* fo = roff + (int64_t)frame * H;
    uint32_t ws[kRbWords];   // the row's words in SGPRs before its first store
#pragma unroll
    for (int i = 0; i < kRbWords; ++i) ws[i] = fb[y * kRbWords + i];
    uint32_t word = fb[y * kRbWords + (lane_id() >> 1)];   // the lane's own word (pixels 16 lane ..)
    int32_t first = fo[y];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const int yn = y + 4;
        uint32_t wn[kRbWords], wordn = 0;
        int32_t fn = 0;
        const bool more = r + 1 < RPW && yn < H;   // uniform
        if (more) {
#pragma unroll
            for (int i = 0; i < kRbWords; ++i) wn[i] = fb[yn * kRbWords + i];
            wordn = fb[yn * kRbWords + (lane_id() >> 1)];
            fn = fo[yn];
        }
        road_row<NT, NTI>(ws, word, first, frame, y, H, cap, img, nzout, bgr, paint);
        if (!more) break;
#pragma unroll
        for (int i = 0; i < kRbWords; ++i) ws[i] = wn[i];
        word = wordn;
        first = fn;
        y = yn;
    }
}

hipError_t launch_road_bits(const uint32_t* bits, int frames, int H, int W, int32_t* roff, int64_t cap,
                            uint8_t* img, int32_t* nzout, int64_t* nzcount, const uint8_t* bgr, uint8_t* paint,
                            hipStream_t s) {
    if (frames <= 0) return hipSuccess;
    if (W != kRbWords * 32 || H <= 0 || H > 1024 || (paint && !bgr)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(road_rowscan_kernel, dim3(frames), dim3(256), 0, s, bits, H, roff, nzcount);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // The walk's entries as ordinary stores: a pass's run starts at any 8-byte offset, and the partial lines at
    // its ends merge with the neighbouring passes' in L2 before they reach HBM; written non-temporal each partial
    // line went out on its own: 2.46 vs 2.99 ms per 4096 frames (profiles/r04/ab_road_walk_nt.txt); the image
    // rows too (2.40 vs 2.41-2.49 ms, profiles/r04/ab_road_img_nt.txt). A/B (diagnostic build): SVX_ROAD_NT=1 /
    // SVX_ROAD_IMG_NT=1 make the walk / image stores non-temporal.
    const char* nt = svx_knob("SVX_ROAD_NT");
    const char* nti = svx_knob("SVX_ROAD_IMG_NT");
    const bool wnt = nt && nt[0] == '1', int_ = nti && nti[0] == '1';
    // rows a wave: 2 (SVX_ROAD_RPW, DIAGNOSTIC A/B: 1 / 2 / 4 took 1.557 / 1.422 / 1.498 ms per 4096 frames in one
    // process, profiles/r05/probe_road_rpw_s8.txt)
    const char* rk = svx_knob("SVX_ROAD_RPW");
    const int rpw = rk ? std::atoi(rk) : 2;
#define SVX_ROAD_ROWS(R)                                                                                            \
    do {                                                                                                            \
        const dim3 g((H + 4 * (R) - 1) / (4 * (R)), frames);                                                        \
        if (wnt && int_)                                                                                            \
            hipLaunchKernelGGL((road_rows_kernel<true, true, R>), g, dim3(256), 0, s, bits, H, roff, cap, img,     \
                               nzout, bgr, paint);                                                                  \
        else if (wnt)                                                                                               \
            hipLaunchKernelGGL((road_rows_kernel<true, false, R>), g, dim3(256), 0, s, bits, H, roff, cap, img,    \
                               nzout, bgr, paint);                                                                  \
        else if (int_)                                                                                              \
            hipLaunchKernelGGL((road_rows_kernel<false, true, R>), g, dim3(256), 0, s, bits, H, roff, cap, img,    \
                               nzout, bgr, paint);                                                                  \
        else                                                                                                        \
            hipLaunchKernelGGL((road_rows_kernel<false, false, R>), g, dim3(256), 0, s, bits, H, roff, cap, img,   \
                               nzout, bgr, paint);                                                                  \
    } while (0)
    if (rpw >= 4) SVX_ROAD_ROWS(4);
    else if (rpw == 2) SVX_ROAD_ROWS(2);
    else SVX_ROAD_ROWS(1);
#undef SVX_ROAD_ROWS
    return hipGetLastError();
}

hipError_t launch_road(const uint32_t* pxy, const int64_t* counts, int64_t cap, uint8_t* img,
                       int frames, int H, int W, int Wu, int32_t* nzout, int64_t* nzcount, const uint8_t* bgr,
                       uint8_t* paint, hipStream_t s) {
    if (frames <= 0) return hipSuccess;
    if (W <= 0 || W > 4096 || W % 8 || H <= 0 || Wu <= 0 || Wu > W || (int64_t)H * W >= (1ll << 28))
        return hipErrorInvalidValue;
    int bytes = kRoadBandBytes;   // SVX_ROAD_BAND: A/B knob
    if (const char* e = svx_knob("SVX_ROAD_BAND")) bytes = std::max(4096, std::min(65536, std::atoi(e)));
    const int R = std::max(1, bytes / W);   // rows per band
    const size_t dyn = ((size_t)R * W + 15) / 16 * 16;
    if (dyn > 65536 || (paint && (!bgr || (size_t)R * W * 3 >= 98304))) return hipErrorInvalidValue;
    const uint64_t m40 = (((uint64_t)1 << 40) + (uint64_t)W - 1) / (uint64_t)W;
    // vec: the point planes and the walk's output 16-byte aligned at every frame (cap % 4 == 0), so a lane takes
    // its 4 points with one load per plane and writes two walk outputs with one store
    if (H > 65536) return hipErrorInvalidValue;   // packed walk entries: y < 65536
    const bool vec = cap % 4 == 0 && (reinterpret_cast<uintptr_t>(pxy) & 15u) == 0;
    hipLaunchKernelGGL(road_kernel, dim3(frames), dim3(256), dyn, s, pxy, counts, cap, img, H, W, Wu, R, m40, nzout,
                       nzcount, bgr, paint, vec);
    return hipGetLastError();
}

hipError_t launch_nonzero(const uint8_t* img, int frames, int64_t px, int W, int32_t* out, int64_t cap, int64_t* counts,
                          bool packed, hipStream_t s) {
    if (frames <= 0) return hipSuccess;
    if (px % 4 || px >= (1ll << 28) || W <= 0 || W > 4096 || (packed && px / W > 65536)) return hipErrorInvalidValue;
    const uint64_t m40 = (((uint64_t)1 << 40) + (uint64_t)W - 1) / (uint64_t)W;
    if (packed)
        hipLaunchKernelGGL(nonzero_kernel<true>, dim3(frames), dim3(256), 0, s, img, px, W, m40, out, cap, counts);
    else
        hipLaunchKernelGGL(nonzero_kernel<false>, dim3(frames), dim3(256), 0, s, img, px, W, m40, out, cap, counts);
    return hipGetLastError();
}

}  // namespace svx
