// Host-side launchers for the svx kernels (one TU per kernel family).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "svx_device.h"

namespace svx {

// kernels/project.hip -------------------------------------------------------
hipError_t launch_synth(const KParams& p, uint8_t* disp, uint8_t* bgr, int frames,
                        int64_t first_frame, hipStream_t s);
// K1: dense fp32 projection over frames * Hg * Q quads; qpl = quads per lane (1, 2, 4).
// kname (nullable): the launched instance's name as rocprofv3 prints it.
hipError_t launch_project_dense(const KParams& p, const uint8_t* disp, float* X, float* Y, float* Z,
                                int frames, int qpl, int nontemporal, hipStream_t s, const char** kname = nullptr);
// Drop-in projection: fp64 XYZ, compacted in raster order (any H, W, step).
hipError_t launch_project_compact_f64(const KParams& p, const uint8_t* disp, int64_t ld_disp,
                                      const uint8_t* bgr, int64_t ld_bgr, double* xyz, uint8_t* rgb,
                                      uint64_t* status, uint32_t* ticket, uint32_t* count,
                                      uint32_t* err, hipStream_t s);
hipError_t launch_rows6(const double* xyz, const uint8_t* rgb, int64_t n, double* rows, hipStream_t s);
hipError_t launch_backproject_f64(const double* xyz, int64_t n, int64_t ld, double f, double cw,
                                  double ch, double* xy, hipStream_t s);
int project_compact_tiles(const KParams& p);

// kernels/tables.hip --------------------------------------------------------
hipError_t launch_hue_lut(int16_t* lut, int variant, hipStream_t s);
// dx bits [256][dx_words], dy bits [256][dy_words]; optional int8 tables.
// dxT / dyT (PipeBuffers) from dxbits / dybits: 8 x 32 dx_words + 8 x 32 dy_words words
hipError_t launch_delta_transpose(const KParams& p, const uint32_t* dxbits, const uint32_t* dybits, uint32_t* dxT,
                                  uint32_t* dyT, hipStream_t s);
hipError_t launch_delta_tables(const KParams& p, uint32_t* dxbits, uint32_t* dybits, int8_t* dx8,
                               int8_t* dy8, hipStream_t s);

// kernels/pipeline.hip ------------------------------------------------------
struct PipeBuffers {
    const uint8_t* disp;
    const uint8_t* bgr;
    uint32_t* hist;      // frames x 1024
    int64_t* counts;     // frames x 4 (N_valid, N_kept, N_kept2, spare)
    uint16_t* kbits;     // frames x tiles x 256: keep1 (pass 1) -> keep2 (offsets) bit 4*i+k of each lane's quads
    uint32_t* tcount;    // frames x tiles: keep1 count per tile (pass 1)
    uint32_t* toff;      // frames x tiles: output offset of each tile (offsets kernel)
    uint32_t* pres;      // frames x tiles x 32: hue bins present among the tile's keep1 points
    float* ox;           // frame f's X[cap] at ox + f * ofs (Y, Z likewise): three planes of frames x cap
    float* oy;           //   (ofs = cap), or SoA per frame (ofs = 3 cap, oy = ox + cap, oz = ox + 2 cap)
    float* oz;
    int64_t ofs;
    uint32_t* pxy;       // the back-projection (planePoints): one word a point, pp_pack(x, y), frames x cap
                         //   (frame f's at f * cap; widened to int32 pairs on read-back)
    const uint32_t* dxbits;
    const uint32_t* dybits;
    // the same bits transposed: word j of coordinate c holds d = 32 j .. 32 j + 31 (bit d mod 32), as
    // dxT[j * 32 dx_words + x] and dyT[j * 32 dy_words + y] (launch_delta_transpose)
    const uint32_t* dxT = nullptr;
    const uint32_t* dyT = nullptr;
    int64_t cap;         // points per frame (Ng)
    const FramePlane* planes = nullptr;   // device planes: frame f uses planes[f * plane_stride] (else the KParams plane)
    int plane_stride = 1;                 // 0: one device plane for every frame (a broadcast plane)
    // optional (resident kernel, 1024-wide frames at step 1): a bitmap of the pixels the int32 points mark
    // (generatePointsAsImage's road image, numpy's -1 wrap included), frames x rb_H rows x 32 words, written by
    // pass 2 as it makes the points; the road pass then reads 68 KB a frame instead of the points
    uint32_t* rbits = nullptr;
    int rb_H = 0, rb_Wu = 0;              // the image rows and the frame's own width (x = -1 wraps to rb_Wu - 1)
};
int pipeline_tiles_per_frame(const KParams& p);
// The whole chain for frames [0, frames) in chunks: chunks + 2 fused stage
// launches on stream sa, one offsets launch per chunk on stream sb, ordered by
// the 2 * chunks events in ev.
hipError_t launch_pipeline(const KParams& p, const PipeBuffers& b, int frames, int chunk, hipStream_t sa,
                           hipStream_t sb, hipEvent_t* ev);

// kernels/resident.hip -----------------------------------------------------
// One workgroup per frame (both passes, LDS histogram, running output offset).
// keep1 per grid point from the frame's plane (b.planes, device memory, required):
// the fp32 division-free test with the fp64 reference arithmetic inside its
// guard; chunks the plane rules out are skipped.
bool resident_supported(const KParams& p);
// One workgroup per frame (pass 1 then pass 2); prefetch = pass 2 loads the
// next chunk before issuing this chunk's stores (costs registers).
// kname (nullable): the launched instance's name as rocprofv3 prints it.
hipError_t launch_pipeline_resident(const KParams& p, const PipeBuffers& b, int frames,
                                    bool prefetch, hipStream_t s, bool prefetch1 = false,
                                    const char** kname = nullptr);
// b.rbits can be filled: W == 1024 at step 1 with lane-contiguous quads (4 grid rows a chunk, 32 words a row)
bool resident_road_bits_supported(const KParams& p);
// *dst = v on stream s (the resident kernel reads its planes from device memory).
hipError_t launch_store_plane(const FramePlane& v, FramePlane* dst, hipStream_t s);

// kernels/prepass.hip ------------------------------------------------------
// fillDisparity frame recurrence / fillAltDisparity row means / maskDisparity.
// frame_px % 4 == 0 (W % 4 == 0); mask_ff = 0x00/0xFF bytes (launch_mask_bytes).
hipError_t launch_mask_bytes(const uint8_t* m, uint8_t* out, int64_t n, hipStream_t s);
hipError_t launch_fill_prev(const uint8_t* raw, uint8_t* out, uint8_t* masked, const uint8_t* mask_ff,
                            const uint8_t* prev0, int frames, int64_t frame_px, hipStream_t s);
// rows of Wrow pixels stored at stride W (W % 4 == 0, Wrow <= W; the padding is left alone)
hipError_t launch_fill_mean(uint8_t* disp, uint8_t* masked, const uint8_t* mask_ff, int frames, int H, int W,
                            int Wrow, hipStream_t s);
hipError_t launch_mask(const uint8_t* disp, uint8_t* out, const uint8_t* mask_ff, int frames, int64_t frame_px,
                       hipStream_t s);

// kernels/raster.hip -------------------------------------------------------
// Road raster (points -> 255 on a zeroed image) and the raster-order non-zero walk.
// counts: NULL -> cap points per frame, else counts[frame * cstride + cidx].
// images of H rows at stride W; Wu = the image width (numpy's negative-index wrap). Point i of frame f:
// (px[(f cap + i) ps], py[(f cap + i) ps]): ps = 2 for interleaved (x, y) pairs; ps = 0: px holds pp_pack words
// (a batch's planePoints), py unused.
hipError_t launch_raster(const int32_t* px, const int32_t* py, int ps, const int64_t* counts, int cstride, int cidx,
                         int64_t cap, uint8_t* img, int frames, int H, int W, int Wu, hipStream_t s);
// The batch's road images and walks in one pass (road_kernel): the pipeline's points (two planes, frame f's
// counts[4f + 2] points at f * cap, in the pipeline's raster order) -> img (frames x H x W, W % 8 == 0) and the
// raster-order [j, i] of every non-zero pixel (frames x cap pairs) + nzcount[frame]; with paint != nullptr also
// imageRoadMap (stereovision.py:131-133): bgr (frames x H x W x 3) with [0, 255, 0] at the marked pixels -> paint.
hipError_t launch_road(const uint32_t* pxy, const int64_t* counts, int64_t cap, uint8_t* img,
                       int frames, int H, int W, int Wu, int32_t* nzout, int64_t* nzcount, const uint8_t* bgr,
                       uint8_t* paint, hipStream_t s);
// img frames x px (px % 4 == 0, rows of W <= 4096 pixels)
// The road pass from the resident pipeline's bitmap (PipeBuffers::rbits; W == 1024, H <= 1024): images, walks
// (roff: frames x H scratch, the walk index of each row's first pixel) and, when paint != nullptr, the
// imageRoadMap copies of bgr.
hipError_t launch_road_bits(const uint32_t* bits, int frames, int H, int W, int32_t* roff, int64_t cap,
                            uint8_t* img, int32_t* nzout, int64_t* nzcount, const uint8_t* bgr, uint8_t* paint,
                            hipStream_t s);
hipError_t launch_nonzero(const uint8_t* img, int frames, int64_t px, int W, int32_t* out, int64_t cap, int64_t* counts, bool packed,
                          hipStream_t s);

// kernels/ransac.hip -------------------------------------------------------
// Host: replay CPython's random draws of RANSAC (functions.py:240-298) from a
// random.getstate() word vector (624 MT words + index; updated in place);
// returns the number of trials drawn (0 when n < k: sample raises first).
int ransac_draw(uint32_t* state625, const double* pts, int64_t n, int64_t ld, int trials, int k, int32_t* sidx,
                int32_t* tri);
// Device: abc, mean distance and a 0/1/2 (ok/singular/ill-conditioned) flag per trial.
hipError_t launch_ransac_eval(const double* pts, int64_t ld, const int32_t* sidx, const int32_t* tri, int trials,
                              int k, double* abc, double* err, uint8_t* flag, hipStream_t s);

// kernels/ransac_batch.hip -------------------------------------------------
// maskpoints of every frame: the d > 0 points of (disp & mask_ff) on the step-2
// grid, raster order, as packed words x | y << 12 | d << 24 (frames x cap,
// H, W <= 4096), counts[frame]; their fp64 X, Y, Z are computed where used
// (launch_maskpoints_xyz, and inside the RANSAC kernels).
hipError_t launch_maskpoints(const uint8_t* disp, const uint8_t* mask_ff, int frames, int H, int W, const KParams& p,
                             uint32_t* packed, int64_t cap, int64_t* counts, hipStream_t s);
// fp64 X (per x / 2, d), Y (per y / 2, d) and Z (per d) of the step-2 grid of an H x W frame, the reference's
// arithmetic (functions.py:191-193): ransac_tables_bytes(H, W) bytes
size_t ransac_tables_bytes(int H, int W);
hipError_t launch_ransac_tables(int H, int W, const KParams& p, double* tab, hipStream_t s);
// n packed maskpoints -> n x 3 fp64 X, Y, Z (from the tables)
hipError_t launch_maskpoints_xyz(const uint32_t* packed, int64_t n, const double* tab, int H, int W, double* out,
                                 hipStream_t s);
// RANSAC of every frame with random.seed(seed_base + first_frame + frame):
// abc (frames x 3), err, winning trial (-1: none ran), flags (1 a singular
// trial, 2 ill-conditioned winner, 4 near-tie). cap <= 163,840, k <= 1024.
// trace (optional): frames x trace_trials x (k + 3) drawn indices (sample, then P1..P3).
// frame_planes: the keep1 plane fields of every frame from its RANSAC result.
// cp: the camera's fp32 fields (B32, fB32, cw/ch hi-lo) for the fp32 screen of every trial.
// random.sample's set-branch threshold: 21 + 4 ** ceil(log4(3k)) for k > 5 (3k is never a power of 4)
__host__ __device__ inline int64_t ransac_setsize(int k) {
    int64_t setsize = 21;
    if (k > 5) {
        int64_t pw = 1;
        while (pw < 3ll * k) pw *= 4;
        setsize += pw;
    }
    return setsize;
}
// Per-trial scratch of the two RANSAC kernels: every trial's sample (u16 when
// every frame has < 65536 points, else int32: ransac_sidx_bytes), its record
// (a, b, c, |abc|, flag: frames x trials x 5 doubles) and per frame the status
// and the number of trials drawn (frames x 2 int32).
struct RansacScratch {
    void* sidx;
    double* tri;
    int32_t* fstat;
};
size_t ransac_sidx_bytes(int64_t max_n, int frames, int trials, int k);
// max_n: the largest frame's point count; max_pool_n: the largest count that takes random.sample's pool
// branch (n <= setsize(k)), 0 if none (both size the draw kernel's LDS). trials <= 4096. phases: 1 = the draw
// kernel, 2 = the evaluation kernel, 3 = both (in that order; the frame loop runs them as separate stages).
hipError_t launch_ransac_batch(const uint32_t* packed, const double* tab, int H, int W, int64_t cap, const KParams& cp,
                               const int64_t* counts, int64_t max_n, int64_t max_pool_n, uint64_t seed_base,
                               int64_t first_frame, int frames, int trials, int k, const RansacScratch& rs, double* abc,
                               double* err, int32_t* trial, uint32_t* flags, int32_t* trace, int trace_trials,
                               int ablate, int phases, uint64_t* started, uint64_t epoch, hipStream_t s);
// the frame loop's dispatch gate: returns once *flag >= epoch (the draw kernel's last workgroup, launched with
// started = flag, is resident) or after max_ms of wall clock
hipError_t launch_loop_gate(const uint64_t* flag, uint64_t epoch, double max_ms, hipStream_t s);
// out[i] = plane_fields of abc[3i..3i+2] (trial[i] < 0, or trial NULL and a NaN plane: valid = 0);
// trial may be NULL (a device plane, e.g. the RCCL broadcast buffer).
hipError_t launch_frame_planes(const double* abc, const int32_t* trial, int frames, const KParams& p, double thr,
                               FramePlane* out, hipStream_t s);

// kernels/stages.hip -------------------------------------------------------
// a2: |(P.abc - 1) / d| per point (abcd = a, b, c, d); a4/a5: hue bin per point,
// bin counts and first point per bin (hist zeroed, first INT32_MAX-filled);
// a3/a6: stable selection (mode 0: vals < thr, mode 1: ok[bins] != 0).
hipError_t launch_point_errors(const double* xyz, int64_t n, int64_t ld, const double* abcd, double* out,
                               hipStream_t s);
hipError_t launch_hue_hist(const uint8_t* rgb, int64_t n, int64_t ld, int16_t* bins, uint32_t* hist, int32_t* first,
                           hipStream_t s);
hipError_t launch_select(int mode, const double* vals, double thr, const int16_t* bins, const uint8_t* ok, int64_t n,
                         int64_t* out_idx, int64_t* out_n, hipStream_t s);

// kernels/digest.hip -------------------------------------------------------
// Per-frame verification digests (out: frames x 8 u64, see sv_batch_digest).
hipError_t launch_digest_pipe(const KParams& p, const uint8_t* disp, const uint32_t* hist, const int64_t* counts,
                              const PipeBuffers& bf, int frames, uint64_t* out, hipStream_t s);
hipError_t launch_digest_dense(const KParams& p, const uint8_t* disp, const float* X, const float* Y, const float* Z,
                               int frames, uint64_t* out, hipStream_t s);

}  // namespace svx
