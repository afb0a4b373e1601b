/*
 * svx — MI355X-native disparity -> 3D point-cloud hot path (C ABI).
 *
 * Drop-in boundary for thien/stereo.vision. The reference has no native/FFI
 * API: its boundary is the Python module `functions`, whose attributes
 * stereovision.py resolves at call time (stereovision.py:3, :84-113). The
 * Python binding (stereo.vision_amd/svx/_abi.py, ctypes) binds exactly these
 * symbols and re-exposes the reference's signatures (svx/dropin.py).
 *
 * Conventions
 *   - every entry point returns 0 on success, a negative SV_E* code on error;
 *     sv_last_error() gives a thread-local message. The Python wrapper raises
 *     RuntimeError(message), which lands in the reference's own try/except
 *     (stereovision.py:92-126) exactly like a reference exception would.
 *   - host buffers are allocated by the caller; device buffers are owned by
 *     the library (sv_batch) and stay resident in HBM.
 *   - the "host" entry points (sv_project_frame, sv_backproject,
 *     sv_pipeline_frame) are synchronous: they return after the D2H copy.
 *   - plain pointers and sizes only; no torch / no C++ types.
 */
#ifndef SVX_H
#define SVX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SV_OK 0
#define SV_E_ARG -1     /* bad argument / unsupported shape                */
#define SV_E_HIP -2     /* HIP runtime error                               */
#define SV_E_CAP -3     /* caller's output capacity too small              */
#define SV_E_STATE -4   /* not initialised / wrong object                  */
#define SV_E_COMM -5    /* RCCL error                                      */
#define SV_E_DEVICE -6  /* a kernel reported an internal failure (timeout) */
#define SV_E_RANGE -7   /* input outside the supported value range          */

/* functions.py:15,19,21,22 — focal length (px), baseline (m), image centre. */
typedef struct { double f, B, cw, ch; } sv_camera;
/* Plane a*X + b*Y + c*Z = 1 (functions.py:267, consumed at :300-312). */
typedef struct { double a, b, c; } sv_plane;

/* ---- library / device ------------------------------------------------- */
const char* sv_version(void);
const char* sv_last_error(void);
int sv_device_count(int* n);
int sv_init(int device);                 /* select + warm the device          */

/* ---- drop-in (host buffers, synchronous) -------------------------------- */

/* Replaces functions.py:178-198 projectDisparityTo3d(disparity, max_disparity,
 * rgb=[]). Grid y in range(0,H-1,step) x range(0,W-1,step), raster order,
 * d == 0 skipped, fp64 X,Y,Z bit-identical to the reference arithmetic.
 * bgr may be NULL (the `rgb=[]` case, stereovision.py:85); out_rgb receives
 * (R,G,B) = bgr[...,2], bgr[...,1], bgr[...,0] (functions.py:195).
 * cap = rows available in out_xyz/out_rgb; *out_n = rows written. */
int sv_project_frame(const uint8_t* disp, int H, int W, int64_t ld_disp,
                     const uint8_t* bgr, int64_t ld_bgr, int step, const sv_camera* cam,
                     double* out_xyz, uint8_t* out_rgb, int64_t cap, int64_t* out_n);

/* projectDisparityTo3d's rows as the drop-in returns them (functions.py:178-198, the same points and bits as
 * sv_project_frame): out_rows holds cap rows of `cols` doubles — X, Y, Z (cols 3; bgr may be NULL) or X, Y, Z, R,
 * G, B (cols 6, bgr required) — laid out on the device and copied back in one transfer, a direct DMA when out_rows
 * is page-locked (sv_host_alloc). *out_n = rows written. */
int sv_project_rows(const uint8_t* disp, int H, int W, int64_t ld_disp, const uint8_t* bgr, int64_t ld_bgr,
                    int step, const sv_camera* cam, double* out_rows, int cols, int64_t cap, int64_t* out_n);

/* Page-locked host memory for drop-in outputs (hipHostMalloc / hipHostFree): the Python binding pools these blocks
 * and hands them out as numpy arrays that return to the pool when the last view is gone (svx/_abi.py). */
int sv_host_alloc(int64_t bytes, void** out);
int sv_host_free(void* p);

/* Replaces functions.py:201-209 project3DPointsTo2DImagePoints(points):
 * x = ((X*f)/Z)+cw, y = ((Y*f)/Z)+ch in fp64, bit-identical. xyz rows have
 * stride ld (>= 3) doubles; out_xy is n x 2. */
int sv_backproject(const double* xyz, int64_t n, int64_t ld, const sv_camera* cam, double* out_xy);

/* Fused chain of stereovision.py:84,97-113 for one host frame: projection ->
 * calculatePointErrors (functions.py:300-312) -> computePlanarThreshold
 * (:314-323) -> calculateColourHistogram (:215-226) -> filterPointsByHistogram
 * (:228-230) -> back-projection + int32 trunc (stereovision.py:111-113).
 * out_counts[3] = N_valid, N_kept, N_kept2; out_hist[1024] = hue-bin counts of
 * the plane-kept points (bin k <-> key str(k/1000)); out_xyz (cap x 3, fp32,
 * NULL ok) and out_pts (cap x 2 int32) hold the N_kept2 surviving points in
 * reference order. Any W >= 2 (rows are staged at a stride rounded up to 8). */
int sv_pipeline_frame(const uint8_t* disp, const uint8_t* bgr, int H, int W, int step,
                      const sv_camera* cam, const sv_plane* plane, double point_thr, int hist_thr,
                      int64_t* out_counts, uint32_t* out_hist, float* out_xyz, int32_t* out_pts,
                      int64_t cap);

/* ---- disparity pre-pass, host frames, synchronous ---- */

/* Replaces functions.py:141-148 fillDisparity(disparity, previousDisparity):
 * out = d > 2 ? d : min(255, d + prev) per pixel (cv2.threshold BINARY at 2,
 * bitwise_not, masked copy of prev, saturating cv2.add); prev NULL -> copy. */
int sv_fill_previous(const uint8_t* disp, const uint8_t* prev, int H, int W, uint8_t* out);
/* Replaces functions.py:150-162 fillAltDisparity(disparity), IN PLACE like the
 * reference: pixels < 2 of each row <- trunc(mean of the row's non-zero values). */
int sv_fill_mean(uint8_t* disp, int H, int W);
/* Replaces functions.py:169-172 maskDisparity(disparity) with the caller's
 * carmask (functions.py:35): out = mask != 0 ? d : 0. */
int sv_mask_disparity(const uint8_t* disp, const uint8_t* mask, int H, int W, uint8_t* out);

/* ---- road raster + non-zero walk, host, synchronous -- */

/* Replaces functions.py:339-344 generatePointsAsImage(points): an H x W grey
 * image, 0 except 255 at every [x, y] of pts (n x 2 int32, the planePoints of
 * stereovision.py:112-113). Negative indices wrap like numpy's; a point past
 * [-W, W) x [-H, H) fails with SV_E_ARG (numpy raises IndexError). */
int sv_road_raster(const int32_t* pts, int64_t n, int H, int W, uint8_t* out_img);
/* The pixel walk at the end of functions.py:355-366 (sanitiseRoadImage):
 * out = [j, i] (int32) of every non-zero pixel, raster order. W <= 4096. */
int sv_nonzero_points(const uint8_t* img, int H, int W, int32_t* out, int64_t cap, int64_t* out_n);

/* ---- the stages a2-a6 one by one (the stage drop-ins) ---------------------- */

/* calculatePointErrors (functions.py:300-312): out[i] = |(P_i . abc - 1) / d|
 * in fp64 with P.abc = fma(z, c, fma(x, a, y * b)) (OpenBLAS dgemv's order for
 * (N,3) x (3,1)); abcd = {a, b, c, d}, d as the reference's
 * math.sqrt computes it. xyz: n rows of stride ld >= 3 doubles. */
int sv_point_errors(const double* xyz, int64_t n, int64_t ld, const double* abcd, double* out);
/* BGRtoHSVHue + calculateColourHistogram (functions.py:73-78, :215-226): the
 * hue bin rint(h * 1000) of every (R, G, B) row (stride ld bytes; out_bins
 * nullable), the count of every bin (out_hist[1000]) and the index of its
 * first row (out_first[1000], -1 if empty; the dict's insertion order). */
int sv_hue_histogram(const uint8_t* rgb, int64_t n, int64_t ld, int16_t* out_bins, uint32_t* out_hist,
                     int64_t* out_first);
/* computePlanarThreshold (functions.py:314-323): indices i with vals[i] < thr
 * (NaN never), in order. filterPointsByHistogram (functions.py:228-230): indices
 * i with ok[bins[i]] != 0 (ok[1000] = hist[bin] > threshold), in order. */
int sv_select_less(const double* vals, int64_t n, double thr, int64_t* out_idx, int64_t* out_n);
int sv_select_bins(const int16_t* bins, int64_t n, const uint8_t* ok, int64_t* out_idx, int64_t* out_n);

/* ---- RANSAC plane fit --------------------------------- */

/* The draws of functions.py:278-298 RANSAC(points, trials), replayed exactly
 * as CPython's `random` makes them (MT19937, _randbelow, random.sample's pool
 * and set branches; per trial sample(points, k) then the non-collinear
 * triple of functions.py:240-260), starting from mt_state = random.getstate()'s
 * 624 words + index (advanced in place, for random.setstate). pts: n rows of
 * stride ld >= 3 doubles (X, Y, Z first). Outputs per trial: sidx (k indices),
 * tri (3 indices). *out_trials = trials, or 0 when n < k (sample raises before
 * drawing, so no trial runs and the state is untouched). Host only. */
int sv_ransac_draw(uint32_t* mt_state, const double* pts, int64_t n, int64_t ld, int trials, int k, int32_t* sidx,
                   int32_t* tri, int* out_trials);
/* sv_ransac_draw, then every trial on the GPU: out_abc (trials x 3) =
 * inv([P1;P2;P3]) 1 (functions.py:267), out_err = mean |P.abc - 1| / |abc| over
 * the trial's sample (functions.py:269-275, :289), out_flag = 0 ok, 1 singular,
 * 2 ill-conditioned (the caller re-decides flagged trials and the near-best
 * ones with the reference's own numpy calls). */
int sv_ransac(uint32_t* mt_state, const double* pts, int64_t n, int64_t ld, int trials, int k, int32_t* sidx,
              int32_t* tri, double* out_abc, double* out_err, uint8_t* out_flag, int* out_trials);

/* ---- disparity stage, host images, synchronous ------ */

/* cv2.StereoSGBM_create(minDisparity, numDisparities, blockSize, P1, P2,
 * disp12MaxDiff, preFilterCap, uniquenessRatio) — functions.py:26 creates it
 * as (0, 128, 21) with the other fields 0. OpenCV's substitutions for zero
 * fields are applied (P1 -> 2, P2 -> max(5, P1 + 1), preFilterCap ->
 * max(cap, 15) | 1, disp12MaxDiff -> 1, uniquenessRatio < 0 -> 10); mode is
 * MODE_SGBM, speckleWindowSize 0. Supported: min_disp 0, num_disp 128, odd
 * block <= 63, 128 + block/2 < W <= 2048. */
typedef struct {
    int min_disp, num_disp, block, P1, P2, disp12_max_diff, prefilter_cap, uniqueness;
} sv_sgbm_params;

/* cv2.LUT(image, table) of gammaChange (functions.py:61-67): out[i] = lut[in[i]]
 * over n bytes (any channel count; the table is built by the caller, as the
 * reference builds it in numpy). */
int sv_lut_u8(const uint8_t* in, int64_t n, const uint8_t* lut, uint8_t* out);
/* One image of greyscale (functions.py:89-97): cv2.cvtColor(BGR2GRAY)
 * (fixed point, (B*1868 + G*9617 + R*4899 + 2^13) >> 14) then
 * cv2.equalizeHist. bgr: H x W x 3 contiguous. */
int sv_grey_equalize(const uint8_t* bgr, int H, int W, uint8_t* out);
/* stereoProcessor.compute(grayL, grayR) (functions.py:108): H x W int16
 * disparity x16, -16 where invalid — computeDisparitySGBM followed, as in
 * OpenCV's StereoSGBM::compute, by medianBlur(disp, disp, 3) (exact 3 x 3
 * median, replicated border). SV_E_RANGE when a path cost leaves int16
 * (block cost sums above 32,763; OpenCV's int16 buffers would truncate). */
int sv_sgbm_compute(const uint8_t* L, const uint8_t* R, int H, int W, const sv_sgbm_params* prm, int16_t* out);
/* cv2.filterSpeckles(img, newVal, maxSpeckleSize, maxDiff) on int16, in place
 * (functions.py:111): 4-connected regions of pixels != newVal joined where
 * neighbours differ by <= maxDiff; regions of <= maxSpeckleSize pixels are set
 * to newVal. */
int sv_filter_speckles(int16_t* img, int H, int W, int new_val, int max_size, int max_diff);
/* functions.py:104-128 disparity(grayL, grayR, max_disparity, crop_disparity):
 * SGBM -> filterSpeckles(0, 4000, max_disparity - 5) -> threshold TOZERO at 0
 * -> (d / 16.).astype(uint8) -> crop [0:390, 135:W] when crop != 0 ->
 * (x * (256. / max_disparity)).astype(uint8). out: rows x cols u8 with rows =
 * crop ? min(390, H) : H, cols = crop ? W - 135 : W. raw16 / filt16 (nullable,
 * H x W): the compute() result (after its medianBlur) before / after
 * filterSpeckles. */
int sv_disparity(const uint8_t* L, const uint8_t* R, int H, int W, const sv_sgbm_params* prm, int max_disparity,
                 int crop, uint8_t* out, int16_t* raw16, int16_t* filt16);

/* ---- batched, device-resident API ------------- */
typedef struct sv_batch sv_batch;

/* frames x H x W uint8 disparity (+ frames x H x W x 3 BGR if with_bgr) in
 * HBM. Any W >= 2: rows are stored at a stride of round_up(W, 8) bytes (the
 * pad columns lie outside every grid; uploads and read-backs use W), so the
 * 390 x 889 frames of crop_disparity=True (functions.py:122-124) run fused;
 * sv_batch_synth / the batched SGBM need W % 8 == 0. Dense outputs: 3 fp32 planes (X, Y, Z) of
 * frames x Hg x pitch, pitch = round_up(Wg, 4); Z == 0 marks d == 0 / pad. */
int sv_batch_create(int device, int frames, int H, int W, int step, int with_bgr,
                    int with_points, sv_batch** out);
int sv_batch_destroy(sv_batch* b);
int sv_batch_info(const sv_batch* b, int64_t* out8); /* Hg, Wg, pitch, Ng, bytes, frames, H, W */
/* K1 launch shape: qpl = quads (4 grid points) per lane, 1, 2 or 4 (0 = 1);
 * nontemporal = 1 for non-temporal (streaming) stores, 2 for the same kernel
 * (qpl 1, non-temporal) as a separately named instance: a profiler keeps its
 * launches in a statistics row of their own. */
int sv_batch_tune(sv_batch* b, int qpl, int nontemporal);

/* Counter-based synthetic frames for global frame ids first..first+frames-1
 * (SURVEY §8d), generated on the device: inputs never cross PCIe. */
int sv_batch_synth(sv_batch* b, int64_t first_frame_id);
/* Upload one host frame (tests / real data). bgr may be NULL. */
int sv_batch_upload(sv_batch* b, int frame, const uint8_t* disp, const uint8_t* bgr);

/* K1: dense projection of every frame (configs 2/3). Asynchronous on the
 * batch stream unless sync != 0. */
int sv_batch_project(sv_batch* b, const sv_camera* cam, int sync);

/* K2+K3: plane threshold + hue histogram + stable compaction + int32
 * back-projection for every frame (config 4). chunk = frames per
 * histogram/compaction wave (0 = library default). */
int sv_batch_pipeline(sv_batch* b, const sv_camera* cam, const sv_plane* plane,
                      double point_thr, int hist_thr, int chunk, int sync);

/* The pipeline with every frame's own plane: the plane the last
 * sv_batch_ransac found for it (stereovision.py:94-113 per frame). A frame
 * without a plane (trial -1: the reference's plane step raises) keeps no
 * points. Same kernel families as sv_batch_pipeline (the frame-resident
 * kernel reads each frame's plane). sv_batch_read_frame_plane: a, b, c and
 * |abc| (-1 without a plane) as the kernels use them. */
int sv_batch_pipeline_planes(sv_batch* b, const sv_camera* cam, double point_thr, int hist_thr, int chunk,
                             int sync);
/* sv_batch_pipeline with the plane in DEVICE memory (3 doubles a, b, c on the
 * batch's device, e.g. the buffer an RCCL broadcast wrote): read by the
 * device, so the call needs no host copy of the plane and no host sync. */
int sv_batch_pipeline_dev(sv_batch* b, const sv_camera* cam, const double* dplane, double point_thr, int hist_thr,
                          int chunk, int sync);
int sv_batch_read_frame_plane(sv_batch* b, int frame, double* out4);

/* Pipeline kernel family: 0 = auto (frame-resident for >= 512 frames when the
 * frame fits, else tiled), 1 = tiled (tiles of 4096 points across workgroups,
 * offsets kernel between the passes), 2 = frame-resident (one workgroup per
 * frame, LDS histogram; frames of <= 1M grid points and <= 2048 grid points a
 * side, else SV_E_ARG; chunks the plane rules out are skipped; both passes
 * prefetch the next chunk; no host sync), 3 = frame-resident without prefetch,
 * 4 = frame-resident with the pass-2 prefetch only. Results are identical;
 * only the speed differs. */
int sv_batch_pipeline_mode(sv_batch* b, int mode);

/* Pre-pass over the batch's frames in order (stereovision.py:53-76): option
 * 1 = fillDisparity with the previous CLEANED frame (frame 0 uses prev0, or is
 * left as is when prev0 is NULL), 2 = fillAltDisparity, 0 = none. The cleaned
 * disparity replaces the batch's; with a mask set (sv_batch_set_mask, the grey
 * carmask, NULL clears it) the masked disparity of functions.py:169-172 is
 * also written (sv_batch_read_disp). capDisparity (functions.py:164-167)
 * returns its input unchanged, so it has no kernel. */
int sv_batch_set_mask(sv_batch* b, const uint8_t* mask);
int sv_batch_prepass(sv_batch* b, int option, const uint8_t* prev0, int sync);
int sv_batch_read_disp(sv_batch* b, int frame, uint8_t* disp, uint8_t* masked);

/* Road images of the pipeline's int32 points (generatePointsAsImage per
 * frame), their raster-order non-zero walks, and read-back (img and/or the
 * walk; n receives the walk's length). sv_batch_road_raster writes the images
 * and their walks in one pass (the walks are then already current and
 * sv_batch_nonzero only orders/syncs); with SVX_ROAD_FUSED=0 (diagnostic
 * build only) it writes the images only and sv_batch_nonzero walks them. */
int sv_batch_road_raster(sv_batch* b, int sync);
int sv_batch_nonzero(sv_batch* b, int sync);
int sv_batch_read_road(sv_batch* b, int frame, uint8_t* img, int32_t* nzpts, int64_t cap, int64_t* n);
/* stereovision.py:131-133 imageRoadMap: with enable != 0, later
 * sv_batch_road_raster calls also write, in the same pass, a copy of each
 * frame's BGR (the corrected imgL the pipeline read its colours from) with
 * [0, 255, 0] at every [x, y] of its int32 planePoints (numpy's negative
 * indices wrap as in the road image). Needs a with_bgr batch. For a batch of
 * crop_disparity=True frames the map covers the batch's H x W (the top-left of
 * the 544 x 1024 imgL; the rest of imgL is unpainted, as the pipeline's points
 * never leave the disparity's own grid). Read-back: H x W x 3 u8. */
int sv_batch_road_map(sv_batch* b, int enable);
/* With enable != 0, later frame-resident pipeline calls on 1024-wide frames at step 1 also write a bitmap of
 * the pixels their int32 points mark (pass 2 marks them as it makes the points; 68 KB a frame), and the next
 * sv_batch_road_raster builds the images, walks and imageRoadMap from it — one wave a row — instead of
 * re-reading the points (8 B each). The outputs are the same either way; other shapes and the tiled kernels
 * keep the points path. */
int sv_batch_road_bits(sv_batch* b, int enable);
int sv_batch_read_road_map(sv_batch* b, int frame, uint8_t* out);

/* Batched RANSAC (stereovision.py:84-94 for every frame):
 * maskpoints = the fp64 step-2 projection of the batch's disparity under the
 * mask set by sv_batch_set_mask (functions.py:169-172, :178-198), then
 * RANSAC(maskpoints, trials) (functions.py:278-298) with the draws CPython
 * makes after random.seed(seed_base + first_frame + frame) — replayed on the
 * device, one workgroup per frame. Per frame: abc (the plane), err (its mean
 * distance), trial (the winning trial, -1 when fewer than k points: the
 * reference returns (None, None)), flags (1: a trial was singular and
 * skipped; 2: unused since round 3; 4: the runner-up's error is within 1e-9
 * relative, information only: planes, errors and the choice are computed with
 * numpy's rounding — LAPACK dgesv + dot, gemv, pairwise mean — so abc, err and
 * trial equal the reference's bit for bit; 8: every triple drawn in 65,536 attempts was collinear
 * — the reference never returns there — trial = -1; 16: more than 2^28
 * draws in one frame, trial = -1; 32: a frame above the launch's size bound,
 * trial = -1 — cannot happen while the bound holds). Step-2 grids of
 * <= 163,840 points, frames up to 4096 x 4096; 1 <= k <= 1024. The kernels'
 * LDS is sized for the largest frame: with a mask set (the reference always
 * masks, stereovision.py:74-85) from the mask's own step-2 points, an upper
 * bound of every frame's count, so the call enqueues everything without a
 * host wait; without a mask (or a mask too large for 8 KiB of sample LDS) it
 * waits for the maskpoints counts (one small read-back). `sync` then applies
 * to the RANSAC kernels. */
int sv_batch_ransac(sv_batch* b, const sv_camera* cam, uint64_t seed_base, int64_t first_frame, int trials, int k,
                    int sync);
int sv_batch_read_ransac(sv_batch* b, int frame, double* abc, double* err, int32_t* trial, uint32_t* flags);
int sv_batch_read_maskpoints(sv_batch* b, int frame, double* xyz, int64_t cap, int64_t* n);
/* Draw-level verification: record the first `trials` trials' drawn indices of
 * every frame in later sv_batch_ransac calls (0 = off); read one frame's as
 * trials x (k + 3) int32 (the sample, then P1..P3 of the accepted triple;
 * -1 where a trial did not run), trials and k being those of the last
 * sv_batch_ransac (*out_trials, *out_k; out NULL: sizes only; cap = int32
 * capacity of out, SV_E_CAP if smaller). */
int sv_batch_ransac_trace(sv_batch* b, int trials);
int sv_batch_read_ransac_trace(sv_batch* b, int frame, int32_t* out, int64_t cap, int* out_trials, int* out_k);

/* Stereo pairs resident in HBM (frames x Hp x Wp grey left / right) and the
 * batched disparity stage: sv_batch_sgbm runs functions.py:104-128 on every
 * pair and writes the batch's disparity (frames x H x W u8), the input of the
 * pre-pass, K1 and the pipeline. The pairs have the batch's shape (no crop)
 * unless sv_batch_pair_shape(b, Hp, Wp) sets the uncropped one: then the batch
 * (H = min(390, Hp), W = Wp - 135) receives disparity_scaled[0:390, 135:Wp],
 * crop_disparity=True (functions.py:122-124). Wp % 8 == 0. chunk = frames per
 * cost-volume chunk (0 = 32; 4 x 125 MB of int16 volumes per 1024 x 544
 * frame). Synchronous per chunk (the int16 range flags are read back).
 * sv_batch_synth_pair: synthetic rectified pairs for global frame ids
 * first.., generated on the device (row y's true disparity is the synthetic
 * road's, halved: clamp(floor(3(y - 200) / 10), 0, 127)). */
int sv_batch_pair_shape(sv_batch* b, int H, int W);
/* The front end of performStereoVision (stereovision.py:44-46) for the batch:
 * BGR stereo pairs (frames x Hp x Wp x 3, the pair shape above) uploaded or
 * generated on the device, then sv_batch_preprocess applies the gamma table
 * `lut` (256 bytes: functions.py:61-67's table for gamma 1.4, built by the
 * caller) to both images in place (preProcessImages, :81-87), writes
 * BGR2GRAY + equalizeHist of both (greyscale, :89-97) as the SGBM pairs, and,
 * for a batch with BGR, copies the corrected left image's top-left H x W into
 * the batch's BGR (the colours projectDisparityTo3d reads at the disparity's
 * own (y, x), cropped or not). */
int sv_batch_upload_bgr_pair(sv_batch* b, int frame, const uint8_t* L, const uint8_t* R);
int sv_batch_synth_bgr_pair(sv_batch* b, int64_t first_frame_id);
int sv_batch_preprocess(sv_batch* b, const uint8_t* lut, int sync);
int sv_batch_synth_pair(sv_batch* b, int64_t first_frame_id);
int sv_batch_upload_pair(sv_batch* b, int frame, const uint8_t* L, const uint8_t* R);
int sv_batch_sgbm(sv_batch* b, const sv_sgbm_params* prm, int max_disparity, int chunk);

int sv_batch_sync(sv_batch* b);
/* ms of the last sv_batch_project / sv_batch_pipeline / sv_batch_sgbm, from
 * HIP events recorded on the batch stream around the kernels. which: 0 =
 * project, 1 = pipeline, 2 = sgbm. */
int sv_batch_last_ms(sv_batch* b, int which, float* ms);
/* Sum of the per-launch durations (HIP events on the batch stream around each
 * K1 launch / each pipeline call) since the last reset, and their count.
 * Synchronises the batch stream. */
int sv_batch_timing(sv_batch* b, int which, double* total_ms, int64_t* count);
int sv_batch_timing_reset(sv_batch* b);
/* The placement probe of a large batch's first call (which: 0 = K1's X/Y/Z planes, k1_place; 1 = the resident
 * pipeline's four output planes (X, Y, Z and the packed planePoints word), pipe_place; 2 = the SGBM cost volumes, sgbm_place): up to 3 (SGBM: 2) sets are
 * allocated and one call is timed on each (the pipeline: the faster of two passes; SGBM: the first chunk's
 * compute, the second of two runs); the fastest set is kept. ms[0..n-1] = each set's timed call, *kept = the
 * kept set's index (-1 when no probe ran: small batch or chunk, too little free memory). */
int sv_batch_placement(sv_batch* b, int which, float* ms, int cap, int* n, int* kept);
/* The kernel instance the last sv_batch_project (which 0) / sv_batch_pipeline* (1) call launched, as rocprofv3
 * names it (e.g. "svx::resident_fused_kernel<1, 4, true, true, true, false>"; the tiled pipeline's two kernels;
 * 2: "sgbm stage"), NUL-terminated into buf[cap]: a PMC profile of that name is the timed kernel's. SV_E_STATE
 * before the first call. */
int sv_batch_kernel_name(sv_batch* b, int which, char* buf, int cap);
/* sha256 (16 hex) of the sources this library's K1 (which 0: kernels/project.hip + the device headers) or resident
 * pipeline (1: kernels/resident.hip, kernels/tables.hip + the device headers) was compiled from, fixed at build time:
 * a PMC profile records it, and a profile counts for the timed kernel only when the ids agree. */
int sv_source_id(int which, char* buf, int cap);

/* Read back. */
int sv_batch_read_dense(sv_batch* b, int frame, float* X, float* Y, float* Z);
int sv_batch_read_counts(sv_batch* b, int64_t* counts /* frames x 3 */);
int sv_batch_read_hist(sv_batch* b, int frame, uint32_t* hist /* 1024 */);
int sv_batch_read_points(sv_batch* b, int frame, float* xyz, int32_t* pts, int64_t cap, int64_t* n);

/* ---- software-pipelined frame loop (stereovision.py:53-136, minus the cv2 drawing) -------------- */
/* The reference's per-frame loop (loop.py:59-78 -> performStereoVision) over a SEQUENCE of device batches:
 * every batch goes through input -> pre-pass (functions.py:130-172) -> maskpoints (stereovision.py:74-85) ->
 * RANSAC (functions.py:278-298, stereovision.py:94) -> the pipeline with each frame's own plane
 * (stereovision.py:97-113) -> road raster + non-zero walk (+ imageRoadMap) (stereovision.py:131-156,
 * functions.py:339-365), on its slot's stream; RANSAC runs as two stages (the draw replay, the evaluation).
 * Each stage of batch k also waits for the same stage of batch k - 1, and the evaluation for batch k - 1's
 * road pass, so with slots = 2 the draw of batch k + 1 (one wave's dependent chain per frame) runs beside the
 * HBM-bound pipeline and road pass of batch k, and the evaluation of batch k + 1 (a CU's LDS per frame)
 * beside the pre-pass and maskpoints of batch k + 2. fillDisparity's previous cleaned frame is carried from batch to
 * batch, so the results equal one long batch's (frame g draws after random.seed(seed_base + g)). */
typedef struct {
    int frames;          /* frames per batch                                                          */
    int H, W, step;      /* frame shape; pipeline grid step (1, or the reference's 2)                  */
    int slots;           /* batches in flight (1..8; 2 = the software pipeline)                        */
    int source;          /* 0: the caller fills each batch (sv_loop_acquire + sv_batch_upload / sv_batch_sgbm);
                            1: synthetic frames of the batch's global ids, generated on the device      */
    int prepass;         /* 0 none, 1 fillDisparity with the previous cleaned frame, 2 fillAltDisparity */
    int trials, k;       /* RANSAC trials and sample size (600, 600)                                    */
    uint64_t seed_base;  /* frame g draws what CPython draws after random.seed(seed_base + g)           */
    double point_thr;    /* computePlanarThreshold threshold (0.05)                                    */
    int hist_thr;        /* filterPointsByHistogram threshold (10)                                     */
    int road;            /* 0 none, 1 road raster + walk, 2 + imageRoadMap                             */
} sv_loop_params;
typedef struct sv_loop sv_loop;
/* carmask: the grey H x W mask of maskDisparity (functions.py:35, :169-172), NULL for none. */
int sv_loop_create(int device, const sv_loop_params* prm, const sv_camera* cam, const uint8_t* carmask,
                   sv_loop** out);
int sv_loop_destroy(sv_loop* L);
/* The batch the next sv_loop_submit runs (waits on the host until its slot's previous batch is done): with
 * source 0 the caller uploads its frames (or runs sv_batch_sgbm on it) before submitting. */
int sv_loop_acquire(sv_loop* L, sv_batch** out);
/* Enqueue one batch (global frame ids first_frame_id..) through every stage; returns its sequence number. With a
 * carmask the host waits for nothing (the mask's step-2 points bound every frame's maskpoints count and size the
 * RANSAC launches); without one it waits for this batch's maskpoint counts, whose copy is enqueued on the slot's
 * stream behind the slot's earlier work (with two slots: batch k - 2's pipeline and road pass, and batch k - 1's
 * pre-pass). Batch k's own pipeline and road pass are enqueued by the next submit (or by sv_loop_wait / _batch /
 * _timeline). */
int sv_loop_submit(sv_loop* L, int64_t first_frame_id, int64_t* out_seq);
/* Wait for batch seq's last stage. sv_loop_batch: the batch holding seq's results (sv_batch_read_* work on it)
 * until batch seq + slots is acquired or submitted; it enqueues seq's pending stages and waits for them first. sv_loop_timeline: the start and end of each of the seven
 * stages (input, pre-pass, maskpoints, RANSAC draw, RANSAC evaluation, pipeline, road) in ms since the loop's
 * first submit, 14 doubles. */
int sv_loop_wait(sv_loop* L, int64_t seq);
int sv_loop_batch(sv_loop* L, int64_t seq, sv_batch** out, int64_t* first_frame_id);
int sv_loop_timeline(sv_loop* L, int64_t seq, double* out);

/* ---- verification helpers (device computes, host compares) -------------- */
/* Per-frame verification digests of the batch's current outputs (test and
 * bench support, not timed): which = 0 checks the K1 dense planes, 1 the
 * pipeline outputs. out = frames x 8 uint64: n_valid, n_kept, n_kept2,
 * disp_hash, hist_hash, pts_hash, bad, 0 — the definitions of
 * oracle/svx_oracle.c svo_frame_digest, recomputed on the device from the
 * outputs (kernels/digest.hip); `bad` counts outputs outside 1e-5 relative of
 * the fp64 reference values or inconsistent with the disparity. Synchronous. */
int sv_batch_digest(sv_batch* b, const sv_camera* cam, int which, uint64_t* out);


/* Hue bin of all 2^24 colours, index R<<16|G<<8|B (for exhaustive tests):
 * sv_hue_lut the exact device function (stage kernels, tiled pipeline);
 * sv_hue_lut_variant 0 the same, 1 the resident pipeline's fp32 path
 * (hue_bin_sel: rcp + rint, the exact path in the tie band). */
int sv_hue_lut(int device, int16_t* out_lut);
int sv_hue_lut_variant(int device, int variant, int16_t* out_lut);
/* Back-projection delta tables as computed on the device: dx[d][x], dy[d][y]. */
int sv_delta_tables(int device, int H, int W, const sv_camera* cam, int8_t* dx, int8_t* dy);
/* Regenerate one synthetic frame on the device and copy it back. */
int sv_synth_frame(int device, int64_t frame_id, int H, int W, uint8_t* disp, uint8_t* bgr);

/* ---- image I/O (host only): PNG ingest of the stereo pairs and masks ---------
 * Replaces cv2.imread at functions.py:29-34 (the masks) and :52-55 (loadImages)
 * for 8-bit non-interlaced PNGs; svx.io.imread inflates the IDAT stream (zlib) and
 * this undoes the scanline filters: `in` holds H rows of 1 filter byte + rowbytes,
 * `out` H x rowbytes; bpp = bytes a pixel (the filters' left neighbour). SV_E_ARG
 * on a filter type above 4 (a corrupt stream). No device work. */
int sv_png_unfilter(const uint8_t* in, int H, int rowbytes, int bpp, uint8_t* out);

/* ---- stage drop-ins: host-side row gathers (no device work) ---------------
 * The one-by-one drop-ins of stereovision.py:97-113 hold their points as an index
 * selection of projectDisparityTo3d's (N, ld) float64 rows (svx/points.py); these
 * gather the columns a stage uploads from rows[0..nrows); idx NULL = rows 0..n-1;
 * an index outside [0, nrows) is SV_E_ARG (nothing read).
 * sv_gather_rgb_u8: columns 3..5 (R, G, B) as uint8, n x 3; SV_E_ARG if a value is
 *   not an integer in [0, 255] (the colour stages' input check, svx/stages.py).
 *   Replaces the row conversion inside calculateColourHistogram /
 *   filterPointsByHistogram (functions.py:215-230).
 * sv_gather_f64: columns c0..c0+nc-1, n x nc (project3DPointsTo2DImagePoints'
 *   X, Y, Z, functions.py:201-209). */
int sv_gather_rgb_u8(const double* rows, int64_t nrows, int64_t ld, const int64_t* idx, int64_t n, uint8_t* out);
int sv_gather_f64(const double* rows, int64_t nrows, int64_t ld, const int64_t* idx, int64_t n, int c0, int nc,
                  double* out);

/* ---- multi-GPU: RCCL over xGMI ----------------------------- */
/* Frames shard by contiguous global-id ranges (one sv_batch per GPU); the only
 * device-data collective is the broadcast of the plane. Two drivers:
 *   one process per GPU: rank 0's sv_comm_unique_id, handed to every rank
 *     (svx/control.py), then sv_comm_init on each rank;
 *   one process, every GPU: sv_comm_init_all, then
 *     sv_multi_pipeline (or sv_comm_group_start / .._end around the per-device
 *     sv_comm_broadcast_plane_dev calls). */
typedef struct sv_comm sv_comm;
#define SV_UNIQUE_ID_BYTES 128
int sv_comm_unique_id(uint8_t* out_id /* SV_UNIQUE_ID_BYTES */);
int sv_comm_init(int nranks, int rank, const uint8_t* id, int device, sv_comm** out);
/* ncclCommInitAll over devices[0..n-1] (rank i on devices[i]); out[n]. */
int sv_comm_init_all(int n, const int* devices, sv_comm** out);
int sv_comm_destroy(sv_comm* c);
/* ncclGroupStart / ncclGroupEnd (one process issuing the collectives of several devices). */
int sv_comm_group_start(void);
int sv_comm_group_end(void);
/* Broadcast the plane coefficients from root over RCCL and back to the host
 * (synchronous; reporting and tests). */
int sv_comm_broadcast_plane(sv_comm* c, sv_plane* inout, int root);
/* Broadcast the plane from root into device memory, ordered on batch b's
 * stream (b on the comm's device): the root passes its host plane, the other
 * ranks NULL. *out_dplane = batch b's own device slot (3 doubles a, b, c;
 * one per batch, so batches in flight on other streams and the comm's
 * synchronous calls never overwrite it), valid for stream-ordered use on b's
 * stream (sv_batch_pipeline_dev) until b's next broadcast. No host
 * sync. Inside a group, the broadcast is enqueued at sv_comm_group_end: enqueue
 * the pipelines after it. */
int sv_comm_broadcast_plane_dev(sv_comm* c, sv_batch* b, const sv_plane* plane, int root, const double** out_dplane);
/* One process, n GPUs (SURVEY §8b sv_multi_pipeline): one grouped broadcast
 * of the root's plane to every device, then sv_batch_pipeline_dev on every
 * batches[i] (comms[i]'s device) with that device's copy of the plane.
 * Asynchronous unless sync != 0 (then every batch is synchronised). */
int sv_multi_pipeline(int n, sv_comm* const* comms, sv_batch* const* batches, const sv_camera* cam,
                      const sv_plane* plane, int root, double point_thr, int hist_thr, int sync);
/* Sum int64 counters over ranks (reporting only; host buffers, synchronous). */
int sv_comm_allreduce_i64(sv_comm* c, int64_t* inout, int n);

#ifdef __cplusplus
}
#endif
#endif /* SVX_H */
