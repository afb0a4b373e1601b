// svx runtime: device/stream management, buffers, tables and the C ABI
// declared in include/svx.h. Host-side C++ compiled by hipcc; every compute
// step is a hand-written gfx950 kernel (kernels/*.hip). There is no CPU
// compute path: if a kernel cannot run, the call fails with an error.
#include <hip/hip_runtime.h>

#include <array>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/svx.h"
#include "svx_launch.h"
#include "svx_sgbm.h"

using namespace svx;

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(SV_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                              \
    } while (0)

// ---------------------------------------------------------------------------
// per-device state
// ---------------------------------------------------------------------------
namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    // contiguous: physically contiguous pages (hipDeviceMallocContiguous, falling back to hipMalloc). With
    // hipMalloc's pages, where K1's planes land decides how its three store streams spread over the HBM
    // channels: K1 took 4.35-5.0 ms from one allocation to the next, 4.23-4.34 ms contiguous.
    // SVX_CONTIG: 0 = never, 2 = every large buffer (A/B).
    // exact: no 1/4 growth slack (the SGBM volumes, 16 GB each at 128 frames, whose size follows the chunk)
    hipError_t ensure(size_t n, bool contiguous = false, int tag = 0, bool exact = false) {
        if (n <= bytes) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        size_t want = n < 4096 ? 4096 : exact ? n : n + n / 4;
        hipError_t e = hipErrorUnknown;
        static const int mode = [] {
            const char* v = svx_knob("SVX_CONTIG");
            return v && *v ? std::atoi(v) : 1;
        }();
        // A/B: SVX_CONTIG bit 4 also the pipeline outputs (tag 4), 8 the inputs (tag 8), 16 the masks (tag 16)
        if (mode != 0 && (contiguous || mode == 2 || (mode & tag)) && want >= (256u << 20)) {
            e = hipExtMallocWithFlags(&p, want, hipDeviceMallocContiguous);
            if (svx_knob("SVX_CONTIG_LOG"))
                std::fprintf(stderr, "svx: contiguous %zu bytes: %s\n", want, hipGetErrorString(e));
            if (e != hipSuccess) {
                (void)hipGetLastError();
                p = nullptr;
            }
        }
        if (e != hipSuccess) e = hipMalloc(&p, want);
        if (e == hipSuccess) bytes = want;
        return e;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

// SGBM scratch for a chunk of frames (kernels/sgbm.hip): four int16 cost
// volumes, the int16 disparity, union-find parents / sizes, overflow flags.
struct SgbmBufs {
    DevBuf vol[4], raw, d16, par, size, flags;
    int frames = 0;
    bool placed = false;   // the volumes came from sgbm_place (re-placed when they have to grow)
    hipError_t ensure_rest(const SgbmK& k, int n) {   // the per-pixel scratch (the volumes: sgbm_place)
        const size_t px = (size_t)k.frame_px * n;
        hipError_t e = raw.ensure(px * sizeof(int16_t));
        if (e == hipSuccess) e = d16.ensure(px * sizeof(int16_t));
        if (e == hipSuccess) e = par.ensure(px * sizeof(int32_t));
        if (e == hipSuccess) e = size.ensure(px * sizeof(int32_t));
        if (e == hipSuccess) e = flags.ensure(sizeof(uint32_t) * n);
        return e;
    }
    hipError_t ensure(const SgbmK& k, int n) {
        const size_t vb = sgbm_volume_bytes(k) * n, px = (size_t)k.frame_px * n;
        hipError_t e = hipSuccess;
        // the cost volumes physically contiguous: 32.37 vs 33.09 ms per 128 frames over five alternating
        // processes with every large buffer contiguous (profiles/r04/ab_sgbm_contig.txt); the walks stream them
        // (sgbm_place allocates them first for a large chunk and keeps the faster of two sets)
        for (int i = 0; i < 4 && e == hipSuccess; ++i) e = vol[i].ensure(vb, true, 0, true);
        if (e == hipSuccess) e = raw.ensure(px * sizeof(int16_t));
        if (e == hipSuccess) e = d16.ensure(px * sizeof(int16_t));
        if (e == hipSuccess) e = par.ensure(px * sizeof(int32_t));
        if (e == hipSuccess) e = size.ensure(px * sizeof(int32_t));
        if (e == hipSuccess) e = flags.ensure(sizeof(uint32_t) * n);
        if (e == hipSuccess) frames = n;
        return e;
    }
    size_t held_bytes() const {
        size_t n = 0;
        for (const DevBuf* x : {&vol[0], &vol[1], &vol[2], &vol[3], &raw, &d16, &par, &size}) n += x->bytes;
        return n;
    }
    SgbmScratch scratch() const {
        return SgbmScratch{vol[0].as<uint32_t>(), vol[1].as<uint32_t>(), vol[2].as<uint32_t>(), vol[3].as<uint32_t>(),
                           raw.as<int16_t>(), d16.as<int16_t>(), par.as<int32_t>(), size.as<int32_t>(),
                           flags.as<uint32_t>()};
    }
    void release() {
        for (DevBuf* x : {&vol[0], &vol[1], &vol[2], &vol[3], &raw, &d16, &par, &size, &flags}) {
            if (x->p) (void)hipFree(x->p);
            x->p = nullptr;
            x->bytes = 0;
        }
    }
};

struct Tables {
    bool valid = false;
    int H = 0, W = 0;
    sv_camera cam{};
    DevBuf dx, dy;
    DevBuf dxT, dyT;   // transposed (launch_delta_transpose): the resident pipeline's lane-contiguous delta stage
};

struct Device {
    bool init = false;
    hipStream_t stream = nullptr;
    std::mutex mu;
    // drop-in scratch
    DevBuf disp, bgr, xyz, rgb, ctrl, xy, aux, aux2;
    DevBuf sg_l, sg_r, sg_out, sg_filt, sg_hist;   // host-frame SGBM / grey drop-ins
    SgbmBufs sg;
    Tables tables;
    sv_batch* frame_batch = nullptr;  // cached 1-frame batch for sv_pipeline_frame
};

constexpr int kMaxDev = 64;
// auto mode: one workgroup per frame needs enough frames to fill 256 CUs
constexpr int kResidentMinFrames = 512;
Device g_dev[kMaxDev];
std::mutex g_init_mu;

bool same_cam(const sv_camera& a, const sv_camera& b) {
    return a.f == b.f && a.B == b.B && a.cw == b.cw && a.ch == b.ch;
}

int grid_len(int n, int step) { return n > 1 ? (n - 1 + step - 1) / step : 0; }

// W: the row stride of the frames in memory; Wu: the frame's own width (the
// grid range(0, Wu-1, step) of functions.py:185-186), 0 = W. A batch of any
// width stores its rows at a stride rounded up to 8 bytes (aligned quad loads).
KParams make_params(int H, int W, int step, const sv_camera& cam, int Wu = 0) {
    KParams p;
    std::memset(&p, 0, sizeof p);
    p.H = H;
    p.W = W;
    p.step = step;
    p.Hg = grid_len(H, step);
    p.Wg = grid_len(Wu > 0 ? Wu : W, step);
    p.pitch = (p.Wg + 3) / 4 * 4;
    p.Q = p.pitch / 4;
    p.frame_quads = p.Hg * p.Q;
    p.Q_m40 = p.Q > 0 ? (((uint64_t)1 << 40) + (uint64_t)p.Q - 1) / (uint64_t)p.Q : 0;
    p.frame_px = (int64_t)H * W;
    p.f = cam.f;
    p.B = cam.B;
    p.cw = cam.cw;
    p.ch = cam.ch;
    p.fB = cam.f * cam.B;  // functions.py:191 evaluates f*B in fp64
    p.fB32 = (float)p.fB;
    p.B32 = (float)cam.B;
    p.cw_hi = (float)cam.cw;
    p.cw_lo = (float)(cam.cw - (double)p.cw_hi);
    p.ch_hi = (float)cam.ch;
    p.ch_lo = (float)(cam.ch - (double)p.ch_hi);
    p.dx_words = (W + 31) / 32;
    p.dy_words = (H + 31) / 32;
    return p;
}

void set_plane(KParams& p, const sv_plane& pl, double thr, int hist_thr) {
    p.thr = thr;
    p.thr32 = (float)thr;
    FramePlane fp;
    plane_fields(fp, pl.a, pl.b, pl.c, p.f, p.B, p.cw, p.ch, thr, p.W, p.H);
    apply_plane(p, fp);
    p.hist_thr = hist_thr;
    // Diagnostic ablation for profiling only (documented in DESIGN.md): when set,
    // kernels skip parts of their work and the results are NOT valid.
    const char* ab = svx_knob("SVX_ABLATE");
    p.ablate = ab ? std::atoi(ab) : 0;
}

int dev_get(int device, Device** out) {
    if (device < 0 || device >= kMaxDev) return fail(SV_E_ARG, "device %d out of range", device);
    Device& d = g_dev[device];
    std::lock_guard<std::mutex> lk(g_init_mu);
    if (!d.init) {
        int n = 0;
        HIP_TRY(hipGetDeviceCount(&n));
        if (device >= n) return fail(SV_E_ARG, "device %d not present (%d visible)", device, n);
        HIP_TRY(hipSetDevice(device));
        HIP_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
        d.init = true;
    }
    HIP_TRY(hipSetDevice(device));
    *out = &d;
    return SV_OK;
}

int current_device(int* dev) {
    HIP_TRY(hipGetDevice(dev));
    return SV_OK;
}

// Delta tables for (H, W, camera), built on the device in fp64 (tables.hip).
int ensure_tables(Device& d, int H, int W, const sv_camera& cam, hipStream_t s) {
    Tables& t = d.tables;
    if (t.valid && t.H == H && t.W == W && same_cam(t.cam, cam)) return SV_OK;
    KParams p = make_params(H, W, 1, cam);
    HIP_TRY(t.dx.ensure(sizeof(uint32_t) * 256 * p.dx_words));
    HIP_TRY(t.dy.ensure(sizeof(uint32_t) * 256 * p.dy_words));
    HIP_TRY(launch_delta_tables(p, t.dx.as<uint32_t>(), t.dy.as<uint32_t>(), nullptr, nullptr, s));
    HIP_TRY(t.dxT.ensure(sizeof(uint32_t) * 8 * 32 * p.dx_words));
    HIP_TRY(t.dyT.ensure(sizeof(uint32_t) * 8 * 32 * p.dy_words));
    HIP_TRY(launch_delta_transpose(p, t.dx.as<uint32_t>(), t.dy.as<uint32_t>(), t.dxT.as<uint32_t>(),
                                   t.dyT.as<uint32_t>(), s));
    HIP_TRY(hipStreamSynchronize(s));
    t.valid = true;
    t.H = H;
    t.W = W;
    t.cam = cam;
    return SV_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// batch object
// ---------------------------------------------------------------------------
struct sv_batch;
static uint8_t* input_disp(sv_batch* b);
struct sv_batch {
    int device = 0;
    int frames = 0, H = 0, W = 0, step = 1;
    int Wu = 0;                // the frames' own width; W = row stride = round_up(Wu, 8)
    bool with_bgr = false;
    KParams kp{};
    int64_t Ng = 0;            // grid points per frame
    size_t cap = 0;            // per-frame point capacity of the pipeline outputs (Ng rounded up to 64)
    int64_t dense_per_frame = 0;
    hipStream_t stream = nullptr;    // K1, pass 1 (stream A)
    hipStream_t stream2 = nullptr;   // tiled pipeline's offsets kernels (stream B), beside the stage launches; made
                                     // on the first tiled call: streams share the device's few hardware queues (4),
                                     // and two streams on one queue run in order, so no stream is made unused
    std::vector<hipEvent_t> sync_ev; // pipeline hand-offs between A and B (timing disabled)
    DevBuf disp, bgr, X, Y, Z, xyz, ctrl, masks;
    DevBuf ppxy;                // the pipeline's planePoints: one pp_pack word (x, y as int16 halves) a point
    DevBuf oxb, oyb, ozb;       // pipeline X, Y, Z: three planes of frames x cap (default; SoA in xyz: A/B)
    bool out_planes = false;
    bool pipe_placed = false;   // the resident pipeline's outputs were placed (pipe_place)
    DevBuf carmask;             // maskDisparity's 0x00/0xFF mask (H x W)
    DevBuf road, nz, nzcount;   // road images (frames x H x W), their non-zero walks (frames x cap x 2)
    bool nz_fresh = false;      // nz holds the walk of the current road images (road_kernel wrote both)
    DevBuf rmap;                // imageRoadMap (stereovision.py:131-133): frames x H x W x 3, on request
    bool road_bits = false;     // the resident pipeline also writes the road bitmap (sv_batch_road_bits)
    bool rbits_fresh = false;   // rbits holds the bitmap of the current pipeline points
    DevBuf rbits, roff;         // the bitmap (frames x H x 32 words); the road pass's per-row walk offsets
    bool want_rmap = false, rmap_fresh = false;
    DevBuf mpts, rres;          // one frame's maskpoints as fp64 (read-back scratch); counts + batched RANSAC results
    DevBuf prev0buf, rdbuf;     // the host prev0 of sv_batch_prepass; sv_batch_read_disp's masked frame (batch-owned:
                                // the device-wide drop-in scratch is used on other streams)
    int64_t* hcnt = nullptr;    // pinned host copy of the maskpoints counts (sized frames), read by the RANSAC launch
    hipEvent_t cnt_ev = nullptr;   // the counts' copy has landed in hcnt
    DevBuf rtab;                // fp64 X / Y / Z tables of the step-2 grid (the last sv_batch_ransac's camera)
    DevBuf mpk;                 // maskpoints packed (frames x mcap words x | y << 12 | d << 24): RANSAC's fp32 screen
    DevBuf rtrace;              // optional: frames x trace_trials x (k + 3) drawn indices
    DevBuf rsidx, rtri;         // batched RANSAC scratch: every trial's sample; trial records + frame status
    DevBuf fplanes;             // per-frame keep1 plane fields (FramePlane) for sv_batch_pipeline_planes
    DevBuf dplane;              // the FramePlane of a device plane (sv_batch_pipeline_dev)
    DevBuf abc;                 // this batch's slot for a broadcast plane (sv_comm_broadcast_plane_dev)
    DevBuf pairL, pairR;        // rectified grey stereo pairs (frames x pairH x pairW each), SGBM input
    int pairH = 0, pairW = 0;   // the pairs' shape: the batch's (H, W), or (Hp, Wp) whose crop is the batch
    DevBuf bgrL, bgrR, glut, ghist;   // BGR stereo pairs (frames x pairH x pairW x 3), gamma table, hist scratch
    SgbmBufs sg;                // SGBM scratch for one chunk of frames
    DevBuf sgflags;             // SGBM range flags, one word per frame of the batch
    int64_t mcap = 0;
    int64_t rmax_n = 0, rmax_pool_n = 0;   // the last RANSAC draw launch's largest frame (they size the eval too)
    int64_t rbound = -1;        // the last prepare's device-side bound of the counts (-1: the counts are read back)
    int trace_trials = 0, trace_k = 0, traced_trials = 0;   // requested; k and trials of the recorded trace
    bool have_mask = false;
    // keep_input (a caller-fed frame loop slot): the frames written by synth / upload / sgbm go to `raw`, and the
    // pre-pass reads them there and writes the cleaned frames to `disp`, so resubmitting the slot cleans the same
    // raw frames again (fillDisparity returns a new array, functions.py:140-147)
    bool keep_input = false;
    DevBuf raw;
    int64_t mask_n2 = 0;        // the mask's points on the step-2 grid (an upper bound of every frame's maskpoints)
    // pipeline control block (one memset per call): hist | counts | err
    uint32_t* hist = nullptr;
    int64_t* counts = nullptr;
    uint32_t* err = nullptr;
    size_t ctrl_bytes = 0;
    hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    float last_ms[3] = {0, 0, 0};
    bool have_ms[3] = {false, false, false};
    int qpl = 1;               // K1 quads per lane (1, 2 or 4)
    int nontemporal = 1;       // K1 store flavour (non-temporal: measured faster)
    int pipe_mode = 0;         // 0 auto, 1 tiled (pipeline.hip), 2 frame-resident (resident.hip, both
                               // passes prefetch the next chunk), 3 same without prefetch, 4 pass-2 prefetch only
    // per-launch timing accumulator: event pairs recorded on the batch stream
    std::vector<hipEvent_t> pool;
    std::vector<std::pair<int, int>> pending[3];  // (start idx, end idx) per op kind: project, pipeline, sgbm
    size_t pool_next = 0;
    // the placement probes of the first K1 / resident pipeline call (k1_place / pipe_place): each set's timed
    // call (ms), how many sets were tried and which one was kept (-1: no probe ran)
    float place_ms[3][8] = {};
    int place_n[3] = {0, 0, 0}, place_kept[3] = {-1, -1, -1};
    // the kernel instance the last timed call of each kind launched (rocprofv3's name; sv_batch_kernel_name)
    const char* kname[3] = {nullptr, nullptr, nullptr};
    bool timing = true;        // record per-launch timing events (off for a frame loop's slots: they run unbounded)
    hipError_t timed_event(int* idx) {
        if (!timing) {
            *idx = -1;
            return hipSuccess;
        }
        if (pool_next == pool.size()) {
            hipEvent_t e;
            hipError_t r = hipEventCreate(&e);
            if (r != hipSuccess) return r;
            pool.push_back(e);
        }
        *idx = (int)pool_next++;
        return hipEventRecord(pool[*idx], stream);
    }
};

// where the batch's frames are written: the raw-input buffer (keep_input) or the disparity the stages read
static uint8_t* input_disp(sv_batch* b) { return b->keep_input ? b->raw.as<uint8_t>() : b->disp.as<uint8_t>(); }


extern "C" {

// The pipeline's fp32 outputs: three planes of frames x cap in separate allocations (frame f's X at
// X + f cap), or, with SVX_PIPE_PLANES=0 (A/B), SoA per frame (X[cap] Y[cap] Z[cap] of frame f at 3 cap f).
// The planes were faster and steadier: 5.94-6.06 vs 5.98-6.23 ms for the pipeline, 6.66-6.87 vs 6.63-7.70
// with per-frame planes (five alternating processes each).
static hipError_t ensure_points(sv_batch* b) {
    const size_t plane = sizeof(float) * b->cap * (size_t)b->frames;
    hipError_t e;
    if (b->out_planes) {
        e = b->oxb.ensure(plane, false, 4);
        if (e == hipSuccess) e = b->oyb.ensure(plane, false, 4);
        if (e == hipSuccess) e = b->ozb.ensure(plane, false, 4);
    } else {
        e = b->xyz.ensure(3 * plane, false, 4);
    }
    if (e == hipSuccess) e = b->ppxy.ensure(plane, false, 4);
    return e;
}

static void point_planes(const sv_batch* b, PipeBuffers& bf) {
    if (b->out_planes) {
        bf.ox = b->oxb.as<float>();
        bf.oy = b->oyb.as<float>();
        bf.oz = b->ozb.as<float>();
        bf.ofs = (int64_t)b->cap;
    } else {
        bf.ox = b->xyz.as<float>();
        bf.oy = bf.ox + b->cap;
        bf.oz = bf.oy + b->cap;
        bf.ofs = 3 * (int64_t)b->cap;
    }
    bf.pxy = b->ppxy.as<uint32_t>();
    bf.cap = (int64_t)b->cap;
}

const char* sv_version(void) { return "svx 0.1.0 (gfx950)"; }

const char* sv_last_error(void) { return g_err.c_str(); }

// internal: lets comm.hip report into the same thread-local error slot
int sv_comm_set_error(const char* msg) {
    g_err = msg ? msg : "";
    return 0;
}

// comm.hip: a batch's device, stream (collectives are ordered on the batch's stream) and its own device slot
// for a broadcast plane (3 doubles), so that two batches — or a comm's other calls — never share the buffer
// a pending pipeline reads the plane from
int sv_batch_stream_internal(sv_batch* b, int* device, hipStream_t* stream, double** abc_slot) {
    if (!b) return SV_E_ARG;
    *device = b->device;
    *stream = b->stream;
    if (abc_slot) {
        if (hipSetDevice(b->device) != hipSuccess || b->abc.ensure(sizeof(double) * 3) != hipSuccess) {
            (void)hipGetLastError();
            return SV_E_HIP;
        }
        *abc_slot = b->abc.as<double>();
    }
    return SV_OK;
}

int sv_device_count(int* n) {
    if (!n) return fail(SV_E_ARG, "null out");
    hipError_t e = hipGetDeviceCount(n);
    if (e != hipSuccess) {
        *n = 0;
        return fail(SV_E_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    return SV_OK;
}

int sv_init(int device) {
    Device* d;
    return dev_get(device, &d);
}

// ---------------------------------------------------------------------------
// drop-in: projectDisparityTo3d (functions.py:178-198)
// ---------------------------------------------------------------------------
// The drop-in projection on the device: the frame (and its colours) up, the compact fp64 kernel, the point count
// back (one sync). On success *n is the count and d's xyz / rgb buffers hold the points; the device mutex is held
// by the caller.
static int project_on_device(Device* d, const uint8_t* disp, int H, int W, int64_t ld_disp, const uint8_t* bgr,
                             int64_t ld_bgr, bool want_rgb, const KParams& p, int64_t* n) {
    hipStream_t s = d->stream;
    const int tiles = project_compact_tiles(p);
    const int64_t ng = (int64_t)p.Hg * p.Wg;
    HIP_TRY(d->disp.ensure((size_t)H * W));
    HIP_TRY(d->xyz.ensure(sizeof(double) * 3 * ng));
    HIP_TRY(d->ctrl.ensure(sizeof(uint64_t) * (tiles + 2)));
    HIP_TRY(hipMemcpy2DAsync(d->disp.p, W, disp, ld_disp, W, H, hipMemcpyHostToDevice, s));
    if (want_rgb) {
        HIP_TRY(d->bgr.ensure((size_t)H * W * 3));
        HIP_TRY(d->rgb.ensure(3 * ng));
        HIP_TRY(hipMemcpy2DAsync(d->bgr.p, 3 * (size_t)W, bgr, ld_bgr, 3 * (size_t)W, H,
                                 hipMemcpyHostToDevice, s));
    }
    uint64_t* status = d->ctrl.as<uint64_t>();
    uint32_t* small = reinterpret_cast<uint32_t*>(status + tiles);  // ticket, count, err
    HIP_TRY(hipMemsetAsync(d->ctrl.p, 0, sizeof(uint64_t) * (tiles + 2), s));
    HIP_TRY(launch_project_compact_f64(p, d->disp.as<uint8_t>(), W, want_rgb ? d->bgr.as<uint8_t>() : nullptr,
                                       3ll * W, d->xyz.as<double>(), want_rgb ? d->rgb.as<uint8_t>() : nullptr,
                                       status, small, small + 1, small + 2, s));
    uint32_t hs[3];
    HIP_TRY(hipMemcpyAsync(hs, small, sizeof hs, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (hs[2]) return fail(SV_E_DEVICE, "projection look-back timed out");
    *n = hs[1];
    return SV_OK;
}

int sv_project_frame(const uint8_t* disp, int H, int W, int64_t ld_disp, const uint8_t* bgr,
                     int64_t ld_bgr, int step, const sv_camera* cam, double* out_xyz, uint8_t* out_rgb,
                     int64_t cap, int64_t* out_n) {
    if (!disp || !cam || !out_n || H < 0 || W < 0 || step < 1 || ld_disp < W)
        return fail(SV_E_ARG, "sv_project_frame: bad arguments (H=%d W=%d step=%d)", H, W, step);
    if (bgr && ld_bgr < 3ll * W) return fail(SV_E_ARG, "sv_project_frame: ld_bgr < 3*W");
    *out_n = 0;
    const KParams p = make_params(H, W, step, *cam);
    if ((int64_t)p.Hg * p.Wg == 0) return SV_OK;
    int dev;
    if (int rc = current_device(&dev)) return rc;
    Device* d;
    if (int rc = dev_get(dev, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    hipStream_t s = d->stream;
    const bool want_rgb = bgr && out_rgb;
    int64_t n = 0;
    if (int rc = project_on_device(d, disp, H, W, ld_disp, bgr, ld_bgr, want_rgb, p, &n)) return rc;
    if (n > cap) return fail(SV_E_CAP, "output capacity %lld < %lld points", (long long)cap, (long long)n);
    if (n) {
        HIP_TRY(hipMemcpyAsync(out_xyz, d->xyz.p, sizeof(double) * 3 * n, hipMemcpyDeviceToHost, s));
        if (want_rgb) HIP_TRY(hipMemcpyAsync(out_rgb, d->rgb.p, 3 * n, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    *out_n = n;
    return SV_OK;
}

int sv_project_rows(const uint8_t* disp, int H, int W, int64_t ld_disp, const uint8_t* bgr, int64_t ld_bgr,
                    int step, const sv_camera* cam, double* out_rows, int cols, int64_t cap, int64_t* out_n) {
    if (!disp || !cam || !out_n || H < 0 || W < 0 || step < 1 || ld_disp < W || (cols != 3 && cols != 6) ||
        (cols == 6 && !bgr))
        return fail(SV_E_ARG, "sv_project_rows: bad arguments (H=%d W=%d step=%d cols=%d)", H, W, step, cols);
    if (bgr && ld_bgr < 3ll * W) return fail(SV_E_ARG, "sv_project_rows: ld_bgr < 3*W");
    *out_n = 0;
    const KParams p = make_params(H, W, step, *cam);
    if ((int64_t)p.Hg * p.Wg == 0) return SV_OK;
    int dev;
    if (int rc = current_device(&dev)) return rc;
    Device* d;
    if (int rc = dev_get(dev, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    hipStream_t s = d->stream;
    int64_t n = 0;
    if (int rc = project_on_device(d, disp, H, W, ld_disp, bgr, ld_bgr, cols == 6, p, &n)) return rc;
    if (n > cap) return fail(SV_E_CAP, "output capacity %lld < %lld points", (long long)cap, (long long)n);
    if (!n) return SV_OK;
    if (!out_rows) return fail(SV_E_ARG, "sv_project_rows: null out_rows");
    const double* src = d->xyz.as<double>();
    if (cols == 6) {
        HIP_TRY(d->aux2.ensure(sizeof(double) * 6 * (size_t)n));
        HIP_TRY(launch_rows6(d->xyz.as<double>(), d->rgb.as<uint8_t>(), n, d->aux2.as<double>(), s));
        src = d->aux2.as<double>();
    }
    HIP_TRY(hipMemcpyAsync(out_rows, src, sizeof(double) * cols * (size_t)n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *out_n = n;
    return SV_OK;
}

int sv_host_alloc(int64_t bytes, void** out) {
    if (!out || bytes <= 0) return fail(SV_E_ARG, "sv_host_alloc: bad arguments");
    *out = nullptr;
    int dev;
    if (int rc = current_device(&dev)) return rc;   // (no GPU: fails like every compute entry point)
    HIP_TRY(hipHostMalloc(out, (size_t)bytes, hipHostMallocDefault));
    return SV_OK;
}

int sv_host_free(void* p) {
    if (p) HIP_TRY(hipHostFree(p));
    return SV_OK;
}

// ---------------------------------------------------------------------------
// drop-in: project3DPointsTo2DImagePoints (functions.py:201-209)
// ---------------------------------------------------------------------------
int sv_backproject(const double* xyz, int64_t n, int64_t ld, const sv_camera* cam, double* out_xy) {
    if (n < 0 || ld < 3 || !cam || (n > 0 && (!xyz || !out_xy)))
        return fail(SV_E_ARG, "sv_backproject: bad arguments");
    if (n == 0) return SV_OK;
    int dev;
    if (int rc = current_device(&dev)) return rc;
    Device* d;
    if (int rc = dev_get(dev, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    hipStream_t s = d->stream;
    HIP_TRY(d->xyz.ensure(sizeof(double) * ld * n));
    HIP_TRY(d->xy.ensure(sizeof(double) * 2 * n));
    HIP_TRY(hipMemcpyAsync(d->xyz.p, xyz, sizeof(double) * ld * n, hipMemcpyHostToDevice, s));
    HIP_TRY(launch_backproject_f64(d->xyz.as<double>(), n, ld, cam->f, cam->cw, cam->ch, d->xy.as<double>(), s));
    HIP_TRY(hipMemcpyAsync(out_xy, d->xy.p, sizeof(double) * 2 * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return SV_OK;
}

// ---------------------------------------------------------------------------
// batch API
// ---------------------------------------------------------------------------
int sv_batch_create(int device, int frames, int H, int W, int step, int with_bgr, int with_points,
                    sv_batch** out) {
    if (!out) return fail(SV_E_ARG, "null out");
    *out = nullptr;
    if (frames < 1 || H < 2 || W < 2 || W > 65536 || (step != 1 && step != 2))
        return fail(SV_E_ARG, "sv_batch_create: need frames>=1, H>=2, 2<=W<=65536, step in {1,2} "
                              "(frames=%d H=%d W=%d step=%d)", frames, H, W, step);
    const int Wu = W;
    W = (W + 7) / 8 * 8;
    Device* d;
    if (int rc = dev_get(device, &d)) return rc;
    sv_batch* b = new sv_batch;
    b->device = device;
    b->frames = frames;
    b->H = H;
    b->W = W;
    b->Wu = Wu;
    b->step = step;
    b->with_bgr = with_bgr != 0;
    sv_camera cam0{1, 1, 0, 0};
    b->kp = make_params(H, W, step, cam0, Wu);
    b->Ng = (int64_t)b->kp.Hg * b->kp.Wg;
    b->cap = ((size_t)b->Ng + 63) / 64 * 64;
    if (const char* e = svx_knob("SVX_CAP_PAD")) b->cap += (size_t)std::atoi(e) / 64 * 64;   // A/B: frame stride
    b->dense_per_frame = (int64_t)b->kp.Hg * b->kp.pitch;
    const size_t px = (size_t)frames * H * W;
    hipError_t e = b->disp.ensure(px, false, 8);
    if (e == hipSuccess && b->with_bgr) e = b->bgr.ensure(px * 3, false, 8);
    b->out_planes = true;   // three planes (A/B: SVX_PIPE_PLANES=0 for SoA per frame)
    if (const char* e2 = svx_knob("SVX_PIPE_PLANES")) b->out_planes = *e2 != '0';
    if (e == hipSuccess && with_points) e = ensure_points(b);
    if (e == hipSuccess) {
        const size_t hist_b = sizeof(uint32_t) * kBins * frames, cnt_b = sizeof(int64_t) * 4 * frames;
        e = b->ctrl.ensure(hist_b + cnt_b + 64);
        if (e == hipSuccess) {
            char* base = b->ctrl.as<char>();
            b->hist = reinterpret_cast<uint32_t*>(base);
            b->counts = reinterpret_cast<int64_t*>(base + hist_b);
            b->err = reinterpret_cast<uint32_t*>(base + hist_b + cnt_b);
            b->ctrl_bytes = hist_b + cnt_b + 64;
            e = hipMemset(b->ctrl.p, 0, b->ctrl_bytes);
        }
    }
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking);
    for (int i = 0; i < 6 && e == hipSuccess; ++i) e = hipEventCreate(&b->ev[i]);
    if (e != hipSuccess) {
        sv_batch_destroy(b);
        return fail(SV_E_HIP, "sv_batch_create: %s", hipGetErrorString(e));
    }
    *out = b;
    return SV_OK;
}

int sv_batch_destroy(sv_batch* b) {
    if (!b) return SV_OK;
    (void)hipSetDevice(b->device);
    if (b->stream) (void)hipStreamSynchronize(b->stream);
    for (DevBuf* x : {&b->disp, &b->bgr, &b->X, &b->Y, &b->Z, &b->oxb, &b->oyb, &b->ozb, &b->xyz, &b->ppxy, &b->ctrl, &b->masks,
                      &b->carmask, &b->road, &b->rmap, &b->nz, &b->nzcount, &b->mpts, &b->mpk, &b->rres, &b->rtab, &b->rtrace, &b->fplanes, &b->dplane, &b->abc,
                      &b->pairL, &b->pairR, &b->rsidx, &b->rtri, &b->bgrL, &b->bgrR,
                      &b->glut, &b->ghist, &b->sgflags, &b->prev0buf, &b->rdbuf, &b->rbits, &b->roff, &b->raw})
        if (x->p) (void)hipFree(x->p);
    if (b->hcnt) (void)hipHostFree(b->hcnt);
    if (b->cnt_ev) (void)hipEventDestroy(b->cnt_ev);
    b->sg.release();
    for (auto& ev : b->ev)
        if (ev) (void)hipEventDestroy(ev);
    for (auto& ev : b->pool) (void)hipEventDestroy(ev);
    for (auto& ev : b->sync_ev) (void)hipEventDestroy(ev);
    if (b->stream2) {
        (void)hipStreamSynchronize(b->stream2);
        (void)hipStreamDestroy(b->stream2);
    }
    if (b->stream) (void)hipStreamDestroy(b->stream);
    delete b;
    return SV_OK;
}

int sv_batch_info(const sv_batch* b, int64_t* o) {
    if (!b || !o) return fail(SV_E_ARG, "null");
    o[0] = b->kp.Hg;
    o[1] = b->kp.Wg;
    o[2] = b->kp.pitch;
    o[3] = b->Ng;
    o[4] = (int64_t)(b->disp.bytes + b->bgr.bytes + b->X.bytes * 3 + b->xyz.bytes + b->oxb.bytes * 3 + b->ppxy.bytes +
                     b->ctrl.bytes);
    o[5] = b->frames;
    o[6] = b->H;
    o[7] = b->Wu;
    return SV_OK;
}

int sv_batch_tune(sv_batch* b, int qpl, int nontemporal) {
    if (!b) return fail(SV_E_ARG, "null batch");
    if (qpl == 0) qpl = 1;
    if (qpl != 1 && qpl != 2 && qpl != 4) return fail(SV_E_ARG, "qpl must be 1, 2 or 4");
    if (nontemporal < 0 || nontemporal > 2) return fail(SV_E_ARG, "nontemporal must be 0, 1 or 2");
    b->qpl = qpl;
    b->nontemporal = nontemporal;
    return SV_OK;
}

int sv_batch_synth(sv_batch* b, int64_t first_frame_id) {
    if (!b) return fail(SV_E_ARG, "null batch");
    if (b->Wu != b->W) return fail(SV_E_ARG, "synthetic frames need W %% 8 == 0 (W=%d)", b->Wu);
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(launch_synth(b->kp, input_disp(b), b->with_bgr ? b->bgr.as<uint8_t>() : nullptr,
                         b->frames, first_frame_id, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    return SV_OK;
}

int sv_batch_upload(sv_batch* b, int frame, const uint8_t* disp, const uint8_t* bgr) {
    if (!b || !disp || frame < 0 || frame >= b->frames) return fail(SV_E_ARG, "sv_batch_upload: bad args");
    if (bgr && !b->with_bgr) return fail(SV_E_ARG, "batch created without bgr");
    HIP_TRY(hipSetDevice(b->device));
    const size_t px = (size_t)b->H * b->W;
    uint8_t* dd = input_disp(b) + px * frame;
    if (b->Wu == b->W) {
        HIP_TRY(hipMemcpyAsync(dd, disp, px, hipMemcpyHostToDevice, b->stream));
    } else {   // rows at the padded stride, pad columns zero (outside every grid)
        HIP_TRY(hipMemcpy2DAsync(dd, b->W, disp, b->Wu, b->Wu, b->H, hipMemcpyHostToDevice, b->stream));
        HIP_TRY(hipMemset2DAsync(dd + b->Wu, b->W, 0, b->W - b->Wu, b->H, b->stream));
    }
    if (bgr)
        HIP_TRY(hipMemcpy2DAsync(b->bgr.as<uint8_t>() + 3 * px * frame, 3 * (size_t)b->W, bgr, 3 * (size_t)b->Wu,
                                 3 * (size_t)b->Wu, b->H, hipMemcpyHostToDevice, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    return SV_OK;
}

// K1's planes, placed. K1 is a pure store stream, and where its three planes land in physical memory moves it
// by 12-15 % (4.22 vs 4.9 ms for 4096 frames, the same code and bytes): hipMalloc's pages vary it
// from allocation to allocation, contiguous planes from box state to box state. So a large batch's first
// projection allocates up to SVX_K1_TRIES (default 3) contiguous sets, times one K1 launch on each (all sets
// held until the end, so each lands elsewhere; at most half the free memory), and keeps the fastest.
static int k1_place(sv_batch* b, const KParams& p, size_t plane) {
    int tries = 3;
    if (const char* e = svx_knob("SVX_K1_TRIES")) tries = std::max(1, std::atoi(e));
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
    const size_t set_b = 3 * (plane + plane / 4);   // DevBuf::ensure's slack
    if (b->frames < 1024 || set_b == 0) tries = 1;
    else tries = (int)std::min<size_t>((size_t)tries, std::max<size_t>(1, free_b / 2 / set_b));
    for (DevBuf* x : {&b->X, &b->Y, &b->Z}) {   // a new size: the old planes go
        if (x->p) (void)hipFree(x->p);
        x->p = nullptr;
        x->bytes = 0;
    }
    std::vector<std::array<DevBuf, 3>> sets((size_t)tries);
    int best = -1;
    float best_ms = 0.f;
    for (int t = 0; t < tries; ++t) {
        auto& c = sets[(size_t)t];
        hipError_t e = hipSuccess;
        for (int k = 0; k < 3 && e == hipSuccess; ++k) e = c[k].ensure(plane, true);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            break;
        }
        if (tries > 1) {
            float ms = 0.f;
            for (int rep = 0; rep < 2 && e == hipSuccess; ++rep) {   // the second launch is timed
                e = hipEventRecord(b->ev[0], b->stream);
                if (e == hipSuccess)
                    e = launch_project_dense(p, b->disp.as<uint8_t>(), c[0].as<float>(), c[1].as<float>(),
                                             c[2].as<float>(), b->frames, b->qpl, b->nontemporal, b->stream);
                if (e == hipSuccess) e = hipEventRecord(b->ev[1], b->stream);
                if (e == hipSuccess) e = hipEventSynchronize(b->ev[1]);
                if (e == hipSuccess) e = hipEventElapsedTime(&ms, b->ev[0], b->ev[1]);
            }
            if (e != hipSuccess) break;
            if (svx_knob("SVX_CONTIG_LOG")) std::fprintf(stderr, "svx: K1 placement %d: %.3f ms\n", t, ms);
            if (t < 8) {
                b->place_ms[0][t] = ms;
                b->place_n[0] = t + 1;
            }
            if (best < 0 || ms < best_ms) {
                best = t;
                best_ms = ms;
            }
        } else {
            best = t;
        }
    }
    int rc = SV_OK;
    if (best < 0) rc = fail(SV_E_HIP, "K1 planes: allocation failed (%zu bytes each)", plane);
    b->place_kept[0] = tries > 1 ? best : -1;
    for (int t = 0; t < (int)sets.size(); ++t) {
        for (int k = 0; k < 3; ++k) {
            DevBuf& x = sets[(size_t)t][k];
            if (t == best) {
                DevBuf& dst = k == 0 ? b->X : k == 1 ? b->Y : b->Z;
                dst = x;
            } else if (x.p) {
                (void)hipFree(x.p);
            }
        }
    }
    return rc;
}

int sv_batch_project(sv_batch* b, const sv_camera* cam, int sync) {
    if (!b || !cam) return fail(SV_E_ARG, "null");
    HIP_TRY(hipSetDevice(b->device));
    const size_t plane = sizeof(float) * (size_t)b->dense_per_frame * b->frames;
    KParams p = make_params(b->H, b->W, b->step, *cam, b->Wu);
    if (b->X.bytes < plane || b->Y.bytes < plane || b->Z.bytes < plane)
        if (int rc = k1_place(b, p, plane)) return rc;
    int t0, t1;
    HIP_TRY(hipEventRecord(b->ev[0], b->stream));
    HIP_TRY(b->timed_event(&t0));
    HIP_TRY(launch_project_dense(p, b->disp.as<uint8_t>(), b->X.as<float>(), b->Y.as<float>(), b->Z.as<float>(),
                                 b->frames, b->qpl, b->nontemporal, b->stream, &b->kname[0]));
    HIP_TRY(b->timed_event(&t1));
    HIP_TRY(hipEventRecord(b->ev[1], b->stream));
    if (t0 >= 0) b->pending[0].push_back({t0, t1});
    b->have_ms[0] = true;
    if (sync) HIP_TRY(hipStreamSynchronize(b->stream));
    return SV_OK;
}

namespace {
struct RansacRes {   // layout of b->rres
    double* abc;
    double* err;
    int32_t* trial;
    uint32_t* flags;
    int64_t* mcount;
};
RansacRes ransac_res(sv_batch* b) {
    RansacRes r;
    const size_t F = (size_t)b->frames;
    r.abc = b->rres.as<double>();
    r.err = r.abc + 3 * F;
    r.mcount = reinterpret_cast<int64_t*>(r.err + F);
    r.trial = reinterpret_cast<int32_t*>(r.mcount + F);
    r.flags = reinterpret_cast<uint32_t*>(r.trial + F);
    return r;
}
}  // namespace

// planes: device planes, frame f uses planes[f * plane_stride] (NULL: the host plane)
// The pipeline's four output planes (X, Y, Z, planePoints), placed like K1's (k1_place): where they land moves the resident pipeline
// by up to 8 % (5.85-5.96 ms, one placement in four 6.36-6.46 ms). On a large batch's first resident call,
// up to two more sets are allocated beside the current one (at most half the free memory), one call is timed
// on each (all held), and the fastest set is kept. SVX_PIPE_TRIES=1 turns it off.
static hipError_t pipe_place(sv_batch* b, const KParams& p, PipeBuffers bf, hipStream_t s) {
    int tries = 3;
    if (const char* e = svx_knob("SVX_PIPE_TRIES")) tries = std::max(1, std::atoi(e));
    const size_t plane = sizeof(float) * b->cap * (size_t)b->frames;
    const size_t set_b = 4 * (plane + plane / 4);
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
    tries = (int)std::min<size_t>((size_t)tries, 1 + free_b / 2 / set_b);
    if (tries <= 1) return hipSuccess;
    std::vector<std::array<DevBuf, 4>> sets((size_t)tries);
    sets[0] = {b->oxb, b->oyb, b->ozb, b->ppxy};
    std::vector<float> set_ms((size_t)tries, 0.f);
    int placed = tries;   // sets allocated
    hipError_t e = hipSuccess;
    // Two passes over the sets, each set's time the faster of its two timed calls: the kernel speeds up over
    // its first calls on a cold GPU (clocks; 6.8-7.0 -> 5.8 ms), which a single pass in set order would charge
    // to the first sets.
    for (int pass = 0; pass < 2 && e == hipSuccess; ++pass) {
        for (int t = 0; t < placed && e == hipSuccess; ++t) {
            auto& c = sets[(size_t)t];
            for (int k = 0; k < 4 && e == hipSuccess && t > 0 && pass == 0; ++k) e = c[k].ensure(plane, false, 4);
            if (e != hipSuccess) {   // out of memory: place among the sets held so far
                (void)hipGetLastError();
                for (int k = 0; k < 4; ++k)
                    if (c[k].p) {
                        (void)hipFree(c[k].p);
                        c[k] = DevBuf();
                    }
                e = hipSuccess;
                placed = t;
                break;
            }
            bf.ox = c[0].as<float>();
            bf.oy = c[1].as<float>();
            bf.oz = c[2].as<float>();
            bf.ofs = (int64_t)b->cap;
            bf.pxy = c[3].as<uint32_t>();
            float ms = 0.f;
            for (int rep = pass == 0 ? 0 : 1; rep < 2 && e == hipSuccess; ++rep) {   // the last call is timed
                e = hipEventRecord(b->ev[0], s);
                if (e == hipSuccess) e = launch_pipeline_resident(p, bf, b->frames, true, s, true);
                if (e == hipSuccess) e = hipEventRecord(b->ev[1], s);
                if (e == hipSuccess) e = hipEventSynchronize(b->ev[1]);
                if (e == hipSuccess) e = hipEventElapsedTime(&ms, b->ev[0], b->ev[1]);
            }
            if (e != hipSuccess) break;
            if (svx_knob("SVX_CONTIG_LOG")) std::fprintf(stderr, "svx: pipeline placement %d: %.3f ms\n", t, ms);
            set_ms[(size_t)t] = pass == 0 ? ms : std::min(set_ms[(size_t)t], ms);
        }
    }
    int best = 0;
    for (int t = 1; t < placed; ++t)
        if (set_ms[(size_t)t] < set_ms[(size_t)best]) best = t;
    b->place_n[1] = std::min(placed, 8);
    for (int t = 0; t < b->place_n[1]; ++t) b->place_ms[1][t] = set_ms[(size_t)t];
    b->place_kept[1] = best;
    for (int t = 0; t < (int)sets.size(); ++t)
        for (int k = 0; k < 4; ++k) {
            DevBuf& x = sets[(size_t)t][k];
            if (t == best) {
                DevBuf* dst[4] = {&b->oxb, &b->oyb, &b->ozb, &b->ppxy};
                *dst[k] = x;
            } else if (x.p && (t != 0 || best != 0)) {
                (void)hipFree(x.p);
            }
        }
    return e;
}

static int batch_pipeline_impl(sv_batch* b, const sv_camera* cam, const sv_plane* plane, double point_thr,
                               int hist_thr, int chunk, int sync, Device* d, const FramePlane* planes = nullptr,
                               int plane_stride = 1) {
    if (!b->with_bgr) return fail(SV_E_ARG, "pipeline needs a batch created with bgr");
    KParams p = make_params(b->H, b->W, b->step, *cam, b->Wu);
    if (p.Wg > 4096 || p.Hg > 4096) return fail(SV_E_ARG, "pipeline supports grids up to 4096 x 4096");
    set_plane(p, *plane, point_thr, hist_thr);
    if (chunk <= 0) chunk = 1024;
    if (chunk > b->frames) chunk = b->frames;
    HIP_TRY(ensure_points(b));
    const size_t tiles = (size_t)pipeline_tiles_per_frame(p);
    const size_t kb_bytes = sizeof(uint16_t) * 256 * tiles * b->frames;
    const size_t pres_bytes = sizeof(uint32_t) * (kBins / 32) * tiles * b->frames;
    const size_t tc_bytes = sizeof(uint32_t) * tiles * b->frames;
    HIP_TRY(b->masks.ensure(kb_bytes + pres_bytes + 2 * tc_bytes, false, 16));
    if (int rc = ensure_tables(*d, b->H, b->W, *cam, b->stream)) return rc;
    PipeBuffers bf;
    bf.disp = b->disp.as<uint8_t>();
    bf.bgr = b->bgr.as<uint8_t>();
    bf.hist = b->hist;
    bf.counts = b->counts;
    bf.kbits = b->masks.as<uint16_t>();
    bf.pres = reinterpret_cast<uint32_t*>(b->masks.as<char>() + kb_bytes);
    bf.tcount = reinterpret_cast<uint32_t*>(b->masks.as<char>() + kb_bytes + pres_bytes);
    bf.toff = bf.tcount + tiles * b->frames;
    point_planes(b, bf);
    bf.dxbits = d->tables.dx.as<uint32_t>();
    bf.dybits = d->tables.dy.as<uint32_t>();
    bf.dxT = d->tables.dxT.as<uint32_t>();
    bf.dyT = d->tables.dyT.as<uint32_t>();
    bf.planes = planes;
    bf.plane_stride = plane_stride;
    int mode = b->pipe_mode;
    if (mode == 0) mode = (b->frames >= kResidentMinFrames && resident_supported(p)) ? 2 : 1;
    if (mode >= 2 && !resident_supported(p))
        return fail(SV_E_ARG, "frame-resident pipeline: frame too large (grid %d x %d)", p.Hg, p.Wg);
    if (mode >= 2 && !planes) {   // the host plane, stream-ordered into device memory
        HIP_TRY(b->dplane.ensure(sizeof(FramePlane)));
        FramePlane fp;
        plane_fields(fp, plane->a, plane->b, plane->c, p.f, p.B, p.cw, p.ch, point_thr, p.W, p.H);
        HIP_TRY(launch_store_plane(fp, b->dplane.as<FramePlane>(), b->stream));
        bf.planes = b->dplane.as<FramePlane>();
        bf.plane_stride = 0;
    }
    b->rbits_fresh = false;
    if (mode >= 2 && b->road_bits && resident_road_bits_supported(p)) {   // the road bitmap too (sv_batch_road_bits)
        HIP_TRY(b->rbits.ensure(sizeof(uint32_t) * 32 * (size_t)b->H * b->frames));
        bf.rbits = b->rbits.as<uint32_t>();
        bf.rb_H = b->H;
        bf.rb_Wu = b->Wu;
        b->rbits_fresh = true;
    }
    if (mode == 2 && !b->pipe_placed && b->out_planes && b->frames >= 1024) {   // outside the timed region
        b->pipe_placed = true;
        HIP_TRY(pipe_place(b, p, bf, b->stream));
        point_planes(b, bf);
    }
    int t0, t1;
    HIP_TRY(hipEventRecord(b->ev[2], b->stream));
    HIP_TRY(b->timed_event(&t0));
    if (mode >= 2) {   // every output word (hist, counts, points) is rewritten: no memset, no host sync
        HIP_TRY(launch_pipeline_resident(p, bf, b->frames, mode != 3, b->stream, mode == 2, &b->kname[1]));
    } else {
        b->kname[1] = "svx::stage_kernel + svx::offsets_kernel";
        const int nchunks = (b->frames + chunk - 1) / chunk;
        while ((int)b->sync_ev.size() < 2 * nchunks) {
            hipEvent_t e;
            HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            b->sync_ev.push_back(e);
        }
        if (!b->stream2) HIP_TRY(hipStreamCreateWithFlags(&b->stream2, hipStreamNonBlocking));
        HIP_TRY(hipMemsetAsync(b->ctrl.p, 0, b->ctrl_bytes, b->stream));
        HIP_TRY(launch_pipeline(p, bf, b->frames, chunk, b->stream, b->stream2, b->sync_ev.data()));
    }
    HIP_TRY(b->timed_event(&t1));
    HIP_TRY(hipEventRecord(b->ev[3], b->stream));
    if (t0 >= 0) b->pending[1].push_back({t0, t1});
    b->have_ms[1] = true;
    if (sync) HIP_TRY(hipStreamSynchronize(b->stream));
    return SV_OK;
}

int sv_batch_pipeline(sv_batch* b, const sv_camera* cam, const sv_plane* plane, double point_thr, int hist_thr,
                      int chunk, int sync) {
    if (!b || !cam || !plane) return fail(SV_E_ARG, "null");
    Device* d;
    if (int rc = dev_get(b->device, &d)) return rc;
    return batch_pipeline_impl(b, cam, plane, point_thr, hist_thr, chunk, sync, d);
}

int sv_batch_pipeline_planes(sv_batch* b, const sv_camera* cam, double point_thr, int hist_thr, int chunk,
                             int sync) {
    if (!b || !cam) return fail(SV_E_ARG, "null");
    if (!b->rres.p) return fail(SV_E_STATE, "no per-frame planes (sv_batch_ransac first)");
    Device* d;
    if (int rc = dev_get(b->device, &d)) return rc;
    HIP_TRY(b->fplanes.ensure(sizeof(FramePlane) * (size_t)b->frames));
    const RansacRes r = ransac_res(b);
    const KParams kp = make_params(b->H, b->W, b->step, *cam, b->Wu);
    HIP_TRY(launch_frame_planes(r.abc, r.trial, b->frames, kp, point_thr, b->fplanes.as<FramePlane>(), b->stream));
    const sv_plane none{0.0, 0.0, 0.0};   // per-frame planes replace it
    return batch_pipeline_impl(b, cam, &none, point_thr, hist_thr, chunk, sync, d, b->fplanes.as<FramePlane>());
}

int sv_batch_pipeline_dev(sv_batch* b, const sv_camera* cam, const double* dplane, double point_thr, int hist_thr,
                          int chunk, int sync) {
    if (!b || !cam || !dplane) return fail(SV_E_ARG, "null");
    Device* d;
    if (int rc = dev_get(b->device, &d)) return rc;
    HIP_TRY(b->dplane.ensure(sizeof(FramePlane)));
    const KParams kp = make_params(b->H, b->W, b->step, *cam, b->Wu);
    HIP_TRY(launch_frame_planes(dplane, nullptr, 1, kp, point_thr, b->dplane.as<FramePlane>(), b->stream));
    const sv_plane none{0.0, 0.0, 0.0};   // the device plane replaces it
    return batch_pipeline_impl(b, cam, &none, point_thr, hist_thr, chunk, sync, d, b->dplane.as<FramePlane>(), 0);
}

int sv_batch_read_frame_plane(sv_batch* b, int frame, double* out4) {
    if (!b || frame < 0 || frame >= b->frames || !out4) return fail(SV_E_ARG, "bad args");
    if (!b->fplanes.p) return fail(SV_E_STATE, "no per-frame planes (sv_batch_pipeline_planes first)");
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(hipStreamSynchronize(b->stream));
    FramePlane fp;
    HIP_TRY(hipMemcpy(&fp, b->fplanes.as<FramePlane>() + frame, sizeof fp, hipMemcpyDeviceToHost));
    out4[0] = fp.a;
    out4[1] = fp.b;
    out4[2] = fp.c;
    out4[3] = fp.valid ? fp.nrm : -1.0;
    return SV_OK;
}

int sv_batch_placement(sv_batch* b, int which, float* ms, int cap, int* n, int* kept) {
    if (!b || which < 0 || which > 2 || !n || !kept || cap < 0 || (cap > 0 && !ms))
        return fail(SV_E_ARG, "sv_batch_placement: bad arguments");
    *n = b->place_n[which];
    *kept = b->place_kept[which];
    for (int t = 0; t < std::min(cap, *n); ++t) ms[t] = b->place_ms[which][t];
    return SV_OK;
}

int sv_source_id(int which, char* buf, int cap) {
#ifndef SVX_SRCID_K1
#define SVX_SRCID_K1 "unknown"
#define SVX_SRCID_PIPE "unknown"
#endif
    if (which < 0 || which > 1 || !buf || cap <= 0) return fail(SV_E_ARG, "sv_source_id: bad arguments");
    std::snprintf(buf, (size_t)cap, "%s", which == 0 ? SVX_SRCID_K1 : SVX_SRCID_PIPE);
    return SV_OK;
}

int sv_batch_kernel_name(sv_batch* b, int which, char* buf, int cap) {
    if (!b || which < 0 || which > 2 || !buf || cap <= 0) return fail(SV_E_ARG, "sv_batch_kernel_name: bad arguments");
    const char* n = which == 2 ? (b->have_ms[2] ? "sgbm stage" : nullptr) : b->kname[which];
    if (!n) return fail(SV_E_STATE, "no kernel of this kind launched yet");
    std::snprintf(buf, (size_t)cap, "%s", n);
    return SV_OK;
}

int sv_batch_pipeline_mode(sv_batch* b, int mode) {
    if (!b) return fail(SV_E_ARG, "null batch");
    if (mode < 0 || mode > 4)
        return fail(SV_E_ARG, "pipeline mode must be 0 (auto), 1 (tiled), 2 (resident), 3 (resident, no prefetch) "
                              "or 4 (resident, pass-2 prefetch only)");
    b->pipe_mode = mode;
    return SV_OK;
}

int sv_batch_sync(sv_batch* b) {
    if (!b) return fail(SV_E_ARG, "null");
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(hipStreamSynchronize(b->stream));
    if (b->err) {
        uint32_t err = 0;
        HIP_TRY(hipMemcpy(&err, b->err, 4, hipMemcpyDeviceToHost));
        if (err) return fail(SV_E_DEVICE, "pipeline look-back timed out");
    }
    return SV_OK;
}

int sv_batch_last_ms(sv_batch* b, int which, float* ms) {
    if (!b || !ms || which < 0 || which > 2) return fail(SV_E_ARG, "bad args");
    if (!b->have_ms[which]) return fail(SV_E_STATE, "no timing recorded");
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(hipEventSynchronize(b->ev[2 * which + 1]));
    HIP_TRY(hipEventElapsedTime(ms, b->ev[2 * which], b->ev[2 * which + 1]));
    return SV_OK;
}

int sv_batch_timing(sv_batch* b, int which, double* total_ms, int64_t* count) {
    if (!b || which < 0 || which > 2 || !total_ms || !count) return fail(SV_E_ARG, "bad args");
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(hipStreamSynchronize(b->stream));
    double tot = 0;
    for (auto& pr : b->pending[which]) {
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, b->pool[pr.first], b->pool[pr.second]));
        tot += ms;
    }
    *total_ms = tot;
    *count = (int64_t)b->pending[which].size();
    return SV_OK;
}

int sv_batch_timing_reset(sv_batch* b) {
    if (!b) return fail(SV_E_ARG, "null");
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(hipStreamSynchronize(b->stream));
    for (auto& p : b->pending) p.clear();
    b->pool_next = 0;
    return SV_OK;
}

int sv_batch_read_dense(sv_batch* b, int frame, float* X, float* Y, float* Z) {
    if (!b || frame < 0 || frame >= b->frames || !b->X.p) return fail(SV_E_ARG, "bad args / nothing projected");
    HIP_TRY(hipSetDevice(b->device));
    const size_t n = (size_t)b->dense_per_frame, off = n * frame;
    HIP_TRY(hipStreamSynchronize(b->stream));
    if (X) HIP_TRY(hipMemcpy(X, b->X.as<float>() + off, n * 4, hipMemcpyDeviceToHost));
    if (Y) HIP_TRY(hipMemcpy(Y, b->Y.as<float>() + off, n * 4, hipMemcpyDeviceToHost));
    if (Z) HIP_TRY(hipMemcpy(Z, b->Z.as<float>() + off, n * 4, hipMemcpyDeviceToHost));
    return SV_OK;
}

int sv_batch_read_counts(sv_batch* b, int64_t* counts) {
    if (!b || !counts) return fail(SV_E_ARG, "null");
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(hipStreamSynchronize(b->stream));
    int64_t* tmp = new int64_t[4 * (size_t)b->frames];
    hipError_t e = hipMemcpy(tmp, b->counts, sizeof(int64_t) * 4 * b->frames, hipMemcpyDeviceToHost);
    if (e == hipSuccess)
        for (int f = 0; f < b->frames; ++f)
            for (int k = 0; k < 3; ++k) counts[3 * f + k] = tmp[4 * f + k];
    delete[] tmp;
    HIP_TRY(e);
    return SV_OK;
}

int sv_batch_read_hist(sv_batch* b, int frame, uint32_t* hist) {
    if (!b || !hist || frame < 0 || frame >= b->frames) return fail(SV_E_ARG, "bad args");
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(hipStreamSynchronize(b->stream));
    HIP_TRY(hipMemcpy(hist, b->hist + (size_t)kBins * frame, 4 * kBins, hipMemcpyDeviceToHost));
    return SV_OK;
}

int sv_batch_read_points(sv_batch* b, int frame, float* xyz, int32_t* pts, int64_t cap, int64_t* n) {
    if (!b || !n || frame < 0 || frame >= b->frames || !b->ppxy.p) return fail(SV_E_ARG, "bad args");
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(hipStreamSynchronize(b->stream));
    int64_t c[4];
    HIP_TRY(hipMemcpy(c, b->counts + 4 * (size_t)frame, sizeof c, hipMemcpyDeviceToHost));
    *n = c[2];
    if (c[2] > cap) return fail(SV_E_CAP, "capacity %lld < %lld", (long long)cap, (long long)c[2]);
    const size_t np = (size_t)c[2], cap_f = b->cap;
    if (xyz && np) {   // device layout: X, Y, Z planes of the frame (point_planes)
        std::vector<float> soa(3 * np);
        PipeBuffers bf;
        point_planes(b, bf);
        const float* src[3] = {bf.ox + bf.ofs * frame, bf.oy + bf.ofs * frame, bf.oz + bf.ofs * frame};
        for (int k = 0; k < 3; ++k)
            HIP_TRY(hipMemcpy(soa.data() + k * np, src[k], 4 * np, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < np; ++i)
            for (int k = 0; k < 3; ++k) xyz[3 * i + k] = soa[k * np + i];
    }
    if (pts && np) {   // device layout: one pp_pack word a point; the caller gets the int32 (x, y) pairs
        std::vector<uint32_t> pl(np);
        HIP_TRY(hipMemcpy(pl.data(), b->ppxy.as<uint32_t>() + cap_f * frame, 4 * np, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < np; ++i) {
            pts[2 * i] = pp_x(pl[i]);
            pts[2 * i + 1] = pp_y(pl[i]);
        }
    }
    return SV_OK;
}

int sv_batch_digest(sv_batch* b, const sv_camera* cam, int which, uint64_t* out) {
    if (!b || !cam || !out || which < 0 || which > 1) return fail(SV_E_ARG, "sv_batch_digest: bad args");
    if (which == 0 && !b->Z.p) return fail(SV_E_STATE, "sv_batch_digest: nothing projected");
    if (which == 1 && !b->ppxy.p) return fail(SV_E_STATE, "sv_batch_digest: no pipeline outputs");
    if ((b->kp.frame_px % 4) != 0) return fail(SV_E_ARG, "sv_batch_digest: H * W must be a multiple of 4");
    HIP_TRY(hipSetDevice(b->device));
    KParams p = make_params(b->H, b->W, b->step, *cam, b->Wu);
    DevBuf buf;
    HIP_TRY(buf.ensure(sizeof(uint64_t) * 8 * (size_t)b->frames));
    hipError_t e;
    if (which == 0)
        e = launch_digest_dense(p, b->disp.as<uint8_t>(), b->X.as<float>(), b->Y.as<float>(), b->Z.as<float>(),
                                b->frames, buf.as<uint64_t>(), b->stream);
    else
    {
        PipeBuffers bf;
        point_planes(b, bf);
        e = launch_digest_pipe(p, b->disp.as<uint8_t>(), b->hist, b->counts, bf, b->frames, buf.as<uint64_t>(),
                               b->stream);
    }
    if (e == hipSuccess) e = hipMemcpyAsync(out, buf.p, sizeof(uint64_t) * 8 * (size_t)b->frames, hipMemcpyDeviceToHost,
                                            b->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(b->stream);
    (void)hipFree(buf.p);
    HIP_TRY(e);
    return SV_OK;
}

// ---------------------------------------------------------------------------
// fused one-frame chain (stereovision.py:84,97-113) through a cached batch
// ---------------------------------------------------------------------------
int sv_pipeline_frame(const uint8_t* disp, const uint8_t* bgr, int H, int W, int step, const sv_camera* cam,
                      const sv_plane* plane, double point_thr, int hist_thr, int64_t* out_counts,
                      uint32_t* out_hist, float* out_xyz, int32_t* out_pts, int64_t cap) {
    if (!disp || !bgr || !cam || !plane || !out_counts)
        return fail(SV_E_ARG, "sv_pipeline_frame: null argument");
    int dev;
    if (int rc = current_device(&dev)) return rc;
    Device* d;
    if (int rc = dev_get(dev, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    sv_batch* b = d->frame_batch;
    if (!b || b->H != H || b->W != W || b->step != step) {
        if (b) sv_batch_destroy(b);
        d->frame_batch = nullptr;
        if (int rc = sv_batch_create(dev, 1, H, W, step, 1, 1, &b)) return rc;
        d->frame_batch = b;
    }
    if (int rc = sv_batch_upload(b, 0, disp, bgr)) return rc;
    if (int rc = batch_pipeline_impl(b, cam, plane, point_thr, hist_thr, 1, 1, d)) return rc;
    if (int rc = sv_batch_read_counts(b, out_counts)) return rc;
    if (out_hist)
        if (int rc = sv_batch_read_hist(b, 0, out_hist)) return rc;
    if (out_pts || out_xyz) {
        int64_t n = 0;
        if (int rc = sv_batch_read_points(b, 0, out_xyz, out_pts, cap, &n)) return rc;
    }
    return SV_OK;
}

// ---------------------------------------------------------------------------
// disparity pre-pass (functions.py:131-172): host frames, synchronous
// ---------------------------------------------------------------------------
namespace {
// upload an H x W u8 host image into a pitch = round_up(W, 4) device buffer (zero pad)
int upload_u8(DevBuf& buf, const uint8_t* src, int H, int W, int pitch, hipStream_t s) {
    HIP_TRY(buf.ensure((size_t)H * pitch));
    if (pitch != W) HIP_TRY(hipMemsetAsync(buf.p, 0, (size_t)H * pitch, s));
    HIP_TRY(hipMemcpy2DAsync(buf.p, pitch, src, W, W, H, hipMemcpyHostToDevice, s));
    return SV_OK;
}
int download_u8(uint8_t* dst, const DevBuf& buf, int H, int W, int pitch, hipStream_t s) {
    HIP_TRY(hipMemcpy2DAsync(dst, W, buf.p, pitch, W, H, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return SV_OK;
}
}  // namespace

int sv_fill_previous(const uint8_t* disp, const uint8_t* prev, int H, int W, uint8_t* out) {
    if (!disp || !out || H < 0 || W < 0) return fail(SV_E_ARG, "sv_fill_previous: bad arguments");
    if ((int64_t)H * W == 0) return SV_OK;
    int dev;
    if (int rc = current_device(&dev)) return rc;
    Device* d;
    if (int rc = dev_get(dev, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    const int pitch = (W + 3) / 4 * 4;
    if (int rc = upload_u8(d->disp, disp, H, W, pitch, d->stream)) return rc;
    if (prev)
        if (int rc = upload_u8(d->aux, prev, H, W, pitch, d->stream)) return rc;
    HIP_TRY(launch_fill_prev(d->disp.as<uint8_t>(), d->disp.as<uint8_t>(), nullptr, nullptr,
                             prev ? d->aux.as<uint8_t>() : nullptr, 1, (int64_t)H * pitch, d->stream));
    return download_u8(out, d->disp, H, W, pitch, d->stream);
}

int sv_fill_mean(uint8_t* disp, int H, int W) {
    if (!disp || H < 0 || W < 0) return fail(SV_E_ARG, "sv_fill_mean: bad arguments");
    if ((int64_t)H * W == 0) return SV_OK;
    int dev;
    if (int rc = current_device(&dev)) return rc;
    Device* d;
    if (int rc = dev_get(dev, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    const int pitch = (W + 3) / 4 * 4;
    if (int rc = upload_u8(d->disp, disp, H, W, pitch, d->stream)) return rc;
    HIP_TRY(launch_fill_mean(d->disp.as<uint8_t>(), nullptr, nullptr, 1, H, pitch, W, d->stream));
    return download_u8(disp, d->disp, H, W, pitch, d->stream);
}

int sv_mask_disparity(const uint8_t* disp, const uint8_t* mask, int H, int W, uint8_t* out) {
    if (!disp || !mask || !out || H < 0 || W < 0) return fail(SV_E_ARG, "sv_mask_disparity: bad arguments");
    if ((int64_t)H * W == 0) return SV_OK;
    int dev;
    if (int rc = current_device(&dev)) return rc;
    Device* d;
    if (int rc = dev_get(dev, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    const int pitch = (W + 3) / 4 * 4;
    const int64_t px = (int64_t)H * pitch;
    if (int rc = upload_u8(d->disp, disp, H, W, pitch, d->stream)) return rc;
    if (int rc = upload_u8(d->aux, mask, H, W, pitch, d->stream)) return rc;
    HIP_TRY(d->aux2.ensure((size_t)px));
    HIP_TRY(launch_mask_bytes(d->aux.as<uint8_t>(), d->aux2.as<uint8_t>(), px, d->stream));
    HIP_TRY(launch_mask(d->disp.as<uint8_t>(), d->disp.as<uint8_t>(), d->aux2.as<uint8_t>(), 1, px, d->stream));
    return download_u8(out, d->disp, H, W, pitch, d->stream);
}

int sv_batch_set_mask(sv_batch* b, const uint8_t* mask) {
    if (!b) return fail(SV_E_ARG, "null batch");
    HIP_TRY(hipSetDevice(b->device));
    if (!mask) {
        b->have_mask = false;
        return SV_OK;
    }
    const int64_t px = (int64_t)b->H * b->W;
    HIP_TRY(b->carmask.ensure((size_t)px * 2));
    uint8_t* grey = b->carmask.as<uint8_t>() + px;
    HIP_TRY(hipMemsetAsync(grey, 0, (size_t)px, b->stream));
    HIP_TRY(hipMemcpy2DAsync(grey, b->W, mask, b->Wu, b->Wu, b->H, hipMemcpyHostToDevice, b->stream));
    HIP_TRY(launch_mask_bytes(grey, b->carmask.as<uint8_t>(), px, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    b->have_mask = true;
    // the mask's points on maskpoints' step-2 grid (range(0, H-1, 2) x range(0, W-1, 2)): no frame's masked point
    // count can exceed it, so it sizes the batched RANSAC's launches without reading the counts back (batch_ransac_*)
    int64_t n2 = 0;
    for (int y = 0; y < b->H - 1; y += 2)
        for (int x = 0; x < b->Wu - 1; x += 2) n2 += mask[(int64_t)y * b->Wu + x] != 0;
    b->mask_n2 = n2;
    return SV_OK;
}

// The pre-pass over the batch's frames in order; dprev0: frame 0's previous cleaned frame in device memory (the
// frame loop's carry from the batch before), or null.
static int batch_prepass_impl(sv_batch* b, int option, const uint8_t* dprev0) {
    uint8_t* masked = nullptr;
    const uint8_t* mff = nullptr;
    uint8_t* disp = b->disp.as<uint8_t>();
    const uint8_t* in = input_disp(b);   // keep_input: the raw frames, read here and never written
    const int64_t px = (int64_t)b->H * b->W;
    if (option == 1) {
        HIP_TRY(launch_fill_prev(in, disp, masked, mff, dprev0, b->frames, px, b->stream));
    } else {
        if (in != disp) HIP_TRY(hipMemcpyAsync(disp, in, (size_t)px * b->frames, hipMemcpyDeviceToDevice, b->stream));
        if (option == 2) HIP_TRY(launch_fill_mean(disp, masked, mff, b->frames, b->H, b->W, b->Wu, b->stream));
    }
    return SV_OK;
}

int sv_batch_prepass(sv_batch* b, int option, const uint8_t* prev0, int sync) {
    if (!b) return fail(SV_E_ARG, "null batch");
    if (option < 0 || option > 2) return fail(SV_E_ARG, "prepass option must be 0 (none), 1 (previous) or 2 (mean)");
    HIP_TRY(hipSetDevice(b->device));
    const int64_t px = (int64_t)b->H * b->W;
    // maskDisparity (functions.py:169-172) is not materialised: its only consumer on the device, maskpoints, applies
    // the mask as it reads the cleaned disparity (the fill pass moves 2 B a pixel, not 3); sv_batch_read_disp
    // applies it to the frame it reads back
    const uint8_t* p0 = nullptr;
    if (option == 1 && prev0) {
        HIP_TRY(b->prev0buf.ensure((size_t)px));
        HIP_TRY(hipMemsetAsync(b->prev0buf.p, 0, (size_t)px, b->stream));
        HIP_TRY(hipMemcpy2DAsync(b->prev0buf.p, b->W, prev0, b->Wu, b->Wu, b->H, hipMemcpyHostToDevice, b->stream));
        p0 = b->prev0buf.as<uint8_t>();
    }
    if (int rc = batch_prepass_impl(b, option, p0)) return rc;
    if (sync || prev0) HIP_TRY(hipStreamSynchronize(b->stream));
    return SV_OK;
}

int sv_batch_read_disp(sv_batch* b, int frame, uint8_t* disp, uint8_t* masked) {
    if (!b || frame < 0 || frame >= b->frames) return fail(SV_E_ARG, "bad args");
    if (masked && !b->have_mask) return fail(SV_E_STATE, "no masked disparity (set a mask first)");
    HIP_TRY(hipSetDevice(b->device));
    const size_t px = (size_t)b->H * b->W;
    uint8_t* mframe = nullptr;
    if (masked) {   // maskDisparity of this frame (the batch does not hold masked copies)
        HIP_TRY(b->rdbuf.ensure(px));
        mframe = b->rdbuf.as<uint8_t>();
        HIP_TRY(launch_mask(b->disp.as<uint8_t>() + px * frame, mframe, b->carmask.as<uint8_t>(), 1, (int64_t)px,
                            b->stream));
    }
    HIP_TRY(hipStreamSynchronize(b->stream));
    if (disp)
        HIP_TRY(hipMemcpy2D(disp, b->Wu, b->disp.as<uint8_t>() + px * frame, b->W, b->Wu, b->H, hipMemcpyDeviceToHost));
    if (masked)
        HIP_TRY(hipMemcpy2D(masked, b->Wu, mframe, b->W, b->Wu, b->H,
                            hipMemcpyDeviceToHost));
    return SV_OK;
}

// ---------------------------------------------------------------------------
// road raster + non-zero walk (functions.py:339-344, :359-365)
// ---------------------------------------------------------------------------
int sv_road_raster(const int32_t* pts, int64_t n, int H, int W, uint8_t* out_img) {
    if (n < 0 || H < 0 || W < 0 || !out_img || (n > 0 && !pts)) return fail(SV_E_ARG, "sv_road_raster: bad arguments");
    for (int64_t i = 0; i < n; ++i) {   // numpy raises IndexError past these; negatives wrap
        const int32_t x = pts[2 * i], y = pts[2 * i + 1];
        if (x < -W || x >= W || y < -H || y >= H)
            return fail(SV_E_ARG, "index out of range: point %lld is [%d, %d] for a %d x %d image", (long long)i, x, y, H, W);
    }
    if ((int64_t)H * W == 0) return SV_OK;
    int dev;
    if (int rc = current_device(&dev)) return rc;
    Device* d;
    if (int rc = dev_get(dev, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    hipStream_t s = d->stream;
    HIP_TRY(d->aux.ensure((size_t)H * W));
    HIP_TRY(d->xy.ensure(sizeof(int32_t) * 2 * (size_t)(n > 0 ? n : 1)));
    if (n) HIP_TRY(hipMemcpyAsync(d->xy.p, pts, sizeof(int32_t) * 2 * n, hipMemcpyHostToDevice, s));
    HIP_TRY(launch_raster(d->xy.as<int32_t>(), d->xy.as<int32_t>() + 1, 2, nullptr, 0, 0, n, d->aux.as<uint8_t>(), 1, H,
                          W, W, s));
    HIP_TRY(hipMemcpyAsync(out_img, d->aux.p, (size_t)H * W, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return SV_OK;
}

int sv_nonzero_points(const uint8_t* img, int H, int W, int32_t* out, int64_t cap, int64_t* out_n) {
    if (!img || !out_n || H < 0 || W < 0 || W > 4096 || (int64_t)H * W >= (1ll << 28))
        return fail(SV_E_ARG, "sv_nonzero_points: bad arguments (W <= 4096, H*W < 2^28)");
    *out_n = 0;
    const int64_t px = (int64_t)H * W;
    if (px == 0) return SV_OK;
    int dev;
    if (int rc = current_device(&dev)) return rc;
    Device* d;
    if (int rc = dev_get(dev, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    hipStream_t s = d->stream;
    const int64_t padded = (px + 3) / 4 * 4;   // zero tail: no extra non-zero pixels
    HIP_TRY(d->aux.ensure((size_t)padded));
    if (padded != px) HIP_TRY(hipMemsetAsync(d->aux.as<uint8_t>() + px, 0, (size_t)(padded - px), s));
    HIP_TRY(hipMemcpyAsync(d->aux.p, img, (size_t)px, hipMemcpyHostToDevice, s));
    HIP_TRY(d->xy.ensure(sizeof(int32_t) * 2 * (size_t)px + 64));
    int64_t* cnt = reinterpret_cast<int64_t*>(d->xy.as<char>() + sizeof(int32_t) * 2 * (size_t)px);
    HIP_TRY(launch_nonzero(d->aux.as<uint8_t>(), 1, padded, W, d->xy.as<int32_t>(), px, cnt, false, s));
    int64_t n = 0;
    HIP_TRY(hipMemcpyAsync(&n, cnt, sizeof n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (n > cap) return fail(SV_E_CAP, "capacity %lld < %lld non-zero pixels", (long long)cap, (long long)n);
    if (n) {
        HIP_TRY(hipMemcpyAsync(out, d->xy.p, sizeof(int32_t) * 2 * n, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    *out_n = n;
    return SV_OK;
}

int sv_batch_road_raster(sv_batch* b, int sync) {
    if (!b) return fail(SV_E_ARG, "null batch");
    if (!b->ppxy.p) return fail(SV_E_STATE, "no pipeline points (create the batch with points and run the pipeline)");
    HIP_TRY(hipSetDevice(b->device));
    const size_t px = (size_t)b->H * b->W;
    HIP_TRY(b->road.ensure(px * b->frames));
    HIP_TRY(b->nz.ensure(sizeof(uint32_t) * b->cap * b->frames));   // packed entries x | y << 16 (walk_pk)
    HIP_TRY(b->nzcount.ensure(sizeof(int64_t) * b->frames));
    // the images and their non-zero walks in one pass (road_kernel); SVX_ROAD_FUSED=0: raster, then the walk
    const char* v = svx_knob("SVX_ROAD_FUSED");
    b->nz_fresh = !(v && v[0] == '0');
    b->rmap_fresh = false;
    if (b->nz_fresh) {
        uint8_t* paint = nullptr;
        if (b->want_rmap) {   // imageRoadMap in the same pass (stereovision.py:131-133)
            HIP_TRY(b->rmap.ensure(px * 3 * b->frames));
            paint = b->rmap.as<uint8_t>();
        }
        if (b->rbits_fresh) {   // from the pipeline's bitmap (68 KB a frame) instead of its points (8 B a point)
            HIP_TRY(b->roff.ensure(sizeof(int32_t) * (size_t)b->H * b->frames));
            HIP_TRY(launch_road_bits(b->rbits.as<uint32_t>(), b->frames, b->H, b->W, b->roff.as<int32_t>(),
                                     (int64_t)b->cap, b->road.as<uint8_t>(), b->nz.as<int32_t>(),
                                     b->nzcount.as<int64_t>(), b->bgr.as<uint8_t>(), paint, b->stream));
        } else {
            HIP_TRY(launch_road(b->ppxy.as<uint32_t>(), b->counts, (int64_t)b->cap,
                                b->road.as<uint8_t>(), b->frames, b->H, b->W, b->Wu, b->nz.as<int32_t>(),
                                b->nzcount.as<int64_t>(), b->bgr.as<uint8_t>(), paint, b->stream));
        }
        b->rmap_fresh = paint != nullptr;
    } else {
        HIP_TRY(launch_raster(b->ppxy.as<int32_t>(), nullptr, 0, b->counts, 4, 2, (int64_t)b->cap,
                              b->road.as<uint8_t>(), b->frames, b->H, b->W, b->Wu, b->stream));
    }
    if (sync) HIP_TRY(hipStreamSynchronize(b->stream));
    return SV_OK;
}

int sv_batch_nonzero(sv_batch* b, int sync) {
    if (!b) return fail(SV_E_ARG, "null batch");
    if (!b->road.p) return fail(SV_E_STATE, "no road images (sv_batch_road_raster first)");
    HIP_TRY(hipSetDevice(b->device));
    if (b->nz_fresh) {   // sv_batch_road_raster walked the images it wrote
        if (sync) HIP_TRY(hipStreamSynchronize(b->stream));
        return SV_OK;
    }
    HIP_TRY(b->nz.ensure(sizeof(uint32_t) * b->cap * b->frames));   // packed entries x | y << 16 (walk_pk)
    HIP_TRY(b->nzcount.ensure(sizeof(int64_t) * b->frames));
    HIP_TRY(launch_nonzero(b->road.as<uint8_t>(), b->frames, (int64_t)b->H * b->W, b->W, b->nz.as<int32_t>(),
                           (int64_t)b->cap, b->nzcount.as<int64_t>(), true, b->stream));
    if (sync) HIP_TRY(hipStreamSynchronize(b->stream));
    return SV_OK;
}

int sv_batch_road_bits(sv_batch* b, int enable) {
    if (!b) return fail(SV_E_ARG, "null batch");
    b->road_bits = enable != 0;
    return SV_OK;
}

int sv_batch_road_map(sv_batch* b, int enable) {
    if (!b) return fail(SV_E_ARG, "null batch");
    if (enable && !b->with_bgr) return fail(SV_E_STATE, "imageRoadMap needs the batch's BGR (with_bgr)");
    b->want_rmap = enable != 0;
    return SV_OK;
}

int sv_batch_read_road_map(sv_batch* b, int frame, uint8_t* out) {
    if (!b || !out || frame < 0 || frame >= b->frames) return fail(SV_E_ARG, "bad args");
    if (!b->rmap_fresh) return fail(SV_E_STATE, "no imageRoadMap (sv_batch_road_map(b, 1), then sv_batch_road_raster)");
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(hipStreamSynchronize(b->stream));
    const size_t px3 = (size_t)b->H * b->W * 3;
    HIP_TRY(hipMemcpy2D(out, (size_t)b->Wu * 3, b->rmap.as<uint8_t>() + px3 * frame, (size_t)b->W * 3,
                        (size_t)b->Wu * 3, b->H, hipMemcpyDeviceToHost));
    return SV_OK;
}

int sv_batch_read_road(sv_batch* b, int frame, uint8_t* img, int32_t* nzpts, int64_t cap, int64_t* n) {
    if (!b || frame < 0 || frame >= b->frames) return fail(SV_E_ARG, "bad args");
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(hipStreamSynchronize(b->stream));
    const size_t px = (size_t)b->H * b->W;
    if (img) {
        if (!b->road.p) return fail(SV_E_STATE, "no road images");
        HIP_TRY(hipMemcpy2D(img, b->Wu, b->road.as<uint8_t>() + px * frame, b->W, b->Wu, b->H, hipMemcpyDeviceToHost));
    }
    if (n) {
        if (!b->nz.p) return fail(SV_E_STATE, "no non-zero walk (sv_batch_nonzero first)");
        int64_t k = 0;
        HIP_TRY(hipMemcpy(&k, b->nzcount.as<int64_t>() + frame, sizeof k, hipMemcpyDeviceToHost));
        *n = k;
        if (k > cap) return fail(SV_E_CAP, "capacity %lld < %lld", (long long)cap, (long long)k);
        if (k && nzpts) {   // the packed entries (x | y << 16) widened to the reference's [x, y] int32 pairs
            std::vector<uint32_t> pk((size_t)k);
            HIP_TRY(hipMemcpy(pk.data(), b->nz.as<uint32_t>() + b->cap * frame, sizeof(uint32_t) * k,
                              hipMemcpyDeviceToHost));
            for (int64_t i = 0; i < k; ++i) {
                nzpts[2 * i] = (int32_t)(pk[(size_t)i] & 0xFFFFu);
                nzpts[2 * i + 1] = (int32_t)(pk[(size_t)i] >> 16);
            }
        }
    }
    return SV_OK;
}

// ---------------------------------------------------------------------------
// batched RANSAC (stereovision.py:85-94 per frame, seeded per frame)
// ---------------------------------------------------------------------------

// DIAGNOSTIC ONLY (env SVX_RANSAC_ABLATE, diagnostic build, documented in DESIGN.md): 1 skips the trial
// evaluation (results invalid); 4 evaluates every trial in fp64 (no fp32 screen; results valid, for A/B); draw
// kernel (results invalid): 8 no collinearity test, 16 no random.sample (both also skip the evaluation). Any other
// bit is refused (-1): an undocumented bit once rode along in an A/B run that faulted.
static constexpr int kRansacAblateBits = 1 | 4 | 8 | 16 | 32 | 128;
#ifdef SVX_DIAG
}  // extern "C"
namespace svx {
hipError_t diag_eval_phases(unsigned long long* out, bool reset);
}
extern "C" {
// DIAGNOSTIC (diagnostic build only, not in include/svx.h): the evaluation's phase clocks (SVX_RANSAC_ABLATE bit 32)
extern "C" int sv_diag_eval_phases(unsigned long long* out8, int reset) {
    if (!out8) return fail(SV_E_ARG, "sv_diag_eval_phases: null argument");
    HIP_TRY(diag_eval_phases(out8, reset != 0));
    return SV_OK;
}
#endif

static int ransac_ablate() {
    const char* e = svx_knob("SVX_RANSAC_ABLATE");
    const int v = e ? std::atoi(e) : 0;
    return (v & ~kRansacAblateBits) ? -1 : v;
}

// Batched RANSAC in two phases, so that a caller with other streams to feed (the frame loop) is not held by the
// one read-back: phase 1 enqueues the step-2 tables, maskpoints and the copy of the per-frame counts into pinned
// host memory (+ an event); phase 2 waits for that event — the largest frame sizes the draw kernel's LDS (bitmap /
// pool list) and the sample index width — and enqueues the draw and evaluation kernels.
// An upper bound of every frame's maskpoints count that sizes the RANSAC launches with no read-back, or -1: the
// mask's step-2 grid points when a mask is set and they keep the draw kernel's sample LDS (a bitmap of n bits, or
// the pool branch's k-entry list) within 8 KiB and the sample indices 16-bit; otherwise the counts are read.
static int64_t ransac_device_bound(const sv_batch* b, int k) {
    if (!b->have_mask) return -1;
    // DIAGNOSTIC A/B (diagnostic build): SVX_RANSAC_BOUND=0 sizes the draw from the counts read back even with a mask
    if (const char* e = svx_knob("SVX_RANSAC_BOUND"); e && e[0] == '0') return -1;
    const int64_t n = std::min(b->mask_n2, b->mcap);
    const int64_t words = std::max<int64_t>((n + 31) / 32, k);
    return (words <= 2048 && n <= 65535) ? n : -1;
}

static int batch_ransac_prepare(sv_batch* b, const sv_camera* cam, int trials, int k) {
    if (!b || !cam || trials < 0 || k < 1 || k > 1024)
        return fail(SV_E_ARG, "sv_batch_ransac: bad arguments (1 <= k <= 1024, trials >= 0)");
    if (trials > 4096) return fail(SV_E_ARG, "sv_batch_ransac: trials <= 4096");
    const int Hg = grid_len(b->H, 2), Wg = grid_len(b->W, 2);
    const int64_t mcap = (int64_t)Hg * Wg;
    if (mcap > 163840)
        return fail(SV_E_ARG, "sv_batch_ransac: %lld step-2 grid points per frame > 163,840 (LDS sample bitmap)",
                    (long long)mcap);
    if (b->H > 4096 || b->W > 4096) return fail(SV_E_ARG, "sv_batch_ransac: frames up to 4096 x 4096");
    HIP_TRY(hipSetDevice(b->device));
    const size_t F = (size_t)b->frames;
    HIP_TRY(b->mpk.ensure(sizeof(uint32_t) * (size_t)(mcap > 0 ? mcap : 1) * F));
    HIP_TRY(b->rres.ensure(F * (sizeof(double) * 4 + sizeof(int64_t) + sizeof(int32_t) + sizeof(uint32_t))));
    if (!b->hcnt) HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&b->hcnt), sizeof(int64_t) * F));
    if (!b->cnt_ev) HIP_TRY(hipEventCreateWithFlags(&b->cnt_ev, hipEventDisableTiming));
    b->mcap = mcap;
    const RansacRes r = ransac_res(b);
    const KParams p = make_params(b->H, b->W, 2, *cam, b->Wu);
    // the fp64 X / Y / Z tables of the step-2 grid for this camera (the RANSAC kernels and the read-back gather
    // them instead of dividing)
    HIP_TRY(b->rtab.ensure(ransac_tables_bytes(b->H, b->W)));
    HIP_TRY(launch_ransac_tables(b->H, b->W, p, b->rtab.as<double>(), b->stream));
    const uint8_t* mff = b->have_mask ? b->carmask.as<uint8_t>() : nullptr;
    HIP_TRY(launch_maskpoints(b->disp.as<uint8_t>(), mff, b->frames, b->H, b->W, p, b->mpk.as<uint32_t>(), mcap,
                              r.mcount, b->stream));
    // the launches are sized from an upper bound of every frame's count when one is small enough (the mask's grid
    // points: ransac_device_bound), else from the counts read back (the host waits for them in the launch)
    b->rbound = ransac_device_bound(b, k);
    if (b->rbound < 0) {
        HIP_TRY(hipMemcpyAsync(b->hcnt, r.mcount, sizeof(int64_t) * F, hipMemcpyDeviceToHost, b->stream));
        HIP_TRY(hipEventRecord(b->cnt_ev, b->stream));
    }
    return SV_OK;
}

// phases: 1 = the draw kernel (waits for phase 1's counts on the host), 2 = the evaluation kernel (after a phase-1
// launch with the same arguments), 3 = both. The frame loop enqueues the two as separate stages.
// started / epoch: the frame loop's dispatch signal (the draw kernel's last workgroup stores epoch there)
static int batch_ransac_launch(sv_batch* b, const sv_camera* cam, uint64_t seed_base, int64_t first_frame,
                               int trials, int k, hipStream_t stream, int phases = 3, uint64_t* started = nullptr,
                               uint64_t epoch = 0) {
    if (first_frame < 0) return fail(SV_E_ARG, "sv_batch_ransac: first_frame >= 0");
    HIP_TRY(hipSetDevice(b->device));
    const size_t F = (size_t)b->frames;
    const int64_t mcap = b->mcap;
    const RansacRes r = ransac_res(b);
    const KParams p = make_params(b->H, b->W, 2, *cam, b->Wu);
    int32_t* trace = nullptr;
    if (b->trace_trials > 0 && (phases & 1)) {
        HIP_TRY(b->rtrace.ensure(sizeof(int32_t) * F * b->trace_trials * (size_t)(k + 3)));
        HIP_TRY(hipMemsetAsync(b->rtrace.p, 0xff, sizeof(int32_t) * F * b->trace_trials * (size_t)(k + 3), stream));
        trace = b->rtrace.as<int32_t>();
    }
    if (phases & 1) {
        b->trace_k = k;
        b->traced_trials = trace ? b->trace_trials : 0;   // what rtrace holds now (sv_batch_read_ransac_trace)
    }
    // the largest frame sizes the kernel's LDS (bitmap / pool list): the device bound of batch_ransac_prepare, or
    // the counts phase 1 copied back
    if ((phases & 1) && b->rbound >= 0) {
        b->rmax_n = b->rbound;
        b->rmax_pool_n = b->rbound >= k ? std::min<int64_t>(b->rbound, ransac_setsize(k)) : 0;
    } else if (phases & 1) {
        HIP_TRY(hipEventSynchronize(b->cnt_ev));
        int64_t max_n = 0, max_pool_n = 0;
        const int64_t setsize = ransac_setsize(k);
        for (size_t f = 0; f < F; ++f) {
            const int64_t c = b->hcnt[f];
            max_n = std::max(max_n, c);
            if (c >= k && c <= setsize) max_pool_n = std::max(max_pool_n, c);
        }
        b->rmax_n = max_n;
        b->rmax_pool_n = max_pool_n;
    }
    const int64_t max_n = b->rmax_n, max_pool_n = b->rmax_pool_n;
    const int ablate = ransac_ablate();
    if (ablate < 0)
        return fail(SV_E_ARG, "SVX_RANSAC_ABLATE: only the documented bits 1, 4, 8, 16, 32 and 128 (diagnostic build)");
    HIP_TRY(b->rsidx.ensure(std::max<size_t>(ransac_sidx_bytes(max_n, b->frames, trials, k), 4)));
    HIP_TRY(b->rtri.ensure(sizeof(double) * 5 * F * (size_t)std::max(trials, 1) + sizeof(int32_t) * 2 * F));
    const RansacScratch rs{b->rsidx.p, b->rtri.as<double>(),
                           reinterpret_cast<int32_t*>(b->rtri.as<double>() + 5 * F * (size_t)std::max(trials, 1))};
    HIP_TRY(launch_ransac_batch(b->mpk.as<uint32_t>(), b->rtab.as<double>(), b->H, b->W, mcap, p, r.mcount, max_n,
                                max_pool_n,
                                seed_base, first_frame, b->frames, trials, k, rs, r.abc, r.err, r.trial, r.flags, trace,
                                b->trace_trials, ablate, phases, started, epoch, stream));
    return SV_OK;
}

int sv_batch_ransac(sv_batch* b, const sv_camera* cam, uint64_t seed_base, int64_t first_frame, int trials, int k,
                    int sync) {
    if (first_frame < 0) return fail(SV_E_ARG, "sv_batch_ransac: bad arguments (first_frame >= 0)");
    if (int rc = batch_ransac_prepare(b, cam, trials, k)) return rc;
    if (int rc = batch_ransac_launch(b, cam, seed_base, first_frame, trials, k, b->stream)) return rc;
    if (sync) HIP_TRY(hipStreamSynchronize(b->stream));
    return SV_OK;
}

int sv_batch_read_ransac(sv_batch* b, int frame, double* abc, double* err, int32_t* trial, uint32_t* flags) {
    if (!b || frame < 0 || frame >= b->frames) return fail(SV_E_ARG, "bad args");
    if (!b->rres.p) return fail(SV_E_STATE, "no RANSAC results (sv_batch_ransac first)");
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(hipStreamSynchronize(b->stream));
    const RansacRes r = ransac_res(b);
    if (abc) HIP_TRY(hipMemcpy(abc, r.abc + 3 * frame, 3 * sizeof(double), hipMemcpyDeviceToHost));
    if (err) HIP_TRY(hipMemcpy(err, r.err + frame, sizeof(double), hipMemcpyDeviceToHost));
    if (trial) HIP_TRY(hipMemcpy(trial, r.trial + frame, sizeof(int32_t), hipMemcpyDeviceToHost));
    if (flags) HIP_TRY(hipMemcpy(flags, r.flags + frame, sizeof(uint32_t), hipMemcpyDeviceToHost));
    return SV_OK;
}

int sv_batch_ransac_trace(sv_batch* b, int trials) {
    if (!b || trials < 0) return fail(SV_E_ARG, "bad args");
    b->trace_trials = trials;
    return SV_OK;
}

int sv_batch_read_ransac_trace(sv_batch* b, int frame, int32_t* out, int64_t cap, int* out_trials, int* out_k) {
    if (!b || frame < 0 || frame >= b->frames) return fail(SV_E_ARG, "bad args");
    if (!b->traced_trials || !b->rtrace.p) return fail(SV_E_STATE, "no trace (sv_batch_ransac_trace, then sv_batch_ransac)");
    const size_t per = (size_t)b->traced_trials * (b->trace_k + 3);
    if (out_trials) *out_trials = b->traced_trials;
    if (out_k) *out_k = b->trace_k;
    if (!out) return SV_OK;   // sizes only
    if (cap < (int64_t)per) return fail(SV_E_CAP, "trace needs %zu int32, buffer holds %lld", per, (long long)cap);
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(hipStreamSynchronize(b->stream));
    HIP_TRY(hipMemcpy(out, b->rtrace.as<int32_t>() + per * frame, sizeof(int32_t) * per, hipMemcpyDeviceToHost));
    return SV_OK;
}

int sv_batch_read_maskpoints(sv_batch* b, int frame, double* xyz, int64_t cap, int64_t* n) {
    if (!b || frame < 0 || frame >= b->frames || !n) return fail(SV_E_ARG, "bad args");
    if (!b->rres.p) return fail(SV_E_STATE, "no maskpoints (sv_batch_ransac first)");
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(hipStreamSynchronize(b->stream));
    const RansacRes r = ransac_res(b);
    int64_t k = 0;
    HIP_TRY(hipMemcpy(&k, r.mcount + frame, sizeof k, hipMemcpyDeviceToHost));
    *n = k;
    if (k > cap) return fail(SV_E_CAP, "capacity %lld < %lld", (long long)cap, (long long)k);
    if (k && xyz) {   // the frame's fp64 X, Y, Z from its packed points (the reference's arithmetic)
        HIP_TRY(b->mpts.ensure(sizeof(double) * 3 * (size_t)k));
        HIP_TRY(launch_maskpoints_xyz(b->mpk.as<uint32_t>() + (size_t)b->mcap * frame, k, b->rtab.as<double>(), b->H,
                                      b->W, b->mpts.as<double>(), b->stream));
        HIP_TRY(hipMemcpyAsync(xyz, b->mpts.p, sizeof(double) * 3 * k, hipMemcpyDeviceToHost, b->stream));
        HIP_TRY(hipStreamSynchronize(b->stream));
    }
    return SV_OK;
}

// ---------------------------------------------------------------------------
// RANSAC (functions.py:240-298): exact draw replay on the host, trials on the GPU
// ---------------------------------------------------------------------------
int sv_ransac_draw(uint32_t* mt_state, const double* pts, int64_t n, int64_t ld, int trials, int k, int32_t* sidx,
                   int32_t* tri, int* out_trials) {
    if (!mt_state || !out_trials || trials < 0 || k < 0 || ld < 3 || n < 0 || (n > 0 && !pts) ||
        (trials > 0 && (!sidx || !tri)))
        return fail(SV_E_ARG, "sv_ransac_draw: bad arguments");
    if (mt_state[624] > 624) return fail(SV_E_ARG, "sv_ransac_draw: MT index %u > 624", mt_state[624]);
    *out_trials = ransac_draw(mt_state, pts, n, ld, trials, k, sidx, tri);
    return SV_OK;
}

// The draws are replayed on the host in chunks of trials; each chunk's samples go up (asynchronously when the
// caller's sidx / tri are page-locked, as svx/ransac.py allocates them) and are evaluated on the device while the
// next chunk is drawn, so only the last chunk's evaluation is exposed after the replay.
int sv_ransac(uint32_t* mt_state, const double* pts, int64_t n, int64_t ld, int trials, int k, int32_t* sidx,
              int32_t* tri, double* out_abc, double* out_err, uint8_t* out_flag, int* out_trials) {
    if (!mt_state || !out_trials || trials < 0 || k < 0 || ld < 3 || n < 0 || (n > 0 && !pts) ||
        (trials > 0 && (!sidx || !tri)))
        return fail(SV_E_ARG, "sv_ransac: bad arguments");
    if (mt_state[624] > 624) return fail(SV_E_ARG, "sv_ransac: MT index %u > 624", mt_state[624]);
    *out_trials = 0;
    if (trials == 0 || n < k || n < 1 || n >= (1ll << 31)) return SV_OK;   // random.sample raises: no draw
    if (!out_abc || !out_err || !out_flag) return fail(SV_E_ARG, "sv_ransac: null outputs");
    int dev;
    if (int rc = current_device(&dev)) return rc;
    Device* d;
    if (int rc = dev_get(dev, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    hipStream_t s = d->stream;
    const size_t pbytes = sizeof(double) * (size_t)n * ld;
    const size_t ibytes = sizeof(int32_t) * ((size_t)trials * k + 3 * (size_t)trials);
    const size_t obytes = sizeof(double) * 4 * (size_t)trials + (size_t)trials;
    HIP_TRY(d->xyz.ensure(pbytes));
    HIP_TRY(d->aux.ensure(ibytes));
    HIP_TRY(d->aux2.ensure(obytes));
    int32_t* dsidx = d->aux.as<int32_t>();
    int32_t* dtri = dsidx + (size_t)trials * k;
    double* dabc = d->aux2.as<double>();
    double* derr = dabc + 3 * (size_t)trials;
    uint8_t* dflag = reinterpret_cast<uint8_t*>(derr + trials);
    HIP_TRY(hipMemcpyAsync(d->xyz.p, pts, pbytes, hipMemcpyHostToDevice, s));
    constexpr int kChunks = 4;
    const int per = (trials + kChunks - 1) / kChunks;
    for (int t0 = 0; t0 < trials; t0 += per) {
        const int c = std::min(per, trials - t0);
        if (ransac_draw(mt_state, pts, n, ld, c, k, sidx + (size_t)t0 * k, tri + 3 * (size_t)t0) != c)
            return fail(SV_E_ARG, "sv_ransac: draw replay stopped");
        HIP_TRY(hipMemcpyAsync(dsidx + (size_t)t0 * k, sidx + (size_t)t0 * k, sizeof(int32_t) * (size_t)c * k,
                               hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(dtri + 3 * (size_t)t0, tri + 3 * (size_t)t0, sizeof(int32_t) * 3 * (size_t)c,
                               hipMemcpyHostToDevice, s));
        HIP_TRY(launch_ransac_eval(d->xyz.as<double>(), ld, dsidx + (size_t)t0 * k, dtri + 3 * (size_t)t0, c, k,
                                   dabc + 3 * (size_t)t0, derr + t0, dflag + t0, s));
    }
    HIP_TRY(hipMemcpyAsync(out_abc, dabc, sizeof(double) * 3 * trials, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(out_err, derr, sizeof(double) * trials, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(out_flag, dflag, (size_t)trials, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *out_trials = trials;
    return SV_OK;
}

// ---------------------------------------------------------------------------
// a2-a6 as separate calls (functions.py:212-230, :300-323) for the stage drop-ins
// ---------------------------------------------------------------------------
namespace {
struct Locked {   // the current device's scratch + stream, under its mutex
    Device* d = nullptr;
    std::unique_lock<std::mutex> lk;
};
int lock_current(Locked& L) {
    int dev;
    if (int rc = current_device(&dev)) return rc;
    if (int rc = dev_get(dev, &L.d)) return rc;
    L.lk = std::unique_lock<std::mutex>(L.d->mu);
    return SV_OK;
}
}  // namespace

int sv_point_errors(const double* xyz, int64_t n, int64_t ld, const double* abcd, double* out) {
    if (n < 0 || ld < 3 || !abcd || (n > 0 && (!xyz || !out))) return fail(SV_E_ARG, "sv_point_errors: bad arguments");
    if (n == 0) return SV_OK;
    Locked L;
    if (int rc = lock_current(L)) return rc;
    hipStream_t s = L.d->stream;
    HIP_TRY(L.d->xyz.ensure(sizeof(double) * (size_t)n * ld));
    HIP_TRY(L.d->aux.ensure(sizeof(double) * (size_t)n));
    HIP_TRY(hipMemcpyAsync(L.d->xyz.p, xyz, sizeof(double) * (size_t)n * ld, hipMemcpyHostToDevice, s));
    HIP_TRY(launch_point_errors(L.d->xyz.as<double>(), n, ld, abcd, L.d->aux.as<double>(), s));
    HIP_TRY(hipMemcpyAsync(out, L.d->aux.p, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return SV_OK;
}

int sv_hue_histogram(const uint8_t* rgb, int64_t n, int64_t ld, int16_t* out_bins, uint32_t* out_hist,
                     int64_t* out_first) {
    if (n < 0 || ld < 3 || n >= INT32_MAX || (n > 0 && !rgb) || !out_hist || !out_first)
        return fail(SV_E_ARG, "sv_hue_histogram: bad arguments");
    for (int k = 0; k < 1000; ++k) {
        out_hist[k] = 0;
        out_first[k] = -1;
    }
    if (n == 0) return SV_OK;
    Locked L;
    if (int rc = lock_current(L)) return rc;
    hipStream_t s = L.d->stream;
    HIP_TRY(L.d->rgb.ensure((size_t)n * ld));
    HIP_TRY(L.d->aux.ensure(sizeof(int16_t) * (size_t)n + 8192));
    int16_t* bins = L.d->aux.as<int16_t>();
    uint32_t* hist = reinterpret_cast<uint32_t*>(L.d->aux.as<char>() + (sizeof(int16_t) * (size_t)n + 15) / 16 * 16);
    int32_t* first = reinterpret_cast<int32_t*>(hist + 1000);
    HIP_TRY(hipMemcpyAsync(L.d->rgb.p, rgb, (size_t)n * ld, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(hist, 0, sizeof(uint32_t) * 1000, s));
    HIP_TRY(hipMemsetAsync(first, 0x7f, sizeof(int32_t) * 1000, s));   // 0x7f7f7f7f > any index
    HIP_TRY(launch_hue_hist(L.d->rgb.as<uint8_t>(), n, ld, out_bins ? bins : nullptr, hist, first, s));
    std::vector<int32_t> f(1000);
    HIP_TRY(hipMemcpyAsync(out_hist, hist, sizeof(uint32_t) * 1000, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(f.data(), first, sizeof(int32_t) * 1000, hipMemcpyDeviceToHost, s));
    if (out_bins) HIP_TRY(hipMemcpyAsync(out_bins, bins, sizeof(int16_t) * (size_t)n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (int k = 0; k < 1000; ++k) out_first[k] = out_hist[k] ? (int64_t)f[k] : -1;
    return SV_OK;
}

static int select_impl(int mode, const double* vals, double thr, const int16_t* bins, const uint8_t* ok, int64_t n,
                       int64_t* out_idx, int64_t* out_n) {
    if (n < 0 || !out_n || (n > 0 && !out_idx) || (mode == 0 && n > 0 && !vals) ||
        (mode == 1 && (!ok || (n > 0 && !bins))))
        return fail(SV_E_ARG, "sv_select: bad arguments");
    *out_n = 0;
    if (n == 0) return SV_OK;
    Locked L;
    if (int rc = lock_current(L)) return rc;
    hipStream_t s = L.d->stream;
    const size_t in_bytes = mode == 0 ? sizeof(double) * (size_t)n : sizeof(int16_t) * (size_t)n;
    HIP_TRY(L.d->aux.ensure((in_bytes + 15) / 16 * 16 + 1024));
    HIP_TRY(L.d->aux2.ensure(sizeof(int64_t) * ((size_t)n + 1)));
    char* in = L.d->aux.as<char>();
    uint8_t* dok = reinterpret_cast<uint8_t*>(in + (in_bytes + 15) / 16 * 16);
    int64_t* idx = L.d->aux2.as<int64_t>();
    int64_t* cnt = idx + n;
    HIP_TRY(hipMemcpyAsync(in, mode == 0 ? (const void*)vals : (const void*)bins, in_bytes, hipMemcpyHostToDevice, s));
    if (mode == 1) HIP_TRY(hipMemcpyAsync(dok, ok, 1000, hipMemcpyHostToDevice, s));
    HIP_TRY(launch_select(mode, reinterpret_cast<const double*>(in), thr, reinterpret_cast<const int16_t*>(in), dok, n,
                          idx, cnt, s));
    int64_t k = 0;
    HIP_TRY(hipMemcpyAsync(&k, cnt, sizeof k, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (k) {
        HIP_TRY(hipMemcpyAsync(out_idx, idx, sizeof(int64_t) * (size_t)k, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    *out_n = k;
    return SV_OK;
}

int sv_select_less(const double* vals, int64_t n, double thr, int64_t* out_idx, int64_t* out_n) {
    return select_impl(0, vals, thr, nullptr, nullptr, n, out_idx, out_n);
}

int sv_select_bins(const int16_t* bins, int64_t n, const uint8_t* ok, int64_t* out_idx, int64_t* out_n) {
    for (int64_t i = 0; bins && i < n; ++i)
        if (bins[i] < 0 || bins[i] >= 1000) return fail(SV_E_ARG, "sv_select_bins: bin %d out of range", (int)bins[i]);
    return select_impl(1, nullptr, 0.0, bins, ok, n, out_idx, out_n);
}

// ---------------------------------------------------------------------------
// verification helpers
// ---------------------------------------------------------------------------
int sv_hue_lut(int device, int16_t* out_lut) { return sv_hue_lut_variant(device, 0, out_lut); }

int sv_hue_lut_variant(int device, int variant, int16_t* out_lut) {
    if (!out_lut) return fail(SV_E_ARG, "null");
    if (variant != 0 && variant != 1) return fail(SV_E_ARG, "sv_hue_lut_variant: variant %d not 0 or 1", variant);
    Device* d;
    if (int rc = dev_get(device, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    DevBuf buf;
    HIP_TRY(buf.ensure(sizeof(int16_t) << 24));
    hipError_t e = launch_hue_lut(buf.as<int16_t>(), variant, d->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(out_lut, buf.p, sizeof(int16_t) << 24, hipMemcpyDeviceToHost, d->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(d->stream);
    (void)hipFree(buf.p);
    HIP_TRY(e);
    return SV_OK;
}

int sv_delta_tables(int device, int H, int W, const sv_camera* cam, int8_t* dx, int8_t* dy) {
    if (!cam || !dx || !dy || H < 1 || W < 1) return fail(SV_E_ARG, "bad args");
    Device* d;
    if (int rc = dev_get(device, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    KParams p = make_params(H, W, 1, *cam);
    DevBuf bx, by, b8;
    HIP_TRY(bx.ensure(4 * 256 * p.dx_words));
    HIP_TRY(by.ensure(4 * 256 * p.dy_words));
    HIP_TRY(b8.ensure(256 * (size_t)(H + W)));
    int8_t* dx8 = b8.as<int8_t>();
    int8_t* dy8 = dx8 + 256 * (size_t)W;
    hipError_t e = launch_delta_tables(p, bx.as<uint32_t>(), by.as<uint32_t>(), dx8, dy8, d->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dx, dx8, 256 * (size_t)W, hipMemcpyDeviceToHost, d->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dy, dy8, 256 * (size_t)H, hipMemcpyDeviceToHost, d->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(d->stream);
    (void)hipFree(bx.p);
    (void)hipFree(by.p);
    (void)hipFree(b8.p);
    HIP_TRY(e);
    return SV_OK;
}

int sv_synth_frame(int device, int64_t frame_id, int H, int W, uint8_t* disp, uint8_t* bgr) {
    if (!disp || H < 1 || W < 4 || (W % 4)) return fail(SV_E_ARG, "bad args (W%%4 == 0 required)");
    Device* d;
    if (int rc = dev_get(device, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    sv_camera cam0{1, 1, 0, 0};
    KParams p = make_params(H, W, 1, cam0);
    DevBuf bd, bc;
    HIP_TRY(bd.ensure((size_t)H * W));
    HIP_TRY(bc.ensure((size_t)H * W * 3));
    hipError_t e = launch_synth(p, bd.as<uint8_t>(), bc.as<uint8_t>(), 1, frame_id, d->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(disp, bd.p, (size_t)H * W, hipMemcpyDeviceToHost, d->stream);
    if (e == hipSuccess && bgr) e = hipMemcpyAsync(bgr, bc.p, (size_t)H * W * 3, hipMemcpyDeviceToHost, d->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(d->stream);
    (void)hipFree(bd.p);
    (void)hipFree(bc.p);
    HIP_TRY(e);
    return SV_OK;
}


// ---------------------------------------------------------------------------
// disparity stage (functions.py:61-128)
// ---------------------------------------------------------------------------
namespace {
// StereoSGBM parameters with OpenCV's substitutions for zero / negative values
// (computeDisparitySGBM): P1 -> 2, P2 -> max(5, P1 + 1), preFilterCap ->
// max(cap, 15) | 1, uniquenessRatio < 0 -> 10, disp12MaxDiff <= 0 -> 1.
int make_sgbm(int H, int W, const sv_sgbm_params* prm, int max_disparity, int crop, SgbmK* k) {
    if (!prm) return fail(SV_E_ARG, "null sgbm params");
    if (prm->min_disp != 0) return fail(SV_E_ARG, "minDisparity must be 0 (got %d)", prm->min_disp);
    if (prm->num_disp != kSgD) return fail(SV_E_ARG, "numDisparities must be %d (got %d)", kSgD, prm->num_disp);
    const int SW = prm->block > 0 ? prm->block : 5;
    if (SW % 2 == 0 || SW > 63) return fail(SV_E_ARG, "blockSize must be odd and <= 63 (got %d)", SW);
    if (max_disparity < 1) return fail(SV_E_ARG, "max_disparity must be >= 1");
    std::memset(k, 0, sizeof *k);
    k->H = H;
    k->W = W;
    k->minX1 = kSgD;
    k->width1 = W - kSgD;
    k->SW2 = k->SH2 = SW / 2;
    k->P1 = prm->P1 > 0 ? prm->P1 : 2;
    k->P2 = std::max(prm->P2 > 0 ? prm->P2 : 5, k->P1 + 1);
    k->ftzero = std::max(prm->prefilter_cap, 15) | 1;
    k->uniq = prm->uniqueness >= 0 ? prm->uniqueness : 10;
    k->d12 = prm->disp12_max_diff > 0 ? prm->disp12_max_diff : 1;
    k->frame_px = (int64_t)H * W;
    // functions.py:111 filterSpeckles(disparity, 0, 4000, max_disparity - 5)
    k->new_val = 0;
    k->max_size = 4000;
    k->max_diff = max_disparity - 5;
    k->out_rows = crop ? std::min(390, H) : H;
    k->out_cols = crop ? std::max(W - 135, 0) : W;
    k->out_c0 = crop ? 135 : 0;
    k->out_stride = k->out_cols;
    k->scale = 256. / max_disparity;
    if (H < 1 || W <= kSgD || !sgbm_supported(*k))
        return fail(SV_E_ARG, "SGBM needs 1 <= H, %d + blockSize/2 < W <= 2048 (H=%d W=%d)", kSgD, H, W);
    return SV_OK;
}

int sgbm_check_flags(const uint32_t* flags, int n, hipStream_t s) {
    std::vector<uint32_t> fl(n);
    HIP_TRY(hipMemcpyAsync(fl.data(), flags, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (int i = 0; i < n; ++i)
        if (fl[i])
            return fail(SV_E_RANGE, "SGBM frame %d: a path cost left the int16 range (block cost sums above "
                                    "32,763: unsupported)", i);
    return SV_OK;
}

// upload a grey pair (or take the device's copies) and run StereoSGBM.compute into d->sg.d16
int sgbm_frame(Device* d, const uint8_t* L, const uint8_t* R, const SgbmK& k) {
    const size_t px = (size_t)k.frame_px;
    hipStream_t s = d->stream;
    HIP_TRY(d->sg_l.ensure(px));
    HIP_TRY(d->sg_r.ensure(px));
    HIP_TRY(d->sg.ensure(k, 1));
    HIP_TRY(hipMemcpyAsync(d->sg_l.p, L, px, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d->sg_r.p, R, px, hipMemcpyHostToDevice, s));
    HIP_TRY(launch_sgbm_compute(k, d->sg_l.as<uint8_t>(), d->sg_r.as<uint8_t>(), 1, d->sg.scratch(), s));
    return sgbm_check_flags(d->sg.flags.as<uint32_t>(), 1, s);
}
}  // namespace

int sv_lut_u8(const uint8_t* in, int64_t n, const uint8_t* lut, uint8_t* out) {
    if (n < 0 || (n > 0 && (!in || !out)) || !lut) return fail(SV_E_ARG, "sv_lut_u8: bad arguments");
    if (n == 0) return SV_OK;
    int dev;
    if (int rc = current_device(&dev)) return rc;
    Device* d;
    if (int rc = dev_get(dev, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    hipStream_t s = d->stream;
    HIP_TRY(d->sg_l.ensure((size_t)n));
    HIP_TRY(d->sg_hist.ensure(256));
    HIP_TRY(hipMemcpyAsync(d->sg_l.p, in, (size_t)n, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d->sg_hist.p, lut, 256, hipMemcpyHostToDevice, s));
    HIP_TRY(launch_lut(d->sg_l.as<uint8_t>(), n, d->sg_hist.as<uint8_t>(), d->sg_l.as<uint8_t>(), s));
    HIP_TRY(hipMemcpyAsync(out, d->sg_l.p, (size_t)n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return SV_OK;
}

int sv_grey_equalize(const uint8_t* bgr, int H, int W, uint8_t* out) {
    if (!bgr || !out || H < 0 || W < 0) return fail(SV_E_ARG, "sv_grey_equalize: bad arguments");
    const int64_t px = (int64_t)H * W;
    if (px == 0) return SV_OK;
    int dev;
    if (int rc = current_device(&dev)) return rc;
    Device* d;
    if (int rc = dev_get(dev, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    hipStream_t s = d->stream;
    HIP_TRY(d->sg_l.ensure((size_t)px * 3));
    HIP_TRY(d->sg_r.ensure((size_t)px));
    HIP_TRY(d->sg_hist.ensure(sizeof(uint32_t) * 256));
    HIP_TRY(hipMemcpyAsync(d->sg_l.p, bgr, (size_t)px * 3, hipMemcpyHostToDevice, s));
    HIP_TRY(launch_grey_equalize(d->sg_l.as<uint8_t>(), px, 1, d->sg_r.as<uint8_t>(), d->sg_hist.as<uint32_t>(), s));
    HIP_TRY(hipMemcpyAsync(out, d->sg_r.p, (size_t)px, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return SV_OK;
}

int sv_sgbm_compute(const uint8_t* L, const uint8_t* R, int H, int W, const sv_sgbm_params* prm, int16_t* out) {
    if (!L || !R || !out) return fail(SV_E_ARG, "sv_sgbm_compute: null buffer");
    SgbmK k;
    if (int rc = make_sgbm(H, W, prm, kSgD, 0, &k)) return rc;
    int dev;
    if (int rc = current_device(&dev)) return rc;
    Device* d;
    if (int rc = dev_get(dev, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    if (int rc = sgbm_frame(d, L, R, k)) return rc;
    HIP_TRY(hipMemcpyAsync(out, d->sg.d16.p, sizeof(int16_t) * k.frame_px, hipMemcpyDeviceToHost, d->stream));
    HIP_TRY(hipStreamSynchronize(d->stream));
    return SV_OK;
}

int sv_filter_speckles(int16_t* img, int H, int W, int new_val, int max_size, int max_diff) {
    if (!img || H < 0 || W < 0) return fail(SV_E_ARG, "sv_filter_speckles: bad arguments");
    const int64_t px = (int64_t)H * W;
    if (px == 0) return SV_OK;
    if (px > INT32_MAX) return fail(SV_E_ARG, "sv_filter_speckles: image too large");
    int dev;
    if (int rc = current_device(&dev)) return rc;
    Device* d;
    if (int rc = dev_get(dev, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    hipStream_t s = d->stream;
    SgbmK k;
    std::memset(&k, 0, sizeof k);
    k.H = H;
    k.W = W;
    k.frame_px = px;
    k.new_val = new_val;
    k.max_size = max_size;
    k.max_diff = max_diff;
    k.out_rows = 0;   // no scaled output
    k.scale = 1;
    HIP_TRY(d->sg.d16.ensure(sizeof(int16_t) * px));
    HIP_TRY(d->sg.par.ensure(sizeof(int32_t) * px));
    HIP_TRY(d->sg.size.ensure(sizeof(int32_t) * px));
    HIP_TRY(d->sg_filt.ensure(sizeof(int16_t) * px));
    HIP_TRY(hipMemcpyAsync(d->sg.d16.p, img, sizeof(int16_t) * px, hipMemcpyHostToDevice, s));
    HIP_TRY(launch_speckle_scale(k, 1, d->sg.scratch(), nullptr, d->sg_filt.as<int16_t>(), s));
    HIP_TRY(hipMemcpyAsync(img, d->sg_filt.p, sizeof(int16_t) * px, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return SV_OK;
}

int sv_disparity(const uint8_t* L, const uint8_t* R, int H, int W, const sv_sgbm_params* prm, int max_disparity,
                 int crop, uint8_t* out, int16_t* raw16, int16_t* filt16) {
    if (!L || !R || !out) return fail(SV_E_ARG, "sv_disparity: null buffer");
    SgbmK k;
    if (int rc = make_sgbm(H, W, prm, max_disparity, crop, &k)) return rc;
    int dev;
    if (int rc = current_device(&dev)) return rc;
    Device* d;
    if (int rc = dev_get(dev, &d)) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    hipStream_t s = d->stream;
    if (int rc = sgbm_frame(d, L, R, k)) return rc;
    if (raw16) HIP_TRY(hipMemcpyAsync(raw16, d->sg.d16.p, sizeof(int16_t) * k.frame_px, hipMemcpyDeviceToHost, s));
    const size_t ob = (size_t)k.out_rows * k.out_cols;
    HIP_TRY(d->sg_out.ensure(ob ? ob : 1));
    if (filt16) HIP_TRY(d->sg_filt.ensure(sizeof(int16_t) * k.frame_px));
    HIP_TRY(launch_speckle_scale(k, 1, d->sg.scratch(), d->sg_out.as<uint8_t>(),
                                 filt16 ? d->sg_filt.as<int16_t>() : nullptr, s));
    if (ob) HIP_TRY(hipMemcpyAsync(out, d->sg_out.p, ob, hipMemcpyDeviceToHost, s));
    if (filt16) HIP_TRY(hipMemcpyAsync(filt16, d->sg_filt.p, sizeof(int16_t) * k.frame_px, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return SV_OK;
}

// the pairs' shape: the batch's own, unless sv_batch_pair_shape chose the uncropped one
static void pair_shape(const sv_batch* b, int* H, int* W) {
    *H = b->pairH ? b->pairH : b->H;
    *W = b->pairW ? b->pairW : b->Wu;
}

int sv_batch_pair_shape(sv_batch* b, int H, int W) {
    if (!b) return fail(SV_E_ARG, "null batch");
    const bool own = H == b->H && W == b->Wu;
    // functions.py:122-124: disparity_scaled[0:390, 135:W] of an H x W pair
    if (!own && !(W > 135 && W - 135 == b->Wu && std::min(390, H) == b->H))
        return fail(SV_E_ARG, "pair shape %d x %d: the batch (%d x %d) must be the pair's shape or its crop "
                              "[0:390, 135:W]", H, W, b->H, b->Wu);
    if (!own && W % 8) return fail(SV_E_ARG, "batched SGBM needs the pair width %% 8 == 0 (W=%d)", W);
    int h0, w0;
    pair_shape(b, &h0, &w0);
    if (h0 != H || w0 != W) {   // a new shape: the grey and the BGR pairs are uploaded again
        for (DevBuf* x : {&b->pairL, &b->pairR, &b->bgrL, &b->bgrR}) {
            if (x->p) (void)hipFree(x->p);
            x->p = nullptr;
            x->bytes = 0;
        }
    }
    b->pairH = own ? 0 : H;
    b->pairW = own ? 0 : W;
    return SV_OK;
}

int sv_batch_synth_pair(sv_batch* b, int64_t first_frame_id) {
    if (!b) return fail(SV_E_ARG, "null batch");
    int H, W;
    pair_shape(b, &H, &W);
    if (W % 8) return fail(SV_E_ARG, "batched SGBM needs W %% 8 == 0 (W=%d)", W);
    if (W + kSgD > 4096) return fail(SV_E_ARG, "synthetic pairs need W <= %d", 4096 - kSgD);
    HIP_TRY(hipSetDevice(b->device));
    const size_t px = (size_t)H * W * b->frames;
    HIP_TRY(b->pairL.ensure(px));
    HIP_TRY(b->pairR.ensure(px));
    HIP_TRY(launch_synth_pair(b->pairL.as<uint8_t>(), b->pairR.as<uint8_t>(), H, W, b->frames, first_frame_id,
                              b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    return SV_OK;
}

int sv_batch_upload_pair(sv_batch* b, int frame, const uint8_t* L, const uint8_t* R) {
    if (!b || !L || !R || frame < 0 || frame >= b->frames) return fail(SV_E_ARG, "sv_batch_upload_pair: bad args");
    int H, W;
    pair_shape(b, &H, &W);
    if (W % 8) return fail(SV_E_ARG, "batched SGBM needs W %% 8 == 0 (W=%d)", W);
    HIP_TRY(hipSetDevice(b->device));
    const size_t px = (size_t)H * W;
    HIP_TRY(b->pairL.ensure(px * b->frames));
    HIP_TRY(b->pairR.ensure(px * b->frames));
    HIP_TRY(hipMemcpyAsync(b->pairL.as<uint8_t>() + px * frame, L, px, hipMemcpyHostToDevice, b->stream));
    HIP_TRY(hipMemcpyAsync(b->pairR.as<uint8_t>() + px * frame, R, px, hipMemcpyHostToDevice, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    return SV_OK;
}

int sv_batch_upload_bgr_pair(sv_batch* b, int frame, const uint8_t* L, const uint8_t* R) {
    if (!b || !L || !R || frame < 0 || frame >= b->frames) return fail(SV_E_ARG, "sv_batch_upload_bgr_pair: bad args");
    int H, W;
    pair_shape(b, &H, &W);
    if (W % 8) return fail(SV_E_ARG, "batched SGBM needs W %% 8 == 0 (W=%d)", W);
    HIP_TRY(hipSetDevice(b->device));
    const size_t px3 = (size_t)H * W * 3;
    HIP_TRY(b->bgrL.ensure(px3 * b->frames));
    HIP_TRY(b->bgrR.ensure(px3 * b->frames));
    HIP_TRY(hipMemcpyAsync(b->bgrL.as<uint8_t>() + px3 * frame, L, px3, hipMemcpyHostToDevice, b->stream));
    HIP_TRY(hipMemcpyAsync(b->bgrR.as<uint8_t>() + px3 * frame, R, px3, hipMemcpyHostToDevice, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    return SV_OK;
}

int sv_batch_synth_bgr_pair(sv_batch* b, int64_t first_frame_id) {
    if (!b) return fail(SV_E_ARG, "null batch");
    int H, W;
    pair_shape(b, &H, &W);
    if (W % 8) return fail(SV_E_ARG, "batched SGBM needs W %% 8 == 0 (W=%d)", W);
    if (W + kSgD > 4096) return fail(SV_E_ARG, "synthetic pairs need W <= %d", 4096 - kSgD);
    HIP_TRY(hipSetDevice(b->device));
    const size_t px3 = (size_t)H * W * 3 * b->frames;
    HIP_TRY(b->bgrL.ensure(px3));
    HIP_TRY(b->bgrR.ensure(px3));
    HIP_TRY(launch_synth_bgr_pair(b->bgrL.as<uint8_t>(), b->bgrR.as<uint8_t>(), H, W, b->frames, first_frame_id,
                                  b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    return SV_OK;
}

int sv_batch_preprocess(sv_batch* b, const uint8_t* lut, int sync) {
    if (!b || !lut) return fail(SV_E_ARG, "sv_batch_preprocess: bad args");
    if (!b->bgrL.p || !b->bgrR.p) return fail(SV_E_STATE, "no BGR pairs (sv_batch_synth_bgr_pair / upload_bgr_pair)");
    int H, W;
    pair_shape(b, &H, &W);
    const int64_t px = (int64_t)H * W;
    // the BGR pairs must hold every frame at the current pair shape (a partial upload after a shape change
    // would otherwise be read past its allocation)
    if (b->bgrL.bytes < (size_t)px * 3 * b->frames || b->bgrR.bytes < (size_t)px * 3 * b->frames)
        return fail(SV_E_STATE, "BGR pairs hold fewer bytes than %d frames of %d x %d x 3", b->frames, H, W);
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(b->glut.ensure(256));
    HIP_TRY(b->ghist.ensure(sizeof(uint32_t) * 256 * b->frames));
    HIP_TRY(b->pairL.ensure((size_t)px * b->frames));
    HIP_TRY(b->pairR.ensure((size_t)px * b->frames));
    HIP_TRY(hipMemcpyAsync(b->glut.p, lut, 256, hipMemcpyHostToDevice, b->stream));
    // preProcessImages' gamma table (functions.py:81-87) is applied as the pairs are read: cv2.LUT returns new
    // images, so the stored pairs stay the raw ones and every call corrects them exactly once (stereovision.py:44)
    const uint8_t* lut_d = b->glut.as<uint8_t>();
    // greyscale: BGR2GRAY + equalizeHist of both, functions.py:89-97 -> the SGBM pairs
    HIP_TRY(launch_grey_equalize(b->bgrL.as<uint8_t>(), px, b->frames, b->pairL.as<uint8_t>(),
                                 b->ghist.as<uint32_t>(), b->stream, lut_d));
    HIP_TRY(launch_grey_equalize(b->bgrR.as<uint8_t>(), px, b->frames, b->pairR.as<uint8_t>(),
                                 b->ghist.as<uint32_t>(), b->stream, lut_d));
    // the pipeline's colours: projectDisparityTo3d(disparity, 128, imgL) reads the gamma-corrected left image at
    // the disparity's own (y, x) (stereovision.py:44, :84), the top-left H x W of it when the disparity is cropped
    if (b->with_bgr)
        HIP_TRY(launch_copy_bgr_region(b->bgrL.as<uint8_t>(), H, W, b->bgr.as<uint8_t>(), b->H, b->W, b->Wu, b->frames,
                                       b->stream, lut_d));
    if (sync) HIP_TRY(hipStreamSynchronize(b->stream));
    return SV_OK;
}

// The cost volumes, placed (as K1's planes, k1_place): where the four streamed volumes land moves the walks by
// up to 7 % from one allocation to the next (30.9-33.1 ms per 128 frames over five processes of the same build,
// profiles/r04/ab_sgbm_volcontig.txt). A chunk of >= 64 frames allocates up to SVX_SGBM_TRIES (default 2)
// contiguous sets (all held until the end, at most 7/8 of the free memory), runs the first chunk's SGBM on each
// (the second of two runs timed) and keeps the fastest; the results are the same on every set.
static int sgbm_place(sv_batch* b, const SgbmK& k, int chunk, const uint8_t* left, const uint8_t* right) {
    int tries = 2;
    if (const char* e = svx_knob("SVX_SGBM_TRIES")) tries = std::max(1, std::atoi(e));
    const size_t vb = sgbm_volume_bytes(k) * (size_t)chunk, set_b = 4 * vb;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
    for (DevBuf& v : b->sg.vol) {   // the old volumes go (a new size)
        if (v.p) (void)hipFree(v.p);
        v.p = nullptr;
        v.bytes = 0;
    }
    if (chunk < 64) tries = 1;
    else tries = (int)std::min<size_t>((size_t)tries, std::max<size_t>(1, free_b / 8 * 7 / set_b));
    std::vector<std::array<DevBuf, 4>> sets((size_t)tries);
    int best = -1;
    float best_ms = 0.f;
    for (int t = 0; t < tries; ++t) {
        auto& c = sets[(size_t)t];
        hipError_t e = hipSuccess;
        for (int i = 0; i < 4 && e == hipSuccess; ++i) e = c[i].ensure(vb, true, 0, true);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            break;
        }
        if (tries > 1) {
            for (int i = 0; i < 4; ++i) b->sg.vol[i] = c[i];   // (borrowed: the set's owner is `sets`)
            SgbmScratch sc = b->sg.scratch();
            sc.flags = b->sgflags.as<uint32_t>();
            float ms = 0.f;
            for (int rep = 0; rep < 2 && e == hipSuccess; ++rep) {   // the second run is timed
                e = hipEventRecord(b->ev[0], b->stream);
                if (e == hipSuccess) e = launch_sgbm_compute(k, left, right, chunk, sc, b->stream);
                if (e == hipSuccess) e = hipEventRecord(b->ev[1], b->stream);
                if (e == hipSuccess) e = hipEventSynchronize(b->ev[1]);
                if (e == hipSuccess) e = hipEventElapsedTime(&ms, b->ev[0], b->ev[1]);
            }
            if (e != hipSuccess) break;
            if (t < 8) {
                b->place_ms[2][t] = ms;
                b->place_n[2] = t + 1;
            }
            if (best < 0 || ms < best_ms) {
                best = t;
                best_ms = ms;
            }
        } else {
            best = t;
        }
    }
    for (DevBuf& v : b->sg.vol) v = DevBuf{};
    int rc = SV_OK;
    if (best < 0) rc = fail(SV_E_HIP, "SGBM volumes: allocation failed (%zu bytes each)", vb);
    b->place_kept[2] = tries > 1 ? best : -1;
    for (int t = 0; t < (int)sets.size(); ++t)
        for (int i = 0; i < 4; ++i) {
            DevBuf& x = sets[(size_t)t][i];
            if (t == best) b->sg.vol[i] = x;
            else if (x.p) (void)hipFree(x.p);
        }
    b->sg.placed = rc == SV_OK;
    return rc;
}

int sv_batch_sgbm(sv_batch* b, const sv_sgbm_params* prm, int max_disparity, int chunk) {
    if (!b) return fail(SV_E_ARG, "null batch");
    if (!b->pairL.p || !b->pairR.p) return fail(SV_E_STATE, "no stereo pairs (sv_batch_synth_pair / upload_pair)");
    int H, W;
    pair_shape(b, &H, &W);
    const int crop = b->pairW ? 1 : 0;   // the batch is the pair's [0:390, 135:W] (sv_batch_pair_shape)
    SgbmK k;
    if (int rc = make_sgbm(H, W, prm, max_disparity, crop, &k)) return rc;
    k.out_stride = b->W;   // the batch's row stride (a cropped 889-wide row is stored in 896 bytes)
    if (b->pairL.bytes < (size_t)k.frame_px * b->frames || b->pairR.bytes < (size_t)k.frame_px * b->frames)
        return fail(SV_E_STATE, "stereo pairs hold fewer bytes than %d frames of %d x %d", b->frames, H, W);
    HIP_TRY(hipSetDevice(b->device));
    // 128 frames a chunk (64 GB of volumes at 544 x 1024): the walks' last round of workgroups is a smaller share
    // of a larger launch — 388 vs 401-424 us per frame at 32 and 403 at 64 (128 frames, alternating runs). The
    // default is capped by the device's free memory: the largest chunk whose scratch (what the batch does not
    // hold already, with DevBuf's 1/4 slack) fits in 3/4 of it, at least 1 frame.
    if (chunk <= 0) {
        chunk = std::min(128, b->frames);
        size_t fr = 0, tot = 0;
        HIP_TRY(hipMemGetInfo(&fr, &tot));
        const size_t per = (4 * sgbm_volume_bytes(k) + (size_t)k.frame_px * (2 * sizeof(int16_t) + 2 * sizeof(int32_t))) *
                           5 / 4;
        const size_t held = b->sg.held_bytes();
        const size_t budget = (fr + held) / 4 * 3;
        while (chunk > 1 && (size_t)chunk * per > budget) chunk = chunk * 3 / 4;
    }
    chunk = std::min(chunk, b->frames);
    // the range flags of every frame of the batch, checked once after the last chunk (no host sync between chunks)
    HIP_TRY(b->sgflags.ensure(sizeof(uint32_t) * b->frames));
    const size_t px = (size_t)k.frame_px, opx = (size_t)b->H * b->W;
    if (b->sg.vol[0].bytes < sgbm_volume_bytes(k) * (size_t)chunk) {
        HIP_TRY(b->sg.ensure_rest(k, chunk));
        if (int rc = sgbm_place(b, k, chunk, b->pairL.as<uint8_t>(), b->pairR.as<uint8_t>())) return rc;
    }
    HIP_TRY(b->sg.ensure(k, chunk));
    int t0, t1;
    HIP_TRY(hipEventRecord(b->ev[4], b->stream));
    HIP_TRY(b->timed_event(&t0));
    for (int f0 = 0; f0 < b->frames; f0 += chunk) {
        const int n = std::min(chunk, b->frames - f0);
        SgbmScratch sc = b->sg.scratch();
        sc.flags = b->sgflags.as<uint32_t>() + f0;
        HIP_TRY(launch_sgbm_compute(k, b->pairL.as<uint8_t>() + px * f0, b->pairR.as<uint8_t>() + px * f0, n, sc,
                                    b->stream));
        HIP_TRY(launch_speckle_scale(k, n, sc, input_disp(b) + opx * f0, nullptr, b->stream));
    }
    HIP_TRY(b->timed_event(&t1));
    HIP_TRY(hipEventRecord(b->ev[5], b->stream));
    if (int rc = sgbm_check_flags(b->sgflags.as<uint32_t>(), b->frames, b->stream)) return rc;
    if (t0 >= 0) b->pending[2].push_back({t0, t1});
    b->have_ms[2] = true;
    return SV_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// software-pipelined frame loop (stereovision.py:53-136 minus the cv2 drawing, over a sequence of batches)
// ---------------------------------------------------------------------------
// Every batch goes through the same stages on its slot's stream: input -> pre-pass -> maskpoints -> RANSAC draw ->
// RANSAC evaluation -> pipeline with the frames' own planes -> road raster + walk. A stage of batch k also waits
// for the same stage of batch k - 1 (an event on the other slot's stream), so each stage handles one batch at a
// time and in order; the evaluation of batch k also waits for batch k - 1's road pass. With two slots the steady
// state alternates two phases: batch k's evaluation beside batch k + 1's pre-pass and maskpoints, then batch k's
// pipeline and road pass beside batch k + 1's draw (one wave's dependent chain per frame). fillDisparity's previous cleaned frame is carried from
// batch to batch in a loop-owned buffer, so a sequence of batches cleans exactly as one long batch would.
namespace {
enum LoopStage { kLsInput = 0, kLsPrepass, kLsMaskpoints, kLsDraw, kLsEval, kLsPipeline, kLsRoad, kLsCount };
}

struct sv_loop {
    int device = 0;
    sv_loop_params prm{};
    sv_camera cam{};
    std::vector<sv_batch*> slot;
    std::vector<int64_t> slot_seq, slot_first;
    std::vector<std::array<hipEvent_t, kLsCount>> t0, t1;   // per slot: start / end of each stage (its last batch)
    hipEvent_t epoch = nullptr;
    // the previous batch's last cleaned frame (fillDisparity's previousDisparity), double-buffered: a submit reads
    // carry[cur] and writes carry[cur ^ 1], and only a submit that enqueued every stage makes its write current
    DevBuf carry[2];
    int carry_cur = 0;
    bool carry_valid = false;
    DevBuf gate;               // uint64: the last draw kernel whose grid is resident (its epoch = seq + 1)
    int64_t next = 0;          // sequence number of the next submitted batch
    int64_t pending = -1;      // the batch whose pipeline + road pass are not enqueued yet (see sv_loop_submit)
};

extern "C" {

int sv_loop_destroy(sv_loop* L) {
    if (!L) return SV_OK;
    (void)hipSetDevice(L->device);
    for (sv_batch* b : L->slot)
        if (b && b->stream) (void)hipStreamSynchronize(b->stream);
    for (auto& a : L->t0)
        for (auto& e : a)
            if (e) (void)hipEventDestroy(e);
    for (auto& a : L->t1)
        for (auto& e : a)
            if (e) (void)hipEventDestroy(e);
    if (L->epoch) (void)hipEventDestroy(L->epoch);
    for (DevBuf& c : L->carry)
        if (c.p) (void)hipFree(c.p);
    if (L->gate.p) (void)hipFree(L->gate.p);
    for (sv_batch* b : L->slot) sv_batch_destroy(b);
    delete L;
    return SV_OK;
}

int sv_loop_create(int device, const sv_loop_params* prm, const sv_camera* cam, const uint8_t* carmask,
                   sv_loop** out) {
    if (!prm || !cam || !out) return fail(SV_E_ARG, "sv_loop_create: null argument");
    *out = nullptr;
    const sv_loop_params& q = *prm;
    if (q.frames < 1 || q.slots < 1 || q.slots > 8 || (q.source != 0 && q.source != 1) || q.prepass < 0 ||
        q.prepass > 2 || q.road < 0 || q.road > 2 || (q.step != 1 && q.step != 2) || q.trials < 0 || q.k < 1)
        return fail(SV_E_ARG, "sv_loop_create: bad parameters (frames >= 1, 1 <= slots <= 8, source 0/1, prepass "
                              "0..2, road 0..2, step 1/2, trials >= 0, k >= 1)");
    // what a submit would only find out after enqueueing the input and pre-pass stages (the RANSAC and synthetic
    // input limits of batch_ransac_prepare / sv_batch_synth)
    if (q.trials > 4096 || q.k > 1024) return fail(SV_E_ARG, "sv_loop_create: RANSAC trials <= 4096, k <= 1024");
    if (q.H > 4096 || q.W > 4096) return fail(SV_E_ARG, "sv_loop_create: frames up to 4096 x 4096");
    if ((int64_t)grid_len(q.H, 2) * grid_len(q.W, 2) > 163840)
        return fail(SV_E_ARG, "sv_loop_create: more than 163,840 step-2 grid points per frame (RANSAC)");
    if (q.source == 1 && q.W % 8) return fail(SV_E_ARG, "sv_loop_create: synthetic frames need W %% 8 == 0 (W=%d)", q.W);
    sv_loop* L = new sv_loop;
    L->device = device;
    L->prm = q;
    L->cam = *cam;
    L->slot.assign((size_t)q.slots, nullptr);
    L->slot_seq.assign((size_t)q.slots, -1);
    L->slot_first.assign((size_t)q.slots, 0);
    L->t0.resize((size_t)q.slots);
    L->t1.resize((size_t)q.slots);
    for (auto& a : L->t0) a.fill(nullptr);
    for (auto& a : L->t1) a.fill(nullptr);
    int rc = SV_OK;
    for (int i = 0; i < q.slots && rc == SV_OK; ++i) {
        rc = sv_batch_create(device, q.frames, q.H, q.W, q.step, 1, 1, &L->slot[(size_t)i]);
        if (rc == SV_OK) L->slot[(size_t)i]->timing = false;
        if (rc == SV_OK && q.source == 0) {   // caller-fed: the frames the caller writes stay as written
            sv_batch* sb = L->slot[(size_t)i];
            const hipError_t ee = sb->raw.ensure(sb->disp.bytes);
            if (ee != hipSuccess) rc = fail(SV_E_HIP, "sv_loop_create: %s", hipGetErrorString(ee));
            else sb->keep_input = true;
        }
        if (rc == SV_OK && carmask) rc = sv_batch_set_mask(L->slot[(size_t)i], carmask);
        if (rc == SV_OK && q.road == 2) rc = sv_batch_road_map(L->slot[(size_t)i], 1);
        if (rc == SV_OK && q.road) rc = sv_batch_road_bits(L->slot[(size_t)i], 1);
    }
    hipError_t e = hipSuccess;
    if (rc == SV_OK) {
        e = hipSetDevice(device);
        for (int i = 0; i < q.slots && e == hipSuccess; ++i)
            for (int st = 0; st < kLsCount && e == hipSuccess; ++st) {
                e = hipEventCreate(&L->t0[(size_t)i][st]);
                if (e == hipSuccess) e = hipEventCreate(&L->t1[(size_t)i][st]);
            }
        if (e == hipSuccess) e = hipEventCreate(&L->epoch);
        for (DevBuf& c : L->carry)
            if (e == hipSuccess) e = c.ensure((size_t)L->slot[0]->H * L->slot[0]->W);
        if (e == hipSuccess) e = L->gate.ensure(sizeof(uint64_t));
        if (e == hipSuccess) e = hipMemset(L->gate.p, 0, sizeof(uint64_t));
        if (e != hipSuccess) rc = fail(SV_E_HIP, "sv_loop_create: %s", hipGetErrorString(e));
    }
    if (rc != SV_OK) {
        const std::string msg = g_err;
        sv_loop_destroy(L);
        g_err = msg;
        return rc;
    }
    *out = L;
    return SV_OK;
}

static int loop_flush(sv_loop* L);

// The batch the next sv_loop_submit processes (source 0: the caller fills it first); waits on the host until
// the batch that last used its slot has finished every stage.
int sv_loop_acquire(sv_loop* L, sv_batch** out) {
    if (!L || !out) return fail(SV_E_ARG, "sv_loop_acquire: null argument");
    const size_t s = (size_t)(L->next % L->prm.slots);
    HIP_TRY(hipSetDevice(L->device));
    if (L->pending >= 0 && (size_t)(L->pending % L->prm.slots) == s)
        if (int rc = loop_flush(L)) return rc;   // (one slot) the batch held there still has its tail to run
    if (L->slot_seq[s] >= 0) HIP_TRY(hipEventSynchronize(L->t1[s][kLsRoad]));
    *out = L->slot[s];
    return SV_OK;
}

// The pipeline and road pass of batch seq (slot s), behind a dispatch gate on the draw kernel of batch seq + 1
// when that has been enqueued (gate_epoch > 0): the draw's 4096 one-wave workgroups are a dependent chain each
// and must all be resident to finish in one pass, so they are placed first and the pipeline takes what is left
// of the CUs; launched together, the pipeline's workgroups would take the LDS and the draw would run in rounds.
static int loop_enqueue_tail(sv_loop* L, int64_t seq, uint64_t gate_epoch) {
    const sv_loop_params& q = L->prm;
    const size_t s = (size_t)(seq % q.slots), ps = (size_t)((seq + q.slots - 1) % q.slots);
    sv_batch* b = L->slot[s];
    hipStream_t st = b->stream;
    auto begin = [&](int stage) -> hipError_t {
        if (seq > 0 && ps != s) {
            hipError_t e = hipStreamWaitEvent(st, L->t1[ps][stage], 0);
            if (e != hipSuccess) return e;
        }
        return hipEventRecord(L->t0[s][stage], st);
    };
    auto end = [&](int stage) { return hipEventRecord(L->t1[s][stage], st); };
    if (gate_epoch) HIP_TRY(launch_loop_gate(L->gate.as<uint64_t>(), gate_epoch, 50.0, st));
#ifdef SVX_DIAG
    // DIAGNOSTIC probe (diagnostic build, SVX_LOOP_SIDE=1; results unchanged): one more fill pass over this batch's
    // raw frames into a scratch buffer, on a side stream, beside the pipeline and the next batch's draw — how much
    // does a pre-pass moved into that window slow them? (the three-deep front end)
    if (const char* e = svx_knob("SVX_LOOP_SIDE"); e && e[0] == '1' && b->keep_input) {
        static hipStream_t side = nullptr;
        static hipEvent_t ev = nullptr;
        static DevBuf scratch;
        if (!side) {
            HIP_TRY(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        }
        const int64_t px = (int64_t)b->H * b->W;
        HIP_TRY(scratch.ensure((size_t)px * b->frames));
        HIP_TRY(hipEventRecord(ev, st));
        HIP_TRY(hipStreamWaitEvent(side, ev, 0));
        HIP_TRY(launch_fill_prev(input_disp(b), scratch.as<uint8_t>(), nullptr, nullptr, nullptr, b->frames, px, side));
    }
#endif
    // the pipeline with every frame's own plane (stereovision.py:97-113)
    HIP_TRY(begin(kLsPipeline));
    if (int rc = sv_batch_pipeline_planes(b, &L->cam, q.point_thr, q.hist_thr, 0, 0)) return rc;
    HIP_TRY(end(kLsPipeline));
    // road raster + non-zero walk (+ imageRoadMap) (stereovision.py:131-156)
    HIP_TRY(begin(kLsRoad));
    if (q.road) {
        if (int rc = sv_batch_road_raster(b, 0)) return rc;
    }
    HIP_TRY(end(kLsRoad));
    if (L->pending == seq) L->pending = -1;
    return SV_OK;
}

static int loop_flush(sv_loop* L) {
    if (L->pending < 0) return SV_OK;
    HIP_TRY(hipSetDevice(L->device));
    return loop_enqueue_tail(L, L->pending, 0);
}

// Enqueue order of sv_loop_submit(k), slot s = k % slots, the previous batch k - 1 on slot ps:
//   slot s:  input(k) -> pre-pass(k) -> maskpoints(k)   [without a carmask the host reads k's counts: they size
//            the draw launch; with one, the mask's step-2 points bound them and nothing is read]
//   slot s:  draw(k)  (after batch k - 1's evaluation: a frame's evaluation needs a whole CU's LDS)
//   slot ps: gate(draw(k) resident) -> pipeline(k - 1) -> road(k - 1)
//   slot s:  evaluation(k)  (after road(k - 1): beside pre-pass(k + 1) and maskpoints(k + 1), which use no LDS)
// so batch k's pipeline and road pass are enqueued by the next submit (or by sv_loop_wait / _timeline).
int sv_loop_submit(sv_loop* L, int64_t first_frame_id, int64_t* out_seq) {
    if (!L) return fail(SV_E_ARG, "sv_loop_submit: null loop");
    if (first_frame_id < 0) return fail(SV_E_ARG, "sv_loop_submit: first_frame_id >= 0");
    const sv_loop_params& q = L->prm;
    const int64_t seq = L->next;
    const size_t s = (size_t)(seq % q.slots), ps = (size_t)((seq + q.slots - 1) % q.slots);
    sv_batch* b = L->slot[s];
    hipStream_t st = b->stream;
    HIP_TRY(hipSetDevice(L->device));
    if (q.slots == 1) {   // one slot: nothing to overlap, the previous batch's tail first
        if (int rc = loop_flush(L)) return rc;
    }
    if (seq == 0) HIP_TRY(hipEventRecord(L->epoch, st));
    auto begin = [&](int stage) -> hipError_t {
        if (seq > 0 && ps != s) {   // the same stage of the batch before, on the other slot's stream
            hipError_t e = hipStreamWaitEvent(st, L->t1[ps][stage], 0);
            if (e != hipSuccess) return e;
        }
        return hipEventRecord(L->t0[s][stage], st);
    };
    auto end = [&](int stage) { return hipEventRecord(L->t1[s][stage], st); };
    // input: for synthetic frames, the batch's global frame ids generated on the device
    HIP_TRY(begin(kLsInput));
    if (q.source == 1) {
        if (b->Wu != b->W) return fail(SV_E_ARG, "synthetic frames need W %% 8 == 0 (W=%d)", b->Wu);
        HIP_TRY(launch_synth(b->kp, input_disp(b), b->bgr.as<uint8_t>(), b->frames, first_frame_id, st));
    }
    HIP_TRY(end(kLsInput));
    // pre-pass (stereovision.py:53-76): frame 0 cleaned with the previous batch's last cleaned frame
    HIP_TRY(begin(kLsPrepass));
    bool carried = false;
    {   // option 0 (no pre-pass) still runs: a caller-fed slot (keep_input) holds its frames in `raw`, and the
        // impl copies them into `disp`, which every later stage reads
        const uint8_t* prev = q.prepass == 1 && L->carry_valid ? L->carry[L->carry_cur].as<uint8_t>() : nullptr;
        if (int rc = batch_prepass_impl(b, q.prepass, prev)) return rc;
        if (q.prepass == 1) {
            const size_t px = (size_t)b->H * b->W;
            HIP_TRY(hipMemcpyAsync(L->carry[L->carry_cur ^ 1].p, b->disp.as<uint8_t>() + px * (b->frames - 1), px,
                                   hipMemcpyDeviceToDevice, st));
            carried = true;
        }
    }
    HIP_TRY(end(kLsPrepass));
    // maskpoints (stereovision.py:74-85): the masked step-2 points of every frame, their counts to the host
    HIP_TRY(begin(kLsMaskpoints));
    if (int rc = batch_ransac_prepare(b, &L->cam, q.trials, q.k)) return rc;
    HIP_TRY(end(kLsMaskpoints));
    // RANSAC draw (stereovision.py:94): frame g draws after random.seed(seed_base + g); sized from the carmask's
    // bound of the counts (no host wait; without a mask the host waits here for this batch's counts, with the
    // previous batch's evaluation already enqueued)
    if (seq > 0 && ps != s) HIP_TRY(hipStreamWaitEvent(st, L->t1[ps][kLsEval], 0));
    HIP_TRY(begin(kLsDraw));
    if (int rc = batch_ransac_launch(b, &L->cam, q.seed_base, first_frame_id, q.trials, q.k, st, 1,
                                     L->gate.as<uint64_t>(), (uint64_t)seq + 1))
        return rc;
    HIP_TRY(end(kLsDraw));
    // the previous batch's pipeline and road pass, gated on this draw's dispatch
    if (L->pending >= 0) {
        if (int rc = loop_enqueue_tail(L, L->pending, (uint64_t)seq + 1)) return rc;
    }
    // RANSAC evaluation, after the previous batch's road pass (SVX_LOOP_EVAL_AFTER=pipeline, diagnostic build:
    // after its pipeline, beside the road pass)
    {   // (SVX_LOOP_EVAL_AFTER=none, diagnostic build: after this batch's draw only, so its workgroups take the CUs
        // the previous batch's pipeline drains, beside that batch's road pass)
        const char* ea = svx_knob("SVX_LOOP_EVAL_AFTER");
        const int dep = ea && ea[0] == 'p' ? kLsPipeline : ea && ea[0] == 'n' ? -1 : kLsRoad;
        if (seq > 0 && ps != s && dep >= 0) HIP_TRY(hipStreamWaitEvent(st, L->t1[ps][dep], 0));
    }
    HIP_TRY(begin(kLsEval));
    if (int rc = batch_ransac_launch(b, &L->cam, q.seed_base, first_frame_id, q.trials, q.k, st, 2)) return rc;
    HIP_TRY(end(kLsEval));
    if (carried) {   // every stage enqueued: this batch's last cleaned frame is the next batch's previous one
        L->carry_cur ^= 1;
        L->carry_valid = true;
    }
    L->pending = seq;
    L->slot_seq[s] = seq;
    L->slot_first[s] = first_frame_id;
    L->next = seq + 1;
    if (out_seq) *out_seq = seq;
    return SV_OK;
}

static int loop_slot_of(sv_loop* L, int64_t seq, size_t* out) {
    if (!L || seq < 0) return fail(SV_E_ARG, "sv_loop: bad arguments");
    const size_t s = (size_t)(seq % L->prm.slots);
    if (L->slot_seq[s] != seq)
        return fail(SV_E_STATE, "sv_loop: batch %lld is not held (submitted: %lld, slots: %d)", (long long)seq,
                    (long long)L->next, L->prm.slots);
    *out = s;
    return SV_OK;
}

int sv_loop_wait(sv_loop* L, int64_t seq) {
    size_t s;
    if (int rc = loop_slot_of(L, seq, &s)) return rc;
    if (int rc = loop_flush(L)) return rc;
    HIP_TRY(hipSetDevice(L->device));
    HIP_TRY(hipEventSynchronize(L->t1[s][kLsRoad]));
    return SV_OK;
}

int sv_loop_batch(sv_loop* L, int64_t seq, sv_batch** out, int64_t* first_frame_id) {
    size_t s;
    if (!out) return fail(SV_E_ARG, "sv_loop_batch: null out");
    if (int rc = loop_slot_of(L, seq, &s)) return rc;
    // the batch's pipeline and road pass may not be enqueued yet (the next submit enqueues them): enqueue them and
    // wait for them, so that sv_batch_read_* of the returned batch never mixes this batch's RANSAC with the points
    // and road images of the batch the slot held before
    if (L->pending == seq)
        if (int rc = loop_flush(L)) return rc;
    HIP_TRY(hipSetDevice(L->device));
    HIP_TRY(hipEventSynchronize(L->t1[s][kLsRoad]));
    *out = L->slot[s];
    if (first_frame_id) *first_frame_id = L->slot_first[s];
    return SV_OK;
}

int sv_loop_timeline(sv_loop* L, int64_t seq, double* out) {
    size_t s;
    if (!out) return fail(SV_E_ARG, "sv_loop_timeline: null out");
    if (int rc = loop_slot_of(L, seq, &s)) return rc;
    if (int rc = loop_flush(L)) return rc;
    HIP_TRY(hipSetDevice(L->device));
    HIP_TRY(hipEventSynchronize(L->t1[s][kLsRoad]));
    for (int st = 0; st < kLsCount; ++st) {
        float a = 0.f, z = 0.f;
        HIP_TRY(hipEventElapsedTime(&a, L->epoch, L->t0[s][st]));
        HIP_TRY(hipEventElapsedTime(&z, L->epoch, L->t1[s][st]));
        out[2 * st] = a;
        out[2 * st + 1] = z;
    }
    return SV_OK;
}

}  // extern "C"
