// SGBM stage: parameters, scratch and launchers
// (kernels/sgbm.hip). numDisparities is fixed at 128 (functions.py:18,26:
// max_disparity = 128): the kernels hold one pixel's 128 path costs as 64
// lanes x 2; minDisparity is 0 as in the reference.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace svx {

constexpr int kSgD = 128;      // numDisparities
constexpr int kSgScale = 16;   // StereoMatcher::DISP_SCALE

struct SgbmK {
    int H, W, width1, minX1;          // width1 = W - 128 cost columns (image columns 128..W-1)
    int SW2, SH2, P1, P2, ftzero, uniq, d12;
    int64_t frame_px;
    int new_val, max_size, max_diff;  // filterSpeckles
    int out_rows, out_cols, out_c0;   // scaled output geometry (crop: 390 x (W - 135) at column 135)
    int out_stride;                   // bytes between output rows (>= out_cols); a frame is out_rows of them
    double scale;                     // 256. / max_disparity
};

// Device scratch for a chunk of frames: four int16 cost volumes (frames x H x
// width1 x 128) — hl1 holds the horizontal sums, then L1, then P — plus the
// int16 disparity (raw: computeDisparitySGBM's; d16: after compute's medianBlur),
// union-find parents, component sizes and overflow flags.
struct SgbmScratch {
    uint32_t *hl1, *c, *l2, *l3;
    int16_t *raw, *d16;
    int32_t *parent, *size;
    uint32_t* flags;   // per frame: 1 = an L value left int16 (unsupported)
};

bool sgbm_supported(const SgbmK& k);
size_t sgbm_volume_bytes(const SgbmK& k);   // one volume, one frame
// StereoSGBM.compute of every frame into s.d16 (frames x H x W int16, x16):
// computeDisparitySGBM into s.raw, then medianBlur 3 into s.d16.
hipError_t launch_sgbm_compute(const SgbmK& k, const uint8_t* left, const uint8_t* right, int frames,
                               const SgbmScratch& s, hipStream_t st);
// filterSpeckles of s.d16 (frames x H x W) + TOZERO + scaling into out.
hipError_t launch_speckle_scale(const SgbmK& k, int frames, const SgbmScratch& s, uint8_t* out, int16_t* filt,
                                hipStream_t st);
hipError_t launch_lut(const uint8_t* in, int64_t n, const uint8_t* lut, uint8_t* out, hipStream_t s);
// BGR2GRAY + equalizeHist of `frames` images of px pixels; hist: frames x 256 scratch; lut (nullable): a table
// applied to every channel as it is read (the gamma of preProcessImages; the input is not rewritten).
hipError_t launch_grey_equalize(const uint8_t* bgr, int64_t px, int frames, uint8_t* grey, uint32_t* hist,
                                hipStream_t s, const uint8_t* lut = nullptr);
hipError_t launch_synth_pair(uint8_t* left, uint8_t* right, int H, int W, int frames, int64_t first, hipStream_t s);
// Synthetic BGR pairs: the synthetic pair's texture with a per-source-pixel channel jitter (so left (y, x) and
// right (y, x - D) carry the same colour), frames x H x W x 3 each.
hipError_t launch_synth_bgr_pair(uint8_t* left, uint8_t* right, int H, int W, int frames, int64_t first,
                                 hipStream_t s);
// dst rows (frames x H rows of Wu * 3 bytes at a stride of W * 3) from the top-left of src frames of Hp x Wp x 3,
// through lut (nullable) byte by byte
hipError_t launch_copy_bgr_region(const uint8_t* src, int Hp, int Wp, uint8_t* dst, int H, int W, int Wu, int frames,
                                  hipStream_t s, const uint8_t* lut = nullptr);

// Synthetic rectified pair (numpy twin: oracle/sgbm.py synth_pair): texture
// T(frame, y, u) from the splitmix64 finaliser; row y's true disparity is the
// synthetic road's in SGBM units; left(y, x) = T(y, x), right(y, x) = T(y, x + D(y)).
__host__ __device__ inline int sgbm_pair_disparity(int y) {
    int t = 3 * (y - 200);
    t = t >= 0 ? t / 10 : -((-t + 9) / 10);
    return t < 0 ? 0 : (t > 127 ? 127 : t);
}

__host__ __device__ inline uint8_t sgbm_pair_texture(int64_t frame, int H, int y, int u) {
    uint64_t z = ((uint64_t)frame * (uint64_t)H + (uint64_t)y) * 4096ull + (uint64_t)u + 0x57E2E0000000000ull;
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint8_t)(48 + (z & 0x9F));
}

}  // namespace svx
