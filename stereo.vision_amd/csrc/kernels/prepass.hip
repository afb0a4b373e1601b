// Disparity pre-pass kernels (gfx950): the per-pixel uint8 stages that feed
// the projection, all HBM-bound byte streams.
//
//  * fill_prev_kernel  — fillDisparity (functions.py:141-148) applied frame
//                        after frame as performStereoVision does with
//                        prev_disp (stereovision.py:56-60, functions.py:131-135):
//                        cleaned_f = raw_f > 2 ? raw_f : sat8(raw_f + cleaned_{f-1})
//                        (cv2.threshold(..., 2, 255, BINARY) -> NOT -> masked
//                        copy of prev -> cv2.add, saturating). The frame
//                        recurrence runs in registers: one lane owns 4 pixels
//                        and walks the batch's frames in order, 8 frames of
//                        loads in flight.
//  * fill_mean_kernel  — fillAltDisparity (functions.py:150-162): per row, the
//                        mean of the non-zero values (0 if none), assigned with
//                        numpy's float->uint8 truncation to every pixel < 2.
//                        The mean of uint8 values is exact in fp64 until the
//                        final division, and a non-integer S/C is >= 1/C away
//                        from an integer, so trunc(S/C) == S div C.
//                        One wave per row.
//  * mask_kernel       — maskDisparity (functions.py:169-172):
//                        bitwise_and(d, d, mask=carmask) = carmask != 0 ? d : 0,
//                        with the mask pre-expanded to 0x00 / 0xFF bytes.
#include "../svx_launch.h"

namespace svx {

__device__ __forceinline__ uint32_t fill4(uint32_t raw, uint32_t prev) {
    uint32_t out = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t r = (raw >> (8 * k)) & 0xFF, q = (prev >> (8 * k)) & 0xFF;
        const uint32_t s = r + q;
        out |= (r > 2 ? r : (s > 255 ? 255 : s)) << (8 * k);
    }
    return out;
}

// words = pixels / 4 per frame; disp may equal out (in place). U frames of loads in flight per lane.
template <int U>
__global__ __launch_bounds__(256) void fill_prev_kernel(const uint32_t* raw, uint32_t* out, uint32_t* masked,
                                                        const uint32_t* __restrict__ mask, const uint32_t* prev0,
                                                        int frames, int64_t words) {
    constexpr int kFillUnroll = U;
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= words) return;
    uint32_t c = prev0 ? prev0[i] : 0u;
    bool have = prev0 != nullptr;
    const uint32_t m = mask ? mask[i] : 0u;
    for (int f0 = 0; f0 < frames; f0 += kFillUnroll) {
        uint32_t r[kFillUnroll];
#pragma unroll
        for (int u = 0; u < kFillUnroll; ++u)
            r[u] = f0 + u < frames ? raw[(int64_t)(f0 + u) * words + i] : 0u;
#pragma unroll
        for (int u = 0; u < kFillUnroll; ++u) {
            if (f0 + u >= frames) break;
            c = have ? fill4(r[u], c) : r[u];
            have = true;
            out[(int64_t)(f0 + u) * words + i] = c;
            if (masked) masked[(int64_t)(f0 + u) * words + i] = c & m;
        }
    }
}

// The same recurrence with loads and stores in different waves. gfx9's vmcnt counts a wave's loads and stores
// together, in issue order, so in fill_prev_kernel every wait for the next frames' loads also waits for the
// acknowledgements of the stores issued before them: the store latency sits on the load chain. Here each
// 128-lane workgroup owns 64 words of the frame: wave 0 only loads (F frames of its 64 words, waits for them, puts
// them in an LDS slot), wave 1 only computes and stores (its 64 words' recurrence in registers, the cleaned words
// out), two LDS slots of F frames alternating, one barrier per F frames. Wave 1 never waits on vmcnt (the barrier
// here is s_barrier with an LDS wait only, no global fence), and wave 0's next F frames are in flight while wave 1
// works through the previous slot. disp may equal out (in place): a frame's word is loaded before it is written.
template <int F>
__global__ __launch_bounds__(128) void fill_prev_split_kernel(const uint32_t* raw, uint32_t* out, uint32_t* masked,
                                                              const uint32_t* __restrict__ mask,
                                                              const uint32_t* prev0, int frames, int64_t words) {
    __shared__ uint32_t ring[2][F][64];
    const int lane = threadIdx.x & 63;
    const bool loader = threadIdx.x < 64;
    const int64_t i = blockIdx.x * 64ll + lane;
    const bool in = i < words;
    const int64_t ic = in ? i : words - 1;   // lanes past the frame load a valid word and store nothing
    const int phases = (frames + F - 1) / F;
    const auto sync = [] {   // LDS writes complete, then the workgroup barrier; no wait on global stores
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    if (loader) {
        uint32_t r[F];
        const auto load = [&](int f0) {   // phase f0 / F: whole phases unconditionally, the last one clamped
            if (f0 + F <= frames) {
#pragma unroll
                for (int u = 0; u < F; ++u) r[u] = __builtin_nontemporal_load(raw + (int64_t)(f0 + u) * words + ic);
            } else {
#pragma unroll
                for (int u = 0; u < F; ++u)
                    r[u] = __builtin_nontemporal_load(raw + (int64_t)min(f0 + u, frames - 1) * words + ic);
            }
        };
        load(0);
        for (int ph = 0; ph < phases; ++ph) {
#pragma unroll
            for (int u = 0; u < F; ++u) ring[ph & 1][u][lane] = r[u];
            if (ph + 1 < phases) load((ph + 1) * F);
            sync();   // slot ph & 1 holds phase ph; the writer has finished phase ph - 1
        }
    } else {
        // fill4(v, 0) = v: without a previous frame the first frame passes through unchanged
        uint32_t c = prev0 ? prev0[ic] : 0u;
        const uint32_t m = masked && mask ? mask[ic] : 0u;
        for (int ph = 0; ph < phases; ++ph) {
            sync();
            const int f0 = ph * F, nf = min(F, frames - f0);
            uint32_t* o = out + (int64_t)f0 * words + i;
            if (nf == F && !masked) {   // uniform: a whole phase, every read issued before the first wait
                uint32_t v[F];
#pragma unroll
                for (int u = 0; u < F; ++u) v[u] = ring[ph & 1][u][lane];
#pragma unroll
                for (int u = 0; u < F; ++u) {
                    c = fill4(v[u], c);
                    if (in) o[(int64_t)u * words] = c;
                }
            } else {   // the batch's last, partial phase, or a masked copy too
                for (int u = 0; u < nf; ++u) {
                    c = fill4(ring[ph & 1][u][lane], c);
                    if (in) {
                        o[(int64_t)u * words] = c;
                        if (masked) masked[(int64_t)(f0 + u) * words + i] = c & m;
                    }
                }
            }
        }
    }
}

// One wave per row of W bytes (W % 4 == 0); rows = frames * H.
__global__ __launch_bounds__(256) void fill_mean_kernel(uint8_t* disp, uint8_t* masked, const uint8_t* __restrict__ mask,
                                                        int64_t rows, int H, int W, int Wrow) {
    const int64_t row = blockIdx.x * 4ll + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int lane = lane_id();
    uint32_t* rp = reinterpret_cast<uint32_t*>(disp + row * W);
    const int words = W / 4;
    uint32_t sum = 0, cnt = 0;
    for (int w = lane; w < words; w += kWave) {
        const uint32_t v = rp[w];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t b = 4 * w + k < Wrow ? (v >> (8 * k)) & 0xFF : 0u;   // stride padding: not the row's
            sum += b;
            cnt += b != 0;
        }
    }
    sum = wave_sum(sum);
    cnt = wave_sum(cnt);
    const uint32_t mean = cnt ? sum / cnt : 0u;   // numpy: nan mean -> 0.0; uint8 <- trunc(mean)
    const int64_t mrow = (row % H) * (int64_t)W;
    uint32_t* mp = masked ? reinterpret_cast<uint32_t*>(masked + row * W) : nullptr;
    const uint32_t* kp = mask ? reinterpret_cast<const uint32_t*>(mask + mrow) : nullptr;
    for (int w = lane; w < words; w += kWave) {
        const uint32_t v = rp[w];
        uint32_t o = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t b = (v >> (8 * k)) & 0xFF;
            o |= (b < 2 && 4 * w + k < Wrow ? mean : b) << (8 * k);
        }
        rp[w] = o;
        if (mp) mp[w] = o & kp[w];
    }
}

__global__ __launch_bounds__(256) void mask_kernel(const uint32_t* disp, uint32_t* out, const uint32_t* __restrict__ mask,
                                                   int64_t words_per_frame, int64_t total_words) {
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total_words; i += (int64_t)gridDim.x * 256)
        out[i] = disp[i] & mask[i % words_per_frame];
}

// Expand a grey mask to 0x00 / 0xFF bytes: bitwise_and(..., mask=m) keeps a pixel iff m != 0.
__global__ __launch_bounds__(256) void mask_bytes_kernel(const uint8_t* m, uint8_t* out, int64_t n) {
    const int64_t i = blockIdx.x * 256ll + threadIdx.x;
    if (i < n) out[i] = m[i] ? 0xFF : 0x00;
}

hipError_t launch_mask_bytes(const uint8_t* m, uint8_t* out, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(mask_bytes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, m, out, n);
    return hipGetLastError();
}

constexpr int kFillSplitFrames = 0;   // measured: the split is not faster

hipError_t launch_fill_prev(const uint8_t* raw, uint8_t* out, uint8_t* masked, const uint8_t* mask_ff,
                            const uint8_t* prev0, int frames, int64_t frame_px, hipStream_t s) {
    if (frames <= 0 || frame_px <= 0) return hipSuccess;
    if (frame_px % 4) return hipErrorInvalidValue;
    const int64_t words = frame_px / 4;
    // A/B knob SVX_FILL="U,B": frames of loads in flight per lane (8, 16, 32) and the workgroup size. 64-lane
    // workgroups spread a frame's 2,176 waves evenly over the 256 CUs (256-lane ones leave 32 CUs a third
    // workgroup): 1.47 vs 1.53 ms per 4096 frames; 16 and 32 frames in flight are slower (1.58-1.63, 1.77 ms)
    int U = 8, B = 64;
    if (const char* e = svx_knob("SVX_FILL")) std::sscanf(e, "%d,%d", &U, &B);
    if (B != 64 && B != 128 && B != 256) B = 256;
    const dim3 grid((unsigned)((words + B - 1) / B)), block(B);
    const auto* r = reinterpret_cast<const uint32_t*>(raw);
    auto* o = reinterpret_cast<uint32_t*>(out);
    auto* m = reinterpret_cast<uint32_t*>(masked);
    const auto* k = reinterpret_cast<const uint32_t*>(mask_ff);
    const auto* p = reinterpret_cast<const uint32_t*>(prev0);
    // the loader / writer split (fill_prev_split_kernel), F frames a phase; SVX_FILL_SPLIT=0 (diagnostic build)
    // keeps the one-wave kernel below for A/B
    int F = kFillSplitFrames;
    if (const char* e = svx_knob("SVX_FILL_SPLIT")) F = std::atoi(e);
    if (F > 0) {
        const dim3 g2((unsigned)((words + 63) / 64)), b2(128);
        if (F >= 32) hipLaunchKernelGGL(fill_prev_split_kernel<32>, g2, b2, 0, s, r, o, m, k, p, frames, words);
        else if (F >= 16) hipLaunchKernelGGL(fill_prev_split_kernel<16>, g2, b2, 0, s, r, o, m, k, p, frames, words);
        else hipLaunchKernelGGL(fill_prev_split_kernel<8>, g2, b2, 0, s, r, o, m, k, p, frames, words);
        return hipGetLastError();
    }
    if (U >= 32) hipLaunchKernelGGL(fill_prev_kernel<32>, grid, block, 0, s, r, o, m, k, p, frames, words);
    else if (U >= 16) hipLaunchKernelGGL(fill_prev_kernel<16>, grid, block, 0, s, r, o, m, k, p, frames, words);
    else hipLaunchKernelGGL(fill_prev_kernel<8>, grid, block, 0, s, r, o, m, k, p, frames, words);
    return hipGetLastError();
}

hipError_t launch_fill_mean(uint8_t* disp, uint8_t* masked, const uint8_t* mask_ff, int frames, int H, int W,
                            int Wrow, hipStream_t s) {
    const int64_t rows = (int64_t)frames * H;
    if (rows <= 0) return hipSuccess;
    if (W % 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(fill_mean_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, disp, masked, mask_ff,
                       rows, H, W, Wrow);
    return hipGetLastError();
}

hipError_t launch_mask(const uint8_t* disp, uint8_t* out, const uint8_t* mask_ff, int frames, int64_t frame_px,
                       hipStream_t s) {
    if (frames <= 0 || frame_px <= 0) return hipSuccess;
    if (frame_px % 4) return hipErrorInvalidValue;
    const int64_t wpf = frame_px / 4, total = wpf * frames;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(mask_kernel, dim3((unsigned)blocks), dim3(256), 0, s, reinterpret_cast<const uint32_t*>(disp),
                       reinterpret_cast<uint32_t*>(out), reinterpret_cast<const uint32_t*>(mask_ff), wpf, total);
    return hipGetLastError();
}

}  // namespace svx
