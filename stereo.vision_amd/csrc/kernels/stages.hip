// The reference's per-stage functions a2-a6 as separate device
// calls, for the drop-ins that replace them one by one (functions.py:212-230,
// :300-323). The fused batch pipeline computes the same decisions in one pass;
// these serve a caller that runs the stages itself (stereovision.py:97-106).
//
//  * point_errors_kernel — calculatePointErrors (functions.py:300-312):
//      |(P.abc - 1) / d| in fp64, P.abc in the order OpenBLAS' dgemv uses for
//      an (N,3) x (3,1) product, fma(z, c, fma(x, a, y * b)).
//  * hue_hist_kernel     — the hue bin of every point (BGRtoHSVHue, functions.py:
//      73-78, exact: hue_bin), the bin counts (calculateColourHistogram,
//      functions.py:215-226) and each bin's first point (the dict's insertion
//      order). LDS histogram per block, merged with global atomics.
//  * select_kernel       — a stable, order-preserving selection of indices
//      (computePlanarThreshold: dist < thr, functions.py:314-323;
//      filterPointsByHistogram: hist[bin] > thr, functions.py:228-230). One
//      workgroup; chunks of 256 lanes x 16 elements, block scan, running offset.
#include "../svx_launch.h"

namespace svx {

__global__ __launch_bounds__(256) void point_errors_kernel(const double* __restrict__ xyz, int64_t n, int64_t ld,
                                                           double a, double b, double c, double d,
                                                           double* __restrict__ out) {
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const double* p = xyz + i * ld;
        const double dot = __builtin_fma(p[2], c, __builtin_fma(p[0], a, p[1] * b));
        out[i] = __builtin_fabs((dot - 1.0) / d);
    }
}

hipError_t launch_point_errors(const double* xyz, int64_t n, int64_t ld, const double* abcd, double* out,
                               hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(point_errors_kernel, dim3((unsigned)blocks), dim3(256), 0, s, xyz, n, ld, abcd[0], abcd[1],
                       abcd[2], abcd[3], out);
    return hipGetLastError();
}

// rgb: n rows of stride ld bytes, (R, G, B) first. hist[1000] / first[1000]
// must be zero / INT32_MAX-filled by the caller.
__global__ __launch_bounds__(256) void hue_hist_kernel(const uint8_t* __restrict__ rgb, int64_t n, int64_t ld,
                                                       int16_t* __restrict__ bins, uint32_t* __restrict__ hist,
                                                       int32_t* __restrict__ first) {
    __shared__ uint32_t sh_hist[1000];
    __shared__ int32_t sh_first[1000];
    for (int i = threadIdx.x; i < 1000; i += 256) {
        sh_hist[i] = 0;
        sh_first[i] = INT32_MAX;
    }
    __syncthreads();
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const uint8_t* p = rgb + i * ld;
        const int k = hue_bin(p[0], p[1], p[2]);
        if (bins) bins[i] = (int16_t)k;
        atomicAdd(&sh_hist[k], 1u);
        atomicMin(&sh_first[k], (int32_t)i);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < 1000; k += 256) {
        if (sh_hist[k]) {
            atomicAdd(&hist[k], sh_hist[k]);
            atomicMin(&first[k], sh_first[k]);
        }
    }
}

hipError_t launch_hue_hist(const uint8_t* rgb, int64_t n, int64_t ld, int16_t* bins, uint32_t* hist, int32_t* first,
                           hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (n >= INT32_MAX) return hipErrorInvalidValue;
    int64_t blocks = (n + 1023) / 1024;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(hue_hist_kernel, dim3((unsigned)blocks), dim3(256), 0, s, rgb, n, ld, bins, hist, first);
    return hipGetLastError();
}

// keep i iff (mode 0) vals[i] < thr (NaN: not kept, as Python's `<`), or
// (mode 1) ok[bins[i]] != 0. Kept indices in order -> out_idx, count -> *out_n.
__global__ __launch_bounds__(256) void select_kernel(int mode, const double* __restrict__ vals, double thr,
                                                     const int16_t* __restrict__ bins, const uint8_t* __restrict__ ok,
                                                     int64_t n, int64_t* __restrict__ out_idx,
                                                     int64_t* __restrict__ out_n) {
    __shared__ uint32_t wtot[4];
    __shared__ uint8_t sh_ok[1024];
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    if (mode == 1)
        for (int k = tid; k < 1024; k += 256) sh_ok[k] = k < 1000 ? ok[k] : 0;
    __syncthreads();
    int64_t running = 0;
    for (int64_t base = 0; base < n; base += 256 * 16) {
        const int64_t i0 = base + 16 * (int64_t)tid;
        uint32_t bits = 0;
        for (int k = 0; k < 16; ++k) {
            const int64_t i = i0 + k;
            if (i >= n) break;
            const bool keep = mode == 0 ? (vals[i] < thr) : (sh_ok[bins[i] & 1023] != 0);
            bits |= (uint32_t)keep << k;
        }
        const uint32_t cnt = __builtin_popcount(bits);
        const uint32_t inc = wave_incl_scan(cnt);
        if (lane == 63) wtot[wave] = inc;
        __syncthreads();
        uint32_t wbase = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            wbase += w < wave ? wtot[w] : 0u;
            tot += wtot[w];
        }
        __syncthreads();   // wtot is rewritten next chunk
        int64_t o = running + wbase + inc - cnt;
        while (bits) {
            const int k = __builtin_ctz(bits);
            bits &= bits - 1;
            out_idx[o++] = i0 + k;
        }
        running += tot;
    }
    if (tid == 0) *out_n = running;
}

hipError_t launch_select(int mode, const double* vals, double thr, const int16_t* bins, const uint8_t* ok, int64_t n,
                         int64_t* out_idx, int64_t* out_n, hipStream_t s) {
    hipLaunchKernelGGL(select_kernel, dim3(1), dim3(256), 0, s, mode, vals, thr, bins, ok, n, out_idx, out_n);
    return hipGetLastError();
}

}  // namespace svx
