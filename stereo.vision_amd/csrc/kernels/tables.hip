// Table kernels (gfx950): built once, read through L1/L2 by the pipeline.
//
//  * hue_lut_kernel      — the device hue-bin function over all 2^24 colours;
//                          exists so tests can compare the GPU's binning with
//                          the reference exhaustively (SURVEY §8c digest).
//  * delta_tables_kernel — back-projection deltas (functions.py:191-193 then
//                          :206-207, int32 trunc at stereovision.py:112):
//                          trunc(((X(x,d)*f)/Z(d))+cw) - x in {-1, 0}, computed
//                          in fp64 with the reference's op order, packed 1 bit
//                          per (d, coordinate): 256 x ceil(W/32) + 256 x ceil(H/32)
//                          words (~49 KB at 1024 x 544).
#include "../svx_launch.h"

namespace svx {

// variant 0: hue_bin (exact; the stage kernels and the tiled pipeline), 1: hue_bin_sel (the resident pipeline's
// fp32 path). Colour i = R << 16 | G << 8 | B.
__global__ __launch_bounds__(256) void hue_lut_kernel(int16_t* __restrict__ lut, int variant) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= (1u << 24)) return;
    lut[i] = variant ? (int16_t)hue_bin_sel(i)
                     : (int16_t)hue_bin((int)(i >> 16), (int)((i >> 8) & 255), (int)(i & 255));
}

hipError_t launch_hue_lut(int16_t* lut, int variant, hipStream_t s) {
    hipLaunchKernelGGL(hue_lut_kernel, dim3((1u << 24) / 256), dim3(256), 0, s, lut, variant);
    return hipGetLastError();
}

__device__ __forceinline__ int round_trip_delta(int coord, double centre, int d, const KParams& p) {
    const double Z = p.fB / (double)d;
    const double V = (((double)coord - centre) * Z) / p.f;
    return (int)(((V * p.f) / Z) + centre) - coord;
}

// One lane per (d, 32-coordinate word) of either table.
__global__ __launch_bounds__(256) void delta_tables_kernel(uint32_t* __restrict__ dxbits,
                                                           uint32_t* __restrict__ dybits,
                                                           int8_t* __restrict__ dx8, int8_t* __restrict__ dy8,
                                                           KParams p) {
    const int nx = 256 * p.dx_words, ny = 256 * p.dy_words;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nx + ny) return;
    const bool is_x = i < nx;
    const int j = is_x ? i : i - nx;
    const int words = is_x ? p.dx_words : p.dy_words;
    const int d = j / words, w = j - d * words;
    const int lim = is_x ? p.W : p.H;
    const double centre = is_x ? p.cw : p.ch;
    uint32_t bits = 0;
    for (int b = 0; b < 32; ++b) {
        const int c = 32 * w + b;
        if (c >= lim) break;
        const int delta = d ? round_trip_delta(c, centre, d, p) : 0;
        if (delta == -1) bits |= 1u << b;
        int8_t* t8 = is_x ? dx8 : dy8;
        if (t8) t8[(size_t)d * lim + c] = (int8_t)delta;
    }
    (is_x ? dxbits : dybits)[j] = bits;
}

hipError_t launch_delta_tables(const KParams& p, uint32_t* dxbits, uint32_t* dybits, int8_t* dx8,
                               int8_t* dy8, hipStream_t s) {
    const int n = 256 * (p.dx_words + p.dy_words);
    hipLaunchKernelGGL(delta_tables_kernel, dim3((n + 255) / 256), dim3(256), 0, s, dxbits, dybits, dx8,
                       dy8, p);
    return hipGetLastError();
}

// One lane per (j, coordinate) of either transposed table: bit b of the word = the delta bit of d = 32 j + b.
__global__ __launch_bounds__(256) void delta_transpose_kernel(const uint32_t* __restrict__ dxbits,
                                                              const uint32_t* __restrict__ dybits,
                                                              uint32_t* __restrict__ dxT, uint32_t* __restrict__ dyT,
                                                              int dx_words, int dy_words) {
    const int nx = 8 * 32 * dx_words, ny = 8 * 32 * dy_words;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nx + ny) return;
    const bool is_x = i < nx;
    const int j0 = is_x ? i : i - nx;
    const int words = is_x ? dx_words : dy_words;
    const int n = 32 * words;
    const int j = j0 / n, c = j0 - j * n;
    const uint32_t* src = is_x ? dxbits : dybits;
    uint32_t bits = 0;
    for (int b = 0; b < 32; ++b) bits |= ((src[(32 * j + b) * words + (c >> 5)] >> (c & 31)) & 1u) << b;
    (is_x ? dxT : dyT)[j0] = bits;
}

hipError_t launch_delta_transpose(const KParams& p, const uint32_t* dxbits, const uint32_t* dybits, uint32_t* dxT,
                                  uint32_t* dyT, hipStream_t s) {
    const int n = 8 * 32 * (p.dx_words + p.dy_words);
    hipLaunchKernelGGL(delta_transpose_kernel, dim3((n + 255) / 256), dim3(256), 0, s, dxbits, dybits, dxT, dyT,
                       p.dx_words, p.dy_words);
    return hipGetLastError();
}

}  // namespace svx
