// RANSAC plane fit (functions.py:240-298), SURVEY §8f rank 1: the trial evaluation of the drop-in.
//
// The draws (CPython's random, replayed exactly) are host code: replay.cpp. The numeric work — per trial
// abc = inv([P1;P2;P3]) 1 (functions.py:267), d = |abc| (:269) and the mean distance of the 600 sampled points
// (:274-275, :289) — is one workgroup per trial on the GPU, in fp64. Trials whose 3x3 system is singular or
// ill-conditioned are flagged so the caller re-decides them with the reference's own numpy calls (it also
// re-derives the winner's plane that way, so the plane it returns is bit-identical).
#include <cmath>
#include <vector>

#include "../svx_launch.h"

namespace svx {

// ---------------------------------------------------------------------------
// Trial evaluation: one workgroup per trial.
// flag: 0 ok, 1 singular (det == 0), 2 ill-conditioned (|det| < 1e-6 |r1||r2||r3|)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ransac_eval_kernel(const double* __restrict__ pts, int64_t ld,
                                                          const int32_t* __restrict__ sidx,
                                                          const int32_t* __restrict__ tri, int k,
                                                          double* __restrict__ abc_out, double* __restrict__ err_out,
                                                          uint8_t* __restrict__ flag_out) {
    __shared__ double part[4];
    const int t = blockIdx.x, tid = threadIdx.x;
    const double* r1 = pts + (int64_t)tri[3 * t + 0] * ld;
    const double* r2 = pts + (int64_t)tri[3 * t + 1] * ld;
    const double* r3 = pts + (int64_t)tri[3 * t + 2] * ld;
    // inv(P) 1 = (r2 x r3 + r3 x r1 + r1 x r2) / det, det = r1 . (r2 x r3)
    const double c23[3] = {r2[1] * r3[2] - r2[2] * r3[1], r2[2] * r3[0] - r2[0] * r3[2], r2[0] * r3[1] - r2[1] * r3[0]};
    const double c31[3] = {r3[1] * r1[2] - r3[2] * r1[1], r3[2] * r1[0] - r3[0] * r1[2], r3[0] * r1[1] - r3[1] * r1[0]};
    const double c12[3] = {r1[1] * r2[2] - r1[2] * r2[1], r1[2] * r2[0] - r1[0] * r2[2], r1[0] * r2[1] - r1[1] * r2[0]};
    const double det = r1[0] * c23[0] + r1[1] * c23[1] + r1[2] * c23[2];
    const double a = (c23[0] + c31[0] + c12[0]) / det;
    const double b = (c23[1] + c31[1] + c12[1]) / det;
    const double c = (c23[2] + c31[2] + c12[2]) / det;
    const double nrm = sqrt(a * a + b * b + c * c);
    const double* sp = nullptr;
    double s = 0.0;
    const int32_t* ti = sidx + (int64_t)t * k;
    for (int j = tid; j < k; j += 256) {
        sp = pts + (int64_t)ti[j] * ld;
        s += fabs((sp[0] * a + sp[1] * b + sp[2] * c - 1.0) / nrm);
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, kWave);
    if (lane_id() == 0) part[tid >> 6] = s;
    __syncthreads();
    if (tid == 0) {
        const double e = (part[0] + part[1] + part[2] + part[3]) / k;
        const double n1 = sqrt(r1[0] * r1[0] + r1[1] * r1[1] + r1[2] * r1[2]);
        const double n2 = sqrt(r2[0] * r2[0] + r2[1] * r2[1] + r2[2] * r2[2]);
        const double n3 = sqrt(r3[0] * r3[0] + r3[1] * r3[1] + r3[2] * r3[2]);
        uint8_t fl = 0;
        if (det == 0.0) fl = 1;
        else if (!(fabs(det) >= 1e-6 * n1 * n2 * n3) || !isfinite(e)) fl = 2;
        err_out[t] = e;
        abc_out[3 * t + 0] = a;
        abc_out[3 * t + 1] = b;
        abc_out[3 * t + 2] = c;
        flag_out[t] = fl;
    }
}

hipError_t launch_ransac_eval(const double* pts, int64_t ld, const int32_t* sidx, const int32_t* tri, int trials,
                              int k, double* abc, double* err, uint8_t* flag, hipStream_t s) {
    if (trials <= 0) return hipSuccess;
    hipLaunchKernelGGL(ransac_eval_kernel, dim3(trials), dim3(256), 0, s, pts, ld, sidx, tri, k, abc, err, flag);
    return hipGetLastError();
}

}  // namespace svx
