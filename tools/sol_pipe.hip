// Speed-of-light probe for the pipeline's data movement (diagnostic, not product).
//
// The resident pipeline (kernels/resident.hip) moves, per 4096-frame call, the
// disparity (1 B/px) and BGR (3 B/px) of every frame in, and 20 B per kept point
// out, as five frame-strided planes (X, Y, Z f32; x, y i32) at frame * cap. This
// program moves the same bytes with the same layout and no arithmetic, one
// workgroup per frame, so its rate is the practical ceiling of that traffic mix:
//   mode 0  read the frame (disparity + BGR), then write its outputs   (the pipeline's order)
//   mode 1  reads and writes interleaved chunk by chunk
//   mode 2  reads only
//   mode 3  writes only
//   mode 4  mode 0 with the reads done twice (pass 1 and pass 2 both read the disparity)
// and, writes only, other output layouts of the same bytes:
//   mode 5  five planes, frame stride = kept (dense frames)
//   mode 6  one plane, 20 B per point (AoS), frame stride 5 x cap
//   mode 7  five planes, frame stride cap + 64 (another channel phase per frame)
//   mode 8  five dense planes swept in 4 KiB tiles across frames (K1's pattern: no per-frame streams)
//   mode 9  five planes, frame stride cap, each lane writing 2 x 16 B contiguous per plane
//   mode 10 read-then-write, each frame's output region taken from a global counter (atomicAdd) after its reads
//   mode 11 five planes, frame stride cap, every frame writing all cap outputs (no gaps; more bytes)
//   mode 12 mode 1 (chunk-interleaved reads and writes) into a region taken from the counter after the first chunk's reads
//   mode 13..17  the resident pipeline's shape: all of the frame read (pass 1), then pass 2 re-reading the
//           disparity and writing, in groups of K = 1, 2, 4, 8, 64 chunks (K chunks' disparity reads, then
//           their K chunks' writes), into a region taken from the counter after pass 1
//   mode 18..22  the same with the frame-strided planes (no counter)
//   mode 27..29  mode 18's shape (K = 1) with frame-interleaved tiles: output o of frame f at
//           ((o / B) * frames + f) * B + o % B, B = 256, 1024, 4096 outputs (round 3, session 3)
//   mode 30..32  writes only, the same three tiled layouts
//   mode 33..36  persistent: 1280 workgroups (the resident kernel's 5 a CU), each taking frames
//           blockIdx + r * 1280, launched cooperatively: 33 mode 18's shape (no barriers); 34 the same with a
//           grid barrier after every round's pass 1 and after its pass 2 (so the whole chip reads, then writes);
//           35 mode 34 with pass 2 as K = 64 (all re-reads, then all writes); 36 mode 34 with only the barrier
//           after pass 1
// argv: frames (4096), outputs per frame (277200), 1 = output planes physically contiguous (0);
//       or: r05 frames kept skip reps (the round-5 probe of the 16-B layout, shape16_kernel)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_sol_pipe tools/sol_pipe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));

struct Args {
    const uint4* disp;   // frames x px bytes
    const uint4* bgr;    // frames x 3 px bytes
    float* o[5];         // frames x cap
    uint32_t* sink;
    int64_t px16;        // 16-byte words of disparity per frame
    int64_t cap;         // outputs per frame (multiple of 4)
    int64_t kept;        // outputs written per frame (multiple of 4)
    int mode;
    int64_t stride;      // floats between frames in a plane (writes)
    int nplanes;         // planes written
    int64_t nper;        // floats per plane per frame
    unsigned long long* counter;
    int kgroup;          // modes 13..22: chunks per read/write group
    int lb;              // modes 27..32: log2 of the tile (outputs)
    unsigned* bar;       // modes 33..36: grid barrier counter
    int frames;
};

__device__ __forceinline__ uint32_t read_range(const Args& a, int f, int64_t w0, int64_t w1) {
    uint32_t acc = 0;
    const uint4* d = a.disp + f * a.px16;
    const uint4* c = a.bgr + f * a.px16 * 3;
    for (int64_t w = w0 + threadIdx.x; w < w1; w += 256) {
        const uint4 x = *(d + w);
        const uint4 y0 = *(c + 3 * w), y1 = *(c + 3 * w + 1),
                    y2 = *(c + 3 * w + 2);
        acc ^= x.x ^ x.y ^ x.z ^ x.w ^ y0.x ^ y0.w ^ y1.y ^ y1.z ^ y2.x ^ y2.w;
    }
    return acc;
}

__device__ __forceinline__ void write_range(const Args& a, int f, int64_t g0, int64_t g1, float v) {
    for (int64_t g = g0 + 4 * threadIdx.x; g < g1; g += 1024) {
        const v4f q = {v, v, v, v};
#pragma unroll
        for (int k = 0; k < 5; ++k) __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(a.o[k] + f * a.cap + g));
    }
}

__device__ __forceinline__ void write_layout(const Args& a, int f, float v) {
    const v4f q = {v, v, v, v};
    if (a.mode == 9) {
        for (int64_t g = 8 * threadIdx.x; g < a.nper; g += 2048)
            for (int k = 0; k < 5; ++k) {
                __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(a.o[k] + f * a.stride + g));
                if (g + 8 <= a.nper) __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(a.o[k] + f * a.stride + g + 4));
            }
        return;
    }
    for (int64_t g = 4 * threadIdx.x; g < a.nper; g += 1024)
        for (int k = 0; k < a.nplanes; ++k)
            __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(a.o[k] + f * a.stride + g));
}

__global__ __launch_bounds__(256) void sweep_kernel(Args a, int64_t total) {   // mode 8
    const v4f q = {1.f, 1.f, 1.f, 1.f};
    for (int64_t t = blockIdx.x; t * 1024 < total; t += gridDim.x) {
        const int64_t g = t * 1024 + 4 * threadIdx.x;
        if (g < total)
            for (int k = 0; k < 5; ++k) __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(a.o[k] + g));
    }
}

__device__ __forceinline__ int64_t tiled(const Args& a, int f, int64_t g) {
    return ((((g >> a.lb) * a.frames) + f) << a.lb) + (g & ((1 << a.lb) - 1));
}

__device__ void grid_barrier(unsigned* ctr, unsigned target) {
    __syncthreads();
    if (threadIdx.x == 0) {
        // relaxed: the phases order no data here (an agent-scope release / acquire per arrival and poll is an L2
        // write-back / invalidate on gfx950: 14-16 ms instead of 6 with them, profiles/r03/sol_pipe_persist.txt)
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(8);
    }
    __syncthreads();
}

__global__ __launch_bounds__(256) void persist_kernel(Args a) {   // modes 33..36
    const int G = gridDim.x;
    uint32_t acc = 0;
    unsigned nb = 0;
    const int rounds = (a.frames + G - 1) / G;
    for (int r = 0; r < rounds; ++r) {
        const int f = blockIdx.x + r * G;
        const bool live = f < a.frames;
        if (live) acc ^= read_range(a, f, 0, a.px16);   // pass 1
        if (a.mode >= 34) grid_barrier(a.bar, ++nb * G);
        if (live) {
            const float v = (float)f;
            const uint4* d = a.disp + f * a.px16;
            const int n = 64, K = a.mode == 35 ? 64 : 1;
            for (int c0 = 0; c0 < n; c0 += K) {
                for (int c = c0; c < c0 + K; ++c)
                    for (int64_t w = a.px16 * c / n + threadIdx.x; w < a.px16 * (c + 1) / n; w += 256) {
                        const uint4 x = *(d + w);
                        acc ^= x.x ^ x.w;
                    }
                const int64_t g0 = (a.kept / 4 * c0 / n) * 4, g1 = (a.kept / 4 * (c0 + K) / n) * 4;
                for (int64_t g = g0 + 4 * threadIdx.x; g < g1; g += 1024) {
                    const v4f q = {v, v, v, v};
#pragma unroll
                    for (int k = 0; k < 5; ++k)
                        __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(a.o[k] + (int64_t)f * a.cap + g));
                }
            }
        }
        if (a.mode == 34 || a.mode == 35) grid_barrier(a.bar, ++nb * G);
    }
    if (acc == 0x12345678u) a.sink[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void sol_kernel(Args a) {
    const int f = blockIdx.x;
    uint32_t acc = 0;
    const float v = (float)f;
    if (a.mode >= 30) {
        for (int64_t g = 4 * threadIdx.x; g < a.kept; g += 1024) {
            const v4f q = {v, v, v, v};
#pragma unroll
            for (int k = 0; k < 5; ++k) __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(a.o[k] + tiled(a, f, g)));
        }
    } else if (a.mode >= 27) {
        const int n = 64;
        acc ^= read_range(a, f, 0, a.px16);   // pass 1
        const uint4* d = a.disp + f * a.px16;
        for (int c = 0; c < n; ++c) {
            for (int64_t w = a.px16 * c / n + threadIdx.x; w < a.px16 * (c + 1) / n; w += 256) {
                const uint4 x = *(d + w);
                acc ^= x.x ^ x.w;
            }
            const int64_t g0 = (a.kept / 4 * c / n) * 4, g1 = (a.kept / 4 * (c + 1) / n) * 4;
            for (int64_t g = g0 + 4 * threadIdx.x; g < g1; g += 1024) {
                const v4f q = {v, v, v, v};
#pragma unroll
                for (int k = 0; k < 5; ++k) __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(a.o[k] + tiled(a, f, g)));
            }
        }
    } else if (a.mode >= 13) {
        // 23 / 24: as 13 / 18 (K = 1) with pass 2 walking the chunks last to first (what pass 1 read last is
        // re-read first, while it may still be cached); 25 / 26: pass 1 + the re-read only (no writes),
        // first to last / last to first
        const int K = a.kgroup, n = 64;
        const bool rev = a.mode == 23 || a.mode == 24 || a.mode == 26;
        const bool nowr = a.mode >= 25;
        acc ^= read_range(a, f, 0, a.px16);   // pass 1
        __shared__ int64_t base13;
        if (threadIdx.x == 0)
            base13 = (a.mode <= 17 || a.mode == 23) ? (int64_t)atomicAdd(a.counter, (unsigned long long)a.kept)
                                                    : (int64_t)f * a.cap;
        __syncthreads();
        const uint4* d = a.disp + f * a.px16;
        for (int cc = 0; cc < n; cc += K) {
            const int c0 = rev ? n - K - cc : cc;
            for (int c = c0; c < c0 + K; ++c)
                for (int64_t w = a.px16 * c / n + threadIdx.x; w < a.px16 * (c + 1) / n; w += 256) {
                    const uint4 x = *(d + w);
                    acc ^= x.x ^ x.w;
                }
            if (nowr) continue;
            const int64_t g0 = (a.kept / 4 * c0 / n) * 4, g1 = (a.kept / 4 * (c0 + K) / n) * 4;
            for (int64_t g = g0 + 4 * threadIdx.x; g < g1; g += 1024) {
                const v4f q = {v, v, v, v};
#pragma unroll
                for (int k = 0; k < 5; ++k) __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(a.o[k] + base13 + g));
            }
        }
    } else if (a.mode == 12) {
        const int n = 64;   // chunks
        __shared__ int64_t base12;
        for (int c = 0; c < n; ++c) {
            acc ^= read_range(a, f, a.px16 * c / n, a.px16 * (c + 1) / n);
            if (c == 0) {
                if (threadIdx.x == 0) base12 = (int64_t)atomicAdd(a.counter, (unsigned long long)a.kept);
                __syncthreads();
            }
            const int64_t g0 = (a.kept / 4 * c / n) * 4, g1 = (a.kept / 4 * (c + 1) / n) * 4;
            for (int64_t g = g0 + 4 * threadIdx.x; g < g1; g += 1024) {
                const v4f q = {v, v, v, v};
#pragma unroll
                for (int k = 0; k < 5; ++k) __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(a.o[k] + base12 + g));
            }
        }
    } else if (a.mode == 10) {
        acc ^= read_range(a, f, 0, a.px16);
        __shared__ int64_t base;
        if (threadIdx.x == 0) base = (int64_t)atomicAdd(a.counter, (unsigned long long)a.kept);
        __syncthreads();
        for (int64_t g = 4 * threadIdx.x; g < a.kept; g += 1024) {
            const v4f q = {v, v, v, v};
#pragma unroll
            for (int k = 0; k < 5; ++k) __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(a.o[k] + base + g));
        }
    } else if (a.mode >= 5) {
        write_layout(a, f, v);
    } else if (a.mode == 1) {
        const int n = 64;   // chunks
        for (int c = 0; c < n; ++c) {
            acc ^= read_range(a, f, a.px16 * c / n, a.px16 * (c + 1) / n);
            write_range(a, f, (a.kept / 4 * c / n) * 4, (a.kept / 4 * (c + 1) / n) * 4, v);
        }
    } else {
        if (a.mode != 3) acc ^= read_range(a, f, 0, a.px16);
        if (a.mode == 4) {   // pass 2 re-reads the disparity
            const uint4* d = a.disp + f * a.px16;
            for (int64_t w = threadIdx.x; w < a.px16; w += 256) {
                const uint4 x = *(d + w);
                acc ^= x.x ^ x.w;
            }
        }
        if (a.mode != 2) write_range(a, f, 0, a.kept, v);
    }
    if (acc == 0x12345678u) a.sink[f] = acc;   // keeps the loads
}

// Round 5: the resident kernel's shape at its 16-B layout (three f32 planes X, Y, Z + one packed planePoints
// word a point, round 4). A frame has `nch` chunks (the kernel's 4096 grid points each: 136 at 1024 x 544); the
// first `skip` of them are chunks the plane rules out (the rows above the horizon: pass 1 reads their disparity
// only, pass 2 skips them), the rest hold the frame's `kept` outputs evenly. Pass 1 reads disparity + BGR, pass 2
// re-reads the disparity and writes its chunk's outputs, K chunks' reads before their writes.
//   r5 mode 0  K = 1, frame-strided planes (the kernel)          1  K = 1, atomic regions (dense frames)
//           2  K = whole frame, strided                          3  K = whole frame, atomic regions
//           4  pass 1 reads only                                 5  pass-2 writes only (strided)
//           6  mode 0 without the pass-2 disparity re-read       7  writes only, dense frames
//           8  pass-2 writes only, one AoS plane of 16-B records   9  mode 0 with the AoS records
//          10  K = 1, the next chunk's pass-2 read issued before this chunk's writes and waited for with
//              s_waitcnt vmcnt(12) (the writes stay outstanding): is K = 1's cost the loads waiting behind the
//              stores' acknowledgements (gfx9 counts both in vmcnt)?
//          11  mode 0 with each chunk's outputs starting on a 128-byte line (multiples of 32 outputs, as the
//              kernel writes them: whole lines, the tail carried)      12  mode 11 without the pass-2 re-read
//          13  mode 11 at the kernel's occupancy (32 KB of LDS a workgroup: 5 a CU)
//          14  mode 13 with the kernel's two workgroup barriers a chunk in pass 2 and one a chunk in pass 1
struct Args5 {
    const uint8_t* disp;
    const uint8_t* bgr;
    float* o[4];
    uint32_t* sink;
    int64_t px, cap, kept;
    int nch, skip, mode;
    unsigned long long* counter;
};

__global__ __launch_bounds__(256) void shape16_kernel(Args5 a) {
    const int f = blockIdx.x;
    const int64_t chunk_px = (a.px + a.nch - 1) / a.nch;   // bytes of disparity a chunk covers
    const uint4* d = reinterpret_cast<const uint4*>(a.disp + (int64_t)f * a.px);
    const uint4* c = reinterpret_cast<const uint4*>(a.bgr + (int64_t)f * a.px * 3);
    uint32_t acc = 0;
    const int live = a.nch - a.skip;
    const auto cw0 = [&](int ch) { return (int64_t)ch * chunk_px / 16; };
    const auto cw1 = [&](int ch) { return min((int64_t)(ch + 1) * chunk_px, a.px) / 16; };
    extern __shared__ uint32_t occ_lds[];   // modes 13, 14: launched with 32 KB (the kernel's occupancy)
    if ((a.mode == 13 || a.mode == 14) && threadIdx.x == 0) occ_lds[0] = 0u;
    if (a.mode != 5 && a.mode != 7 && a.mode != 8) {   // pass 1
        for (int ch = 0; ch < a.nch; ++ch) {
            if (a.mode == 14) __syncthreads();
            const bool bgr = ch >= a.skip;
            for (int64_t w = cw0(ch) + threadIdx.x; w < cw1(ch); w += 256) {
                const uint4 x = d[w];
                acc ^= x.x ^ x.w;
                if (bgr) {
                    const uint4 y0 = c[3 * w], y1 = c[3 * w + 1], y2 = c[3 * w + 2];
                    acc ^= y0.x ^ y1.y ^ y2.w;
                }
            }
        }
    }
    if (a.mode == 4) {
        if (acc == 0x12345678u) a.sink[f] = acc;
        return;
    }
    __shared__ int64_t base;
    if (threadIdx.x == 0)
        base = (a.mode == 1 || a.mode == 3 || a.mode == 7) ? (int64_t)atomicAdd(a.counter, (unsigned long long)a.kept)
                                                           : (int64_t)f * a.cap;
    __syncthreads();
    if (a.mode == 10) {   // one 16-byte disparity load a lane a chunk (4096 B = 256 lanes x 16 B)
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const float v = (float)f;
        u32x4 xn;
        const u32x4* dv = reinterpret_cast<const u32x4*>(d);
        const auto ld = [&](int ch) {   // the compiler does not track this load: the waits below are ours
            u32x4 r;
            const u32x4* ptr = dv + cw0(a.skip + ch) + threadIdx.x;
            __asm__ volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(ptr) : "memory");
            return r;
        };
        xn = ld(0);
        for (int c0 = 0; c0 < live; ++c0) {
            if (c0 == 0) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else __asm__ volatile("s_waitcnt vmcnt(12)" ::: "memory");   // >= 12 stores of the last chunk a lane
            const u32x4 x = xn;
            if (c0 + 1 < live) xn = ld(c0 + 1);
            acc ^= x.x ^ x.w;
            const int64_t g0 = (a.kept / 4 * c0 / live) * 4, g1 = (a.kept / 4 * (c0 + 1) / live) * 4;
            for (int64_t g = g0 + 4 * threadIdx.x; g < g1; g += 1024) {
                const v4f q = {v, v, v, v};
#pragma unroll
                for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(a.o[k] + base + g));
            }
        }
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (acc == 0x12345678u) a.sink[f] = acc;
        return;
    }
    const int K = (a.mode == 2 || a.mode == 3) ? live : 1;
    const float v = (float)f;
    for (int c0 = 0; c0 < live; c0 += K) {
        if (a.mode != 5 && a.mode != 6 && a.mode != 7 && a.mode != 8 && a.mode != 12)   // (13, 14 read)
            for (int ch = c0; ch < min(c0 + K, live); ++ch)
                for (int64_t w = cw0(a.skip + ch) + threadIdx.x; w < cw1(a.skip + ch); w += 256) {
                    const uint4 x = d[w];
                    acc ^= x.x ^ x.w;
                }
        int64_t g0 = (a.kept / 4 * c0 / live) * 4, g1 = (a.kept / 4 * min(c0 + K, live) / live) * 4;
        if (a.mode == 14) __syncthreads();
        if (a.mode >= 11 && a.mode <= 14) {   // whole 128-byte lines a chunk (the last chunk ends at kept)
            g0 &= ~31ll;
            g1 = min(c0 + K, live) == live ? a.kept : (g1 & ~31ll);
        }
        if (a.mode == 8 || a.mode == 9) {   // record g = X, Y, Z, P of output g: 1 KiB contiguous a wave-store
            for (int64_t g = g0 + threadIdx.x; g < g1; g += 256) {
                const v4f q = {v, v, v, v};
                __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(a.o[0]) + base + g);
            }
        } else {
            for (int64_t g = g0 + 4 * threadIdx.x; g < g1; g += 1024) {
                const v4f q = {v, v, v, v};
#pragma unroll
                for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(a.o[k] + base + g));
            }
        }
        if (a.mode == 14) __syncthreads();
    }
    if (acc == 0x12345678u) a.sink[f] = acc;
}

static int main_r05(int argc, char** argv) {
    // argv: r05 frames kept skip_of_136 reps
    const int frames = argc > 2 ? std::atoi(argv[2]) : 4096;
    const int64_t kept = argc > 3 ? std::atoll(argv[3]) : 277200;
    const int skip = argc > 4 ? std::atoi(argv[4]) : 50;
    const int reps = argc > 5 ? std::atoi(argv[5]) : 5;
    const int64_t px = 544 * 1024, cap = (555489 + 63) / 64 * 64;
    Args5 a{};
    void* p;
    CK(hipMalloc(&p, frames * px));
    CK(hipMemset(p, 1, frames * px));
    a.disp = (const uint8_t*)p;
    CK(hipMalloc(&p, frames * px * 3));
    CK(hipMemset(p, 2, frames * px * 3));
    a.bgr = (const uint8_t*)p;
    for (int k = 0; k < 4; ++k) {   // plane 0 holds the AoS records too (4 x cap floats)
        CK(hipMalloc(&p, frames * cap * (k == 0 ? 16 : 4)));
        a.o[k] = (float*)p;
    }
    CK(hipMalloc(&p, frames * 4));
    a.sink = (uint32_t*)p;
    CK(hipMalloc(&p, 8));
    a.counter = (unsigned long long*)p;
    a.px = px;
    a.cap = cap;
    a.kept = kept;
    a.nch = 136;
    a.skip = skip;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[] = {"K=1 strided (the kernel's shape)", "K=1 atomic regions", "K=frame strided",
                           "K=frame atomic regions", "pass 1 reads only", "pass-2 writes only, strided",
                           "K=1 strided, no pass-2 re-read", "writes only, atomic regions",
                           "pass-2 writes only, AoS records", "K=1, AoS records",
                           "K=1, next read before the writes, vmcnt(12)", "K=1, chunks on whole lines",
                           "K=1, whole lines, no pass-2 re-read", "K=1, whole lines, 5 workgroups a CU",
                           "K=1, whole lines, 5 a CU, the kernel's barriers"};
    const int live = a.nch - skip;
    for (int round = 0; round < 2; ++round)
        for (int mode = 0; mode < 15; ++mode) {
            a.mode = mode;
            float best = 1e30f, tot = 0.f;
            CK(hipMemset(a.counter, 0, 8));
            const size_t lds = (mode == 13 || mode == 14) ? 32768 : 0;
            hipLaunchKernelGGL(shape16_kernel, dim3(frames), dim3(256), lds, 0, a);
            for (int r = 0; r < reps; ++r) {
                CK(hipMemset(a.counter, 0, 8));
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(shape16_kernel, dim3(frames), dim3(256), lds, 0, a);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
                tot += ms;
            }
            const double p1 = (mode == 5 || mode == 7 || mode == 8) ? 0. : px * frames * (1. + 3. * live / a.nch);
            const double p2r = (mode <= 3 || mode == 9 || mode == 10 || mode == 11 || mode == 13 || mode == 14)
                                   ? px * frames * (double)live / a.nch
                                                                                    : 0.;
            const double wr = mode == 4 ? 0. : 16. * kept * frames;
            std::printf("{\"round\": %d, \"r5mode\": %d, \"what\": \"%s\", \"skip\": %d, \"kept\": %lld, "
                        "\"GB\": %.2f, \"best_ms\": %.3f, \"mean_ms\": %.3f, \"TBps_best\": %.2f}\n",
                        round, mode, names[mode], skip, (long long)kept, (p1 + p2r + wr) / 1e9, best, tot / reps,
                        (p1 + p2r + wr) / best / 1e9);
            std::fflush(stdout);
        }
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "r05") return main_r05(argc, argv);
    const int frames = argc > 1 ? std::atoi(argv[1]) : 4096;
    const int64_t px = 544 * 1024;
    const int64_t kept = argc > 2 ? std::atoll(argv[2]) : 277200;   // 1.135 G kept points / 4096 frames (the bench pipeline)
    const int64_t cap = (555489 + 3) / 4 * 4 + 64;   // room for mode 7's padding
    Args a{};
    void* p;
    CK(hipMalloc(&p, frames * px));
    CK(hipMemset(p, 1, frames * px));
    a.disp = (const uint4*)p;
    CK(hipMalloc(&p, frames * px * 3));
    CK(hipMemset(p, 2, frames * px * 3));
    a.bgr = (const uint4*)p;
    const bool contig = argc > 3 && std::atoi(argv[3]) != 0;   // outputs physically contiguous
    for (int k = 0; k < 5; ++k) {
        const size_t bytes = frames * cap * 4 * (k == 0 ? 5 : 1);   // plane 0 also holds mode 6's AoS
        if (contig) CK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocContiguous));
        else CK(hipMalloc(&p, bytes));
        a.o[k] = (float*)p;
    }
    CK(hipMalloc(&p, frames * 4));
    a.sink = (uint32_t*)p;
    CK(hipMalloc(&p, 8));
    a.counter = (unsigned long long*)p;
    CK(hipMalloc(&p, 8));
    a.bar = (unsigned*)p;
    a.px16 = px / 16;
    a.cap = cap;
    a.kept = kept;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[] = {"read-then-write", "interleaved", "read only", "write only", "read, re-read disp, write",
                           "write: dense frames", "write: one AoS plane", "write: stride cap+64", "write: dense sweep",
                           "write: 32 B per lane", "read-then-write, atomic regions", "write: full frames, stride cap",
                           "interleaved, atomic regions", "pass1 + K-grouped pass2, atomic regions",
                           "pass1 + K-grouped pass2, atomic regions", "pass1 + K-grouped pass2, atomic regions",
                           "pass1 + K-grouped pass2, atomic regions", "pass1 + K-grouped pass2, atomic regions",
                           "pass1 + K-grouped pass2, strided", "pass1 + K-grouped pass2, strided",
                           "pass1 + K-grouped pass2, strided", "pass1 + K-grouped pass2, strided",
                           "pass1 + K-grouped pass2, strided", "pass1 + pass2 last chunk first, atomic regions",
                           "pass1 + pass2 last chunk first, strided", "pass1 + re-read only, first chunk first",
                           "pass1 + re-read only, last chunk first", "pass1 + pass2, tiles of 256",
                           "pass1 + pass2, tiles of 1024", "pass1 + pass2, tiles of 4096", "write: tiles of 256",
                           "write: tiles of 1024", "write: tiles of 4096", "persistent, no barriers",
                           "persistent, barrier after pass 1 and pass 2", "persistent, barriers, pass 2 K = 64",
                           "persistent, barrier after pass 1"};
    const int kgroups[5] = {1, 2, 4, 8, 64};
    const int64_t cap0 = cap - 64;
    for (int round = 0; round < 2; ++round)
        for (int mode = 0; mode < 37; ++mode) {
            // earlier results: profiles/r02/sol_pipe_session8.txt, r03/sol_pipe_kgroup.txt, r03/sol_pipe_reverse.txt,
            // r03/sol_pipe_tiles.txt
            if (!(mode == 18 || mode >= 33)) continue;
            a.mode = mode;
            a.kgroup = mode >= 13 && mode <= 22 ? kgroups[(mode - 13) % 5] : 1;
            a.nplanes = 5;
            a.frames = frames;
            a.lb = mode >= 27 ? (const int[]){8, 10, 12}[(mode - 27) % 3] : 0;
            a.nper = kept;
            a.stride = cap0;
            if (mode == 5) a.stride = kept;
            if (mode == 6) {
                a.nplanes = 1;
                a.nper = 5 * kept;
                a.stride = 5 * cap0;
            }
            if (mode == 7) a.stride = cap;
            if (mode == 11) a.nper = cap0;
            auto launch = [&]() {
                if (mode >= 33) {
                    CK(hipMemsetAsync(a.bar, 0, 4, 0));
                    void* kargs[] = {&a};
                    CK(hipLaunchCooperativeKernel((const void*)persist_kernel, dim3(1280), dim3(256), kargs, 0, 0));
                } else if (mode == 8) hipLaunchKernelGGL(sweep_kernel, dim3(4096), dim3(256), 0, 0, a, kept * frames);
                else hipLaunchKernelGGL(sol_kernel, dim3(frames), dim3(256), 0, 0, a);
            };
            float best = 1e30f, tot = 0.f;
            const int reps = 5;
            CK(hipMemset(a.counter, 0, 8));
            launch();
            for (int r = 0; r < reps; ++r) {
                CK(hipMemset(a.counter, 0, 8));
                CK(hipEventRecord(e0, 0));
                launch();
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
                tot += ms;
            }
            const double rd = ((mode == 3 || mode >= 5) && mode != 10 && (mode < 12 || (mode >= 30 && mode < 33)) ? 0. : 4. * px * frames) +
                              ((mode == 4 || mode >= 13) && (mode < 30 || mode >= 33) ? 1. * px * frames : 0.);
            const double wr = (mode == 2 || (mode >= 25 && mode < 27)) ? 0. : 20. * (mode == 11 ? cap0 : kept) * frames;
            std::printf("{\"round\": %d, \"mode\": %d, \"what\": \"%s\", \"K\": %d, \"GB\": %.2f, \"best_ms\": %.3f, "
                        "\"mean_ms\": %.3f, \"TBps_best\": %.2f}\n",
                        round, mode, names[mode], a.kgroup, (rd + wr) / 1e9, best, tot / reps, (rd + wr) / best / 1e9);
            std::fflush(stdout);
        }
    return 0;
}
