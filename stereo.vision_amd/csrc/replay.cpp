// Host replay of CPython's random draws for the RANSAC drop-in (functions.py:240-298), SURVEY §8f rank 1:
// sv_ransac_draw and the draw side of sv_ransac (runtime.hip). Plain C++ for the host compiler; the trial
// evaluation kernels are kernels/ransac.hip.
//
// The reference draws from Python's global `random` (unseeded). To be a drop-in whose effect on the program is
// identical, the draws are replayed exactly: CPython's MT19937 (genrand_uint32), getrandbits(k) = word >> (32-k)
// for k <= 32, _randbelow_with_getrandbits (rejection on k = n.bit_length() bits) and random.sample's two branches
// (pool swap for n <= setsize, set rejection otherwise), starting from the caller's random.getstate() and handing
// the advanced state back. The draw order per trial is the reference's: sample(points, 600) (functions.py:286),
// then randomNonCollinearPoints' three sample(points, 1) until numpy's cross(P1-P2, P2-P3) is not all zero
// (functions.py:240-260, products rounded before the subtraction as numpy.cross does).
#include <immintrin.h>

#include <cmath>
#include <cstdint>
#include <vector>

namespace svx {

int ransac_draw(uint32_t* state625, const double* pts, int64_t n, int64_t ld, int trials, int k, int32_t* sidx,
                int32_t* tri);   // (declared for the runtime in svx_launch.h)

// ---------------------------------------------------------------------------
// CPython Random (Modules/_randommodule.c + Lib/random.py, 3.10)
// ---------------------------------------------------------------------------
struct PyMT {
    uint32_t mt[624];
    int index;
    // the tempered outputs of the current state (out[i] = temper(mt[i])), made once per twist: the twist and the
    // tempering run as straight loops over the 624 words (vectorised), and a draw is one load
    uint32_t out[624];
    bool out_valid = false;

    void twist() {
        constexpr uint32_t UPPER = 0x80000000u, LOWER = 0x7fffffffu, A = 0x9908b0dfu;
        int kk;
        for (kk = 0; kk < 624 - 397; kk++) {
            const uint32_t y = (mt[kk] & UPPER) | (mt[kk + 1] & LOWER);
            mt[kk] = mt[kk + 397] ^ (y >> 1) ^ ((0u - (y & 1u)) & A);
        }
        for (; kk < 623; kk++) {
            const uint32_t y = (mt[kk] & UPPER) | (mt[kk + 1] & LOWER);
            mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ ((0u - (y & 1u)) & A);
        }
        const uint32_t y = (mt[623] & UPPER) | (mt[0] & LOWER);
        mt[623] = mt[396] ^ (y >> 1) ^ ((0u - (y & 1u)) & A);
        index = 0;
        out_valid = false;
    }
    void temper_all() {
        for (int i = 0; i < 624; ++i) {
            uint32_t y = mt[i];
            y ^= (y >> 11);
            y ^= (y << 7) & 0x9d2c5680u;
            y ^= (y << 15) & 0xefc60000u;
            y ^= (y >> 18);
            out[i] = y;
        }
        out_valid = true;
    }
    uint32_t genrand() {   // CPython's genrand_uint32
        if (index >= 624) twist();
        if (!out_valid) temper_all();
        return out[index++];
    }
    uint32_t getrandbits(int k) { return k == 0 ? 0u : genrand() >> (32 - k); }   // k <= 32
    uint32_t randbelow(uint32_t n) {
        if (!n) return 0;
        const int k = 32 - __builtin_clz(n);   // n.bit_length()
        uint32_t r = getrandbits(k);
        while (r >= n) r = getrandbits(k);
        return r;
    }
};

// random.sample's setsize (Lib/random.py): the pool branch for n <= setsize, the set branch above it
static int64_t sample_setsize(int k) {
    int64_t setsize = 21;
    if (k > 5) setsize += (int64_t)std::pow(4.0, std::ceil(std::log((double)k * 3) / std::log(4.0)));
    return setsize;
}

// random.sample(range(n), k) -> out[0..k). Caller guarantees 0 <= k <= n.
// The set branch's `selected` is a bitmap of n bits (cleared bit by bit after
// the sample): membership is what the reference's set answers, at a fraction
// of a hash set's cost.
static void py_sample(PyMT& rng, uint32_t n, int k, int32_t* out, std::vector<uint32_t>& pool,
                      std::vector<uint64_t>& selected) {
    if ((int64_t)n <= sample_setsize(k)) {
        pool.resize(n);
        for (uint32_t i = 0; i < n; ++i) pool[i] = i;
        for (int i = 0; i < k; ++i) {
            const uint32_t j = rng.randbelow(n - i);
            out[i] = (int32_t)pool[j];
            pool[j] = pool[n - i - 1];
        }
    } else {
        // `j = randbelow(n); while j in selected: j = randbelow(n)` consumes the stream one word at a time and
        // keeps a word iff its top n.bit_length() bits are < n and not selected yet: one flat, branch-free loop
        // over the tempered words (a rejected word writes its bit into a spare word past the bitmap)
        const uint32_t nw = (n + 63) / 64;
        if (selected.size() < nw + 1) selected.assign(nw + 1, 0);
        const int sh = __builtin_clz(n);   // 32 - n.bit_length()
        uint64_t* __restrict__ sel = selected.data();
        int32_t* __restrict__ dst = out;   // (distinct from the state and the bitmap: no reload after each store)
        int cnt = 0;
        while (cnt < k) {
            if (rng.index >= 624) rng.twist();
            if (!rng.out_valid) rng.temper_all();
            const uint32_t* __restrict__ src = rng.out;
            int i = rng.index;
            for (; i < 624 && cnt < k; ++i) {
                const uint32_t j = src[i] >> sh;
                const uint32_t jj = j < n ? j : 64u * nw;   // the spare word
                const uint64_t w = sel[jj >> 6], bit = 1ull << (jj & 63);
                const uint32_t take = (uint32_t)(j < n) & (uint32_t)((w & bit) == 0);
                sel[jj >> 6] = w | (take ? bit : 0ull);
                dst[cnt] = (int32_t)j;
                cnt += (int)take;
            }
            rng.index = i;
        }
        for (int i = 0; i < k; ++i) sel[(uint32_t)out[i] >> 6] = 0;   // every word that got a bit
        sel[nw] = 0;
    }
}

// numpy.cross(P1 - P2, P2 - P3) == 0 in every component (functions.py:255-258)
static bool collinear(const double* p1, const double* p2, const double* p3) {
    volatile double a0 = p1[0] - p2[0], a1 = p1[1] - p2[1], a2 = p1[2] - p2[2];
    volatile double b0 = p2[0] - p3[0], b1 = p2[1] - p3[1], b2 = p2[2] - p3[2];
    volatile double t0 = a1 * b2, u0 = a2 * b1, t1 = a2 * b0, u1 = a0 * b2, t2 = a0 * b1, u2 = a1 * b0;
    const double c0 = t0 - u0, c1 = t1 - u1, c2 = t2 - u2;
    return c0 == 0.0 && c1 == 0.0 && c2 == 0.0;
}

// set branch fast path: every draw of the call is randbelow(n) for one n (sample(points, k) with n > setsize, and
// the triples' sample(points, 1)), i.e. a word is taken iff its top bit_length(n) bits are < n. The words of each
// twist block are compacted into the accepted values (branch-free), then consumed in order.
// The compaction of one block's words into the accepted values (top bits < n) and their positions, in stream
// order: scalar (branch-free), or AVX2, 8 words a step (compare, movemask, a permutation from a 256-entry table,
// one store of the packed values and one of the positions), chosen once by the CPU's features. The host replay is
// compiled by the host compiler (g++): clang's build of the same loops ran 1.6x slower.
static int compact_scalar(const uint32_t* __restrict__ src, int i0, uint32_t n, int sh, uint32_t* __restrict__ v,
                          uint16_t* __restrict__ p) {
    int k = 0;
    for (int i = i0; i < 624; ++i) {
        const uint32_t j = src[i] >> sh;
        v[k] = j;
        p[k] = (uint16_t)i;
        k += (int)(j < n);
    }
    return k;
}

struct PackTable {   // entry m: the lanes of mask m, packed low (byte j = the j-th set lane)
    uint64_t e[256];
    PackTable() {
        for (int m = 0; m < 256; ++m) {
            uint64_t v = 0;
            int j = 0;
            for (int l = 0; l < 8; ++l)
                if (m >> l & 1) v |= (uint64_t)l << (8 * j++);
            e[m] = v;
        }
    }
};
static const PackTable g_pack;
static const bool g_avx2 = (__builtin_cpu_init(), __builtin_cpu_supports("avx2") != 0);

__attribute__((target("avx2"))) static int compact_avx2(const uint32_t* __restrict__ src, int i0, uint32_t n, int sh,
                                                        uint32_t* __restrict__ v, uint16_t* __restrict__ p) {
    int k = 0, i = i0;
    const __m256i flip = _mm256_set1_epi32((int)0x80000000u);
    const __m256i lim = _mm256_xor_si256(_mm256_set1_epi32((int)(n - 1)), flip);   // j < n <=> j <= n - 1
    const __m128i shc = _mm_cvtsi32_si128(sh);
    const __m256i lanes = _mm256_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7);
    for (; i + 8 <= 624; i += 8) {
        const __m256i j = _mm256_srl_epi32(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i)), shc);
        const __m256i rej = _mm256_cmpgt_epi32(_mm256_xor_si256(j, flip), lim);
        const uint32_t acc = ~(uint32_t)_mm256_movemask_ps(_mm256_castsi256_ps(rej)) & 0xFFu;
        const __m256i perm = _mm256_cvtepu8_epi32(_mm_cvtsi64_si128((long long)g_pack.e[acc]));
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(v + k), _mm256_permutevar8x32_epi32(j, perm));
        const __m256i ix = _mm256_add_epi32(_mm256_set1_epi32(i), _mm256_permutevar8x32_epi32(lanes, perm));
        _mm_storeu_si128(reinterpret_cast<__m128i*>(p + k),
                         _mm_packus_epi32(_mm256_castsi256_si128(ix), _mm256_extracti128_si256(ix, 1)));
        k += __builtin_popcount(acc);
    }
    return k + compact_scalar(src, i, n, sh, v + k, p + k);
}

struct AccStream {
    PyMT& rng;
    uint32_t n;
    int sh;
    alignas(32) uint32_t vals[632];   // (8 spare: the vector compaction stores whole groups of 8)
    alignas(32) uint16_t pos[632];
    int m = 0, c = 0;
    bool started = false;   // nothing is compacted (and the state not twisted) before the first value is taken
    AccStream(PyMT& r, uint32_t n_) : rng(r), n(n_), sh(__builtin_clz(n_)) {}
    void compact() {   // the accepted values of the current block from rng.index on
        if (rng.index >= 624) rng.twist();
        if (!rng.out_valid) rng.temper_all();
        const int i0 = rng.index;
        m = g_avx2 ? compact_avx2(rng.out, i0, n, sh, vals, pos) : compact_scalar(rng.out, i0, n, sh, vals, pos);
        c = 0;
    }
    __attribute__((noinline)) void refill() {
        if (!started) {   // the first value: the current block from the caller's position
            started = true;
            compact();
            if (m > 0) return;
        }
        do {   // the block's remaining words are all rejected: consumed, then the next block
            rng.index = 624;
            compact();
        } while (m == 0);
    }
    inline uint32_t next() {
        if (__builtin_expect(c == m, 0)) refill();
        return vals[c++];
    }
    // the stream position after the last value taken (the words after it in the block are not consumed)
    void finish() {
        if (c > 0) rng.index = pos[c - 1] + 1;
    }
};

static void ransac_draw_set(PyMT& rng, const double* pts, int64_t n, int64_t ld, int trials, int k, int32_t* sidx,
                            int32_t* tri) {
    std::vector<uint64_t> selected(((uint64_t)n + 63) / 64, 0);
    uint64_t* __restrict__ sel = selected.data();
    AccStream as(rng, (uint32_t)n);
    for (int t = 0; t < trials; ++t) {
        int32_t* __restrict__ dst = sidx + (int64_t)t * k;
        for (int q = 0; q < k;) {
            const uint32_t v = as.next();
            uint64_t& wd = sel[v >> 6];
            const uint64_t b = 1ull << (v & 63);
            if (__builtin_expect((wd & b) != 0, 0)) continue;   // drawn before in this sample: rejected
            wd |= b;
            dst[q++] = (int32_t)v;
        }
        for (int q = 0; q < k; ++q) sel[(uint32_t)dst[q] >> 6] = 0;
        uint32_t i1, i2, i3;
        do {
            i1 = as.next();
            i2 = as.next();
            i3 = as.next();
        } while (collinear(pts + i1 * ld, pts + i2 * ld, pts + i3 * ld));
        tri[3 * t + 0] = (int32_t)i1;
        tri[3 * t + 1] = (int32_t)i2;
        tri[3 * t + 2] = (int32_t)i3;
    }
    as.finish();
}

int ransac_draw(uint32_t* state625, const double* pts, int64_t n, int64_t ld, int trials, int k, int32_t* sidx,
                int32_t* tri) {
    if (n < k || n < 1 || n >= (1ll << 31)) return 0;   // random.sample raises before drawing: no trial runs
    PyMT rng;
    for (int i = 0; i < 624; ++i) rng.mt[i] = state625[i];
    rng.index = (int)state625[624];
    if ((int64_t)n > sample_setsize(k)) {   // every draw of the call is randbelow(n): the compacted stream
        ransac_draw_set(rng, pts, n, ld, trials, k, sidx, tri);
        for (int i = 0; i < 624; ++i) state625[i] = rng.mt[i];
        state625[624] = (uint32_t)rng.index;
        return trials;
    }
    std::vector<uint32_t> pool;
    std::vector<uint64_t> selected;
    for (int t = 0; t < trials; ++t) {
        py_sample(rng, (uint32_t)n, k, sidx + (int64_t)t * k, pool, selected);
        uint32_t i1, i2, i3;
        do {   // randomNonCollinearPoints: three sample(points, 1) per attempt
            i1 = rng.randbelow((uint32_t)n);
            i2 = rng.randbelow((uint32_t)n);
            i3 = rng.randbelow((uint32_t)n);
        } while (collinear(pts + i1 * ld, pts + i2 * ld, pts + i3 * ld));
        tri[3 * t + 0] = (int32_t)i1;
        tri[3 * t + 1] = (int32_t)i2;
        tri[3 * t + 2] = (int32_t)i3;
    }
    for (int i = 0; i < 624; ++i) state625[i] = rng.mt[i];
    state625[624] = (uint32_t)rng.index;
    return trials;
}

}  // namespace svx
