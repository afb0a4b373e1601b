// Host-side row gathers of the C ABI (include/svx.h) for the one-by-one stage drop-ins (svx/stages.py,
// svx/dropin.py). The reference passes points between stereovision.py:97-113's stages as a list of rows; the
// drop-ins keep them as an index selection of projectDisparityTo3d's (N, 6) float64 array (svx/points.py), so a
// stage's device input is a gather of some of its columns. numpy's fancy indexing of the whole rows plus a
// dtype conversion cost 1-3 ms a stage at 60-90K points (extras.dropin_frame_chain a5-a7); one pass here reads
// only the columns the stage uploads. Host code only: no device work.
#include <cstdint>

#include "../../include/svx.h"

// every index must name one of the nrows rows (idx NULL: rows 0..n-1, n <= nrows)
static bool rows_ok(int64_t nrows, const int64_t* idx, int64_t n) {
    if (!idx) return n <= nrows;
    for (int64_t i = 0; i < n; ++i)
        if ((uint64_t)idx[i] >= (uint64_t)nrows) return false;
    return true;
}

extern "C" int sv_gather_rgb_u8(const double* rows, int64_t nrows, int64_t ld, const int64_t* idx, int64_t n,
                                uint8_t* out) {
    if (!rows || !out || ld < 6 || n < 0 || !rows_ok(nrows, idx, n)) return SV_E_ARG;
    for (int64_t i = 0; i < n; ++i) {
        const double* r = rows + (idx ? idx[i] : i) * ld + 3;
        for (int c = 0; c < 3; ++c) {
            const double v = r[c];
            // the colour stages hash integer colours only (functions.py:73-78 keys): an integer in [0, 255]
            if (!(v >= 0.0 && v <= 255.0) || v != (double)(int)v) return SV_E_ARG;
            out[3 * i + c] = (uint8_t)(int)v;
        }
    }
    return SV_OK;
}

extern "C" int sv_gather_f64(const double* rows, int64_t nrows, int64_t ld, const int64_t* idx, int64_t n, int c0,
                             int nc, double* out) {
    if (!rows || !out || n < 0 || c0 < 0 || nc < 1 || c0 + nc > ld || !rows_ok(nrows, idx, n)) return SV_E_ARG;
    for (int64_t i = 0; i < n; ++i) {
        const double* r = rows + (idx ? idx[i] : i) * ld + c0;
        double* o = out + i * nc;
        for (int c = 0; c < nc; ++c) o[c] = r[c];
    }
    return SV_OK;
}
