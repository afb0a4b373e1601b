// Host-side image I/O helpers of the C ABI (include/svx.h): the PNG scanline unfilter behind svx.io.imread, the
// reader of the reference's stereo pairs and masks (functions.py:29-35, 41-55, cv2.imread). Host code only: no
// device work (the frames then go to a batch with sv_batch_upload*).
#include <cstdint>
#include <cstdlib>

#include "../../include/svx.h"

namespace {

inline int paeth(int a, int b, int c) {   // PNG 1.2 §9.4: the neighbour nearest a + b - c, ties a, b, c
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}

}  // namespace

extern "C" int sv_png_unfilter(const uint8_t* in, int H, int rowbytes, int bpp, uint8_t* out) {
    if (!in || !out || H < 0 || rowbytes < 0 || bpp < 1 || bpp > 8) return SV_E_ARG;
    const uint8_t* prev = nullptr;   // row above (none for the first: zeros)
    for (int y = 0; y < H; ++y) {
        const uint8_t* s = in + (int64_t)y * (rowbytes + 1);
        uint8_t* d = out + (int64_t)y * rowbytes;
        const int ft = s[0];
        ++s;
        switch (ft) {
        case 0:   // None
            for (int i = 0; i < rowbytes; ++i) d[i] = s[i];
            break;
        case 1:   // Sub
            for (int i = 0; i < rowbytes; ++i) d[i] = (uint8_t)(s[i] + (i >= bpp ? d[i - bpp] : 0));
            break;
        case 2:   // Up
            for (int i = 0; i < rowbytes; ++i) d[i] = (uint8_t)(s[i] + (prev ? prev[i] : 0));
            break;
        case 3:   // Average
            for (int i = 0; i < rowbytes; ++i) {
                const int a = i >= bpp ? d[i - bpp] : 0, b = prev ? prev[i] : 0;
                d[i] = (uint8_t)(s[i] + ((a + b) >> 1));
            }
            break;
        case 4:   // Paeth
            for (int i = 0; i < rowbytes; ++i) {
                const int a = i >= bpp ? d[i - bpp] : 0, b = prev ? prev[i] : 0;
                const int c = (i >= bpp && prev) ? prev[i - bpp] : 0;
                d[i] = (uint8_t)(s[i] + paeth(a, b, c));
            }
            break;
        default:
            return SV_E_ARG;   // not a PNG filter type: a corrupt stream
        }
        prev = d;
    }
    return SV_OK;
}
