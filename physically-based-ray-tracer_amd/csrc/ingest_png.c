/* ingest_png.c -- PNG scanline reconstruction for the scene ingest (prt/ingest.py), the part of
 * stb_image's PNG path (template/surface.cpp:51 -> stbi_load) that is sequential per byte.  Host-only,
 * not on the hot path; zlib inflation stays in Python.  See include/prt_ingest.h. */
#include <stdint.h>
#include <stdlib.h>

#include "../../include/prt_ingest.h"

static int paeth(int a, int b, int c) {
    const int p = a + b - c, pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
    return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

int prt_png_unfilter(const uint8_t* raw, int64_t raw_len, int32_t width, int32_t height, int32_t bpp, uint8_t* out) {
    if (!raw || !out || width <= 0 || height <= 0 || bpp <= 0) return -1;
    const int64_t stride = (int64_t)width * bpp;
    if (raw_len < (stride + 1) * height) return -1;
    for (int32_t y = 0; y < height; y++) {
        const uint8_t* in = raw + y * (stride + 1);
        const int ft = in[0];
        in++;
        uint8_t* cur = out + y * stride;
        const uint8_t* prev = y > 0 ? out + (y - 1) * stride : NULL;
        for (int64_t x = 0; x < stride; x++) {
            const int a = x >= bpp ? cur[x - bpp] : 0, b = prev ? prev[x] : 0, c = (prev && x >= bpp) ? prev[x - bpp] : 0;
            int p;
            switch (ft) {
                case 0: p = 0; break;
                case 1: p = a; break;
                case 2: p = b; break;
                case 3: p = (a + b) >> 1; break;
                case 4: p = paeth(a, b, c); break;
                default: return -2;
            }
            cur[x] = (uint8_t)(in[x] + p);
        }
    }
    return 0;
}
