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

/* ---- Renderer::Capture (Core/Renderer.cpp:437-465): the 0x00RRGGBB screen as an 8-bit RGB PNG.
 * stb_image_write picks a filter per row; the decoded pixels are what the capture pins, so every row
 * is written with filter 0 here. */
#include <stdio.h>
#include <string.h>
#include <zlib.h>

static void put_be32(uint8_t* p, uint32_t v) { p[0] = v >> 24; p[1] = v >> 16; p[2] = v >> 8; p[3] = v; }

static int put_chunk(FILE* f, const char* kind, const uint8_t* body, uint32_t len) {
    uint8_t hdr[8];
    put_be32(hdr, len);
    memcpy(hdr + 4, kind, 4);
    uLong crc = crc32(0L, (const Bytef*)kind, 4);
    if (len) crc = crc32(crc, body, len);
    uint8_t tail[4];
    put_be32(tail, (uint32_t)crc);
    return fwrite(hdr, 1, 8, f) == 8 && (len == 0 || fwrite(body, 1, len, f) == len) && fwrite(tail, 1, 4, f) == 4;
}

int prt_capture_png(const char* path, const uint32_t* rgb8, int32_t width, int32_t height) {
    if (!path || !rgb8 || width <= 0 || height <= 0) return -1;
    const size_t stride = (size_t)width * 3 + 1, raw_len = stride * (size_t)height;
    uint8_t* raw = (uint8_t*)malloc(raw_len);
    uLongf zlen = compressBound((uLong)raw_len);
    uint8_t* z = (uint8_t*)malloc(zlen);
    if (!raw || !z) { free(raw); free(z); return -3; }
    for (int32_t y = 0; y < height; y++) {
        uint8_t* row = raw + y * stride;
        row[0] = 0;
        for (int32_t x = 0; x < width; x++) {
            const uint32_t px = rgb8[(size_t)y * width + x];
            row[1 + 3 * x] = (uint8_t)(px >> 16);
            row[2 + 3 * x] = (uint8_t)(px >> 8);
            row[3 + 3 * x] = (uint8_t)px;
        }
    }
    int rc = compress2(z, &zlen, raw, (uLong)raw_len, 6) == Z_OK ? 0 : -3;
    FILE* f = rc ? NULL : fopen(path, "wb");
    if (!rc && !f) rc = -2;
    if (!rc) {
        static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
        uint8_t ihdr[13];
        put_be32(ihdr, (uint32_t)width);
        put_be32(ihdr + 4, (uint32_t)height);
        ihdr[8] = 8; ihdr[9] = 2; ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;  /* 8-bit RGB */
        if (fwrite(sig, 1, 8, f) != 8 || !put_chunk(f, "IHDR", ihdr, 13) || !put_chunk(f, "IDAT", z, (uint32_t)zlen) ||
            !put_chunk(f, "IEND", NULL, 0))
            rc = -2;
        if (fclose(f) != 0) rc = -2;
    }
    free(raw);
    free(z);
    return rc;
}
