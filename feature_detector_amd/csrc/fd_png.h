// PNG decode of the ingest front end (fd_png.cpp, host only, g++).
#pragma once

#include <stddef.h>
#include <stdint.h>

namespace fdp {

enum { kPngOk = 0, kPngBadFile = 1, kPngUnsupported = 2, kPngCapacity = 3 };

struct PngInfo {
    int rows = 0, cols = 0, channels = 0;  // channels: 1 gray, 2 gray+alpha, 3 RGB, 4 RGBA (8 bits each)
};

int png_info(const uint8_t *png, size_t len, PngInfo &info);
// Samples as stored, row-major, interleaved channels; cap = bytes available at out.
int png_decode(const uint8_t *png, size_t len, uint8_t *out, size_t cap, PngInfo &info);
// n images on `threads` worker threads, image i at out + i * per_image_cap; first error wins.
int png_decode_batch(const uint8_t *const *pngs, const size_t *lens, int n, uint8_t *out, size_t per_image_cap,
                     PngInfo *infos, int threads);

}  // namespace fdp
