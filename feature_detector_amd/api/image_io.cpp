// LoadImage over fd_png_decode (include/feature_detector/image_io.h).
#include "feature_detector/image_io.h"

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fd_hip.h"

namespace feature_detector {

bool LoadImage(const std::string &path, GrayImage &image) {
    FILE *f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    std::vector<uint8_t> data;
    uint8_t chunk[1 << 16];
    size_t n;
    while ((n = std::fread(chunk, 1, sizeof chunk, f)) > 0) data.insert(data.end(), chunk, chunk + n);
    std::fclose(f);
    int32_t rows = 0, cols = 0, channels = 0;
    if (fd_png_info(data.data(), data.size(), &rows, &cols, &channels) != FD_OK) return false;
    const size_t npx = static_cast<size_t>(rows) * cols;
    uint8_t *buf = static_cast<uint8_t *>(std::malloc(npx));
    if (!buf) return false;
    if (fd_png_decode(data.data(), data.size(), buf, npx, &rows, &cols) != FD_OK) {
        std::free(buf);
        return false;
    }
    image.SetImage(buf, rows, cols, true);
    return true;
}

}  // namespace feature_detector
