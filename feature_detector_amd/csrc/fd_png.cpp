// fd_png.cpp -- PNG decode for the ingest front end: the reference loads its frames
// with Visualizor2D::LoadImage (test/test_feature_point_detector.cpp:104, un-vendored).
//
// Host part of fd_png_decode / fd_png_to_frames (fd_runtime.cpp): zlib inflate of the IDAT stream and
// the per-row PNG filters (None / Sub / Up / Average / Paeth, PNG spec §9), which are serial along a
// row and from row to row -- CPU work, done per image on worker threads. The output is the image's
// samples as stored (gray or RGB / RGBA / gray+alpha, 8 bits); colour images become gray on the GPU
// (k_rgb_gray). Supported: bit depth 8, colour types 0, 2, 4, 6, no interlace (the reference's
// examples: image.png is 8-bit gray, image2.png 8-bit RGB).
#include "fd_png.h"

#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace fdp {

namespace {

uint32_t be32(const uint8_t *p) {
    return (static_cast<uint32_t>(p[0]) << 24) | (static_cast<uint32_t>(p[1]) << 16) |
           (static_cast<uint32_t>(p[2]) << 8) | static_cast<uint32_t>(p[3]);
}

int channels_of(int ctype) {
    switch (ctype) {
        case 0: return 1;  // gray
        case 2: return 3;  // RGB
        case 4: return 2;  // gray + alpha
        case 6: return 4;  // RGBA
        default: return 0;
    }
}

// Chunks of the stream: IHDR geometry and the concatenated IDAT payload.
int parse(const uint8_t *png, size_t len, PngInfo &info, std::vector<uint8_t> *idat) {
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    if (!png || len < 8 + 25 || std::memcmp(png, sig, 8) != 0) return kPngBadFile;
    size_t pos = 8;
    bool have_hdr = false;
    while (pos + 12 <= len) {
        const uint32_t n = be32(png + pos);
        const uint8_t *type = png + pos + 4;
        const uint8_t *body = png + pos + 8;
        if (n > len - pos - 12) return kPngBadFile;
        if (std::memcmp(type, "IHDR", 4) == 0) {
            if (n < 13) return kPngBadFile;
            info.cols = static_cast<int>(be32(body));
            info.rows = static_cast<int>(be32(body + 4));
            const int depth = body[8], ctype = body[9], interlace = body[12];
            info.channels = channels_of(ctype);
            if (depth != 8 || info.channels == 0 || interlace != 0) return kPngUnsupported;
            if (info.rows <= 0 || info.cols <= 0 || static_cast<int64_t>(info.rows) * info.cols >= (int64_t(1) << 31))
                return kPngBadFile;
            have_hdr = true;
        } else if (std::memcmp(type, "IDAT", 4) == 0) {
            if (idat) idat->insert(idat->end(), body, body + n);
        } else if (std::memcmp(type, "IEND", 4) == 0) {
            break;
        }
        pos += 12 + static_cast<size_t>(n);
    }
    return have_hdr ? kPngOk : kPngBadFile;
}

inline int paeth(int a, int b, int c) {
    const int p = a + b - c;
    const int pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

}  // namespace

int png_info(const uint8_t *png, size_t len, PngInfo &info) { return parse(png, len, info, nullptr); }

int png_decode(const uint8_t *png, size_t len, uint8_t *out, size_t cap, PngInfo &info) {
    std::vector<uint8_t> idat;
    int rc = parse(png, len, info, &idat);
    if (rc) return rc;
    const size_t bpp = static_cast<size_t>(info.channels);
    const size_t stride = static_cast<size_t>(info.cols) * bpp;
    const size_t need = stride * static_cast<size_t>(info.rows);
    if (cap < need) return kPngCapacity;
    // inflate: every row is one filter-type byte + stride bytes
    std::vector<uint8_t> raw((stride + 1) * static_cast<size_t>(info.rows));
    z_stream zs{};
    if (inflateInit(&zs) != Z_OK) return kPngBadFile;
    zs.next_in = idat.data();
    zs.avail_in = static_cast<uInt>(idat.size());
    zs.next_out = raw.data();
    zs.avail_out = static_cast<uInt>(raw.size());
    const int zr = inflate(&zs, Z_FINISH);
    const size_t got = raw.size() - zs.avail_out;
    inflateEnd(&zs);
    if ((zr != Z_STREAM_END && zr != Z_OK) || got != raw.size()) return kPngBadFile;
    // unfilter in place into out (PNG spec §9.2; a = left, b = up, c = up-left, 0 outside)
    for (int r = 0; r < info.rows; ++r) {
        const uint8_t ft = raw[static_cast<size_t>(r) * (stride + 1)];
        const uint8_t *src = raw.data() + static_cast<size_t>(r) * (stride + 1) + 1;
        uint8_t *dst = out + static_cast<size_t>(r) * stride;
        const uint8_t *up = r > 0 ? dst - stride : nullptr;
        for (size_t i = 0; i < stride; ++i) {
            const int a = i >= bpp ? dst[i - bpp] : 0;
            const int b = up ? up[i] : 0;
            const int c = (up && i >= bpp) ? up[i - bpp] : 0;
            int p;
            switch (ft) {
                case 0: p = 0; break;
                case 1: p = a; break;
                case 2: p = b; break;
                case 3: p = (a + b) >> 1; break;
                case 4: p = paeth(a, b, c); break;
                default: return kPngBadFile;
            }
            dst[i] = static_cast<uint8_t>(src[i] + p);
        }
    }
    return kPngOk;
}

int png_decode_batch(const uint8_t *const *pngs, const size_t *lens, int n, uint8_t *out, size_t per_image_cap,
                     PngInfo *infos, int threads) {
    std::atomic<int> next{0}, err{kPngOk};
    auto worker = [&]() {
        for (int i = next.fetch_add(1); i < n; i = next.fetch_add(1)) {
            const int rc = png_decode(pngs[i], lens[i], out + static_cast<size_t>(i) * per_image_cap, per_image_cap,
                                      infos[i]);
            if (rc) {
                int expected = kPngOk;
                err.compare_exchange_strong(expected, rc);
            }
        }
    };
    threads = std::max(1, std::min(threads, n));
    if (threads == 1) {
        worker();
    } else {
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; ++t) pool.emplace_back(worker);
        for (auto &t : pool) t.join();
    }
    return err.load();
}

}  // namespace fdp
