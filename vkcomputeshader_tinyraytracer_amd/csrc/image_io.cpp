// image_io.cpp — frame files.  The reference only presents its storage image
// through the swapchain (main.cpp:2181-2205) and never writes a file; these writers are the
// build's way to hand a rendered RGBA8 frame (trt_render's out_rgba8, optionally with
// TRT_FLAG_SRGB_OUT = "as displayed") to the outside world.
//   PPM: binary P6, RGB, alpha dropped.
//   PNG: 8-bit RGBA, non-interlaced, per-row filter 1 (Sub), zlib deflate level 6.
#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/trt/abi.h"

namespace {

bool valid(const char* path, const uint8_t* rgba8, uint32_t w, uint32_t h) {
    return path && rgba8 && w && h && (uint64_t)w * h <= (1ull << 31);
}

void be32(std::vector<uint8_t>& b, uint32_t v) {
    b.push_back((uint8_t)(v >> 24));
    b.push_back((uint8_t)(v >> 16));
    b.push_back((uint8_t)(v >> 8));
    b.push_back((uint8_t)v);
}

void chunk(std::vector<uint8_t>& out, const char type[4], const uint8_t* data, size_t n) {
    be32(out, (uint32_t)n);
    const size_t at = out.size();
    out.insert(out.end(), type, type + 4);
    if (n) out.insert(out.end(), data, data + n);
    be32(out, (uint32_t)crc32(0L, out.data() + at, (uInt)(n + 4)));
}

int write_all(const char* path, const uint8_t* p, size_t n) {
    FILE* f = std::fopen(path, "wb");
    if (!f) return TRT_ERR_IO;
    const bool ok = std::fwrite(p, 1, n, f) == n;
    return (std::fclose(f) == 0 && ok) ? TRT_OK : TRT_ERR_IO;
}

} // namespace

extern "C" int trt_write_ppm(const char* path, const uint8_t* rgba8, uint32_t w, uint32_t h) {
    if (!valid(path, rgba8, w, h)) return TRT_ERR_INVALID;
    char hdr[64];
    const int nh = std::snprintf(hdr, sizeof hdr, "P6\n%u %u\n255\n", w, h);
    std::vector<uint8_t> buf((size_t)nh + (size_t)w * h * 3);
    std::memcpy(buf.data(), hdr, (size_t)nh);
    uint8_t* d = buf.data() + nh;
    for (size_t i = 0, n = (size_t)w * h; i < n; ++i) {
        d[3 * i + 0] = rgba8[4 * i + 0];
        d[3 * i + 1] = rgba8[4 * i + 1];
        d[3 * i + 2] = rgba8[4 * i + 2];
    }
    return write_all(path, buf.data(), buf.size());
}

extern "C" int trt_write_png(const char* path, const uint8_t* rgba8, uint32_t w, uint32_t h) {
    if (!valid(path, rgba8, w, h)) return TRT_ERR_INVALID;
    const size_t row = (size_t)w * 4;
    std::vector<uint8_t> raw((row + 1) * h);
    for (uint32_t y = 0; y < h; ++y) { // filter 1 (Sub): byte - byte 4 to the left, mod 256
        uint8_t* d = raw.data() + (row + 1) * y;
        const uint8_t* s = rgba8 + row * y;
        d[0] = 1;
        for (size_t i = 0; i < row; ++i) d[1 + i] = (uint8_t)(s[i] - (i >= 4 ? s[i - 4] : 0));
    }
    uLongf zn = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zn);
    if (compress2(z.data(), &zn, raw.data(), (uLong)raw.size(), 6) != Z_OK) return TRT_ERR_OOM;
    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<uint8_t> ihdr;
    be32(ihdr, w);
    be32(ihdr, h);
    const uint8_t rest[5] = {8, 6, 0, 0, 0}; // 8-bit, RGBA, deflate, adaptive filters, no interlace
    ihdr.insert(ihdr.end(), rest, rest + 5);
    chunk(out, "IHDR", ihdr.data(), ihdr.size());
    chunk(out, "IDAT", z.data(), zn);
    chunk(out, "IEND", nullptr, 0);
    return write_all(path, out.data(), out.size());
}
