// Minimal PNG (RGB8, filter 0, zlib deflate) writer for the headless dump path: the GPU box has no
// window to glReadPixels from, so frames leave through vr_frame_to_rgb8 + this instead of
// saveImage's stbi_write_png (myApp.cu:1942-1956).  Rows are written top to bottom as given.
#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "scene.h"

namespace vr {

namespace {
void put_be32(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back((uint8_t)(x >> 24)); v.push_back((uint8_t)(x >> 16));
    v.push_back((uint8_t)(x >> 8));  v.push_back((uint8_t)x);
}

void chunk(std::FILE* f, const char type[4], const std::vector<uint8_t>& data) {
    std::vector<uint8_t> buf;
    put_be32(buf, (uint32_t)data.size());
    buf.insert(buf.end(), type, type + 4);
    buf.insert(buf.end(), data.begin(), data.end());
    const uLong crc = crc32(crc32(0L, Z_NULL, 0), buf.data() + 4, (uInt)(buf.size() - 4));
    put_be32(buf, (uint32_t)crc);
    if (std::fwrite(buf.data(), 1, buf.size(), f) != buf.size()) throw std::runtime_error("png: write failed");
}
}  // namespace

void write_png_rgb8(const std::string& path, int W, int H, const uint8_t* rgb) {
    if (W <= 0 || H <= 0 || !rgb) throw std::invalid_argument("png: bad image");
    std::vector<uint8_t> raw((size_t)H * (3 * (size_t)W + 1));
    for (int r = 0; r < H; ++r) {
        uint8_t* row = raw.data() + (size_t)r * (3 * (size_t)W + 1);
        row[0] = 0;   // filter: none
        std::copy(rgb + (size_t)r * 3 * W, rgb + (size_t)(r + 1) * 3 * W, row + 1);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK)
        throw std::runtime_error("png: deflate failed");
    z.resize(zlen);
    std::FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("png: cannot open " + path);
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0d, 0x0a, 0x1a, 0x0a};
    try {
        if (std::fwrite(sig, 1, 8, f) != 8) throw std::runtime_error("png: write failed");
        std::vector<uint8_t> ihdr;
        put_be32(ihdr, (uint32_t)W); put_be32(ihdr, (uint32_t)H);
        ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});   // 8-bit, truecolour, deflate, filter 0, no interlace
        chunk(f, "IHDR", ihdr);
        chunk(f, "IDAT", z);
        chunk(f, "IEND", {});
    } catch (...) {
        std::fclose(f);
        throw;
    }
    if (std::fclose(f) != 0) throw std::runtime_error("png: close failed");
}

}  // namespace vr
