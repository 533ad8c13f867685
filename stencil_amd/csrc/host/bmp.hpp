// bmp.hpp -- 24-bit BMP dump of a grid: the colour map of
// the reference's Stencil::to_bmp (src/stencil/stencil.cpp:153-188, blue ->
// cyan -> green -> yellow -> red by quarters of [0, 1]) and the uncompressed
// BITMAPINFOHEADER layout its BMPImage writes (src/stencil/bmp_image.cpp):
// 54-byte header, rows bottom-up, each padded to 4 bytes, pixels as B, G, R.
#pragma once

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

struct BmpPixel {
    std::uint8_t b, g, r;
};

// Quarter-wise heat map of a value in [0, 1] (values are clamped).
inline BmpPixel heat_color(double v) {
    if (!(v >= 0.0)) v = 0.0;  // also maps NaN to 0
    if (v > 1.0) v = 1.0;
    auto c = [](double x) { return static_cast<std::uint8_t>(x * 255.0); };
    if (v < 0.25) return {255, c(4.0 * v), 0};
    if (v < 0.5) return {c(1.0 + 4.0 * (0.25 - v)), 255, 0};
    if (v < 0.75) return {0, 255, c(4.0 * (v - 0.5))};
    return {0, c(1.0 + 4.0 * (0.75 - v)), 255};
}

inline void put_u32(unsigned char* p, std::uint32_t v) {
    p[0] = std::uint8_t(v);
    p[1] = std::uint8_t(v >> 8);
    p[2] = std::uint8_t(v >> 16);
    p[3] = std::uint8_t(v >> 24);
}

// Write width x height pixels (row 0 first = bottom row of the image).
inline bool write_bmp24(const std::string& path, std::uint32_t width, std::uint32_t height,
                        const std::vector<BmpPixel>& px) {
    if (px.size() != std::size_t(width) * height) return false;
    const std::uint32_t pad = (4 - (width * 3) % 4) % 4;
    const std::uint32_t row_bytes = width * 3 + pad;
    unsigned char hdr[54] = {'B', 'M'};
    put_u32(hdr + 2, 54 + row_bytes * height);  // file size
    put_u32(hdr + 10, 54);                      // pixel array offset
    put_u32(hdr + 14, 40);                      // BITMAPINFOHEADER size
    put_u32(hdr + 18, width);
    put_u32(hdr + 22, height);
    hdr[26] = 1;   // colour planes
    hdr[28] = 24;  // bits per pixel
    std::FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    bool ok = std::fwrite(hdr, 1, sizeof hdr, f) == sizeof hdr;
    const unsigned char zeros[4] = {0, 0, 0, 0};
    std::vector<unsigned char> row(row_bytes, 0);
    for (std::uint32_t y = 0; ok && y < height; ++y) {
        for (std::uint32_t x = 0; x < width; ++x) {
            const BmpPixel& p = px[std::size_t(y) * width + x];
            row[3 * x] = p.b;
            row[3 * x + 1] = p.g;
            row[3 * x + 2] = p.r;
        }
        for (std::uint32_t k = 0; k < pad; ++k) row[width * 3 + k] = zeros[k];
        ok = std::fwrite(row.data(), 1, row_bytes, f) == row_bytes;
    }
    return std::fclose(f) == 0 && ok;
}
