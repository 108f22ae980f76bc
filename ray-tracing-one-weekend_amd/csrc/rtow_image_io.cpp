// rtow_image_io.cpp — writing frames: the reference's BMP output
// (WINDIBBitmap::writeBMPToFile, winDIBbitmap.cpp:20-168, called at
// main.cpp:774 with the BGRA frame buffer) and a PPM for inspection.
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/rtow.h"
#include "rtow_internal.h"

namespace {

void put16(std::vector<uint8_t>& b, uint16_t v) {
    b.push_back((uint8_t)(v & 0xff));
    b.push_back((uint8_t)(v >> 8));
}
void put32(std::vector<uint8_t>& b, uint32_t v) {
    for (int k = 0; k < 4; k++) b.push_back((uint8_t)(v >> (8 * k)));
}

int writeAll(const char* path, const std::vector<uint8_t>& bytes) {
    FILE* f = std::fopen(path, "wb");
    if (!f) return set_error(RTOW_E_IO, std::string("cannot open ") + path);
    const size_t n = std::fwrite(bytes.data(), 1, bytes.size(), f);
    const bool ok = n == bytes.size() && std::fclose(f) == 0;
    if (n != bytes.size()) std::fclose(f);
    return ok ? RTOW_OK : set_error(RTOW_E_IO, std::string("short write to ") + path);
}

}  // namespace

extern "C" {

// The file winDIBbitmap.cpp writes: a 14-byte BMP header and a 40-byte
// BITMAPINFOHEADER (height POSITIVE, so a reader shows the top-down frame
// buffer upside down, as the reference's test.bmp is), then the buffer rows in
// order, each zero-padded to a multiple of 4 bytes (winDIBbitmap.cpp:33-63).
int rtow_write_bmp(const char* path, const uint8_t* pixels, uint64_t size_bytes, uint32_t width, uint32_t height,
                   uint32_t bits_per_pixel) {
    if (!path || !pixels || width == 0 || height == 0) return set_error(RTOW_E_INVALID, "bad BMP arguments");
    if (bits_per_pixel != 8 && bits_per_pixel != 16 && bits_per_pixel != 24 && bits_per_pixel != 32)
        return set_error(RTOW_E_INVALID, "bits_per_pixel must be 8, 16, 24 or 32");
    const uint64_t row = (uint64_t)width * (bits_per_pixel / 8);
    if (size_bytes != row * height) return set_error(RTOW_E_INVALID, "buffer size != width * height * bpp/8");
    const uint64_t padded = ((uint64_t)bits_per_pixel * width + 31) / 32 * 4;  // ceil(bits*W/32)*4
    const uint64_t data = padded * height;
    if (54 + data > 0x7fffffffull) return set_error(RTOW_E_INVALID, "image too large for a BMP");
    std::vector<uint8_t> b;
    b.reserve(54 + data);
    b.push_back('B');
    b.push_back('M');
    put32(b, (uint32_t)(54 + data));  // bmpSize
    put16(b, 0);                      // reserved0
    put16(b, 0);                      // reserved1
    put32(b, 54);                     // pixelArrayOffset
    put32(b, 40);                     // dibHeaderSize
    put32(b, width);
    put32(b, height);
    put16(b, 1);  // colorPlanes
    put16(b, (uint16_t)bits_per_pixel);
    put32(b, 0);  // pixelArrayCompression (BI_RGB)
    put32(b, (uint32_t)data);
    put32(b, 0);  // horizontalRes
    put32(b, 0);  // verticalRes
    put32(b, 0);  // colorsInPalette
    put32(b, 0);  // importantColors
    for (uint32_t y = 0; y < height; y++) {
        b.insert(b.end(), pixels + (size_t)y * row, pixels + (size_t)(y + 1) * row);
        b.insert(b.end(), (size_t)(padded - row), 0);
    }
    return writeAll(path, b);
}

// Binary PPM (P6) of a BGRA frame, top row first: the image as displayed.
int rtow_write_ppm(const char* path, const uint8_t* bgra, uint32_t width, uint32_t height) {
    if (!path || !bgra || width == 0 || height == 0) return set_error(RTOW_E_INVALID, "bad PPM arguments");
    const std::string hdr = "P6\n" + std::to_string(width) + " " + std::to_string(height) + "\n255\n";
    std::vector<uint8_t> b(hdr.begin(), hdr.end());
    b.reserve(hdr.size() + (size_t)width * height * 3);
    for (size_t i = 0; i < (size_t)width * height; i++) {
        b.push_back(bgra[4 * i + 2]);
        b.push_back(bgra[4 * i + 1]);
        b.push_back(bgra[4 * i + 0]);
    }
    return writeAll(path, b);
}

}  // extern "C"
