// oracle/ref_bmp.cpp — TEST INFRASTRUCTURE ONLY (never shipped).
// Drives the reference's own BMP writer, WINDIBBitmap::writeBMPToFile
// (winDIBbitmap.cpp:20-168, compiled from /root/reference by `make -C oracle
// ref`), so tests/golden can pin rtow_write_bmp byte for byte.
//
//   ref_bmp OUT_DIR IN.raw WIDTH HEIGHT BITS_PER_PIXEL
// reads IN.raw (width*height*bpp/8 bytes, the frame buffer as main.cpp:774
// hands it over), chdirs to OUT_DIR and lets the reference write test.bmp.
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <vector>

#include "winDIBbitmap.h"

int main(int argc, char** argv) {
    if (argc != 6) {
        std::fprintf(stderr, "usage: ref_bmp OUT_DIR IN.raw WIDTH HEIGHT BPP\n");
        return 2;
    }
    std::ifstream in(argv[2], std::ios::binary);
    std::vector<uint8_t> buf((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    const uint32_t w = (uint32_t)std::atoi(argv[3]), h = (uint32_t)std::atoi(argv[4]);
    const uint8_t bpp = (uint8_t)std::atoi(argv[5]);
    if (buf.size() != (size_t)w * h * (bpp / 8)) {
        std::fprintf(stderr, "input size %zu != %u x %u x %u\n", buf.size(), w, h, bpp / 8);
        return 2;
    }
    if (chdir(argv[1]) != 0) return 3;
    return (int)WINDIBBitmap::writeBMPToFile(buf.data(), (uint32_t)buf.size(), w, h, bpp);
}
