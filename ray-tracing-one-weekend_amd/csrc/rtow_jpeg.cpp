// rtow_jpeg.cpp -- the JPEG reader on the texture path: what stbi_load() (the
// reference's stb_image.h v2.22, scenes.h:140) returns for a JPEG, restated.
//
// stb_image (https://github.com/nothings/stb, the reference vendors v2.22 as
// stb_image.h) is by Sean Barrett and contributors, dual-licensed: public
// domain (unlicense.org) or MIT.  MIT notice for the restated parts:
//   Copyright (c) 2017 Sean Barrett.  Permission is hereby granted, free of
//   charge, to any person obtaining a copy of this software and associated
//   documentation files (the "Software"), to deal in the Software without
//   restriction, including without limitation the rights to use, copy, modify,
//   merge, publish, distribute, sublicense, and/or sell copies of the
//   Software, and to permit persons to whom the Software is furnished to do
//   so, subject to the following conditions: The above copyright notice and
//   this permission notice shall be included in all copies or substantial
//   portions of the Software.  THE SOFTWARE IS PROVIDED "AS IS", WITHOUT
//   WARRANTY OF ANY KIND, EXPRESS OR IMPLIED.
//
// scenes.h:140 loads ./input_images/1_earth_8k.jpg with stbi_load(path, &nx,
// &ny, &nn, 0) and hands the pixels to ImageTexture.  rtow_image_decode_jpeg
// produces the same bytes: baseline and progressive Huffman JPEG, 8-bit,
// 1/3/4 components, any sampling factors, restart intervals; the
// reference's x86-64 build runs stb's SSE2 kernels (stbi__setup_jpeg,
// stb_image.h:3618-3630), whose results equal the scalar ones restated here
// (stb_image.h:2344-2346, 3454-3455; the IDCT's 16-bit intermediates are
// reproduced below).  Pinned bit for bit against the reference's own stb
// build (tests/test_jpeg.py: tests/golden/jpeg fixtures from
// oracle/_ref/ref_harness `decode`, and the reference's input_images where
// present).  Host code: decoding happens once per scene upload.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rtow.h"
#include "rtow_internal.h"

namespace {

// zigzag position -> row-major index (stb_image.h:2007-2020; the tail lets
// corrupt input run past 63 harmlessly)
const uint8_t kDezigzag[64 + 15] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
    13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45,
    38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};
const uint32_t kMask[17] = {0, 1, 3, 7, 15, 31, 63, 127, 255, 511, 1023, 2047, 4095, 8191, 16383, 32767, 65535};
const int kBias[16] = {0, -1, -3, -7, -15, -31, -63, -127, -255, -511, -1023, -2047, -4095, -8191, -16383, -32767};

struct Huffman {  // canonical code tables (stb_image.h:1823-1863, without the fast lookup)
    uint16_t code[256];
    uint8_t values[256];
    uint8_t size[257];
    uint32_t maxcode[18];
    int delta[17];
};

struct Component {
    int id = 0, h = 1, v = 1, tq = 0, hd = 0, ha = 0, dc_pred = 0;
    int x = 0, y = 0, w2 = 0, h2 = 0;
    std::vector<uint8_t> data;    // w2 x h2 samples
    std::vector<int16_t> coeff;   // progressive: coeff_w x coeff_h blocks of 64
    int coeff_w = 0, coeff_h = 0;
};

struct Decoder {
    const uint8_t* buf;
    size_t len, pos = 0;
    std::string err;

    Huffman huff_dc[4], huff_ac[4];
    uint16_t dequant[4][64] = {};
    int img_x = 0, img_y = 0, img_n = 0;
    int h_max = 1, v_max = 1, mcu_x = 0, mcu_y = 0;
    Component comp[4];
    uint32_t code_buffer = 0;
    int code_bits = 0;
    uint8_t marker = 0xff;  // STBI__MARKER_none
    bool nomore = false;
    bool progressive = false;
    int spec_start = 0, spec_end = 0, succ_high = 0, succ_low = 0, eob_run = 0;
    bool jfif = false;
    int app14 = -1;
    int rgb = 0;
    int scan_n = 0, order[4] = {0, 0, 0, 0};
    int restart_interval = 0, todo = 0;

    Decoder(const uint8_t* b, size_t n) : buf(b), len(n) {}

    bool fail(const char* why) {
        if (err.empty()) err = why;
        return false;
    }
    // stbi__get8: 0 past the end of the data
    int get8() { return pos < len ? buf[pos++] : 0; }
    int get16() {
        const int z = get8();
        return (z << 8) + get8();
    }
    bool at_eof() const { return pos >= len; }
    void skip(int n) { pos = n < 0 ? len : std::min(len, pos + (size_t)n); }

    // ---- entropy decoder (stb_image.h:1892-2003) ---------------------------
    void grow() {
        do {
            uint32_t b = nomore ? 0u : (uint32_t)get8();
            if (b == 0xff) {
                int c = get8();
                while (c == 0xff) c = get8();  // fill bytes
                if (c != 0) {
                    marker = (uint8_t)c;
                    nomore = true;
                    return;
                }
            }
            code_buffer |= b << (24 - code_bits);
            code_bits += 8;
        } while (code_bits <= 24);
    }
    int huff_decode(const Huffman& h) {
        if (code_bits < 16) grow();
        const uint32_t temp = code_buffer >> 16;
        int k = 1;
        while (k < 17 && temp >= h.maxcode[k]) k++;
        if (k == 17) {
            code_bits -= 16;
            return -1;
        }
        if (k > code_bits) return -1;
        const int c = (int)((code_buffer >> (32 - k)) & kMask[k]) + h.delta[k];
        code_bits -= k;
        code_buffer <<= k;
        return h.values[c & 255];
    }
    int extend_receive(int n) {
        if (code_bits < n) grow();
        const int sgn = (int32_t)code_buffer >> 31;
        uint32_t k = n ? (code_buffer << n) | (code_buffer >> (32 - n)) : code_buffer;
        code_buffer = k & ~kMask[n];
        k &= kMask[n];
        code_bits -= n;
        return (int)k + (kBias[n] & ~sgn);
    }
    int get_bits(int n) {
        if (code_bits < n) grow();
        uint32_t k = n ? (code_buffer << n) | (code_buffer >> (32 - n)) : code_buffer;
        code_buffer = k & ~kMask[n];
        k &= kMask[n];
        code_bits -= n;
        return (int)k;
    }
    bool get_bit() {
        if (code_bits < 1) grow();
        const uint32_t k = code_buffer;
        code_buffer <<= 1;
        --code_bits;
        return (k & 0x80000000u) != 0;
    }

    static bool build_huffman(Huffman& h, const int* count) {
        int k = 0;
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < count[i]; ++j) {
                if (k >= 256) return false;
                h.size[k++] = (uint8_t)(i + 1);
            }
        h.size[k] = 0;
        uint32_t code = 0;
        k = 0;
        int j;
        for (j = 1; j <= 16; ++j) {
            h.delta[j] = k - (int)code;
            if (h.size[k] == j) {
                while (h.size[k] == j) h.code[k++] = (uint16_t)(code++);
                if (code - 1 >= (1u << j)) return false;  // bad code lengths
            }
            h.maxcode[j] = code << (16 - j);
            code <<= 1;
        }
        h.maxcode[j] = 0xffffffffu;
        return true;
    }

    // ---- blocks (stb_image.h:2023-2229) ------------------------------------
    bool decode_block(int16_t* data, const Huffman& hdc, const Huffman& hac, int b, const uint16_t* dq) {
        if (code_bits < 16) grow();
        const int t = huff_decode(hdc);
        if (t < 0 || t > 15) return fail("bad huffman code");
        std::memset(data, 0, 64 * sizeof(int16_t));
        const int diff = t ? extend_receive(t) : 0;
        const int dc = comp[b].dc_pred + diff;
        comp[b].dc_pred = dc;
        data[0] = (int16_t)(dc * dq[0]);
        int k = 1;
        do {
            const int rs = huff_decode(hac);
            if (rs < 0) return fail("bad huffman code");
            const int s = rs & 15, r = rs >> 4;
            if (s == 0) {
                if (rs != 0xf0) break;  // end of block
                k += 16;
            } else {
                k += r;
                const int zig = kDezigzag[k++];
                data[zig] = (int16_t)(extend_receive(s) * dq[zig]);
            }
        } while (k < 64);
        return true;
    }
    bool decode_block_prog_dc(int16_t* data, const Huffman& hdc, int b) {
        if (spec_end != 0) return fail("can't merge dc and ac");
        if (code_bits < 16) grow();
        if (succ_high == 0) {
            std::memset(data, 0, 64 * sizeof(int16_t));
            const int t = huff_decode(hdc);
            if (t < 0 || t > 15) return fail("bad huffman code");
            const int diff = t ? extend_receive(t) : 0;
            const int dc = comp[b].dc_pred + diff;
            comp[b].dc_pred = dc;
            data[0] = (int16_t)(dc * (1 << succ_low));
        } else if (get_bit()) {
            data[0] = (int16_t)(data[0] + (1 << succ_low));
        }
        return true;
    }
    bool decode_block_prog_ac(int16_t* data, const Huffman& hac) {
        if (spec_start == 0) return fail("can't merge dc and ac");
        if (succ_high == 0) {
            const int shift = succ_low;
            if (eob_run) {
                --eob_run;
                return true;
            }
            int k = spec_start;
            do {
                const int rs = huff_decode(hac);
                if (rs < 0) return fail("bad huffman code");
                const int s = rs & 15, r = rs >> 4;
                if (s == 0) {
                    if (r < 15) {
                        eob_run = 1 << r;
                        if (r) eob_run += get_bits(r);
                        --eob_run;
                        break;
                    }
                    k += 16;
                } else {
                    k += r;
                    const int zig = kDezigzag[k++];
                    data[zig] = (int16_t)(extend_receive(s) * (1 << shift));
                }
            } while (k <= spec_end);
        } else {
            const int16_t bit = (int16_t)(1 << succ_low);
            if (eob_run) {
                --eob_run;
                for (int k = spec_start; k <= spec_end; ++k) {
                    int16_t* p = &data[kDezigzag[k]];
                    if (*p != 0 && get_bit() && (*p & bit) == 0) *p = (int16_t)(*p > 0 ? *p + bit : *p - bit);
                }
            } else {
                int k = spec_start;
                do {
                    const int rs = huff_decode(hac);
                    if (rs < 0) return fail("bad huffman code");
                    int s = rs & 15, r = rs >> 4;
                    if (s == 0) {
                        if (r < 15) {
                            eob_run = (1 << r) - 1;
                            if (r) eob_run += get_bits(r);
                            r = 64;  // force end of block
                        }
                        // r == 15, s == 0: a run of 15 zeros, then a zero
                    } else {
                        if (s != 1) return fail("bad huffman code");
                        s = get_bit() ? bit : -bit;
                    }
                    while (k <= spec_end) {
                        int16_t* p = &data[kDezigzag[k++]];
                        if (*p != 0) {
                            if (get_bit() && (*p & bit) == 0) *p = (int16_t)(*p > 0 ? *p + bit : *p - bit);
                        } else {
                            if (r == 0) {
                                *p = (int16_t)s;
                                break;
                            }
                            --r;
                        }
                    }
                } while (k <= spec_end);
            }
        }
        return true;
    }

    // ---- IDCT (stb_image.h:2242-2341; the SSE2 kernel the reference build
    // runs keeps 16-bit values between the passes and forms the 0+4 / 1+7 /
    // 3+5 sums in 16 bits: done here too) -----------------------------------
    static int f2f(double x) { return (int)(x * 4096 + 0.5); }
    static uint8_t clamp8(int x) { return (uint8_t)(x < 0 ? 0 : (x > 255 ? 255 : x)); }
    static int16_t sat16(int x) { return (int16_t)(x < -32768 ? -32768 : (x > 32767 ? 32767 : x)); }
    // one 1-D pass of STBI__IDCT_1D over s[0..7 * stride]: out = (x +- t + bias) >> shift
    static void idct_1d(const int16_t* s, int stride, int bias, int shift, int* out) {
        const int s0 = s[0], s1 = s[stride], s2 = s[2 * stride], s3 = s[3 * stride];
        const int s4 = s[4 * stride], s5 = s[5 * stride], s6 = s[6 * stride], s7 = s[7 * stride];
        // even part
        const int p1e = (s2 + s6) * f2f(0.5411961f);
        const int t2e = p1e + s6 * f2f(-1.847759065f);
        const int t3e = p1e + s2 * f2f(0.765366865f);
        const int t0e = (int16_t)(s0 + s4) * 4096, t1e = (int16_t)(s0 - s4) * 4096;
        const int x0 = t0e + t3e + bias, x3 = t0e - t3e + bias, x1 = t1e + t2e + bias, x2 = t1e - t2e + bias;
        // odd part (p1 = s7 + s1 and p2 = s5 + s3 formed in 16 bits, as the SSE2 kernel does)
        const int sum17 = (int16_t)(s1 + s7), sum35 = (int16_t)(s3 + s5);
        const int p5 = (sum17 + sum35) * f2f(1.175875602f);
        int t0 = s7 * f2f(0.298631336f);
        int t1 = s5 * f2f(2.053119869f);
        int t2 = s3 * f2f(3.072711026f);
        int t3 = s1 * f2f(1.501321110f);
        const int p1 = p5 + sum17 * f2f(-0.899976223f);
        const int p2 = p5 + sum35 * f2f(-2.562915447f);
        const int p3 = s7 * f2f(-1.961570560f) + s3 * f2f(-1.961570560f);
        const int p4 = s5 * f2f(-0.390180644f) + s1 * f2f(-0.390180644f);
        t3 += p1 + p4;
        t2 += p2 + p3;
        t1 += p2 + p4;
        t0 += p1 + p3;
        out[0] = (x0 + t3) >> shift;
        out[7] = (x0 - t3) >> shift;
        out[1] = (x1 + t2) >> shift;
        out[6] = (x1 - t2) >> shift;
        out[2] = (x2 + t1) >> shift;
        out[5] = (x2 - t1) >> shift;
        out[3] = (x3 + t0) >> shift;
        out[4] = (x3 - t0) >> shift;
    }
    static void idct_block(uint8_t* out, int out_stride, const int16_t* data) {
        int16_t mid[64];
        int o[8];
        for (int i = 0; i < 8; ++i) {  // columns, bias 512, >> 10, saturated to 16 bits
            idct_1d(data + i, 8, 512, 10, o);
            for (int r = 0; r < 8; ++r) mid[r * 8 + i] = sat16(o[r]);
        }
        for (int i = 0; i < 8; ++i) {  // rows, bias 0.5 * 2^17 + (128 << 17), >> 17
            idct_1d(mid + i * 8, 1, 65536 + (128 << 17), 17, o);
            for (int c = 0; c < 8; ++c) out[i * out_stride + c] = clamp8(sat16(o[c]));
        }
    }

    // ---- markers and headers (stb_image.h:2736-3244) -----------------------
    int get_marker() {
        if (marker != 0xff) {
            const int x = marker;
            marker = 0xff;
            return x;
        }
        int x = get8();
        if (x != 0xff) return 0xff;
        while (x == 0xff) x = get8();
        return x;
    }
    void reset() {
        code_bits = 0;
        code_buffer = 0;
        nomore = false;
        for (auto& c : comp) c.dc_pred = 0;
        marker = 0xff;
        todo = restart_interval ? restart_interval : 0x7fffffff;
        eob_run = 0;
    }
    bool process_marker(int m) {
        int L;
        switch (m) {
        case 0xff:
            return fail("expected marker");
        case 0xdd:  // DRI
            if (get16() != 4) return fail("bad DRI len");
            restart_interval = get16();
            return true;
        case 0xdb:  // DQT
            L = get16() - 2;
            while (L > 0) {
                const int q = get8();
                const int p = q >> 4, t = q & 15;
                if (p != 0 && p != 1) return fail("bad DQT type");
                if (t > 3) return fail("bad DQT table");
                for (int i = 0; i < 64; ++i) dequant[t][kDezigzag[i]] = (uint16_t)(p ? get16() : get8());
                L -= p ? 129 : 65;
            }
            return L == 0 || fail("bad DQT len");
        case 0xc4:  // DHT
            L = get16() - 2;
            while (L > 0) {
                const int q = get8();
                const int tc = q >> 4, th = q & 15;
                if (tc > 1 || th > 3) return fail("bad DHT header");
                int sizes[16], n = 0;
                for (int i = 0; i < 16; ++i) {
                    sizes[i] = get8();
                    n += sizes[i];
                }
                L -= 17;
                Huffman& h = tc == 0 ? huff_dc[th] : huff_ac[th];
                if (!build_huffman(h, sizes)) return fail("bad code lengths");
                for (int i = 0; i < n; ++i) h.values[i & 255] = (uint8_t)get8();
                L -= n;
            }
            return L == 0 || fail("bad DHT len");
        }
        if ((m >= 0xe0 && m <= 0xef) || m == 0xfe) {  // APPn, COM
            L = get16();
            if (L < 2) return fail("bad APP len");
            L -= 2;
            if (m == 0xe0 && L >= 5) {  // JFIF
                static const uint8_t tag[5] = {'J', 'F', 'I', 'F', 0};
                bool ok = true;
                for (int i = 0; i < 5; ++i) ok = get8() == tag[i] && ok;
                L -= 5;
                if (ok) jfif = true;
            } else if (m == 0xee && L >= 12) {  // Adobe APP14
                static const uint8_t tag[6] = {'A', 'd', 'o', 'b', 'e', 0};
                bool ok = true;
                for (int i = 0; i < 6; ++i) ok = get8() == tag[i] && ok;
                L -= 6;
                if (ok) {
                    get8();
                    get16();
                    get16();
                    app14 = get8();
                    L -= 6;
                }
            }
            skip(L);
            return true;
        }
        return fail("unknown marker");
    }
    bool scan_header() {
        const int Ls = get16();
        scan_n = get8();
        if (scan_n < 1 || scan_n > 4 || scan_n > img_n) return fail("bad SOS component count");
        if (Ls != 6 + 2 * scan_n) return fail("bad SOS len");
        for (int i = 0; i < scan_n; ++i) {
            const int id = get8(), q = get8();
            int which = 0;
            while (which < img_n && comp[which].id != id) which++;
            if (which == img_n) return fail("bad SOS component");
            comp[which].hd = q >> 4;
            comp[which].ha = q & 15;
            if (comp[which].hd > 3 || comp[which].ha > 3) return fail("bad huffman table id");
            order[i] = which;
        }
        spec_start = get8();
        spec_end = get8();
        const int aa = get8();
        succ_high = aa >> 4;
        succ_low = aa & 15;
        if (progressive) {
            if (spec_start > 63 || spec_end > 63 || spec_start > spec_end || succ_high > 13 || succ_low > 13)
                return fail("bad SOS");
        } else {
            if (spec_start != 0 || succ_high != 0 || succ_low != 0) return fail("bad SOS");
            spec_end = 63;
        }
        return true;
    }
    bool frame_header() {
        const int Lf = get16();
        if (Lf < 11) return fail("bad SOF len");
        if (get8() != 8) return fail("only 8-bit");
        img_y = get16();
        if (img_y == 0) return fail("no header height");
        img_x = get16();
        if (img_x == 0) return fail("0 width");
        const int c = get8();
        if (c != 3 && c != 1 && c != 4) return fail("bad component count");
        img_n = c;
        if (Lf != 8 + 3 * img_n) return fail("bad SOF len");
        rgb = 0;
        for (int i = 0; i < img_n; ++i) {
            static const uint8_t rgbid[3] = {'R', 'G', 'B'};
            comp[i].id = get8();
            if (img_n == 3 && comp[i].id == rgbid[i]) ++rgb;
            const int q = get8();
            comp[i].h = q >> 4;
            comp[i].v = q & 15;
            comp[i].tq = get8();
            if (!comp[i].h || comp[i].h > 4) return fail("bad H");
            if (!comp[i].v || comp[i].v > 4) return fail("bad V");
            if (comp[i].tq > 3) return fail("bad TQ");
        }
        if ((uint64_t)img_x * img_y * img_n > (1ull << 31)) return fail("too large");
        for (int i = 0; i < img_n; ++i) {
            h_max = std::max(h_max, comp[i].h);
            v_max = std::max(v_max, comp[i].v);
        }
        // sampling factors that do not divide the maximum (H=3 beside H=2)
        // would make the colour conversion read a row past a component plane
        // (stb 2.22 accepts them; later stb versions reject them the same way,
        // and 2.22's output for such files is undefined)
        for (int i = 0; i < img_n; ++i) {
            if (h_max % comp[i].h != 0) return fail("bad H");
            if (v_max % comp[i].v != 0) return fail("bad V");
        }
        mcu_x = (img_x + h_max * 8 - 1) / (h_max * 8);
        mcu_y = (img_y + v_max * 8 - 1) / (v_max * 8);
        for (int i = 0; i < img_n; ++i) {
            Component& C = comp[i];
            C.x = (img_x * C.h + h_max - 1) / h_max;
            C.y = (img_y * C.v + v_max - 1) / v_max;
            C.w2 = mcu_x * C.h * 8;
            C.h2 = mcu_y * C.v * 8;
            C.data.assign((size_t)C.w2 * C.h2, 0);
            if (progressive) {
                C.coeff_w = C.w2 / 8;
                C.coeff_h = C.h2 / 8;
                C.coeff.assign((size_t)C.w2 * C.h2, 0);
            }
        }
        return true;
    }
    // after every MCU: the restart interval (stb_image.h:2786-2792)
    bool restart_due(bool& stop) {
        stop = false;
        if (--todo <= 0) {
            if (code_bits < 24) grow();
            if (!(marker >= 0xd0 && marker <= 0xd7)) {
                stop = true;  // not a restart: keep what was decoded
                return true;
            }
            reset();
        }
        return true;
    }
    bool entropy_data() {
        reset();
        alignas(16) int16_t data[64];
        bool stop = false;
        if (scan_n == 1) {  // non-interleaved: every block is an MCU
            const int n = order[0];
            Component& C = comp[n];
            const int w = (C.x + 7) >> 3, h = (C.y + 7) >> 3;
            for (int j = 0; j < h; ++j)
                for (int i = 0; i < w; ++i) {
                    if (!progressive) {
                        if (!decode_block(data, huff_dc[C.hd], huff_ac[C.ha], n, dequant[C.tq])) return false;
                        idct_block(C.data.data() + (size_t)C.w2 * j * 8 + i * 8, C.w2, data);
                    } else {
                        int16_t* d = C.coeff.data() + 64 * ((size_t)i + (size_t)j * C.coeff_w);
                        if (spec_start == 0) {
                            if (!decode_block_prog_dc(d, huff_dc[C.hd], n)) return false;
                        } else if (!decode_block_prog_ac(d, huff_ac[C.ha])) {
                            return false;
                        }
                    }
                    restart_due(stop);
                    if (stop) return true;
                }
            return true;
        }
        for (int j = 0; j < mcu_y; ++j)  // interleaved MCUs
            for (int i = 0; i < mcu_x; ++i) {
                for (int k = 0; k < scan_n; ++k) {
                    const int n = order[k];
                    Component& C = comp[n];
                    for (int y = 0; y < C.v; ++y)
                        for (int x = 0; x < C.h; ++x) {
                            const int x2 = i * C.h + x, y2 = j * C.v + y;
                            if (!progressive) {
                                if (!decode_block(data, huff_dc[C.hd], huff_ac[C.ha], n, dequant[C.tq])) return false;
                                idct_block(C.data.data() + (size_t)C.w2 * y2 * 8 + x2 * 8, C.w2, data);
                            } else if (!decode_block_prog_dc(C.coeff.data() + 64 * ((size_t)x2 + (size_t)y2 * C.coeff_w),
                                                             huff_dc[C.hd], n)) {
                                return false;
                            }
                        }
                }
                restart_due(stop);
                if (stop) return true;
            }
        return true;
    }
    void finish_progressive() {  // dequantize + IDCT every block (stb_image.h:2901-2918)
        for (int n = 0; n < img_n; ++n) {
            Component& C = comp[n];
            const int w = (C.x + 7) >> 3, h = (C.y + 7) >> 3;
            for (int j = 0; j < h; ++j)
                for (int i = 0; i < w; ++i) {
                    int16_t* d = C.coeff.data() + 64 * ((size_t)i + (size_t)j * C.coeff_w);
                    for (int q = 0; q < 64; ++q) d[q] = (int16_t)(d[q] * dequant[C.tq][q]);
                    idct_block(C.data.data() + (size_t)C.w2 * j * 8 + i * 8, C.w2, d);
                }
        }
    }
    bool decode() {
        marker = 0xff;
        if (get_marker() != 0xd8) return fail("no SOI");
        int m = get_marker();
        while (!(m == 0xc0 || m == 0xc1 || m == 0xc2)) {
            if (!process_marker(m)) return false;
            m = get_marker();
            while (m == 0xff) {
                if (at_eof()) return fail("no SOF");
                m = get_marker();
            }
        }
        progressive = m == 0xc2;
        if (!frame_header()) return false;
        m = get_marker();
        while (m != 0xd9) {
            if (m == 0xda) {
                if (!scan_header() || !entropy_data()) return false;
                if (marker == 0xff) {  // zeros at the end of the data: look for the next marker
                    while (!at_eof()) {
                        if (get8() == 255) {
                            marker = (uint8_t)get8();
                            break;
                        }
                    }
                }
            } else if (m == 0xdc) {  // DNL
                const int Ld = get16();
                const int NL = get16();
                if (Ld != 4) return fail("bad DNL len");
                if (NL != img_y) return fail("bad DNL height");
            } else if (!process_marker(m)) {
                return false;
            }
            m = get_marker();
            if (m == 0xff && at_eof()) return fail("no EOI");
        }
        if (progressive) finish_progressive();
        return true;
    }
};

// ---- upsampling and colour (stb_image.h:3251-3480, 3656-3828) --------------
inline uint8_t div4(int x) { return (uint8_t)(x >> 2); }
inline uint8_t div16(int x) { return (uint8_t)(x >> 4); }

const uint8_t* resample(int hs, int vs, uint8_t* out, const uint8_t* in_near, const uint8_t* in_far, int w) {
    if (hs == 1 && vs == 1) return in_near;
    if (hs == 1 && vs == 2) {
        for (int i = 0; i < w; ++i) out[i] = div4(3 * in_near[i] + in_far[i] + 2);
        return out;
    }
    if (hs == 2 && vs == 1) {
        const uint8_t* in = in_near;
        if (w == 1) {
            out[0] = out[1] = in[0];
            return out;
        }
        out[0] = in[0];
        out[1] = div4(in[0] * 3 + in[1] + 2);
        int i;
        for (i = 1; i < w - 1; ++i) {
            const int n = 3 * in[i] + 2;
            out[i * 2 + 0] = div4(n + in[i - 1]);
            out[i * 2 + 1] = div4(n + in[i + 1]);
        }
        out[i * 2 + 0] = div4(in[w - 2] * 3 + in[w - 1] + 2);
        out[i * 2 + 1] = in[w - 1];
        return out;
    }
    if (hs == 2 && vs == 2) {
        if (w == 1) {
            out[0] = out[1] = div4(3 * in_near[0] + in_far[0] + 2);
            return out;
        }
        int t1 = 3 * in_near[0] + in_far[0], t0;
        out[0] = div4(t1 + 2);
        for (int i = 1; i < w; ++i) {
            t0 = t1;
            t1 = 3 * in_near[i] + in_far[i];
            out[i * 2 - 1] = div16(3 * t0 + t1 + 8);
            out[i * 2] = div16(3 * t1 + t0 + 8);
        }
        out[w * 2 - 1] = div4(t1 + 2);
        return out;
    }
    for (int i = 0; i < w; ++i)  // nearest neighbour
        for (int j = 0; j < hs; ++j) out[i * hs + j] = in_near[i];
    return out;
}

inline int float2fixed(float x) { return ((int)(x * 4096.0f + 0.5f)) << 8; }

void ycbcr_to_rgb(uint8_t* out, const uint8_t* y, const uint8_t* pcb, const uint8_t* pcr, int count, int step) {
    for (int i = 0; i < count; ++i) {
        const int y_fixed = (y[i] << 20) + (1 << 19);
        const int cr = pcr[i] - 128, cb = pcb[i] - 128;
        int r = y_fixed + cr * float2fixed(1.40200f);
        int g = y_fixed + cr * -float2fixed(0.71414f) + (int)((unsigned)(cb * -float2fixed(0.34414f)) & 0xffff0000u);
        int b = y_fixed + cb * float2fixed(1.77200f);
        r >>= 20;
        g >>= 20;
        b >>= 20;
        out[0] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
        out[1] = (uint8_t)(g < 0 ? 0 : (g > 255 ? 255 : g));
        out[2] = (uint8_t)(b < 0 ? 0 : (b > 255 ? 255 : b));
        out += step;
    }
}

inline uint8_t blinn(uint8_t x, uint8_t y) {
    const unsigned t = (unsigned)x * y + 128;
    return (uint8_t)((t + (t >> 8)) >> 8);
}

}  // namespace

extern "C" int rtow_image_decode_jpeg(const uint8_t* data, size_t size, uint8_t** pixels, uint32_t* nx, uint32_t* ny,
                                      uint32_t* channels) {
    if (!data || !pixels || !nx || !ny || !channels) return set_error(RTOW_E_INVALID, "NULL argument");
    *pixels = nullptr;
    Decoder z(data, size);
    if (!z.decode()) return set_error(RTOW_E_IO, "JPEG: " + z.err);
    // stbi_load(..., 0): 3 channels for 3/4-component images, 1 otherwise
    const int n = z.img_n >= 3 ? 3 : 1;
    const bool is_rgb = z.img_n == 3 && (z.rgb == 3 || (z.app14 == 0 && !z.jfif));
    const int decode_n = z.img_n;
    struct Res {
        int hs, vs, ystep, w_lores, ypos;
        const uint8_t *line0, *line1;
    } res[4];
    std::vector<uint8_t> linebuf[4];
    for (int k = 0; k < decode_n; ++k) {
        Res& r = res[k];
        linebuf[k].assign((size_t)z.img_x + 3, 0);
        r.hs = z.h_max / z.comp[k].h;
        r.vs = z.v_max / z.comp[k].v;
        r.ystep = r.vs >> 1;
        r.w_lores = (z.img_x + r.hs - 1) / r.hs;
        r.ypos = 0;
        r.line0 = r.line1 = z.comp[k].data.data();
    }
    const size_t bytes = (size_t)n * z.img_x * z.img_y;
    uint8_t* out_all = static_cast<uint8_t*>(std::malloc(bytes + 1));
    if (!out_all) return set_error(RTOW_E_NOMEM, "JPEG: out of memory");
    const uint8_t* co[4] = {nullptr, nullptr, nullptr, nullptr};
    for (int j = 0; j < z.img_y; ++j) {
        uint8_t* out = out_all + (size_t)n * z.img_x * j;
        for (int k = 0; k < decode_n; ++k) {
            Res& r = res[k];
            const bool y_bot = r.ystep >= (r.vs >> 1);
            co[k] = resample(r.hs, r.vs, linebuf[k].data(), y_bot ? r.line1 : r.line0, y_bot ? r.line0 : r.line1,
                             r.w_lores);
            if (++r.ystep >= r.vs) {
                r.ystep = 0;
                r.line0 = r.line1;
                if (++r.ypos < z.comp[k].y) r.line1 += z.comp[k].w2;
            }
        }
        if (n == 3) {
            if (z.img_n == 3) {
                if (is_rgb) {
                    for (int i = 0; i < z.img_x; ++i, out += 3) {
                        out[0] = co[0][i];
                        out[1] = co[1][i];
                        out[2] = co[2][i];
                    }
                } else {
                    ycbcr_to_rgb(out, co[0], co[1], co[2], z.img_x, 3);
                }
            } else if (z.app14 == 0) {  // CMYK
                for (int i = 0; i < z.img_x; ++i, out += 3) {
                    const uint8_t m = co[3][i];
                    out[0] = blinn(co[0][i], m);
                    out[1] = blinn(co[1][i], m);
                    out[2] = blinn(co[2][i], m);
                }
            } else if (z.app14 == 2) {  // YCCK
                ycbcr_to_rgb(out, co[0], co[1], co[2], z.img_x, 3);
                for (int i = 0; i < z.img_x; ++i, out += 3) {
                    const uint8_t m = co[3][i];
                    out[0] = blinn((uint8_t)(255 - out[0]), m);
                    out[1] = blinn((uint8_t)(255 - out[1]), m);
                    out[2] = blinn((uint8_t)(255 - out[2]), m);
                }
            } else {  // YCbCr + a fourth channel stb ignores
                ycbcr_to_rgb(out, co[0], co[1], co[2], z.img_x, 3);
            }
        } else {
            std::memcpy(out, co[0], (size_t)z.img_x);
        }
    }
    *pixels = out_all;
    *nx = (uint32_t)z.img_x;
    *ny = (uint32_t)z.img_y;
    *channels = (uint32_t)n;
    return RTOW_OK;
}

extern "C" int rtow_image_load_jpeg(const char* path, uint8_t** pixels, uint32_t* nx, uint32_t* ny,
                                    uint32_t* channels) {
    if (!path) return set_error(RTOW_E_INVALID, "NULL path");
    FILE* f = std::fopen(path, "rb");
    if (!f) return set_error(RTOW_E_IO, std::string("cannot open ") + path);
    std::vector<uint8_t> bytes;
    uint8_t chunk[1 << 16];
    size_t got;
    while ((got = std::fread(chunk, 1, sizeof chunk, f)) > 0) bytes.insert(bytes.end(), chunk, chunk + got);
    std::fclose(f);
    return rtow_image_decode_jpeg(bytes.data(), bytes.size(), pixels, nx, ny, channels);
}

extern "C" void rtow_image_free(uint8_t* pixels) { std::free(pixels); }
