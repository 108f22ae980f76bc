"""The float identities the device kernels lean on, checked on the host
(IEEE binary32 arithmetic is the same there; the C is compiled with gcc).

div_by (rtow_device.hip): x / a == fma(fma(-q0, a, x), y, q0) with
y = RN(1/a), q0 = RN(x*y) -- the sphere roots, sphere normals and rectangle
planes divide this way, from a reciprocal hoisted per ray or per sphere."""
import os
import shutil
import subprocess

import pytest

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static uint64_t s = 88172645463325252ull;
static uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static float mk(uint32_t e, uint32_t m, int neg) { uint32_t b = (e << 23) | m | (neg ? 0x80000000u : 0); float f; memcpy(&f, &b, 4); return f; }
static int check(float x, float a) {
    float y = 1.0f / a, q0 = x * y, r = fmaf(-q0, a, x), q1 = fmaf(r, y, q0), q = x / a;
    return q1 == q || (q == 0 && q1 == 0);
}
int main(void) {
    long bad = 0, n = 0;
    const uint32_t special[] = {0, 1, 2, 0x7fffff, 0x7ffffe, 0x400000, 0x3fffff, 0x555555};
    for (int k = 0; k < 8; k++)
        for (uint32_t ea = 118; ea < 138; ea++)
            for (uint32_t mx = 0; mx < 0x800000; mx += 7) { bad += !check(mk(124, mx, mx & 1), mk(ea, special[k], 0)); n++; }
    for (long i = 0; i < 20000000L; i++) {
        float a = mk(117 + (uint32_t)(xr() % 30), (uint32_t)(xr() & 0x7fffff), 0);
        float x = mk(97 + (uint32_t)(xr() % 60), (uint32_t)(xr() & 0x7fffff), (int)(xr() & 1));
        bad += !check(x, a); n++;
    }
    printf("%ld %ld\n", bad, n);
    return 0;
}
"""


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_fma_corrected_division_is_the_ieee_quotient(tmp_path):
    c = tmp_path / "div.c"
    c.write_text(SRC)
    exe = tmp_path / "div"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(c), "-lm"], check=True)
    bad, n = map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split())
    assert n > 40_000_000 and bad == 0


SRC_F64 = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static inline double mk(double x, double d, double r) { double q0 = x * r; return fma(fma(-q0, d, x), r, q0); }
int main(int argc, char** argv) {
    const long step = 97;  /* the device claim was checked for every float; this samples them */
    const double d1 = 2 * M_PI, r1 = 1.0 / d1, d2 = M_PI, r2 = 1.0 / d2;
    long bad = 0, n = 0;
    for (long u = 0; u < (1L << 32); u += step) {
        float f; uint32_t b = (uint32_t)u; memcpy(&f, &b, 4);
        if (f >= -3.14159274f && f <= 3.14159274f) { double x = (double)f + M_PI; bad += x / d1 != mk(x, d1, r1); n++; }
        if (f >= -1.57079637f && f <= 1.57079637f) { double x = (double)f + M_PI / 2; bad += x / d2 != mk(x, d2, r2); n++; }
    }
    const float r = 1.0f / 255.0f;
    for (int i = 0; i < 256; i++) {
        float x = (float)i, q0 = x * r, q = fmaf(fmaf(-q0, 255.0f, x), r, q0);
        bad += q != (float)(i / 255.0); n++;
    }
    printf("%ld %ld\n", bad, n);
    return 0;
}
"""


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_uv_and_texel_divisions(tmp_path):
    """sphere_uv's (phi + pi) / 2pi and (theta + pi/2) / pi (mathUtilities.h:
    62-68) in double via the reciprocal and one fma residual step equal the
    IEEE quotients for the floats atan2f / asinf return (every one of the
    4.3e9 was checked once; this samples every 97th bit pattern), and
    ImageTexture's c / 255.0 (texture.h:76), rounded to float, is div_by's
    float result for all 256 byte values."""
    src = tmp_path / "f64.c"
    src.write_text(SRC_F64)
    exe = tmp_path / "f64"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(src), "-lm"], check=True)
    bad, n = (int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split())
    assert n > 40_000_000 and bad == 0
