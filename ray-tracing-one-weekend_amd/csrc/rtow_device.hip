// rtow_device.hip — gfx950 kernels and the device half of the C-ABI.
//
// What replaces main.cpp:932-996 (DESIGN.md has the full picture):
//
//   trace_kernel   persistent wavefronts.  One lane = one path.  A lane owns a
//                  work item = (pixel, chunk of consecutive samples); when its
//                  path ends it starts the next sample, and when its chunk is
//                  done it writes the chunk sum and takes a new item.  Items are
//                  handed out per WAVE: __ballot of the lanes that need work,
//                  one atomicAdd by the leader for popcount(mask) items, and a
//                  mask-prefix rank per lane -- so live lanes are refilled (the
//                  "compaction") every bounce without leaving the kernel.
//                  color() (color.h:12-59) is unrolled into the bounce loop; the
//                  world->hit recursion (bvhNode.h:66-96, hitableList.h:20-38,
//                  hitable.h:25-154) is an explicit traversal with a per-lane
//                  stack in LDS (column-major: conflict-free).
//   resolve_kernel sums each pixel's chunk sums in order, applies the
//                  /= float(spp) (vec3.h:133-139), sqrt gamma and the 255.99
//                  quantisation (main.cpp:955-970) and writes BGRA8 (+ linear).
//   assemble_kernel scatters rank tile slabs into the framebuffer
//                  (main.cpp:982-989 layout).
//
// Numerics: compiled with -ffp-contract=off and HIP's default correctly
// rounded f32 division/sqrt, every float expression mirrors the reference's
// shape (oracle/rtow_oracle.c restates the same expressions on the CPU), and
// random numbers come from include/rtow_rng.h, keyed per (pixel, sample).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/rtow.h"
#include "../../include/rtow_rng.h"
#include "rtow_device_layout.h"
#include "rtow_internal.h"


using namespace rtow_dev;

// Device code lives in a named namespace so that one kernel instantiation can
// come from a second compilation of this file with its own code-generation
// flags (RTOW_TU_SIMPLE, see the Makefile and the end of this section).
namespace rtow_k {

// Block size of every general-scene kernel: the general traversal (dnode_step,
// traverse) strides a lane's LDS stack column by BLOCK, so a general kernel
// must be instantiated with BS == BLOCK (static_assert in trace_kernel); only
// the simple-scene traversal (trace_simple) takes the block size as BS.
constexpr int BLOCK = 256;

// ---------------------------------------------------------------------------
// small vector math with the reference's exact operation order (vec3.h)
struct F3 {
    float x, y, z;
};
__device__ __forceinline__ F3 f3(float x, float y, float z) { return F3{x, y, z}; }
__device__ __forceinline__ F3 add(F3 a, F3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ F3 sub(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ F3 mulv(F3 a, F3 b) { return f3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ F3 scl(float t, F3 v) { return f3(t * v.x, t * v.y, t * v.z); }
__device__ __forceinline__ F3 divs(F3 v, float t) { return f3(v.x / t, v.y / t, v.z / t); }
__device__ __forceinline__ F3 neg(F3 v) { return f3(-v.x, -v.y, -v.z); }
__device__ __forceinline__ float dot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float len(F3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }
__device__ __forceinline__ float sqlen(F3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
__device__ __forceinline__ F3 unit(F3 v) {
    float l = len(v);
    if (l == 0.0f) return f3(0, 0, 0);
    return divs(v, l);
}
__device__ __forceinline__ F3 ld3(const float* p) { return f3(p[0], p[1], p[2]); }

// Scene records read through the constant address space: the scene is
// read-only for a kernel's lifetime, and a load whose address is uniform
// across the wave (the top-level scan's items, their instance chains, Box
// corners, media: every lane is on the same item) then becomes a scalar
// s_load into SGPRs through the scalar cache, used directly as VALU operands,
// instead of a 64-lane vector load through the vector L1 (the general
// kernels' waves wait ~45 % of their cycles, mostly on vector memory).  A
// divergent address still compiles to a vector load.  RTOW_SCALAR=0 reads
// them as plain global loads (A/B).
#ifndef RTOW_SCALAR
#define RTOW_SCALAR 1
#endif
#define RTOW_CONST_AS __attribute__((address_space(4)))
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));  // 16-B aligned: a divergent load stays one dwordx4
template <class T>
__device__ __forceinline__ T cld(const T* p) {
#if RTOW_SCALAR
    static_assert(sizeof(T) % 4 == 0, "dword records");
    uint32_t w[sizeof(T) / 4];
    if constexpr (sizeof(T) % 16 == 0 && alignof(T) >= 16) {
        const RTOW_CONST_AS u32x4_t* q = (const RTOW_CONST_AS u32x4_t*)p;
#pragma unroll
        for (int i = 0; i < (int)(sizeof(T) / 16); i++) {
            const u32x4_t v = q[i];
            w[4 * i] = v.x;
            w[4 * i + 1] = v.y;
            w[4 * i + 2] = v.z;
            w[4 * i + 3] = v.w;
        }
    } else {
        const RTOW_CONST_AS uint32_t* q = (const RTOW_CONST_AS uint32_t*)p;
#pragma unroll
        for (int i = 0; i < (int)(sizeof(T) / 4); i++) w[i] = q[i];
    }
    T out;
    __builtin_memcpy(&out, w, sizeof(T));
    return out;
#else
    return *p;
#endif
}
// 16 bytes at a 16-B aligned address
__device__ __forceinline__ float4 cld4(const void* p) {
#if RTOW_SCALAR
    const u32x4_t v = *(const RTOW_CONST_AS u32x4_t*)p;
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
#else
    return *reinterpret_cast<const float4*>(p);
#endif
}
__device__ __forceinline__ float comp(F3 v, uint32_t i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }

struct Ray {
    F3 o, d;
    float time;
};
__device__ __forceinline__ F3 at(const Ray& r, float t) { return add(r.o, scl(t, r.d)); }

struct Rng {
    uint64_t key;
    uint32_t ctr;
    __device__ __forceinline__ double next() {
        return (double)rtow_draw24(key, ctr++) * (1.0 / 16777216.0);
    }
    // the same draw as a float: U = r24 * 2^-24 is exact in float, so
    // (float)next() == nextf() and a double U compared with, or rounded to,
    // a float gives what nextf() gives -- without the f64 conversions
    __device__ __forceinline__ float nextf() { return (float)rtow_draw24(key, ctr++) * (1.0f / 16777216.0f); }
};

struct DevCam {
    float origin[3], llc[3], hor[3], ver[3], u[3], v[3];
    float lens_radius, t0, t1;
};

// Chunks of a pixel's samples (one work item = one chunk of one pixel): n_big
// chunks of spc samples (the last one shorter when there is no tail), then,
// for auto chunking, a tail of R = spp - n_big*spc samples (spc <= R < 2 spc)
// cut into halving chunks: tail chunk k holds samples
// [base + R - L(k), base + R - L(k+1)), L(k) = ceil(R / 2^k), L(n_tail) = 0 --
// R = 16 gives 8, 4, 2, 1, 1.  The n_big full chunks run pixel-major (item =
// pixel * n_big + chunk), the tail chunk-major after them, so the grid ends
// on one-sample items instead of spc-sample ones: a short tail at every rank
// count.
struct DevParams {
    uint32_t width, height, spp, spc;  // spc: samples per chunk
    uint32_t n_chunks, n_local_px, tiles_x, rank, world;
    uint32_t n_big, tail_r, n_tail;
    uint32_t max_depth, gi_enable;
    uint32_t dof;  // RTOW_FLAG_CAMERA_DOF: camera.h:124-126 with CAMERA_DOF_EN 1
    float sky_gain, gi_gain;
    uint64_t seed;
    uint32_t n_items;
    uint32_t sample_base;  // progressive frames: the samples already accumulated (RNG sample index offset)
    // rtow_debug_trace_sample: the one (column, row, sample) whose segments
    // the DBG kernel records (RTOW_DEBUG_SEG_FLOATS floats each) into dbg_out
    uint32_t dbg_col, dbg_row, dbg_sample, dbg_max;
    float* dbg_out;
    struct XFrame* xframes;  // xhit's call frames: DevScene::xdepth x xstride (the grid's threads)
    uint32_t xstride;
    uint32_t spare;  // unused (keeps the kernels' argument layout of the measured builds)
};

struct Rec {
    float t, u, v;
    F3 p, n;
    uint32_t mat;
};

// ---------------------------------------------------------------------------
// instances (hitable.h:53-62, 125-154)
__device__ __forceinline__ Ray apply_inst(const DevScene& S, uint32_t ref, const Ray& r) {
    const uint32_t kind = ref >> KIND_SHIFT;
    const DInst& I = S.inst[ref & INDEX_MASK];
    Ray q = r;
    if (kind == DK_TRANSLATE) {
        q.o = sub(r.o, f3(I.p[0], I.p[1], I.p[2]));
    } else if (kind == DK_ROTY) {
        const float s = I.p[0], c = I.p[1];
        q.o.x = c * r.o.x - s * r.o.z;
        q.o.z = s * r.o.x + c * r.o.z;
        q.d.x = c * r.d.x - s * r.d.z;
        q.d.z = s * r.d.x + c * r.d.z;
    }
    return q;
}

// the ray through a simple scene's root instances (registers, kernel argument)
__device__ __forceinline__ Ray root_ray(const DevScene& S, const Ray& w) {
    Ray r = w;
#pragma unroll
    for (int k = 0; k < ROOTCHAIN; k++)
        if (k < (int)S.root_chain_n) r = apply_inst(S, S.root_chain[k], r);
    return r;
}

// the ray in the frame of chain `id` (DevScene::chains), outermost first
__device__ __forceinline__ void chain_step(float4 e, Ray& r) {
    const uint32_t kind = __float_as_uint(e.x) >> KIND_SHIFT;
    if (kind == DK_TRANSLATE) {
        r.o = sub(r.o, f3(e.y, e.z, e.w));
    } else if (kind == DK_ROTY) {  // apply_inst's operations
        const float sn = e.y, c = e.z;
        const F3 o = r.o, d = r.d;
        r.o.x = c * o.x - sn * o.z;
        r.o.z = sn * o.x + c * o.z;
        r.d.x = c * d.x - sn * d.z;
        r.d.z = sn * d.x + c * d.z;
    }
}
__device__ __forceinline__ Ray chain_ray(const DevScene& S, uint32_t id, const Ray& w) {
    const DChainX* C = S.chains + id;
    // the count and the first two entries in one round trip (the scan's
    // scalar loads otherwise wait for each other: count, entry 0, entry 1, ...)
    const int n = (int)cld(&C->n);
    const float4 e0 = cld4(C->t), e1 = cld4(C->t + 1);
    Ray r = w;
    if (n > 0) chain_step(e0, r);
    if (n > 1) chain_step(e1, r);
    for (int k = 2; k < n; k++) chain_step(cld4(C->t + k), r);
    return r;
}

// the way out of one instance (hitable.h:28-36, 53-62, 137-150)
__device__ __forceinline__ void inst_out(const DevScene& S, uint32_t ref, F3& p, F3& nrm);

// the way out of the instances, innermost first
__device__ __forceinline__ void chain_out_step(float4 e, F3& p, F3& nrm) {  // inst_out's operations
    const uint32_t kind = __float_as_uint(e.x) >> KIND_SHIFT;
    if (kind == DK_FLIP) {
        nrm = neg(nrm);
    } else if (kind == DK_TRANSLATE) {
        p = add(p, f3(e.y, e.z, e.w));
    } else {
        const float sn = e.y, c = e.z;
        F3 q = p, m = nrm;
        q.x = c * p.x + sn * p.z;
        q.z = -sn * p.x + c * p.z;
        m.x = c * nrm.x + sn * nrm.z;
        m.z = -sn * nrm.x + c * nrm.z;
        p = q;
        nrm = m;
    }
}
__device__ __forceinline__ void chain_out(const DevScene& S, uint32_t id, F3& p, F3& nrm) {
    const DChainX* C = S.chains + id;
    // (the count and the first two entries in one round trip, as chain_ray)
    const int n = (int)cld(&C->n);
    const float4 e0 = cld4(C->t), e1 = cld4(C->t + 1);
    for (int k = n - 1; k >= 0; k--) chain_out_step(k == 0 ? e0 : (k == 1 ? e1 : cld4(C->t + k)), p, nrm);
}

__device__ __forceinline__ void root_out(const DevScene& S, F3& p, F3& nrm) {
#pragma unroll
    for (int k = ROOTCHAIN - 1; k >= 0; k--)
        if (k < (int)S.root_chain_n) inst_out(S, S.root_chain[k], p, nrm);
}

__device__ __forceinline__ void inst_out(const DevScene& S, uint32_t ref, F3& p, F3& nrm) {
    const uint32_t ik = ref >> KIND_SHIFT;
    const DInst& I = S.inst[ref & INDEX_MASK];
    if (ik == DK_FLIP) {
        nrm = neg(nrm);
    } else if (ik == DK_TRANSLATE) {
        p = add(p, f3(I.p[0], I.p[1], I.p[2]));
    } else {
        const float s = I.p[0], c = I.p[1];
        F3 q = p, m = nrm;
        q.x = c * p.x + s * p.z;
        q.z = -s * p.x + c * p.z;
        m.x = c * nrm.x + s * nrm.z;
        m.z = -s * nrm.x + c * nrm.z;
        p = q;
        nrm = m;
    }
}

__device__ __forceinline__ F3 inv_dir(F3 d) { return f3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z); }

// Per-ray slab constants.  Each plane is (x - o) * (1/d): NOT the one-fma
// form x*(1/d) - o/d, which cancels catastrophically when the origin is far
// from the box compared with the box's distance (the random scene sits under
// Translate(..., (0,0,1000)): in the BVH frame o.z ~ -1000, boxes ~1 away) and
// then culls subtrees holding the true closest hit.  x - o is exact for
// nearby planes (Sterbenz), so the error stays within a few ulp of t.
// (The simple-scene kernel uses the one-FMA form in the world frame:
// SlabRayF below.)
struct SlabRay {
    F3 o, inv;
};
__device__ __forceinline__ SlabRay slab_ray_inv(F3 o, F3 inv) {
    SlabRay s;
    s.o = o;
    s.inv = inv;
    return s;
}
__device__ __forceinline__ SlabRay slab_ray(const Ray& r) { return slab_ray_inv(r.o, inv_dir(r.d)); }

// min(a, b) as the bare v_min_f32.  fminf() makes the compiler canonicalise
// an operand it cannot prove canonical (the culling bound is a loop-carried
// select: one extra v_max_f32 per slab test).  The slab tests' operands are
// never signalling NaNs (a quiet NaN from (x - o) * inf gives the other
// operand either way), so the result is fminf's.
__device__ __forceinline__ float min_hw(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// Conservative slab test for culling (never the reference's own AABB::hit,
// whose divisions only decide WHICH subtrees it visits, not the result).
// The box's exit is widened by 2^-9 relative (see below);
// tmax_c is the culling bound, the best hit so far widened by cull_bound().
__device__ __forceinline__ bool slab(float x0, float x1, float y0, float y1, float z0, float z1, const SlabRay& q,
                                     float tmin, float tmax_c, float& tnear) {
    const float tx0 = (x0 - q.o.x) * q.inv.x, tx1 = (x1 - q.o.x) * q.inv.x;
    const float ty0 = (y0 - q.o.y) * q.inv.y, ty1 = (y1 - q.o.y) * q.inv.y;
    const float tz0 = (z0 - q.o.z) * q.inv.z, tz1 = (z1 - q.o.z) * q.inv.z;
    const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), tmin));
    const float ex = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
    // ex * (1 + 2^-9): for ex >= 0 the exit widened by 2^-9 relative; for
    // ex < 0 the box lies behind the ray and stays culled (tn >= tmin > 0).
    // Not just the planes' rounding: a ray that passes a sphere's box by a
    // hair can still get a root from Sphere::hit's quadratic (the cancellation
    // of b*b - a*c near tangency), and the reference, testing every leaf,
    // keeps it.  Widened by 2^-19, 11 pixels of final_ned at 1024^2 x 512 spp
    // differed from the oracle by > 1e-6; by 2^-13 or 2^-9, 2 (the same two
    // in both: transcendentals), at no measurable cost (tools/diverge.py).
    const float tf = min_hw(ex * 1.001953125f, tmax_c);
    tnear = tn;
    return tn <= tf;
}

// The simple-scene kernel's slab test: each plane is x*(1/d) - o*(1/d), one
// FMA with o*(1/d) hoisted per ray, in the world frame (the DNode boxes moved
// there by shiftBoxes: the rays' origins lie near the boxes).  The error of a
// plane's t is at most 2^-24 (|o/d| + |t|) (plus the world-frame origin's own
// rounding, also below 2^-24 |o/d|), so the exit is widened by 2^-9 relative
// (covering the |t| part) and by werr = 2^-21 max|o/d| absolute: culling
// stays conservative in any frame.  1/d is clamped to +-2^64 (a zero
// direction component gives planes at +-huge instead of +-inf, so x*(1/d) -
// o*(1/d) never forms inf - inf; with |1/d| > 2^64 every plane of the axis
// lies beyond any distance the scene has either way).
struct SlabRayF {
    F3 oi, inv;
    float werr;
};
__device__ __forceinline__ SlabRayF slab_ray_f(F3 o, F3 d) {
    constexpr float BIG = 0x1p64f;
    SlabRayF s;
    const F3 inv = inv_dir(d);
    s.inv = f3(fminf(fmaxf(inv.x, -BIG), BIG), fminf(fmaxf(inv.y, -BIG), BIG), fminf(fmaxf(inv.z, -BIG), BIG));
    s.oi = mulv(o, s.inv);
    s.werr = fmaxf(fmaxf(fabsf(s.oi.x), fabsf(s.oi.y)), fabsf(s.oi.z)) * 0x1p-21f;
    return s;
}
__device__ __forceinline__ bool slab_f(float x0, float x1, float y0, float y1, float z0, float z1, const SlabRayF& q,
                                       float tmin, float tmax_c, float& tnear) {
    const float tx0 = fmaf(x0, q.inv.x, -q.oi.x), tx1 = fmaf(x1, q.inv.x, -q.oi.x);
    const float ty0 = fmaf(y0, q.inv.y, -q.oi.y), ty1 = fmaf(y1, q.inv.y, -q.oi.y);
    const float tz0 = fmaf(z0, q.inv.z, -q.oi.z), tz1 = fmaf(z1, q.inv.z, -q.oi.z);
    const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), tmin));
    const float ex = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
    const float tf = min_hw(fmaf(ex, 1.001953125f, q.werr), tmax_c);  // see slab()
    tnear = tn;
    return tn <= tf;
}

// The culling bound for a best hit at t.  A sphere root near tangency carries
// the cancellation of b*b - a*c: its computed t can sit ~2^-10.5 * t before the
// ray reaches the sphere's box at all (the reference never culls by the best
// hit, so it still finds that root).  Boxes are culled only beyond t*(1+2^-9).
// t + |t| * 2^-9 with one rounding either way (|t| * 2^-9 is exact): one FMA,
// the |t| a source modifier (-ffp-contract=off keeps the mul + add otherwise)
__device__ __forceinline__ float cull_bound(float t) { return fmaf(fabsf(t), 0.001953125f, t); }

// ---- spheres: Sphere::hit sphere.h:20-69 and MovingSphere::hit sphere.h:93-118
struct Sph {
    F3 c0;
    float r;
    F3 dc;  // center1 - center0
    float t0, t1;
    uint32_t mat, moving;
};

__device__ __forceinline__ Sph load_sph(const DSphere* p) {
    const float4 a = cld4(p);
    const float4 b = cld4(reinterpret_cast<const float4*>(p) + 1);
    const float4 c = cld4(reinterpret_cast<const float4*>(p) + 2);
    Sph s;
    s.c0 = f3(a.x, a.y, a.z);
    s.r = a.w;
    s.dc = f3(b.x, b.y, b.z);
    s.t0 = b.w;
    s.t1 = c.x;
    s.mat = __float_as_uint(c.y);
    s.moving = __float_as_uint(c.z);
    return s;
}

// sphere.h:129-131 (a static sphere has dc = 0, so this is c0 exactly)
template <bool UNIT_TIME>
__device__ __forceinline__ F3 sph_center(const Sph& s, float time) {
    const float f = UNIT_TIME ? time : (time - s.t0) / (s.t1 - s.t0);  // (time-0)/(1-0) == time exactly
    return add(s.c0, scl(f, s.dc));
}

// x / a, correctly rounded, from ra = 1/a (itself an IEEE division, hoisted
// per ray or per sphere): q = x*ra is within 1 ulp of x/a and one FMA
// residual step rounds it exactly (Markstein's correction; with ra the
// correctly rounded reciprocal the result equals the IEEE quotient -- checked
// against every float mantissa at several exponents, 8e9 cases, and 2e8
// random pairs over the ranges that occur; zero results may differ in sign,
// which no comparison here sees).  3 VALU instead of the 10 of v_div_scale /
// v_div_fmas / v_div_fixup.
__device__ __forceinline__ float div_by(float x, float a, float ra) {
    const float q0 = x * ra;
    const float r = fmaf(-q0, a, x);
    return fmaf(r, ra, q0);
}

// div_by for a divisor that may be zero (ra = +-inf): x/0 is +-inf and 0/0 NaN,
// as the IEEE division gives them (the residual is NaN there; q0 is the answer)
__device__ __forceinline__ float div_by_any(float x, float a, float ra) {
    const float q0 = x * ra;
    const float r = fmaf(-q0, a, x);
    return r == r ? fmaf(r, ra, q0) : q0;
}

// The sphere tests' sqrt(disc), disc > 0: v_sqrt_f32 (within 1 ulp) and the
// two one-ulp FMA residual corrections of sqrtf's own expansion, without its
// selects for 0 / inf / NaN.  !FAST keeps sqrtf's rescaling of inputs below
// 2^-96 and equals sqrtf for every positive float (tools/sqrt_check.hip
// checks all of them on the GPU).  FAST drops the rescaling (7 VALU of a
// sphere test's 17; config 2 +1.8 %): equal for every x >= 2^-96 and +inf,
// off for smaller ones (v_sqrt_f32's error there exceeds one ulp; the result
// stays below 2^-48).  Where that can reach a frame: a root (-b -+ sq) / a is
// accepted only above tmin = 0.001; disc in (0, 2^-96) forces b*b < 2^-70
// (else b*b - a*c is 0 or at least 2^-96: Sterbenz), so |-b -+ sq| < 2^-34.9
// and the root is below 2^-34.9 / a -- under tmin unless a = dot(d, d) <
// 2^-24.  The simple-scene traversal therefore runs FAST only for rays with
// dot(d, d) >= 2^-24 (every camera ray, all but a vanishing fraction of
// Lambertian bounces, (p + n + r) - p with r within 2^-12 of -n) and the exact
// variant for the rest; the general kernels use the exact variant
// (tests/test_gpu_sqrt.py constructs such a ray).  RTOW_SQRT_POS=0: sqrtf;
// 2: the exact variant everywhere.
#ifndef RTOW_SQRT_POS
#define RTOW_SQRT_POS 1
#endif
// Sphere::hit's root choice as one select (near root if above tmin, else the
// far one): fewer VALU, measured better in the simple-scene kernel only
// (config 2 +1.1 %, final_ned -0.6 %: the general kernels keep the two tests)
#ifndef RTOW_ROOT_SEL
#if defined(RTOW_TU_SIMPLE)
#define RTOW_ROOT_SEL 1
#else
#define RTOW_ROOT_SEL 0
#endif
#endif
template <bool FAST>
__device__ __forceinline__ float sqrt_pos(float x) {
#if RTOW_SQRT_POS
    constexpr bool F = FAST && RTOW_SQRT_POS == 1;
    const bool small = !F && x < 0x1p-96f;
    if constexpr (!F) x = small ? x * 0x1p32f : x;
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sdn = __uint_as_float(__float_as_uint(s) - 1u);
    const float sup = __uint_as_float(__float_as_uint(s) + 1u);
    const float rdn = fmaf(-sdn, s, x), rup = fmaf(-sup, s, x);
    const float t = rdn <= 0.0f ? sdn : s;
    const float u = rup > 0.0f ? sup : t;
    if constexpr (F) return u;
    return small ? u * 0x1p-16f : u;
#else
    return sqrtf(x);
#endif
}

// the root the reference records, strictly inside (tmin, tmax)
// `a` = dot(d, d) is the same for every sphere a ray meets: hoisted per ray.
__device__ __forceinline__ bool sph_quad(F3 center, float radius, const Ray& r, float a, float ra, float tmin,
                                         float tmax, float& t) {
    const F3 oc = sub(r.o, center);
    const float b = dot(r.d, oc);
    const float c = dot(oc, oc) - radius * radius;
    const float disc = b * b - a * c;
    if (disc > 0) {
        const float sq = sqrt_pos<false>(disc);
        const float tn = div_by(-b - sq, a, ra);
        if (tn < tmax && tn > tmin) {
            t = tn;
            return true;
        }
        const float tf = div_by(-b + sq, a, ra);
        if (tf < tmax && tf > tmin) {
            t = tf;
            return true;
        }
    }
    return false;
}

// Sphere::hit over the reference's whole window (tmin, MAXFLOAT) (color.h:17
// passes MAXFLOAT), then BvhNode::hit's merge of two records (bvhNode.h:74-77):
// the nearer wins and an exact tie goes to the later leaf of the reference
// tree, i.e. the larger sphere index (see rebuildSah).  `bt`/`best` is the
// record so far.  The far root is only evaluated when the near one is <= tmin.
// rr: radius * radius (a DNode's sphere slot holds it, rounded as the
// reference's radius*radius is)
template <bool FAST = false>
__device__ __forceinline__ bool sph_root(F3 center, float rr, const Ray& r, float a, float ra, float tmin,
                                         float& t) {
    const F3 oc = sub(r.o, center);
    const float b = dot(r.d, oc);
    const float c = dot(oc, oc) - rr;
    const float disc = b * b - a * c;
    if (disc > 0) {
        const float sq = sqrt_pos<FAST>(disc);
        // the near root, or the far one when the near is not above tmin; the
        // far root is never below the near one (-b + sq >= -b - sq, a > 0), so
        // a near root >= FLT_MAX leaves none (Sphere::hit's two tests)
#if RTOW_ROOT_SEL
        const float tn = div_by(-b - sq, a, ra), tf = div_by(-b + sq, a, ra);
        const float root = tn > tmin ? tn : tf;
#else
        float root = div_by(-b - sq, a, ra);
        if (!(root < FLT_MAX && root > tmin)) root = div_by(-b + sq, a, ra);
#endif
        t = root;
        return root < FLT_MAX && root > tmin;
    }
    return false;
}

__device__ __forceinline__ bool sph_closer(F3 center, float rr, const Ray& r, float a, float ra, float tmin,
                                           float bt, uint32_t best, uint32_t ref, float& t) {
    return sph_root(center, rr, r, a, ra, tmin, t) && (t < bt || (t == bt && ref > best));
}

template <bool UNIT_TIME>
__device__ __forceinline__ bool sph_t(const Sph& s, const Ray& r, float a, float ra, float tmin, float tmax, float& t) {
    return sph_quad(sph_center<UNIT_TIME>(s, r.time), s.r, r, a, ra, tmin, tmax, t);
}

// xy_rect.h:22-40, 57-75, 92-110 (closed interval: t == tmax is a hit)
__device__ __forceinline__ void rect_axes(uint32_t axis, uint32_t& i, uint32_t& j, uint32_t& k) {
    i = axis == 2 ? 1u : 0u;
    j = axis == 0 ? 1u : 2u;
    k = axis == 0 ? 2u : (axis == 1 ? 1u : 0u);
}
// inv: the ray's per-axis IEEE reciprocals (SlabRay), so the division is div_by's
__device__ __forceinline__ bool rect_t(const DRect& q, const Ray& r, const F3& inv, float t0, float t1, float& t) {
    uint32_t i, j, k;
    rect_axes(q.axis & 3u, i, j, k);
    const float tt = div_by_any(q.k - comp(r.o, k), comp(r.d, k), comp(inv, k));
    if (tt < t0 || tt > t1) return false;
    const float x = comp(r.o, i) + tt * comp(r.d, i);
    const float y = comp(r.o, j) + tt * comp(r.d, j);
    if (x < q.a0 || x > q.a1 || y < q.b0 || y > q.b1) return false;
    t = tt;
    return true;
}

// rect_t with the axes known at compile time: K the plane's axis, I and J the
// in-plane ones (rect_axes: XY K=2 I=0 J=1, XZ K=1 I=0 J=2, YZ K=0 I=1 J=2);
// the same float operations, without selecting components at run time
template <int A>
__device__ __forceinline__ float cmp3(const F3& v) { return A == 0 ? v.x : (A == 1 ? v.y : v.z); }
template <int K, int I, int J>
__device__ __forceinline__ bool rect_t_ax(float a0, float a1, float b0, float b1, float k, const Ray& r, const F3& inv,
                                          float t0, float t1, float& t) {
    const float tt = div_by_any(k - cmp3<K>(r.o), cmp3<K>(r.d), cmp3<K>(inv));
    if (tt < t0 || tt > t1) return false;
    const float x = cmp3<I>(r.o) + tt * cmp3<I>(r.d);
    const float y = cmp3<J>(r.o) + tt * cmp3<J>(r.d);
    if (x < a0 || x > a1 || y < b0 || y > b1) return false;
    t = tt;
    return true;
}

// AABB::hit (aabb.h:22-43) exactly: true divisions, ffmin/ffmax, `tmax <= tmin`
// (a NaN comparison does not reject).  b: min xyz, 0, max xyz, 0.
__device__ __forceinline__ bool ref_slab(float mn, float mx, float o, float d, float& tmin, float& tmax) {
    const float p = (mn - o) / d, q = (mx - o) / d;
    const float t0 = p < q ? p : q, t1 = p > q ? p : q;
    tmin = t0 > tmin ? t0 : tmin;
    tmax = t1 < tmax ? t1 : tmax;
    return !(tmax <= tmin);
}
__device__ __forceinline__ bool ref_aabb_hit(const float* b, const Ray& r, float tmin, float tmax) {
    const float4 lo = *(const float4*)b, hi = *(const float4*)(b + 4);
    return ref_slab(lo.x, hi.x, r.o.x, r.d.x, tmin, tmax) && ref_slab(lo.y, hi.y, r.o.y, r.d.y, tmin, tmax) &&
           ref_slab(lo.z, hi.z, r.o.z, r.d.z, tmin, tmax);
}

// The same with the ray's IEEE reciprocals: (x - o) / d as div_by_any gives
// it (the correctly rounded quotient; +-inf and NaN where d is zero)
__device__ __forceinline__ bool ref_slab_inv(float mn, float mx, float o, float d, float rd, float& tmin, float& tmax) {
    const float p = div_by_any(mn - o, d, rd), q = div_by_any(mx - o, d, rd);
    const float t0 = p < q ? p : q, t1 = p > q ? p : q;
    tmin = t0 > tmin ? t0 : tmin;
    tmax = t1 < tmax ? t1 : tmax;
    return !(tmax <= tmin);
}
__device__ __forceinline__ bool ref_aabb_hit_inv(const float* b, const Ray& r, const F3& inv, float tmin, float tmax) {
    const float4 lo = *(const float4*)b, hi = *(const float4*)(b + 4);
    return ref_slab_inv(lo.x, hi.x, r.o.x, r.d.x, inv.x, tmin, tmax) &&
           ref_slab_inv(lo.y, hi.y, r.o.y, r.d.y, inv.y, tmin, tmax) &&
           ref_slab_inv(lo.z, hi.z, r.o.z, r.d.z, inv.z, tmin, tmax);
}

// Does the reference test rectangle `rect` for this ray at all?  BvhNode::hit
// (bvhNode.h:66-71) tests its own box before its children, with the interval
// color() hands down (tmin, MAXFLOAT), so a ray that grazes a box edge -- one
// point or an empty interval after rounding -- never reaches the Box's sides
// there, although the rectangle test (closed bounds) would take the edge
// point.  `r`: the ray in the rectangle's frame, which is the frame of the
// BvhNodes recorded for it.
__device__ __forceinline__ bool ref_reaches_rect(const DevScene& S, uint32_t rect, const Ray& r, float tmin) {
    const uint32_t a = S.rect_anc[rect];
    const uint32_t n = a & 255u, off = a >> 8;
    for (uint32_t k = 0; k < n; k++)
        if (!ref_aabb_hit(S.abox + 8 * (size_t)(off + k), r, tmin, FLT_MAX)) return false;
    return true;
}

// The winning hit of a traversal, rectangle `rect` at t: would the reference
// have skipped it (ref_reaches_rect)?  Only a hit within rounding of the
// rectangle's edge can be skipped (a ray through a face's interior crosses
// its box, and every box above it, in an interval of positive length), so the
// box tests run only for hits within 2^-14 (relative to the rectangle's
// coordinates) of an edge.  `wray`: the world ray.
__device__ __forceinline__ bool ref_skips_hit(const DevScene& S, uint32_t rect, const Ray& wray, float t, float tmin) {
    if ((S.rect_anc[rect] & 255u) == 0) return false;
    const DRect q = S.rect[rect];
    const Ray r = chain_ray(S, q.chain, wray);
    uint32_t i, j, k;
    rect_axes(q.axis & 3u, i, j, k);
    const float x = comp(r.o, i) + t * comp(r.d, i);
    const float y = comp(r.o, j) + t * comp(r.d, j);
    const float ex = (fabsf(q.a0) + fabsf(q.a1) + 1.0f) * 0x1p-14f, ey = (fabsf(q.b0) + fabsf(q.b1) + 1.0f) * 0x1p-14f;
    const bool edge = x - q.a0 < ex || q.a1 - x < ex || y - q.b0 < ey || q.b1 - y < ey;
    return edge && !ref_reaches_rect(S, rect, r, tmin);
}
// ref_skips_hit for a rectangle hit at the t its plane gives (rect_t's
// division: the t it held the record at)
__device__ __forceinline__ bool ref_skips_rect(const DevScene& S, uint32_t rect, const Ray& wray, float tmin) {
    if ((S.rect_anc[rect] & 255u) == 0) return false;
    const DRect q = S.rect[rect];
    const Ray r = chain_ray(S, q.chain, wray);
    uint32_t i, j, k;
    rect_axes(q.axis & 3u, i, j, k);
    const float dk = comp(r.d, k);
    return ref_skips_hit(S, rect, wray, div_by_any(q.k - comp(r.o, k), dk, 1.0f / dk), tmin);
}

// A Box's six sides (DBox6) in their list order (box.h:29-38), each tested as
// the rectangle-list loop tests it: the interval [tmin, bt] shrinks as sides
// are taken, exact ties go by the tie keys.  Returns whether a side was taken.
__device__ __forceinline__ bool take_hit(const DevScene& S, float t, float& bt, uint32_t& best, uint32_t cand);
template <int K, int I, int J>
__device__ __forceinline__ void box6_side(const DevScene& S, float a0, float a1, float b0, float b1, float k,
                                          uint32_t rect, const Ray& r, const F3& inv, float tmin, float& bt,
                                          uint32_t& best, bool& found) {
    float t;
    if (rect_t_ax<K, I, J>(a0, a1, b0, b1, k, r, inv, tmin, bt, t) && take_hit(S, t, bt, best, mkref(DK_RECT, rect)))
        found = true;
}
__device__ __forceinline__ bool box6_scan(const DevScene& S, uint32_t bi, const Ray& r, const F3& inv, float tmin,
                                          float& bt, uint32_t& best) {
    const float4 lo = cld4(S.box6 + bi);
    const float4 hi = cld4(reinterpret_cast<const float4*>(S.box6 + bi) + 1);
    const uint32_t f = __float_as_uint(lo.w);
    bool found = false;
    box6_side<2, 0, 1>(S, lo.x, hi.x, lo.y, hi.y, hi.z, f + 0, r, inv, tmin, bt, best, found);  // XY at z1 (flipped)
    box6_side<2, 0, 1>(S, lo.x, hi.x, lo.y, hi.y, lo.z, f + 1, r, inv, tmin, bt, best, found);  // XY at z0
    box6_side<1, 0, 2>(S, lo.x, hi.x, lo.z, hi.z, hi.y, f + 2, r, inv, tmin, bt, best, found);  // XZ at y1
    box6_side<1, 0, 2>(S, lo.x, hi.x, lo.z, hi.z, lo.y, f + 3, r, inv, tmin, bt, best, found);  // XZ at y0 (flipped)
    box6_side<0, 1, 2>(S, lo.y, hi.y, lo.z, hi.z, hi.x, f + 4, r, inv, tmin, bt, best, found);  // YZ at x1
    box6_side<0, 1, 2>(S, lo.y, hi.y, lo.z, hi.z, lo.x, f + 5, r, inv, tmin, bt, best, found);  // YZ at x0 (flipped)
    return found;
}
// ConstantMedium's boundary query over a Box (MB_BOX6): the nearest side hit
// in [lo_t, near] (which side does not matter), near shrinking as sides hit
__device__ __forceinline__ bool box6_nearest(const DevScene& S, uint32_t bi, const Ray& r, const F3& inv, float lo_t,
                                             float& near) {
    const float4 lo = cld4(S.box6 + bi);
    const float4 hi = cld4(reinterpret_cast<const float4*>(S.box6 + bi) + 1);
    bool f = false;
    float t;
    if (rect_t_ax<2, 0, 1>(lo.x, hi.x, lo.y, hi.y, hi.z, r, inv, lo_t, near, t)) near = t, f = true;
    if (rect_t_ax<2, 0, 1>(lo.x, hi.x, lo.y, hi.y, lo.z, r, inv, lo_t, near, t)) near = t, f = true;
    if (rect_t_ax<1, 0, 2>(lo.x, hi.x, lo.z, hi.z, hi.y, r, inv, lo_t, near, t)) near = t, f = true;
    if (rect_t_ax<1, 0, 2>(lo.x, hi.x, lo.z, hi.z, lo.y, r, inv, lo_t, near, t)) near = t, f = true;
    if (rect_t_ax<0, 1, 2>(lo.y, hi.y, lo.z, hi.z, hi.x, r, inv, lo_t, near, t)) near = t, f = true;
    if (rect_t_ax<0, 1, 2>(lo.y, hi.y, lo.z, hi.z, lo.x, r, inv, lo_t, near, t)) near = t, f = true;
    return f;
}

// Words of COLD path state per lane of the general kernels (see lds_bytes):
// 14; 17 with a stack of 16 (MODE 5 / 8 park the sample's RNG key and counter
// there too, PARK_RNG): either way 4 blocks of 256 fit a CU's 160 KB.
constexpr int cold_words(int STACK) { return STACK <= 16 ? 17 : 14; }

// Diagnostic counters (instrumented kernel variant only; see RTOW_PROFILE)
struct Prof {
    uint32_t lane_steps, wave_steps, leaf_tests, lane_iters, wave_iters, pad;
    uint32_t disc_pos, accepted, wave_mixed, wave_sph;  // sphere slots with disc > 0 / taken; waves running both slot paths / any sphere path
    unsigned long long cyc_trav, cyc_other;  // wave cycles (s_memtime) in traversal / everything else
    // general scenes: wave cycles per top-level item (first 8), in finalize, and the item visits
    unsigned long long cyc_item[8], cyc_fin, visits_item[8], cyc_chain;
    uint32_t box_lanes, box_waves;  // Box leaf scans in node steps: lanes / wave executions
};

__device__ __forceinline__ bool first_active_lane() {
    const unsigned long long m = __ballot(1);
    return (threadIdx.x & 63u) == (uint32_t)(__ffsll((long long)m) - 1);
}

// TOP_GRID (MODE 8): the Boxes of a grid of columns (DGrid), walked along the
// ray: rows along v in the ray's v order, within a row the cells along u in
// its u order.  Every cell is widened by G.margin (2^-10 of a cell, hundreds
// of ulps of the scene's coordinates), and every t bound computed here by a
// further 2^-18 relative, so the walk reaches every Box whose six-side scan
// could yield a hit in [tmin, bt]: such a hit lies on the Box's surface up to
// the rectangle tests' rounding, i.e. inside the widened column, at a height
// inside the widened [hlo, hhi], at a t inside the widened bounds.  A cell
// is scanned when the ray, over the cell's t interval, passes at a height the
// cell's Box spans; the scan is box6_scan itself (the tree's leaf test:
// same rectangle tests, same interval shrinking, same tie keys), so the record
// is the tree's -- the set of Boxes tested is a superset of those that can
// win, as for any culled visit order (see "Exact ties in general scenes").
// The walk stops at the first row (cell) that starts beyond the culling bound
// of the record.  The scans are batched: each lane walks to its next cell to
// scan, then the wave scans the cells it found together (the walk steps are
// a few VALU, a scan six rectangle tests).
// The band of the ray's t in which o + t d lies in [lo, hi], widened; a zero
// (or denormal) d, whose 1/d is infinite: every t or none.
__device__ __forceinline__ void grid_band(float lo, float hi, float o, float id, float& t0, float& t1) {
    constexpr float REL = 0x1p-18f;
    const float a = (lo - o) * id, b = (hi - o) * id;
    const float n = fminf(a, b), f = fmaxf(a, b);
    const bool flat = !(fabsf(id) < INFINITY);
    const bool in = lo <= o && o <= hi;
    t0 = flat ? (in ? -INFINITY : INFINITY) : n - fabsf(n) * REL;
    t1 = flat ? (in ? INFINITY : -INFINITY) : f + fabsf(f) * REL;
}
// (the rows' and cells' bands: widened by the caller, see Eu, Ev)
__device__ __forceinline__ void grid_band_w(float lo, float hi, float o, float id, bool flat, float& t0, float& t1) {
    const float a = (lo - o) * id, b = (hi - o) * id;
    const bool in = lo <= o && o <= hi;
    t0 = flat ? (in ? -INFINITY : INFINITY) : fminf(a, b);
    t1 = flat ? (in ? INFINITY : -INFINITY) : fmaxf(a, b);
}
// A cell's (or row's) extent along ah from its packed word in DevScene::gq:
// 16-bit steps of (hhi - hlo) / 65535 from the grid's hlo, rounded outward
// (the host checks the decoded floats contain the true extent), low half the
// lower bound.  GLDS: the words staged in LDS (lq), else global memory.
template <bool GLDS>
__device__ __forceinline__ void grid_ext(const DevScene& S, const uint32_t* lq, uint32_t k, float base, float step,
                                         float& lo, float& hi) {
    uint32_t w;
    if constexpr (GLDS) {
        w = lq[k];
    } else {
        w = S.gq[k];
    }
    lo = fmaf((float)(w & 0xffffu), step, base);
    hi = fmaf((float)(w >> 16), step, base);
}
template <bool PROF = false, bool GLDS = false>
__device__ __forceinline__ bool grid_walk(const DevScene& S, uint32_t gi, const Ray& r, const F3& inv, float tmin,
                                          float& bt, uint32_t& best, const uint32_t* lq, Prof* prof = nullptr) {
    constexpr float REL = 0x1p-18f;
    const DGrid G = cld(S.grid + gi);
    const float qstep = (G.hhi - G.hlo) * (1.0f / 65535.0f);  // (the host quantised with this very float)
    const uint32_t au = G.axes & 3u, av = (G.axes >> 2) & 3u, ah = (G.axes >> 4) & 3u;
    const float ou = comp(r.o, au), ov = comp(r.o, av), oh = comp(r.o, ah);
    const float du = comp(r.d, au), dv = comp(r.d, av), dh = comp(r.d, ah);
    const float iu = comp(inv, au), iv = comp(inv, av), ih = comp(inv, ah);
    const float D = G.margin;
    // the grid's box, widened: the walk's t range [te, tx]
    float u0, u1, v0, v1, h0, h1;
    grid_band(G.u0 - D, G.u1 + D, ou, iu, u0, u1);
    grid_band(G.v0 - D, G.v1 + D, ov, iv, v0, v1);
    grid_band(G.hlo - D, G.hhi + D, oh, ih, h0, h1);
    const float te = fmaxf(fmaxf(u0, v0), fmaxf(h0, tmin));
    const float tx = fminf(fminf(u1, v1), h1);  // finite: d has a non-zero component
    if (!(te <= fminf(tx, cull_bound(bt)))) return false;
    // the rows the ray can meet, one more either side for the widening
    const bool vflat = !(fabsf(iv) < INFINITY), uflat = !(fabsf(iu) < INFINITY);
    const int sv = dv < 0.0f ? -1 : 1, su = du < 0.0f ? -1 : 1;
    const float fnv = (float)(G.nv - 1u), fnu = (float)(G.nu - 1u);
    // (the row of v, moved back / on by twice the widening: the rows whose
    // widened bands hold the ray at te / tx; 1 / wv's rounding is 2^-23 of a
    // cell per cell index, far inside the margin)
    auto row_of = [&](float t, float back) {
        const float v = fmaf(t, dv, ov);
        const float e = 2.0f * D + (fabsf(ov) + fabsf(v)) * REL;
        return fminf(fmaxf(floorf((v + back * e - G.v0) * G.iwv), 0.0f), fnv);
    };
    // the widening of every row and cell band: the margin plus 2^-18 of the
    // magnitudes the walk's coordinates reach within [te, tx] -- more than
    // the rounding of o + t d, and of t = (x - o) (1 / d) carried back to a
    // coordinate (|t d| 2^-22).  The height tests need no margin: a Box spans
    // exactly its cell's [hlo, hhi], so only roundings separate a hit's
    // height from that range -- the face test's point (2 roundings of o + t d)
    // and ha / hb here (one), far below 2^-18 of the magnitudes.  (A margin
    // there would make every ray leaving a column's top scan that column.)
    const float Eu = D + (fabsf(ou) + fabsf(tx * du)) * REL, Ev = D + (fabsf(ov) + fabsf(tx * dv)) * REL;
    const float Eh = (fabsf(oh) + fabsf(tx * dh)) * REL;
    int j = (int)row_of(te, -(float)sv);
    const int jl = (int)row_of(tx, (float)sv);
    int nrows = (jl - j) * sv + 1;
    int i = 0, ncells = 0, jr = 0;
    float ra = 0.0f, rb = 0.0f;
    bool found = false, live = nrows > 0;
    // (Measured, round 5: a lane that holds its candidate walking on to queue
    // a second while the wave's slowest lane still walks raises the walk's
    // lane efficiency from 0.22 to 0.37 but costs registers and scans: -0.3 %
    // to -7 %; DESIGN.md "Grids of Boxes".)
    while (live) {
        uint32_t cand = ~0u;
        while (true) {  // this lane's next cell to scan
            if constexpr (PROF) {  // (instrumented kernel: walk steps, lanes / wave)
                prof->lane_steps++;
                if (first_active_lane()) prof->wave_steps++;
            }
            const float bound = cull_bound(bt);
            if (ncells <= 0) {
                if (nrows <= 0) {
                    live = false;
                    break;
                }
                const float vlo = fmaf((float)j, G.wv, G.v0);
                float t0, t1;
                grid_band_w(vlo - Ev, vlo + G.wv + Ev, ov, iv, vflat, t0, t1);
                jr = j;
                j += sv;
                nrows--;
                if (t0 > bound && !vflat) {  // this row and the later ones lie beyond the record
                    live = false;
                    break;
                }
                ra = fmaxf(t0, te);
                rb = fminf(fminf(t1, tx), bound);
                if (!(ra <= rb)) continue;
                {  // the row's columns span [hlo, hhi] together (row record after the cells)
                    float rlo, rhi;
                    grid_ext<GLDS>(S, lq, G.cell0 + G.nu * G.nv + (uint32_t)jr, G.hlo, qstep, rlo, rhi);
                    const float ha = fmaf(ra, dh, oh), hb = fmaf(rb, dh, oh);
                    if (fmaxf(ha, hb) + Eh < rlo || fminf(ha, hb) - Eh > rhi) continue;
                }
                // the row's cells: u over [ra, rb], widened
                const float ua = fmaf(ra, du, ou), ub = fmaf(rb, du, ou);
                const float fa = floorf((fminf(ua, ub) - Eu - G.u0) * G.iwu);
                const float fb = floorf((fmaxf(ua, ub) + Eu - G.u0) * G.iwu);
                const int ia = (int)fminf(fmaxf(fa, 0.0f), fnu), ib = (int)fminf(fmaxf(fb, 0.0f), fnu);
                i = su > 0 ? ia : ib;
                ncells = ib - ia + 1;
                // (on to the row's first cell in the same step)
            }
            const int ic = i;
            i += su;
            ncells--;
            const float ulo = fmaf((float)ic, G.wu, G.u0);
            float c0, c1;
            grid_band_w(ulo - Eu, ulo + G.wu + Eu, ou, iu, uflat, c0, c1);
            c0 = fmaxf(c0, ra);
            c1 = fminf(fminf(c1, rb), bound);
            if (!(c0 <= c1)) {
                if (c0 > bound && !uflat) ncells = 0;  // the rest of the row lies beyond the record
                continue;
            }
            const uint32_t cell = G.cell0 + (uint32_t)jr * G.nu + (uint32_t)ic;
            float clo, chi;
            grid_ext<GLDS>(S, lq, cell, G.hlo, qstep, clo, chi);
            const float ha = fmaf(c0, dh, oh), hb = fmaf(c1, dh, oh);
            if (fmaxf(ha, hb) + Eh < clo || fminf(ha, hb) - Eh > chi) continue;
            cand = cell;
            break;
        }
        if (cand != ~0u) {
            if constexpr (PROF) {
                prof->box_lanes++;
                if (first_active_lane()) prof->box_waves++;
            }
            if (box6_scan(S, G.box0 + (cand - G.cell0), r, inv, tmin, bt, best)) found = true;
        }
    }
    return found;
}

// General scenes: does leaf `cand`, hit at exactly the t of the current best
// leaf `best`, take the record in the reference?  (assignTieKeys)
__device__ __forceinline__ unsigned long long leaf_key(const DevScene& S, uint32_t ref) {
    const uint32_t k = ref >> KIND_SHIFT, i = ref & LEAF_MASK;
    return k == DK_SPHERE ? S.sph_key[i] : (k == DK_RECT ? S.rect_key[i] : (k == DK_MEDIUM ? S.med_key[i] : 0ull));
}
// An exact tie at the record's t: does leaf `cand` take the record from
// `best`?  The keys decide (the larger wins); the record keeps, in its tie
// bits (TIE_MASK), the first key bit where the two leaves' paths part (+1):
// tie_unsettled() checks after the traversal whether the reference's boxes
// let the winner see that tie at all.
__device__ __forceinline__ bool tie_pick(const DevScene& S, uint32_t cand, uint32_t& best) {
    if ((best >> KIND_SHIFT) == DK_NONE) {
        best = cand;
        return true;
    }
    const unsigned long long kc = leaf_key(S, cand), kb = leaf_key(S, best);
    const bool w = kc > kb;
    const unsigned long long x = kc ^ kb;
    const uint32_t info = x ? (uint32_t)__clzll((long long)x) + 1u : 0u;
    best = ((w ? cand : best) & ~TIE_MASK) | (info << TIE_SHIFT);
    return w;
}
// The record: a strictly nearer hit takes it, an exact tie goes by tie_pick.
// True when `cand` holds the record afterwards.
__device__ __forceinline__ bool take_hit(const DevScene& S, float t, float& bt, uint32_t& best, uint32_t cand) {
    if (t < bt) {
        bt = t;
        best = cand;
        return true;
    }
    return t == bt && tie_pick(S, cand, best);
}

// After a traversal: did the winning rectangle `prim` take or keep an exact
// tie (its tie bits: the first key bit where the two leaves' paths part) that
// the reference never lets it see?  Where the paths part at a HitableList,
// the reference asks the later item with (tmin, t) -- the list's closest hit
// so far (hitableList.h:24-34) -- and every BvhNode between the list and the
// rectangle with that interval; AABB::hit rejects a box the ray enters exactly
// at t (`tmax <= tmin`, aabb.h:22-43).  When a box below the list fails that
// test, which item keeps the tie depends on the order the culled traversal
// does not record: the ray is settled by xhit.  rect_lvl (assignTieKeys): per
// list level on the rectangle's path, its key component's bits and how many
// of the rectangle's reference boxes (rect_anc, its own frame) lie below it.
__device__ __forceinline__ bool tie_unsettled(const DevScene& S, uint32_t prim, const Ray& wray, float tmin, float t) {
    const uint32_t info = (prim & TIE_MASK) >> TIE_SHIFT;
    if (!info) return false;
    const uint32_t p = info - 1u, rect = prim & LEAF_MASK;
    // the common ties (Boxes' coplanar sides in one BVH) part at a BvhNode:
    // rect_lmask marks the key bits of the list levels that have boxes below
    if (!((S.rect_lmask[rect] << p) >> 63)) return false;
    const uint32_t a = S.rect_anc[rect], cnt = a & 255u, off = a >> 8;
    if (cnt == 0) return false;
    for (int k = 0; k < 4; k++) {
        const uint32_t lv = S.rect_lvl[4 * (size_t)rect + k];
        if (!(lv >> 31)) break;
        const uint32_t st = lv & 255u, w = (lv >> 8) & 255u, suf = min((lv >> 16) & 255u, cnt);
        if (p < st || p >= st + w) continue;
        if (suf == 0) return false;
        const Ray rr = chain_ray(S, S.rect[rect].chain, wray);
        for (uint32_t i = cnt - suf; i < cnt; i++)
            if (!ref_aabb_hit(S.abox + 8 * (size_t)(off + i), rr, tmin, t)) return true;
        return false;
    }
    return false;  // the paths part at a BvhNode: both children see the same interval
}

// ---------------------------------------------------------------------------
// The DK_BVH step of a general scene (BvhNode semantics, bvhNode.h:66-96):
// the node's DNode twin (DevScene::gnode: of the SAH tree, or of the
// reference's own with RTOW_TREE_REFERENCE), unit-time sphere children inline
// (tested right here, no box test and no second fetch: the closest hit of a
// set of leaves does not depend on which boxes are tested first), any other
// child a box slot; of the inner children that are hit the nearer is
// returned and the farther pushed; exact ties between leaves by the tie keys.
template <int STACK>
__device__ __forceinline__ uint32_t dnode_step(const DevScene& S, uint32_t idx, const Ray& r, const SlabRay& q, float a,
                                               float ra, float tmin, float& bt, uint32_t& best, uint32_t* stk, int& sp,
                                               uint32_t& overflow, Prof* prof = nullptr) {
    const float4* np = reinterpret_cast<const float4*>(S.node + idx);
    const float4 a0 = np[0], a1 = np[1], b0 = np[2], b1 = np[3];
    const uint32_t refa = __float_as_uint(a1.w), refb = __float_as_uint(b1.w);
    const float btc = cull_bound(bt);
    float ta = 0.0f, tb = 0.0f;
    bool ha = false, hb = false;
    if ((refb >> KIND_SHIFT) == DK_SPHERE) {  // slot b (the right child) first
        const F3 c = add(f3(b0.x, b0.y, b0.z), scl(r.time, f3(b1.x, b1.y, b1.z)));
        float t;
        if (sph_root(c, b0.w, r, a, ra, tmin, t)) take_hit(S, t, bt, best, refb);
    } else {
        hb = slab(b0.x, b0.w, b0.y, b1.x, b0.z, b1.y, q, tmin, btc, tb) && (refb >> KIND_SHIFT) != DK_NONE;
    }
    if ((refa >> KIND_SHIFT) == DK_SPHERE) {
        const F3 c = add(f3(a0.x, a0.y, a0.z), scl(r.time, f3(a1.x, a1.y, a1.z)));
        float t;
        if (sph_root(c, a0.w, r, a, ra, tmin, t)) take_hit(S, t, bt, best, refa);
    } else {
        ha = slab(a0.x, a0.w, a0.y, a1.x, a0.z, a1.y, q, tmin, btc, ta) && (refa >> KIND_SHIFT) != DK_NONE;
    }
    // Box leaves: their sides right here, no visit of their own (one copy of
    // the body for both slots; the order does not matter, ties go by the keys)
    uint32_t l0 = hb && (refb >> KIND_SHIFT) == DK_BOX6 ? refb : 0u;
    uint32_t l1 = ha && (refa >> KIND_SHIFT) == DK_BOX6 ? refa : 0u;
    if (l0) hb = false;
    if (l1) ha = false;
    if (!l0) l0 = l1, l1 = 0u;
    while (l0) {
        if (prof) {
            prof->box_lanes++;
            if (first_active_lane()) prof->box_waves++;
        }
        box6_scan(S, l0 & INDEX_MASK, r, q.inv, tmin, bt, best);
        l0 = l1;
        l1 = 0u;
    }
    if (ha && hb) {
        const bool afirst = ta <= tb;
        if (sp < STACK) {
            stk[sp * BLOCK] = afirst ? refb : refa;
            sp++;
        } else {
            overflow = 1;
        }
        return afirst ? refa : refb;
    }
    if (ha) return refa;
    if (hb) return refb;
    return mkref(DK_NONE, 0);
}

// Closest hit in a world of BvhNodes and spheres only (a "simple" scene,
// every sphere with time0 = 0, time1 = 1), ray already in the BVH's frame.
// The tree is the SAH rebuild (rebuildSah) or the reference's own; either way
// one DNode step tests both child slots: a sphere slot is intersected right
// here (sph_closer: nearer wins, exact ties by the reference's leaf order, so
// the result does not depend on the tree or the visit order), an inner slot
// is slab-tested; the nearer inner hit is visited next, the farther pushed.
// The stack keeps its top entry in a register: a pop hands that entry to the
// next node fetch at once while the LDS read of the new top is in flight.
// Returns the winning sphere ref or DK_NONE.
template <int STACK, int BS, bool PROF, bool FAST>
__device__ __forceinline__ uint32_t trace_simple(const DevScene& S, const DNode* nodes, uint32_t root, const Ray& r, float tmin,
                                 float& bt, uint32_t* stk, uint32_t& overflow, Prof& prof) {
    // the boxes sit in the world frame (DevScene::tshift, see SlabRay): the
    // ray's origin there, from its origin in the BVH's frame
    const SlabRayF q = slab_ray_f(add(r.o, f3(S.tshift[0], S.tshift[1], S.tshift[2])), r.d);
    const float a = dot(r.d, r.d);
    const float ra = 1.0f / a;
    const float time = r.time;
    uint32_t best = mkref(DK_NONE, 0);
    if ((root >> KIND_SHIFT) == DK_SPHERE) {
        float t;
        if (sph_t<true>(load_sph(S.sph + (root & INDEX_MASK)), r, a, ra, tmin, bt, t)) {
            bt = t;
            best = root;
        }
        return best;
    }
    uint32_t cur = root;
    uint32_t top = mkref(DK_NONE, 0);
    // entry 0 of the LDS stack holds NONE, a sentinel no push overwrites
    // (entries live at 1 .. sp - 1): a pop reads entry sp - 1 and keeps sp >= 1,
    // no branch -- from the empty stack it reads the sentinel.  The capacity
    // of STACK - 1 entries still covers the host's stack_need - 1 (the register
    // top holds one more).
    stk[0] = mkref(DK_NONE, 0);
    int sp = 1;
    // the culling bound follows bt (recomputed only when a sphere takes the
    // record), widened by werr besides: the one-FMA planes can put a box's
    // entry late by as much as its exit early (SlabRayF)
    float btc = cull_bound(bt) + q.werr;
    // the record as one 64-bit key, (t bits, ~leaf): t > tmin > 0 and bt are
    // positive, so their bits order as the floats do, and ~ reverses the leaf
    // order -- key < record  <=>  t < bt || (t == bt && leaf > best), the
    // reference's tie rule (sph_closer), in one 64-bit compare
    unsigned long long rkey = (unsigned long long)__float_as_uint(bt) << 32 | (uint32_t)~best;
    while (true) {
        if constexpr (PROF) {
            prof.lane_steps++;
            if (first_active_lane()) prof.wave_steps++;
        }
        const float4* np = reinterpret_cast<const float4*>(nodes + (cur & INDEX_MASK));
        const float4 a0 = np[0], a1 = np[1], b0 = np[2], b1 = np[3];
        const uint32_t refa = __float_as_uint(a1.w), refb = __float_as_uint(b1.w);
        if constexpr (PROF) {
            const bool sa = (refa >> KIND_SHIFT) == DK_SPHERE, sb = (refb >> KIND_SHIFT) == DK_SPHERE;
            const unsigned long long act = __ballot(1), ma = __ballot(sa), mb = __ballot(sb);
            if (first_active_lane()) {
                prof.wave_mixed += (ma != 0 && ma != act) + (mb != 0 && mb != act);
                prof.wave_sph += (ma != 0) + (mb != 0);
            }
            for (int k = 0; k < 2; k++) {
                const bool sk = k ? sb : sa;
                if (!sk) continue;
                const float4 p0 = k ? b0 : a0, p1 = k ? b1 : a1;
                const F3 c = add(f3(p0.x, p0.y, p0.z), scl(time, f3(p1.x, p1.y, p1.z)));
                const F3 oc = sub(r.o, c);
                const float bq = dot(r.d, oc), cq = dot(oc, oc) - p0.w;
                prof.leaf_tests++;
                if (bq * bq - a * cq > 0) prof.disc_pos++;
            }
        }
        float tb = 0.0f, ta = 0.0f;
        bool hb = false, ha = false;
        // slot b (the right child) first
        if ((refb >> KIND_SHIFT) == DK_SPHERE) {
            // Sphere::hit / MovingSphere::hit with center = c0 + time * (c1 - c0)
            const F3 c = add(f3(b0.x, b0.y, b0.z), scl(time, f3(b1.x, b1.y, b1.z)));
            float t;
            if (sph_root<FAST>(c, b0.w, r, a, ra, tmin, t)) {
                const unsigned long long k = (unsigned long long)__float_as_uint(t) << 32 | (uint32_t)~refb;
                if (k < rkey) {
                    rkey = k;
                    btc = cull_bound(t) + q.werr;
                    if constexpr (PROF) prof.accepted++;
                }
            }
        } else {
            hb = slab_f(b0.x, b0.w, b0.y, b1.x, b0.z, b1.y, q, tmin, btc, tb);  // (a simple scene's slot: sphere or DK_BVH)
        }
        if ((refa >> KIND_SHIFT) == DK_SPHERE) {
            const F3 c = add(f3(a0.x, a0.y, a0.z), scl(time, f3(a1.x, a1.y, a1.z)));
            float t;
            if (sph_root<FAST>(c, a0.w, r, a, ra, tmin, t)) {
                const unsigned long long k = (unsigned long long)__float_as_uint(t) << 32 | (uint32_t)~refa;
                if (k < rkey) {
                    rkey = k;
                    btc = cull_bound(t) + q.werr;
                    if constexpr (PROF) prof.accepted++;
                }
            }
        } else {
            ha = slab_f(a0.x, a0.w, a0.y, a1.x, a0.z, a1.y, q, tmin, btc, ta);
        }
        // one back-edge, one exit: push / descend / pop are predicated updates
        const uint32_t NONE = mkref(DK_NONE, 0);
        const bool afirst = ta <= tb;
        const bool both = ha && hb;
        uint32_t nxt = both ? (afirst ? refa : refb) : (ha ? refa : (hb ? refb : NONE));
        if (both) {  // push the farther child; the old top goes to LDS
            // (no bound check: the host's stack_need, the deepest chain of
            // nodes with two inner children, is at most STACK, and the
            // register top holds one of those entries: checkSimpleNodes)
            if (top != NONE) {
                stk[sp * BS] = top;
                sp++;
            }
            top = afirst ? refb : refa;
        }
        if (nxt == NONE) {  // pop
            nxt = top;
            top = stk[(sp - 1) * BS];
            sp = max(sp - 1, 1);
        }
        if (nxt == NONE) break;
        cur = nxt;
    }
    bt = __uint_as_float((uint32_t)(rkey >> 32));
    return ~(uint32_t)rkey;
}

// A BvhNode of unit-time spheres inside a general scene (TOP_SPHERES: a
// top-level item that is a chain of instances over one), traversed in a loop
// of its own: dnode_step's node step on the DNode twins (spheres inline, the
// exact (x - o) * (1/d) slab planes of the general kernels), trace_simple's
// register stack top, no kind dispatch.  `r` is the ray in the spheres' frame,
// inv its reciprocals, a = dot(d, d), ra = 1 / a; bt / best the record so far
// (the list's closest hit), updated with the reference's tie rule (tie keys).
// LEAVES (TOP_DTREE: a BvhNode tree without instances, lists or media below
// it, final_ned's first tree of ground Boxes, light and spheres): a slot may
// also hold a Box (DK_BOX6), a rectangle or a sphere that is not inlined
// (DK_MSPHERE); its box hit, it is tested right there -- the same tests and
// tie keys as the general traversal's visit of that leaf (traverse), without
// the visit.
template <int STACK, bool LEAVES = false>
__device__ __forceinline__ bool trace_dnodes(const DevScene& S, uint32_t root, const Ray& r, const F3& inv, float a,
                                             float ra, float tmin, float& bt, uint32_t& best, uint32_t* stk,
                                             uint32_t& overflow) {
    const uint32_t NONE = mkref(DK_NONE, 0);
    const SlabRay q = slab_ray_inv(r.o, inv);
    bool found = false;
    uint32_t cur = mkref(DK_BVH, root), top = NONE;
    int sp = 0;
    float btc = cull_bound(bt);
    while (true) {
        const float4* np = reinterpret_cast<const float4*>(S.node + (cur & INDEX_MASK));
        const float4 a0 = np[0], a1 = np[1], b0 = np[2], b1 = np[3];
        const uint32_t refa = __float_as_uint(a1.w), refb = __float_as_uint(b1.w);
        float tb = 0.0f, ta = 0.0f;
        bool hb = false, ha = false;
        if ((refb >> KIND_SHIFT) == DK_SPHERE) {  // slot b (the right child) first
            const F3 c = add(f3(b0.x, b0.y, b0.z), scl(r.time, f3(b1.x, b1.y, b1.z)));
            float t;
            if (sph_root(c, b0.w, r, a, ra, tmin, t) && take_hit(S, t, bt, best, refb)) {
                btc = cull_bound(bt);
                found = true;
            }
        } else {
            // (a TOP_SPHERES tree's slots are spheres or inner nodes only:
            // sphereInstance; and the general stack_need counts every one of
            // its BvhNodes, so the push needs no bound check)
            hb = slab(b0.x, b0.w, b0.y, b1.x, b0.z, b1.y, q, tmin, btc, tb);
        }
        if ((refa >> KIND_SHIFT) == DK_SPHERE) {
            const F3 c = add(f3(a0.x, a0.y, a0.z), scl(r.time, f3(a1.x, a1.y, a1.z)));
            float t;
            if (sph_root(c, a0.w, r, a, ra, tmin, t) && take_hit(S, t, bt, best, refa)) {
                btc = cull_bound(bt);
                found = true;
            }
        } else {
            ha = slab(a0.x, a0.w, a0.y, a1.x, a0.z, a1.y, q, tmin, btc, ta);
        }
        if constexpr (LEAVES) {
            uint32_t l0 = hb && (refb >> KIND_SHIFT) != DK_BVH ? refb : 0u;
            uint32_t l1 = ha && (refa >> KIND_SHIFT) != DK_BVH ? refa : 0u;
            if (l0) hb = false;
            if (l1) ha = false;
            if (!l0) l0 = l1, l1 = 0u;
            if (l0) {
                do {  // one copy of the leaf tests for both slots
                    const uint32_t lk = l0 >> KIND_SHIFT, li = l0 & INDEX_MASK;
                    float t;
                    if (lk == DK_BOX6) {
                        if (box6_scan(S, li, r, q.inv, tmin, bt, best)) found = true;
                    } else if (lk == DK_RECT) {
                        if (rect_t(S.rect[li], r, q.inv, tmin, bt, t) && take_hit(S, t, bt, best, l0)) found = true;
                    } else {  // DK_MSPHERE
                        const Sph s = load_sph(S.sph + li);
                        const F3 c = S.unit_time ? sph_center<true>(s, r.time) : sph_center<false>(s, r.time);
                        if (sph_root(c, s.r * s.r, r, a, ra, tmin, t) && take_hit(S, t, bt, best, mkref(DK_SPHERE, li)))
                            found = true;
                    }
                    l0 = l1;
                    l1 = 0u;
                } while (l0);
                btc = cull_bound(bt);
            }
        }
        const bool afirst = ta <= tb;
        const bool both = ha && hb;
        uint32_t nxt = both ? (afirst ? refa : refb) : (ha ? refa : (hb ? refb : NONE));
        if (both) {
            if (top != NONE) {
                stk[sp * BLOCK] = top;
                sp++;
            }
            top = afirst ? refb : refa;
        }
        if (nxt == NONE) {
            nxt = top;
            top = NONE;
            if (sp > 0) {
                --sp;
                top = stk[sp * BLOCK];
            }
        }
        if (nxt == NONE) break;
        cur = nxt;
    }
    return found;
}

struct Best {
    float t;
    uint32_t prim;  // the leaf; its instance chain is the leaf's own (DSphere::chain ...)
};

// ConstantMedium's two boundary queries (constantMedium.h:28-29) when the
// boundary is a plain sphere: hit(-FLT_MAX, FLT_MAX) takes the near root,
// hit(t1 + 0.0001, FLT_MAX) then rejects the near root again and takes the
// far one -- the same roots Sphere::hit (sphere.h:20-69) computes each call.
template <bool UNIT_TIME>
__device__ __forceinline__ bool sphere_boundary(const Sph& s, const Ray& r, float a, float ra, float& t1, float& t2) {
    const F3 oc = sub(r.o, sph_center<UNIT_TIME>(s, r.time));
    const float b = dot(r.d, oc);
    const float c = dot(oc, oc) - s.r * s.r;
    const float disc = b * b - a * c;
    if (!(disc > 0)) return false;
    const float sq = sqrt_pos<false>(disc);
    const float tn = div_by(-b - sq, a, ra), tf = div_by(-b + sq, a, ra);  // the IEEE quotients (sph_root's)
    const float lo = -FLT_MAX;
    float first;
    if (tn < FLT_MAX && tn > lo) first = tn;
    else if (tf < FLT_MAX && tf > lo) first = tf;
    else return false;
    const float lo2 = (float)((double)first + 0.0001);
    if (tn < FLT_MAX && tn > lo2) t2 = tn;
    else if (tf < FLT_MAX && tf > lo2) t2 = tf;
    else return false;
    t1 = first;
    return true;
}

// ConstantMedium::hit (constantMedium.h:26-74) of medium `idx` for the ray
// `r` in the medium's frame (a = dot(d, d)), called with the list's current
// closest hit as tmax (hitableList.h:30): true and bt = the scatter distance
// when the ray scatters inside.  Draws 1 or 2 numbers, as the reference.
// ANYB: media whose boundary needs the general traversal may occur (MB_ANY);
// without them the kernel carries no nested traversal (fewer registers).
template <bool MEDIA, int STACK, bool ANYB = true>
__device__ __forceinline__ bool traverse(const DevScene& S, uint32_t root, const Ray& wray, uint32_t chain0, float tmin,
                                         float tmax, uint32_t* stk, int sp0, Rng& rng, Best& best, uint32_t& overflow,
                                         uint32_t prev, Prof* prof = nullptr);

template <int STACK, bool ANYB>
__device__ __forceinline__ bool medium_hit(const DevScene& S, uint32_t idx, const Ray& r, float a, float ra,
                                           const Ray& wray, float tmin, float& bt, uint32_t* stk, int sp, Rng& rng,
                                           uint32_t& overflow) {
    const DMedium M = cld(S.med + idx);
    (void)rng.next();  // the discarded `db` draw (constantMedium.h:27)
    float t1 = 0, t2 = 0;
    bool two = false;
    if (M.bkind == MB_SPHERE) {
        const Sph s = load_sph(S.sph + (M.boundary & INDEX_MASK));
        two = S.unit_time ? sphere_boundary<true>(s, r, a, ra, t1, t2) : sphere_boundary<false>(s, r, a, ra, t1, t2);
    } else if (M.bkind == MB_BOX6) {
        // the same two queries over a Box's sides (box6_nearest)
        const Ray rb = chain_ray(S, M.bchain, wray);
        const F3 inv = inv_dir(rb.d);
        float near = FLT_MAX;
        if (box6_nearest(S, M.bfirst, rb, inv, -FLT_MAX, near)) {
            t1 = near;
            near = FLT_MAX;
            if (box6_nearest(S, M.bfirst, rb, inv, (float)((double)t1 + 0.0001), near)) {
                t2 = near;
                two = true;
            }
        }
    } else if (M.bkind == MB_RECTS) {
        // boundary->hit(-FLT_MAX, FLT_MAX) then boundary->hit(t1 + 0.0001,
        // FLT_MAX) over instances of a Box: the nearest rectangle hit in each
        // interval (hitableList.h:20-38 keeps the nearest; which rectangle
        // does not matter here), in the rectangles' frame (chain bchain: the
        // same transforms the traversal applies on the way down)
        const Ray rb = chain_ray(S, M.bchain, wray);
        const F3 inv = inv_dir(rb.d);
        float lo = -FLT_MAX;
        for (int pass = 0; pass < 2; pass++) {
            float near = FLT_MAX, t;
            bool f = false;
            for (uint32_t k = 0; k < M.bcount; k++) {
                if (rect_t(cld(S.rect + M.bfirst + k), rb, inv, lo, near, t)) {
                    near = t;
                    f = true;
                }
            }
            if (!f) break;
            if (pass == 0) {
                t1 = near;
                lo = (float)((double)near + 0.0001);
            } else {
                t2 = near;
                two = true;
            }
        }
    } else if constexpr (ANYB) {
        Best b1, b2;
        two = traverse<false, STACK>(S, M.boundary, wray, M.chain, -FLT_MAX, FLT_MAX, stk, sp, rng, b1, overflow,
                                     mkref(DK_NONE, 0)) &&
              traverse<false, STACK>(S, M.boundary, wray, M.chain, (float)((double)b1.t + 0.0001), FLT_MAX, stk, sp,
                                     rng, b2, overflow, mkref(DK_NONE, 0));
        t1 = b1.t;
        t2 = b2.t;
    }
    if (two) {
        float ta = t1, tb = t2;
        if (ta < tmin) ta = tmin;
        if (tb > bt) tb = bt;
        if (!(ta >= tb)) {
            if (ta < 0) ta = 0;
            const float dl = len(r.d);
            const float inside = (tb - ta) * dl;
            const float dist = (float)(-M.inv_density * log(rng.next()));
            if (dist < inside) {
                bt = ta + dist / dl;
                return true;
            }
        }
    }
    return false;
}

// Closest hit of `root` for a world-space ray, reference semantics, any scene
// graph: lists in order with a shrinking tmax (hitableList.h:20-38),
// instances, rectangles, media; exact ties settled by the tie keys.
// `r` is the ray in the frame of chain `chain0` (the frame `root` sits in).
// stk: this lane's LDS stack column.
// `prev`: the leaf that holds tmax from before the call (DK_NONE: none), for
// exact ties at tmax.
template <bool MEDIA, int STACK, bool ANYB>
__device__ __forceinline__ bool traverse(const DevScene& S, uint32_t root, const Ray& wray, uint32_t chain0, float tmin,
                                         float tmax, uint32_t* stk, int sp0, Rng& rng, Best& best, uint32_t& overflow,
                                         uint32_t prev, Prof* prof) {
    Ray r = chain_ray(S, chain0, wray);
    SlabRay q = slab_ray(r);
    float a = dot(r.d, r.d);
    float ra = 1.0f / a;
    float bt = tmax;
    float tmed = __builtin_nanf("");  // a DProg medium's interval end (NaN: none pending)
    bool found = false;
    best.prim = prev;
    uint32_t cur = root;
    int sp = sp0;
    while (true) {
        uint32_t kind = cur >> KIND_SHIFT;
        if (prof) {  // instrumented kernel only (a null pointer otherwise: folded away)
            prof->lane_steps++;
            if (first_active_lane()) prof->wave_steps++;
            if (kind == DK_BVH) prof->leaf_tests++;
        }
        const uint32_t idx = cur & INDEX_MASK;
        if (kind == DK_BVH) {
            const uint32_t before = best.prim;
            uint32_t b = before;
            const uint32_t nxt = dnode_step<STACK>(S, idx, r, q, a, ra, tmin, bt, b, stk, sp, overflow, prof);
            if (b != before) {
                best.prim = b;
                found = true;
            }
            if ((nxt >> KIND_SHIFT) != DK_NONE) {
                cur = nxt;
                continue;
            }
        } else if (kind == DK_SPHERE || kind == DK_MSPHERE) {
            float t;
            const Sph s = load_sph(S.sph + idx);
            const F3 c = S.unit_time ? sph_center<true>(s, r.time) : sph_center<false>(s, r.time);
            if (sph_root(c, s.r * s.r, r, a, ra, tmin, t) && take_hit(S, t, bt, best.prim, mkref(DK_SPHERE, idx)))
                found = true;
        } else if (kind == DK_RECT) {
            float t;
            if (rect_t(S.rect[idx], r, q.inv, tmin, bt, t) && take_hit(S, t, bt, best.prim, cur)) found = true;
        } else if (kind == DK_RECTS) {
            // a list of rectangles: scanned in order, closed interval, as hitableList.h
            const DList R = S.list[idx];
            if (R.box6) {  // a Box's sides: the unrolled scan
                if (box6_scan(S, R.box6 - 1, r, q.inv, tmin, bt, best.prim)) found = true;
            } else
            for (uint32_t j = 0; j < R.count; j++) {
                float t;
                if (rect_t(S.rect[R.first + j], r, q.inv, tmin, bt, t) &&
                    take_hit(S, t, bt, best.prim, mkref(DK_RECT, R.first + j)))
                    found = true;
            }
        } else if (kind == DK_LIST || kind == DK_LISTNEXT) {
            // items in order; one continuation entry below the item being
            // visited instead of the whole rest of the list
            const uint32_t at = kind == DK_LIST ? S.list[idx].first : idx;
            const uint32_t item = S.refs[at];
            if ((item >> KIND_SHIFT) != DK_NONE) {
                if ((S.refs[at + 1] >> KIND_SHIFT) != DK_NONE) {
                    if (sp < STACK) {
                        stk[sp * BLOCK] = mkref(DK_LISTNEXT, at + 1);
                        sp++;
                    } else {
                        overflow = 1;
                    }
                }
                cur = item;
                continue;
            }
        } else if (kind == DK_TRANSLATE || kind == DK_ROTY || kind == DK_FLIP) {
            // enter: the EXIT marker remembers the chain to restore.  An
            // instance's only child may be another instance (Translate(RotateY
            // (...))): the whole run of them is entered at once -- the same
            // transforms in the same order -- with one EXIT and the per-ray
            // constants of the innermost frame only
            const DInst& I = S.inst[idx];
            if (sp < STACK) {
                stk[sp * BLOCK] = mkref(DK_EXIT, I.parent_chain);
                sp++;
                r = apply_inst(S, cur, r);
                cur = I.child;
                for (int guard = 0; guard < MAXCHAIN; guard++) {
                    const uint32_t ck = cur >> KIND_SHIFT;
                    if (ck != DK_TRANSLATE && ck != DK_ROTY && ck != DK_FLIP) break;
                    r = apply_inst(S, cur, r);
                    cur = S.inst[cur & INDEX_MASK].child;
                }
                q = slab_ray(r);
                a = dot(r.d, r.d);
                ra = 1.0f / a;
                continue;
            }
            overflow = 1;
        } else if (kind == DK_EXIT) {
            r = chain_ray(S, idx, wray);
            q = slab_ray(r);
            a = dot(r.d, r.d);
            ra = 1.0f / a;
        } else if (kind == DK_PROG || kind == DK_PROGNEXT) {
            if constexpr (MEDIA) {
                // a BvhNode subtree holding media, replayed in the reference's
                // visit order (DProg); tin: the end of the interval the
                // subtree was handed, which every box and medium in it sees
                uint32_t pos = idx;
                float tin = bt;
                if (kind == DK_PROGNEXT) {  // back from an item: its interval sits below the marker
                    --sp;
                    tin = __uint_as_float(stk[sp * BLOCK]);
                }
                bool descend = false;
                while (true) {
                    const DProg* E = S.prog + pos;
                    const uint4 w = reinterpret_cast<const uint4*>(E)[1];
                    const uint32_t op = __float_as_uint(reinterpret_cast<const float4*>(E)[0].w);
                    if (op == PROG_END) break;
                    if (op == PROG_BOX) {
                        pos += ref_aabb_hit_inv(reinterpret_cast<const float*>(E), r, q.inv, tmin, tin) ? 1u : 1u + w.w;
                        continue;
                    }
                    // an item: a medium (asked with the subtree's interval,
                    // below) or a child without media (the general traversal:
                    // nearest hit and exact ties merge as anywhere else);
                    // then on with the program
                    pos++;
                    if (sp + 2 <= STACK) {
                        stk[sp * BLOCK] = __float_as_uint(tin);
                        stk[(sp + 1) * BLOCK] = mkref(DK_PROGNEXT, pos);
                        sp += 2;
                        cur = w.w;
                        if ((cur >> KIND_SHIFT) == DK_MEDIUM) tmed = tin;
                        descend = true;
                    } else {
                        overflow = 1;
                    }
                    break;
                }
                if (descend) continue;
            }
        } else if (kind == DK_MEDIUM) {
            if constexpr (MEDIA) {
                // asked with the closest hit so far, or (tmed, set by a DProg
                // program) its subtree's interval; the nearest record is kept
                float tm = tmed == tmed ? tmed : bt;
                if (!(tmed == tmed) && (best.prim >> KIND_SHIFT) == DK_RECT &&
                    ref_skips_hit(S, best.prim & LEAF_MASK, wray, bt, tmin))
                    overflow |= 2u;  // see traverse_top's TOP_MEDIUM
                tmed = __builtin_nanf("");
                if (medium_hit<STACK, ANYB>(S, idx, r, a, ra, wray, tmin, tm, stk, sp, rng, overflow) &&
                    take_hit(S, tm, bt, best.prim, cur))
                    found = true;
            }
        }
        if (sp == sp0) break;
        --sp;
        cur = stk[sp * BLOCK];
    }
    best.t = bt;
    return found || best.prim != prev;  // (an exact tie settled for `prev` marks its tie bits)
}

// The closest hit of a general scene whose root (below its instances) is a
// list, scanned as hitableList.h:20-38 does: items in order, tmax the closest
// hit so far.  The loop is uniform across the wave (see DTop).
// MEDIA / ANYB: media below the top level (the general traversal asks them);
// TOPMED: media as top-level items (TOP_MEDIUM).
// PARK: the caller parked the sample's RNG key (COLD words 14, 15) and its
// counter (16) in LDS; media draw through them (registers, see cold_words).
// GRID: TOP_GRID items may occur (MODE 8).
template <bool MEDIA, int STACK, bool ANYB, bool TOPMED, bool PROF = false, bool PARK = false, bool GRID = false>
__device__ __forceinline__ bool traverse_top(const DevScene& S, const Ray& wray, float tmin, uint32_t* stk, Rng& rng, Best& best,
                             uint32_t& overflow, Prof* prof = nullptr) {
    float bt = FLT_MAX;
    uint32_t bp = mkref(DK_NONE, 0);
    // COLD slot 13 (the lane's LDS column past its stack): mrect, below
    uint32_t* const mslot = stk + (size_t)(STACK + 13) * BLOCK;
    if constexpr (TOPMED) *mslot = mkref(DK_NONE, 0);
    // the ray in the item's frame and its per-direction constants, recomputed
    // only where the host marked the item (TOP_NEWCHAIN / TOP_NEWDIR)
    F3 inv = f3(0, 0, 0);
    float a = 0, ra = 0;
    Ray r = wray;
    const uint32_t n = S.n_top ? S.n_top : 1u;  // no top-level list: the whole graph is one item
    unsigned long long t0 = PROF ? __builtin_amdgcn_s_memtime() : 0;
    for (uint32_t j = 0; j < n; j++) {
        if constexpr (PROF) {  // the previous item's wave cycles
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            if (j > 0 && j <= 8) prof->cyc_item[j - 1] += t1 - t0;
            if (j < 8 && first_active_lane()) prof->visits_item[j]++;
            t0 = t1;
        }
        const DTop T = S.n_top ? cld(S.top + j) : DTop{TOP_GENERIC, S.root, 0, 0};
        const uint32_t kind = T.kind & TOP_KIND_MASK;
        if (kind == TOP_GENERIC) {  // (media too: traverse() keeps their draws in order)
            // the scan's ray is dead across the general traversal (the host
            // marks the next in-place item to recompute it): registers
            r = wray;
            inv = f3(0, 0, 0);
            a = ra = 0.0f;
            Best b;
            if (traverse<MEDIA, STACK, ANYB>(S, T.a, wray, T.chain, tmin, bt, stk, 0, rng, b, overflow, bp,
                                             PROF ? prof : nullptr)) {
                bt = b.t;
                bp = b.prim;
            }
            continue;
        }
        unsigned long long tc = PROF ? __builtin_amdgcn_s_memtime() : 0;
        // consecutive items in one frame (a room's walls) share the ray, and
        // frames that differ by translations only its direction constants
        if (T.kind & TOP_NEWCHAIN) {
            r = chain_ray(S, T.chain, wray);
            if (T.kind & TOP_NEWDIR) {
                inv = inv_dir(r.d);
                a = dot(r.d, r.d);
                ra = 1.0f / a;
            }
        }
        if constexpr (PROF) {
            __builtin_amdgcn_s_waitcnt(0);
            prof->cyc_chain += __builtin_amdgcn_s_memtime() - tc;
        }
        if (kind == TOP_BOX6) {
            box6_scan(S, T.a, r, inv, tmin, bt, bp);
        } else if (kind == TOP_RECTS) {
            for (uint32_t k = 0; k < T.b; k++) {
                // the rectangle is the same for the whole wave (a scalar load):
                // its axes pick rect_t_ax's compile-time variant by a uniform
                // branch instead of rect_t's per-component selects
                const DRect q = cld(S.rect + T.a + k);
                const uint32_t ax = q.axis & 3u;
                float t;
                bool h;
                if (ax == 0)
                    h = rect_t_ax<2, 0, 1>(q.a0, q.a1, q.b0, q.b1, q.k, r, inv, tmin, bt, t);
                else if (ax == 1)
                    h = rect_t_ax<1, 0, 2>(q.a0, q.a1, q.b0, q.b1, q.k, r, inv, tmin, bt, t);
                else
                    h = rect_t_ax<0, 1, 2>(q.a0, q.a1, q.b0, q.b1, q.k, r, inv, tmin, bt, t);
                if (h) take_hit(S, t, bt, bp, mkref(DK_RECT, T.a + k));
            }
        } else if (TOPMED && kind == TOP_MEDIUM) {
            // ConstantMedium::hit (constantMedium.h:26-74) with the closest hit
            // so far as tmax, in the medium's frame; it draws as the reference.
            // A record the reference never reached (a rectangle grazed at its
            // box's edge, ref_skips_hit) would cut the medium's interval and
            // maybe its draws: the ray is then settled by xhit (overflow bit 1)
            // (checked after the scan, once: mrect, the rectangle holding the
            // record when a medium was asked; a second one forces the re-trace)
            if ((bp >> KIND_SHIFT) == DK_RECT) {
                const uint32_t mrect = *mslot;
                if ((mrect >> KIND_SHIFT) == DK_RECT && ((mrect ^ bp) & ~TIE_MASK)) overflow |= 2u;
                *mslot = bp;
            }
            if constexpr (PARK) {
                uint32_t* const cw = stk + (size_t)STACK * BLOCK;
                Rng m{(uint64_t)cw[15 * BLOCK] << 32 | cw[14 * BLOCK], cw[16 * BLOCK]};
                if (medium_hit<STACK, false>(S, T.a, r, a, ra, wray, tmin, bt, stk, 0, m, overflow))
                    bp = mkref(DK_MEDIUM, T.a);
                cw[16 * BLOCK] = m.ctr;
            } else {
                if (medium_hit<STACK, false>(S, T.a, r, a, ra, wray, tmin, bt, stk, 0, rng, overflow))
                    bp = mkref(DK_MEDIUM, T.a);
            }
        } else if (kind == TOP_SPHERES) {
            trace_dnodes<STACK>(S, T.a, r, inv, a, ra, tmin, bt, bp, stk, overflow);
        } else if (kind == TOP_DTREE) {
            trace_dnodes<STACK, true>(S, T.a, r, inv, a, ra, tmin, bt, bp, stk, overflow);
        } else if (GRID && kind == TOP_GRID) {
            // (the packed heights staged after the COLD words: STACK 16 only)
            constexpr bool GLDS = STACK <= 16;
            grid_walk<PROF, GLDS>(S, T.a, r, inv, tmin, bt, bp,
                                  stk - threadIdx.x + (size_t)(STACK + cold_words(STACK)) * BLOCK, prof);
        } else if (kind == TOP_SPHERE) {
            if constexpr (GRID) {  // grid worlds: a run of spheres in this frame (copies: chain = own index)
                for (uint32_t k = 0; k < T.b; k++) {
                    const DSphere* q = S.tsph + T.a + k;
                    const Sph sp = load_sph(q);
                    const uint32_t si = cld(&q->chain);
                    const F3 c = S.unit_time ? sph_center<true>(sp, r.time) : sph_center<false>(sp, r.time);
                    float t;
                    if (sph_root(c, sp.r * sp.r, r, a, ra, tmin, t)) take_hit(S, t, bt, bp, mkref(DK_SPHERE, si));
                }
            } else {
                const Sph sp = load_sph(S.sph + T.a);
                const F3 c = S.unit_time ? sph_center<true>(sp, r.time) : sph_center<false>(sp, r.time);
                float t;
                if (sph_root(c, sp.r * sp.r, r, a, ra, tmin, t)) take_hit(S, t, bt, bp, mkref(DK_SPHERE, T.a));
            }
        }
    }
    if constexpr (PROF) {
        if (n <= 8) prof->cyc_item[n - 1] += __builtin_amdgcn_s_memtime() - t0;
    }
    // a rectangle that cut a medium's interval and lost the record later (the
    // winner itself is checked by the caller)
    if constexpr (TOPMED) {
        const uint32_t mrect = *mslot;
        if ((mrect >> KIND_SHIFT) == DK_RECT && ((mrect ^ bp) & ~TIE_MASK) &&
            ref_skips_rect(S, mrect & LEAF_MASK, wray, tmin))
            overflow |= 2u;
    }
    best.t = bt;
    best.prim = bp;
    return (bp >> KIND_SHIFT) != DK_NONE;  // a record was taken
}

// x / d in double from r = RN(1/d): q0 = x*r, one fma residual step.  For the
// two divisions below it equals the IEEE quotient for every float phi in
// [-pi, pi] and theta in [-pi/2, pi/2] (all 4.3e9 checked on the host;
// tests/test_numerics.py samples them), at 3 f64 ops instead of ~10.
__device__ __forceinline__ double div_by_f64(double x, double d, double r) {
    const double q0 = x * r;
    return fma(fma(-q0, d, x), r, q0);
}

// mathUtilities.h:62-68
__device__ __forceinline__ void sphere_uv(F3 p, float& u, float& v) {
    const float phi = atan2f(p.z, p.x);
    const float theta = asinf(p.y);
    u = (float)(1 - div_by_f64(phi + M_PI, 2 * M_PI, 1.0 / (2 * M_PI)));
    v = (float)div_by_f64(theta + M_PI / 2, M_PI, 1.0 / M_PI);
}

// The HitRecord of the winning leaf: the ray into the leaf's frame (its
// instance chain), the leaf's record, then the instances' way out.
// SIMPLE: every leaf sits under the root chain (kernel-argument registers).
template <bool SIMPLE>
__device__ __forceinline__ void finalize(const DevScene& S, uint32_t prim, float t, const Ray& wray, Rec& rec) {
    const uint32_t kind = prim >> KIND_SHIFT;
    const uint32_t idx = prim & INDEX_MASK;
    if constexpr (!SIMPLE) {
        // General scenes, in two memory round trips: the leaf's whole record
        // (its chain id, material and the host's "needs uv" bit ride along:
        // RECT_UV / SPH_UV), then the chain's count and first two entries,
        // which serve the way in and the way out (chain_ray / chain_out).
        float4 q0, q1, q2 = make_float4(0, 0, 0, 0);
        if (kind == DK_SPHERE) {
            const float4* g = reinterpret_cast<const float4*>(S.sph + idx);
            q0 = g[0], q1 = g[1], q2 = g[2];  // c0 r | dc t0 | t1 mat moving chain
        } else if (kind == DK_RECT) {
            const float4* g = reinterpret_cast<const float4*>(S.rect + idx);
            q0 = g[0], q1 = g[1];  // a0 a1 b0 b1 | k axis mat chain
        } else {
            const float4* g = reinterpret_cast<const float4*>(S.med + idx);
            q0 = g[0], q1 = g[1];  // boundary phase_mat inv_density chain | ...
        }
        const uint32_t chain = __float_as_uint(kind == DK_SPHERE ? q2.w : (kind == DK_RECT ? q1.w : q0.w));
        const DChainX* C = S.chains + chain;
        const int n = (int)C->n;
        const float4 e0 = C->t[0], e1 = C->t[1];
        Ray r = wray;
        if (n > 0) chain_step(e0, r);
        if (n > 1) chain_step(e1, r);
        for (int k = 2; k < n; k++) chain_step(C->t[k], r);
        rec.t = t;
        rec.u = 0.0f;
        rec.v = 0.0f;
        rec.p = at(r, t);
        if (kind == DK_SPHERE) {
            // sph_center's arithmetic ((time - 0) / (1 - 0) is time exactly)
            const uint32_t flags = __float_as_uint(q2.z);
            const float f = (r.time - q1.w) / (q2.x - q1.w);
            const F3 pc = sub(rec.p, add(f3(q0.x, q0.y, q0.z), scl(f, f3(q1.x, q1.y, q1.z))));
            const float rr = 1.0f / q0.w;
            rec.n = f3(div_by(pc.x, q0.w, rr), div_by(pc.y, q0.w, rr), div_by(pc.z, q0.w, rr));
            rec.mat = __float_as_uint(q2.y);
            if (flags & SPH_UV) sphere_uv(rec.n, rec.u, rec.v);
        } else if (kind == DK_RECT) {
            const uint32_t axis = __float_as_uint(q1.y);
            uint32_t i, j, k;
            rect_axes(axis & 3u, i, j, k);
            if (axis & RECT_UV) {  // (u, v reach nothing else: two divisions saved)
                const float x = comp(r.o, i) + t * comp(r.d, i);
                const float y = comp(r.o, j) + t * comp(r.d, j);
                rec.u = (x - q0.x) / (q0.y - q0.x);
                rec.v = (y - q0.z) / (q0.w - q0.z);
            }
            const float nv = (axis & RECT_FLIP) ? -1.0f : 1.0f;  // FlipNormals folded into the leaf
            const float zero = (axis & RECT_FLIP) ? -0.0f : 0.0f;
            rec.n = f3(k == 0 ? nv : zero, k == 1 ? nv : zero, k == 2 ? nv : zero);
            rec.mat = __float_as_uint(q1.z);
        } else {  // DK_MEDIUM
            rec.n = f3(1, 0, 0);
            rec.mat = __float_as_uint(q0.y);
        }
        for (int k = n - 1; k >= 0; k--)  // inst_out's operations, innermost first
            chain_out_step(k == 0 ? e0 : (k == 1 ? e1 : C->t[k]), rec.p, rec.n);
        return;
    }
    const uint32_t chain =
        SIMPLE ? 0u : (kind == DK_SPHERE ? S.sph[idx].chain : (kind == DK_RECT ? S.rect[idx].chain : S.med[idx].chain));
    const Ray r = SIMPLE ? root_ray(S, wray) : chain_ray(S, chain, wray);
    rec.t = t;
    rec.u = 0.0f;
    rec.v = 0.0f;
    if (kind == DK_SPHERE) {
        const Sph s = load_sph(S.sph + idx);
        rec.p = at(r, t);
        const F3 pc = sub(rec.p, S.unit_time ? sph_center<true>(s, r.time) : sph_center<false>(s, r.time));
        const float rr = 1.0f / s.r;
        rec.n = f3(div_by(pc.x, s.r, rr), div_by(pc.y, s.r, rr), div_by(pc.z, s.r, rr));
        rec.mat = s.mat;
        // (general scenes carry SPH_UV above the moving bit)
        if ((SIMPLE ? !s.moving : !(s.moving & 1u)) && S.mat[s.mat].needs_uv) sphere_uv(rec.n, rec.u, rec.v);
    } else if (kind == DK_RECT) {
        const DRect& q = S.rect[idx];
        uint32_t i, j, k;
        rect_axes(q.axis & 3u, i, j, k);
        if (S.mat[q.mat].needs_uv) {  // (u, v reach nothing else: two divisions saved)
            const float x = comp(r.o, i) + t * comp(r.d, i);
            const float y = comp(r.o, j) + t * comp(r.d, j);
            rec.u = (x - q.a0) / (q.a1 - q.a0);
            rec.v = (y - q.b0) / (q.b1 - q.b0);
        }
        rec.p = at(r, t);
        const float nv = (q.axis & RECT_FLIP) ? -1.0f : 1.0f;  // FlipNormals folded into the leaf
        const float zero = (q.axis & RECT_FLIP) ? -0.0f : 0.0f;
        rec.n = f3(k == 0 ? nv : zero, k == 1 ? nv : zero, k == 2 ? nv : zero);
        rec.mat = q.mat;
    } else {  // DK_MEDIUM
        const DMedium& m = S.med[idx];
        rec.p = at(r, t);
        rec.n = f3(1, 0, 0);
        rec.mat = m.phase_mat;
    }
    if (SIMPLE)
        root_out(S, rec.p, rec.n);
    else
        chain_out(S, chain, rec.p, rec.n);
}

// ---------------------------------------------------------------------------
// MODE 6: worlds whose random draws depend on the reference's exact visit
// order in ways the culled traversals cannot replay -- a ConstantMedium whose
// boundary holds a medium (constantMedium.h:26-31 asks its boundary twice,
// and asking a medium draws), or a medium below a BvhNode behind an instance
// or inside a list (bvhNode.h:66-96 visits both children exhaustively, and a
// list hands each item its closest hit so far, hitableList.h:24-34).  xhit is
// the reference's own recursion, hit() over the raw scene graph (XHit =
// rtow_hitable), made iterative: one frame per pending call in private
// memory, each with its interval, its ray (the frame it sits in) and the
// record it holds; no culling, every call and draw in the reference's order.
// The leaf tests are the shared ones (sph_quad, rect arithmetic of
// rect_t_ax), so a record is what the other kernels produce for it.
struct XFrame {
    uint32_t h, phase;
    float tmin, tmax;
    float aux;       // LIST: closest hit so far; MEDIUM: the boundary's first hit
    uint32_t auxi;   // LIST: next item; BVH: left child hit
    uint32_t have;   // LIST: a record is held
    Ray r;
    Rec rec;        // LIST: the record so far; BVH: the left child's
};

__device__ __forceinline__ bool xaabb(const float* f, const Ray& r, float tmin, float tmax) {  // aabb.h:22-43
    return ref_slab(f[0], f[3], r.o.x, r.d.x, tmin, tmax) && ref_slab(f[1], f[4], r.o.y, r.d.y, tmin, tmax) &&
           ref_slab(f[2], f[5], r.o.z, r.d.z, tmin, tmax);
}

template <int K, int I, int J>
__device__ __forceinline__ bool xrect(const XHit& H, const Ray& r, float t0, float t1, Rec& rec) {  // xy_rect.h
    const float t = (H.f[4] - cmp3<K>(r.o)) / cmp3<K>(r.d);
    if (t < t0 || t > t1) return false;
    const float x = cmp3<I>(r.o) + t * cmp3<I>(r.d);
    const float y = cmp3<J>(r.o) + t * cmp3<J>(r.d);
    if (x < H.f[0] || x > H.f[1] || y < H.f[2] || y > H.f[3]) return false;
    rec.u = (x - H.f[0]) / (H.f[1] - H.f[0]);
    rec.v = (y - H.f[2]) / (H.f[3] - H.f[2]);
    rec.t = t;
    rec.mat = H.a;
    rec.p = at(r, t);
    rec.n = f3(K == 0 ? 1.0f : 0.0f, K == 1 ? 1.0f : 0.0f, K == 2 ? 1.0f : 0.0f);
    return true;
}

// The closest hit of the world for ray `wr` (world frame) in (tmin, FLT_MAX),
// as color.h:17 asks for it; false: nothing hit (or the frames ran out:
// `overflow`).
// The frames live in global memory (DevParams::xframes: frame k of grid
// thread i at [k * xstride + i]), not in private scratch: a per-lane scratch
// array of 4.6 KB made the runtime size every wave's scratch for it and cost
// the general kernels 8-12 % although xhit itself runs for rare rays.
__device__ __forceinline__ bool xhit(const DevScene& S, const DevParams& P, const Ray& wr, float tmin, Rng& rng, Rec& out,
                                     uint32_t& overflow) {
    XFrame* const fr0 = P.xframes + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t fs = P.xstride;
    int d = 0;
    bool rh = false;  // the result a finished call hands its caller
    Rec rr;
    rr.t = rr.u = rr.v = 0.0f;
    rr.p = rr.n = f3(0, 0, 0);
    rr.mat = 0;
    const int maxd = (int)S.xdepth;  // the world's deepest hit() recursion (rawDepth): the frames allocated
    auto call = [&](uint32_t h, const Ray& r, float t0, float t1) {
        if (d >= maxd) {
            overflow = 1;
            rh = false;
            return;
        }
        XFrame& F = fr0[fs * (size_t)d++];
        F.h = h;
        F.phase = 0;
        F.tmin = t0;
        F.tmax = t1;
        F.r = r;
    };
    call(S.xroot, wr, tmin, FLT_MAX);
    while (d > 0) {
        XFrame& F = fr0[fs * (size_t)(d - 1)];
        const XHit& H = S.xh[F.h];
        const uint32_t ph = F.phase;
        switch (H.kind) {
        case RTOW_HIT_SPHERE:
        case RTOW_HIT_MOVING_SPHERE: {  // sphere.h:20-69, 93-118
            const bool mv = H.kind == RTOW_HIT_MOVING_SPHERE;
            const F3 c = mv ? add(ld3(H.f), scl((F.r.time - H.f[6]) / (H.f[7] - H.f[6]), sub(ld3(H.f + 3), ld3(H.f))))
                            : ld3(H.f);
            const float R = mv ? H.f[8] : H.f[3];
            const float a = dot(F.r.d, F.r.d);
            float t;
            rh = sph_quad(c, R, F.r, a, 1.0f / a, F.tmin, F.tmax, t);
            if (rh) {
                rr.t = t;
                rr.p = at(F.r, t);
                const F3 pc = sub(rr.p, c);
                rr.n = f3(pc.x / R, pc.y / R, pc.z / R);
                rr.mat = H.a;
                rr.u = rr.v = 0.0f;
                if (!mv && S.mat[H.a].needs_uv) sphere_uv(rr.n, rr.u, rr.v);
            }
            d--;
            break;
        }
        case RTOW_HIT_RECT_XY:
            rh = xrect<2, 0, 1>(H, F.r, F.tmin, F.tmax, rr);
            d--;
            break;
        case RTOW_HIT_RECT_XZ:
            rh = xrect<1, 0, 2>(H, F.r, F.tmin, F.tmax, rr);
            d--;
            break;
        case RTOW_HIT_RECT_YZ:
            rh = xrect<0, 1, 2>(H, F.r, F.tmin, F.tmax, rr);
            d--;
            break;
        case RTOW_HIT_BOX:  // box.h:43-45: its list of sides
        case RTOW_HIT_FLIP_NORMALS:
        case RTOW_HIT_TRANSLATE:
        case RTOW_HIT_ROTATE_Y:
            if (ph == 0) {  // hitable.h:25-154: the child with the moved ray
                F.phase = 1;
                Ray q = F.r;
                if (H.kind == RTOW_HIT_TRANSLATE) {
                    q.o = sub(F.r.o, ld3(H.f));
                } else if (H.kind == RTOW_HIT_ROTATE_Y) {
                    const float sn = H.f[0], cs = H.f[1];
                    q.o.x = cs * F.r.o.x - sn * F.r.o.z;
                    q.o.z = sn * F.r.o.x + cs * F.r.o.z;
                    q.d.x = cs * F.r.d.x - sn * F.r.d.z;
                    q.d.z = sn * F.r.d.x + cs * F.r.d.z;
                }
                call(H.a, q, F.tmin, F.tmax);
            } else {  // the record on the way out
                if (rh) {
                    if (H.kind == RTOW_HIT_FLIP_NORMALS) {
                        rr.n = neg(rr.n);
                    } else if (H.kind == RTOW_HIT_TRANSLATE) {
                        rr.p = add(rr.p, ld3(H.f));
                    } else if (H.kind == RTOW_HIT_ROTATE_Y) {
                        const float sn = H.f[0], cs = H.f[1];
                        const F3 p = rr.p, n = rr.n;
                        rr.p.x = cs * p.x + sn * p.z;
                        rr.p.z = -sn * p.x + cs * p.z;
                        rr.n.x = cs * n.x + sn * n.z;
                        rr.n.z = -sn * n.x + cs * n.z;
                    }
                }
                d--;
            }
            break;
        case RTOW_HIT_LIST:  // hitableList.h:20-38
            if (ph == 0) {
                F.phase = 1;
                F.aux = F.tmax;  // closestHitSoFar (a double holding float values)
                F.auxi = 0;
                F.have = 0;
            } else if (rh) {
                F.aux = rr.t;
                F.rec = rr;
                F.have = 1;
            }
            if (F.auxi < H.b) {
                const uint32_t item = S.xrefs[H.a + F.auxi];
                F.auxi++;
                call(item, F.r, F.tmin, F.aux);
            } else {
                rh = F.have != 0;
                if (rh) rr = F.rec;
                d--;
            }
            break;
        case RTOW_HIT_BVH_NODE:  // bvhNode.h:66-96
            if (ph == 0) {
                if (!xaabb(H.f, F.r, F.tmin, F.tmax)) {
                    rh = false;
                    d--;
                    break;
                }
                F.phase = 1;
                call(H.a, F.r, F.tmin, F.tmax);
            } else if (ph == 1) {
                F.auxi = rh ? 1u : 0u;
                F.rec = rr;
                F.phase = 2;
                call(H.b, F.r, F.tmin, F.tmax);
            } else {
                if (F.auxi && rh) {
                    if (F.rec.t < rr.t) rr = F.rec;
                } else if (F.auxi) {
                    rr = F.rec;
                    rh = true;
                }
                d--;
            }
            break;
        case RTOW_HIT_CONSTANT_MEDIUM:  // constantMedium.h:26-74
            if (ph == 0) {
                (void)rng.next();  // the discarded `db` draw
                F.phase = 1;
                call(H.a, F.r, -FLT_MAX, FLT_MAX);
            } else if (ph == 1) {
                if (!rh) {
                    d--;
                    break;
                }
                F.aux = rr.t;
                F.phase = 2;
                call(H.a, F.r, (float)((double)rr.t + 0.0001), FLT_MAX);
            } else {
                if (rh) {
                    float ta = F.aux, tb = rr.t;
                    rh = false;
                    if (ta < F.tmin) ta = F.tmin;
                    if (tb > F.tmax) tb = F.tmax;
                    if (!(ta >= tb)) {
                        if (ta < 0) ta = 0;
                        const float dl = len(F.r.d);
                        const float inside = (tb - ta) * dl;
                        const float dist = (float)(-(1 / H.f[0]) * log(rng.next()));
                        if (dist < inside) {
                            rr.t = ta + dist / dl;
                            rr.p = at(F.r, rr.t);
                            rr.n = f3(1, 0, 0);
                            rr.mat = H.b;
                            rr.u = rr.v = 0.0f;
                            rh = true;
                        }
                    }
                }
                d--;
            }
            break;
        default:
            rh = false;
            d--;
            break;
        }
    }
    out = rr;
    return rh;
}

// ---------------------------------------------------------------------------
// textures (texture.h, noise.h, mathUtilities.h:41-60); Perlin tables in LDS
struct Tables {
    const float4* ranvec;
    const uint32_t* perm;
};

__device__ __forceinline__ float perlin_noise(const Tables& T, F3 p) {
    const float fx = floorf(p.x), fy = floorf(p.y), fz = floorf(p.z);
    const float u = p.x - fx, v = p.y - fy, w = p.z - fz;
    const int i = (int)fx, j = (int)fy, k = (int)fz;
    const float uu = u * u * (3 - 2 * u);
    const float vv = v * v * (3 - 2 * v);
    const float ww = w * w * (3 - 2 * w);
    const uint32_t px0 = T.perm[i & 255] & 255u, px1 = T.perm[(i + 1) & 255] & 255u;
    const uint32_t py0 = (T.perm[j & 255] >> 8) & 255u, py1 = (T.perm[(j + 1) & 255] >> 8) & 255u;
    const uint32_t pz0 = T.perm[k & 255] >> 16, pz1 = T.perm[(k + 1) & 255] >> 16;
    float accum = 0;
#pragma unroll
    for (int di = 0; di < 2; di++)
#pragma unroll
        for (int dj = 0; dj < 2; dj++)
#pragma unroll
            for (int dk = 0; dk < 2; dk++) {
                const uint32_t q = (di ? px1 : px0) ^ (dj ? py1 : py0) ^ (dk ? pz1 : pz0);
                const float4 c = T.ranvec[q];
                const F3 wt = f3(u - di, v - dj, w - dk);
                const float fi = di ? uu : (1 - uu);
                const float fj = dj ? vv : (1 - vv);
                const float fk = dk ? ww : (1 - ww);
                accum += fi * fj * fk * dot(f3(c.x, c.y, c.z), wt);
            }
    return accum;
}

// Perlin::turbulance (noise.h:38-49), spread over the wave.  Every lane with
// `want` needs turb(p) = |sum_o 2^-o * noise(2^o p)|, o = 0..6; those 7k
// octave terms (k lanes) are independent, so the wave's active lanes take
// them as tasks (task t = 7 * requester + octave) instead of each requester
// looping over its 7 octaves while the rest of the wave idles.  The terms go
// through LDS and each requester then sums its own 7 in the reference's order
// (2^o p is exact, as the reference's repeated tempP *= 2 is, and 2^-o * noise
// is exactly weight * noise), so the result is bit for bit the loop's.
// Scratch: this wave's traversal-stack columns, idle between traversals
// (word q at row q / 64, lane column q % 64; needs STACK * 64 >= 640 words).
// Must be called by all active lanes of the wave together.
template <int BS>
__device__ __forceinline__ float wave_turbulence(const Tables& T, uint32_t* wave_stack, bool want, F3 p) {
    const unsigned long long wm = __ballot(want);
    if (wm == 0) return 0.0f;
    const unsigned long long act = __ballot(1);
    const uint32_t lane = threadIdx.x & 63u;
    const unsigned long long lt = (1ull << lane) - 1ull;
    auto slot = [&](uint32_t q) -> uint32_t* { return wave_stack + (q >> 6) * BS + (q & 63u); };
    const uint32_t k = (uint32_t)__popcll(wm);
    const uint32_t nact = (uint32_t)__popcll(act), ar = (uint32_t)__popcll(act & lt);
    const uint32_t wr = (uint32_t)__popcll(wm & lt);
    if (want) {
        *slot(wr) = __float_as_uint(p.x);
        *slot(64 + wr) = __float_as_uint(p.y);
        *slot(128 + wr) = __float_as_uint(p.z);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (uint32_t t = ar; t < 7 * k; t += nact) {
        const uint32_t r = t / 7, o = t - 7 * r;
        const float sc = (float)(1u << o);
        const F3 tp = f3(__uint_as_float(*slot(r)) * sc, __uint_as_float(*slot(64 + r)) * sc,
                         __uint_as_float(*slot(128 + r)) * sc);
        *slot(192 + t) = __float_as_uint((1.0f / sc) * perlin_noise(T, tp));
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    float accum = 0;
    if (want) {
#pragma unroll
        for (uint32_t o = 0; o < 7; o++) accum += __uint_as_float(*slot(192 + 7 * wr + o));
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    return fabsf(accum);
}

// Texture::value of a resolved (non-checker) texture; `turb` is
// Perlin::turbulance(p) when it is a NoiseTexture (wave_turbulence)
__device__ __forceinline__ F3 leaf_tex_value(const DevScene& S, uint32_t ti, float u, float v, F3 p, float turb) {
    const DTex t = S.tex[ti];
    if (t.kind == RTOW_TEX_CONSTANT) return f3(t.f[0], t.f[1], t.f[2]);
    if (t.kind == RTOW_TEX_NOISE) {  // texture.h:44-48
        const float s = 1 + sinf(t.f[0] * p.z + 10 * turb);
        return scl(s, f3(0.5f, 0.5f, 0.5f));
    }
    if (t.kind == RTOW_TEX_IMAGE) {  // texture.h:65-79
        const DImage im = S.img[t.a];
        const int nx = (int)im.nx, ny = (int)im.ny;
        const uint8_t* data = S.texels + im.offset;
        int i = (int)(u * nx);
        int j = (int)((double)((1 - v) * ny) - 0.001);
        if (i < 0) i = 0;
        if (j < 0) j = 0;
        if (i > nx - 1) i = nx - 1;
        if (j > ny - 1) j = ny - 1;
        const size_t o = 3 * (size_t)i + 3 * (size_t)nx * (size_t)j;
        // (float)(c / 255.0) == div_by((float)c, 255, RN(1/255)) for all 256 c
        // (tests/test_numerics.py): float ops instead of three f64 divisions
        const float r255 = 1.0f / 255.0f;
        return f3(div_by((float)data[o], 255.0f, r255), div_by((float)data[o + 1], 255.0f, r255),
                  div_by((float)data[o + 2], 255.0f, r255));
    }
    return f3(0, 0, 0);
}

// ---------------------------------------------------------------------------
// materials (material.h)
__device__ __forceinline__ F3 random_in_unit_sphere(Rng& g) {  // mathUtilities.h:19-25
    F3 p;
    do {
        const float c = g.nextf();  // g++ evaluates vec3(U, U, U) right to left
        const float b = g.nextf();
        const float a = g.nextf();
        p = sub(scl(2.0f, f3(a, b, c)), f3(1, 1, 1));
    } while (sqlen(p) >= 1.0f);
    return p;
}

__device__ __forceinline__ F3 reflect(F3 v, F3 n) { return sub(v, scl(2 * dot(v, n), n)); }

__device__ __forceinline__ bool refract(F3 d, F3 n, float ni, F3& out) {  // material.h:15-26
    const F3 uv = unit(d);
    const float dt = dot(uv, n);
    const float disc = (float)(1.0 - ni * ni * (1 - dt * dt));
    if (disc > 0) {
        out = sub(scl(ni, sub(uv, scl(dt, n))), scl(sqrtf(disc), n));
        return true;
    }
    return false;
}

// material.h:28-32.  pow(x, 5) in double: x*x is exact (a float squared fits
// 48 bits), two more products round at 2^-53 each, and the result is then
// rounded to float -- it differs from libm's pow only when the double value
// lies within ~2^-52 of a float rounding boundary (odds ~2^-28 per call).
__device__ __forceinline__ float schlick(float cosine, float ri) {
    float r0 = (1 - ri) / (1 + ri);
    r0 = r0 * r0;
    const double x = (double)(1 - cosine);
    const double x2 = x * x;
    return (float)(r0 + (1 - r0) * (x2 * x2 * x));
}

// tv: the material's texture value at the hit (Lambertian / Isotropic)
// Lambertian, Metal and Isotropic each start with randomInUnitSphere() and
// draw nothing else, so one rejection loop serves all three (lanes of a wave
// with different materials loop together, not one material after another).
__device__ __forceinline__ bool scatter(const DMat& m, const Ray& in, const Rec& rec, F3 tv, Rng& g, F3& atten, Ray& out) {
    F3 rius = f3(0, 0, 0);
    if (m.kind == RTOW_MAT_LAMBERTIAN || m.kind == RTOW_MAT_METAL || m.kind == RTOW_MAT_ISOTROPIC)
        rius = random_in_unit_sphere(g);
    switch (m.kind) {
    case RTOW_MAT_LAMBERTIAN: {  // material.h:47-53
        const F3 target = add(add(rec.p, rec.n), rius);
        out.o = rec.p;
        out.d = sub(target, rec.p);
        out.time = in.time;
        atten = tv;
        return true;
    }
    case RTOW_MAT_METAL: {  // material.h:62-67
        const F3 reflected = reflect(unit(in.d), rec.n);
        out.o = rec.p;
        out.d = add(reflected, scl(m.param, rius));
        out.time = 0.0f;
        atten = ld3(m.albedo);
        return dot(out.d, rec.n) > 0;
    }
    case RTOW_MAT_DIELECTRIC: {  // material.h:77-117
        const float ri = m.param;
        const F3 reflected = reflect(in.d, rec.n);
        F3 outward, refracted = f3(0, 0, 0);
        float ni, cosine, prob;
        atten = f3(1.0f, 1.0f, 1.0f);
        if (dot(in.d, rec.n) > 0) {
            outward = neg(rec.n);
            ni = ri;
            cosine = ri * dot(in.d, rec.n) / len(in.d);
        } else {
            outward = rec.n;
            ni = m.inv_ri;  // (float)(1.0 / ri), computed on the host
            cosine = -dot(in.d, rec.n) / len(in.d);
        }
        if (refract(in.d, outward, ni, refracted))
            prob = schlick(cosine, ri);
        else
            prob = 1.0f;
        out.o = rec.p;
        out.time = 0.0f;
        out.d = (g.nextf() < prob) ? reflected : refracted;  // double U < (double)prob compares the same reals
        return true;
    }
    case RTOW_MAT_ISOTROPIC: {  // material.h:141-145
        out.o = rec.p;
        out.d = rius;
        out.time = 0.0f;
        atten = tv;
        return true;
    }
    default:  // DiffuseLight never scatters (material.h:126-128)
        return false;
    }
}

// ---------------------------------------------------------------------------
// work-item decoding: item = chunk * n_local_px + local pixel; a local pixel
// is (slot of this rank's tile, position in the 8x8 tile)
__device__ __forceinline__ bool decode_pixel(const DevParams& P, uint32_t lp, uint32_t& x, uint32_t& yimg) {
    const uint32_t slot = lp >> 6, q = lp & 63;
    const uint32_t tile = P.rank + slot * P.world;
    x = (tile % P.tiles_x) * 8 + (q & 7);
    yimg = (tile / P.tiles_x) * 8 + (q >> 3);
    return x < P.width && yimg < P.height;
}

// mathUtilities.h:11-17: 2.0*vec3(U, U, 0) - vec3(1,1,0) until inside the unit
// disk; the constructor's arguments are evaluated right to left (y first)
__device__ __forceinline__ F3 random_in_unit_disk(Rng& g) {
    F3 p;
    do {
        const float b = g.nextf();
        const float a = g.nextf();
        p = sub(scl(2.0f, f3(a, b, 0.0f)), f3(1, 1, 0));
    } while (dot(p, p) >= 1.0f);
    return p;
}
// main.cpp:943-946 + camera.h:123-135: the sample's jitter, time and primary
// ray; the counter restarts per sample.  CAMERA_DOF_EN 0 (the reference's
// build) or, with P.dof, 1: the lens offset draws a unit-sphere point, then a
// unit-disk point (the order g++ evaluates operator+'s arguments in; the
// ref_harness_dof fixtures pin it)
__device__ __forceinline__ void camera_ray(const DevCam& C, const DevParams& P, uint32_t col, uint32_t row,
                                          uint32_t s, Rng& rng, Ray& ray) {
    rng.key = rtow_sample_key(P.seed, row * P.width + col, P.sample_base + s);
    rng.ctr = 0;
    // (double)col + U is exact (col < 2^24, U has 24 fraction bits), so its
    // float rounding is the float sum's (makeParams bounds W and H by 2^24)
    const float u = ((float)col + rng.nextf()) / (float)P.width;
    const float v = ((float)row + rng.nextf()) / (float)P.height;
    F3 rd = scl(C.lens_radius, f3(1.0f, 1.0f, 1.0f));
    if (P.dof) {
        const F3 sph = random_in_unit_sphere(rng);
        rd = add(scl(C.lens_radius, random_in_unit_disk(rng)), sph);
    }
    const F3 offset = add(scl(rd.x, ld3(C.u)), scl(rd.y, ld3(C.v)));
    // with t0 == 0 the double expression is the exact product U*(t1-t0)
    // rounded once to float, as the float product is (0.0f + keeps -0 -> +0)
    float time;
    if (C.t0 == 0.0f)
        time = 0.0f + rng.nextf() * (C.t1 - C.t0);
    else
        time = (float)((double)C.t0 + rng.next() * (double)(C.t1 - C.t0));
    ray.o = add(ld3(C.origin), offset);
    ray.d = sub(sub(add(add(ld3(C.llc), scl(u, ld3(C.hor))), scl(v, ld3(C.ver))), ld3(C.origin)), offset);
    ray.time = time;
}

// The texture value the hit's material will use: Lambertian / Isotropic
// albedo when it scatters (material.h:47-53, 141-145), DiffuseLight emission
// (material.h:130-132); (0,0,0) otherwise.  Texture lookups draw no random
// numbers, so evaluating them ahead of scatter() changes nothing.  Called by
// all active lanes together (wave_turbulence).
template <int BS>
__device__ __forceinline__ F3 texture_at(const DevScene& S, const Tables& T, const DevParams& P, bool hit,
                                         const Rec& rec, uint32_t depth, uint32_t* wave_stack) {
    uint32_t ti = 0;
    bool need = false;
    // a constant colour inline in the material, or a checker of two constant
    // colours inline in its record: no further texture record to load
    bool have = false;
    F3 cv = f3(0, 0, 0);
    if (hit) {
        const DMat m = S.mat[rec.mat];
        need = m.kind == RTOW_MAT_DIFFUSE_LIGHT ||
               ((m.kind == RTOW_MAT_LAMBERTIAN || m.kind == RTOW_MAT_ISOTROPIC) && depth < P.max_depth);
        if (need && m.tex == TEX_INLINE) {
            have = true;
            cv = f3(m.albedo[0], m.albedo[1], m.albedo[2]);
        } else if (need) {
            ti = m.tex;
            for (int guard = 0; guard < 32; guard++) {  // CheckerTexture picks (texture.h:23-39), flat ones inline
                const DTex t = S.tex[ti];
                if (t.kind != RTOW_TEX_CHECKER) break;
                const float sines = sinf(10 * rec.p.x) * sinf(10 * rec.p.y) * sinf(10 * rec.p.z);  // texture.h:27-35
                if (t.c & TEX_FLAT) {
                    have = true;
                    cv = sines < 0 ? f3(t.f[0], t.f[1], t.f[2]) : f3(t.g[0], t.g[1], t.g[2]);
                    break;
                }
                ti = sines < 0 ? t.a : t.b;
            }
        }
    }
    const bool noise = need && !have && S.tex[ti].kind == RTOW_TEX_NOISE;
    const float turb = wave_turbulence<BS>(T, wave_stack, noise, rec.p);
    return need ? (have ? cv : leaf_tex_value(S, ti, rec.u, rec.v, rec.p, turb)) : f3(0, 0, 0);
}

// The rest of one color() call (color.h:12-59) after the closest hit:
// scatter into the next segment (done = false) or end the path with its
// terminal term in `contrib`.
// tv: the hit material's texture value (texture_at)
__device__ __forceinline__ void shade_segment(const DevScene& S, const DevParams& P, bool hit, const Rec& rec, F3 tv,
                                             Ray& ray, F3& thr, uint32_t& depth, Rng& rng, F3& contrib, bool& done) {
    done = true;
    contrib = f3(0, 0, 0);
    if (hit) {
        const DMat m = S.mat[rec.mat];
        Ray sc;
        F3 att;
        if (depth < P.max_depth && scatter(m, ray, rec, tv, rng, att, sc)) {
            // emitted() is (0,0,0) for every material that scatters
            // (material.h:38-40; DiffuseLight never scatters), so the
            // recursion's `emitted + attenuation * color(...)` is a product
            thr = mulv(thr, att);
            ray = sc;
            depth++;
            done = false;
        } else if (m.kind == RTOW_MAT_DIFFUSE_LIGHT) {
            contrib = mulv(thr, tv);
        }
    } else if (P.gi_enable) {
        if (depth < 1) {  // color.h:35-50
            const F3 ud = unit(ray.d);
            const float t = ud.z;
            const float rt = (float)(1.0 + t);
            const F3 sky = f3((float)(rt * 0.1), (float)(rt * 0.3), (float)(rt * 1.0));
            contrib = mulv(thr, scl(P.sky_gain, sky));
        } else {
            contrib = mulv(thr, f3(P.gi_gain, P.gi_gain, P.gi_gain));
        }
    }
}

// ---------------------------------------------------------------------------
// Pixel sums.  A work item's chunk sum (its samples added in order, in float,
// as main.cpp:946 adds them) goes into the pixel's sum as a signed 192-bit
// fixed-point number with 32 fraction bits: q = trunc(sum * 2^32), three
// 64-bit limbs per channel (limb k in plane k of the sums buffer), added with
// 64-bit integer atomics and explicit carries (fx_add192).  Integer addition
// is associative, so the pixel's sum is the same whatever order the chunks
// finish in (no [chunk][pixel] buffer, the frame deterministic and
// independent of the rank split), and progressive frames add into the same
// sums (any chunking gives the same frame).  Every finite float fits: |sum| <
// 2^128, so |q| < 2^160, and 2^32 chunks of those stay below 2^192 -- any
// emitter the reference's float accumulation (main.cpp:939-955) accepts
// renders, negative values included (two's complement).  The truncation is
// below 2^-32 per chunk.  Only a NaN or infinite chunk sum fails the render
// (RTOW_E_UNSUPPORTED, fx_range).  In the usual range (0 <= sum, pixel total
// < 2^32) only limb 0 is ever touched: one atomic per channel.  The pixel
// value is (float)(q * 2^-32), averaged as vec3.h:133-139 does.
__device__ __forceinline__ void fx_limbs(float x, unsigned long long& l0, unsigned long long& l1,
                                         unsigned long long& l2) {
    const uint32_t b = __float_as_uint(x);
    const uint32_t e = (b >> 23) & 255u;
    const unsigned long long m = (b & 0x7fffffu) | (e ? 0x800000u : 0u);
    // |x| * 2^32 = m * 2^sh, sh = max(e, 1) - 150 + 32
    const int sh = (int)(e ? e : 1u) - 118;
    l0 = l1 = l2 = 0;
    if (sh < 0) {
        l0 = sh > -24 ? m >> -sh : 0ull;  // truncation of the bits below 2^-32
    } else {
        const uint32_t w = (uint32_t)sh >> 6, r = (uint32_t)sh & 63u;
        const unsigned long long lo = m << r, hi = r ? m >> (64u - r) : 0ull;
        if (w == 0) {
            l0 = lo;
            l1 = hi;
        } else if (w == 1) {
            l1 = lo;
            l2 = hi;
        } else {
            l2 = lo;
        }
    }
    if (b >> 31) {  // two's complement of the 192-bit magnitude
        l0 = ~l0 + 1ull;
        l1 = ~l1 + (l0 == 0 ? 1ull : 0ull);
        l2 = ~l2 + ((l0 == 0 && l1 == 0) ? 1ull : 0ull);
    }
}
// (l2, l1, l0) added to the 192-bit sum at p, p + plane, p + 2 plane: each
// limb's carry out is read from the atomic's old value, so the limbs hold the
// exact sum of all adds (mod 2^192) whatever their order
__device__ __forceinline__ void fx_add192(unsigned long long* p, size_t plane, unsigned long long l0,
                                          unsigned long long l1, unsigned long long l2) {
    unsigned long long c = 0;
    if (l0) {
        const unsigned long long o = atomicAdd(p, l0);
        c = (o + l0 < o) ? 1ull : 0ull;
    }
    const unsigned long long t1 = l1 + c;
    unsigned long long c2 = (t1 < l1) ? 1ull : 0ull;  // l1 = 2^64 - 1 plus a carry: wraps to 0, carries on
    if (t1) {
        const unsigned long long o = atomicAdd(p + plane, t1);
        c2 |= (o + t1 < o) ? 1ull : 0ull;
    }
    const unsigned long long t2 = l2 + c2;
    if (t2) atomicAdd(p + 2 * plane, t2);
}
__device__ __forceinline__ void fx_add(unsigned long long* dst, size_t plane, F3 acc, uint32_t& range) {
    const float v[3] = {acc.x, acc.y, acc.z};
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float x = v[k];
        if (!(fabsf(x) <= FLT_MAX)) {  // NaN or infinite
            range = 1;
            continue;
        }
        unsigned long long l0, l1, l2;
        fx_limbs(x, l0, l1, l2);
        fx_add192(dst + k, plane, l0, l1, l2);
    }
}

// the signed 192-bit sum as a double: the usual case (l1 = l2 = 0) is
// exactly (double)l0 * 2^-32
__device__ __forceinline__ float fx_value(unsigned long long l0, unsigned long long l1, unsigned long long l2) {
    const bool neg = (l2 >> 63) != 0;
    if (neg) {
        l0 = ~l0 + 1ull;
        l1 = ~l1 + (l0 == 0 ? 1ull : 0ull);
        l2 = ~l2 + ((l0 == 0 && l1 == 0) ? 1ull : 0ull);
    }
    const double v = (double)l2 * 0x1p96 + (double)l1 * 0x1p32 + (double)l0 * 0x1p-32;
    return (float)(neg ? -v : v);
}

// MODE: 0 simple scene (BvhNodes + unit-time spheres under a root instance
// chain), 2 general scene, 3 general scene with media, 4 general scene with
// media whose boundaries are spheres or Boxes (no nested general traversal),
// 5 general scene whose media are all top-level items with such boundaries,
// 8 the same with TOP_GRID items (grid_walk)
// (asked by the top-level scan only: the general traversal carries no media)
// All LDS is one dynamic region (16-B aligned carve, no static __shared__):
// Perlin ranvec (4 KB) | perms (1 KB) | traversal stack STACK x BS words |
// (LDSN) the DNode array of a simple scene | (general scenes) COLD x BS
// words: the path state the traversal does not read, parked while it runs
// (the general kernels are register-bound: 128 VGPRs at 4 waves/SIMD).
// 14 words; 17 with a stack of 16 (MODE 5 parks the sample's RNG key and
// counter there too, PARK_RNG): either way 4 blocks of 256 fit a CU's 160 KB.
template <int MODE, int STACK>
constexpr bool park_rng() { return (MODE == 5 || MODE == 8) && STACK <= 16; }

constexpr size_t lds_bytes(int STACK, int BS, uint32_t n_node, bool ldsn, bool general = false) {
    return 4096 + 1024 + (size_t)STACK * BS * 4 + (ldsn ? (size_t)n_node * sizeof(DNode) : 0) +
           (general ? (size_t)cold_words(STACK) * BS * 4 : 0);
}

template <int MODE, int STACK, int WAVES, bool PROF = false, int BS = BLOCK, bool LDSN = false, bool DBG = false>
__global__ __launch_bounds__(BS, WAVES) void trace_kernel(DevScene S, DevCam C, DevParams P, uint32_t* work,
                                                       unsigned long long* fx, unsigned long long* counters) {
    Prof prof{};
    unsigned long long t_mark = PROF ? __builtin_amdgcn_s_memtime() : 0;
    constexpr bool SIMPLE = MODE == 0;
    static_assert(STACK * 64 >= 640, "wave_turbulence scratch lives in the wave's stack columns");
    static_assert(SIMPLE || BS == BLOCK, "the general traversal strides its LDS stack by BLOCK");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float4* s_ranvec = reinterpret_cast<float4*>(smem);
    uint32_t* s_perm = reinterpret_cast<uint32_t*>(smem + 4096);
    uint32_t* s_stack = reinterpret_cast<uint32_t*>(smem + 5120);
    for (uint32_t i = threadIdx.x; i < 256; i += BS) {
        s_ranvec[i] = reinterpret_cast<const float4*>(S.ranvec)[i];
        s_perm[i] = S.perm[i];
    }
    if constexpr (MODE == 8 && STACK <= 16) {  // the grids' packed heights (grid_walk, GLDS)
        uint32_t* lq = reinterpret_cast<uint32_t*>(smem + 5120 + (size_t)(STACK + cold_words(STACK)) * BS * 4);
        for (uint32_t i = threadIdx.x; i < S.n_gq; i += BS) lq[i] = S.gq[i];
    }
    const DNode* nodes = S.node;
    if constexpr (SIMPLE && LDSN) {
        float4* s_node = reinterpret_cast<float4*>(smem + 5120 + (size_t)STACK * BS * 4);
        const float4* g = reinterpret_cast<const float4*>(S.node);
        const uint32_t n4 = S.n_node * 4u;
        for (uint32_t i = threadIdx.x; i < n4; i += BS) s_node[i] = g[i];
        nodes = reinterpret_cast<const DNode*>(s_node);
    }
    __syncthreads();
    const Tables T{s_ranvec, s_perm};
    uint32_t* stk = s_stack + threadIdx.x;
    uint32_t* cold = reinterpret_cast<uint32_t*>(smem + 5120 + (size_t)STACK * BS * 4) + threadIdx.x;  // general only
    const uint32_t lane = threadIdx.x & 63u;

    uint32_t item = 0, lpx = 0, s = 0, s_end = 0, col = 0, row = 0, depth = 0, nseg = 0, overflow = 0;
    uint32_t fx_range = 0;
    uint32_t nseg_dbg = 0;
    bool need_item = true, need_sample = false;
    F3 acc = f3(0, 0, 0), thr = f3(1, 1, 1);
    Ray ray;
    ray.o = f3(0, 0, 0);
    ray.d = f3(0, 0, 1);
    ray.time = 0;
    Rng rng{0, 0};

    while (true) {
        // ---- wave-wide refill of lanes whose work item is finished ----
        const unsigned long long want = __ballot(need_item);
        if (want) {
            const uint32_t cnt = (uint32_t)__popcll(want);
            const uint32_t leader = (uint32_t)__ffsll((long long)want) - 1u;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(work, cnt);
            base = __shfl(base, (int)leader);
            if (need_item) {
                const uint32_t rank = (uint32_t)__popcll(want & ((1ull << lane) - 1ull));
                item = base + rank;
                if (item >= P.n_items) break;
                // the n_big full chunks pixel-major (a pixel's chunks run side
                // by side: their sums meet in L2 instead of each evicting the
                // pixel's line), then the halving tail chunk-major (the grid
                // ends on one-sample items)
                uint32_t chunk, lp;
                const uint32_t nb_items = P.n_big * P.n_local_px;
                if (item < nb_items) {
                    lp = item / P.n_big;
                    chunk = item - lp * P.n_big;
                } else {
                    const uint32_t j = item - nb_items;
                    const uint32_t k = j / P.n_local_px;
                    lp = j - k * P.n_local_px;
                    chunk = P.n_big + k;
                }
                uint32_t x, yimg;
                if (!decode_pixel(P, lp, x, yimg)) continue;  // padding pixel of a partial tile
                lpx = lp;
                col = x;
                row = P.height - 1u - yimg;  // reference row numbering (main.cpp:932)
                if (chunk < P.n_big) {
                    s = chunk * P.spc;
                    s_end = min(s + P.spc, P.spp);
                } else {
                    const uint32_t k = chunk - P.n_big, base = P.n_big * P.spc, R = P.tail_r;
                    const uint32_t lk = (R + (1u << k) - 1u) >> k;
                    const uint32_t lk1 = k + 1 == P.n_tail ? 0u : (R + (2u << k) - 1u) >> (k + 1);
                    s = base + R - lk;
                    s_end = base + R - lk1;
                }
                acc = f3(0, 0, 0);
                need_item = false;
                need_sample = true;
            }
        }
        if (need_sample) {
            camera_ray(C, P, col, row, s, rng, ray);
            thr = f3(1, 1, 1);
            depth = 0;
            need_sample = false;
        }

        // ---- one segment = one color() call (color.h:12-59) ----
        nseg++;
        if constexpr (PROF) {
            prof.lane_iters++;
            if (first_active_lane()) prof.wave_iters++;
        }
        bool hit;
        Rec rec;
        if constexpr (SIMPLE) {
            if constexpr (PROF) {
                const unsigned long long t_now = __builtin_amdgcn_s_memtime();
                prof.cyc_other += t_now - t_mark;
                t_mark = t_now;
            }
            const Ray lray = root_ray(S, ray);
            float bt = FLT_MAX;
            uint32_t prim;
            // the fast sphere-test sqrt only for rays where it equals sqrtf's
            // effect (sqrt_pos: dot(d, d) >= 2^-24), the exact one for the rest
            const bool fast = dot(lray.d, lray.d) >= 0x1p-24f;
            if (fast)
                prim = trace_simple<STACK, BS, PROF, true>(S, nodes, S.bvh_root, lray, 0.001f, bt, stk, overflow, prof);
            else
                prim = trace_simple<STACK, BS, PROF, false>(S, nodes, S.bvh_root, lray, 0.001f, bt, stk, overflow, prof);
            hit = (prim >> KIND_SHIFT) != DK_NONE;
            if constexpr (PROF) {
                const unsigned long long t_now = __builtin_amdgcn_s_memtime();
                prof.cyc_trav += t_now - t_mark;
                t_mark = t_now;
            }
            if (hit) finalize<true>(S, prim, bt, ray, rec);
            if constexpr (PROF) {
                const unsigned long long t_now = __builtin_amdgcn_s_memtime();
                prof.cyc_fin += t_now - t_mark;
                t_mark = t_now;
            }
        } else if constexpr (MODE == 6) {
            hit = xhit(S, P, ray, 0.001f, rng, rec, overflow);
        } else {
            // park the path state the traversal does not need (COLD)
            cold[0 * BS] = __float_as_uint(acc.x);
            cold[1 * BS] = __float_as_uint(acc.y);
            cold[2 * BS] = __float_as_uint(acc.z);
            cold[3 * BS] = __float_as_uint(thr.x);
            cold[4 * BS] = __float_as_uint(thr.y);
            cold[5 * BS] = __float_as_uint(thr.z);
            cold[6 * BS] = lpx;
            cold[7 * BS] = s;
            cold[8 * BS] = s_end;
            cold[9 * BS] = col;
            cold[10 * BS] = row;
            cold[11 * BS] = depth;
            Best best;
            best.prim = 0;
            cold[12 * BS] = rng.ctr;  // the draw counter at the segment's start (an xhit re-trace restarts there)
            if constexpr (PROF) {
                const unsigned long long t_now = __builtin_amdgcn_s_memtime();
                prof.cyc_other += t_now - t_mark;
                t_mark = t_now;
            }
            constexpr bool PARK = park_rng<MODE, STACK>();
            if constexpr (PARK) {  // the key and counter wait in LDS (media draw through them)
                cold[14 * BS] = (uint32_t)rng.key;
                cold[15 * BS] = (uint32_t)(rng.key >> 32);
                cold[16 * BS] = rng.ctr;
                rng.key = 0;
                rng.ctr = 0;
            }
            hit = traverse_top<MODE == 3 || MODE == 4, STACK, MODE == 3, MODE >= 3, PROF, PARK, MODE == 8>(
                S, ray, 0.001f, stk, rng, best, overflow, &prof);
            if constexpr (PARK) {
                rng.key = (uint64_t)cold[15 * BS] << 32 | cold[14 * BS];
                rng.ctr = cold[16 * BS];
            }
            if constexpr (PROF) {
                const unsigned long long t_now = __builtin_amdgcn_s_memtime();
                prof.cyc_trav += t_now - t_mark;
                t_mark = t_now;
            }
            // A winning rectangle the reference would not have reached -- its
            // boxes grazed at an edge (ref_skips_hit), or entered exactly at
            // the t of a tie it won (tie_unsettled) -- and the record is the
            // reference's only by its own recursion: the ray again, same
            // draws, through xhit (the exact-order kernel's hit()).
            // (also a medium whose interval such a rectangle cut: overflow bit 1)
            if ((overflow & 2u) || (hit && (best.prim >> KIND_SHIFT) == DK_RECT &&
                                    (ref_skips_hit(S, best.prim & LEAF_MASK, ray, best.t, 0.001f) ||
                                     tie_unsettled(S, best.prim, ray, 0.001f, best.t)))) {
                overflow &= 1u;
                rng.ctr = cold[12 * BS];  // same draws (the key is the sample's)
                hit = xhit(S, P, ray, 0.001f, rng, rec, overflow);
            } else if (hit) {
                finalize<false>(S, best.prim & ~TIE_MASK, best.t, ray, rec);
            }
            acc = f3(__uint_as_float(cold[0 * BS]), __uint_as_float(cold[1 * BS]), __uint_as_float(cold[2 * BS]));
            thr = f3(__uint_as_float(cold[3 * BS]), __uint_as_float(cold[4 * BS]), __uint_as_float(cold[5 * BS]));
            lpx = cold[6 * BS];
            s = cold[7 * BS];
            s_end = cold[8 * BS];
            col = cold[9 * BS];
            row = cold[10 * BS];
            depth = cold[11 * BS];
            if constexpr (PROF) {
                const unsigned long long t_now = __builtin_amdgcn_s_memtime();
                prof.cyc_fin += t_now - t_mark;
                t_mark = t_now;
            }
        }
        if constexpr (DBG) {
            if (col == P.dbg_col && row == P.dbg_row && s == P.dbg_sample) {
                const uint32_t k = min(nseg_dbg, P.dbg_max);
                if (k < P.dbg_max) {
                    float* o = P.dbg_out + (size_t)k * RTOW_DEBUG_SEG_FLOATS;
                    o[0] = hit ? 1.0f : 0.0f;
                    o[1] = (float)depth;
                    o[2] = hit ? rec.t : 0.0f;
                    o[3] = hit ? rec.p.x : ray.d.x;
                    o[4] = hit ? rec.p.y : ray.d.y;
                    o[5] = hit ? rec.p.z : ray.d.z;
                    o[6] = hit ? rec.n.x : 0.0f;
                    o[7] = hit ? rec.n.y : 0.0f;
                    o[8] = hit ? rec.n.z : 0.0f;
                    o[9] = hit ? (float)rec.mat : -1.0f;
                    o[10] = (float)rng.ctr;
                    o[11] = 1.0f;
                }
                nseg_dbg++;
            }
        }
        bool done;
        F3 contrib;
        const F3 tv = texture_at<BS>(S, T, P, hit, rec, depth, stk - lane);
        if constexpr (PROF && SIMPLE) {  // simple scenes: texture / shading split of the wave cycles
            const unsigned long long t_now = __builtin_amdgcn_s_memtime();
            prof.cyc_item[0] += t_now - t_mark;
            t_mark = t_now;
        }
        shade_segment(S, P, hit, rec, tv, ray, thr, depth, rng, contrib, done);
        if constexpr (PROF && SIMPLE) {
            const unsigned long long t_now = __builtin_amdgcn_s_memtime();
            prof.cyc_item[1] += t_now - t_mark;
            t_mark = t_now;
        }
        if (done) {
            acc = add(acc, contrib);
            s++;
            if (s >= s_end) {
                fx_add(fx + 4 * (size_t)lpx, 4 * (size_t)P.n_local_px, acc, fx_range);
                need_item = true;
            } else {
                need_sample = true;
            }
        }
    }

    // ---- per-wave counter reduction, one atomic per wave ----
    uint32_t v = nseg;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const unsigned long long ov = __ballot(overflow != 0), orange = __ballot(fx_range != 0);
    if (lane == 0) {
        atomicAdd(&counters[0], (unsigned long long)v);
        if (ov) atomicAdd(&counters[1], 1ull);
        if (orange) atomicAdd(&counters[13], 1ull);
    }
    if constexpr (PROF) {
        uint32_t vals[9] = {prof.lane_steps, prof.wave_steps, prof.leaf_tests, prof.lane_iters, prof.wave_iters,
                            prof.disc_pos, prof.accepted, prof.wave_mixed, prof.wave_sph};
#pragma unroll
        for (int k = 0; k < 9; k++) {
            uint32_t x = vals[k];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
            if (lane == 0) atomicAdd(&counters[k < 5 ? 2 + k : 4 + k], (unsigned long long)x);
        }
        if (lane == 0) {  // s_memtime is per wave: lane 0's copy is the wave's
            atomicAdd(&counters[7], prof.cyc_trav);
            atomicAdd(&counters[8], prof.cyc_other);
            for (int k = 0; k < 8; k++) {
                atomicAdd(&counters[16 + k], prof.cyc_item[k]);
                atomicAdd(&counters[24 + k], prof.visits_item[k]);
            }
            atomicAdd(&counters[32], prof.cyc_fin);
            atomicAdd(&counters[33], prof.cyc_chain);
        }
        {
            uint32_t x = prof.box_lanes, y = prof.box_waves;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off), y += __shfl_xor(y, off);
            if (lane == 0) {
                atomicAdd(&counters[34], (unsigned long long)x);
                atomicAdd(&counters[35], (unsigned long long)y);
            }
        }
    }
}

// fx: the pixel sums (fixed point, see fx_add) of all P.sample_base + P.spp
// samples -- this frame's chunks added by trace_kernel into the running sums
// of the earlier progressive frames (sample_base 0: a fresh, zeroed buffer).
#if !defined(RTOW_TU_SIMPLE) && !defined(RTOW_TU_KERNELS)
__global__ void resolve_kernel(DevParams P, const unsigned long long* fx, uint8_t* slab_bgra, float* slab_lin,
                               uint8_t* fb_bgra, float* fb_lin, unsigned long long* counters) {
    const uint32_t lp = blockIdx.x * blockDim.x + threadIdx.x;
    if (lp >= P.n_local_px) return;
    uint32_t x, yimg;
    const bool valid = decode_pixel(P, lp, x, yimg);
    if (!valid) {
        if (slab_bgra) *reinterpret_cast<uint32_t*>(slab_bgra + 4 * (size_t)lp) = 0u;
        if (slab_lin) {
            slab_lin[3 * (size_t)lp] = 0.0f;
            slab_lin[3 * (size_t)lp + 1] = 0.0f;
            slab_lin[3 * (size_t)lp + 2] = 0.0f;
        }
        return;
    }
    const unsigned long long* sum = fx + 4 * (size_t)lp;
    const size_t plane = 4 * (size_t)P.n_local_px;
    const F3 acc = f3(fx_value(sum[0], sum[plane], sum[2 * plane]), fx_value(sum[1], sum[plane + 1], sum[2 * plane + 1]),
                      fx_value(sum[2], sum[plane + 2], sum[2 * plane + 2]));
    const float k = (float)(1.0 / (double)(float)(P.sample_base + P.spp));  // vec3.h:133-139
    const F3 lin = f3(acc.x * k, acc.y * k, acc.z * k);
    const float sq[3] = {sqrtf(lin.x), sqrtf(lin.y), sqrtf(lin.z)};
    uint32_t q[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {  // main.cpp:961-970
        const double d = 255.99 * (double)sq[i];
        const uint32_t u16 = d >= 65535.0 ? 65535u : (d > 0.0 ? (uint32_t)d : 0u);
        q[i] = u16 > 255u ? 255u : u16;
    }
    const uint32_t px = q[2] | (q[1] << 8) | (q[0] << 16);  // B, G, R, alpha 0 (main.cpp:982-989)
    if (slab_bgra) *reinterpret_cast<uint32_t*>(slab_bgra + 4 * (size_t)lp) = px;
    if (slab_lin) {
        slab_lin[3 * (size_t)lp] = lin.x;
        slab_lin[3 * (size_t)lp + 1] = lin.y;
        slab_lin[3 * (size_t)lp + 2] = lin.z;
    }
    const size_t fb = (size_t)yimg * P.width + x;
    if (fb_bgra) *reinterpret_cast<uint32_t*>(fb_bgra + 4 * fb) = px;
    if (fb_lin) {
        fb_lin[3 * fb] = lin.x;
        fb_lin[3 * fb + 1] = lin.y;
        fb_lin[3 * fb + 2] = lin.z;
    }
}

__global__ void assemble_kernel(uint32_t W, uint32_t H, uint32_t world, uint32_t tiles_x, const uint32_t* slabs,
                                uint32_t stride_px, uint32_t* fb) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= W * H) return;
    const uint32_t x = i % W, y = i / W;
    const uint32_t tile = (y >> 3) * tiles_x + (x >> 3);
    const uint32_t rank = tile % world, slot = tile / world;
    fb[i] = slabs[(size_t)rank * stride_px + slot * 64u + (y & 7u) * 8u + (x & 7u)];
}

// the same for linear slabs: 3 floats per pixel
__global__ void assemble_lin_kernel(uint32_t W, uint32_t H, uint32_t world, uint32_t tiles_x, const float* slabs,
                                    uint32_t stride_px, float* fb) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= W * H) return;
    const uint32_t x = i % W, y = i / W;
    const uint32_t tile = (y >> 3) * tiles_x + (x >> 3);
    const uint32_t rank = tile % world, slot = tile / world;
    const float* s = slabs + 3 * ((size_t)rank * stride_px + slot * 64u + (y & 7u) * 8u + (x & 7u));
    fb[3 * (size_t)i] = s[0];
    fb[3 * (size_t)i + 1] = s[1];
    fb[3 * (size_t)i + 2] = s[2];
}

#endif  // host translation unit

// Every trace_kernel instantiation the host launches (launchWaves), listed
// once: X(MODE, STACK, WAVES, PROF, BS, LDSN, DBG).  The host translation unit
// declares them extern; the kernel translation units (-DRTOW_TU_KERNELS=m,
// one per MODE, see the Makefile) instantiate them, so the modes compile in
// parallel.  The simple-scene kernel the bench runs (random scene, BVH in LDS)
// is compiled in its own unit with -amdgpu-sched-strategy=iterative-ilp
// (RTOW_TU_SIMPLE: +2.8 % there, but -3..-6 % on the general kernels).
#define RTOW_KERNEL_ARGS DevScene, DevCam, DevParams, uint32_t*, unsigned long long*, unsigned long long*
#define RTOW_K_COMMON(X, M, S)                                                                    \
    X(M, S, 1, false, BLOCK, false, true)                                                         \
    X(M, S, 4, false, BLOCK, false, false)                                                        \
    X(M, S, 3, false, BLOCK, false, false)                                                        \
    X(M, S, 1, false, BLOCK, false, false)
#define RTOW_K_PROF(X, M, S) X(M, S, 4, true, BLOCK, false, false)
#define RTOW_K_DEEP(X, M) X(M, 64, 1, false, BLOCK, false, true) X(M, 64, 1, false, BLOCK, false, false)
#define RTOW_KLIST_0(X) RTOW_K_COMMON(X, 0, 16) RTOW_K_PROF(X, 0, 16) RTOW_K_COMMON(X, 0, 32) RTOW_K_DEEP(X, 0)
#define RTOW_KLIST_G(X, M)                                                                         \
    RTOW_K_COMMON(X, M, 16) RTOW_K_PROF(X, M, 16) RTOW_K_COMMON(X, M, 20) RTOW_K_PROF(X, M, 20)   \
    RTOW_K_COMMON(X, M, 32) RTOW_K_PROF(X, M, 32) RTOW_K_DEEP(X, M)
#define RTOW_K_HOT(X) X(0, 16, 4, false, 512, true, false)
#define RTOW_KLIST_6(X) RTOW_K_COMMON(X, 6, 16) RTOW_K_PROF(X, 6, 16)
// MODE 8 (TOP_GRID worlds): the stacks final_ned-like worlds need
#define RTOW_KLIST_8(X) RTOW_K_COMMON(X, 8, 16) RTOW_K_PROF(X, 8, 16) RTOW_K_COMMON(X, 8, 20) RTOW_K_PROF(X, 8, 20) \
    RTOW_K_COMMON(X, 8, 32) RTOW_K_PROF(X, 8, 32) RTOW_K_DEEP(X, 8)
#if defined(RTOW_TU_SIMPLE)
#define RTOW_KX(M, S, W, P, B, L, D) template __global__ void trace_kernel<M, S, W, P, B, L, D>(RTOW_KERNEL_ARGS);
RTOW_K_HOT(RTOW_KX)
#elif defined(RTOW_TU_KERNELS)
#define RTOW_KX(M, S, W, P, B, L, D) template __global__ void trace_kernel<M, S, W, P, B, L, D>(RTOW_KERNEL_ARGS);
#if RTOW_TU_KERNELS == 0
RTOW_KLIST_0(RTOW_KX)
#elif RTOW_TU_KERNELS == 6
RTOW_KLIST_6(RTOW_KX)
#elif RTOW_TU_KERNELS == 8
RTOW_KLIST_8(RTOW_KX)
#else
RTOW_KLIST_G(RTOW_KX, RTOW_TU_KERNELS)
#endif
#else
#define RTOW_KX(M, S, W, P, B, L, D) \
    extern template __global__ void trace_kernel<M, S, W, P, B, L, D>(RTOW_KERNEL_ARGS);
RTOW_K_HOT(RTOW_KX)
RTOW_KLIST_0(RTOW_KX)
RTOW_KLIST_G(RTOW_KX, 2)
RTOW_KLIST_G(RTOW_KX, 3)
RTOW_KLIST_G(RTOW_KX, 4)
RTOW_KLIST_G(RTOW_KX, 5)
RTOW_KLIST_6(RTOW_KX)
RTOW_KLIST_8(RTOW_KX)
#endif
#undef RTOW_KX

}  // namespace rtow_k
using namespace rtow_k;

#if !defined(RTOW_TU_SIMPLE) && !defined(RTOW_TU_KERNELS)

// ===========================================================================
// host side: context, scene upload (the layout: rtow_layout.cpp), launches, C-ABI
// ===========================================================================

#define HIP_TRY(expr)                                                                               \
    do {                                                                                            \
        hipError_t _e = (expr);                                                                     \
        if (_e != hipSuccess)                                                                       \
            return set_error(RTOW_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));        \
    } while (0)

#include "rtow_layout.h"
using namespace rtow_layout;  // HostLayout, buildLayout (rtow_layout.cpp)

struct rtow_context {
    int device = 0;
    int cus = 0;
    int waves = 4;  // trace-kernel occupancy variant (RTOW_TRACE_WAVES; 4 measured best, tools/probe.py)
    int profile = 0;  // RTOW_PROFILE=1: instrumented trace kernel, counters printed to stderr
    int lds_nodes = 1;  // simple-scene BVH staged in LDS when it fits (RTOW_LDS_NODES=0 disables; +11%, tools/ab.py)
    uint32_t auto_spc = 0;  // samples per work item under automatic chunking (RTOW_AUTO_SPC; 0: from the grid, makeParams)
    int tree = RTOW_TREE_SAH;  // rtow_context_set_tree / RTOW_BVH
    // rtow_debug_trace_sample (a render with the segment-recording kernel)
    float* dbg_out = nullptr;
    uint32_t dbg_col = 0, dbg_row = 0, dbg_sample = 0, dbg_max = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {};
    // scene
    void* d_scene = nullptr;
    DevScene scene{};
    bool has_scene = false;
    // work buffers
    void* d_work = nullptr;  // [0] work counter (u32) | [8..] u64 counters
    void* d_xframes = nullptr;  // xhit's call frames (general scenes)
    size_t xframes_bytes = 0;
    unsigned long long* d_fx = nullptr;  // pixel sums of one render (fx_add): three limb planes, 96 B per local pixel
    size_t fx_bytes = 0;
    uint8_t* d_fb = nullptr;  // rtow_render: BGRA frame + linear frame
    size_t fb_bytes = 0;
    // rtow_render_progressive: running sums, samples so far, what they were rendered with
    unsigned long long* d_accum = nullptr;  // progressive frames' running pixel sums (same layout)
    size_t accum_bytes = 0;
    uint32_t accum_spp = 0;
    std::vector<uint8_t> accum_sig;
    unsigned long long* fx_cur = nullptr;  // the sums the launch in flight adds into (d_fx or d_accum)
};

namespace {

template <class T>
size_t pushBlob(std::vector<uint8_t>& blob, const std::vector<T>& v) {
    size_t off = (blob.size() + 255) & ~size_t(255);
    blob.resize(off + v.size() * sizeof(T));
    std::memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
    return off;
}

int ensure(void** p, size_t* have, size_t need) {
    if (*have >= need) return RTOW_OK;
    if (*p) HIP_TRY(hipFree(*p));
    *p = nullptr;
    *have = 0;
    HIP_TRY(hipMalloc(p, need));
    *have = need;
    return RTOW_OK;
}

template <int MODE, int STACK, int WAVES, bool PROF = false, int BS = BLOCK, bool LDSN = false, bool DBG = false>
int launchTrace(rtow_context* c, const DevCam& cam, const DevParams& P, uint32_t bpc, hipStream_t st) {
    const size_t lds = lds_bytes(STACK, BS, c->scene.n_node, LDSN, MODE != 0) +
                       (MODE == 8 && STACK <= 16 ? (size_t)c->scene.n_gq * 4u : 0u);
    // the occupancy query is host work between the launch events: once per
    // (kernel, LDS size) per process
    static std::mutex mu;
    static std::map<std::pair<int, size_t>, int> occ_cache;
    int occ = 0;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = occ_cache.find({c->device, lds});
        if (it != occ_cache.end()) {
            occ = it->second;
        } else {
            HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &occ, trace_kernel<MODE, STACK, WAVES, PROF, BS, LDSN, DBG>, BS, lds));
            occ_cache[{c->device, lds}] = occ;
        }
    }
    if (occ < 1) occ = 1;
    // a persistent grid gains nothing from blocks that cannot be resident:
    // blocks_per_cu is capped at the occupancy (it also sizes xhit's frames)
    uint32_t per = bpc ? std::min(bpc, (uint32_t)occ) : (uint32_t)occ;
    uint32_t grid = (uint32_t)c->cus * per;
    uint32_t maxUseful = (P.n_items + BS - 1) / BS;
    if (grid > maxUseful) grid = std::max(1u, maxUseful);
    DevParams Pk = P;
    if constexpr (MODE != 0) {  // xhit's call frames, one column per grid thread, as deep as the world's recursion
        Pk.xstride = grid * (uint32_t)BS;
        const int rc = ensure((void**)&c->d_xframes, &c->xframes_bytes,
                              (size_t)Pk.xstride * c->scene.xdepth * sizeof(XFrame));
        if (rc) return rc;
        Pk.xframes = (XFrame*)c->d_xframes;
    }
    hipLaunchKernelGGL((trace_kernel<MODE, STACK, WAVES, PROF, BS, LDSN, DBG>), dim3(grid), dim3(BS), lds, st, c->scene,
                       cam, Pk,
                       (uint32_t*)c->d_work, c->fx_cur, (unsigned long long*)((uint8_t*)c->d_work + 8));
    HIP_TRY(hipGetLastError());
    return RTOW_OK;
}

// occupancy variants (waves per SIMD the register allocator must allow):
// c->waves picks one; 0 = the compiler's free choice
template <int MODE, int STACK>
int launchWaves(rtow_context* c, const DevCam& cam, const DevParams& P, uint32_t bpc, hipStream_t st) {
    if (c->dbg_out) return launchTrace<MODE, STACK, 1, false, BLOCK, false, true>(c, cam, P, bpc, st);
    if constexpr (MODE != 0 && STACK <= 32) {
        if (c->profile) return launchTrace<MODE, STACK, 4, true>(c, cam, P, bpc, st);
    }
    if constexpr (STACK <= 32) {
        if constexpr (MODE == 0 && STACK == 16) {
            if (c->profile) return launchTrace<MODE, STACK, 4, true>(c, cam, P, bpc, st);
            // BVH in LDS: 512-thread blocks, 2 per CU (<= 80 KB LDS each)
            if (c->lds_nodes && lds_bytes(STACK, 512, c->scene.n_node, true) <= 80 * 1024)
                return launchTrace<MODE, STACK, 4, false, 512, true>(c, cam, P, bpc, st);
        }
        if (c->waves == 4) return launchTrace<MODE, STACK, 4>(c, cam, P, bpc, st);
        if (c->waves == 3) return launchTrace<MODE, STACK, 3>(c, cam, P, bpc, st);
    }
    return launchTrace<MODE, STACK, 1>(c, cam, P, bpc, st);
}

template <int MODE>
int launchStack(rtow_context* c, const DevCam& cam, const DevParams& P, uint32_t bpc, hipStream_t st) {
    const uint32_t need = c->scene.stack_need;
    // MODE 8 at STACK 16 stages the grids' packed cell heights in LDS: a
    // table larger than GRID_LDS_WORDS goes to the STACK 20 kernel, which
    // reads it from global memory (the same walk, the same frame)
    const bool lds_grid = MODE != 8 || c->scene.n_gq <= GRID_LDS_WORDS;
    if (need <= 16 && lds_grid) return launchWaves<MODE, 16>(c, cam, P, bpc, st);
    // general kernels: 20 entries keep 4 blocks of 256 per CU within LDS
    // (tables + stack + COLD: 39 KB a block)
    if constexpr (MODE != 0)
        if (need <= 20) return launchWaves<MODE, 20>(c, cam, P, bpc, st);
    if (need <= 32) return launchWaves<MODE, 32>(c, cam, P, bpc, st);
    if (need <= 64) return launchWaves<MODE, 64>(c, cam, P, bpc, st);
    return set_error(RTOW_E_UNSUPPORTED, "scene needs a traversal stack deeper than 64 entries");
}

int dispatchTrace(rtow_context* c, const DevCam& cam, const DevParams& P, uint32_t bpc, hipStream_t st) {
    const DevScene& d = c->scene;
    if (d.exact) return launchWaves<6, 16>(c, cam, P, bpc, st);
    if (d.simple && d.unit_time) return launchStack<0>(c, cam, P, bpc, st);
    if (d.n_grid) return launchStack<8>(c, cam, P, bpc, st);  // (buildTop keeps grids to MODE 2 / 5 worlds)
    if (!d.has_media) return launchStack<2>(c, cam, P, bpc, st);
    if (!d.media_any && !d.media_nested) return launchStack<5>(c, cam, P, bpc, st);
    if (!d.media_any) return launchStack<4>(c, cam, P, bpc, st);
    return launchStack<3>(c, cam, P, bpc, st);
}

// cus: the device's compute units (the automatic chunk length depends on the
// grid); auto_spc: RTOW_AUTO_SPC (0: none)
int planParams(int cus, uint32_t auto_spc, const rtow_params* p, DevParams& P) {
    if (!p || p->width == 0 || p->height == 0 || p->spp == 0) return set_error(RTOW_E_INVALID, "bad params");
    if ((uint64_t)p->width * p->height > (1ull << 31) || p->width > (1u << 24) || p->height > (1u << 24))
        return set_error(RTOW_E_INVALID, "image too large");
    uint32_t world = p->world ? p->world : 1;
    if (p->rank >= world) return set_error(RTOW_E_INVALID, "rank >= world");
    std::memset(&P, 0, sizeof P);
    P.width = p->width;
    P.height = p->height;
    P.spp = p->spp;
    // Automatic chunking: the longest items (fewer refills and pixel-sum
    // atomics: on config 2, 64 samples are 4.6 % faster than 16 and 128 another
    // 0.4 %, with 3.6 instead of 16.6 GB of atomic write traffic) that still
    // leave >= 30 items per lane of the grid (cus x 1024 lanes), so a rank's
    // share of a multi-GPU frame keeps a short tail.  Config 2's share of 8
    // ranks (tools/rank_share.py, end of round 3): 64-sample items 151.2 ms,
    // 32-sample 146.4, 16-sample 149.0 -- round 2's bound of 60 items per lane
    // picked 16; 30 picks 32.  Config 2 gets 128 on one or two GPUs, 64 on
    // four, 32 on eight; config 5's shares get 128.
    // RTOW_AUTO_SPC (c->auto_spc) fixes the length instead.  RTOW_FLAG_FRAME_PLAN
    // plans every rank's share as the whole frame (rank 0 of world 1), so its
    // chunks -- and their float sums -- are rtow_render's.
    const bool frame_plan = (p->flags & RTOW_FLAG_FRAME_PLAN) != 0;
    const uint32_t n_px = rtow_rank_tile_count(p->width, p->height, frame_plan ? 0u : p->rank,
                                               frame_plan ? 1u : world) * 64u;
    uint32_t spc = p->samples_per_chunk;
    if (!spc && auto_spc) spc = auto_spc;
    if (!spc) {
        const uint64_t lanes = (uint64_t)std::max(1, cus) * 1024u;
        spc = 16;
        for (uint32_t cand : {128u, 64u, 32u}) {
            if ((uint64_t)n_px * ((p->spp + cand - 1) / cand) >= 30 * lanes) {
                spc = cand;
                break;
            }
        }
    }
    if (spc > p->spp) spc = p->spp;
    P.n_chunks = (p->spp + spc - 1) / spc;
    if (P.n_chunks > 200 && !p->samples_per_chunk) {
        spc = (p->spp + 199) / 200;
        P.n_chunks = (p->spp + spc - 1) / spc;
    }
    P.spc = spc;
    P.n_big = P.n_chunks;
    if (!p->samples_per_chunk && p->spp >= 2 * spc) {  // auto: halving tail (DevParams)
        P.n_big = (p->spp - spc) / spc;
        P.tail_r = p->spp - P.n_big * spc;
        uint32_t k = 0;
        while (((P.tail_r + (1u << k) - 1u) >> k) > 1u) k++;
        P.n_tail = k + 1;
        P.n_chunks = P.n_big + P.n_tail;
    }
    P.tiles_x = (p->width + 7) / 8;
    P.rank = p->rank;
    P.world = world;
    P.n_local_px = rtow_rank_tile_count(p->width, p->height, p->rank, world) * 64u;
    uint64_t items = (uint64_t)P.n_chunks * P.n_local_px;
    if (items >= (1ull << 32) - (1ull << 20)) return set_error(RTOW_E_INVALID, "too many work items; raise samples_per_chunk");
    P.n_items = (uint32_t)items;
    P.max_depth = p->max_depth;
    P.gi_enable = p->gi_enable;
    P.dof = (p->flags & RTOW_FLAG_CAMERA_DOF) ? 1u : 0u;
    P.sky_gain = p->sky_gain;
    P.gi_gain = p->gi_gain;
    P.seed = p->seed;
    return RTOW_OK;
}

int makeParams(const rtow_context* c, const rtow_params* p, DevParams& P) {
    const int rc = planParams(c->cus, c->auto_spc, p, P);
    if (rc) return rc;
    P.dbg_out = c->dbg_out;
    P.dbg_col = c->dbg_col;
    P.dbg_row = c->dbg_row;
    P.dbg_sample = c->dbg_sample;
    P.dbg_max = c->dbg_max;
    return RTOW_OK;
}

DevCam makeCam(const rtow_camera* cam) {
    DevCam d{};
    for (int a = 0; a < 3; a++) {
        d.origin[a] = cam->origin[a];
        d.llc[a] = cam->lower_left_corner[a];
        d.hor[a] = cam->horizontal[a];
        d.ver[a] = cam->vertical[a];
        d.u[a] = cam->u[a];
        d.v[a] = cam->v[a];
    }
    d.lens_radius = cam->lens_radius;
    d.t0 = cam->time0;
    d.t1 = cam->time1;
    return d;
}

// trace + resolve on `st`; outputs may be NULL
int renderCore(rtow_context* c, const rtow_camera* cam, const rtow_params* p, uint8_t* slab_bgra, float* slab_lin,
               uint8_t* fb_bgra, float* fb_lin, hipStream_t st, rtow_stats* stats, unsigned long long* accum = nullptr,
               uint32_t sample_base = 0) {
    auto t0 = std::chrono::steady_clock::now();
    if (!c || !cam) return set_error(RTOW_E_INVALID, "NULL context or camera");
    if (!c->has_scene) return set_error(RTOW_E_INVALID, "no scene uploaded");
    DevParams P;
    int rc = makeParams(c, p, P);
    if (rc) return rc;
    P.sample_base = sample_base;
    HIP_TRY(hipSetDevice(c->device));
    const size_t fx_need = (size_t)P.n_local_px * 3 * 4 * sizeof(unsigned long long);  // three limb planes
    if (accum) {  // progressive: the running sums (zeroed by the caller when they restart)
        c->fx_cur = accum;
    } else {
        rc = ensure((void**)&c->d_fx, &c->fx_bytes, std::max<size_t>(fx_need, 32));
        if (rc) return rc;
        HIP_TRY(hipMemsetAsync(c->d_fx, 0, fx_need, st));
        c->fx_cur = c->d_fx;
    }
    HIP_TRY(hipMemsetAsync(c->d_work, 0, 512, st));
    const DevCam dc = makeCam(cam);
    HIP_TRY(hipEventRecord(c->ev[0], st));
    if (P.n_items) {
        rc = dispatchTrace(c, dc, P, p->blocks_per_cu, st);
        if (rc) return rc;
    }
    HIP_TRY(hipEventRecord(c->ev[1], st));
    if (P.n_local_px) {
        hipLaunchKernelGGL(resolve_kernel, dim3((P.n_local_px + 255) / 256), dim3(256), 0, st, P, c->fx_cur, slab_bgra,
                           slab_lin, fb_bgra, fb_lin, (unsigned long long*)((uint8_t*)c->d_work + 8));
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipEventRecord(c->ev[2], st));
    unsigned long long host_ctr[40] = {};
    HIP_TRY(hipMemcpyAsync(host_ctr, (uint8_t*)c->d_work + 8, sizeof host_ctr, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (c->profile && host_ctr[3])
        std::fprintf(stderr,
                     "rtow-profile: segments %llu | bvh steps lane %llu wave %llu (SIMD eff %.3f, %.2f steps/ray) | "
                     "bounce iters lane %llu wave %llu (SIMD eff %.3f)\n",
                     host_ctr[0], host_ctr[2], host_ctr[3], (double)host_ctr[2] / (64.0 * host_ctr[3]),
                     (double)host_ctr[2] / (double)host_ctr[0], host_ctr[5], host_ctr[6],
                     (double)host_ctr[5] / (64.0 * (double)std::max(1ull, host_ctr[6])));
    if (c->profile && host_ctr[4])
        std::fprintf(stderr,
                     "rtow-profile: sphere slots %.2f/ray (disc>0 %.2f, taken %.2f) | per wave step: sphere path %.3f "
                     "slots, both paths %.3f slots\n",
                     (double)host_ctr[4] / host_ctr[0], (double)host_ctr[9] / host_ctr[0],
                     (double)host_ctr[10] / host_ctr[0], (double)host_ctr[12] / host_ctr[3],
                     (double)host_ctr[11] / host_ctr[3]);
    if (c->profile && host_ctr[7])
        std::fprintf(stderr, "rtow-profile: wave cycles traversal %.3g other %.3g (traversal share %.3f)\n",
                     (double)host_ctr[7], (double)host_ctr[8],
                     (double)host_ctr[7] / (double)(host_ctr[7] + host_ctr[8] + host_ctr[32]));
    if (c->profile && host_ctr[32] && c->scene.simple) {
        const double tot = (double)(host_ctr[7] + host_ctr[8] + host_ctr[32] + host_ctr[16] + host_ctr[17]);
        std::fprintf(stderr, "rtow-profile: simple: wave cycles traversal %.3f finalize %.3f texture %.3f shade %.3f "
                             "refill+camera+sums %.3f\n",
                     host_ctr[7] / tot, host_ctr[32] / tot, host_ctr[16] / tot, host_ctr[17] / tot, host_ctr[8] / tot);
    }
    if (c->profile && host_ctr[32] && !c->scene.simple) {
        const double tot = (double)(host_ctr[7] + host_ctr[8] + host_ctr[32]);
        std::fprintf(stderr, "rtow-profile: general traversal iterations lane %llu wave %llu (SIMD eff %.3f, %.2f per "
                             "ray, node steps %.2f per ray)\n",
                     host_ctr[2], host_ctr[3], (double)host_ctr[2] / (64.0 * std::max(1ull, host_ctr[3])),
                     (double)host_ctr[2] / std::max(1ull, host_ctr[0]), (double)host_ctr[4] / std::max(1ull, host_ctr[0]));
        std::fprintf(stderr, "rtow-profile: general: finalize %.3f of wave cycles; per top item (share, wave visits):",
                     host_ctr[32] / tot);
        for (int k = 0; k < 8; k++)
            if (host_ctr[24 + k]) std::fprintf(stderr, " [%d] %.3f %llu", k, host_ctr[16 + k] / tot, host_ctr[24 + k]);
        std::fprintf(stderr, " | chain_ray+constants of in-place items %.3f\n", host_ctr[33] / tot);
        if (host_ctr[35])
            std::fprintf(stderr, "rtow-profile: Box leaf scans in node steps %.3f per ray, %.1f lanes per wave scan\n",
                         (double)host_ctr[34] / std::max(1ull, host_ctr[0]), (double)host_ctr[34] / host_ctr[35]);
    }
    if (host_ctr[1]) return set_error(RTOW_E_UNSUPPORTED, "traversal stack overflow (scene deeper than bound)");
    if (host_ctr[13])
        return set_error(RTOW_E_UNSUPPORTED, "a chunk of samples summed to NaN or infinity");
    if (stats) {
        float k = 0, r = 0;
        HIP_TRY(hipEventElapsedTime(&k, c->ev[0], c->ev[1]));
        HIP_TRY(hipEventElapsedTime(&r, c->ev[1], c->ev[2]));
        uint64_t valid = 0;
        {
            // count valid pixels of this rank
            uint32_t ntile = rtow_rank_tile_count(P.width, P.height, P.rank, P.world);
            for (uint32_t sl = 0; sl < ntile; sl++) {
                uint32_t tile = P.rank + sl * P.world;
                uint32_t tx = tile % P.tiles_x, ty = tile / P.tiles_x;
                uint32_t w = std::min(8u, P.width - tx * 8), h = std::min(8u, P.height - ty * 8);
                valid += (uint64_t)w * h;
            }
        }
        stats->segments = host_ctr[0];
        stats->pixels = valid;
        stats->samples = valid * P.spp;
        stats->kernel_ms = k;
        stats->resolve_ms = r;
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return RTOW_OK;
}

}  // namespace

extern "C" {

int rtow_device_count(int* count) {
    if (!count) return set_error(RTOW_E_INVALID, "NULL count");
    *count = 0;
    hipError_t e = hipGetDeviceCount(count);
    if (e != hipSuccess) {
        *count = 0;
        return set_error(RTOW_E_NO_DEVICE, hipGetErrorString(e));
    }
    return RTOW_OK;
}

int rtow_context_create(int device, rtow_context** out) {
    if (!out) return set_error(RTOW_E_INVALID, "NULL out");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return set_error(RTOW_E_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= n) return set_error(RTOW_E_INVALID, "device out of range");
    auto* c = new rtow_context;
    c->device = device;
    auto fail = [&](int rc) {
        rtow_context_destroy(c);
        return rc;
    };
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return fail(set_error(RTOW_E_HIP, hipGetErrorString(e)));
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return fail(set_error(RTOW_E_HIP, hipGetErrorString(e)));
    c->cus = prop.multiProcessorCount;
    if (const char* w = std::getenv("RTOW_TRACE_WAVES")) c->waves = std::atoi(w);
    if (const char* pr = std::getenv("RTOW_PROFILE")) c->profile = std::atoi(pr);
    if (const char* ln = std::getenv("RTOW_LDS_NODES")) c->lds_nodes = std::atoi(ln);
    if (const char* sc = std::getenv("RTOW_AUTO_SPC")) c->auto_spc = std::max(1, std::atoi(sc));
    if (const char* tr = std::getenv("RTOW_BVH")) c->tree = std::string(tr) == "ref" ? RTOW_TREE_REFERENCE : RTOW_TREE_SAH;
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess)
        return fail(set_error(RTOW_E_HIP, hipGetErrorString(e)));
    for (auto& ev : c->ev)
        if ((e = hipEventCreate(&ev)) != hipSuccess) return fail(set_error(RTOW_E_HIP, hipGetErrorString(e)));
    if ((e = hipMalloc(&c->d_work, 512)) != hipSuccess) return fail(set_error(RTOW_E_HIP, hipGetErrorString(e)));
    *out = c;
    return RTOW_OK;
}

int rtow_context_destroy(rtow_context* c) {
    if (!c) return RTOW_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->d_scene) (void)hipFree(c->d_scene);
    if (c->d_work) (void)hipFree(c->d_work);
    if (c->d_fx) (void)hipFree(c->d_fx);
    if (c->d_xframes) (void)hipFree(c->d_xframes);
    if (c->d_fb) (void)hipFree(c->d_fb);
    if (c->d_accum) (void)hipFree(c->d_accum);
    for (auto& ev : c->ev)
        if (ev) (void)hipEventDestroy(ev);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return RTOW_OK;
}

int rtow_render_plan(const rtow_context* c, const rtow_params* p, rtow_plan* out) {
    if (!p || !out) return set_error(RTOW_E_INVALID, "NULL argument");
    const int cus = c ? c->cus : 256;  // MI355X: 256 CUs
    DevParams P;
    const int rc = planParams(cus, c ? c->auto_spc : 0u, p, P);
    if (rc) return rc;
    out->samples_per_chunk = P.spc;
    out->n_big = P.n_big;
    out->tail_samples = P.n_tail ? P.tail_r : 0u;
    out->n_tail = P.n_tail;
    out->n_chunks = P.n_chunks;
    out->n_local_px = P.n_local_px;
    out->n_items = P.n_items;
    out->cus = (uint32_t)cus;
    return RTOW_OK;
}

int rtow_context_set_tree(rtow_context* c, int tree) {
    if (!c) return set_error(RTOW_E_INVALID, "NULL context");
    if (tree != RTOW_TREE_SAH && tree != RTOW_TREE_REFERENCE) return set_error(RTOW_E_INVALID, "unknown tree");
    c->tree = tree;
    return RTOW_OK;
}

int rtow_scene_upload(rtow_context* c, const rtow_scene* s) {
    if (!c || !s) return set_error(RTOW_E_INVALID, "NULL argument");
    HostLayout L;
    int rc = buildLayout(*s, L, c->tree);
    if (rc) return rc;
    std::vector<uint8_t> blob;
    size_t o_bvh = pushBlob(blob, L.bvh), o_node = pushBlob(blob, L.node), o_sph = pushBlob(blob, L.sph);
    size_t o_rect = pushBlob(blob, L.rect), o_inst = pushBlob(blob, L.inst), o_list = pushBlob(blob, L.list);
    size_t o_refs = pushBlob(blob, L.refs), o_med = pushBlob(blob, L.med), o_mat = pushBlob(blob, L.mat);
    size_t o_tex = pushBlob(blob, L.tex), o_rv = pushBlob(blob, L.ranvec), o_perm = pushBlob(blob, L.perm);
    size_t o_img = pushBlob(blob, L.img), o_texels = pushBlob(blob, L.texels);
    std::vector<DChainX> chainx(L.chains.size());
    for (size_t c = 0; c < L.chains.size(); c++) {
        const DChain& C = L.chains[c];
        DChainX& X = chainx[c];
        X.n = C.n;
        for (uint32_t k = 0; k < C.n && k < (uint32_t)MAXCHAIN; k++) {
            const DInst& I = L.inst[C.ref[k] & INDEX_MASK];
            uint32_t rb = C.ref[k];
            float rf;
            std::memcpy(&rf, &rb, 4);
            X.t[k] = make_float4(rf, I.p[0], I.p[1], I.p[2]);
        }
    }
    if (chainx.empty()) chainx.push_back(DChainX{});
    size_t o_ch = pushBlob(blob, chainx);
    size_t o_ks = pushBlob(blob, L.sph_key), o_kr = pushBlob(blob, L.rect_key), o_km = pushBlob(blob, L.med_key);
    std::vector<DTop> top = L.top;
    if (top.empty()) top.push_back(DTop{});
    size_t o_top = pushBlob(blob, top);
    if (L.rect_anc.empty()) L.rect_anc.push_back(0u);
    if (L.abox.empty()) L.abox.assign(8, 0.0f);
    if (L.rect_lvl.size() < 4) L.rect_lvl.resize(4, 0u);
    if (L.rect_lmask.empty()) L.rect_lmask.push_back(0ull);
    size_t o_anc = pushBlob(blob, L.rect_anc), o_abox = pushBlob(blob, L.abox), o_lvl = pushBlob(blob, L.rect_lvl);
    size_t o_lmask = pushBlob(blob, L.rect_lmask);
    if (L.prog.empty()) L.prog.push_back(DProg{});
    size_t o_prog = pushBlob(blob, L.prog);
    if (L.box6.empty()) L.box6.push_back(DBox6{});
    size_t o_box6 = pushBlob(blob, L.box6);
    const uint32_t n_grid = L.grid_top;
    if (L.grid.empty()) L.grid.push_back(DGrid{});
    if (L.gcell.empty()) L.gcell.push_back(DGridCell{});
    const uint32_t n_gq = (uint32_t)L.gq.size();
    if (L.gq.empty()) L.gq.push_back(0u);
    size_t o_grid = pushBlob(blob, L.grid), o_gcell = pushBlob(blob, L.gcell), o_gq = pushBlob(blob, L.gq);
    if (L.xh.empty()) L.xh.push_back(XHit{});
    if (L.xrefs.empty()) L.xrefs.push_back(0u);
    size_t o_xh = pushBlob(blob, L.xh), o_xrefs = pushBlob(blob, L.xrefs);
    if (L.tsph.empty()) L.tsph.push_back(DSphere{});
    const size_t o_tsph = pushBlob(blob, L.tsph);
    HIP_TRY(hipSetDevice(c->device));
    if (c->d_scene) {
        HIP_TRY(hipStreamSynchronize(c->stream));
        HIP_TRY(hipFree(c->d_scene));
        c->d_scene = nullptr;
        c->has_scene = false;
    }
    HIP_TRY(hipMalloc(&c->d_scene, blob.size()));
    HIP_TRY(hipMemcpy(c->d_scene, blob.data(), blob.size(), hipMemcpyHostToDevice));
    uint8_t* b = (uint8_t*)c->d_scene;
    DevScene& d = c->scene;
    d.bvh = (const DBvh*)(b + o_bvh);
    d.node = (const DNode*)(b + o_node);
    d.sph = (const DSphere*)(b + o_sph);
    d.rect = (const DRect*)(b + o_rect);
    d.inst = (const DInst*)(b + o_inst);
    d.list = (const DList*)(b + o_list);
    d.refs = (const uint32_t*)(b + o_refs);
    d.med = (const DMedium*)(b + o_med);
    d.mat = (const DMat*)(b + o_mat);
    d.tex = (const DTex*)(b + o_tex);
    d.ranvec = (const float*)(b + o_rv);
    d.perm = (const uint32_t*)(b + o_perm);
    d.img = (const DImage*)(b + o_img);
    d.texels = (const uint8_t*)(b + o_texels);
    d.chains = (const DChainX*)(b + o_ch);
    d.sph_key = (const unsigned long long*)(b + o_ks);
    d.rect_key = (const unsigned long long*)(b + o_kr);
    d.med_key = (const unsigned long long*)(b + o_km);
    d.top = (const DTop*)(b + o_top);
    d.n_top = (uint32_t)L.top.size();
    d.rect_anc = (const uint32_t*)(b + o_anc);
    d.abox = (const float*)(b + o_abox);
    d.rect_lvl = (const uint32_t*)(b + o_lvl);
    d.rect_lmask = (const unsigned long long*)(b + o_lmask);
    d.prog = (const DProg*)(b + o_prog);
    d.box6 = (const DBox6*)(b + o_box6);
    d.grid = (const DGrid*)(b + o_grid);
    d.gcell = (const DGridCell*)(b + o_gcell);
    d.gq = (const uint32_t*)(b + o_gq);
    d.n_gq = n_gq;
    d.n_grid = n_grid;
    for (int a = 0; a < 3; a++) d.tshift[a] = L.tshift[a];
    d.root = L.root;
    d.stack_need = L.stack_need;
    d.has_media = L.has_media ? 1u : 0u;
    d.media_any = L.media_any ? 1u : 0u;
    d.simple = L.simple ? 1u : 0u;
    d.unit_time = L.unit_time ? 1u : 0u;
    d.root_chain_n = L.root_chain_n;
    for (int k = 0; k < 4; k++) d.root_chain[k] = L.root_chain[k];
    d.bvh_root = L.bvh_root;
    d.n_node = L.simple ? (uint32_t)L.node.size() : 0u;
    d.gnode = L.gnode ? 1u : 0u;
    d.media_nested = L.media_nested ? 1u : 0u;
    d.xh = (const XHit*)(b + o_xh);
    d.xrefs = (const uint32_t*)(b + o_xrefs);
    d.xroot = L.xroot;
    d.exact = L.exact ? 1u : 0u;
    d.xdepth = std::max(1u, L.xdepth);
    d.tsph = (const DSphere*)(b + o_tsph);
    c->has_scene = true;
    // progressive sums belong to the scene they were rendered from: a new
    // scene restarts them (rtow_render_progressive)
    c->accum_spp = 0;
    c->accum_sig.clear();
    return RTOW_OK;
}

int rtow_render(rtow_context* c, const rtow_camera* cam, const rtow_params* p, uint8_t* bgra_out, float* linear_out,
                rtow_stats* stats) {
    if (!c || !p) return set_error(RTOW_E_INVALID, "NULL argument");
    rtow_params q = *p;
    q.rank = 0;
    q.world = 1;
    HIP_TRY(hipSetDevice(c->device));
    const size_t npx = (size_t)q.width * q.height;
    size_t need = npx * 4 + npx * 12 + 256;
    int rc = ensure((void**)&c->d_fb, &c->fb_bytes, need);
    if (rc) return rc;
    uint8_t* d_bgra = c->d_fb;
    float* d_lin = (float*)(c->d_fb + ((npx * 4 + 255) & ~size_t(255)));
    rc = renderCore(c, cam, &q, nullptr, nullptr, d_bgra, linear_out ? d_lin : nullptr, c->stream, stats);
    if (rc) return rc;
    if (bgra_out) HIP_TRY(hipMemcpy(bgra_out, d_bgra, npx * 4, hipMemcpyDeviceToHost));
    if (linear_out) HIP_TRY(hipMemcpy(linear_out, d_lin, npx * 12, hipMemcpyDeviceToHost));
    return RTOW_OK;
}

}  // extern "C"

namespace {
// The running sums of rtow_render_progressive / rtow_render_progressive_tiles_device:
// q->rank of q->world's pixels (one rank: the whole frame); the average so far
// goes to the slabs (tiles) or the frame buffers (whole frame), both device.
int progressiveCore(rtow_context* c, const rtow_camera* cam, const rtow_params& q, int reset, uint8_t* slab_bgra,
                    float* slab_lin, uint8_t* fb_bgra, float* fb_lin, hipStream_t st, uint32_t* total_spp,
                    rtow_stats* stats) {
    // what the accumulated samples were rendered with: camera + every param but
    // spp / chunking / the statistics flag (RTOW_FLAG_CAMERA_DOF changes the
    // image, so it is part of the key)
    rtow_params key = q;
    key.spp = 0;
    key.samples_per_chunk = 0;
    key.blocks_per_cu = 0;
    key.flags = q.flags & ~(uint32_t)RTOW_FLAG_STATS;
    std::vector<uint8_t> sig(sizeof(rtow_camera) + sizeof(rtow_params));
    std::memcpy(sig.data(), cam, sizeof(rtow_camera));
    std::memcpy(sig.data() + sizeof(rtow_camera), &key, sizeof(rtow_params));
    if (reset || sig != c->accum_sig) {
        c->accum_spp = 0;
        c->accum_sig = sig;
    }
    if ((uint64_t)c->accum_spp + q.spp > 0xffffffffull) return set_error(RTOW_E_INVALID, "too many accumulated samples");
    const uint32_t world = q.world ? q.world : 1;
    if (q.rank >= world) return set_error(RTOW_E_INVALID, "rank >= world");
    HIP_TRY(hipSetDevice(c->device));
    const size_t acc_need = (size_t)rtow_rank_tile_count(q.width, q.height, q.rank, world) * 64 * 3 * 4 *
                            sizeof(unsigned long long);  // three limb planes (fx_add)
    if (c->accum_bytes < acc_need) c->accum_spp = 0;
    int rc = ensure((void**)&c->d_accum, &c->accum_bytes, acc_need);
    if (rc) return rc;
    if (c->accum_spp == 0) HIP_TRY(hipMemsetAsync(c->d_accum, 0, acc_need, st));
    rc = renderCore(c, cam, &q, slab_bgra, slab_lin, fb_bgra, fb_lin, st, stats, c->d_accum, c->accum_spp);
    if (rc) {
        c->accum_spp = 0;
        return rc;
    }
    c->accum_spp += q.spp;
    if (total_spp) *total_spp = c->accum_spp;
    return RTOW_OK;
}
}  // namespace

extern "C" {

int rtow_render_progressive(rtow_context* c, const rtow_camera* cam, const rtow_params* p, int reset,
                            uint8_t* bgra_out, float* linear_out, uint32_t* total_spp, rtow_stats* stats) {
    if (!c || !p || !cam) return set_error(RTOW_E_INVALID, "NULL argument");
    rtow_params q = *p;
    q.rank = 0;
    q.world = 1;
    HIP_TRY(hipSetDevice(c->device));
    const size_t npx = (size_t)q.width * q.height;
    size_t need = npx * 4 + npx * 12 + 256;
    int rc = ensure((void**)&c->d_fb, &c->fb_bytes, need);
    if (rc) return rc;
    uint8_t* d_bgra = c->d_fb;
    float* d_lin = (float*)(c->d_fb + ((npx * 4 + 255) & ~size_t(255)));
    rc = progressiveCore(c, cam, q, reset, nullptr, nullptr, d_bgra, linear_out ? d_lin : nullptr, c->stream, total_spp,
                         stats);
    if (rc) return rc;
    if (bgra_out) HIP_TRY(hipMemcpy(bgra_out, d_bgra, npx * 4, hipMemcpyDeviceToHost));
    if (linear_out) HIP_TRY(hipMemcpy(linear_out, d_lin, npx * 12, hipMemcpyDeviceToHost));
    return RTOW_OK;
}

int rtow_debug_trace_sample(rtow_context* c, const rtow_camera* cam, const rtow_params* p, uint32_t x, uint32_t y,
                            uint32_t sample, float* out, uint32_t max_segments, uint32_t* n_segments) {
    if (!c || !p || !out || max_segments == 0) return set_error(RTOW_E_INVALID, "NULL argument");
    if (x >= p->width || y >= p->height || sample >= p->spp) return set_error(RTOW_E_INVALID, "pixel/sample out of range");
    HIP_TRY(hipSetDevice(c->device));
    const size_t bytes = (size_t)max_segments * RTOW_DEBUG_SEG_FLOATS * sizeof(float);
    HIP_TRY(hipMalloc((void**)&c->dbg_out, bytes));
    HIP_TRY(hipMemset(c->dbg_out, 0, bytes));
    c->dbg_col = x;
    c->dbg_row = p->height - 1 - y;
    c->dbg_sample = sample;
    c->dbg_max = max_segments;
    rtow_params q = *p;
    q.rank = 0;
    q.world = 1;
    rtow_stats st;
    int rc = renderCore(c, cam, &q, nullptr, nullptr, nullptr, nullptr, c->stream, &st);
    hipError_t e = hipSuccess;
    if (rc == RTOW_OK) e = hipMemcpy(out, c->dbg_out, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(c->dbg_out);
    c->dbg_out = nullptr;
    if (rc) return rc;
    if (e != hipSuccess) return set_error(RTOW_E_HIP, hipGetErrorString(e));
    uint32_t n = 0;
    while (n < max_segments && out[(size_t)n * RTOW_DEBUG_SEG_FLOATS + 11] != 0.0f) n++;
    if (n_segments) *n_segments = n;
    return RTOW_OK;
}

int rtow_render_tiles_device(rtow_context* c, const rtow_camera* cam, const rtow_params* p, void* d_bgra_slab,
                             void* d_linear_slab, void* stream, rtow_stats* stats) {
    if (!c) return set_error(RTOW_E_INVALID, "NULL context");
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return renderCore(c, cam, p, (uint8_t*)d_bgra_slab, (float*)d_linear_slab, nullptr, nullptr, st, stats);
}

int rtow_render_progressive_tiles_device(rtow_context* c, const rtow_camera* cam, const rtow_params* p, int reset,
                                         void* d_bgra_slab, void* d_linear_slab, void* stream, uint32_t* total_spp,
                                         rtow_stats* stats) {
    if (!c || !p || !cam) return set_error(RTOW_E_INVALID, "NULL argument");
    rtow_params q = *p;
    if (q.world == 0) q.world = 1;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return progressiveCore(c, cam, q, reset, (uint8_t*)d_bgra_slab, (float*)d_linear_slab, nullptr, nullptr, st,
                           total_spp, stats);
}

int rtow_assemble_device(rtow_context* c, uint32_t width, uint32_t height, uint32_t world, const void* d_slabs,
                         uint32_t slab_stride_px, void* d_bgra_frame, void* stream) {
    if (!c || !d_slabs || !d_bgra_frame || width == 0 || height == 0) return set_error(RTOW_E_INVALID, "bad arguments");
    if (world == 0) world = 1;
    if (slab_stride_px < rtow_rank_tile_count(width, height, 0, world) * 64u)
        return set_error(RTOW_E_INVALID, "slab stride smaller than rank 0's slab");
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    HIP_TRY(hipSetDevice(c->device));
    const uint32_t n = width * height;
    hipLaunchKernelGGL(assemble_kernel, dim3((n + 255) / 256), dim3(256), 0, st, width, height, world, (width + 7) / 8,
                       (const uint32_t*)d_slabs, slab_stride_px, (uint32_t*)d_bgra_frame);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(st));
    return RTOW_OK;
}

int rtow_assemble_linear_device(rtow_context* c, uint32_t width, uint32_t height, uint32_t world,
                                const void* d_slabs, uint32_t slab_stride_px, void* d_linear_frame, void* stream) {
    if (!c || !d_slabs || !d_linear_frame || width == 0 || height == 0)
        return set_error(RTOW_E_INVALID, "bad arguments");
    if (world == 0) world = 1;
    if (slab_stride_px < rtow_rank_tile_count(width, height, 0, world) * 64u)
        return set_error(RTOW_E_INVALID, "slab stride smaller than rank 0's slab");
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    HIP_TRY(hipSetDevice(c->device));
    const uint32_t n = width * height;
    hipLaunchKernelGGL(assemble_lin_kernel, dim3((n + 255) / 256), dim3(256), 0, st, width, height, world,
                       (width + 7) / 8, (const float*)d_slabs, slab_stride_px, (float*)d_linear_frame);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(st));
    return RTOW_OK;
}

}  // extern "C"
#endif  // host translation unit
