/* regroup_emu.c -- the bench kernel's traversal (trace_simple,
 * ray-tracing-one-weekend_amd/csrc/rtow_device.hip) restated on the CPU for
 * tools/regroup_emulate.py: for every ray, the node steps it takes and, per
 * step, which code paths its two slots run -- the input of a lockstep model
 * of 64-lane waves.  Same tree (the uploaded DNodes, RTOW_LAYOUT_DUMP), same
 * float operations (-ffp-contract=off; the one-FMA world-frame slabs, the
 * culling bound, the 64-bit record key), sqrtf for the sphere roots.
 *
 *   gcc -O2 -shared -fPIC -ffp-contract=off -o tools/_build/regroup_emu.so tools/regroup_emu.c -lm
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct {
    float a[7];
    uint32_t ref_a;
    float b[7];
    uint32_t ref_b;
} dnode;

enum { KIND_SHIFT = 28, DK_BVH = 0, DK_SPHERE = 1, DK_NONE = 15 };
#define INDEX_MASK ((1u << KIND_SHIFT) - 1u)
#define NONE ((uint32_t)DK_NONE << KIND_SHIFT)

static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float cull_bound(float t) { return fmaf(fabsf(t), 0.001953125f, t); }

/* slab_f: one-FMA planes in the world frame */
static int slab_f(const float* s, const float* oi, const float* inv, float werr, float tmin, float tmax_c,
                  float* tnear) {
    const float tx0 = fmaf(s[0], inv[0], -oi[0]), tx1 = fmaf(s[3], inv[0], -oi[0]);
    const float ty0 = fmaf(s[1], inv[1], -oi[1]), ty1 = fmaf(s[4], inv[1], -oi[1]);
    const float tz0 = fmaf(s[2], inv[2], -oi[2]), tz1 = fmaf(s[5], inv[2], -oi[2]);
    const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), tmin));
    const float ex = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
    float tf = fmaf(ex, 1.001953125f, werr);
    tf = tf < tmax_c ? tf : tmax_c;
    *tnear = tn;
    return tn <= tf;
}

/* sph_root: the root Sphere::hit records; *disc_pos: b*b - a*c > 0 */
static int sph_root(const float* s, float time, const float* o, const float* d, float a, float tmin, float* t,
                    int* disc_pos) {
    const float c[3] = {s[0] + time * s[4], s[1] + time * s[5], s[2] + time * s[6]};
    const float oc[3] = {o[0] - c[0], o[1] - c[1], o[2] - c[2]};
    const float b = d[0] * oc[0] + d[1] * oc[1] + d[2] * oc[2];
    const float cc = (oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2]) - s[3];
    const float disc = b * b - a * cc;
    *disc_pos = disc > 0;
    if (!(disc > 0)) return 0;
    const float sq = sqrtf(disc);
    const float tn = (-b - sq) / a, tf = (-b + sq) / a;
    const float root = tn > tmin ? tn : tf;
    *t = root;
    return root < 3.4028235e38f && root > tmin;
}

/* Trace n rays (7 floats each: origin in the BVH frame, direction, time).
 * codes[i * maxs + k]: step k of ray i -- bit 0 slot b is a sphere, bit 1
 * slot a is a sphere, bit 2 slot b's sphere has disc > 0, bit 3 the same for
 * a, bit 4 slot b's slab test hit, bit 5 slot a's.  steps[i]: the step count
 * (capped at maxs), prim[i] / bt[i]: the record. */
int trace_rays_seeded(const dnode* nodes, uint32_t n_nodes, uint32_t root, const float* tshift, const float* rays,
                      int n, uint8_t* codes, int maxs, int* steps, uint32_t* prim, float* bt_out, const float* seed_t,
                      const uint32_t* seed_ref);
int trace_rays(const dnode* nodes, uint32_t n_nodes, uint32_t root, const float* tshift, const float* rays, int n,
               uint8_t* codes, int maxs, int* steps, uint32_t* prim, float* bt_out) {
    return trace_rays_seeded(nodes, n_nodes, root, tshift, rays, n, codes, maxs, steps, prim, bt_out, 0, 0);
}

/* Sphere::hit of one sphere (c0, radius^2, dc as a DNode slot holds them) for
 * ray i: the root or -1 (the seed a lane could take from a predicted sphere) */
float sphere_t(const float* slot, const float* R) {
    const float o[3] = {R[0], R[1], R[2]}, d[3] = {R[3], R[4], R[5]};
    const float a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    float t;
    int dp;
    return sph_root(slot, R[6], o, d, a, 0.001f, &t, &dp) ? t : -1.0f;
}

/* The same with a seed per ray (seed_ref NONE: none): the record starts as
 * that sphere's hit, as if the lane had tested it before the traversal. */
int trace_rays_seeded(const dnode* nodes, uint32_t n_nodes, uint32_t root, const float* tshift, const float* rays,
                      int n, uint8_t* codes, int maxs, int* steps, uint32_t* prim, float* bt_out, const float* seed_t,
                      const uint32_t* seed_ref) {
    for (int i = 0; i < n; i++) {
        const float* R = rays + 7 * (size_t)i;
        const float o[3] = {R[0], R[1], R[2]}, d[3] = {R[3], R[4], R[5]};
        const float time = R[6];
        const float ow[3] = {o[0] + tshift[0], o[1] + tshift[1], o[2] + tshift[2]};
        const float BIG = 18446744073709551616.0f;
        float inv[3], oi[3];
        for (int k = 0; k < 3; k++) {
            const float v = 1.0f / d[k];
            inv[k] = fminf(fmaxf(v, -BIG), BIG);
            oi[k] = ow[k] * inv[k];
        }
        const float werr = fmaxf(fmaxf(fabsf(oi[0]), fabsf(oi[1])), fabsf(oi[2])) * 0x1p-21f;
        const float a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        const float tmin = 0.001f;
        float bt = 3.4028235e38f;
        uint32_t best = NONE;
        if (seed_ref && seed_ref[i] != NONE) {
            bt = seed_t[i];
            best = seed_ref[i];
        }
        float btc = cull_bound(bt) + werr;
        unsigned long long rkey = (unsigned long long)f2u(bt) << 32 | (uint32_t)~best;
        uint32_t stack[128];
        int sp = 0;
        uint32_t cur = root, top = NONE;
        int ns = 0;
        for (;;) {
            if ((cur & INDEX_MASK) >= n_nodes) return -1;
            const dnode* nd = nodes + (cur & INDEX_MASK);
            uint8_t code = 0;
            float ta = 0.0f, tb = 0.0f;
            int ha = 0, hb = 0;
            for (int slot = 1; slot >= 0; slot--) {  /* slot b first */
                const float* f = slot ? nd->b : nd->a;
                const uint32_t ref = slot ? nd->ref_b : nd->ref_a;
                if ((ref >> KIND_SHIFT) == DK_SPHERE) {
                    code |= slot ? 1 : 2;
                    float t;
                    int dp;
                    if (sph_root(f, time, o, d, a, tmin, &t, &dp)) {
                        const unsigned long long k = (unsigned long long)f2u(t) << 32 | (uint32_t)~ref;
                        if (k < rkey) {
                            rkey = k;
                            btc = cull_bound(t) + werr;
                        }
                    }
                    if (dp) code |= slot ? 4 : 8;
                } else {
                    float tn;
                    const int h = slab_f(f, oi, inv, werr, tmin, btc, &tn);
                    if (slot) hb = h, tb = tn; else ha = h, ta = tn;
                    if (h) code |= slot ? 16 : 32;
                }
            }
            if (ns < maxs) codes[(size_t)i * maxs + ns] = code;
            ns++;
            const int afirst = ta <= tb;
            const int both = ha && hb;
            uint32_t nxt = both ? (afirst ? nd->ref_a : nd->ref_b) : (ha ? nd->ref_a : (hb ? nd->ref_b : NONE));
            if (both) {
                if (top != NONE) {
                    if (sp >= 127) return -2;
                    stack[sp++] = top;
                }
                top = afirst ? nd->ref_b : nd->ref_a;
            }
            if (nxt == NONE) {
                nxt = top;
                top = sp > 0 ? stack[--sp] : NONE;
            }
            if (nxt == NONE) break;
            cur = nxt;
        }
        steps[i] = ns;
        prim[i] = ~(uint32_t)rkey;
        bt_out[i] = u2f((uint32_t)(rkey >> 32));
    }
    return 0;
}
