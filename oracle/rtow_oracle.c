/*
 * rtow_oracle.c — TEST INFRASTRUCTURE ONLY: the C restatement of the
 * reference render path.  See rtow_oracle.h.  Every function cites the
 * reference file:line it follows (paths relative to rayTracingOneWeekend/).
 *
 * Float semantics notes: C float arithmetic here is
 * IEEE single (x86-64 SSE, FLT_EVAL_METHOD 0) and the Makefile forbids FMA
 * contraction.  Where the reference mixes in a double literal or a double
 * function (unifRand, M_PI, 255.99, pow, log, 1.0/x) the promotion to double
 * is written out explicitly.  float overloads of the C++ <cmath> calls map to
 * sqrtf/sinf/atan2f/asinf/floorf/fabsf.
 */
#define _GNU_SOURCE
#include "rtow_oracle.h"
#include "../include/rtow_rng.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---- vec3 / ray (vec3.h, ray.h) ---------------------------------------- */
typedef struct { float x, y, z; } v3;
typedef struct { v3 o, d; float time; } ray_t;

static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }      /* vec3.h:58 */
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }      /* vec3.h:62 */
static inline v3 mulv(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }     /* vec3.h:66 */
static inline v3 scl(float t, v3 v) { return mk(t * v.x, t * v.y, t * v.z); }         /* vec3.h:74,78 */
static inline v3 divs(v3 v, float t) { return mk(v.x / t, v.y / t, v.z / t); }        /* vec3.h:82 */
static inline v3 neg(v3 v) { return mk(-v.x, -v.y, -v.z); }                          /* vec3.h:19 */
static inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }    /* vec3.h:86 */
static inline float len(v3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }   /* vec3.h:30 */
static inline float sqlen(v3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }        /* vec3.h:34 */
static inline v3 unit(v3 v) {                                                         /* vec3.h:141-148 */
    if (len(v) == 0.0) return mk(0.0f, 0.0f, 0.0f);
    return divs(v, len(v));
}
static inline v3 at(const ray_t* r, float t) { return add(r->o, scl(t, r->d)); }      /* ray.h:11 */
static inline v3 ld3(const float* f) { return mk(f[0], f[1], f[2]); }

/* ---- RNG (rngs.h:9-11 replaced, include/rtow_rng.h) --------------------- */
typedef struct { uint64_t key; uint32_t ctr; } rng_t;

typedef struct {
    const rtow_scene* s;
    rtow_oracle_counters c;
    float* trace; /* rtow_oracle_trace_sample: segment records, or NULL */
    uint32_t trace_max, trace_n;
    float* rays;  /* rtow_oracle_trace_rays: each color() call's ray (o, d, time), or NULL */
    uint32_t rays_max, rays_n;
} ctx_t;

static inline double unif(ctx_t* cx, rng_t* g) {
    cx->c.draws++;
    return (double)rtow_draw24(g->key, g->ctr++) * (1.0 / 16777216.0);
}

/* ---- HitRecord (hitable.h:9-17) ---------------------------------------- */
typedef struct {
    float t, u, v;
    v3 p, n;
    uint32_t mat;
} hitrec;

/* mathUtilities.h:11-17: 2.0*vec3(U, U, 0) - vec3(1,1,0), the constructor's
 * arguments evaluated right to left (y drawn first) */
static v3 random_in_unit_disk(ctx_t* cx, rng_t* g) {
    v3 p;
    do {
        double b = unif(cx, g);
        double a = unif(cx, g);
        p = sub(scl(2.0f, mk((float)a, (float)b, 0.0f)), mk(1, 1, 0));
    } while (dot(p, p) >= 1.0);
    return p;
}

/* mathUtilities.h:19-25 */
static v3 random_in_unit_sphere(ctx_t* cx, rng_t* g) {
    v3 p;
    do {
        /* 2.0*vec3(U, U, U) - vec3(1,1,1); g++ evaluates the constructor's
         * arguments right to left, so the first draw is z */
        double c = unif(cx, g);
        double b = unif(cx, g);
        double a = unif(cx, g);
        p = sub(scl(2.0f, mk((float)a, (float)b, (float)c)), mk(1, 1, 1));
    } while (sqlen(p) >= 1.0);
    return p;
}

/* mathUtilities.h:62-68 */
static void sphere_uv(v3 p, float* u, float* v) {
    float phi = atan2f(p.z, p.x);
    float theta = asinf(p.y);
    *u = (float)(1 - (phi + M_PI) / (2 * M_PI));
    *v = (float)((theta + M_PI / 2) / M_PI);
}

/* aabb.h:8-9, 22-43 */
static inline float ffmin(float a, float b) { return a < b ? a : b; }
static inline float ffmax(float a, float b) { return a > b ? a : b; }
static int aabb_hit(const float* mn, const float* mx, const ray_t* r, float tmin, float tmax) {
    const float o[3] = {r->o.x, r->o.y, r->o.z};
    const float d[3] = {r->d.x, r->d.y, r->d.z};
    for (int a = 0; a < 3; a++) {
        float t0 = ffmin((mn[a] - o[a]) / d[a], (mx[a] - o[a]) / d[a]);
        float t1 = ffmax((mn[a] - o[a]) / d[a], (mx[a] - o[a]) / d[a]);
        tmin = ffmax(t0, tmin);
        tmax = ffmin(t1, tmax);
        if (tmax <= tmin) return 0;
    }
    return 1;
}

static int hit(ctx_t* cx, rng_t* g, uint32_t idx, const ray_t* r, float tmin, float tmax, hitrec* rec);

/* sphere.h:20-69 */
static int hit_sphere(const rtow_hitable* h, const ray_t* r, float tmin, float tmax, hitrec* rec) {
    v3 c = ld3(h->f);
    float R = h->f[3];
    v3 oc = sub(r->o, c);
    float a = dot(r->d, r->d);
    float b = dot(r->d, oc);
    float cc = dot(oc, oc) - R * R;
    float disc = b * b - a * cc;
    if (disc > 0) {
        float temp = (-b - sqrtf(b * b - a * cc)) / a;
        if (temp < tmax && temp > tmin) {
            rec->t = temp;
            rec->p = at(r, temp);
            sphere_uv(divs(sub(rec->p, c), R), &rec->u, &rec->v);
            rec->n = divs(sub(rec->p, c), R);
            rec->mat = h->a;
            return 1;
        }
        temp = (-b + sqrtf(b * b - a * cc)) / a;
        if (temp < tmax && temp > tmin) {
            rec->t = temp;
            rec->p = at(r, temp);
            sphere_uv(divs(sub(rec->p, c), R), &rec->u, &rec->v);
            rec->n = divs(sub(rec->p, c), R);
            rec->mat = h->a;
            return 1;
        }
    }
    return 0;
}

/* sphere.h:129-131 */
static v3 moving_center(const rtow_hitable* h, float time) {
    v3 c0 = ld3(h->f), c1 = ld3(h->f + 3);
    return add(c0, scl((time - h->f[6]) / (h->f[7] - h->f[6]), sub(c1, c0)));
}

/* sphere.h:93-118 (u, v are not written) */
static int hit_moving_sphere(const rtow_hitable* h, const ray_t* r, float tmin, float tmax, hitrec* rec) {
    float R = h->f[8];
    v3 oc = sub(r->o, moving_center(h, r->time));
    float a = dot(r->d, r->d);
    float b = dot(oc, r->d);
    float c = dot(oc, oc) - R * R;
    float disc = b * b - a * c;
    if (disc > 0) {
        float temp = (-b - sqrtf(disc)) / a;
        if (temp < tmax && temp > tmin) {
            rec->t = temp;
            rec->p = at(r, temp);
            rec->n = divs(sub(rec->p, moving_center(h, r->time)), R);
            rec->mat = h->a;
            return 1;
        }
        temp = (-b + sqrtf(disc)) / a;
        if (temp < tmax && temp > tmin) {
            rec->t = temp;
            rec->p = at(r, temp);
            rec->n = divs(sub(rec->p, moving_center(h, r->time)), R);
            rec->mat = h->a;
            return 1;
        }
    }
    return 0;
}

/* xy_rect.h:22-40 / 57-75 / 92-110: axis k is the plane normal, (i, j) the
 * in-plane axes in the order the reference names them. */
static int hit_rect(const rtow_hitable* h, int i, int j, int k, v3 normal, const ray_t* r, float t0,
                    float t1, hitrec* rec) {
    const float o[3] = {r->o.x, r->o.y, r->o.z};
    const float d[3] = {r->d.x, r->d.y, r->d.z};
    float t = (h->f[4] - o[k]) / d[k];
    if (t < t0 || t > t1) return 0;
    float x = o[i] + t * d[i];
    float y = o[j] + t * d[j];
    if (x < h->f[0] || x > h->f[1] || y < h->f[2] || y > h->f[3]) return 0;
    rec->u = (x - h->f[0]) / (h->f[1] - h->f[0]);
    rec->v = (y - h->f[2]) / (h->f[3] - h->f[2]);
    rec->t = t;
    rec->mat = h->a;
    rec->p = at(r, t);
    rec->n = normal;
    return 1;
}

/* hitableList.h:20-38 */
static int hit_list(ctx_t* cx, rng_t* g, const rtow_hitable* h, const ray_t* r, float tmin, float tmax,
                    hitrec* rec) {
    hitrec tmp;
    memset(&tmp, 0, sizeof tmp);
    int any = 0;
    double closest = tmax;
    cx->c.list_visits++;
    for (uint32_t i = 0; i < h->b; i++) {
        if (hit(cx, g, cx->s->refs[h->a + i], r, tmin, (float)closest, &tmp)) {
            any = 1;
            closest = tmp.t;
            *rec = tmp;
        }
    }
    return any;
}

/* constantMedium.h:26-74 */
static int hit_medium(ctx_t* cx, rng_t* g, const rtow_hitable* h, const ray_t* r, float tmin, float tmax,
                      hitrec* rec) {
    cx->c.medium_calls++;
    (void)unif(cx, g); /* the discarded `db` draw, constantMedium.h:27 */
    hitrec ra, rb;
    memset(&ra, 0, sizeof ra);
    memset(&rb, 0, sizeof rb);
    if (hit(cx, g, h->a, r, -FLT_MAX, FLT_MAX, &ra)) {
        if (hit(cx, g, h->a, r, (float)((double)ra.t + 0.0001), FLT_MAX, &rb)) {
            if (ra.t < tmin) ra.t = tmin;
            if (rb.t > tmax) rb.t = tmax;
            if (ra.t >= rb.t) return 0;
            if (ra.t < 0) ra.t = 0;
            float inside = (rb.t - ra.t) * len(r->d);
            float dist = (float)(-(1 / h->f[0]) * log(unif(cx, g)));
            if (dist < inside) {
                rec->t = ra.t + dist / len(r->d);
                rec->p = at(r, rec->t);
                rec->n = mk(1, 0, 0);
                rec->mat = h->b;
                return 1;
            }
        }
    }
    return 0;
}

static int hit(ctx_t* cx, rng_t* g, uint32_t idx, const ray_t* r, float tmin, float tmax, hitrec* rec) {
    const rtow_hitable* h = &cx->s->hitables[idx];
    switch (h->kind) {
    case RTOW_HIT_SPHERE:
        cx->c.sphere_tests++;
        return hit_sphere(h, r, tmin, tmax, rec);
    case RTOW_HIT_MOVING_SPHERE:
        cx->c.moving_sphere_tests++;
        return hit_moving_sphere(h, r, tmin, tmax, rec);
    case RTOW_HIT_RECT_XY:
        cx->c.rect_tests++;
        return hit_rect(h, 0, 1, 2, mk(0, 0, 1), r, tmin, tmax, rec);
    case RTOW_HIT_RECT_XZ:
        cx->c.rect_tests++;
        return hit_rect(h, 0, 2, 1, mk(0, 1, 0), r, tmin, tmax, rec);
    case RTOW_HIT_RECT_YZ:
        cx->c.rect_tests++;
        return hit_rect(h, 1, 2, 0, mk(1, 0, 0), r, tmin, tmax, rec);
    case RTOW_HIT_FLIP_NORMALS: /* hitable.h:28-36 */
        if (hit(cx, g, h->a, r, tmin, tmax, rec)) {
            rec->n = neg(rec->n);
            return 1;
        }
        return 0;
    case RTOW_HIT_TRANSLATE: { /* hitable.h:53-62 */
        ray_t moved = {sub(r->o, ld3(h->f)), r->d, r->time};
        if (hit(cx, g, h->a, &moved, tmin, tmax, rec)) {
            rec->p = add(rec->p, ld3(h->f));
            return 1;
        }
        return 0;
    }
    case RTOW_HIT_ROTATE_Y: { /* hitable.h:125-154 */
        float s = h->f[0], c = h->f[1];
        ray_t rr = *r;
        rr.o.x = c * r->o.x - s * r->o.z;
        rr.o.z = s * r->o.x + c * r->o.z;
        rr.d.x = c * r->d.x - s * r->d.z;
        rr.d.z = s * r->d.x + c * r->d.z;
        if (hit(cx, g, h->a, &rr, tmin, tmax, rec)) {
            v3 p = rec->p, n = rec->n;
            p.x = c * rec->p.x + s * rec->p.z;
            p.z = -s * rec->p.x + c * rec->p.z;
            n.x = c * rec->n.x + s * rec->n.z;
            n.z = -s * rec->n.x + c * rec->n.z;
            rec->p = p;
            rec->n = n;
            return 1;
        }
        return 0;
    }
    case RTOW_HIT_LIST:
        return hit_list(cx, g, h, r, tmin, tmax, rec);
    case RTOW_HIT_BOX: /* box.h:43-45 */
        return hit(cx, g, h->a, r, tmin, tmax, rec);
    case RTOW_HIT_BVH_NODE: { /* bvhNode.h:66-96 */
        cx->c.bvh_visits++;
        if (!aabb_hit(h->f, h->f + 3, r, tmin, tmax)) return 0;
        cx->c.bvh_box_pass++;
        hitrec lr, rr;
        memset(&lr, 0, sizeof lr);
        memset(&rr, 0, sizeof rr);
        int hl = hit(cx, g, h->a, r, tmin, tmax, &lr);
        int hr = hit(cx, g, h->b, r, tmin, tmax, &rr);
        if (hl && hr) {
            *rec = lr.t < rr.t ? lr : rr;
            return 1;
        }
        if (hl) { *rec = lr; return 1; }
        if (hr) { *rec = rr; return 1; }
        return 0;
    }
    case RTOW_HIT_CONSTANT_MEDIUM:
        return hit_medium(cx, g, h, r, tmin, tmax, rec);
    default:
        return 0;
    }
}

/* ---- textures (texture.h, noise.h) --------------------------------------- */

/* mathUtilities.h:41-60 */
static float perlin_interp(v3 c[2][2][2], float u, float v, float w) {
    float uu = u * u * (3 - 2 * u);
    float vv = v * v * (3 - 2 * v);
    float ww = w * w * (3 - 2 * w);
    float accum = 0;
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
            for (int k = 0; k < 2; k++) {
                v3 wt = mk(u - i, v - j, w - k);
                accum += (i * uu + (1 - i) * (1 - uu)) * (j * vv + (1 - j) * (1 - vv)) *
                         (k * ww + (1 - k) * (1 - ww)) * dot(c[i][j][k], wt);
            }
    return accum;
}

/* noise.h:11-36 (filter = true path; NoiseTexture::value always asks for it) */
static float perlin_noise(const rtow_perlin* pt, v3 p) {
    float u = p.x - floorf(p.x);
    float v = p.y - floorf(p.y);
    float w = p.z - floorf(p.z);
    int i = (int)floorf(p.x);
    int j = (int)floorf(p.y);
    int k = (int)floorf(p.z);
    v3 c[2][2][2];
    for (int di = 0; di < 2; di++)
        for (int dj = 0; dj < 2; dj++)
            for (int dk = 0; dk < 2; dk++) {
                int q = pt->perm_x[(i + di) & 255] ^ pt->perm_y[(j + dj) & 255] ^ pt->perm_z[(k + dk) & 255];
                c[di][dj][dk] = ld3(pt->ranvec[q]);
            }
    return perlin_interp(c, u, v, w);
}

/* noise.h:38-49 */
static float turbulence(const rtow_perlin* pt, v3 p) {
    float accum = 0;
    v3 tp = p;
    float weight = 1.0;
    for (int i = 0; i < 7; i++) {
        accum += weight * perlin_noise(pt, tp);
        weight *= 0.5;
        tp = scl(2.0f, tp);
    }
    return fabsf(accum);
}

static v3 tex_value(ctx_t* cx, uint32_t ti, float u, float v, v3 p) {
    const rtow_texture* t = &cx->s->textures[ti];
    switch (t->kind) {
    case RTOW_TEX_CONSTANT: /* texture.h:16-18 */
        return ld3(t->f);
    case RTOW_TEX_CHECKER: { /* texture.h:27-35 */
        float sines = sinf(10 * p.x) * sinf(10 * p.y) * sinf(10 * p.z);
        if (sines < 0) return tex_value(cx, t->a, u, v, p);
        return tex_value(cx, t->b, u, v, p);
    }
    case RTOW_TEX_NOISE: { /* texture.h:44-48 */
        float s = 1 + sinf(t->f[0] * p.z + 10 * turbulence(cx->s->perlin, p));
        return scl(s, mk(0.5f, 0.5f, 0.5f));
    }
    case RTOW_TEX_IMAGE: { /* texture.h:65-79 */
        const rtow_image* im = &cx->s->images[t->a];
        int nx = (int)im->nx, ny = (int)im->ny;
        const uint8_t* data = cx->s->texels + im->offset;
        int i = (int)(u * nx);
        int j = (int)((double)((1 - v) * ny) - 0.001);
        if (i < 0) i = 0;
        if (j < 0) j = 0;
        if (i > nx - 1) i = nx - 1;
        if (j > ny - 1) j = ny - 1;
        float r = (float)(data[3 * i + 3 * nx * j] / 255.0);
        float g = (float)(data[3 * i + 3 * nx * j + 1] / 255.0);
        float b = (float)(data[3 * i + 3 * nx * j + 2] / 255.0);
        return mk(r, g, b);
    }
    default:
        return mk(0, 0, 0);
    }
}

/* ---- materials (material.h) --------------------------------------------- */

static v3 reflect(v3 v, v3 n) { return sub(v, scl(2 * dot(v, n), n)); } /* material.h:11-13 */

/* material.h:15-26 */
static int refract(v3 d, v3 n, float ni, v3* out) {
    v3 uv = unit(d);
    float dt = dot(uv, n);
    float disc = (float)(1.0 - ni * ni * (1 - dt * dt));
    if (disc > 0) {
        *out = sub(scl(ni, sub(uv, scl(dt, n))), scl(sqrtf(disc), n));
        return 1;
    }
    return 0;
}

/* material.h:28-32 */
static float schlick(float cosine, float ri) {
    float r0 = (1 - ri) / (1 + ri);
    r0 = r0 * r0;
    return (float)(r0 + (1 - r0) * pow((double)(1 - cosine), 5.0));
}

static v3 emitted(ctx_t* cx, const rtow_material* m, const hitrec* rec) {
    if (m->kind == RTOW_MAT_DIFFUSE_LIGHT) /* material.h:130-132 */
        return tex_value(cx, m->texture, rec->u, rec->v, rec->p);
    return mk(0, 0, 0); /* material.h:38-40 */
}

static int scatter(ctx_t* cx, rng_t* g, const rtow_material* m, const ray_t* in, const hitrec* rec,
                   v3* atten, ray_t* out) {
    switch (m->kind) {
    case RTOW_MAT_LAMBERTIAN: { /* material.h:47-53 */
        v3 target = add(add(rec->p, rec->n), random_in_unit_sphere(cx, g));
        out->o = rec->p;
        out->d = sub(target, rec->p);
        out->time = in->time;
        *atten = tex_value(cx, m->texture, rec->u, rec->v, rec->p);
        return 1;
    }
    case RTOW_MAT_METAL: { /* material.h:62-67 */
        v3 reflected = reflect(unit(in->d), rec->n);
        out->o = rec->p;
        out->d = add(reflected, scl(m->param, random_in_unit_sphere(cx, g)));
        out->time = 0.0f;
        *atten = ld3(m->albedo);
        return dot(out->d, rec->n) > 0;
    }
    case RTOW_MAT_DIELECTRIC: { /* material.h:77-117 */
        v3 outward, refracted = mk(0, 0, 0);
        v3 reflected = reflect(in->d, rec->n);
        float ni, prob, cosine;
        float ri = m->param;
        *atten = mk(1.0f, 1.0f, 1.0f);
        if (dot(in->d, rec->n) > 0) {
            outward = neg(rec->n);
            ni = ri;
            cosine = ri * dot(in->d, rec->n) / len(in->d);
        } else {
            outward = rec->n;
            ni = (float)(1.0 / ri);
            cosine = -dot(in->d, rec->n) / len(in->d);
        }
        if (refract(in->d, outward, ni, &refracted)) {
            prob = schlick(cosine, ri);
        } else {
            prob = 1.0f;
        }
        out->o = rec->p;
        out->time = 0.0f;
        if (unif(cx, g) < prob)
            out->d = reflected;
        else
            out->d = refracted;
        return 1;
    }
    case RTOW_MAT_ISOTROPIC: { /* material.h:141-145 */
        out->o = rec->p;
        out->d = random_in_unit_sphere(cx, g);
        out->time = 0.0f;
        *atten = tex_value(cx, m->texture, rec->u, rec->v, rec->p);
        return 1;
    }
    default: /* DiffuseLight::scatter material.h:126-128 */
        return 0;
    }
}

/* ---- integrator (color.h:12-59) ------------------------------------------ */
static v3 color(ctx_t* cx, rng_t* g, const rtow_params* P, const ray_t* r, int depth) {
    hitrec rec;
    memset(&rec, 0, sizeof rec);
    cx->c.segments++;
    const int hit_any = hit(cx, g, cx->s->root, r, 0.001f, FLT_MAX, &rec);
    if (cx->rays && cx->rays_n < cx->rays_max) {
        float* o = cx->rays + (size_t)cx->rays_n * 7;
        o[0] = r->o.x, o[1] = r->o.y, o[2] = r->o.z;
        o[3] = r->d.x, o[4] = r->d.y, o[5] = r->d.z;
        o[6] = r->time;
        cx->rays_n++;
    }
    if (cx->trace && cx->trace_n < cx->trace_max) {
        float* o = cx->trace + (size_t)cx->trace_n * RTOW_DEBUG_SEG_FLOATS;
        o[0] = hit_any ? 1.0f : 0.0f;
        o[1] = (float)depth;
        o[2] = hit_any ? rec.t : 0.0f;
        o[3] = hit_any ? rec.p.x : r->d.x;
        o[4] = hit_any ? rec.p.y : r->d.y;
        o[5] = hit_any ? rec.p.z : r->d.z;
        o[6] = hit_any ? rec.n.x : 0.0f;
        o[7] = hit_any ? rec.n.y : 0.0f;
        o[8] = hit_any ? rec.n.z : 0.0f;
        o[9] = hit_any ? (float)rec.mat : -1.0f;
        o[10] = (float)g->ctr;
        o[11] = 1.0f;
        cx->trace_n++;
    }
    if (hit_any) {
        const rtow_material* m = &cx->s->materials[rec.mat];
        ray_t scattered;
        v3 atten;
        v3 e = emitted(cx, m, &rec);
        if (depth < (int)P->max_depth && scatter(cx, g, m, r, &rec, &atten, &scattered))
            return add(e, mulv(atten, color(cx, g, P, &scattered, depth + 1)));
        return e;
    }
    if (P->gi_enable) {
        if (depth < 1) {
            v3 ud = unit(r->d);
            float t = ud.z;
            float rt = (float)(1.0 + t), gt = (float)(1.0 + t), bt = (float)(1.0 + t);
            v3 sky = mk((float)(rt * 0.1), (float)(gt * 0.3), (float)(bt * 1.0));
            return scl(P->sky_gain, sky);
        }
        return mk(P->gi_gain, P->gi_gain, P->gi_gain);
    }
    return mk(0, 0, 0);
}

/* ---- render loop (main.cpp:932-996 + camera.h:123-135) ------------------- */
/* main.cpp:942-944 + Camera::getRay (camera.h:123-135): the sample's primary ray */
static ray_t camera_ray(ctx_t* cx, rng_t* gp, const rtow_camera* C, const rtow_params* P, int column, int row) {
    const uint32_t W = P->width, H = P->height;
    rng_t g = *gp;
    {
        float u = (float)(column + unif(cx, &g)) / (float)W;
        float v = (float)(row + unif(cx, &g)) / (float)H;
        /* camera.h:123-135: CAMERA_DOF_EN 0 (the reference default) or, with
         * RTOW_FLAG_CAMERA_DOF, CAMERA_DOF_EN 1 */
        float lr = C->lens_radius;
        v3 rd;
        if (P->flags & RTOW_FLAG_CAMERA_DOF) {
            /* camera.h:125: _lensRadius * randomInUnitDisk() + randomInUnitSphere();
             * g++ evaluates operator+'s arguments right to left: the sphere's
             * draws come first (pinned by the ref_harness_dof fixtures) */
            v3 sph = random_in_unit_sphere(cx, &g);
            v3 disk = random_in_unit_disk(cx, &g);
            rd = add(scl(lr, disk), sph);
        } else {
            rd = scl(lr, mk(1.0f, 1.0f, 1.0f));
        }
        v3 offset = add(scl(rd.x, ld3(C->u)), scl(rd.y, ld3(C->v)));
        float time = (float)(C->time0 + unif(cx, &g) * (double)(C->time1 - C->time0));
        ray_t r;
        r.o = add(ld3(C->origin), offset);
        r.d = sub(sub(add(add(ld3(C->lower_left_corner), scl(u, ld3(C->horizontal))), scl(v, ld3(C->vertical))),
                      ld3(C->origin)),
                  offset);
        r.time = time;
        *gp = g;
        return r;
    }
}

static v3 sample_color(ctx_t* cx, const rtow_camera* C, const rtow_params* P, int column, int row, uint32_t s) {
    const uint32_t W = P->width;
    {
        rng_t g;
        g.key = rtow_sample_key(P->seed, (uint32_t)row * W + (uint32_t)column, s);
        g.ctr = 0;
        uint64_t d0 = cx->c.draws;
        ray_t r = camera_ray(cx, &g, C, P, column, row);
        v3 c = color(cx, &g, P, &r, 0);
        cx->c.samples++;
        uint64_t nd = cx->c.draws - d0;
        if (nd > cx->c.max_draws_per_sample) cx->c.max_draws_per_sample = nd;
        return c;
    }
}

static v3 render_pixel(ctx_t* cx, const rtow_camera* C, const rtow_params* P, uint32_t fb_index) {
    const uint32_t W = P->width, H = P->height;
    uint32_t x = fb_index % W, y = fb_index / W;
    int column = (int)x, row = (int)(H - 1 - y);
    v3 out = mk(0, 0, 0);
    for (uint32_t s = 0; s < P->spp; s++) out = add(out, sample_color(cx, C, P, column, row, s));
    float k = (float)(1.0 / (float)P->spp); /* vec3.h:133-139 */
    return mk(out.x * k, out.y * k, out.z * k);
}

static void quantize(v3 c, uint8_t* px) { /* main.cpp:957-989 */
    float s[3] = {sqrtf(c.x), sqrtf(c.y), sqrtf(c.z)};
    uint8_t o[3];
    for (int i = 0; i < 3; i++) {
        double q = 255.99 * s[i];
        uint32_t v = q >= 65535.0 ? 65535u : (q > 0 ? (uint32_t)(uint16_t)q : 0u);
        o[i] = v > 255 ? 255 : (uint8_t)v;
    }
    px[0] = o[2];
    px[1] = o[1];
    px[2] = o[0];
    px[3] = 0;
}

typedef struct {
    const rtow_scene* s;
    const rtow_camera* cam;
    const rtow_params* p;
    const uint32_t* pixels;
    uint32_t n;
    int tid, nt;
    float* lin;
    uint8_t* bgra;
    rtow_oracle_counters c;
} job_t;

static void* worker(void* arg) {
    job_t* j = (job_t*)arg;
    ctx_t cx;
    memset(&cx, 0, sizeof cx);
    cx.s = j->s;
    for (uint32_t i = (uint32_t)j->tid; i < j->n; i += (uint32_t)j->nt) {
        uint32_t fb = j->pixels ? j->pixels[i] : i;
        v3 c = render_pixel(&cx, j->cam, j->p, fb);
        if (j->lin) {
            j->lin[3 * (size_t)i + 0] = c.x;
            j->lin[3 * (size_t)i + 1] = c.y;
            j->lin[3 * (size_t)i + 2] = c.z;
        }
        if (j->bgra) quantize(c, j->bgra + 4 * (size_t)i);
    }
    j->c = cx.c;
    return NULL;
}

static int validate(const rtow_scene* s, const rtow_params* p) {
    if (!s || !p || p->width == 0 || p->height == 0 || p->spp == 0) return RTOW_E_INVALID;
    if (s->root >= s->n_hitables || !s->perlin) return RTOW_E_INVALID;
    for (uint32_t i = 0; i < s->n_hitables; i++) {
        const rtow_hitable* h = &s->hitables[i];
        if (h->kind < RTOW_HIT_SPHERE || h->kind > RTOW_HIT_CONSTANT_MEDIUM) return RTOW_E_INVALID;
    }
    return 0;
}

int rtow_oracle_render_pixels(const rtow_scene* scene, const rtow_camera* cam, const rtow_params* p,
                              const uint32_t* pixels, uint32_t n_pixels, int threads, float* lin,
                              uint8_t* bgra, rtow_oracle_counters* counters) {
    int rc = validate(scene, p);
    if (rc) return rc;
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    job_t* jobs = (job_t*)calloc((size_t)threads, sizeof(job_t));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    if (!jobs || !th) { free(jobs); free(th); return RTOW_E_NOMEM; }
    for (int t = 0; t < threads; t++) {
        job_t j = {scene, cam, p, pixels, n_pixels, t, threads, lin, bgra, {0}};
        jobs[t] = j;
        if (threads > 1)
            pthread_create(&th[t], NULL, worker, &jobs[t]);
        else
            worker(&jobs[t]);
    }
    rtow_oracle_counters sum;
    memset(&sum, 0, sizeof sum);
    for (int t = 0; t < threads; t++) {
        if (threads > 1) pthread_join(th[t], NULL);
        const rtow_oracle_counters* c = &jobs[t].c;
        sum.samples += c->samples;
        sum.segments += c->segments;
        sum.bvh_visits += c->bvh_visits;
        sum.bvh_box_pass += c->bvh_box_pass;
        sum.sphere_tests += c->sphere_tests;
        sum.moving_sphere_tests += c->moving_sphere_tests;
        sum.rect_tests += c->rect_tests;
        sum.medium_calls += c->medium_calls;
        sum.list_visits += c->list_visits;
        sum.draws += c->draws;
        if (c->max_draws_per_sample > sum.max_draws_per_sample) sum.max_draws_per_sample = c->max_draws_per_sample;
    }
    if (counters) *counters = sum;
    free(jobs);
    free(th);
    return 0;
}

int rtow_oracle_render(const rtow_scene* scene, const rtow_camera* cam, const rtow_params* p, int threads,
                       float* lin, uint8_t* bgra, rtow_oracle_counters* counters) {
    if (!p) return RTOW_E_INVALID;
    return rtow_oracle_render_pixels(scene, cam, p, NULL, p->width * p->height, threads, lin, bgra,
                                     counters);
}

int rtow_oracle_trace_sample(const rtow_scene* scene, const rtow_camera* cam, const rtow_params* p, uint32_t x,
                             uint32_t y, uint32_t sample, float* out, uint32_t max_segments, uint32_t* n_segments) {
    int rc = validate(scene, p);
    if (rc) return rc;
    if (!cam || !out || x >= p->width || y >= p->height || sample >= p->spp) return RTOW_E_INVALID;
    ctx_t cx;
    memset(&cx, 0, sizeof cx);
    cx.s = scene;
    cx.trace = out;
    cx.trace_max = max_segments;
    (void)sample_color(&cx, cam, p, (int)x, (int)(p->height - 1 - y), sample);
    if (n_segments) *n_segments = cx.trace_n;
    return 0;
}

int rtow_oracle_trace_rays(const rtow_scene* scene, const rtow_camera* cam, const rtow_params* p, uint32_t x,
                           uint32_t y, uint32_t sample, float* out, uint32_t max_segments, uint32_t* n_segments) {
    int rc = validate(scene, p);
    if (rc) return rc;
    if (!cam || !out || x >= p->width || y >= p->height || sample >= p->spp) return RTOW_E_INVALID;
    ctx_t cx;
    memset(&cx, 0, sizeof cx);
    cx.s = scene;
    cx.rays = out;
    cx.rays_max = max_segments;
    (void)sample_color(&cx, cam, p, (int)x, (int)(p->height - 1 - y), sample);
    if (n_segments) *n_segments = cx.rays_n;
    return 0;
}

/* ---- scene file loader ("RTOWSCN1") ---------------------------- */
struct rtow_oracle_scene {
    rtow_scene view;
    void* blob;
};

int rtow_oracle_load(const char* path, rtow_oracle_scene** out) {
    FILE* f = fopen(path, "rb");
    if (!f) return RTOW_E_IO;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t* b = (uint8_t*)malloc((size_t)sz);
    if (!b) { fclose(f); return RTOW_E_NOMEM; }
    if (fread(b, 1, (size_t)sz, f) != (size_t)sz) { fclose(f); free(b); return RTOW_E_IO; }
    fclose(f);
    if (sz < 56 || memcmp(b, "RTOWSCN1", 8) != 0) { free(b); return RTOW_E_IO; }
    uint32_t hdr[10];
    uint64_t ntex;
    memcpy(hdr, b + 8, 40);
    memcpy(&ntex, b + 48, 8);
    rtow_oracle_scene* s = (rtow_oracle_scene*)calloc(1, sizeof *s);
    if (!s) { free(b); return RTOW_E_NOMEM; }
    s->blob = b;
    size_t off = 56;
    rtow_scene* v = &s->view;
    v->root = hdr[1];
    v->n_hitables = hdr[2];
    v->n_refs = hdr[3];
    v->n_materials = hdr[4];
    v->n_textures = hdr[5];
    v->n_images = hdr[6];
    v->n_texel_bytes = ntex;
    size_t need = off + (size_t)v->n_hitables * sizeof(rtow_hitable) + (size_t)v->n_refs * 4 +
                  (size_t)v->n_materials * sizeof(rtow_material) + (size_t)v->n_textures * sizeof(rtow_texture) +
                  (hdr[7] ? sizeof(rtow_perlin) : 0) + (size_t)v->n_images * sizeof(rtow_image) + ntex;
    if (need != (size_t)sz) { free(b); free(s); return RTOW_E_IO; }
    v->hitables = (const rtow_hitable*)(b + off); off += (size_t)v->n_hitables * sizeof(rtow_hitable);
    v->refs = (const uint32_t*)(b + off); off += (size_t)v->n_refs * 4;
    v->materials = (const rtow_material*)(b + off); off += (size_t)v->n_materials * sizeof(rtow_material);
    v->textures = (const rtow_texture*)(b + off); off += (size_t)v->n_textures * sizeof(rtow_texture);
    if (hdr[7]) { v->perlin = (const rtow_perlin*)(b + off); off += sizeof(rtow_perlin); }
    v->images = (const rtow_image*)(b + off); off += (size_t)v->n_images * sizeof(rtow_image);
    v->texels = b + off;
    *out = s;
    return 0;
}

const rtow_scene* rtow_oracle_view(const rtow_oracle_scene* s) { return s ? &s->view : NULL; }

void rtow_oracle_free(rtow_oracle_scene* s) {
    if (!s) return;
    free(s->blob);
    free(s);
}

/* The primary ray of one sample (column, row in the reference's numbering:
 * row 0 = the bottom image row), as the render loop computes it: origin xyz,
 * direction xyz, time.  Test infrastructure (tests/golden/make_graze_golden.py
 * builds a world around one exact ray). */
int rtow_oracle_camera_ray(const rtow_camera* cam, const rtow_params* p, uint32_t column, uint32_t row,
                           uint32_t sample, float* out7) {
    if (!cam || !p || !out7 || column >= p->width || row >= p->height) return RTOW_E_INVALID;
    ctx_t cx;
    memset(&cx, 0, sizeof cx);
    rng_t g;
    g.key = rtow_sample_key(p->seed, row * p->width + column, sample);
    g.ctr = 0;
    ray_t r = camera_ray(&cx, &g, cam, p, (int)column, (int)row);
    out7[0] = r.o.x, out7[1] = r.o.y, out7[2] = r.o.z;
    out7[3] = r.d.x, out7[4] = r.d.y, out7[5] = r.d.z;
    out7[6] = r.time;
    return 0;
}
