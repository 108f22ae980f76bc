/*
 * rtow_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * A CPU restatement, in plain C, of the reference's render path
 * (main.cpp:932-996 -> Camera::getRay camera.h:123-135 -> color() color.h:12-59
 * -> Hitable::hit / Material::scatter / Texture::value), evaluated over the
 * flattened scene graph of include/rtow.h.  It keeps the reference's own
 * traversal (BvhNode tests both children with the same interval, lists scan
 * in order, ConstantMedium draws on every call) and its float/double
 * expression shapes, so it reproduces the compiled reference bit for bit
 * (pinned by tests/golden, generated from the reference itself by
 * oracle/_ref/ref_harness).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
 * it, and only as the checker / CPU baseline; the product never links it.
 */
#ifndef RTOW_ORACLE_H
#define RTOW_ORACLE_H

#include <stdint.h>
#include "../include/rtow.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Traversal counters, summed over all samples rendered. */
typedef struct rtow_oracle_counters {
    uint64_t samples;
    uint64_t segments;       /* color() calls */
    uint64_t bvh_visits;     /* BvhNode::hit calls */
    uint64_t bvh_box_pass;   /* ... whose AABB test passed */
    uint64_t sphere_tests;
    uint64_t moving_sphere_tests;
    uint64_t rect_tests;
    uint64_t medium_calls;
    uint64_t list_visits;
    uint64_t draws;          /* random numbers consumed */
    uint64_t max_draws_per_sample;
} rtow_oracle_counters;

typedef struct rtow_oracle_scene rtow_oracle_scene;

/* Load an "RTOWSCN1" scene file (format: DESIGN.md). */
int rtow_oracle_load(const char* path, rtow_oracle_scene** out);
const rtow_scene* rtow_oracle_view(const rtow_oracle_scene* s);
void rtow_oracle_free(rtow_oracle_scene* s);

/* Render the listed framebuffer pixels (index = y*W + x, y = 0 the TOP row,
 * i.e. reference row H-1-y).  lin receives 3 floats per listed pixel (the
 * average before sqrt), bgra (may be NULL) 4 bytes per listed pixel.  Pixels
 * are split over `threads` std threads by index modulo.  Returns 0 or <0. */
int rtow_oracle_render_pixels(const rtow_scene* scene, const rtow_camera* cam, const rtow_params* p,
                              const uint32_t* pixels, uint32_t n_pixels, int threads,
                              float* lin, uint8_t* bgra, rtow_oracle_counters* counters);

/* Whole frame, framebuffer order: lin W*H*3, bgra W*H*4 (either may be NULL). */
int rtow_oracle_render(const rtow_scene* scene, const rtow_camera* cam, const rtow_params* p,
                       int threads, float* lin, uint8_t* bgra, rtow_oracle_counters* counters);
/* The primary ray of one sample: origin xyz, direction xyz, time. */
int rtow_oracle_camera_ray(const rtow_camera* cam, const rtow_params* p, uint32_t column, uint32_t row,
                           uint32_t sample, float* out7);

/* The path of one sample (pixel x, y of the top-down frame): per color() call
 * RTOW_DEBUG_SEG_FLOATS floats, the records rtow_debug_trace_sample writes. */
int rtow_oracle_trace_sample(const rtow_scene* scene, const rtow_camera* cam, const rtow_params* p, uint32_t x,
                             uint32_t y, uint32_t sample, float* out, uint32_t max_segments, uint32_t* n_segments);
/* The rays of the same sample's color() calls (world frame, in call order):
 * 7 floats each, origin xyz, direction xyz, time -- the rays the device's
 * traversal is handed (tools/regroup_emulate.py prices traversal orders on
 * them). */
int rtow_oracle_trace_rays(const rtow_scene* scene, const rtow_camera* cam, const rtow_params* p, uint32_t x,
                           uint32_t y, uint32_t sample, float* out, uint32_t max_segments, uint32_t* n_segments);

#ifdef __cplusplus
}
#endif

#endif
