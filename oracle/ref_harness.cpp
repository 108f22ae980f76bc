// ref_harness.cpp — TEST INFRASTRUCTURE ONLY (builds into oracle/_ref/, never
// shipped, never linked into the product).
//
// Compiles the reference's own hot-path headers, unmodified, straight from
// /root/reference/rayTracingOneWeekend (-I on the g++ line, see Makefile) and
// uses them to produce the golden fixtures in tests/golden/:
//   * the scene graph the reference builds (scenes.h), flattened to the
//     rtow_scene layout of include/rtow.h by walking the reference objects;
//   * the camera basis (camera.h:315-342);
//   * rendered images: the loop of main.cpp:932-996 re-stated below (main.cpp
//     itself is Win32-only), calling the reference's Camera::getRay and color().
//
// The reference's RNG (rngs.h:9, one global std::mt19937_64 seeded from the
// clock) is replaced WITHOUT editing any reference file: `mt19937_64` is
// #defined to an engine that returns rtow_draw24(key, ctr++) << 40 from
// thread-local (key, ctr), so uniform_real_distribution<double> yields exactly
// r24 * 2^-24 (include/rtow_rng.h).  The loop sets key = rtow_sample_key(seed,
// row*W + column, sample), ctr = 0 before each sample's jitter draws.
//
// Usage:
//   ref_harness dump   <scene> <out.scn> [opts]
//   ref_harness camera <W> <H> <out.cam>
//   ref_harness decode <file.jpg> <out.img>   (stbi_load(path, .., 0): u32 nx, ny, n + pixels)
//   ref_harness camera_oriented <W> <H> <lookfrom xyz> <view xyz> <east xyz> <down xyz> <out.cam>
//   ref_harness render <scene> <W> <H> <spp> <out_prefix> [opts]
//   ref_harness bench  <scene> <W> <H> <spp> <pixels.u32> [opts]   (timing, JSON line)
//       --racy: render with the reference's own shared std::mt19937_64 (see g_racy)
//       writes <out_prefix>.lin (W*H*3 float32, framebuffer order) and
//       <out_prefix>.bgra (W*H*4 bytes, main.cpp:982-989)
// scenes: three_sphere | random_ned | cornell | cornell_smoke | final_ned
// opts:   --n N  --scene-seed S  --seed S  --threads T  --cwd DIR
// The scene stream seed is read from RTOW_SCENE_SEED (environment) because the
// Perlin tables are drawn during static initialisation (noise.h:112-116),
// before main() runs.

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <limits>
#include <map>
#include <memory>
#include <random>
#include <sstream>
#include <string>
#include <thread>
#include <vector>
#include <unistd.h>

#include "../include/rtow.h"
#include "../include/rtow_rng.h"

static uint64_t harness_env_scene_key() {
    const char* s = std::getenv("RTOW_SCENE_SEED");
    uint64_t seed = s ? std::strtoull(s, nullptr, 0) : 1ull;
    return rtow_scene_key(seed);
}

// `bench --racy`: the reference as written (rngs.h:9-11, main.cpp:942-943):
// every render thread draws from ONE std::mt19937_64, unsynchronised (a data
// race, as in the reference).  The real engine type is named before the
// #define below turns `mt19937_64` into the counter engine.
using RealMt64 = std::mt19937_64;
static RealMt64 g_shared_mt(5489u);
static bool g_racy = false;

struct CbEngine {
    using result_type = uint64_t;
    static constexpr uint64_t min() { return 0; }
    static constexpr uint64_t max() { return ~0ull; }
    static thread_local uint64_t key;
    static thread_local uint32_t ctr;
    static thread_local uint64_t total;
    uint64_t operator()() {
        ++total;
        if (g_racy) return g_shared_mt();
        return (uint64_t)rtow_draw24(key, ctr++) << 40;
    }
    void seed(uint64_t) {}
    template <class S> void seed(S&) {}
};
thread_local uint64_t CbEngine::key = harness_env_scene_key();
thread_local uint32_t CbEngine::ctr = 0;
thread_local uint64_t CbEngine::total = 0;
namespace std { using cbrng_engine = ::CbEngine; }
#define mt19937_64 cbrng_engine

// The camera basis is private (camera.h:352-379); the harness reads it.
#define private public
#define protected public
#include "defines.h"
#ifdef RTOW_HARNESS_DOF
// the ref_harness_dof build: camera.h:124-126 compiled with CAMERA_DOF_EN 1
// (defines.h is #pragma once, so this value is the one camera.h sees)
#undef CAMERA_DOF_EN
#define CAMERA_DOF_EN 1
#endif
#include "vec3.h"
#include "scenes.h"
#undef private
#undef protected

// ---------------------------------------------------------------------------
// Scene graph: the reference objects flattened by the product's own
// reference-side adapter (include/rtow_reference.hpp, compiled here in the
// reference's translation unit exactly as a main.cpp binding would compile
// it), written as an .scn file (the layout rtow_scene_save writes).
#include "../include/rtow_reference.hpp"

static void v3(float* d, const vec3& v) { d[0] = v.x(); d[1] = v.y(); d[2] = v.z(); }

static void writeScene(const char* path, const rtow_scene& s) {
    FILE* f = std::fopen(path, "wb");
    if (!f) { std::perror(path); std::exit(2); }
    uint32_t hdr[10] = {1u, s.root, s.n_hitables, s.n_refs, s.n_materials, s.n_textures, s.n_images, 1u, 0u, 0u};
    uint64_t ntex = s.n_texel_bytes;
    std::fwrite("RTOWSCN1", 1, 8, f);
    std::fwrite(hdr, 4, 10, f);
    std::fwrite(&ntex, 8, 1, f);
    std::fwrite(s.hitables, sizeof(rtow_hitable), s.n_hitables, f);
    std::fwrite(s.refs, 4, s.n_refs, f);
    std::fwrite(s.materials, sizeof(rtow_material), s.n_materials, f);
    std::fwrite(s.textures, sizeof(rtow_texture), s.n_textures, f);
    std::fwrite(s.perlin, sizeof(rtow_perlin), 1, f);
    std::fwrite(s.images, sizeof(rtow_image), s.n_images, f);
    std::fwrite(s.texels, 1, s.n_texel_bytes, f);
    std::fclose(f);
}

// ---------------------------------------------------------------------------
// Scene composition.  Scenes the reference provides are called directly;
// configurations BASELINE.json names but the reference has no function for are
// composed from reference classes and documented here.

// randomScene_NED with n other than its hard-coded 100 (scenes.h:124): the same
// construction, with every random draw sequenced explicitly in the order g++
// evaluates the reference's expressions (checked: at n = 100 this produces a
// scene graph byte-identical to the reference's own randomScene_NED()).
static double U() { return unifRand(randomNumberGenerator); }

static Hitable* randomSceneNedN(int n, bool* usedImage) {
    Hitable** list = new Hitable*[n + 1];
    Texture* checker = new CheckerTexture(new ConstantTexture(vec3(0.2, 0.2, 0.8)),
                                          new ConstantTexture(vec3(0.9, 0.9, 0.9)));
    Texture* perlin = new NoiseTexture(true, 8.0f);
    Material* emitterMat = new DiffuseLight(new ConstantTexture(vec3(20, 0, 0)));
    int nx = 0, ny = 0, nn = 0;
    unsigned char* texData = stbi_load("./input_images/1_earth_8k.jpg", &nx, &ny, &nn, 0);
    Material* imageMat = new Lambertian(new ImageTexture(texData, nx, ny));
    const float R = 1000.0f;
    const float zOff = -1 * R;
    list[0] = new Sphere(vec3(0, 0, 0), R, new Lambertian(perlin));
    int i = 1;
    const int xMod = 10, yMod = 10;
    int cx = xMod, cy = yMod;
    while (i < n - 3) {
        float choose = (float)U();
        double uy = U();  // g++ evaluates the vec3 constructor's arguments right to left
        double ux = U();
        vec3 center(cx * ux, cy * uy, zOff - 1);
        if ((center - vec3(4, 0.2, 0)).length() > 0.9) {
            if (choose < 0.8) {
                double up = U();
                list[i++] = new MovingSphere(center, center + vec3(0, 0.5 * up, 0), 0.0, 1.0, 0.2,
                                             new Lambertian(checker));
            } else if (choose < 0.95) {
                double az = U();  // albedo arguments right to left, then the fuzz
                double ay = U();
                double ax = U();
                double fz = U();
                list[i++] = new Sphere(center, 0.2,
                                       new Metal(vec3(0.5 * (1 + ax), 0.5 * (1 + ay), 0.5 * (1 + az)),
                                                 0.5 * (1 + fz)));
            } else {
                list[i++] = new Sphere(center, 0.5, new Dielectric(1.5));
            }
        }
        if (cx < xMod) cx++; else { cx = -xMod; cy++; }
        if (cy > yMod) cy = -yMod;
    }
    *usedImage = texData != nullptr;
    if (texData)
        list[i++] = new Sphere(vec3(20.0, 0.0, zOff - 25.0), 10.0, imageMat);
    else
        list[i++] = new Sphere(vec3(20.0, 0.0, zOff - 25.0), 10.0, new Dielectric(1.5));
    list[i++] = new Sphere(vec3(100, -70, zOff), 50.0, new Lambertian(perlin));
    list[i++] = new Sphere(vec3(100, 70, zOff), 50.0, new Metal(vec3(0.7, 0.6, 0.5), 0.0));
    list[i++] = new Sphere(vec3(0, 0, zOff - 500), 100.0, emitterMat);
    return new BvhNode(list, i, 0.0, 1.0);
}

// Config 1: "three-sphere lambertian scene" has no reference function; three
// Sphere + Lambertian(ConstantTexture) in a HitableList, NED frame, in view of
// the main.cpp camera (which looks down +x, main.cpp:111-125, camera.h:76-81).
static Hitable* threeSphereNed() {
    Hitable** list = new Hitable*[3];
    list[0] = new Sphere(vec3(10, 0, 101), 100, new Lambertian(new ConstantTexture(vec3(0.8, 0.8, 0.0))));
    list[1] = new Sphere(vec3(10, 0, 0), 1, new Lambertian(new ConstantTexture(vec3(0.1, 0.2, 0.5))));
    list[2] = new Sphere(vec3(10, -2.2, 0), 1, new Lambertian(new ConstantTexture(vec3(0.8, 0.3, 0.3))));
    return new HitableList(list, 3);
}

// Not a reference scene: ConstantMedium below a BvhNode (the reference allows
// it; its draws then follow BvhNode::hit's exhaustive both-children visit,
// bvhNode.h:66-96, with the caller's interval, and an n == 1 node calls its
// one leaf twice, bvhNode.h:38-39).  Built from the reference's classes in
// the frame of threeSphereNed (camera at the origin looking along +x).
static Hitable* mediumBvhNed() {
    Texture* white = new ConstantTexture(vec3(0.9, 0.9, 0.9));
    Texture* teal = new ConstantTexture(vec3(0.2, 0.8, 0.7));
    Hitable** items = new Hitable*[6];
    items[0] = new Sphere(vec3(10, 0, 0), 1, new Lambertian(new ConstantTexture(vec3(0.1, 0.2, 0.5))));
    items[1] = new ConstantMedium(new Sphere(vec3(10, -2.2, 0), 1, new Dielectric(1.5)), 0.8f, white);
    items[2] = new ConstantMedium(new Box(vec3(8, 1.5, -1), vec3(9.5, 3, 1), new Lambertian(white)), 0.5f, teal);
    items[3] = new Sphere(vec3(10, 2.2, -1.6), 0.5, new Metal(vec3(0.8, 0.8, 0.9), 0.1));
    items[4] = new ConstantMedium(new Sphere(vec3(12, 0, -2.5), 1.2, new Dielectric(1.5)), 0.3f, teal);
    items[5] = new ConstantMedium(new Sphere(vec3(9, -0.9, -1.3), 0.4, new Dielectric(1.5)), 2.0f, white);
    Hitable** list = new Hitable*[3];
    list[0] = new Sphere(vec3(10, 0, 101), 100, new Lambertian(new ConstantTexture(vec3(0.8, 0.8, 0.0))));
    list[1] = new BvhNode(items, 6, 0.0f, 1.0f);
    list[2] = new Sphere(vec3(7, 0.5, -4), 0.6, new DiffuseLight(new ConstantTexture(vec3(4, 4, 4))));
    return new HitableList(list, 3);
}

// Media the reference composes freely (constantMedium.h:26-31: the boundary is
// any Hitable; hitableList.h:24-34: a list hands each item its closest hit so
// far): a medium whose boundary is another medium, or a list holding one; and
// media below a BvhNode behind an instance or inside a list.
static Hitable* mediumNestedNed() {
    Texture* white = new ConstantTexture(vec3(0.9, 0.9, 0.9));
    Texture* teal = new ConstantTexture(vec3(0.2, 0.8, 0.7));
    Texture* rose = new ConstantTexture(vec3(0.9, 0.4, 0.5));
    Material* glass = new Dielectric(1.5);
    Hitable** list = new Hitable*[6];
    list[0] = new Sphere(vec3(10, 0, 101), 100, new Lambertian(new ConstantTexture(vec3(0.8, 0.8, 0.0))));
    // a medium whose boundary is a medium
    list[1] = new ConstantMedium(new ConstantMedium(new Sphere(vec3(10, -1.5, 0), 1.2, glass), 0.7f, white), 0.9f, teal);
    // a medium whose boundary is a list holding a sphere and a medium over a Box
    Hitable** inner = new Hitable*[2];
    inner[0] = new Sphere(vec3(10, 1.6, 0.2), 0.8, glass);
    inner[1] = new ConstantMedium(new Box(vec3(9.2, 1.2, -1.4), vec3(10.4, 2.8, -0.4), new Lambertian(white)), 1.5f, rose);
    list[2] = new ConstantMedium(new HitableList(inner, 2), 0.6f, white);
    list[3] = new Sphere(vec3(11, 0.2, -1.8), 0.6, new Metal(vec3(0.8, 0.8, 0.9), 0.1));
    list[4] = new Sphere(vec3(7, 0.5, -4), 0.6, new DiffuseLight(new ConstantTexture(vec3(4, 4, 4))));
    list[5] = new Sphere(vec3(12, -3, -1), 0.9, new Lambertian(new ConstantTexture(vec3(0.1, 0.2, 0.5))));
    return new HitableList(list, 6);
}

static Hitable* mediumBvhWrappedNed() {
    Texture* white = new ConstantTexture(vec3(0.9, 0.9, 0.9));
    Texture* teal = new ConstantTexture(vec3(0.2, 0.8, 0.7));
    Material* glass = new Dielectric(1.5);
    Hitable** items = new Hitable*[5];
    items[0] = new Sphere(vec3(10, 0, 0), 1, new Lambertian(new ConstantTexture(vec3(0.1, 0.2, 0.5))));
    // behind a Translate
    items[1] = new Translate(new ConstantMedium(new Sphere(vec3(0, 0, 0), 1, glass), 0.8f, white), vec3(10, -2.2, 0));
    // inside a list: handed the list's closest hit so far (hitableList.h:24-34)
    Hitable** l2 = new Hitable*[3];
    l2[0] = new Sphere(vec3(9.4, 2.0, 0.3), 0.5, new Metal(vec3(0.8, 0.8, 0.9), 0.1));
    l2[1] = new ConstantMedium(new Box(vec3(8, 1.5, -1), vec3(9.5, 3, 1), new Lambertian(white)), 0.5f, teal);
    l2[2] = new Sphere(vec3(10.5, 2.6, -0.8), 0.4, new Lambertian(new ConstantTexture(vec3(0.7, 0.3, 0.2))));
    items[2] = new HitableList(l2, 3);
    // behind a RotateY over a Translate
    items[3] = new RotateY(new Translate(new ConstantMedium(new Box(vec3(-0.6, -0.6, -0.6), vec3(0.6, 0.6, 0.6),
                                                                     new Lambertian(white)), 1.2f, teal),
                                         vec3(10.5, 0.8, -2.2)), 8);
    items[4] = new ConstantMedium(new Sphere(vec3(12, 0, -2.5), 1.2, glass), 0.3f, white);
    Hitable** list = new Hitable*[3];
    list[0] = new Sphere(vec3(10, 0, 101), 100, new Lambertian(new ConstantTexture(vec3(0.8, 0.8, 0.0))));
    list[1] = new BvhNode(items, 5, 0.0f, 1.0f);
    list[2] = new Sphere(vec3(7, 0.5, -4), 0.6, new DiffuseLight(new ConstantTexture(vec3(4, 4, 4))));
    return new HitableList(list, 3);
}

// An exact tie between a list item and a BvhNode item entered exactly at the
// tied t: the wall rectangle (item 0) and the near faces of two Boxes in a
// BvhNode (item 1) share the plane x = 10.  A ray through the overlap hits the
// wall at t*, then HitableList::hit asks the BvhNode with (tmin, t*)
// (hitableList.h:24-34); AABB::hit sees its box entered at exactly t* and
// returns `tmax <= tmin` (aabb.h:22-43), so the Boxes' faces -- which would
// take t == t* (closed interval, xy_rect.h) -- are never tested: the wall keeps
// the record.  A third Box sits in a BvhNode whose box starts before the
// plane (a sphere in front of it): there the face is tested and takes the tie.
static Hitable* tieBvhEntryNed() {
    Material* red = new Lambertian(new ConstantTexture(vec3(0.8, 0.1, 0.1)));
    Material* blue = new Lambertian(new ConstantTexture(vec3(0.1, 0.2, 0.8)));
    Material* green = new Lambertian(new ConstantTexture(vec3(0.1, 0.8, 0.2)));
    Hitable** boxes = new Hitable*[2];
    boxes[0] = new Box(vec3(10, -2.5, -1.5), vec3(11, -0.5, 0.5), blue);
    boxes[1] = new Box(vec3(10, 0.5, -1.5), vec3(11.5, 2.5, 0.5), blue);
    Hitable** front = new Hitable*[2];
    front[0] = new Box(vec3(10, -1.0, 0.8), vec3(11, 1.0, 2.0), green);
    front[1] = new Sphere(vec3(8.5, 3.0, 1.5), 0.3, green);
    Hitable** list = new Hitable*[5];
    list[0] = new YZRectangle(-3, 3, -2, 2.5, 10, red);
    list[1] = new BvhNode(boxes, 2, 0.0f, 1.0f);
    list[2] = new BvhNode(front, 2, 0.0f, 1.0f);
    list[3] = new Sphere(vec3(7, 0.5, -4), 0.6, new DiffuseLight(new ConstantTexture(vec3(4, 4, 4))));
    list[4] = new Sphere(vec3(10, 0, 101.5), 100, new Lambertian(new ConstantTexture(vec3(0.8, 0.8, 0.0))));
    return new HitableList(list, 5);
}

// Residual corner (i): one exact primary ray (tests/golden/make_graze_golden.py
// computes it with the oracle and writes the world's 14 parameters, C hex
// floats, to the file $RTOW_GRAZE_PARAMS) grazes the edge of a Box held by an
// n == 1 BvhNode: AABB::hit sees `tmax <= tmin` (aabb.h:22-43) and the Box's
// sides are never tested, although the side's rectangle (closed bounds,
// xy_rect.h) would take the edge point.  Behind it in the list a
// ConstantMedium whose boundary the ray enters beyond that point, then a
// sphere in front of both: the reference asks the medium with the whole
// interval and draws its scatter distance; a traversal that took the grazed
// side would hand the medium that side's t, skip the draw, and end at the
// same sphere with the stream one draw behind.
static Hitable* grazeMediumNed() {
    const char* path = std::getenv("RTOW_GRAZE_PARAMS");
    float q[14] = {};
    FILE* f = path ? std::fopen(path, "r") : nullptr;
    if (!f) { std::fprintf(stderr, "RTOW_GRAZE_PARAMS not readable\n"); std::exit(2); }
    for (int k = 0; k < 14; k++) {
        char buf[64];
        if (std::fscanf(f, "%63s", buf) != 1) { std::fprintf(stderr, "short graze params\n"); std::exit(2); }
        q[k] = std::strtof(buf, nullptr);
    }
    std::fclose(f);
    Material* blue = new Lambertian(new ConstantTexture(vec3(0.1, 0.2, 0.8)));
    Hitable** box = new Hitable*[1];
    box[0] = new Box(vec3(q[0], q[1], q[2]), vec3(q[3], q[4], q[5]), blue);
    Hitable** list = new Hitable*[4];
    list[0] = new BvhNode(box, 1, 0.0f, 1.0f);
    list[1] = new ConstantMedium(new Sphere(vec3(q[6], q[7], q[8]), q[9], new Dielectric(1.5)), 0.4f,
                                 new ConstantTexture(vec3(0.9, 0.9, 0.9)));
    list[2] = new Sphere(vec3(q[10], q[11], q[12]), q[13], new Lambertian(new ConstantTexture(vec3(0.8, 0.3, 0.2))));
    list[3] = new Sphere(vec3(q[0], q[1], q[2] - 40), 10, new DiffuseLight(new ConstantTexture(vec3(3, 3, 3))));
    return new HitableList(list, 4);
}

// Config 4: cornellBox_NED() with the smoke box that scenes.h:461-470 keeps
// commented out, inserted at the position that code occupies (after the
// rotated box, before the sphere medium).
static Hitable* cornellSmokeNed() {
    HitableList* l = dynamic_cast<HitableList*>(cornellBox_NED());
    Material* green = new Lambertian(new ConstantTexture(vec3(0.12, 0.95, 0.15)));
    Hitable* box = new Translate(new RotateY(new Box(vec3(0, 0, 0), vec3(160, 300, 160), green), -25),
                                 vec3(-100, -50, 200));
    Hitable* smoke = new ConstantMedium(box, 0.01, new ConstantTexture(vec3(0.2, 0.9, 0.4)));
    const uint32_t at = 9;  // 6 panels + 3 boxes precede it
    for (uint32_t k = l->_listSize; k > at; k--) l->_hitableList[k] = l->_hitableList[k - 1];
    l->_hitableList[at] = smoke;
    l->_listSize += 1;
    return l;
}

// Config 5: book 2's final scene ("The Next Week", final chapter) has no
// reference function; composed here from reference classes and transcribed to
// the reference's NED frame: NED (x north, y east, z down) = (book z, book x,
// -book y).  The book rotates its sphere cloud about its vertical axis, which
// is NED z, for which the reference has no class: RotateY (about NED y, the
// reference's only rotation) takes its place.  Every random draw is sequenced
// explicitly.  main.cpp-style root Translate puts the book's look-at point
// (278, 278, 0) straight ahead of the main camera, 600 units out.
static Hitable* finalSceneNed(bool* usedImage) {
    Hitable** list = new Hitable*[16];
    Hitable** boxes = new Hitable*[400];
    Hitable** cloud = new Hitable*[1000];
    Material* white = new Lambertian(new ConstantTexture(vec3(0.73, 0.73, 0.73)));
    Material* ground = new Lambertian(new ConstantTexture(vec3(0.48, 0.83, 0.53)));
    int b = 0;
    for (int i = 0; i < 20; i++) {
        for (int j = 0; j < 20; j++) {
            float w = 100;
            float x0 = -1000 + i * w;
            float z0 = -1000 + j * w;
            float x1 = x0 + w;
            float y1 = 100 * (U() + 0.01);
            float z1 = z0 + w;
            boxes[b++] = new Box(vec3(z0, x0, -y1), vec3(z1, x1, 0), ground);
        }
    }
    int l = 0;
    list[l++] = new BvhNode(boxes, b, 0, 1);
    Material* light = new DiffuseLight(new ConstantTexture(vec3(7, 7, 7)));
    list[l++] = new XYRectangle(147, 412, 123, 423, -554, light);
    vec3 center(200, 400, -400);
    list[l++] = new MovingSphere(center, center + vec3(0, 30, 0), 0, 1, 50,
                                 new Lambertian(new ConstantTexture(vec3(0.7, 0.3, 0.1))));
    list[l++] = new Sphere(vec3(45, 260, -150), 50, new Dielectric(1.5));
    list[l++] = new Sphere(vec3(145, 0, -150), 50, new Metal(vec3(0.8, 0.8, 0.9), 10.0));
    Hitable* boundary = new Sphere(vec3(145, 360, -150), 70, new Dielectric(1.5));
    list[l++] = boundary;
    list[l++] = new ConstantMedium(boundary, 0.2, new ConstantTexture(vec3(0.2, 0.4, 0.9)));
    boundary = new Sphere(vec3(0, 0, 0), 5000, new Dielectric(1.5));
    list[l++] = new ConstantMedium(boundary, 0.0001, new ConstantTexture(vec3(1.0, 1.0, 1.0)));
    int nx = 0, ny = 0, nn = 0;
    unsigned char* texData = stbi_load("./input_images/1_earth_8k.jpg", &nx, &ny, &nn, 0);
    *usedImage = texData != nullptr;
    Material* emat = texData ? (Material*)new Lambertian(new ImageTexture(texData, nx, ny))
                             : (Material*)new Dielectric(1.5);
    list[l++] = new Sphere(vec3(400, 400, -200), 100, emat);
    list[l++] = new Sphere(vec3(300, 220, -280), 80, new Lambertian(new NoiseTexture(true, 0.1f)));
    for (int j = 0; j < 1000; j++) {
        double bx = U();
        double by = U();
        double bz = U();
        cloud[j] = new Sphere(vec3(165 * bz, 165 * bx, -165 * by), 10, white);
    }
    list[l++] = new Translate(new RotateY(new BvhNode(cloud, 1000, 0.0, 1.0), 15), vec3(395, -100, -270));
    return new HitableList(list, l);
}

struct Opts {
    int n = 100;
    uint64_t seed = 1;
    int threads = 0;
    bool racy = false;
    int ranks = 0;  // dropin_multi: ranks over device 0 (0: every visible device once)
    std::string cwd;
};

static Hitable* buildWorld(const std::string& name, const Opts& o) {
    if (!o.cwd.empty() && chdir(o.cwd.c_str()) != 0) { std::perror("chdir"); std::exit(2); }
    // main.cpp:132 / 136 wrap the scene in a root Translate.
    if (name == "random_ned") {
        Hitable* s;
        if (o.n == 100) {
            s = randomScene_NED();
        } else {
            bool used;
            s = randomSceneNedN(o.n, &used);
        }
        return new Translate(s, vec3(0, 0, 1000));
    }
    if (name == "random_ned_restated") {  // for the n = 100 equivalence check only
        bool used;
        return new Translate(randomSceneNedN(o.n, &used), vec3(0, 0, 1000));
    }
    // the reference's non-NED builders, called directly (main.cpp selects the
    // NED ones, so no root Translate): scenes.h:29-120 loads
    // ./input_images/earth1300x1300.jpg relative to the working directory
    if (name == "random") return randomScene();
    if (name == "cornell_box") return cornellBox();
    if (name == "cornell") return new Translate(cornellBox_NED(), vec3(800, 0, 0));
    if (name == "cornell_smoke") return new Translate(cornellSmokeNed(), vec3(800, 0, 0));
    if (name == "three_sphere") return threeSphereNed();
    if (name == "medium_bvh") return mediumBvhNed();
    if (name == "medium_nested") return mediumNestedNed();
    if (name == "tie_bvh_entry") return tieBvhEntryNed();
    if (name == "graze_medium") return grazeMediumNed();
    if (name == "medium_bvh_wrapped") return mediumBvhWrappedNed();
    if (name == "final_ned") {
        bool used;
        return new Translate(finalSceneNed(&used), vec3(600, -278, 278));
    }
    std::fprintf(stderr, "unknown scene %s\n", name.c_str());
    std::exit(2);
}

// main.cpp:111-125
static Camera* mainCamera(uint32_t W, uint32_t H) {
    vec3 lookFrom(0, 0, 0), lookAt(1, 0, 0), worldUp(0, 0, -1);
    float distToFocus = 1000;
    float aperture = 2.0;
    float aspectRatio = float(W) / float(H);
    float vFoV = 60.0;
    std::streambuf* old = std::cout.rdbuf(nullptr);  // the constructor prints its basis
    Camera* c = new Camera(lookFrom, lookAt, worldUp, vFoV, aspectRatio, aperture, distToFocus, 0.0, 1.0);
    std::cout.rdbuf(old);
    return c;
}

// the camera's private basis (camera.h:352-379), read directly
static rtow_camera privateBasis(Camera* c) {
    rtow_camera rc{};
    v3(rc.origin, c->_origin);
    v3(rc.lower_left_corner, c->_lowerLeftCorner);
    v3(rc.horizontal, c->_horizontal);
    v3(rc.vertical, c->_vertical);
    v3(rc.u, c->_u);
    v3(rc.v, c->_v);
    v3(rc.w, c->_w);
    rc.lens_radius = c->_lensRadius;
    rc.time0 = c->_time0;
    rc.time1 = c->_time1;
    return rc;
}

// the main camera after the frame loop's updates (main.cpp:476/554, 624-628):
// setOrientationMatrix(rows view/east/down) + setLookFromPoint
static void orientCamera(Camera* c, const float* v) {
    mat4x4 m;
    m.m[0] = vec4(v[3], v[4], v[5], 0.0f);
    m.m[1] = vec4(v[6], v[7], v[8], 0.0f);
    m.m[2] = vec4(v[9], v[10], v[11], 0.0f);
    m.m[3] = vec4(0.0f, 0.0f, 0.0f, 1.0f);
    c->setOrientationMatrix(m);
    c->setLookFromPoint(vec3(v[0], v[1], v[2]));
}

static void writeCamera(const char* path, Camera* c) {
    const rtow_camera rc = privateBasis(c);
    FILE* f = std::fopen(path, "wb");
    if (!f) { std::perror(path); std::exit(2); }
    std::fwrite(&rc, sizeof(rc), 1, f);
    std::fclose(f);
}

// main.cpp:932-996, re-stated; thread id / count interleave columns as
// main.cpp:936 does.  Output in framebuffer order.
static void renderWorker(int id, int nthreads, Camera* cam, Hitable* world, uint32_t W, uint32_t H,
                         uint32_t spp, uint64_t seed, float* lin, uint8_t* bgra) {
    const uint32_t bytesPerPixel = 4;
    const uint32_t sizeInBytes = W * H * bytesPerPixel;
    for (int row = (int)H - 1; row >= 0; row--) {
        for (int i = 0; i < (int)W; i++) {
            int column = id + nthreads * i;
            if (column >= (int)W) break;
            vec3 outputColor(0, 0, 0);
            for (uint32_t sample = 0; sample < spp; sample++) {
                CbEngine::key = rtow_sample_key(seed, (uint32_t)row * W + (uint32_t)column, sample);
                CbEngine::ctr = 0;
                float u = (float)(column + unifRand(randomNumberGenerator)) / (float)W;
                float v = (float)(row + unifRand(randomNumberGenerator)) / (float)H;
                ray rayCast = cam->getRay(u, v);
                outputColor += color(rayCast, world, 0);
            }
            outputColor /= float(spp);
            uint32_t px = (H - 1 - (uint32_t)row) * W + (uint32_t)column;
            lin[3 * px + 0] = outputColor[0];
            lin[3 * px + 1] = outputColor[1];
            lin[3 * px + 2] = outputColor[2];
            outputColor = vec3(sqrt(outputColor[0]), sqrt(outputColor[1]), sqrt(outputColor[2]));
            uint16_t irO = uint16_t(255.99 * outputColor[0]);
            uint16_t igO = uint16_t(255.99 * outputColor[1]);
            uint16_t ibO = uint16_t(255.99 * outputColor[2]);
            uint8_t ir = irO > 255 ? 255 : uint8_t(irO);
            uint8_t ig = igO > 255 ? 255 : uint8_t(igO);
            uint8_t ib = ibO > 255 ? 255 : uint8_t(ibO);
            uint32_t rowIndex = row * W * bytesPerPixel;
            uint32_t columnIndex = (W * bytesPerPixel) - column * bytesPerPixel;
            uint32_t bufferIndex = sizeInBytes - (rowIndex + columnIndex);
            bgra[bufferIndex] = ib;
            bgra[bufferIndex + 1] = ig;
            bgra[bufferIndex + 2] = ir;
            bgra[bufferIndex + 3] = 0;
        }
    }
}

// `bench`: the same loop body over a list of framebuffer pixels (x + W*y,
// top-down, as the oracle's rtow_oracle_render_pixels takes them), T threads
// interleaving the list -- the reference's own code timed on a bounded
// sample of a frame (bench.py's cpu_baseline, kind "reference").
static void benchWorker(int id, int nthreads, Camera* cam, Hitable* world, uint32_t W, uint32_t H, uint32_t spp,
                        uint64_t seed, const std::vector<uint32_t>* pix, double* sum) {
    double acc = 0.0;
    for (size_t i = (size_t)id; i < pix->size(); i += (size_t)nthreads) {
        const uint32_t fb = (*pix)[i];
        const int column = (int)(fb % W), row = (int)(H - 1 - fb / W);
        vec3 outputColor(0, 0, 0);
        for (uint32_t sample = 0; sample < spp; sample++) {
            CbEngine::key = rtow_sample_key(seed, (uint32_t)row * W + (uint32_t)column, sample);
            CbEngine::ctr = 0;
            float u = (float)(column + unifRand(randomNumberGenerator)) / (float)W;
            float v = (float)(row + unifRand(randomNumberGenerator)) / (float)H;
            ray rayCast = cam->getRay(u, v);
            outputColor += color(rayCast, world, 0);
        }
        outputColor /= float(spp);
        acc += (double)outputColor[0] + (double)outputColor[1] + (double)outputColor[2];
    }
    *sum = acc;
}

static Opts parseOpts(int argc, char** argv, int first) {
    Opts o;
    for (int k = first; k < argc; k++) {
        std::string a = argv[k];
        auto next = [&]() -> const char* {
            if (k + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); }
            return argv[++k];
        };
        if (a == "--n") o.n = std::atoi(next());
        else if (a == "--seed") o.seed = std::strtoull(next(), nullptr, 0);
        else if (a == "--threads") o.threads = std::atoi(next());
        else if (a == "--cwd") o.cwd = next();
        else if (a == "--racy") o.racy = true;
        else if (a == "--ranks") o.ranks = std::atoi(next());
        else { std::fprintf(stderr, "unknown option %s\n", a.c_str()); std::exit(2); }
    }
    return o;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: see header\n");
        return 2;
    }
    std::string cmd = argv[1];
    if (cmd == "dump" && argc >= 4) {
        Opts o = parseOpts(argc, argv, 4);
        Hitable* world = buildWorld(argv[2], o);
        rtow_ref::World w(world);
        if (w.status() != RTOW_OK) { std::fprintf(stderr, "unknown object class\n"); return 3; }
        writeScene(argv[3], *w.view());
        std::printf("draws %llu hitables %u\n", (unsigned long long)CbEngine::total, w.view()->n_hitables);
        return 0;
    }
    if (cmd == "decode" && argc >= 4) {
        // the reference's own stb_image (scenes.h:26-27, stb_image.h v2.22)
        // on a file, as scenes.h:140 calls it: uint32 nx, ny, channels, then
        // the pixels (tests/golden/jpeg/make_jpeg_golden.py)
        int x = 0, y = 0, n = 0;
        unsigned char* px = stbi_load(argv[2], &x, &y, &n, 0);
        if (!px) { std::fprintf(stderr, "stbi_load: %s\n", stbi_failure_reason()); return 5; }
        FILE* f = std::fopen(argv[3], "wb");
        if (!f) { std::perror(argv[3]); return 2; }
        const uint32_t hdr[3] = {(uint32_t)x, (uint32_t)y, (uint32_t)n};
        std::fwrite(hdr, 4, 3, f);
        std::fwrite(px, 1, (size_t)x * y * n, f);
        std::fclose(f);
        stbi_image_free(px);
        return 0;
    }
    if (cmd == "camera" && argc >= 5) {
        Camera* c = mainCamera((uint32_t)std::atoi(argv[2]), (uint32_t)std::atoi(argv[3]));
        writeCamera(argv[4], c);
        return 0;
    }
    if (cmd == "camera_oriented" && argc >= 17) {
        // the main camera after the frame loop's updates (main.cpp:476/554,
        // 624-628): setOrientationMatrix(rows view/east/down) + setLookFromPoint
        Camera* c = mainCamera((uint32_t)std::atoi(argv[2]), (uint32_t)std::atoi(argv[3]));
        float v[12];
        for (int k = 0; k < 12; k++) v[k] = (float)std::atof(argv[4 + k]);
        orientCamera(c, v);
        writeCamera(argv[16], c);
        return 0;
    }
    if (cmd == "camera_euler" && argc >= 18) {
        // setCamera_Euler (camera.h:271-313), which the reference's setCamera()
        // compiles out (camera.h:344-350): lookFrom / lookAt / up, vfov,
        // aspect, aperture, focus distance, t0, t1 -- the constructor, then
        // the Euler basis on the same object (protected: public here)
        float v[15];
        for (int k = 0; k < 15; k++) v[k] = (float)std::atof(argv[2 + k]);
        std::streambuf* old = std::cout.rdbuf(nullptr);  // the constructor prints its basis
        Camera* c = new Camera(vec3(v[0], v[1], v[2]), vec3(v[3], v[4], v[5]), vec3(v[6], v[7], v[8]), v[9], v[10],
                               v[11], v[12], v[13], v[14]);
        std::cout.rdbuf(old);
        c->setCamera_Euler();
        writeCamera(argv[17], c);
        return 0;
    }
    if (cmd == "camera_check" && argc >= 16) {
        // rtow_ref::camera (public getters) against the private basis, for
        // the main camera and for it after the frame loop's updates
        Camera* c = mainCamera((uint32_t)std::atoi(argv[2]), (uint32_t)std::atoi(argv[3]));
        int bad = 0;
        for (int pass = 0; pass < 2; pass++) {
            if (pass == 1) {
                float v[12];
                for (int k = 0; k < 12; k++) v[k] = (float)std::atof(argv[4 + k]);
                orientCamera(c, v);
            }
            rtow_camera a{}, b = privateBasis(c);
            if (rtow_ref::camera(*c, &a) != RTOW_OK || std::memcmp(&a, &b, sizeof a) != 0) bad |= 1 << pass;
        }
        std::printf("camera_check %s\n", bad ? "DIFFERS" : "identical");
        return bad ? 1 : 0;
    }
    if (cmd == "render" && argc >= 7) {
        Opts o = parseOpts(argc, argv, 7);
        uint32_t W = (uint32_t)std::atoi(argv[3]), H = (uint32_t)std::atoi(argv[4]);
        uint32_t spp = (uint32_t)std::atoi(argv[5]);
        std::string prefix = argv[6];
        Hitable* world = buildWorld(argv[2], o);
        Camera* cam = mainCamera(W, H);
        std::vector<float> lin((size_t)W * H * 3, 0.0f);
        std::vector<uint8_t> bgra((size_t)W * H * 4, 0);
        int nt = o.threads > 0 ? o.threads : (int)std::thread::hardware_concurrency();
        std::vector<std::thread> ts;
        for (int t = 0; t < nt; t++)
            ts.emplace_back(renderWorker, t, nt, cam, world, W, H, spp, o.seed, lin.data(), bgra.data());
        for (auto& t : ts) t.join();
        FILE* f = std::fopen((prefix + ".lin").c_str(), "wb");
        std::fwrite(lin.data(), 4, lin.size(), f);
        std::fclose(f);
        f = std::fopen((prefix + ".bgra").c_str(), "wb");
        std::fwrite(bgra.data(), 1, bgra.size(), f);
        std::fclose(f);
        return 0;
    }
    if (cmd == "bench" && argc >= 7) {
        Opts o = parseOpts(argc, argv, 7);
        uint32_t W = (uint32_t)std::atoi(argv[3]), H = (uint32_t)std::atoi(argv[4]);
        uint32_t spp = (uint32_t)std::atoi(argv[5]);
        std::vector<uint32_t> pix;
        {
            FILE* f = std::fopen(argv[6], "rb");
            if (!f) { std::perror("pixels"); return 2; }
            uint32_t v;
            while (std::fread(&v, 4, 1, f) == 1)
                if (v < W * H) pix.push_back(v);
            std::fclose(f);
        }
        Hitable* world = buildWorld(argv[2], o);
        Camera* cam = mainCamera(W, H);
        int nt = o.threads > 0 ? o.threads : (int)std::thread::hardware_concurrency();
        std::vector<double> sums((size_t)nt, 0.0);
        g_racy = o.racy;  // the scene is built; the render draws from the shared engine
        std::vector<std::thread> ts;
        auto t0 = std::chrono::steady_clock::now();
        for (int t = 0; t < nt; t++)
            ts.emplace_back(benchWorker, t, nt, cam, world, W, H, spp, o.seed, &pix, &sums[(size_t)t]);
        for (auto& t : ts) t.join();
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        double sum = 0.0;
        for (double x : sums) sum += x;
        std::printf("{\"seconds\": %.6f, \"pixels\": %zu, \"samples\": %llu, \"threads\": %d, \"checksum\": %.9g, "
                    "\"racy\": %s}\n",
                    sec, pix.size(), (unsigned long long)pix.size() * spp, nt, sum, o.racy ? "true" : "false");
        return 0;
    }
#ifdef RTOW_HARNESS_DROPIN
    if (cmd == "dropin" && argc >= 7) {
        // The drop-in as a main.cpp binding would do it: the
        // reference builds its world and camera (main.cpp:111-137),
        // rtow_reference.hpp flattens both, librtow_hip.so renders the frame
        // main.cpp:932-996 would have rendered.  Writes <prefix>.bgra/.lin.
        Opts o = parseOpts(argc, argv, 7);
        uint32_t W = (uint32_t)std::atoi(argv[3]), H = (uint32_t)std::atoi(argv[4]);
        uint32_t spp = (uint32_t)std::atoi(argv[5]);
        std::string prefix = argv[6];
        Hitable* world = buildWorld(argv[2], o);
        Camera* cam = mainCamera(W, H);
        rtow_ref::World w(world);
        rtow_camera rc;
        if (w.status() != RTOW_OK || rtow_ref::camera(*cam, &rc) != RTOW_OK) return 3;
        rtow_context* ctx = nullptr;
        int rc2 = rtow_context_create(0, &ctx);
        if (rc2 == RTOW_OK) rc2 = rtow_scene_upload(ctx, w.view());
        rtow_params p;
        rtow_ref::params(W, H, spp, &p);  // this build's defines.h
        p.seed = o.seed;
        std::vector<uint8_t> bgra((size_t)W * H * 4);
        std::vector<float> lin((size_t)W * H * 3);
        rtow_stats st{};
        if (rc2 == RTOW_OK) rc2 = rtow_render(ctx, &rc, &p, bgra.data(), lin.data(), &st);
        if (rc2 != RTOW_OK) {
            std::fprintf(stderr, "dropin: %s (%s)\n", rtow_error_string(rc2), rtow_last_error());
            return 4;
        }
        rtow_context_destroy(ctx);
        FILE* f = std::fopen((prefix + ".lin").c_str(), "wb");
        std::fwrite(lin.data(), 4, lin.size(), f);
        std::fclose(f);
        f = std::fopen((prefix + ".bgra").c_str(), "wb");
        std::fwrite(bgra.data(), 1, bgra.size(), f);
        std::fclose(f);
        std::printf("{\"segments\": %llu, \"samples\": %llu, \"kernel_ms\": %.3f}\n",
                    (unsigned long long)st.segments, (unsigned long long)st.samples, st.kernel_ms);
        return 0;
    }
    if (cmd == "dropin_multi" && argc >= 7) {
        // The multi-GPU binding of INTEGRATION.md, in the reference's own TU:
        // every visible device renders its share of the frame main.cpp's N
        // worker threads would have split by columns (main.cpp:182-195, 936),
        // one RCCL gather, the frame assembled on device 0 (rtow_render_devices).
        // --ranks k instead lists device 0 k times (ranks sharing one device,
        // gathered by device copies).  Prints which librccl the process loaded.
        Opts o = parseOpts(argc, argv, 7);
        uint32_t W = (uint32_t)std::atoi(argv[3]), H = (uint32_t)std::atoi(argv[4]);
        uint32_t spp = (uint32_t)std::atoi(argv[5]);
        std::string prefix = argv[6];
        Hitable* world = buildWorld(argv[2], o);
        Camera* cam = mainCamera(W, H);
        rtow_ref::World w(world);
        rtow_camera rc;
        if (w.status() != RTOW_OK || rtow_ref::camera(*cam, &rc) != RTOW_OK) return 3;
        int count = 0;
        if (rtow_device_count(&count) != RTOW_OK || count < 1) {
            std::fprintf(stderr, "dropin_multi: no device (%s)\n", rtow_last_error());
            return 4;
        }
        std::vector<int> devices;
        if (o.ranks > 0) devices.assign((size_t)o.ranks, 0);
        else for (int d = 0; d < count; d++) devices.push_back(d);
        rtow_params p;
        rtow_ref::params(W, H, spp, &p);
        p.seed = o.seed;
        std::vector<uint8_t> bgra((size_t)W * H * 4);
        std::vector<float> lin((size_t)W * H * 3);
        rtow_stats st{};
        int rc2 = rtow_render_devices(devices.data(), (uint32_t)devices.size(), w.view(), &rc, &p, bgra.data(),
                                      lin.data(), &st);
        if (rc2 != RTOW_OK) {
            std::fprintf(stderr, "dropin_multi: %s (%s)\n", rtow_error_string(rc2), rtow_last_error());
            return 4;
        }
        std::string rccl = "none";
        if (FILE* maps = std::fopen("/proc/self/maps", "r")) {
            char line[4096];
            while (std::fgets(line, sizeof line, maps))
                if (const char* q = std::strstr(line, "/librccl.so")) {
                    const char* b = std::strchr(line, '/');
                    rccl.assign(b, q + std::strlen("/librccl.so") - b);
                    break;
                }
            std::fclose(maps);
        }
        FILE* f = std::fopen((prefix + ".lin").c_str(), "wb");
        std::fwrite(lin.data(), 4, lin.size(), f);
        std::fclose(f);
        f = std::fopen((prefix + ".bgra").c_str(), "wb");
        std::fwrite(bgra.data(), 1, bgra.size(), f);
        std::fclose(f);
        std::printf("{\"segments\": %llu, \"samples\": %llu, \"kernel_ms\": %.3f, \"total_ms\": %.3f, "
                    "\"ranks\": %zu, \"devices_visible\": %d, \"librccl\": \"%s\"}\n",
                    (unsigned long long)st.segments, (unsigned long long)st.samples, st.kernel_ms, st.total_ms,
                    devices.size(), count, rccl.c_str());
        return 0;
    }
#endif
    std::fprintf(stderr, "bad command\n");
    return 2;
}
