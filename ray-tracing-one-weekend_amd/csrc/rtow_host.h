// rtow_host.h — host-side C++ API of the MI355X path tracer.
//
// Mirrors the reference's scene-description interfaces so code that builds a
// world for the reference builds one for this renderer unchanged:
//   vec3 / ray                           vec3.h, ray.h
//   AABB, surroundingBox                 aabb.h:11-79
//   Hitable::boundingBox                 hitable.h:19-23
//   Sphere, MovingSphere                 sphere.h
//   XYRectangle, XZRectangle, YZRectangle xy_rect.h
//   FlipNormals, Translate, RotateY      hitable.h:25-154
//   HitableList, Box, BvhNode            hitableList.h, box.h, bvhNode.h
//   ConstantMedium                       constantMedium.h
//   Lambertian, Metal, Dielectric, DiffuseLight, Isotropic   material.h
//   ConstantTexture, CheckerTexture, NoiseTexture, ImageTexture  texture.h
//   Perlin tables                        noise.h:51-116
//   Camera (ctor, getters, basis)        camera.h
//   randomScene_NED, cornellBox_NED      scenes.h
// The classes describe the scene; hit/scatter/value run on the GPU (the
// device kernels in rtow_device.hip), reached through rtow_render() after the
// world is flattened (flattenWorld) into the rtow_scene arrays of
// include/rtow.h.  Objects live in an Arena (the reference leaks them).
//
// Scene construction consumes the counter-based scene stream
// (include/rtow_rng.h) in exactly the reference's draw order, so a world built
// here is byte-identical, once flattened, to the one the reference builds
// (tests/test_scene_graph.py checks this against tests/golden).
#pragma once

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <memory>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/rtow.h"
#include "../../include/rtow_rng.h"

namespace rtow {

// ---- math ---------------------------------------------------------------
struct vec3 {
    float e[3];
    vec3() : e{0, 0, 0} {}
    vec3(float a, float b, float c) : e{a, b, c} {}
    float x() const { return e[0]; }
    float y() const { return e[1]; }
    float z() const { return e[2]; }
    float operator[](int i) const { return e[i]; }
    float& operator[](int i) { return e[i]; }
    float length() const { return std::sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]); }
    float squared_length() const { return e[0] * e[0] + e[1] * e[1] + e[2] * e[2]; }
};
inline vec3 operator+(const vec3& a, const vec3& b) { return vec3(a.e[0] + b.e[0], a.e[1] + b.e[1], a.e[2] + b.e[2]); }
inline vec3 operator-(const vec3& a, const vec3& b) { return vec3(a.e[0] - b.e[0], a.e[1] - b.e[1], a.e[2] - b.e[2]); }
inline vec3 operator-(const vec3& a) { return vec3(-a.e[0], -a.e[1], -a.e[2]); }
inline vec3 operator*(float t, const vec3& v) { return vec3(t * v.e[0], t * v.e[1], t * v.e[2]); }
inline vec3 operator*(const vec3& v, float t) { return vec3(t * v.e[0], t * v.e[1], t * v.e[2]); }
inline vec3 operator/(const vec3& v, float t) { return vec3(v.e[0] / t, v.e[1] / t, v.e[2] / t); }
inline float dot(const vec3& a, const vec3& b) { return a.e[0] * b.e[0] + a.e[1] * b.e[1] + a.e[2] * b.e[2]; }
inline vec3 cross(const vec3& v1, const vec3& v2) {  // vec3.h:90-96
    return vec3((v1.e[1] * v2.e[2] - v1.e[2] * v2.e[1]), (-(v1.e[0] * v2.e[2] - v1.e[2] * v2.e[0])),
                (v1.e[0] * v2.e[1] - v1.e[1] * v2.e[0]));
}
inline vec3 unit_vector(const vec3& v) {  // vec3.h:141-148
    if (v.length() == 0.0) return vec3(0, 0, 0);
    return v / v.length();
}

struct ray {
    vec3 _a, _b;
    float _time = 0;
    ray() {}
    ray(const vec3& a, const vec3& b, float t = 0.0f) : _a(a), _b(b), _time(t) {}
    vec3 origin() const { return _a; }
    vec3 direction() const { return _b; }
    float time() const { return _time; }
    vec3 pointAtParameter(float t) const { return _a + t * _b; }
};

struct AABB {
    vec3 _min, _max;
    AABB() {}
    AABB(const vec3& a, const vec3& b) : _min(a), _max(b) {}
    vec3 min() const { return _min; }
    vec3 max() const { return _max; }
};
AABB surroundingBox(const AABB& a, const AABB& b);  // aabb.h:66-79

// ---- scene stream ---------------------------------------------------------
// The reference's global engine + unifRand (rngs.h:9-11), as one counter
// stream per scene build.
class SceneRng {
public:
    explicit SceneRng(uint64_t sceneSeed) : _key(rtow_scene_key(sceneSeed)) {}
    double operator()() { return (double)rtow_draw24(_key, _ctr++) * (1.0 / 16777216.0); }
    uint32_t draws() const { return _ctr; }

private:
    uint64_t _key;
    uint32_t _ctr = 0;
};

class Arena;
class GraphWriter;

// ---- textures --------------------------------------------------------------
class Texture {
public:
    virtual ~Texture() = default;
    virtual uint32_t flatten(GraphWriter& w) const = 0;
};
class ConstantTexture : public Texture {
public:
    explicit ConstantTexture(vec3 c) : _color(c) {}
    uint32_t flatten(GraphWriter& w) const override;
    vec3 _color;
};
class CheckerTexture : public Texture {
public:
    CheckerTexture(Texture* even, Texture* odd) : _odd(odd), _even(even) {}
    uint32_t flatten(GraphWriter& w) const override;
    Texture* _odd;
    Texture* _even;
};
class NoiseTexture : public Texture {  // uses the global Perlin tables
public:
    NoiseTexture(bool filter, float scale) : _scaled(scale), _filter(filter) {}
    uint32_t flatten(GraphWriter& w) const override;
    float _scaled;
    bool _filter;
};
// Image data as stbi_load returns it: nx*ny*3 RGB bytes.  Not owned.
class ImageTexture : public Texture {
public:
    ImageTexture(const unsigned char* pixels, int nx, int ny) : _data(pixels), _nx(nx), _ny(ny) {}
    uint32_t flatten(GraphWriter& w) const override;
    const unsigned char* _data;
    int _nx, _ny;
};

// Perlin tables (noise.h:51-116), drawn from the scene stream in the order the
// reference's static initialisers run (randFloat, randVector, permX/Y/Z).
struct PerlinTables {
    rtow_perlin t;
    void generate(SceneRng& rng);
};

// ---- materials -------------------------------------------------------------
class Material {
public:
    virtual ~Material() = default;
    virtual uint32_t flatten(GraphWriter& w) const = 0;
};
class Lambertian : public Material {
public:
    explicit Lambertian(Texture* a) : _albedo(a) {}
    uint32_t flatten(GraphWriter& w) const override;
    Texture* _albedo;
};
class Metal : public Material {
public:
    Metal(const vec3& a, float f) : _albedo(a), _fuzz(f < 1 ? f : 1) {}  // material.h:60
    uint32_t flatten(GraphWriter& w) const override;
    vec3 _albedo;
    float _fuzz;
};
class Dielectric : public Material {
public:
    explicit Dielectric(float ri) : _refIndex(ri) {}
    uint32_t flatten(GraphWriter& w) const override;
    float _refIndex;
};
class DiffuseLight : public Material {
public:
    explicit DiffuseLight(Texture* a) : _emit(a) {}
    uint32_t flatten(GraphWriter& w) const override;
    Texture* _emit;
};
class Isotropic : public Material {
public:
    explicit Isotropic(Texture* a) : _albedo(a) {}
    uint32_t flatten(GraphWriter& w) const override;
    Texture* _albedo;
};

// ---- hitables --------------------------------------------------------------
class Hitable {
public:
    virtual ~Hitable() = default;
    virtual bool boundingBox(float t0, float t1, AABB& box) const = 0;
    virtual uint32_t flatten(GraphWriter& w) const = 0;
};

class Sphere : public Hitable {
public:
    Sphere(vec3 c, float r, Material* m) : _center(c), _radius(r), _materialPointer(m) {}
    bool boundingBox(float, float, AABB& box) const override;
    uint32_t flatten(GraphWriter& w) const override;
    vec3 _center;
    float _radius;
    Material* _materialPointer;
};
class MovingSphere : public Hitable {
public:
    MovingSphere(vec3 c0, vec3 c1, float t0, float t1, float r, Material* m)
        : _center0(c0), _center1(c1), _time0(t0), _time1(t1), _radius(r), _materialPointer(m) {}
    bool boundingBox(float, float, AABB& box) const override;
    uint32_t flatten(GraphWriter& w) const override;
    vec3 center(float time) const;
    vec3 _center0, _center1;
    float _time0, _time1, _radius;
    Material* _materialPointer;
};

// XY (axis 2), XZ (axis 1), YZ (axis 0) rectangles share one shape.
class AxisRectangle : public Hitable {
public:
    AxisRectangle(uint32_t kind, float a0, float a1, float b0, float b1, float k, Material* m)
        : _kind(kind), _a0(a0), _a1(a1), _b0(b0), _b1(b1), _k(k), _material(m) {}
    bool boundingBox(float, float, AABB& box) const override;
    uint32_t flatten(GraphWriter& w) const override;
    uint32_t _kind;
    float _a0, _a1, _b0, _b1, _k;
    Material* _material;
};
class XYRectangle : public AxisRectangle {
public:
    XYRectangle(float x0, float x1, float y0, float y1, float k, Material* m)
        : AxisRectangle(RTOW_HIT_RECT_XY, x0, x1, y0, y1, k, m) {}
};
class XZRectangle : public AxisRectangle {
public:
    XZRectangle(float x0, float x1, float z0, float z1, float k, Material* m)
        : AxisRectangle(RTOW_HIT_RECT_XZ, x0, x1, z0, z1, k, m) {}
};
class YZRectangle : public AxisRectangle {
public:
    YZRectangle(float y0, float y1, float z0, float z1, float k, Material* m)
        : AxisRectangle(RTOW_HIT_RECT_YZ, y0, y1, z0, z1, k, m) {}
};

class FlipNormals : public Hitable {
public:
    explicit FlipNormals(Hitable* h) : _hitable(h) {}
    bool boundingBox(float t0, float t1, AABB& box) const override { return _hitable->boundingBox(t0, t1, box); }
    uint32_t flatten(GraphWriter& w) const override;
    Hitable* _hitable;
};
class Translate : public Hitable {
public:
    Translate(Hitable* h, const vec3& offset) : _hitablePointer(h), _offset(offset) {}
    bool boundingBox(float t0, float t1, AABB& box) const override;
    uint32_t flatten(GraphWriter& w) const override;
    Hitable* _hitablePointer;
    vec3 _offset;
};
class RotateY : public Hitable {
public:
    RotateY(Hitable* h, float angle);
    bool boundingBox(float, float, AABB& box) const override {
        box = _boundBox;
        return _hasBox;
    }
    uint32_t flatten(GraphWriter& w) const override;
    Hitable* _pointer;
    float _sinTheta, _cosTheta;
    bool _hasBox;
    AABB _boundBox;
};
class HitableList : public Hitable {
public:
    HitableList(Hitable** list, uint32_t n) : _hitableList(list, list + n) {}
    explicit HitableList(std::vector<Hitable*> list) : _hitableList(std::move(list)) {}
    bool boundingBox(float t0, float t1, AABB& box) const override;
    uint32_t flatten(GraphWriter& w) const override;
    std::vector<Hitable*> _hitableList;
};
class Box : public Hitable {
public:
    Box(Arena& arena, const vec3& p0, const vec3& p1, Material* m);
    bool boundingBox(float, float, AABB& box) const override {
        box = AABB(_pMin, _pMax);
        return true;
    }
    uint32_t flatten(GraphWriter& w) const override;
    vec3 _pMin, _pMax;
    Hitable* _hitableList;
};
class BvhNode : public Hitable {
public:
    // bvhNode.h:25-59: random split axis (one scene-stream draw), qsort by box
    // minimum with the reference's comparators, median split.
    BvhNode(Arena& arena, SceneRng& rng, Hitable** l, int n, float time0, float time1);
    bool boundingBox(float, float, AABB& box) const override {
        box = _box;
        return true;
    }
    uint32_t flatten(GraphWriter& w) const override;
    Hitable* _left;
    Hitable* _right;
    AABB _box;
};
class ConstantMedium : public Hitable {
public:
    ConstantMedium(Arena& arena, Hitable* boundary, float density, Texture* a);
    bool boundingBox(float t0, float t1, AABB& box) const override { return _boundary->boundingBox(t0, t1, box); }
    uint32_t flatten(GraphWriter& w) const override;
    Hitable* _boundary;
    float _density;
    Material* _phaseFunction;
};

// ---- ownership -------------------------------------------------------------
class Arena {
public:
    template <class T, class... A>
    T* make(A&&... a) {
        T* p = new T(std::forward<A>(a)...);
        _owned.emplace_back(p, [](void* q) { delete static_cast<T*>(q); });
        return p;
    }
    Hitable** list(size_t n) {
        _lists.emplace_back(new Hitable*[n]());
        return _lists.back().get();
    }

private:
    std::vector<std::unique_ptr<void, void (*)(void*)>> _owned;
    std::vector<std::unique_ptr<Hitable*[]>> _lists;
};

// ---- flattening ------------------------------------------------------------
// Object graph -> rtow_scene arrays, in the canonical order include/rtow.h
// documents.
class GraphWriter {
public:
    explicit GraphWriter(const PerlinTables& perlin) : _perlin(perlin.t) {}
    uint32_t hitable(const Hitable* h);
    uint32_t material(const Material* m);
    uint32_t texture(const Texture* t);
    uint32_t image(const unsigned char* data, int nx, int ny);

    // used by the flatten() overrides
    uint32_t beginHitable(const Hitable* h, bool* fresh);
    uint32_t beginMaterial(const Material* m, bool* fresh);
    uint32_t beginTexture(const Texture* t, bool* fresh);
    std::vector<rtow_hitable> hit;
    std::vector<uint32_t> refs;
    std::vector<rtow_material> mats;
    std::vector<rtow_texture> texs;
    std::vector<rtow_image> imgs;
    std::vector<uint8_t> texels;
    rtow_perlin _perlin;

private:
    std::unordered_map<const void*, uint32_t> _hmap, _mmap, _tmap, _imap;
};

// ---- camera (camera.h) -----------------------------------------------------
class Camera {
public:
    // camera.h:13-121 with setCamera_QuaternionMatrix (camera.h:315-342): the
    // basis comes from the NED orientation matrix rows; lookAt and up are kept
    // but, as in the reference, do not steer the view.
    Camera(vec3 lookFrom, vec3 lookAt, vec3 up, float vFoV, float aspect, float aperture, float focusDist,
           float t0, float t1);
    vec3 getU() const { return _u; }
    vec3 getV() const { return _v; }
    vec3 getW() const { return _w; }
    vec3 getLookFromPoint() const { return _lookFromPoint; }
    vec3 getLookAt() const { return _lookAt; }
    void getTime(float& t0, float& t1) const { t0 = _time0; t1 = _time1; }
    // orientation rows (camera.h:76-81 initial NED basis), see setOrientationMatrix camera.h:231-235
    void setOrientationRows(const vec3& w, const vec3& u, const vec3& v);
    void setLookFromPoint(vec3 p) { _lookFromPoint = p; setCamera(); }
    void setVerticalFoV(float f) { _vFoV = f; setCamera(); }
    void setAspect(float a) { _aspect = a; setCamera(); }
    void setAperture(float a) { _aperture = a; setCamera(); }
    void setFocusDistance(float d) { _focusDistance = d; setCamera(); }
    void setTime(float t0, float t1) { _time0 = t0; _time1 = t1; setCamera(); }
    // setCamera_Euler (camera.h:271-313): the basis from lookFrom, lookAt and
    // up instead of the orientation rows (the reference compiles it out of
    // setCamera, camera.h:344-350; here it is selectable)
    void setCamera_Euler();
    rtow_camera toDevice() const;

private:
    void setCamera();
    vec3 _lookFromPoint, _lookAt, _upDirection;
    float _vFoV, _aspect, _aperture, _focusDistance;
    vec3 _rowW, _rowU, _rowV;
    vec3 _origin, _lowerLeftCorner, _horizontal, _vertical, _u, _v, _w;
    float _lensRadius = 0;
    float _time0, _time1;
};

// main.cpp:111-125
Camera mainCamera(uint32_t width, uint32_t height);

// ---- scenes (scenes.h) -------------------------------------------------------
struct Image {
    int nx = 0, ny = 0;
    std::vector<unsigned char> rgb;
    bool empty() const { return rgb.empty(); }
};

// Everything a built world needs kept alive.
struct World {
    Arena arena;
    PerlinTables perlin;
    std::vector<Image> images;
    Hitable* root = nullptr;
    uint32_t draws = 0;
};

// scenes.h:122-218 with n parameterised (the reference hard-codes 100).
// `earth` empty reproduces the reference's stbi_load-failed fallback.
Hitable* randomScene_NED(World& w, SceneRng& rng, int n, const Image* earth);
Hitable* cornellBox_NED(World& w);                 // scenes.h:355-483
Hitable* cornellSmoke_NED(World& w);               // + smoke box of scenes.h:461-470
Hitable* threeSphere_NED(World& w);                // config 1 (composed)
// config 5 (composed); per_side: the ground's Boxes per side (the book's 20)
Hitable* finalScene_NED(World& w, SceneRng& rng, const Image* earth, int per_side = 20);
// the reference's non-NED builders: randomScene scenes.h:29-120 (n
// parameterised, `earth` its earth1300x1300.jpg) and cornellBox scenes.h:220-353
Hitable* randomScene(World& w, SceneRng& rng, int n, const Image* earth);
Hitable* cornellBox(World& w);

// Build one of the RTOW_SCENE_* worlds the way main.cpp does (Perlin tables
// first, then the scene, then main.cpp's root Translate when opts.wrap_world).
int buildWorld(int sceneId, const rtow_build_opts& opts, World& out);

// Flattened, self-contained scene (owns its arrays).
struct SceneGraph {
    std::vector<rtow_hitable> hitables;
    std::vector<uint32_t> refs;
    std::vector<rtow_material> materials;
    std::vector<rtow_texture> textures;
    rtow_perlin perlin;
    std::vector<rtow_image> images;
    std::vector<uint8_t> texels;
    uint32_t root = 0;
    uint32_t draws = 0;
    rtow_scene view() const;
};
SceneGraph flattenWorld(const Hitable* root, const PerlinTables& perlin);

Image syntheticImage(int nx, int ny);

}  // namespace rtow
