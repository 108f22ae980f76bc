// rtow_scene.cpp — host side: scene classes, builders, flattening, camera and
// the device-independent part of the C-ABI (include/rtow.h).
//
// Expression shapes that feed stored floats follow the reference exactly
// (double literals promote, float members truncate), because the flattened
// scene must be byte-identical to the reference's (tests/golden).
#include "rtow_host.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <new>
#include <string>

#include "rtow_internal.h"

namespace rtow {

// ---- aabb.h:66-79 -----------------------------------------------------------
AABB surroundingBox(const AABB& box0, const AABB& box1) {
    vec3 small(std::fmin(box0.min().x(), box1.min().x()), std::fmin(box0.min().y(), box1.min().y()),
               std::fmin(box0.min().z(), box1.min().z()));
    vec3 big(std::fmax(box0.max().x(), box1.max().x()), std::fmax(box0.max().y(), box1.max().y()),
             std::fmax(box0.max().z(), box1.max().z()));
    return AABB(small, big);
}

// ---- bounding boxes -----------------------------------------------------------
bool Sphere::boundingBox(float, float, AABB& box) const {  // sphere.h:71-74
    box = AABB(_center - vec3(_radius, _radius, _radius), _center + vec3(_radius, _radius, _radius));
    return true;
}

vec3 MovingSphere::center(float time) const {  // sphere.h:129-131
    return _center0 + ((time - _time0) / (_time1 - _time0)) * (_center1 - _center0);
}

bool MovingSphere::boundingBox(float, float, AABB& box) const {  // sphere.h:120-127
    vec3 r(_radius, _radius, _radius);
    AABB b0(center(_time0) - r, center(_time0) + r);
    AABB b1(center(_time1) - r, center(_time1) + r);
    box = surroundingBox(b0, b1);
    return true;
}

bool AxisRectangle::boundingBox(float, float, AABB& box) const {  // xy_rect.h:13-16, 48-51, 83-86
    float lo = (float)(_k - 0.0001), hi = (float)(_k + 0.0001);
    switch (_kind) {
    case RTOW_HIT_RECT_XY: box = AABB(vec3(_a0, _b0, lo), vec3(_a1, _b1, hi)); break;
    case RTOW_HIT_RECT_XZ: box = AABB(vec3(_a0, lo, _b0), vec3(_a1, hi, _b1)); break;
    default: box = AABB(vec3(lo, _a0, _b0), vec3(hi, _a1, _b1)); break;
    }
    return true;
}

bool Translate::boundingBox(float t0, float t1, AABB& box) const {  // hitable.h:64-72
    if (_hitablePointer->boundingBox(t0, t1, box)) {
        box = AABB(box.min() + _offset, box.max() + _offset);
        return true;
    }
    return false;
}

RotateY::RotateY(Hitable* h, float angle) : _pointer(h) {  // hitable.h:90-123
    float radians = (float)((M_PI / 180.0) * angle);
    _sinTheta = std::sin(radians);
    _cosTheta = std::cos(radians);
    _hasBox = _pointer->boundingBox(0, 1, _boundBox);
    vec3 mn(FLT_MAX, FLT_MAX, FLT_MAX), mx(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
            for (int k = 0; k < 2; k++) {
                float x = i * _boundBox.max().x() + (1 - i) * _boundBox.min().x();
                float y = j * _boundBox.max().y() + (1 - j) * _boundBox.min().y();
                float z = k * _boundBox.max().z() + (1 - k) * _boundBox.min().z();
                float nx = _cosTheta * x + _sinTheta * z;
                float nz = -_sinTheta * x + _cosTheta * z;
                vec3 t(nx, y, nz);
                for (int c = 0; c < 3; c++) {
                    if (t[c] > mx[c]) mx[c] = t[c];
                    if (t[c] < mn[c]) mn[c] = t[c];
                }
            }
    _boundBox = AABB(mn, mx);
}

bool HitableList::boundingBox(float t0, float t1, AABB& box) const {
    // hitableList.h:40-60, including its bug: every iteration re-reads item 0.
    if (_hitableList.empty()) return false;
    AABB tmp;
    if (!_hitableList[0]->boundingBox(t0, t1, tmp)) return false;
    box = tmp;
    for (size_t i = 0; i < _hitableList.size(); i++) {
        if (_hitableList[0]->boundingBox(t0, t1, tmp))
            box = surroundingBox(box, tmp);
        else
            return false;
    }
    return true;
}

Box::Box(Arena& arena, const vec3& p0, const vec3& p1, Material* m) : _pMin(p0), _pMax(p1) {  // box.h:25-41
    std::vector<Hitable*> sides(6);
    sides[0] = arena.make<FlipNormals>(arena.make<XYRectangle>(p0.x(), p1.x(), p0.y(), p1.y(), p1.z(), m));
    sides[1] = arena.make<XYRectangle>(p0.x(), p1.x(), p0.y(), p1.y(), p0.z(), m);
    sides[2] = arena.make<XZRectangle>(p0.x(), p1.x(), p0.z(), p1.z(), p1.y(), m);
    sides[3] = arena.make<FlipNormals>(arena.make<XZRectangle>(p0.x(), p1.x(), p0.z(), p1.z(), p0.y(), m));
    sides[4] = arena.make<YZRectangle>(p0.y(), p1.y(), p0.z(), p1.z(), p1.x(), m);
    sides[5] = arena.make<FlipNormals>(arena.make<YZRectangle>(p0.y(), p1.y(), p0.z(), p1.z(), p0.x(), m));
    _hitableList = arena.make<HitableList>(std::move(sides));
}

ConstantMedium::ConstantMedium(Arena& arena, Hitable* boundary, float density, Texture* a)
    : _boundary(boundary), _density(density), _phaseFunction(arena.make<Isotropic>(a)) {}  // constantMedium.h:12-14

// bvhNode.h:98-144: never returns 0, so the order qsort leaves depends on the
// C library's algorithm -- the same glibc qsort the reference build calls.
template <int AXIS>
static int boxCompare(const void* a, const void* b) {
    AABB l, r;
    const Hitable* ah = *(Hitable* const*)a;
    const Hitable* bh = *(Hitable* const*)b;
    ah->boundingBox(0, 0, l);
    bh->boundingBox(0, 0, r);
    return (l.min()[AXIS] - r.min()[AXIS] < 0.0) ? -1 : 1;
}

BvhNode::BvhNode(Arena& arena, SceneRng& rng, Hitable** l, int n, float time0, float time1) {  // bvhNode.h:25-59
    int axis = int(3 * rng());
    if (axis == 0)
        std::qsort(l, (size_t)n, sizeof(Hitable*), boxCompare<0>);
    else if (axis == 1)
        std::qsort(l, (size_t)n, sizeof(Hitable*), boxCompare<1>);
    else
        std::qsort(l, (size_t)n, sizeof(Hitable*), boxCompare<2>);
    if (n == 1) {
        _left = _right = l[0];
    } else if (n == 2) {
        _left = l[0];
        _right = l[1];
    } else {
        _left = arena.make<BvhNode>(arena, rng, l, n / 2, time0, time1);
        _right = arena.make<BvhNode>(arena, rng, l + n / 2, n - n / 2, time0, time1);
    }
    AABB bl, br;
    if (!_left->boundingBox(time0, time1, bl) || !_right->boundingBox(time0, time1, br))
        std::fprintf(stderr, "rtow: BvhNode child without a bounding box\n");
    _box = surroundingBox(bl, br);
}

// ---- Perlin tables (noise.h:58-116) -------------------------------------------
void PerlinTables::generate(SceneRng& rng) {
    for (int i = 0; i < 256; ++i) t.ranfloat[i] = (float)rng();
    for (int i = 0; i < 256; ++i) {
        double a = rng(), b = rng(), c = rng();
        vec3 v = unit_vector(vec3((float)(-1 + 2 * a), (float)(-1 + 2 * b), (float)(-1 + 2 * c)));
        t.ranvec[i][0] = v.x();
        t.ranvec[i][1] = v.y();
        t.ranvec[i][2] = v.z();
    }
    int32_t* perms[3] = {t.perm_x, t.perm_y, t.perm_z};
    for (int32_t* p : perms) {
        for (int i = 0; i < 256; i++) p[i] = i;
        for (int i = 255; i > 0; i--) {
            int target = int(rng() * (i + 1));
            int32_t tmp = p[i];
            p[i] = p[target];
            p[target] = tmp;
        }
    }
}

// ---- flattening (include/rtow.h canonical order) ------------------------------
static void put3(float* d, const vec3& v) {
    d[0] = v.x();
    d[1] = v.y();
    d[2] = v.z();
}

uint32_t GraphWriter::beginHitable(const Hitable* h, bool* fresh) {
    auto it = _hmap.find(h);
    if (it != _hmap.end()) {
        *fresh = false;
        return it->second;
    }
    uint32_t idx = (uint32_t)hit.size();
    hit.push_back(rtow_hitable{});
    _hmap[h] = idx;
    *fresh = true;
    return idx;
}
uint32_t GraphWriter::beginMaterial(const Material* m, bool* fresh) {
    auto it = _mmap.find(m);
    if (it != _mmap.end()) {
        *fresh = false;
        return it->second;
    }
    uint32_t idx = (uint32_t)mats.size();
    mats.push_back(rtow_material{});
    _mmap[m] = idx;
    *fresh = true;
    return idx;
}
uint32_t GraphWriter::beginTexture(const Texture* t, bool* fresh) {
    auto it = _tmap.find(t);
    if (it != _tmap.end()) {
        *fresh = false;
        return it->second;
    }
    uint32_t idx = (uint32_t)texs.size();
    texs.push_back(rtow_texture{});
    _tmap[t] = idx;
    *fresh = true;
    return idx;
}
uint32_t GraphWriter::hitable(const Hitable* h) { return h->flatten(*this); }
uint32_t GraphWriter::material(const Material* m) { return m->flatten(*this); }
uint32_t GraphWriter::texture(const Texture* t) { return t->flatten(*this); }
uint32_t GraphWriter::image(const unsigned char* data, int nx, int ny) {
    auto it = _imap.find(data);
    if (it != _imap.end()) return it->second;
    uint32_t idx = (uint32_t)imgs.size();
    rtow_image im{};
    im.nx = (uint32_t)nx;
    im.ny = (uint32_t)ny;
    im.channels = 3;
    im.offset = texels.size();
    texels.insert(texels.end(), data, data + (size_t)nx * (size_t)ny * 3);
    imgs.push_back(im);
    _imap[data] = idx;
    return idx;
}

#define RTOW_TEXTURE_FLATTEN(T, BODY)                     \
    uint32_t T::flatten(GraphWriter& w) const {           \
        bool fresh;                                       \
        uint32_t idx = w.beginTexture(this, &fresh);      \
        if (!fresh) return idx;                           \
        rtow_texture r{};                                 \
        BODY;                                             \
        w.texs[idx] = r;                                  \
        return idx;                                       \
    }
RTOW_TEXTURE_FLATTEN(ConstantTexture, r.kind = RTOW_TEX_CONSTANT; put3(r.f, _color))
RTOW_TEXTURE_FLATTEN(CheckerTexture, r.kind = RTOW_TEX_CHECKER; r.a = w.texture(_odd); r.b = w.texture(_even))
RTOW_TEXTURE_FLATTEN(NoiseTexture, r.kind = RTOW_TEX_NOISE; r.f[0] = _scaled; r.a = _filter ? 1 : 0)
RTOW_TEXTURE_FLATTEN(ImageTexture, r.kind = RTOW_TEX_IMAGE; r.a = w.image(_data, _nx, _ny))

#define RTOW_MATERIAL_FLATTEN(T, BODY)                    \
    uint32_t T::flatten(GraphWriter& w) const {           \
        bool fresh;                                       \
        uint32_t idx = w.beginMaterial(this, &fresh);     \
        if (!fresh) return idx;                           \
        rtow_material r{};                                \
        BODY;                                             \
        w.mats[idx] = r;                                  \
        return idx;                                       \
    }
RTOW_MATERIAL_FLATTEN(Lambertian, r.kind = RTOW_MAT_LAMBERTIAN; r.texture = w.texture(_albedo))
RTOW_MATERIAL_FLATTEN(Metal, r.kind = RTOW_MAT_METAL; put3(r.albedo, _albedo); r.param = _fuzz)
RTOW_MATERIAL_FLATTEN(Dielectric, r.kind = RTOW_MAT_DIELECTRIC; r.param = _refIndex)
RTOW_MATERIAL_FLATTEN(DiffuseLight, r.kind = RTOW_MAT_DIFFUSE_LIGHT; r.texture = w.texture(_emit))
RTOW_MATERIAL_FLATTEN(Isotropic, r.kind = RTOW_MAT_ISOTROPIC; r.texture = w.texture(_albedo))

#define RTOW_HITABLE_FLATTEN(T, BODY)                     \
    uint32_t T::flatten(GraphWriter& w) const {           \
        bool fresh;                                       \
        uint32_t idx = w.beginHitable(this, &fresh);      \
        if (!fresh) return idx;                           \
        rtow_hitable r{};                                 \
        BODY;                                             \
        w.hit[idx] = r;                                   \
        return idx;                                       \
    }
RTOW_HITABLE_FLATTEN(Sphere, r.kind = RTOW_HIT_SPHERE; put3(r.f, _center); r.f[3] = _radius;
                     r.a = w.material(_materialPointer))
RTOW_HITABLE_FLATTEN(MovingSphere, r.kind = RTOW_HIT_MOVING_SPHERE; put3(r.f, _center0); put3(r.f + 3, _center1);
                     r.f[6] = _time0; r.f[7] = _time1; r.f[8] = _radius; r.a = w.material(_materialPointer))
RTOW_HITABLE_FLATTEN(AxisRectangle, r.kind = _kind; r.f[0] = _a0; r.f[1] = _a1; r.f[2] = _b0; r.f[3] = _b1;
                     r.f[4] = _k; r.a = w.material(_material))
RTOW_HITABLE_FLATTEN(FlipNormals, r.kind = RTOW_HIT_FLIP_NORMALS; r.a = w.hitable(_hitable))
RTOW_HITABLE_FLATTEN(Translate, r.kind = RTOW_HIT_TRANSLATE; put3(r.f, _offset); r.a = w.hitable(_hitablePointer))
RTOW_HITABLE_FLATTEN(RotateY, r.kind = RTOW_HIT_ROTATE_Y; r.f[0] = _sinTheta; r.f[1] = _cosTheta;
                     r.b = _hasBox ? 1 : 0; put3(r.f + 2, _boundBox.min()); put3(r.f + 5, _boundBox.max());
                     r.a = w.hitable(_pointer))
RTOW_HITABLE_FLATTEN(HitableList, r.kind = RTOW_HIT_LIST; r.a = (uint32_t)w.refs.size();
                     r.b = (uint32_t)_hitableList.size(); w.refs.resize(w.refs.size() + _hitableList.size());
                     for (size_t i = 0; i < _hitableList.size(); i++) {
                         uint32_t c = w.hitable(_hitableList[i]);
                         w.refs[r.a + i] = c;
                     })
RTOW_HITABLE_FLATTEN(Box, r.kind = RTOW_HIT_BOX; put3(r.f, _pMin); put3(r.f + 3, _pMax); r.a = w.hitable(_hitableList))
RTOW_HITABLE_FLATTEN(BvhNode, r.kind = RTOW_HIT_BVH_NODE; put3(r.f, _box.min()); put3(r.f + 3, _box.max());
                     r.a = w.hitable(_left); r.b = w.hitable(_right))
RTOW_HITABLE_FLATTEN(ConstantMedium, r.kind = RTOW_HIT_CONSTANT_MEDIUM; r.f[0] = _density;
                     r.a = w.hitable(_boundary); r.b = w.material(_phaseFunction))

rtow_scene SceneGraph::view() const {
    rtow_scene s{};
    s.root = root;
    s.n_hitables = (uint32_t)hitables.size();
    s.hitables = hitables.data();
    s.n_refs = (uint32_t)refs.size();
    s.refs = refs.empty() ? nullptr : refs.data();
    s.n_materials = (uint32_t)materials.size();
    s.materials = materials.data();
    s.n_textures = (uint32_t)textures.size();
    s.textures = textures.data();
    s.perlin = &perlin;
    s.n_images = (uint32_t)images.size();
    s.images = images.empty() ? nullptr : images.data();
    s.n_texel_bytes = texels.size();
    s.texels = texels.empty() ? nullptr : texels.data();
    return s;
}

SceneGraph flattenWorld(const Hitable* root, const PerlinTables& perlin) {
    GraphWriter w(perlin);
    SceneGraph g;
    g.root = w.hitable(root);
    g.hitables = std::move(w.hit);
    g.refs = std::move(w.refs);
    g.materials = std::move(w.mats);
    g.textures = std::move(w.texs);
    g.perlin = perlin.t;
    g.images = std::move(w.imgs);
    g.texels = std::move(w.texels);
    return g;
}

// ---- camera (camera.h:13-121, 315-342) --------------------------------------------
Camera::Camera(vec3 lookFrom, vec3 lookAt, vec3 up, float vFoV, float aspect, float aperture, float focusDist,
               float t0, float t1)
    : _lookFromPoint(lookFrom), _lookAt(lookAt), _upDirection(up), _vFoV(vFoV), _aspect(aspect),
      _aperture(aperture), _focusDistance(focusDist), _rowW(-1, 0, 0), _rowU(0, 1, 0), _rowV(0, 0, -1),
      _time0(t0), _time1(t1) {
    setCamera();
}

void Camera::setOrientationRows(const vec3& w, const vec3& u, const vec3& v) {
    _rowW = w;
    _rowU = u;
    _rowV = v;
    setCamera();
}

void Camera::setCamera() {
    _lensRadius = _aperture / 2;
    float theta = (float)(_vFoV * M_PI / 180);
    float half_height = std::tan(theta / 2);
    float half_width = _aspect * half_height;
    _origin = _lookFromPoint;
    _w = _rowW;
    _u = _rowU;
    _v = _rowV;
    _lowerLeftCorner = _origin - half_width * _focusDistance * _u - half_height * _focusDistance * _v -
                       _focusDistance * _w;
    _horizontal = 2 * half_width * _focusDistance * _u;
    _vertical = 2 * half_height * _focusDistance * _v;
}

void Camera::setCamera_Euler() {  // camera.h:271-313
    _lensRadius = _aperture / 2;
    float theta = (float)(_vFoV * M_PI / 180);
    float half_height = std::tan(theta / 2);
    float half_width = _aspect * half_height;
    _origin = _lookFromPoint;
    _w = unit_vector(_lookFromPoint - _lookAt);
    _u = unit_vector(cross(_upDirection, _w));
    _v = cross(_w, _u);
    _lowerLeftCorner = _origin - half_width * _focusDistance * _u - half_height * _focusDistance * _v -
                       _focusDistance * _w;
    _horizontal = 2 * half_width * _focusDistance * _u;
    _vertical = 2 * half_height * _focusDistance * _v;
}

rtow_camera Camera::toDevice() const {
    rtow_camera c{};
    put3(c.origin, _origin);
    put3(c.lower_left_corner, _lowerLeftCorner);
    put3(c.horizontal, _horizontal);
    put3(c.vertical, _vertical);
    put3(c.u, _u);
    put3(c.v, _v);
    put3(c.w, _w);
    c.lens_radius = _lensRadius;
    c.time0 = _time0;
    c.time1 = _time1;
    return c;
}

Camera mainCamera(uint32_t width, uint32_t height) {  // main.cpp:111-125
    float aspect = float(width) / float(height);
    return Camera(vec3(0, 0, 0), vec3(1, 0, 0), vec3(0, 0, -1), 60.0f, aspect, 2.0f, 1000.0f, 0.0f, 1.0f);
}

// ---- scenes (scenes.h) ------------------------------------------------------------
Image syntheticImage(int nx, int ny) {
    Image im;
    im.nx = nx;
    im.ny = ny;
    im.rgb.resize((size_t)nx * (size_t)ny * 3);
    rtow_synthetic_image((uint32_t)nx, (uint32_t)ny, im.rgb.data());
    return im;
}

Hitable* randomScene_NED(World& w, SceneRng& rng, int n, const Image* earth) {  // scenes.h:122-218
    Arena& A = w.arena;
    Hitable** list = A.list((size_t)n + 1);
    Texture* checker = A.make<CheckerTexture>(A.make<ConstantTexture>(vec3(0.2f, 0.2f, 0.8f)),
                                              A.make<ConstantTexture>(vec3(0.9f, 0.9f, 0.9f)));
    Texture* perlin = A.make<NoiseTexture>(true, 8.0f);
    Material* emitterMat = A.make<DiffuseLight>(A.make<ConstantTexture>(vec3(20 * 1, 20 * 0, 20 * 0)));
    Material* imageMat = nullptr;
    if (earth && !earth->empty())
        imageMat = A.make<Lambertian>(A.make<ImageTexture>(earth->rgb.data(), earth->nx, earth->ny));
    const float R = 1000.0f;
    const float zOff = -1 * R;
    list[0] = A.make<Sphere>(vec3(0, 0, 0), R, A.make<Lambertian>(perlin));
    int i = 1;
    const int xMod = 10, yMod = 10;
    int cx = xMod, cy = yMod;
    while (i < n - 3) {
        float choose = (float)rng();
        // The reference's vec3 arguments are evaluated right to left (g++):
        // the y draw comes before the x draw.
        double uy = rng();
        double ux = rng();
        vec3 center((float)(cx * ux), (float)(cy * uy), zOff - 1);
        if ((center - vec3(4, 0.2f, 0)).length() > 0.9) {
            if (choose < 0.8) {
                double up = rng();
                list[i++] = A.make<MovingSphere>(center, center + vec3(0, (float)(0.5 * up), 0), 0.0f, 1.0f, 0.2f,
                                                 A.make<Lambertian>(checker));
            } else if (choose < 0.95) {
                double az = rng(), ay = rng(), ax = rng(), fz = rng();
                list[i++] = A.make<Sphere>(
                    center, 0.2f,
                    A.make<Metal>(vec3((float)(0.5 * (1 + ax)), (float)(0.5 * (1 + ay)), (float)(0.5 * (1 + az))),
                                  (float)(0.5 * (1 + fz))));
            } else {
                list[i++] = A.make<Sphere>(center, 0.5f, A.make<Dielectric>(1.5f));
            }
        }
        if (cx < xMod) {
            cx++;
        } else {
            cx = -xMod;
            cy++;
        }
        if (cy > yMod) cy = -yMod;
    }
    const float earthZ = (float)(zOff - 25.0);
    if (imageMat)
        list[i++] = A.make<Sphere>(vec3(20.0f, 0.0f, earthZ), 10.0f, imageMat);
    else
        list[i++] = A.make<Sphere>(vec3(20.0f, 0.0f, earthZ), 10.0f, A.make<Dielectric>(1.5f));
    list[i++] = A.make<Sphere>(vec3(100, -70, zOff), 50.0f, A.make<Lambertian>(perlin));
    list[i++] = A.make<Sphere>(vec3(100, 70, zOff), 50.0f, A.make<Metal>(vec3(0.7f, 0.6f, 0.5f), 0.0f));
    list[i++] = A.make<Sphere>(vec3(0, 0, zOff - 500), 100.0f, emitterMat);
    return A.make<BvhNode>(A, rng, list, i, 0.0f, 1.0f);
}

// scenes.h:29-120, the reference's first random scene (its own frame, no
// root Translate: main.cpp renders the NED builders), n parameterised like
// randomScene_NED (the reference hard-codes 100).  The same draws in the same
// (g++: right-to-left argument) order as the reference.
Hitable* randomScene(World& w, SceneRng& rng, int n, const Image* earth) {
    Arena& A = w.arena;
    Hitable** list = A.list((size_t)n + 1);
    Texture* checker = A.make<CheckerTexture>(A.make<ConstantTexture>(vec3(0.2f, 0.2f, 0.8f)),
                                              A.make<ConstantTexture>(vec3(0.9f, 0.9f, 0.9f)));
    Texture* perlin = A.make<NoiseTexture>(true, 8.0f);
    Material* emitterMat = A.make<DiffuseLight>(A.make<ConstantTexture>(vec3(20 * 1, 20 * 0, 20 * 0)));
    Material* imageMat = nullptr;  // scenes.h:47: ./input_images/earth1300x1300.jpg
    if (earth && !earth->empty())
        imageMat = A.make<Lambertian>(A.make<ImageTexture>(earth->rgb.data(), earth->nx, earth->ny));
    list[0] = A.make<Sphere>(vec3(0, 1000, 0), 1000.0f, A.make<Lambertian>(perlin));
    int i = 1;
    const int xMod = 5, yMod = 5;
    int cx = -xMod, cy = -yMod;
    while (i < n - 3) {
        float choose = (float)rng();
        double uz = rng();  // vec3(x, y, z)'s arguments right to left: z's draw first
        double ux = rng();
        vec3 center((float)(cx + 0.9 * ux), -0.2f, (float)(cy + 0.9 * uz));
        if ((center - vec3(4, 0.2f, 0)).length() > 0.9) {
            if (choose < 0.8) {
                double up = rng();
                list[i++] = A.make<MovingSphere>(center, center + vec3(0, (float)(0.5 * up), 0), 0.0f, 1.0f, 0.2f,
                                                 A.make<Lambertian>(checker));
            } else if (choose < 0.95) {
                double az = rng(), ay = rng(), ax = rng(), fz = rng();
                list[i++] = A.make<Sphere>(
                    center, 0.2f,
                    A.make<Metal>(vec3((float)(0.5 * (1 + ax)), (float)(0.5 * (1 + ay)), (float)(0.5 * (1 + az))),
                                  (float)(0.5 * (1 + fz))));
            } else {
                list[i++] = A.make<Sphere>(center, 0.2f, A.make<Dielectric>(1.5f));
            }
        }
        if (cx < xMod) {
            cx++;
        } else {
            cx = -xMod;
            cy++;
        }
        if (cy > yMod) cy = -yMod;
    }
    if (imageMat)
        list[i++] = A.make<Sphere>(vec3(0, -2.0f, 20), 2.0f, imageMat);
    else
        list[i++] = A.make<Sphere>(vec3(5, -1.0f, 0), 1.0f, A.make<Dielectric>(1.5f));
    list[i++] = A.make<Sphere>(vec3(-4, -1.0f, 0), 1.0f, A.make<Lambertian>(perlin));
    list[i++] = A.make<Sphere>(vec3(4, -1.0f, 0), 1.0f, A.make<Metal>(vec3(0.7f, 0.6f, 0.5f), 0.0f));
    list[i++] = A.make<Sphere>(vec3(0, -400, 10), 100.0f, emitterMat);  // the "sun"
    return A.make<BvhNode>(A, rng, list, i, 0.0f, 1.0f);
}

// scenes.h:220-353, the reference's first Cornell box (its own frame, no root
// Translate): the light, five walls (the back one under Translate(0, 0, 0)),
// the medium inside the glass sphere.  The reference computes the extents in
// int arithmetic (planeWidth = planeHeight = planeAxisDepthOffset = 500,
// xCoord = yCoord = 0); these are its values.
Hitable* cornellBox(World& w) {
    Arena& A = w.arena;
    std::vector<Hitable*> L;
    Material* white = A.make<Lambertian>(A.make<ConstantTexture>(vec3(0.73f, 0.73f, 0.73f)));
    Material* red = A.make<Lambertian>(A.make<ConstantTexture>(vec3(0.65f, 0.05f, 0.05f)));
    Material* blue = A.make<Lambertian>(A.make<ConstantTexture>(vec3(0.12f, 0.12f, 0.45f)));
    Material* light = A.make<DiffuseLight>(A.make<ConstantTexture>(vec3(3, 3, 3)));
    L.push_back(A.make<XZRectangle>(-175, 175, 75, 425, -249, light));                           // light panel
    L.push_back(A.make<XZRectangle>(-250, 250, 0, 500, -250, white));                            // top
    L.push_back(A.make<YZRectangle>(-250, 250, 0, 500, -250, red));                              // left
    L.push_back(A.make<Translate>(A.make<FlipNormals>(A.make<XYRectangle>(-250, 250, -250, 250, 500, white)),
                                  vec3(0, 0, 0)));                                               // back
    L.push_back(A.make<FlipNormals>(A.make<YZRectangle>(-250, 250, 0, 500, 250, blue)));        // right
    L.push_back(A.make<FlipNormals>(A.make<XZRectangle>(-250, 250, 0, 500, 250, white)));       // bottom
    Material* innerMat = A.make<Lambertian>(A.make<ConstantTexture>(vec3(0.9f, 0.05f, 0.10f)));
    Hitable* outer = A.make<Sphere>(vec3(-150, 150, 200), 100.0f, A.make<Dielectric>(1.5f));
    Hitable* inner = A.make<Sphere>(vec3(-150, 150, 200), 99.0f, innerMat);
    L.push_back(A.make<ConstantMedium>(A, inner, 0.001f, A.make<ConstantTexture>(vec3(0.8f, 0.2f, 0.1f))));
    L.push_back(inner);
    L.push_back(outer);
    return A.make<HitableList>(std::move(L));
}

static void cornellItems(World& w, std::vector<Hitable*>& L) {  // scenes.h:355-480
    Arena& A = w.arena;
    Material* white = A.make<Lambertian>(A.make<ConstantTexture>(vec3(0.73f, 0.73f, 0.73f)));
    Material* red = A.make<Lambertian>(A.make<ConstantTexture>(vec3(0.65f, 0.05f, 0.05f)));
    Material* blue = A.make<Lambertian>(A.make<ConstantTexture>(vec3(0.12f, 0.12f, 0.45f)));
    Material* light = A.make<DiffuseLight>(A.make<ConstantTexture>(vec3(3, 3, 3)));
    const int pw = 1000, ph = 1000;
    L.push_back(A.make<Translate>(A.make<XYRectangle>(0, pw / 2, 0, ph / 2, 0, light),
                                  vec3(-pw / 4, -pw / 4, (-ph / 2) + 1)));                       // light panel
    L.push_back(A.make<Translate>(A.make<XYRectangle>(0, pw, 0, ph, 0, white), vec3(-pw / 2, -pw / 2, -ph / 2)));  // top
    L.push_back(A.make<Translate>(A.make<FlipNormals>(A.make<XYRectangle>(0, pw, 0, ph, 0, white)),
                                  vec3(-pw / 2, -pw / 2, ph / 2)));                              // bottom
    L.push_back(A.make<Translate>(A.make<XZRectangle>(0, pw, 0, ph, 0, red), vec3(-pw / 2, -pw / 2, -ph / 2)));  // left
    L.push_back(A.make<Translate>(A.make<FlipNormals>(A.make<YZRectangle>(0, pw, 0, ph, 0, white)),
                                  vec3(pw / 2, -pw / 2, -ph / 2)));                              // back
    L.push_back(A.make<Translate>(A.make<FlipNormals>(A.make<XZRectangle>(0, pw, 0, ph, 0, blue)),
                                  vec3(-pw / 2, pw / 2, -ph / 2)));                              // right
    L.push_back(A.make<Translate>(A.make<Box>(A, vec3(0, 0, 0), vec3(200, 200, 300), blue), vec3(0, -300, 0)));
    L.push_back(A.make<Translate>(A.make<Box>(A, vec3(0, 0, 0), vec3(200, 200, 300), red), vec3(0, 150, 0)));
    L.push_back(A.make<Translate>(A.make<RotateY>(A.make<Box>(A, vec3(0, 0, 0), vec3(160, 160, 160), blue), 18.0f),
                                  vec3(0, 0, -200)));
}

static void cornellSpheres(World& w, std::vector<Hitable*>& L) {  // scenes.h:472-479
    Arena& A = w.arena;
    Material* innerMat = A.make<Lambertian>(A.make<ConstantTexture>(vec3(0.1f, 0.7f, 0.20f)));
    Hitable* outer = A.make<Sphere>(vec3(0, 0, 150), 100.0f, A.make<Dielectric>(1.5f));
    Hitable* inner = A.make<Sphere>(vec3(0, 0, 150), 99.0f, innerMat);
    L.push_back(A.make<ConstantMedium>(A, inner, 0.001f, A.make<ConstantTexture>(vec3(0.1f, 0.7f, 0.2f))));
    L.push_back(inner);
    L.push_back(outer);
}

Hitable* cornellBox_NED(World& w) {
    std::vector<Hitable*> L;
    cornellItems(w, L);
    cornellSpheres(w, L);
    return w.arena.make<HitableList>(std::move(L));
}

Hitable* cornellSmoke_NED(World& w) {
    // cornellBox_NED with the smoke box scenes.h:461-470 keeps commented out, at
    // the list position that code occupies (after the rotated box).
    Arena& A = w.arena;
    std::vector<Hitable*> L;
    cornellItems(w, L);
    Material* green = A.make<Lambertian>(A.make<ConstantTexture>(vec3(0.12f, 0.95f, 0.15f)));
    Hitable* box = A.make<Translate>(
        A.make<RotateY>(A.make<Box>(A, vec3(0, 0, 0), vec3(160, 300, 160), green), -25.0f), vec3(-100, -50, 200));
    L.push_back(A.make<ConstantMedium>(A, box, 0.01f, A.make<ConstantTexture>(vec3(0.2f, 0.9f, 0.4f))));
    cornellSpheres(w, L);
    return A.make<HitableList>(std::move(L));
}

Hitable* threeSphere_NED(World& w) {
    Arena& A = w.arena;
    std::vector<Hitable*> L;
    L.push_back(A.make<Sphere>(vec3(10, 0, 101), 100.0f,
                               A.make<Lambertian>(A.make<ConstantTexture>(vec3(0.8f, 0.8f, 0.0f)))));
    L.push_back(A.make<Sphere>(vec3(10, 0, 0), 1.0f, A.make<Lambertian>(A.make<ConstantTexture>(vec3(0.1f, 0.2f, 0.5f)))));
    L.push_back(A.make<Sphere>(vec3(10, -2.2f, 0), 1.0f,
                               A.make<Lambertian>(A.make<ConstantTexture>(vec3(0.8f, 0.3f, 0.3f)))));
    return A.make<HitableList>(std::move(L));
}

// Config 5: book 2's final scene ("The Next Week", final chapter), which the
// reference does not have, composed from its classes in its NED frame: NED
// (x, y, z) = (book z, book x, -book y); the sphere cloud turns with RotateY
// (about NED y, the reference's only rotation) where the book turns it about
// its vertical axis.  Draws in this order: 400 box heights, then per cloud
// sphere book x, y, z; plus one per BvhNode (oracle/ref_harness.cpp
// finalSceneNed is the same composition over the reference's own classes).
// per_side: the ground's Boxes per side (the book: 20, each 100 wide; other
// counts keep the ground's 2000 x 2000 extent -- a larger grid for tests).
Hitable* finalScene_NED(World& w, SceneRng& rng, const Image* earth, int per_side) {
    Arena& A = w.arena;
    std::vector<Hitable*> L;
    Hitable** boxes = A.list((size_t)per_side * per_side);
    Hitable** cloud = A.list(1000);
    Material* white = A.make<Lambertian>(A.make<ConstantTexture>(vec3(0.73f, 0.73f, 0.73f)));
    Material* ground = A.make<Lambertian>(A.make<ConstantTexture>(vec3(0.48f, 0.83f, 0.53f)));
    int b = 0;
    for (int i = 0; i < per_side; i++) {
        for (int j = 0; j < per_side; j++) {
            float wd = 2000.0f / (float)per_side;  // (exactly 100 for the book's 20)
            float x0 = -1000 + i * wd;
            float z0 = -1000 + j * wd;
            float x1 = x0 + wd;
            float y1 = (float)(100 * (rng() + 0.01));
            float z1 = z0 + wd;
            boxes[b++] = A.make<Box>(A, vec3(z0, x0, -y1), vec3(z1, x1, 0), ground);
        }
    }
    L.push_back(A.make<BvhNode>(A, rng, boxes, b, 0.0f, 1.0f));
    Material* light = A.make<DiffuseLight>(A.make<ConstantTexture>(vec3(7, 7, 7)));
    L.push_back(A.make<XYRectangle>(147, 412, 123, 423, -554, light));
    vec3 center(200, 400, -400);
    L.push_back(A.make<MovingSphere>(center, center + vec3(0, 30, 0), 0.0f, 1.0f, 50.0f,
                                     A.make<Lambertian>(A.make<ConstantTexture>(vec3(0.7f, 0.3f, 0.1f)))));
    L.push_back(A.make<Sphere>(vec3(45, 260, -150), 50.0f, A.make<Dielectric>(1.5f)));
    L.push_back(A.make<Sphere>(vec3(145, 0, -150), 50.0f, A.make<Metal>(vec3(0.8f, 0.8f, 0.9f), 10.0f)));
    Hitable* boundary = A.make<Sphere>(vec3(145, 360, -150), 70.0f, A.make<Dielectric>(1.5f));
    L.push_back(boundary);
    L.push_back(A.make<ConstantMedium>(A, boundary, 0.2f, A.make<ConstantTexture>(vec3(0.2f, 0.4f, 0.9f))));
    boundary = A.make<Sphere>(vec3(0, 0, 0), 5000.0f, A.make<Dielectric>(1.5f));
    L.push_back(A.make<ConstantMedium>(A, boundary, 0.0001f, A.make<ConstantTexture>(vec3(1.0f, 1.0f, 1.0f))));
    Material* emat = (earth && !earth->empty())
                         ? (Material*)A.make<Lambertian>(A.make<ImageTexture>(earth->rgb.data(), earth->nx, earth->ny))
                         : (Material*)A.make<Dielectric>(1.5f);
    L.push_back(A.make<Sphere>(vec3(400, 400, -200), 100.0f, emat));
    L.push_back(A.make<Sphere>(vec3(300, 220, -280), 80.0f, A.make<Lambertian>(A.make<NoiseTexture>(true, 0.1f))));
    for (int j = 0; j < 1000; j++) {
        double bx = rng();
        double by = rng();
        double bz = rng();
        cloud[j] = A.make<Sphere>(vec3((float)(165 * bz), (float)(165 * bx), (float)(-165 * by)), 10.0f, white);
    }
    L.push_back(A.make<Translate>(A.make<RotateY>(A.make<BvhNode>(A, rng, cloud, 1000, 0.0f, 1.0f), 15.0f),
                                  vec3(395, -100, -270)));
    return A.make<HitableList>(std::move(L));
}

static bool readRaw(const char* path, int nx, int ny, Image& im) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    im.nx = nx;
    im.ny = ny;
    im.rgb.resize((size_t)nx * (size_t)ny * 3);
    f.read(reinterpret_cast<char*>(im.rgb.data()), (std::streamsize)im.rgb.size());
    return (size_t)f.gcount() == im.rgb.size();
}

int buildWorld(int sceneId, const rtow_build_opts& o, World& out) {
    SceneRng rng(o.scene_seed);
    out.perlin.generate(rng);  // static initialisation happens first (noise.h:112-116)
    Hitable* scene = nullptr;
    Arena& A = out.arena;
    const Image* earth = nullptr;
    if (sceneId == RTOW_SCENE_RANDOM_NED || sceneId == RTOW_SCENE_FINAL_NED || sceneId == RTOW_SCENE_RANDOM) {
        if (o.image_mode == RTOW_IMAGE_SYNTHETIC) {
            out.images.push_back(syntheticImage(2048, 1024));
            earth = &out.images.back();
        } else if (o.image_mode == RTOW_IMAGE_JPEG) {
            uint8_t* px = nullptr;
            uint32_t nx = 0, ny = 0, ch = 0;
            if (!o.image_path) return set_error(RTOW_E_INVALID, "JPEG image mode without image_path");
            const int rc = rtow_image_load_jpeg(o.image_path, &px, &nx, &ny, &ch);
            if (rc != RTOW_OK) return rc;
            if (ch != 3) {
                rtow_image_free(px);
                return set_error(RTOW_E_UNSUPPORTED, "JPEG texture is not 3-channel (ImageTexture reads RGB)");
            }
            Image im;
            im.nx = (int)nx;
            im.ny = (int)ny;
            im.rgb.assign(px, px + (size_t)nx * ny * 3);
            rtow_image_free(px);
            out.images.push_back(std::move(im));
            earth = &out.images.back();
        } else if (o.image_mode == RTOW_IMAGE_RAW) {
            Image im;
            if (!o.image_path || o.image_nx == 0 || o.image_ny == 0 ||
                !readRaw(o.image_path, (int)o.image_nx, (int)o.image_ny, im))
                return set_error(RTOW_E_IO, "cannot read raw RGB8 image");
            out.images.push_back(std::move(im));
            earth = &out.images.back();
        }
    }
    switch (sceneId) {
    case RTOW_SCENE_THREE_SPHERE:
        scene = threeSphere_NED(out);
        break;
    case RTOW_SCENE_RANDOM_NED: {
        if (o.n < 4) return set_error(RTOW_E_INVALID, "random scene needs n >= 4");
        scene = randomScene_NED(out, rng, (int)o.n, earth);
        if (o.wrap_world) scene = A.make<Translate>(scene, vec3(0, 0, 1000));  // main.cpp:132
        break;
    }
    case RTOW_SCENE_RANDOM:
        if (o.n < 4) return set_error(RTOW_E_INVALID, "random scene needs n >= 4");
        scene = randomScene(out, rng, (int)o.n, earth);
        break;
    case RTOW_SCENE_CORNELL:
        scene = cornellBox(out);
        break;
    case RTOW_SCENE_CORNELL_NED:
        scene = cornellBox_NED(out);
        if (o.wrap_world) scene = A.make<Translate>(scene, vec3(800, 0, 0));  // main.cpp:136
        break;
    case RTOW_SCENE_CORNELL_SMOKE:
        scene = cornellSmoke_NED(out);
        if (o.wrap_world) scene = A.make<Translate>(scene, vec3(800, 0, 0));
        break;
    case RTOW_SCENE_FINAL_NED:
        if (o.ground_side > 256) return set_error(RTOW_E_INVALID, "final scene: at most 256 ground Boxes per side");
        scene = finalScene_NED(out, rng, earth, o.ground_side ? (int)o.ground_side : 20);
        if (o.wrap_world) scene = A.make<Translate>(scene, vec3(600, -278, 278));
        break;
    default:
        return set_error(RTOW_E_INVALID, "unknown scene id");
    }
    out.root = scene;
    out.draws = rng.draws();
    return RTOW_OK;
}

}  // namespace rtow

// ============================================================================
// C-ABI, host part
// ============================================================================
using namespace rtow;

struct rtow_scene_buf {
    SceneGraph g;
    rtow_scene view;
};

static thread_local std::string g_last_error;

int set_error(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

extern "C" {

int rtow_abi_version(void) { return RTOW_ABI_VERSION; }

const char* rtow_error_string(int code) {
    switch (code) {
    case RTOW_OK: return "ok";
    case RTOW_E_INVALID: return "invalid argument";
    case RTOW_E_UNSUPPORTED: return "unsupported scene construct";
    case RTOW_E_HIP: return "HIP runtime error";
    case RTOW_E_NO_DEVICE: return "no GPU device";
    case RTOW_E_IO: return "I/O error";
    case RTOW_E_NOMEM: return "out of memory";
    case RTOW_E_RCCL: return "RCCL error";
    default: return "unknown error";
    }
}

const char* rtow_last_error(void) { return g_last_error.c_str(); }

void rtow_params_default(rtow_params* p, uint32_t width, uint32_t height, uint32_t spp) {
    if (!p) return;
    std::memset(p, 0, sizeof *p);
    p->width = width;
    p->height = height;
    p->spp = spp;
    p->max_depth = 50;   // DEPTH_RECURSION defines.h:27
    p->gi_enable = 1;    // GLOBAL_ILLUM_EN defines.h:23
    p->sky_gain = 1.0f;  // SKY_ILLUM_GAIN defines.h:24
    p->gi_gain = 0.3f;   // GLOBAL_ILLUM_GAIN defines.h:25
    p->seed = 1;
    p->world = 1;
}

uint32_t rtow_tile_count(uint32_t width, uint32_t height) {
    return ((width + 7) / 8) * ((height + 7) / 8);
}

uint32_t rtow_rank_tile_count(uint32_t width, uint32_t height, uint32_t rank, uint32_t world) {
    uint32_t n = rtow_tile_count(width, height);
    if (world == 0) world = 1;
    if (rank >= world) return 0;
    return n > rank ? (n - rank + world - 1) / world : 0;
}

void rtow_build_opts_default(rtow_build_opts* o) {
    if (!o) return;
    std::memset(o, 0, sizeof *o);
    o->scene_seed = 1;
    o->n = 100;
    o->image_mode = RTOW_IMAGE_SYNTHETIC;
    o->wrap_world = 1;
}

int rtow_build_scene(int scene_id, const rtow_build_opts* opts, rtow_scene_buf** out) {
    if (!out) return set_error(RTOW_E_INVALID, "out is NULL");
    rtow_build_opts o;
    if (opts)
        o = *opts;
    else
        rtow_build_opts_default(&o);
    try {
        World w;
        int rc = buildWorld(scene_id, o, w);
        if (rc) return rc;
        auto* b = new rtow_scene_buf;
        b->g = flattenWorld(w.root, w.perlin);
        b->g.draws = w.draws;
        b->view = b->g.view();
        *out = b;
        return RTOW_OK;
    } catch (const std::bad_alloc&) {
        return set_error(RTOW_E_NOMEM, "out of memory building scene");
    }
}

const rtow_scene* rtow_scene_view(const rtow_scene_buf* b) { return b ? &b->view : nullptr; }

void rtow_scene_free(rtow_scene_buf* b) { delete b; }

uint32_t rtow_scene_draws(const rtow_scene_buf* b) { return b ? b->g.draws : 0; }

int rtow_scene_save(const rtow_scene* s, const char* path) {
    if (!s || !path) return set_error(RTOW_E_INVALID, "NULL argument");
    FILE* f = std::fopen(path, "wb");
    if (!f) return set_error(RTOW_E_IO, std::string("cannot open ") + path);
    uint32_t hdr[10] = {1u, s->root, s->n_hitables, s->n_refs, s->n_materials, s->n_textures, s->n_images,
                        s->perlin ? 1u : 0u, 0u, 0u};
    uint64_t ntex = s->n_texel_bytes;
    bool ok = std::fwrite("RTOWSCN1", 1, 8, f) == 8 && std::fwrite(hdr, 4, 10, f) == 10 &&
              std::fwrite(&ntex, 8, 1, f) == 1 &&
              std::fwrite(s->hitables, sizeof(rtow_hitable), s->n_hitables, f) == s->n_hitables &&
              std::fwrite(s->refs, 4, s->n_refs, f) == s->n_refs &&
              std::fwrite(s->materials, sizeof(rtow_material), s->n_materials, f) == s->n_materials &&
              std::fwrite(s->textures, sizeof(rtow_texture), s->n_textures, f) == s->n_textures &&
              (!s->perlin || std::fwrite(s->perlin, sizeof(rtow_perlin), 1, f) == 1) &&
              std::fwrite(s->images, sizeof(rtow_image), s->n_images, f) == s->n_images &&
              std::fwrite(s->texels, 1, (size_t)ntex, f) == (size_t)ntex;
    std::fclose(f);
    return ok ? RTOW_OK : set_error(RTOW_E_IO, "short write");
}

int rtow_scene_load(const char* path, rtow_scene_buf** out) {
    if (!path || !out) return set_error(RTOW_E_INVALID, "NULL argument");
    std::ifstream f(path, std::ios::binary);
    if (!f) return set_error(RTOW_E_IO, std::string("cannot open ") + path);
    std::vector<char> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (b.size() < 56 || std::memcmp(b.data(), "RTOWSCN1", 8) != 0) return set_error(RTOW_E_IO, "not a scene file");
    uint32_t hdr[10];
    uint64_t ntex;
    std::memcpy(hdr, b.data() + 8, 40);
    std::memcpy(&ntex, b.data() + 48, 8);
    size_t need = 56 + (size_t)hdr[2] * sizeof(rtow_hitable) + (size_t)hdr[3] * 4 +
                  (size_t)hdr[4] * sizeof(rtow_material) + (size_t)hdr[5] * sizeof(rtow_texture) +
                  (hdr[7] ? sizeof(rtow_perlin) : 0) + (size_t)hdr[6] * sizeof(rtow_image) + ntex;
    if (need != b.size()) return set_error(RTOW_E_IO, "scene file size mismatch");
    auto* sb = new rtow_scene_buf;
    SceneGraph& g = sb->g;
    const char* p = b.data() + 56;
    auto take = [&](auto& vec, size_t n) {
        using T = typename std::decay_t<decltype(vec)>::value_type;
        vec.resize(n);
        std::memcpy(vec.data(), p, n * sizeof(T));
        p += n * sizeof(T);
    };
    g.root = hdr[1];
    take(g.hitables, hdr[2]);
    take(g.refs, hdr[3]);
    take(g.materials, hdr[4]);
    take(g.textures, hdr[5]);
    if (hdr[7]) {
        std::memcpy(&g.perlin, p, sizeof(rtow_perlin));
        p += sizeof(rtow_perlin);
    } else {
        std::memset(&g.perlin, 0, sizeof(rtow_perlin));
    }
    take(g.images, hdr[6]);
    take(g.texels, (size_t)ntex);
    sb->view = g.view();
    *out = sb;
    return RTOW_OK;
}

int rtow_camera_main(uint32_t width, uint32_t height, rtow_camera* out) {
    if (!out || width == 0 || height == 0) return set_error(RTOW_E_INVALID, "bad camera arguments");
    *out = mainCamera(width, height).toDevice();
    return RTOW_OK;
}

int rtow_camera_oriented(uint32_t width, uint32_t height, const float look_from[3], const float rows[9],
                         rtow_camera* out) {
    if (!out || !look_from || !rows || width == 0 || height == 0)
        return set_error(RTOW_E_INVALID, "bad camera arguments");
    Camera c = mainCamera(width, height);
    c.setOrientationRows(vec3(rows[0], rows[1], rows[2]), vec3(rows[3], rows[4], rows[5]),
                         vec3(rows[6], rows[7], rows[8]));
    c.setLookFromPoint(vec3(look_from[0], look_from[1], look_from[2]));
    *out = c.toDevice();
    return RTOW_OK;
}

int rtow_camera_look_at(const float look_from[3], const float look_at[3], const float up[3], float vfov_deg,
                        float aspect, float aperture, float focus_distance, float time0, float time1,
                        rtow_camera* out) {
    if (!out || !look_from || !look_at || !up) return set_error(RTOW_E_INVALID, "bad camera arguments");
    Camera c(vec3(look_from[0], look_from[1], look_from[2]), vec3(look_at[0], look_at[1], look_at[2]),
             vec3(up[0], up[1], up[2]), vfov_deg, aspect, aperture, focus_distance, time0, time1);
    c.setCamera_Euler();
    *out = c.toDevice();
    return RTOW_OK;
}

void rtow_synthetic_image(uint32_t nx, uint32_t ny, uint8_t* rgb) {
    // r = 255*i/(nx-1), g = 255*j/(ny-1), b = 40 + 160*checker32 + (i*j & 31)
    // (tests/scene_io.py:synthetic_image is the same formula)
    const uint64_t dx = nx > 1 ? nx - 1 : 1, dy = ny > 1 ? ny - 1 : 1;
    for (uint64_t j = 0; j < ny; j++)
        for (uint64_t i = 0; i < nx; i++) {
            uint8_t* px = rgb + 3 * (j * nx + i);
            px[0] = (uint8_t)((i * 255) / dx);
            px[1] = (uint8_t)((j * 255) / dy);
            px[2] = (uint8_t)(40 + 160 * (((i >> 5) + (j >> 5)) & 1) + ((i * j) & 31));
        }
}

}  // extern "C"
