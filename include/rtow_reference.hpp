/* rtow_reference.hpp -- the reference-side half of the drop-in (header only).
 *
 * Compiled INSIDE the reference's own translation unit, after its scenes.h
 * (which brings every Hitable / Material / Texture class) and camera.h, it
 * turns what the reference builds into what librtow_hip.so takes:
 *
 *   rtow_ref::World w(world);            // the Hitable* of main.cpp:128-137
 *   if (w.status() != RTOW_OK) ...       // an object class the C-ABI has no record for
 *   rtow_scene_upload(ctx, w.view());    // include/rtow.h
 *   rtow_camera cam;
 *   rtow_ref::camera(mainCamera, &cam);  // the basis Camera::getRay reads
 *   rtow_params params;
 *   rtow_ref::params(W, H, spp, &params);  // defines.h of this build (DOF, GI gains, depth)
 *   rtow_render(ctx, &cam, &params, bgra, nullptr, &stats);
 *
 * World walks the object graph depth first in the canonical order
 * include/rtow.h documents (a node's record is reserved before its children
 * are visited; shared objects are flattened once), so it yields byte for
 * byte the arrays the product's own scene builders produce for the same
 * world (tests/test_reference_binding.py checks that against every golden
 * scene).  Every class is read through its public members; the hit/scatter/
 * value functions of hitable.h:19-23, material.h:34-41 and texture.h:6-9 are
 * not called -- the GPU runs them (rtow_device.hip), the C oracle restates
 * them for the tests.  The Perlin tables are the reference's static ones
 * (noise.h:112-116).
 *
 * camera() reads the Camera through its public getters (camera.h:186-262)
 * and evaluates setCamera_QuaternionMatrix (camera.h:315-342) with the same
 * expressions in the same translation unit, so the basis is the one the
 * Camera holds privately, bit for bit.
 *
 * Needs only include/rtow.h.  Not compiled into librtow_hip.so (it depends
 * on the reference's classes); INTEGRATION.md shows the call site. */
#ifndef RTOW_REFERENCE_HPP
#define RTOW_REFERENCE_HPP

#include <cmath>
#include <cstdint>
#include <map>
#include <vector>

#include "rtow.h"

namespace rtow_ref {

class World {
public:
    explicit World(const Hitable* root) {
        root_ = hitable(root);
        for (int i = 0; i < 256; i++) {  // noise.h:112-116, the static tables
            perlin_.ranfloat[i] = Perlin::randFloat[i];
            perlin_.ranvec[i][0] = Perlin::randVector[i].x();
            perlin_.ranvec[i][1] = Perlin::randVector[i].y();
            perlin_.ranvec[i][2] = Perlin::randVector[i].z();
            perlin_.perm_x[i] = Perlin::permX[i];
            perlin_.perm_y[i] = Perlin::permY[i];
            perlin_.perm_z[i] = Perlin::permZ[i];
        }
        view_.root = root_;
        view_.n_hitables = (uint32_t)hit_.size();
        view_.hitables = hit_.data();
        view_.n_refs = (uint32_t)refs_.size();
        view_.refs = refs_.data();
        view_.n_materials = (uint32_t)mats_.size();
        view_.materials = mats_.data();
        view_.n_textures = (uint32_t)texs_.size();
        view_.textures = texs_.data();
        view_.perlin = &perlin_;
        view_.n_images = (uint32_t)imgs_.size();
        view_.images = imgs_.data();
        view_.n_texel_bytes = texels_.size();
        view_.texels = texels_.data();
    }
    World(const World&) = delete;
    World& operator=(const World&) = delete;

    /* RTOW_OK, or RTOW_E_UNSUPPORTED when the graph holds an object class
     * (or a NULL pointer) the flattened layout has no record for; the
     * offending records are left zeroed and the scene must not be uploaded. */
    int status() const { return unknown_ ? RTOW_E_UNSUPPORTED : RTOW_OK; }
    uint32_t unknown_objects() const { return unknown_; }
    /* Valid as long as this World lives. */
    const rtow_scene* view() const { return &view_; }

private:
    static void v3(float* d, const vec3& v) {
        d[0] = v.x();
        d[1] = v.y();
        d[2] = v.z();
    }

    // ImageTexture pixels (texture.h:55-85: RGB8, nx * ny * 3 bytes)
    uint32_t image(const unsigned char* data, int nx, int ny) {
        auto it = img_of_.find(data);
        if (it != img_of_.end()) return it->second;
        const uint32_t idx = (uint32_t)imgs_.size();
        rtow_image im{};
        im.nx = (uint32_t)nx;
        im.ny = (uint32_t)ny;
        im.channels = 3;
        im.offset = texels_.size();
        if (data && nx > 0 && ny > 0) texels_.insert(texels_.end(), data, data + (size_t)nx * ny * 3);
        imgs_.push_back(im);
        img_of_[data] = idx;
        return idx;
    }

    uint32_t texture(const Texture* t) {  // texture.h, noise.h
        auto it = tex_of_.find(t);
        if (it != tex_of_.end()) return it->second;
        const uint32_t idx = (uint32_t)texs_.size();
        texs_.push_back(rtow_texture{});
        tex_of_[t] = idx;
        rtow_texture r{};
        if (auto c = dynamic_cast<const ConstantTexture*>(t)) {
            r.kind = RTOW_TEX_CONSTANT;
            v3(r.f, c->_color);
        } else if (auto k = dynamic_cast<const CheckerTexture*>(t)) {
            r.kind = RTOW_TEX_CHECKER;
            r.a = texture(k->_odd);
            r.b = texture(k->_even);
        } else if (auto n = dynamic_cast<const NoiseTexture*>(t)) {
            r.kind = RTOW_TEX_NOISE;
            r.f[0] = n->_scaled;
            r.a = n->_filter ? 1 : 0;
        } else if (auto im = dynamic_cast<const ImageTexture*>(t)) {
            r.kind = RTOW_TEX_IMAGE;
            r.a = image(im->_data, im->_nx, im->_ny);
        } else {
            unknown_++;
        }
        texs_[idx] = r;
        return idx;
    }

    uint32_t material(const Material* m) {  // material.h
        auto it = mat_of_.find(m);
        if (it != mat_of_.end()) return it->second;
        const uint32_t idx = (uint32_t)mats_.size();
        mats_.push_back(rtow_material{});
        mat_of_[m] = idx;
        rtow_material r{};
        if (auto l = dynamic_cast<const Lambertian*>(m)) {
            r.kind = RTOW_MAT_LAMBERTIAN;
            r.texture = texture(l->_albedo);
        } else if (auto me = dynamic_cast<const Metal*>(m)) {
            r.kind = RTOW_MAT_METAL;
            v3(r.albedo, me->_albedo);
            r.param = me->_fuzz;
        } else if (auto d = dynamic_cast<const Dielectric*>(m)) {
            r.kind = RTOW_MAT_DIELECTRIC;
            r.param = d->_refIndex;
        } else if (auto dl = dynamic_cast<const DiffuseLight*>(m)) {
            r.kind = RTOW_MAT_DIFFUSE_LIGHT;
            r.texture = texture(dl->_emit);
        } else if (auto is = dynamic_cast<const Isotropic*>(m)) {
            r.kind = RTOW_MAT_ISOTROPIC;
            r.texture = texture(is->_albedo);
        } else {
            unknown_++;
        }
        mats_[idx] = r;
        return idx;
    }

    uint32_t hitable(const Hitable* h) {  // sphere.h, xy_rect.h, hitable.h, hitableList.h, box.h, bvhNode.h, constantMedium.h
        auto it = hit_of_.find(h);
        if (it != hit_of_.end()) return it->second;
        const uint32_t idx = (uint32_t)hit_.size();
        hit_.push_back(rtow_hitable{});
        hit_of_[h] = idx;
        rtow_hitable r{};
        if (auto s = dynamic_cast<const Sphere*>(h)) {
            r.kind = RTOW_HIT_SPHERE;
            v3(r.f, s->_center);
            r.f[3] = s->_radius;
            r.a = material(s->_materialPointer);
        } else if (auto ms = dynamic_cast<const MovingSphere*>(h)) {
            r.kind = RTOW_HIT_MOVING_SPHERE;
            v3(r.f, ms->_center0);
            v3(r.f + 3, ms->_center1);
            r.f[6] = ms->_time0;
            r.f[7] = ms->_time1;
            r.f[8] = ms->_radius;
            r.a = material(ms->_materialPointer);
        } else if (auto q = dynamic_cast<const XYRectangle*>(h)) {
            r.kind = RTOW_HIT_RECT_XY;
            r.f[0] = q->_x0, r.f[1] = q->_x1, r.f[2] = q->_y0, r.f[3] = q->_y1, r.f[4] = q->_k;
            r.a = material(q->_material);
        } else if (auto q = dynamic_cast<const XZRectangle*>(h)) {
            r.kind = RTOW_HIT_RECT_XZ;
            r.f[0] = q->_x0, r.f[1] = q->_x1, r.f[2] = q->_z0, r.f[3] = q->_z1, r.f[4] = q->_k;
            r.a = material(q->_material);
        } else if (auto q = dynamic_cast<const YZRectangle*>(h)) {
            r.kind = RTOW_HIT_RECT_YZ;
            r.f[0] = q->_y0, r.f[1] = q->_y1, r.f[2] = q->_z0, r.f[3] = q->_z1, r.f[4] = q->_k;
            r.a = material(q->_material);
        } else if (auto fl = dynamic_cast<const FlipNormals*>(h)) {
            r.kind = RTOW_HIT_FLIP_NORMALS;
            r.a = hitable(fl->_hitable);
        } else if (auto tr = dynamic_cast<const Translate*>(h)) {
            r.kind = RTOW_HIT_TRANSLATE;
            v3(r.f, tr->_offset);
            r.a = hitable(tr->_hitablePointer);
        } else if (auto ro = dynamic_cast<const RotateY*>(h)) {
            r.kind = RTOW_HIT_ROTATE_Y;
            r.f[0] = ro->_sinTheta;
            r.f[1] = ro->_cosTheta;
            r.b = ro->_hasBox ? 1 : 0;
            v3(r.f + 2, ro->_boundBox.min());
            v3(r.f + 5, ro->_boundBox.max());
            r.a = hitable(ro->_pointer);
        } else if (auto li = dynamic_cast<const HitableList*>(h)) {
            r.kind = RTOW_HIT_LIST;
            r.a = (uint32_t)refs_.size();
            r.b = (uint32_t)li->_listSize;
            refs_.resize(refs_.size() + (size_t)li->_listSize);
            for (uint32_t i = 0; i < r.b; i++) {
                const uint32_t c = hitable(li->_hitableList[i]);
                refs_[r.a + i] = c;
            }
        } else if (auto bx = dynamic_cast<const Box*>(h)) {
            r.kind = RTOW_HIT_BOX;
            v3(r.f, bx->_pMin);
            v3(r.f + 3, bx->_pMax);
            r.a = hitable(bx->_hitableList);
        } else if (auto bv = dynamic_cast<const BvhNode*>(h)) {
            r.kind = RTOW_HIT_BVH_NODE;
            v3(r.f, bv->_box.min());
            v3(r.f + 3, bv->_box.max());
            r.a = hitable(bv->_left);
            r.b = hitable(bv->_right);
        } else if (auto cm = dynamic_cast<const ConstantMedium*>(h)) {
            r.kind = RTOW_HIT_CONSTANT_MEDIUM;
            r.f[0] = cm->_density;
            r.a = hitable(cm->_boundary);
            r.b = material(cm->_phaseFunction);
        } else {
            unknown_++;
        }
        hit_[idx] = r;
        return idx;
    }

    uint32_t root_ = 0, unknown_ = 0;
    std::vector<rtow_hitable> hit_;
    std::vector<uint32_t> refs_;
    std::vector<rtow_material> mats_;
    std::vector<rtow_texture> texs_;
    std::vector<rtow_image> imgs_;
    std::vector<uint8_t> texels_;
    rtow_perlin perlin_{};
    std::map<const void*, uint32_t> hit_of_, mat_of_, tex_of_, img_of_;
    rtow_scene view_{};
};

/* The basis Camera::getRay (camera.h:123-135) reads, from the camera's public
 * getters: setCamera_QuaternionMatrix (camera.h:315-342) evaluated with the
 * same expressions, in the reference's own translation unit. */
inline int camera(Camera& c, rtow_camera* out) {
    if (!out) return RTOW_E_INVALID;
    const vec3 lookFrom = c.getLookFromPoint();
    const mat4x4 om = c.getOrientationMatrix();
    const float vFoV = c.setVerticalFoV(), aspect = c.setAspect();  // the reference's getters carry "set" names
    const float aperture = c.setAperture(), focusDistance = c.setFocusDistance();
    float t0, t1;
    c.getTime(t0, t1);

    const float lensRadius = aperture / 2;
    const float theta = vFoV * M_PI / 180;
    const float half_height = tan(theta / 2);
    const float half_width = aspect * half_height;
    const vec3 origin = lookFrom;
    const vec3 w = vec3(om.m[0][0], om.m[0][1], om.m[0][2]);
    const vec3 u = vec3(om.m[1][0], om.m[1][1], om.m[1][2]);
    const vec3 v = vec3(om.m[2][0], om.m[2][1], om.m[2][2]);
    const vec3 lowerLeftCorner = origin - half_width * focusDistance * u - half_height * focusDistance * v -
                                 focusDistance * w;
    const vec3 horizontal = 2 * half_width * focusDistance * u;
    const vec3 vertical = 2 * half_height * focusDistance * v;

    const vec3* src[7] = {&origin, &lowerLeftCorner, &horizontal, &vertical, &u, &v, &w};
    float* dst[7] = {out->origin, out->lower_left_corner, out->horizontal, out->vertical, out->u, out->v, out->w};
    for (int k = 0; k < 7; k++) {
        dst[k][0] = src[k]->x();
        dst[k][1] = src[k]->y();
        dst[k][2] = src[k]->z();
    }
    out->lens_radius = lensRadius;
    out->time0 = t0;
    out->time1 = t1;
    return RTOW_OK;
}

/* The render parameters of THIS build of the reference: defines.h as the
 * translation unit sees it (GLOBAL_ILLUM_EN, SKY_ILLUM_GAIN,
 * GLOBAL_ILLUM_GAIN, DEPTH_RECURSION, CAMERA_DOF_EN -> RTOW_FLAG_CAMERA_DOF),
 * over rtow_params_default's values for anything defines.h leaves out. */
inline void params(uint32_t width, uint32_t height, uint32_t spp, rtow_params* out) {
    rtow_params_default(out, width, height, spp);
#ifdef GLOBAL_ILLUM_EN
    out->gi_enable = GLOBAL_ILLUM_EN ? 1u : 0u;
#endif
#ifdef SKY_ILLUM_GAIN
    out->sky_gain = (float)SKY_ILLUM_GAIN;
#endif
#ifdef GLOBAL_ILLUM_GAIN
    out->gi_gain = (float)GLOBAL_ILLUM_GAIN;
#endif
#ifdef DEPTH_RECURSION
    out->max_depth = DEPTH_RECURSION;
#endif
#if defined(CAMERA_DOF_EN) && CAMERA_DOF_EN == 1
    out->flags |= RTOW_FLAG_CAMERA_DOF;
#endif
}

}  // namespace rtow_ref

#endif  // RTOW_REFERENCE_HPP
