// rtow_layout.h -- the scene graph (include/rtow.h: one record per reference
// object) converted into the arrays the gfx950 kernels read
// (rtow_device_layout.h).  Host code only: rtow_layout.cpp builds the layout,
// rtow_device.hip's rtow_scene_upload copies it to the device.
#pragma once

#include <hip/hip_runtime.h>  // float4 (DChainX)

#include <cstdint>
#include <unordered_map>
#include <vector>

#include "../../include/rtow.h"
#include "rtow_device_layout.h"

namespace rtow_layout {
using namespace rtow_dev;

struct HostLayout {
    std::vector<DBvh> bvh;
    std::vector<DNode> node;
    std::vector<DSphere> sph;
    std::vector<DRect> rect;
    std::vector<DInst> inst;
    std::vector<DList> list;
    std::vector<uint32_t> refs;
    std::vector<DMedium> med;
    std::vector<DMat> mat;
    std::vector<DTex> tex;
    std::vector<float> ranvec;
    std::vector<uint32_t> perm;
    std::vector<DImage> img;
    std::vector<uint8_t> texels;
    uint32_t root = 0;
    uint32_t stack_need = 0;
    uint32_t chain_need = 0;
    bool has_media = false;
    bool media_any = false;
    bool gnode = false;
    bool media_nested = false;  // a medium the general traversal must ask (not a TOP_MEDIUM item)
    bool simple = false;
    bool unit_time = true;
    uint32_t root_chain_n = 0;
    uint32_t root_chain[4] = {0, 0, 0, 0};
    uint32_t bvh_root = 0;
    std::vector<unsigned long long> sph_key, rect_key, med_key;
    std::vector<DChain> chains;
    std::vector<DTop> top;
    std::vector<DSphere> tsph;       // grid worlds: copies of the top-level spheres, by run (DevScene::tsph)
    std::vector<float> bvh_own;      // 6 per reference BvhNode slot: its own box (bvhNode.h:58)
    // n == 1 BvhNodes (collapsed into their leaf): the leaf's ref -> index of
    // the node's own box (6 floats) in collapsed_own; AABB::hit still tests it
    std::vector<float> collapsed_own;
    std::unordered_map<uint32_t, uint32_t> collapsed_of;
    std::vector<uint32_t> rect_lvl;  // DevScene::rect_lvl
    std::vector<unsigned long long> rect_lmask;  // DevScene::rect_lmask
    std::vector<uint32_t> rect_anc;  // DevScene::rect_anc
    std::vector<float> abox;         // DevScene::abox
    std::vector<DProg> prog;         // DevScene::prog
    std::vector<DBox6> box6;         // DevScene::box6
    std::vector<DGrid> grid;         // DevScene::grid (TOP_GRID)
    std::vector<DGridCell> gcell;    // DevScene::gcell
    std::vector<uint32_t> gq;        // DevScene::gq: gcell's extents packed (grid_ext), one word each
    std::unordered_map<uint32_t, uint32_t> grid_of;  // a grid's BvhNode ref -> its DGrid
    uint32_t grid_top = 0;           // TOP_GRID items of the top-level list (DevScene::n_grid)
    float tshift[3] = {0.0f, 0.0f, 0.0f};  // DevScene::tshift
    // exact-order worlds (MODE 6, xhit): the raw scene graph
    bool exact = false;
    std::vector<XHit> xh;
    std::vector<uint32_t> xrefs;
    uint32_t xroot = 0;
    uint32_t xdepth = 0;  // rawDepth of the raw graph (general and exact worlds): xhit's frames per thread
};

// Convert scene `s` (tree: RTOW_TREE_SAH or RTOW_TREE_REFERENCE) into `L`;
// RTOW_OK or an error code (set_error).
int buildLayout(const rtow_scene& s, HostLayout& L, int tree = RTOW_TREE_SAH);

}  // namespace rtow_layout
