// rtow_device_layout.h — the scene as the gfx950 kernels read it from HBM.
//
// rtow_scene_upload() converts the scene graph (include/rtow.h, one record per
// reference object) into these arrays:
//
//   * references are tagged 32-bit words: kind in bits 28..31, index below;
//   * every reference BvhNode becomes a 64-byte DBvh holding BOTH children's
//     boxes as an x/y/z-plane SoA (three float4 + the two child refs), so one
//     node visit is four 16-byte loads and two slab tests, and traversal can
//     visit the nearer child first.  A BvhNode with left == right
//     (bvhNode.h:38-39, n == 1) collapses into its leaf.  The box stored for a
//     BvhNode child is that node's own box (bvhNode.h:58); a sphere/moving
//     sphere/rectangle child gets its exact bounding box; any other child an
//     infinite box, so a list's buggy box (hitableList.h:52-53) never culls;
//   * Box (box.h:43-45) becomes its 6-side list; FlipNormals/Translate/RotateY
//     are instance records applied on the way in and, for the winning hit, on
//     the way out (hitable.h:25-154).
#pragma once

#include <stdint.h>

namespace rtow_dev {

enum : uint32_t {
    DK_BVH = 0,
    DK_SPHERE = 1,
    DK_MSPHERE = 2,  // a sphere leaf reached through a general DNode's box slot (not inlined: time0/time1 not 0/1)
    DK_RECT = 3,
    DK_LIST = 4,
    DK_TRANSLATE = 5,
    DK_ROTY = 6,
    DK_FLIP = 7,
    DK_MEDIUM = 8,
    DK_EXIT = 9,  // traversal-stack marker: leave the innermost instance
    DK_LISTNEXT = 10,  // traversal-stack marker: continue a list at refs[index]
    DK_RECTS = 11,     // a list of rectangles only (a Box's sides): DList over rect[first, first+count)
    DK_PROG = 12,      // a BvhNode subtree holding media, visited as the reference visits it (DProg)
    DK_PROGNEXT = 13,  // traversal-stack marker: continue a DProg program at prog[index]
    DK_BOX6 = 14,      // a general DNode slot holding a Box (index into box6): its sides scanned in the node step
    DK_NONE = 15
};

constexpr uint32_t KIND_SHIFT = 28;
constexpr uint32_t INDEX_MASK = (1u << KIND_SHIFT) - 1;
constexpr uint32_t mkref(uint32_t kind, uint32_t idx) { return (kind << KIND_SHIFT) | idx; }
// A leaf reference held as a traversal's record (sphere, rectangle, medium)
// carries tie bits above its index: the first key bit where it and the leaf
// it tied with part (+1; 0: no exact tie), for tie_unsettled.  Leaf indices
// stay below 2^21 (checked at upload).
constexpr uint32_t LEAF_BITS = 21;
constexpr uint32_t LEAF_MASK = (1u << LEAF_BITS) - 1;
constexpr uint32_t TIE_SHIFT = LEAF_BITS;
constexpr uint32_t TIE_MASK = 0x7Fu << TIE_SHIFT;

struct alignas(16) DBvh {  // 64 B
    float xs[4];  // left.min.x, left.max.x, right.min.x, right.max.x
    float ys[4];
    float zs[4];
    uint32_t left, right, pad0, pad1;
};

// Node of the "simple scene" traversal (BvhNodes + spheres, every sphere with
// time0 = 0, time1 = 1): 64 B, two 32-B child slots.  A slot holds either an
// inner child (box min xyz, max xyz, 0, ref DK_BVH) or the sphere leaf itself
// (center0 xyz, radius * radius, center1 - center0 xyz, ref DK_SPHERE | sphere index),
// so one node fetch carries everything a step needs.  Empty: ref DK_NONE.
// General scenes (SAH mode, DevScene::gnode) use the same record as the twin
// of every DBvh (same index): a sphere child with time0 = 0, time1 = 1 is
// inlined, any other child is a box slot whose ref is the child (a
// non-inlined sphere as DK_MSPHERE).
struct alignas(16) DNode {
    float a[7];
    uint32_t ref_a;
    float b[7];
    uint32_t ref_b;
};

// Sphere (sphere.h:7-18) and MovingSphere (sphere.h:76-91) share one leaf:
// a static sphere is stored with center1 = center0, time0 = 0, time1 = 1, and
// center(time) = c0 + ((time-0)/(1-0)) * (c0-c0) = c0 exactly, so one test
// reproduces both classes bit for bit.  `moving` keeps MovingSphere's missing
// u,v (sphere.h:93-118 never writes them).
// dc = center1 - center0 is computed once on the host: the same float
// subtraction center() performs on every call (sphere.h:130).
// Leaves carry `chain`: the index in DevScene::chains of the instance chain
// (root first) their path from the root passes through, so a hit record needs
// only the leaf to be carried out of its instances.  (Every node is reached
// on one path: rtow_scene_upload rejects an instance shared under two
// different chains.)
struct alignas(16) DSphere {  // 48 B
    float c0[3], r;
    float dc[3], t0;
    float t1;
    uint32_t mat, moving, chain;
};

// xy_rect.h; axis & 3: 0 XY (k on z), 1 XZ (k on y), 2 YZ (k on x).
// axis & RECT_FLIP: a FlipNormals directly above the rectangle (hitable.h:28-36)
// folded into the leaf.
constexpr uint32_t RECT_FLIP = 4u;
// finalize's "needs uv" bits, set once the materials are known (buildLayout):
// DRect::axis & RECT_UV, DSphere::moving & SPH_UV (a static sphere whose
// material reads (u, v)); bit 0 of DSphere::moving stays "moving"
constexpr uint32_t RECT_UV = 8u;
constexpr uint32_t SPH_UV = 2u;
struct alignas(16) DRect {  // 32 B
    float a0, a1, b0, b1;
    float k;
    uint32_t axis, mat, chain;
};

// TRANSLATE p = offset; ROTY p[0] sin, p[1] cos; FLIP -.  parent_chain: the
// chain in force where the instance sits (restored when the traversal leaves it).
struct alignas(16) DInst {  // 32 B
    uint32_t child, parent_chain;
    float p[6];
};

constexpr int MAXCHAIN = 7;
struct alignas(16) DChain {  // 32 B: instance refs, outermost first
    uint32_t n;
    uint32_t ref[MAXCHAIN];
};
// The device's copy of a chain: the instances' parameters inline (no second
// dependent load per chain walk): per instance (ref bits, p0, p1, p2) --
// Translate offset, or RotateY sine and cosine (DInst::p)
struct alignas(16) DChainX {  // 128 B
    float4 t[MAXCHAIN];
    uint32_t n, pad[3];
};

struct alignas(16) DList {  // 16 B: children at refs[first .. first+count)
    uint32_t first, count;
    uint32_t box6;  // DK_RECTS: 1 + index in DevScene::box6 when the six rectangles are a Box's (0: no)
    uint32_t pad1;
};

// A Box's six sides (box.h:25-41: XY at z1 and z0, XZ at y1 and y0, YZ at x1
// and x0, in that list order) as its two corners: the six rectangle tests of
// rect[first .. first+5] unrolled with their axes known at compile time
// (box6_scan), same arithmetic, same order.
struct alignas(16) DBox6 {  // 32 B
    float lo[3];
    uint32_t first;
    float hi[3];
    uint32_t pad;
};

// bkind: how the kernel queries the boundary (rtow_device.hip medium_hit):
// MB_SPHERE a plain sphere (both roots from one quadratic), MB_RECTS instances
// over a Box's rectangles rect[bfirst, +bcount) whose frame is chain bchain,
// MB_ANY the general traversal.
enum : uint32_t { MB_ANY = 0, MB_SPHERE = 1, MB_RECTS = 2, MB_BOX6 = 3 };  // MB_BOX6: bfirst = box6 index
struct alignas(16) DMedium {  // 32 B, constantMedium.h:21-23
    uint32_t boundary, phase_mat;
    float inv_density;  // 1 / density, the float quotient constantMedium.h:47 forms (host IEEE division)
    uint32_t chain;
    uint32_t bkind, bfirst, bcount, bchain;
};

// A BvhNode subtree with ConstantMedium leaves.  BvhNode::hit (bvhNode.h:66-96)
// tests its own box (AABB::hit, aabb.h:22-43) with the interval it was handed
// and then BOTH children with that same interval; a medium draws a number on
// every call (constantMedium.h:27, a second one when the ray crosses its
// boundary), so which media are called, how often and in what order is the
// reference's exhaustive depth-first visit -- the device replays it as a
// flat program, one entry per step:
//   PROG_BOX  the node's own box (lo, hi); when AABB::hit fails, skip the
//             `arg` entries of its children's programs;
//   PROG_ITEM `arg` is a child the visit order does not matter for (no media
//             below it: its closest hit merges by the tie keys) or a medium,
//             called with the subtree's interval;
//   PROG_END  the end of the program.
// An n == 1 node (bvhNode.h:38-39) calls its one leaf twice: two ITEMs.
enum : uint32_t { PROG_BOX = 0, PROG_ITEM = 1, PROG_END = 2 };
struct alignas(16) DProg {  // 32 B; lo/hi read as ref_aabb_hit's (min xyz, -, max xyz, -)
    float lo[3];
    uint32_t op;
    float hi[3];
    uint32_t arg;
};

// The top-level list of a general scene (below the root's instances), as the
// kernel scans it: item by item with the whole wave on the same item, so the
// descriptors are read with uniform (scalar) loads and the wave stays
// together.  An item that is a chain of instances over one sphere, one
// rectangle or a Box's rectangles is tested in place (the leaf's chain gives
// the ray in the leaf's frame); a medium whose boundary is a sphere or a
// Box's rectangles (MB_SPHERE / MB_RECTS) is asked right there (TOP_MEDIUM,
// with the closest hit so far as its tmax, hitableList.h:30); anything else
// goes to the general traversal -- except a chain of instances over a BvhNode
// of unit-time spheres only (final_ned's cloud, Translate(RotateY(BvhNode of
// 1000 spheres))): TOP_SPHERES runs its DNode tree in a loop of its own
// (trace_dnodes) in the leaves' frame, entered once per ray; and so does a
// BvhNode whose leaves are only spheres, rectangles and Boxes, with no
// instance, list or medium below it (TOP_DTREE: final_ned's first tree).
// A BvhNode whose leaves are Boxes tiling a regular grid of columns (final_ned's
// 20 x 20 ground: equal cells along two axes, any extent along the third) is
// walked as that grid (TOP_GRID, MODE 8): see DGrid.
enum : uint32_t {
    TOP_GENERIC = 0,
    TOP_RECTS = 1,
    TOP_SPHERE = 2,
    TOP_MEDIUM = 3,
    TOP_BOX6 = 4,
    TOP_SPHERES = 5,
    TOP_DTREE = 6,
    TOP_GRID = 7
};
// DTop::kind flags above the kind (buildTop): the item's frame differs from
// the previous in-place item's (the scan recomputes its ray), and so does the
// ray's direction there (it recomputes 1/d and dot(d, d) too)
enum : uint32_t { TOP_KIND_MASK = 255u, TOP_NEWCHAIN = 1u << 8, TOP_NEWDIR = 1u << 9 };
// BOX6: a = box6 index; SPHERES, DTREE: a = the DNode index of the BvhNode
struct alignas(16) DTop {  // 16 B
    uint32_t kind;
    uint32_t a;      // GENERIC: item ref; RECTS: first rectangle; SPHERE: sphere; MEDIUM: medium
    uint32_t b;      // RECTS: count
    uint32_t chain;  // the chain of the leaf's frame (GENERIC: of the list's frame)
};

// TOP_GRID (a = grid index): Boxes whose extents along axes au and av are
// exactly the cells [u0 + i wu, u0 + (i+1) wu] x [v0 + j wv, v0 + (j+1) wv] of an
// nu x nv grid, one Box per cell, any extent [hlo, hhi] along the third axis ah
// (a heightfield of columns).  Cell (i, j) is gcell[cell0 + j nu + i], row j
// (its columns together: hlo, hhi) gcell[cell0 + nu nv + j].  The
// kernel walks the cells the ray crosses in order (rows along v, cells along u
// within a row), every cell widened by `margin`, and scans the Box of every
// cell the ray passes at a height the Box spans -- the same box6_scan the tree
// runs, so the closest hit and its tie keys are the tree's.
struct alignas(16) DGrid {  // 64 B
    float u0, v0, wu, wv;
    float iwu, iwv;   // 1 / wu, 1 / wv (rounded: cell indices are estimates, the margins cover them)
    float hlo, hhi;   // the columns' extent along ah, over all cells
    float u1, v1;     // the grid's far corner (every Box lies within [u0, u1] x [v0, v1])
    uint32_t nu, nv;
    uint32_t axes;    // au | av << 2 | ah << 4
    uint32_t cell0;
    float margin;     // spatial widening of every cell (and of the grid's box)
    uint32_t box0;    // cell (i, j)'s Box is DBox6 box0 + j nu + i (copies in cell order: no index load)
};
struct alignas(16) DGridCell {  // 16 B
    float hlo, hhi;  // the Box's extent along ah
    uint32_t box6;   // its DBox6
    uint32_t pad;
};

struct alignas(16) DMat {  // 32 B
    uint32_t kind, tex, needs_uv;
    float inv_ri;  // Dielectric: (float)(1.0 / ref_idx), material.h:97
    float param;
    float albedo[3];
};

struct alignas(16) DTex {  // 48 B: rtow_texture (32 B), then g
    uint32_t kind, a, b, c;
    float f[4];
    float g[4];  // a CHECKER whose two textures are CONSTANT (c & TEX_FLAT): odd colour in f, even in g
};
// DTex::c of a CheckerTexture: its odd / even colours inline (texture_at), no
// further texture record to load
constexpr uint32_t TEX_FLAT = 1u;
// DMat::tex of a Lambertian / DiffuseLight / Isotropic whose texture is a
// ConstantTexture: the colour is inline in DMat::albedo (texture_at)
constexpr uint32_t TEX_INLINE = 0xffffffffu;

struct alignas(16) DImage {
    uint32_t nx, ny;
    uint64_t offset;
};

// DevScene::root_chain: the instances above a simple scene's BvhNode tree
constexpr int ROOTCHAIN = 4;
// MODE 8 at STACK 16 stages the grids' packed cell heights (DevScene::gq) in
// LDS after the COLD words when they fit in this many words (4 blocks of 256
// threads then take 4 x 40 KB of the CU's 160 KB); larger tables go to the
// STACK 20 kernel, which reads them from global memory.
constexpr uint32_t GRID_LDS_WORDS = 512;

// Pointers into one device allocation + scene-wide facts the launch needs.
struct DevScene {
    const DBvh* bvh;
    const DNode* node;       // simple scenes only
    const DSphere* sph;
    const DRect* rect;
    const DInst* inst;
    const DList* list;
    const uint32_t* refs;
    const DMedium* med;
    const DChainX* chains;
    const DTop* top;         // general scenes: the top-level list, n_top items (0: none)
    const DProg* prog;       // programs of the BvhNode subtrees that hold media (DK_PROG)
    const DBox6* box6;       // Boxes among the rectangle lists (DList::box6, TOP_BOX6, MB_BOX6)
    const DGrid* grid;       // TOP_GRID items (MODE 8)
    const DGridCell* gcell;
    const uint32_t* gq;      // gcell's extents packed to 16-bit steps (grid_ext), staged in LDS by MODE 8
    uint32_t n_gq;
    uint32_t n_grid;
    uint32_t n_top;
    // Per rectangle: (offset << 8) | count of the boxes (8 floats each in
    // abox: min xyz, 0, max xyz, 0) of the reference BvhNodes above it in its
    // own frame -- the boxes the reference's AABB::hit tests before it tests
    // the rectangle at all (see ref_reaches_rect).
    const uint32_t* rect_anc;
    const float* abox;
    // per rectangle, its innermost 4 list levels: start | width << 8 | boxes
    // below (of rect_anc) << 16 | valid << 31 (tie_unsettled)
    const uint32_t* rect_lvl;
    const unsigned long long* rect_lmask;  // per rectangle: the key bits of those levels with boxes below
    // Tie keys (general scenes): per sphere / rectangle / medium leaf, the
    // order in which the reference settles an exact tie in t (see
    // assignTieKeys in rtow_device.hip): the larger key wins.
    const unsigned long long* sph_key;
    const unsigned long long* rect_key;
    const unsigned long long* med_key;
    const DMat* mat;
    const DTex* tex;
    const float* ranvec;     // 256 x float4 (xyz, pad)
    const uint32_t* perm;    // 256 x (px | py << 8 | pz << 16)
    const DImage* img;
    const uint8_t* texels;
    uint32_t root;
    uint32_t stack_need;     // deepest traversal stack a ray can need
    uint32_t has_media;
    uint32_t media_any;      // some medium's boundary needs the general traversal (MB_ANY)
    uint32_t media_nested;   // some medium is not a top-level TOP_MEDIUM item
    // "simple" worlds: a chain of instances at the root, then only BvhNodes
    // and spheres (the random scene) -- traversed by the BVH-only kernel
    uint32_t simple;
    uint32_t unit_time;      // every sphere has time0 = 0, time1 = 1
    uint32_t root_chain_n;
    uint32_t root_chain[ROOTCHAIN];
    uint32_t bvh_root;       // root below the chain
    uint32_t n_node;         // DNode count (simple scenes)
    float tshift[3];         // simple scenes: world-frame offset of the DNode boxes (shiftBoxes)
    uint32_t gnode;          // general scene: node[i] is the DNode twin of bvh[i] (DK_BVH steps read it)
    // exact-order worlds (MODE 6): the scene graph as the reference builds
    // it, one XHit per rtow_hitable (include/rtow.h), interpreted by xhit
    const struct XHit* xh;
    const uint32_t* xrefs;
    uint32_t xroot;
    uint32_t exact;
    uint32_t xdepth;  // the deepest hit() recursion of the raw graph (rawDepth, <= XDEPTH): xhit's frames per thread
    // grid worlds (MODE 8): copies of the top-level spheres, by run -- a
    // TOP_SPHERE run item has a = first copy, b = count (the copy's chain = the
    // sphere's own index)
    const DSphere* tsph;
    // (unused: keep every kernel argument where the measured builds had it --
    // a moved argument cost the MODE 0 kernel 0.6 %, the compiler reloads
    // arguments inside the loop rather than spill them)
    uint32_t spare[3];
};

// One reference Hitable, as rtow_hitable (include/rtow.h) lays it out.
struct alignas(16) XHit {  // 64 B
    uint32_t kind, a, b, c;
    float f[12];
};
// The deepest reference hit() recursion xhit follows (frames in private
// memory); deeper worlds are refused at upload.
constexpr int XDEPTH = 48;

}  // namespace rtow_dev
