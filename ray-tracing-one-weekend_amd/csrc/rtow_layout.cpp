// rtow_layout.cpp -- buildLayout: the scene graph (include/rtow.h, one record
// per reference object, the reference's own tree) converted into the arrays
// the gfx950 kernels read (rtow_device_layout.h; DESIGN.md "Data layout in
// HBM"), and rtow_scene_check, which runs it without a device.  Host code
// only: the traversal kernels and the upload live in rtow_device.hip.
#include "rtow_layout.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <string>

#include "rtow_internal.h"

namespace rtow_layout {
namespace {

// The deepest hit() recursion the reference runs over the raw graph (xhit's
// frames: every call in flight, medium boundary queries included); 0 on a
// cycle or beyond XDEPTH.
uint32_t rawDepth(const rtow_scene& s, uint32_t h, std::vector<int>& memo, int guard = 0) {
    if (h >= s.n_hitables || guard > XDEPTH) return XDEPTH + 1;
    if (memo[h] > 0) return (uint32_t)memo[h];
    if (memo[h] < 0) return XDEPTH + 1;  // on the current path: a cycle
    memo[h] = -1;
    const rtow_hitable& H = s.hitables[h];
    uint32_t below = 0;
    switch (H.kind) {
    case RTOW_HIT_LIST:
        for (uint32_t j = 0; j < H.b; j++) below = std::max(below, rawDepth(s, s.refs[H.a + j], memo, guard + 1));
        break;
    case RTOW_HIT_BVH_NODE:
        below = std::max(rawDepth(s, H.a, memo, guard + 1), rawDepth(s, H.b, memo, guard + 1));
        break;
    case RTOW_HIT_FLIP_NORMALS:
    case RTOW_HIT_TRANSLATE:
    case RTOW_HIT_ROTATE_Y:
    case RTOW_HIT_BOX:
    case RTOW_HIT_CONSTANT_MEDIUM:
        below = rawDepth(s, H.a, memo, guard + 1);
        break;
    default:
        break;
    }
    memo[h] = (int)std::min<uint32_t>(below + 1, XDEPTH + 1);
    return (uint32_t)memo[h];
}

static_assert(sizeof(XHit) == sizeof(rtow_hitable), "XHit mirrors rtow_hitable");
int buildExact(const rtow_scene& s, HostLayout& L) {
    for (uint32_t i = 0; i < s.n_hitables; i++) {
        const rtow_hitable& h = s.hitables[i];
        const bool child = h.kind == RTOW_HIT_FLIP_NORMALS || h.kind == RTOW_HIT_TRANSLATE ||
                           h.kind == RTOW_HIT_ROTATE_Y || h.kind == RTOW_HIT_BOX || h.kind == RTOW_HIT_CONSTANT_MEDIUM;
        if (child && h.a >= s.n_hitables) return set_error(RTOW_E_INVALID, "child index out of range");
        if (h.kind == RTOW_HIT_BVH_NODE && (h.a >= s.n_hitables || h.b >= s.n_hitables))
            return set_error(RTOW_E_INVALID, "BvhNode child out of range");
    }
    for (uint32_t j = 0; j < s.n_refs; j++)
        if (s.refs[j] >= s.n_hitables) return set_error(RTOW_E_INVALID, "list entry out of range");
    std::vector<int> memo(s.n_hitables, 0);
    const uint32_t depth = rawDepth(s, s.root, memo);
    if (depth > (uint32_t)XDEPTH)
        return set_error(RTOW_E_UNSUPPORTED, "scene graph deeper than " + std::to_string(XDEPTH) + " calls (or cyclic)");
    L.exact = true;
    L.xh.resize(s.n_hitables);
    std::memcpy(L.xh.data(), s.hitables, sizeof(XHit) * s.n_hitables);
    L.xrefs.assign(s.refs, s.refs + s.n_refs);
    L.xroot = s.root;
    L.xdepth = depth;
    L.stack_need = depth;
    return RTOW_OK;
}

// ---------------------------------------------------------------------------
// Exact ties in general scenes.  The reference returns, among the leaves hit
// at the minimal t, the one its evaluation order leaves in the record:
// BvhNode::hit hands a tie to the right child (bvhNode.h:74-77); HitableList
// scans items in order with tmax = the closest so far (hitableList.h:20-38),
// so a later item takes a tie only if its leaf accepts t == tmax -- the
// rectangles do (closed interval, xy_rect.h:25), spheres and media do not.
// Per leaf, along its path from the root, one key component per BvhNode
// (left 0, right 1) and per list of N items (item j: N + j for a rectangle,
// N - 1 - j otherwise), packed most significant first: the first component
// where two keys differ is their lowest common ancestor's, and the larger key
// is the reference's winner.  Instances add nothing; leaves under a medium
// boundary are queried for t alone and get no key.  (Not reproduced: a
// BvhNode ITEM of a list whose box the ray enters exactly at the tied t is
// culled by AABB::hit's `tmax <= tmin`, so its leaf cannot take the tie.)
// Instance chains: every leaf / medium / instance gets the id (in L.chains)
// of the chain of instances above it; EXIT markers restore an instance's
// parent chain.  A node met again under a different chain (an instance
// shared between two transforms) is rejected.
struct ChainAssigner {
    HostLayout& L;
    std::map<std::vector<uint32_t>, uint32_t> ids;
    std::vector<uint32_t> cur;
    std::vector<uint32_t> sph, rect, med, inst;  // assigned chain per entity (~0u: not yet)
    std::string err;

    explicit ChainAssigner(HostLayout& l) : L(l) {
        sph.assign(L.sph.size(), ~0u);
        rect.assign(L.rect.size(), ~0u);
        med.assign(L.med.size(), ~0u);
        inst.assign(L.inst.size(), ~0u);
        id();  // chain 0: no instances
    }
    uint32_t id() {
        auto it = ids.find(cur);
        if (it != ids.end()) return it->second;
        DChain c{};
        c.n = (uint32_t)cur.size();
        for (size_t k = 0; k < cur.size() && k < (size_t)MAXCHAIN; k++) c.ref[k] = cur[k];
        L.chains.push_back(c);
        return ids[cur] = (uint32_t)L.chains.size() - 1;
    }
    bool set(std::vector<uint32_t>& v, uint32_t i, uint32_t c) {
        if (v[i] != ~0u && v[i] != c) {
            err = "a hitable is shared under two different instance chains";
            return false;
        }
        v[i] = c;
        return true;
    }
    void walk(uint32_t ref, int depth = 0) {
        if (!err.empty() || depth > 4096) return;
        const uint32_t kind = ref >> KIND_SHIFT, idx = ref & INDEX_MASK;
        if (cur.size() > (size_t)MAXCHAIN) {
            err = "instance nesting deeper than " + std::to_string(MAXCHAIN);
            return;
        }
        const uint32_t c = id();
        switch (kind) {
        case DK_SPHERE:
            if (set(sph, idx, c)) L.sph[idx].chain = c;
            break;
        case DK_RECT:
            if (set(rect, idx, c)) L.rect[idx].chain = c;
            break;
        case DK_MEDIUM:
            if (set(med, idx, c)) {
                L.med[idx].chain = c;
                walk(L.med[idx].boundary, depth + 1);
            }
            break;
        case DK_BVH:
            walk(L.bvh[idx].left, depth + 1);
            walk(L.bvh[idx].right, depth + 1);
            break;
        case DK_LIST: {
            const DList l = L.list[idx];
            for (uint32_t j = 0; j < l.count; j++) walk(L.refs[l.first + j], depth + 1);
            break;
        }
        case DK_RECTS: {
            const DList l = L.list[idx];
            for (uint32_t j = 0; j < l.count; j++) walk(mkref(DK_RECT, l.first + j), depth + 1);
            break;
        }
        case DK_TRANSLATE:
        case DK_ROTY:
        case DK_FLIP:
            if (set(inst, idx, c)) {
                L.inst[idx].parent_chain = c;
                cur.push_back(ref);
                walk(L.inst[idx].child, depth + 1);
                cur.pop_back();
            }
            break;
        default:
            break;
        }
    }
};

struct KeyComp {
    uint32_t bits;
    unsigned long long closed, open;
    // list components: where refAncestors' in-frame box path stood when the
    // list was entered (frame: which instance frame that was)
    bool list = false;
    uint32_t frame = 0, boxes = 0;
};
// refAncestors' box path as assignTieKeys walks the same graph: its length
// in the current frame (a Translate / RotateY starts a new one)
struct TieWalk {
    uint32_t frame = 0, boxes = 0, next_frame = 1;
};

void assignTieKeys(HostLayout& L, uint32_t ref, std::vector<KeyComp>& path, TieWalk& tw, int depth = 0) {
    if (depth > 512) return;
    const uint32_t kind = ref >> KIND_SHIFT, idx = ref & INDEX_MASK;
    auto key = [&](bool closed) {
        unsigned long long k = 0;
        uint32_t used = 0;
        for (const KeyComp& c : path) {
            if (used + c.bits > 64) break;  // deeper levels: ties there stay with the first found
            k = (k << c.bits) | (closed ? c.closed : c.open);
            used += c.bits;
        }
        return used ? k << (64 - used) : 0ull;
    };
    // a rectangle's list levels (DevScene::rect_lvl, tie_unsettled): the
    // innermost four, with how many boxes of its frame lie below each
    auto levels = [&](uint32_t rect) {
        std::vector<uint32_t> lv;
        uint32_t at = 0;
        for (const KeyComp& c : path) {
            if (at + c.bits > 64) break;
            if (c.list) {
                const uint32_t below = c.frame == tw.frame ? tw.boxes - c.boxes : tw.boxes;
                lv.push_back(at | (c.bits << 8) | (std::min(below, 255u) << 16) | 0x80000000u);
            }
            at += c.bits;
        }
        const size_t from = lv.size() > 4 ? lv.size() - 4 : 0;
        unsigned long long mask = 0;
        for (size_t k = from; k < lv.size(); k++) {
            L.rect_lvl[4 * (size_t)rect + (k - from)] = lv[k];
            const uint32_t st = lv[k] & 255u, w = (lv[k] >> 8) & 255u;
            if ((lv[k] >> 16) & 255u)
                for (uint32_t b = st; b < st + w && b < 64; b++) mask |= 1ull << (63 - b);
        }
        L.rect_lmask[rect] = mask;
    };
    const bool collapsed = L.collapsed_of.count(ref) != 0;  // an n == 1 BvhNode's box (refAncestors)
    if (collapsed) tw.boxes++;
    switch (kind) {
    case DK_SPHERE:
        L.sph_key[idx] = key(false);
        break;
    case DK_RECT:
        L.rect_key[idx] = key(true);
        levels(idx);
        break;
    case DK_MEDIUM:
        L.med_key[idx] = key(false);
        break;
    case DK_BVH:
        tw.boxes++;
        for (uint32_t c = 0; c < 2; c++) {
            path.push_back(KeyComp{1, c, c});
            assignTieKeys(L, c ? L.bvh[idx].right : L.bvh[idx].left, path, tw, depth + 1);
            path.pop_back();
        }
        tw.boxes--;
        break;
    case DK_LIST:
    case DK_RECTS: {
        const DList l = L.list[idx];
        uint32_t bits = 1;
        while ((1ull << bits) < 2ull * l.count) bits++;
        for (uint32_t j = 0; j < l.count; j++) {
            path.push_back(KeyComp{bits, (unsigned long long)l.count + j, (unsigned long long)l.count - 1 - j, true,
                                   tw.frame, tw.boxes});
            assignTieKeys(L, kind == DK_RECTS ? mkref(DK_RECT, l.first + j) : L.refs[l.first + j], path, tw, depth + 1);
            path.pop_back();
        }
        break;
    }
    case DK_FLIP:
        assignTieKeys(L, L.inst[idx].child, path, tw, depth + 1);
        break;
    case DK_TRANSLATE:
    case DK_ROTY: {
        const TieWalk saved = tw;
        tw.frame = tw.next_frame++;
        tw.boxes = 0;
        assignTieKeys(L, L.inst[idx].child, path, tw, depth + 1);
        const uint32_t nf = tw.next_frame;
        tw = saved;
        tw.next_frame = nf;
        break;
    }
    default:
        break;
    }
    if (collapsed) tw.boxes--;
}

// ---------------------------------------------------------------------------
// Simple scenes are traversed over a surface-area-heuristic tree rebuilt from
// the same spheres instead of the reference's own BvhNode tree (bvhNode.h:
// 14-58 sorts on a random axis and splits at the median, which leaves the
// R=1000 ground sphere's box on a spine of whole-scene boxes every ray walks).
// The closest hit is a property of the set of leaves, not of the tree, once
// ties are settled the reference's way: BvhNode::hit (bvhNode.h:66-96) keeps
// the nearer record and hands an exact tie to the right subtree, so among the
// leaves at the minimal t the reference returns the LAST one in the tree's
// left-to-right order.  The converter numbers spheres in that order (it
// converts the left subtree first), so the device breaks a tie by the larger
// sphere index, and the result is the reference tree's whatever tree is
// traversed.  RTOW_BVH=ref keeps the reference tree.
struct SahPrim {
    float mn[3], mx[3], c[3];
    uint32_t ref;
};

float sahArea(const float* mn, const float* mx) {
    const double dx = (double)mx[0] - mn[0], dy = (double)mx[1] - mn[1], dz = (double)mx[2] - mn[2];
    return (float)(2.0 * (dx * dy + dy * dz + dz * dx));
}

void sahUnion(float* mn, float* mx, const float* bmn, const float* bmx) {
    for (int a = 0; a < 3; a++) {
        mn[a] = std::min(mn[a], bmn[a]);
        mx[a] = std::max(mx[a], bmx[a]);
    }
}

// Binary SAH build over P[lo, hi) (full sweep over the three centroid axes);
// fills `out` with fused DNodes (sphere children inline) and returns the
// node's ref.  `need` = LDS stack entries its traversal can hold: a push
// happens only where both children are inner nodes and hit.
uint32_t sahBuild(const HostLayout& L, std::vector<SahPrim>& P, size_t lo, size_t hi, std::vector<DNode>& out,
                  uint32_t& need, int depth) {
    const size_t n = hi - lo;
    const uint32_t idx = (uint32_t)out.size();
    out.push_back(DNode{});
    int best_axis = 0;
    size_t best_i = lo + n / 2;
    double best_cost = DBL_MAX;
    std::vector<float> right_area(n + 1);
    for (int axis = 0; axis < 3; axis++) {
        std::sort(P.begin() + lo, P.begin() + hi, [axis](const SahPrim& x, const SahPrim& y) {
            return x.c[axis] < y.c[axis] || (x.c[axis] == y.c[axis] && x.ref < y.ref);
        });
        float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (size_t k = n; k-- > 1;) {
            sahUnion(mn, mx, P[lo + k].mn, P[lo + k].mx);
            right_area[k] = sahArea(mn, mx);
        }
        float lmn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, lmx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (size_t k = 1; k < n; k++) {
            sahUnion(lmn, lmx, P[lo + k - 1].mn, P[lo + k - 1].mx);
            const double cost = (double)sahArea(lmn, lmx) * (double)k + (double)right_area[k] * (double)(n - k);
            if (cost < best_cost) {
                best_cost = cost;
                best_axis = axis;
                best_i = lo + k;
            }
        }
    }
    std::sort(P.begin() + lo, P.begin() + hi, [best_axis](const SahPrim& x, const SahPrim& y) {
        return x.c[best_axis] < y.c[best_axis] || (x.c[best_axis] == y.c[best_axis] && x.ref < y.ref);
    });
    const size_t range[2][2] = {{lo, best_i}, {best_i, hi}};
    uint32_t refs[2], needs[2] = {0, 0};
    float box[2][6];
    for (int k = 0; k < 2; k++) {
        const size_t a = range[k][0], b = range[k][1];
        float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (size_t i = a; i < b; i++) sahUnion(mn, mx, P[i].mn, P[i].mx);
        for (int q = 0; q < 3; q++) {
            box[k][q] = mn[q];
            box[k][3 + q] = mx[q];
        }
        refs[k] = b - a == 1 ? P[a].ref : sahBuild(L, P, a, b, out, needs[k], depth + 1);
    }
    // A node with one sphere child keeps it in slot b: the kernel runs a
    // slot's sphere path (or box path) once for every lane of the wave that
    // needs it, so slot b's box path is left to inner-inner nodes and slot
    // a's sphere path to sphere-sphere nodes.  (Slots carry no order: ties go
    // by sphere index and the nearer inner child is visited first.)  +2 %.
    if ((refs[0] >> KIND_SHIFT) == DK_SPHERE && (refs[1] >> KIND_SHIFT) != DK_SPHERE) {
        std::swap(refs[0], refs[1]);
        std::swap(needs[0], needs[1]);
        for (int q = 0; q < 6; q++) std::swap(box[0][q], box[1][q]);
    }
    DNode& d = out[idx];
    for (int k = 0; k < 2; k++) {
        float* f = k == 0 ? d.a : d.b;
        (k == 0 ? d.ref_a : d.ref_b) = refs[k];
        if ((refs[k] >> KIND_SHIFT) == DK_SPHERE) {
            const DSphere& sp = L.sph[refs[k] & INDEX_MASK];
            f[0] = sp.c0[0]; f[1] = sp.c0[1]; f[2] = sp.c0[2]; f[3] = sp.r * sp.r;
            f[4] = sp.dc[0]; f[5] = sp.dc[1]; f[6] = sp.dc[2];
        } else {
            for (int q = 0; q < 6; q++) f[q] = box[k][q];
            f[6] = 0.0f;
        }
    }
    const bool ia = (refs[0] >> KIND_SHIFT) == DK_BVH, ib = (refs[1] >> KIND_SHIFT) == DK_BVH;
    need = (ia && ib) ? 1 + std::max(needs[0], needs[1]) : (ia ? needs[0] : (ib ? needs[1] : 0u));
    return mkref(DK_BVH, idx);
}

// ---- General scenes: every maximal BvhNode subtree whose leaves all have
// finite boxes (spheres, Boxes) is rebuilt the same way, over those leaves,
// as DBvh nodes; exact ties are settled by the tie keys (assigned before, on
// the reference tree), so the frame does not change.  Leaves keep their
// instance chains (the rebuild only rearranges the BvhNodes above them).
struct GenLeaf {
    float mn[3], mx[3], c[3];
    uint32_t ref;
};

void genLeaves(const HostLayout& L, uint32_t ref, std::vector<GenLeaf>& out, bool& bounded, int depth = 0) {
    const DBvh b = L.bvh[ref & INDEX_MASK];
    for (int k = 0; k < 2; k++) {
        const uint32_t child = k ? b.right : b.left;
        if ((child >> KIND_SHIFT) == DK_BVH && depth < 200) {
            genLeaves(L, child, out, bounded, depth + 1);
            continue;
        }
        GenLeaf g;
        const float mn[3] = {b.xs[2 * k], b.ys[2 * k], b.zs[2 * k]};
        const float mx[3] = {b.xs[2 * k + 1], b.ys[2 * k + 1], b.zs[2 * k + 1]};
        for (int a = 0; a < 3; a++) {
            g.mn[a] = mn[a];
            g.mx[a] = mx[a];
            if (!(std::fabs(mn[a]) < 1e30f && std::fabs(mx[a]) < 1e30f)) bounded = false;
            g.c[a] = 0.5f * (mn[a] + mx[a]);
        }
        g.ref = child;
        out.push_back(g);
    }
}

uint32_t sahBuildBvh(std::vector<GenLeaf>& P, size_t lo, size_t hi, std::vector<DBvh>& out) {
    const size_t n = hi - lo;
    const uint32_t idx = (uint32_t)out.size();
    out.push_back(DBvh{});
    int best_axis = 0;
    size_t best_i = lo + n / 2;
    double best_cost = DBL_MAX;
    std::vector<float> right_area(n + 1);
    auto order = [](int axis) {
        return [axis](const GenLeaf& x, const GenLeaf& y) {
            return x.c[axis] < y.c[axis] || (x.c[axis] == y.c[axis] && x.ref < y.ref);
        };
    };
    for (int axis = 0; axis < 3; axis++) {
        std::sort(P.begin() + lo, P.begin() + hi, order(axis));
        float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (size_t k = n; k-- > 1;) {
            sahUnion(mn, mx, P[lo + k].mn, P[lo + k].mx);
            right_area[k] = sahArea(mn, mx);
        }
        float lmn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, lmx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (size_t k = 1; k < n; k++) {
            sahUnion(lmn, lmx, P[lo + k - 1].mn, P[lo + k - 1].mx);
            const double cost = (double)sahArea(lmn, lmx) * (double)k + (double)right_area[k] * (double)(n - k);
            if (cost < best_cost) {
                best_cost = cost;
                best_axis = axis;
                best_i = lo + k;
            }
        }
    }
    std::sort(P.begin() + lo, P.begin() + hi, order(best_axis));
    const size_t range[2][2] = {{lo, best_i}, {best_i, hi}};
    DBvh d{};
    uint32_t refs[2];
    for (int k = 0; k < 2; k++) {
        const size_t a = range[k][0], b = range[k][1];
        float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (size_t i = a; i < b; i++) sahUnion(mn, mx, P[i].mn, P[i].mx);
        d.xs[2 * k] = mn[0];
        d.xs[2 * k + 1] = mx[0];
        d.ys[2 * k] = mn[1];
        d.ys[2 * k + 1] = mx[1];
        d.zs[2 * k] = mn[2];
        d.zs[2 * k + 1] = mx[2];
        refs[k] = b - a == 1 ? P[a].ref : sahBuildBvh(P, a, b, out);
    }
    d.left = refs[0];
    d.right = refs[1];
    out[idx] = d;
    return mkref(DK_BVH, idx);
}

// Does anything below `ref` draw random numbers during traversal?
bool refHasMedium(const HostLayout& L, uint32_t ref, int depth = 0) {
    const uint32_t kind = ref >> KIND_SHIFT, idx = ref & INDEX_MASK;
    if (depth > 512) return true;
    switch (kind) {
    case DK_MEDIUM:
        return true;
    case DK_BVH:
        return refHasMedium(L, L.bvh[idx].left, depth + 1) || refHasMedium(L, L.bvh[idx].right, depth + 1);
    case DK_LIST: {
        const DList& l = L.list[idx];
        for (uint32_t j = 0; j < l.count; j++)
            if (refHasMedium(L, L.refs[l.first + j], depth + 1)) return true;
        return false;
    }
    case DK_TRANSLATE:
    case DK_ROTY:
    case DK_FLIP:
        return refHasMedium(L, L.inst[idx].child, depth + 1);
    default:
        return false;
    }
}

struct GeneralSah {
    HostLayout& L;
    uint32_t n_old;  // DBvh nodes of the reference trees (new ones come after)

    bool hasMedium(uint32_t ref) const { return refHasMedium(L, ref); }

    // A box holding every hit point of `ref`, in the frame `ref` sits in
    // (false: unbounded).  Only used to cull, so it is padded well beyond the
    // rounding of the hit points and of the instance transforms.
    bool bounds(uint32_t ref, float* mn, float* mx, int depth = 0) const {
        const uint32_t kind = ref >> KIND_SHIFT, idx = ref & INDEX_MASK;
        if (depth > 512) return false;
        for (int a = 0; a < 3; a++) {
            mn[a] = FLT_MAX;
            mx[a] = -FLT_MAX;
        }
        auto grow = [&](const float* bmn, const float* bmx) { sahUnion(mn, mx, bmn, bmx); };
        switch (kind) {
        case DK_SPHERE: {
            const DSphere& q = L.sph[idx];
            for (int a = 0; a < 3; a++) {
                const float c1 = q.c0[a] + q.dc[a];
                mn[a] = std::min(q.c0[a], c1) - q.r;
                mx[a] = std::max(q.c0[a], c1) + q.r;
            }
            break;
        }
        case DK_RECT: {
            const DRect& q = L.rect[idx];
            const uint32_t ax = q.axis & 3u;
            const int i = ax == 2 ? 1 : 0, j = ax == 0 ? 1 : 2, k = ax == 0 ? 2 : (ax == 1 ? 1 : 0);
            mn[i] = q.a0;
            mx[i] = q.a1;
            mn[j] = q.b0;
            mx[j] = q.b1;
            mn[k] = mx[k] = q.k;
            break;
        }
        case DK_RECTS: {
            const DList& l = L.list[idx];
            for (uint32_t j = 0; j < l.count; j++) {
                float a[3], b[3];
                if (!bounds(mkref(DK_RECT, l.first + j), a, b, depth + 1)) return false;
                grow(a, b);
            }
            break;
        }
        case DK_BVH: {
            const DBvh& b = L.bvh[idx];
            const float a0[3] = {b.xs[0], b.ys[0], b.zs[0]}, a1[3] = {b.xs[1], b.ys[1], b.zs[1]};
            const float b0[3] = {b.xs[2], b.ys[2], b.zs[2]}, b1[3] = {b.xs[3], b.ys[3], b.zs[3]};
            grow(a0, a1);
            grow(b0, b1);
            break;
        }
        case DK_LIST: {
            const DList& l = L.list[idx];
            for (uint32_t j = 0; j < l.count; j++) {
                float a[3], b[3];
                if (!bounds(L.refs[l.first + j], a, b, depth + 1)) return false;
                grow(a, b);
            }
            break;
        }
        case DK_TRANSLATE:
        case DK_FLIP:
        case DK_ROTY: {
            const DInst& I = L.inst[idx];
            float a[3], b[3];
            if (!bounds(I.child, a, b, depth + 1)) return false;
            if (kind == DK_FLIP) {
                grow(a, b);
            } else if (kind == DK_TRANSLATE) {
                for (int k = 0; k < 3; k++) {
                    mn[k] = a[k] + I.p[k];
                    mx[k] = b[k] + I.p[k];
                }
            } else {  // the way out (inst_out): x' = c x + s z, z' = -s x + c z
                const double sn = I.p[0], cs = I.p[1];
                for (int c = 0; c < 8; c++) {
                    const double x = (c & 1) ? b[0] : a[0], y = (c & 2) ? b[1] : a[1], z = (c & 4) ? b[2] : a[2];
                    const float q[3] = {(float)(cs * x + sn * z), (float)y, (float)(-sn * x + cs * z)};
                    grow(q, q);
                }
            }
            break;
        }
        default:
            return false;
        }
        for (int a = 0; a < 3; a++) {
            if (!(std::fabs(mn[a]) < 1e30f && std::fabs(mx[a]) < 1e30f && mn[a] <= mx[a])) return false;
            const float pad = 1e-5f * (std::fabs(mn[a]) + std::fabs(mx[a]) + (mx[a] - mn[a])) + 1e-5f;
            mn[a] -= pad;
            mx[a] += pad;
        }
        return true;
    }

    // leaves below `ref` (capped): how much a box around it can save
    uint32_t leafCount(uint32_t ref, int depth = 0) const {
        const uint32_t kind = ref >> KIND_SHIFT, idx = ref & INDEX_MASK;
        if (depth > 64) return 1;
        switch (kind) {
        case DK_BVH:
            return std::min(1u << 20, leafCount(L.bvh[idx].left, depth + 1) + leafCount(L.bvh[idx].right, depth + 1));
        case DK_RECTS:
            return L.list[idx].count;
        case DK_LIST: {
            uint32_t n = 0;
            for (uint32_t j = 0; j < L.list[idx].count; j++)
                n = std::min(1u << 20, n + leafCount(L.refs[L.list[idx].first + j], depth + 1));
            return n;
        }
        case DK_TRANSLATE:
        case DK_ROTY:
        case DK_FLIP:
            return leafCount(L.inst[idx].child, depth + 1);
        default:
            return 1;
        }
    }

    // A list's items in order, with every run of consecutive items that hold
    // no medium and are bounded replaced by one SAH tree over those items
    // when the run holds a large aggregate (>= 16 leaves: culling it pays).
    // Short lists of small items stay a scan: every lane of a wave visits the
    // same item at the same time there, where a tree would split the wave
    // over different items (measured: cornell -13 %, cornell_smoke -51 %;
    // final_ned's two runs +33 %).
    // hitableList.h:20-38 keeps the nearest hit of its items; within such a
    // run that does not depend on the order (exact ties: the tie keys, taken
    // from the reference graph before this), and a medium only sees the
    // nearest hit of the items before it (hitableList.h:30), which the run's
    // tree gives it as the scan did.  Media keep their places.
    // An instance chain over a BvhNode of unit-time spheres with many leaves
    // (final_ned's cloud) stays an item of its own: at the top level it is a
    // TOP_SPHERES item (trace_dnodes) instead of a leaf of the run's tree.
    bool sphereInstance(uint32_t ref) const {
        uint32_t r = ref;
        int n = 0;
        for (; n < 64; n++) {
            const uint32_t k = r >> KIND_SHIFT;
            if (k != DK_TRANSLATE && k != DK_ROTY && k != DK_FLIP) break;
            r = L.inst[r & INDEX_MASK].child;
        }
        return n > 0 && (r >> KIND_SHIFT) == DK_BVH && onlyUnitSpheres(r) && leafCount(r) >= 16;
    }
    bool onlyUnitSpheres(uint32_t ref, int depth = 0) const {
        const uint32_t kind = ref >> KIND_SHIFT, idx = ref & INDEX_MASK;
        if (depth > 200) return false;
        if (kind == DK_SPHERE) return L.sph[idx].t0 == 0.0f && L.sph[idx].t1 == 1.0f;
        if (kind != DK_BVH) return false;
        return onlyUnitSpheres(L.bvh[idx].left, depth + 1) && onlyUnitSpheres(L.bvh[idx].right, depth + 1);
    }

    // grid_ext's packed extents: 16-bit steps of (hhi - hlo) / 65535 (that
    // float, as the kernel computes it) from the grid's hlo, the lower bound
    // rounded down and the upper up (one step more either way); false if a
    // decoded float (fmaf, as the kernel decodes) does not contain the true
    // extent -- then the grid is not used and its tree is traversed instead.
    static bool packHeights(const DGrid& g, const std::vector<DGridCell>& cells, std::vector<uint32_t>& out) {
        const float step = (g.hhi - g.hlo) * (1.0f / 65535.0f);
        out.clear();
        for (const DGridCell& c : cells) {
            uint32_t q[2];
            for (int e = 0; e < 2; e++) {
                const double h = e ? c.hhi : c.hlo;
                double x = step > 0.0f ? (h - (double)g.hlo) / (double)step : 0.0;
                x = e ? std::ceil(x) + 1.0 : std::floor(x) - 1.0;
                q[e] = (uint32_t)std::min(65535.0, std::max(0.0, x));
            }
            const float lo = std::fmaf((float)q[0], step, g.hlo), hi = std::fmaf((float)q[1], step, g.hlo);
            if (!(lo <= c.hlo && hi >= c.hhi)) return false;
            out.push_back(q[0] | q[1] << 16);
        }
        return true;
    }

    // A BvhNode whose leaves are Boxes (rectangle lists with a DBox6), all in
    // one frame, that tile a regular grid of columns along two axes (one Box
    // per cell, within a 2^-12 cell width of the cell; any extent along the
    // third axis): its DGrid is registered (L.grid_of) and the item stays out
    // of the run's tree, so the top-level scan can walk it as a grid
    // (TOP_GRID).  final_ned's ground: 20 x 20 Boxes 100 wide, heights 1..101.
    // RTOW_GRID=0: no grids (A/B).
    bool gridItem(uint32_t ref) {
        if ((ref >> KIND_SHIFT) != DK_BVH) return false;
        if (L.grid_of.count(ref)) return true;
        if (const char* e = std::getenv("RTOW_GRID"))
            if (std::atoi(e) == 0) return false;
        std::vector<GenLeaf> lv;
        bool bounded = true;
        genLeaves(L, ref, lv, bounded);
        if (!bounded || lv.size() < 16) return false;
        std::vector<uint32_t> bx(lv.size());
        uint32_t chain = ~0u;
        for (size_t q = 0; q < lv.size(); q++) {
            const uint32_t r = lv[q].ref;
            if ((r >> KIND_SHIFT) != DK_RECTS) return false;
            const DList& l = L.list[r & INDEX_MASK];
            if (!l.box6) return false;
            for (uint32_t k = 0; k < l.count; k++) {
                const uint32_t c = L.rect[l.first + k].chain;
                if (chain == ~0u) chain = c;
                if (c != chain) return false;
            }
            bx[q] = l.box6 - 1;
        }
        for (uint32_t ah = 0; ah < 3; ah++) {
            const uint32_t au = ah == 0 ? 1u : 0u, av = ah == 2 ? 1u : 2u;
            float u0 = FLT_MAX, v0 = FLT_MAX, u1 = -FLT_MAX, v1 = -FLT_MAX, hlo = FLT_MAX, hhi = -FLT_MAX;
            for (uint32_t b : bx) {
                const DBox6& q = L.box6[b];
                u0 = std::min(u0, q.lo[au]), v0 = std::min(v0, q.lo[av]);
                u1 = std::max(u1, q.hi[au]), v1 = std::max(v1, q.hi[av]);
                hlo = std::min(hlo, q.lo[ah]), hhi = std::max(hhi, q.hi[ah]);
            }
            const DBox6& f = L.box6[bx[0]];
            const double wu = (double)f.hi[au] - f.lo[au], wv = (double)f.hi[av] - f.lo[av];
            if (!(wu > 0 && wv > 0)) continue;
            const double nuf = std::round((u1 - (double)u0) / wu), nvf = std::round((v1 - (double)v0) / wv);
            if (!(nuf >= 1 && nvf >= 1 && nuf * nvf == (double)bx.size())) continue;
            const uint32_t nu = (uint32_t)nuf, nv = (uint32_t)nvf;
            const double tol = std::max(wu, wv) * 0x1p-12;
            std::vector<DGridCell> cells((size_t)nu * nv);
            std::vector<char> seen((size_t)nu * nv, 0);
            bool ok = true;
            for (uint32_t b : bx) {
                const DBox6& q = L.box6[b];
                const double fi = std::round((q.lo[au] - (double)u0) / wu), fj = std::round((q.lo[av] - (double)v0) / wv);
                if (!(fi >= 0 && fi < nu && fj >= 0 && fj < nv)) {
                    ok = false;
                    break;
                }
                const double cu = u0 + fi * wu, cv = v0 + fj * wv;
                if (std::fabs(q.lo[au] - cu) > tol || std::fabs(q.hi[au] - (cu + wu)) > tol ||
                    std::fabs(q.lo[av] - cv) > tol || std::fabs(q.hi[av] - (cv + wv)) > tol || !(q.lo[ah] <= q.hi[ah])) {
                    ok = false;
                    break;
                }
                const size_t c = (size_t)fj * nu + (size_t)fi;
                if (seen[c]) {
                    ok = false;
                    break;
                }
                seen[c] = 1;
                cells[c] = DGridCell{q.lo[ah], q.hi[ah], b, 0u};
            }
            if (!ok) continue;
            // the cell and row extents as packed 16-bit words (gq): the decoded
            // floats must contain every true extent.  The MODE 8 kernel at
            // STACK 16 stages the table in LDS when it holds at most
            // GRID_LDS_WORDS words; a larger one is walked from global memory
            // by the STACK 20 kernel (rtow_device.hip, launchStack)
            DGrid g{};
            g.u0 = u0, g.v0 = v0, g.wu = (float)wu, g.wv = (float)wv;
            g.iwu = (float)(1.0 / wu), g.iwv = (float)(1.0 / wv);
            g.hlo = hlo, g.hhi = hhi, g.u1 = u1, g.v1 = v1;
            g.nu = nu, g.nv = nv;
            g.axes = au | av << 2 | ah << 4;
            g.cell0 = (uint32_t)L.gcell.size();
            g.margin = (float)(std::max(wu, wv) * 0x1p-10);  // 2^2 x the tolerance above
            std::vector<DGridCell> all(cells);
            for (uint32_t j = 0; j < nv; j++) {  // per row: the extent of its columns together
                DGridCell row{FLT_MAX, -FLT_MAX, 0u, 0u};
                for (uint32_t i = 0; i < nu; i++) {
                    row.hlo = std::min(row.hlo, cells[(size_t)j * nu + i].hlo);
                    row.hhi = std::max(row.hhi, cells[(size_t)j * nu + i].hhi);
                }
                all.push_back(row);
            }
            std::vector<uint32_t> packed;
            if (!packHeights(g, all, packed)) continue;
            // the cells' Boxes copied in cell order (the walk computes a
            // candidate's DBox6 instead of loading its index); a copy's first
            // side is the same rectangle, so its tie keys are the Box's
            g.box0 = (uint32_t)L.box6.size();
            for (size_t c = 0; c < cells.size(); c++) {
                const DBox6 b = L.box6[cells[c].box6];
                L.box6.push_back(b);
            }
            L.gcell.insert(L.gcell.end(), all.begin(), all.end());
            L.gq.insert(L.gq.end(), packed.begin(), packed.end());
            L.grid_of[ref] = (uint32_t)L.grid.size();
            L.grid.push_back(g);
            return true;
        }
        return false;
    }

    void treeRuns(const DList& l) {
        std::vector<uint32_t> items(L.refs.begin() + l.first, L.refs.begin() + l.first + l.count), out;
        size_t j = 0;
        while (j < items.size()) {
            std::vector<GenLeaf> run;
            std::vector<uint32_t> alone;  // sphereInstance items of the run
            size_t k = j;
            for (; k < items.size(); k++) {
                GenLeaf g;
                if (hasMedium(items[k]) || !bounds(items[k], g.mn, g.mx)) break;
                if (sphereInstance(items[k]) || gridItem(items[k])) {
                    alone.push_back(items[k]);
                    continue;
                }
                for (int a = 0; a < 3; a++) g.c[a] = 0.5f * (g.mn[a] + g.mx[a]);
                g.ref = items[k];
                run.push_back(g);
            }
            uint32_t big = 0;
            for (const GenLeaf& g : run) big = std::max(big, leafCount(g.ref));
            // (RTOW_RUNTREE=k: the rest of a run an aggregate was taken out of
            // -- a grid, a sphere instance -- as a tree as well when it holds
            // >= k items; A/B)
            const char* rt = std::getenv("RTOW_RUNTREE");
            if (rt && std::atoi(rt) != 0 && !alone.empty() && run.size() >= (size_t)std::max(2, std::atoi(rt))) big = 16;
            if (run.size() >= 2 && big >= 16) {
                out.push_back(sahBuildBvh(run, 0, run.size(), L.bvh));
            } else {
                for (const GenLeaf& g : run) out.push_back(g.ref);
            }
            for (uint32_t a : alone) out.push_back(a);
            if (k < items.size()) out.push_back(items[k]);  // the barrier item
            j = k + 1;
        }
        for (size_t q = 0; q < out.size(); q++) L.refs[l.first + q] = out[q];
        for (size_t q = out.size(); q < l.count; q++) L.refs[l.first + q] = mkref(DK_NONE, 0);
    }

    void patch(uint32_t& ref, int depth = 0) {
        if (depth > 512) return;
        const uint32_t kind = ref >> KIND_SHIFT, idx = ref & INDEX_MASK;
        switch (kind) {
        case DK_BVH: {
            if (idx >= n_old) return;  // already rebuilt (a shared subtree)
            std::vector<GenLeaf> leaves;
            bool bounded = true;
            genLeaves(L, ref, leaves, bounded);
            for (const GenLeaf& g : leaves) {  // BVHs nested below the leaves
                uint32_t r = g.ref;
                patch(r, depth + 1);
            }
            if (bounded && leaves.size() >= 2) ref = sahBuildBvh(leaves, 0, leaves.size(), L.bvh);
            break;
        }
        case DK_LIST: {
            const DList l = L.list[idx];
            for (uint32_t j = 0; j < l.count; j++) patch(L.refs[l.first + j], depth + 1);
            treeRuns(l);
            uint32_t n = 0;
            while (n < l.count && (L.refs[l.first + n] >> KIND_SHIFT) != DK_NONE) n++;
            L.list[idx].count = n;
            break;
        }
        case DK_TRANSLATE:
        case DK_ROTY:
        case DK_FLIP:
            patch(L.inst[idx].child, depth + 1);
            break;
        case DK_MEDIUM:
            patch(L.med[idx].boundary, depth + 1);
            break;
        default:
            break;
        }
    }
};

// leaves of the reference tree left to right
void inorderLeaves(const HostLayout& L, uint32_t ref, std::vector<uint32_t>& out) {
    if ((ref >> KIND_SHIFT) == DK_BVH) {
        inorderLeaves(L, L.bvh[ref & INDEX_MASK].left, out);
        inorderLeaves(L, L.bvh[ref & INDEX_MASK].right, out);
    } else {
        out.push_back(ref);
    }
}

// Replace L.node / L.bvh_root by the SAH tree; false (reference tree kept)
// when the leaves are not numbered in left-to-right order (a shared subtree).
bool rebuildSah(HostLayout& L) {
    std::vector<uint32_t> leaves;
    inorderLeaves(L, L.bvh_root, leaves);
    if (leaves.size() < 2) return false;
    for (size_t i = 1; i < leaves.size(); i++)
        if ((leaves[i] & INDEX_MASK) <= (leaves[i - 1] & INDEX_MASK)) return false;
    std::vector<SahPrim> P(leaves.size());
    for (size_t i = 0; i < leaves.size(); i++) {
        const DSphere& sp = L.sph[leaves[i] & INDEX_MASK];
        SahPrim& q = P[i];
        for (int a = 0; a < 3; a++) {
            // the box every center(time), time in [0, 1], stays in (boxOf)
            const float c1 = sp.c0[a] + sp.dc[a];
            q.mn[a] = std::min(sp.c0[a], c1) - sp.r;
            q.mx[a] = std::max(sp.c0[a], c1) + sp.r;
            q.c[a] = 0.5f * (q.mn[a] + q.mx[a]);
        }
        q.ref = leaves[i];
    }
    std::vector<DNode> nodes;
    uint32_t need = 0;
    const uint32_t root = sahBuild(L, P, 0, P.size(), nodes, need, 0);
    L.node.swap(nodes);
    L.bvh_root = root;
    L.stack_need = need;
    return true;
}

// A simple scene whose root chain is translations only: its DNode boxes move
// to the world frame (rounded outward), where the rays' origins lie near them
// and the one-FMA slab planes stay tight (SlabRay); the kernel shifts each
// ray's origin by the same float offset.  Sphere slots stay in the BVH frame:
// their tests are the reference's arithmetic.
void shiftBoxes(HostLayout& L) {
    float t[3] = {0.0f, 0.0f, 0.0f};
    for (uint32_t k = 0; k < L.root_chain_n; k++) {
        if ((L.root_chain[k] >> KIND_SHIFT) != DK_TRANSLATE) return;
        const DInst& I = L.inst[L.root_chain[k] & INDEX_MASK];
        for (int a = 0; a < 3; a++) t[a] += I.p[a];
    }
    if (t[0] == 0.0f && t[1] == 0.0f && t[2] == 0.0f) return;
    auto down = [](double v) {
        float f = (float)v;
        return (double)f > v ? std::nextafter(f, -INFINITY) : f;
    };
    auto up = [](double v) {
        float f = (float)v;
        return (double)f < v ? std::nextafter(f, INFINITY) : f;
    };
    for (DNode& d : L.node)
        for (int k = 0; k < 2; k++) {
            float* f = k == 0 ? d.a : d.b;
            if (((k == 0 ? d.ref_a : d.ref_b) >> KIND_SHIFT) != DK_BVH) continue;
            for (int a = 0; a < 3; a++) {
                f[a] = down((double)f[a] + t[a]);
                f[3 + a] = up((double)f[3 + a] + t[a]);
            }
        }
    for (int a = 0; a < 3; a++) L.tshift[a] = t[a];
}

// What trace_simple relies on without checking it per step: every slot of
// the DNodes reachable from the root is a sphere or an inner node (no
// DK_NONE), and no chain of nodes with two inner children is longer than the
// stack_need the kernel's STACK is chosen by (launchStack: need <= STACK).
bool checkSimpleNodes(const HostLayout& L) {
    if ((L.bvh_root >> KIND_SHIFT) != DK_BVH) return (L.bvh_root >> KIND_SHIFT) == DK_SPHERE;
    std::vector<uint32_t> memo(L.node.size(), ~0u);
    std::function<uint32_t(uint32_t, int)> need = [&](uint32_t i, int depth) -> uint32_t {
        if (i >= L.node.size() || depth > 4096) return ~0u;
        if (memo[i] != ~0u) return memo[i];
        const DNode& d = L.node[i];
        uint32_t n[2] = {0, 0};
        bool inner[2];
        for (int k = 0; k < 2; k++) {
            const uint32_t ref = k == 0 ? d.ref_a : d.ref_b, kind = ref >> KIND_SHIFT;
            inner[k] = kind == DK_BVH;
            if (kind != DK_SPHERE && kind != DK_BVH) return ~0u;
            if (inner[k] && (n[k] = need(ref & INDEX_MASK, depth + 1)) == ~0u) return ~0u;
        }
        return memo[i] = (inner[0] && inner[1]) ? 1 + std::max(n[0], n[1]) : std::max(n[0], n[1]);
    };
    const uint32_t n = need(L.bvh_root & INDEX_MASK, 0);
    return n != ~0u && n <= L.stack_need;  // (trace_simple's sentinel: LDS entries <= n - 1 <= STACK - 1)
}

// every slot of the DNode twins reachable from node i is an inline sphere or
// an inner node (what trace_dnodes relies on)
bool sphereNodesOnly(const HostLayout& L, uint32_t i, int depth = 0) {
    if (i >= L.node.size() || depth > 4096) return false;
    const DNode& d = L.node[i];
    for (uint32_t ref : {d.ref_a, d.ref_b}) {
        const uint32_t k = ref >> KIND_SHIFT;
        if (k == DK_BVH) {
            if (!sphereNodesOnly(L, ref & INDEX_MASK, depth + 1)) return false;
        } else if (k != DK_SPHERE) {
            return false;
        }
    }
    return true;
}

// every slot of the DNode twins reachable from node i is an inner node or a
// leaf trace_dnodes<LEAVES> tests in place (TOP_DTREE)
bool dtreeNodesOnly(const HostLayout& L, uint32_t i, int depth = 0) {
    if (i >= L.node.size() || depth > 4096) return false;
    const DNode& d = L.node[i];
    for (uint32_t ref : {d.ref_a, d.ref_b}) {
        const uint32_t k = ref >> KIND_SHIFT;
        if (k == DK_BVH) {
            if (!dtreeNodesOnly(L, ref & INDEX_MASK, depth + 1)) return false;
        } else if (k != DK_SPHERE && k != DK_MSPHERE && k != DK_BOX6 && k != DK_RECT) {
            return false;
        }
    }
    return true;
}

// true when `ref` is a BvhNode whose leaves are only spheres, rectangles and
// Boxes (no instance, list or medium below it): its DNode twin holds only the
// slots dtreeNodesOnly accepts (buildGeneralNodes)
bool dtreeLeaves(const HostLayout& L, uint32_t ref, int depth = 0) {
    const uint32_t kind = ref >> KIND_SHIFT, idx = ref & INDEX_MASK;
    if (depth > 4096) return false;
    if (kind == DK_BVH) return dtreeLeaves(L, L.bvh[idx].left, depth + 1) && dtreeLeaves(L, L.bvh[idx].right, depth + 1);
    if (kind == DK_SPHERE || kind == DK_MSPHERE || kind == DK_RECT) return true;
    return kind == DK_RECTS && L.list[idx].box6 != 0;
}

// true when everything below `ref` is BvhNodes and spheres
bool onlyBvhSpheres(const HostLayout& L, uint32_t ref, int depth = 0) {
    const uint32_t kind = ref >> KIND_SHIFT, idx = ref & INDEX_MASK;
    if (depth > 200) return false;
    if (kind == DK_SPHERE) return true;
    if (kind != DK_BVH) return false;
    return onlyBvhSpheres(L, L.bvh[idx].left, depth + 1) && onlyBvhSpheres(L, L.bvh[idx].right, depth + 1);
}

// A rectangle list that is a Box's six sides (box.h:29-38: XY at z1 and z0,
// XZ at y1 and y0, YZ at x1 and x0, each spanning the box): its DBox6, whose
// unrolled scan (box6_scan) performs the same tests in the same order.
// Returns 1 + the DBox6 index, or 0.
uint32_t detectBox6(HostLayout& L, uint32_t first, uint32_t count) {
    if (count != 6) return 0;
    const DRect* q = &L.rect[first];
    const float x0 = q[0].a0, x1 = q[0].a1, y0 = q[0].b0, y1 = q[0].b1, z1 = q[0].k, z0 = q[1].k;
    const float y1b = q[2].k, y0b = q[3].k, x1b = q[4].k, x0b = q[5].k;
    auto same = [](float a, float b) { return std::memcmp(&a, &b, sizeof a) == 0; };
    const uint32_t ax[6] = {0, 0, 1, 1, 2, 2};
    for (int j = 0; j < 6; j++)
        if ((q[j].axis & 3u) != ax[j]) return 0;
    // XY sides: x, y bounds; XZ sides: x, z bounds; YZ sides: y, z bounds
    const float zlo = q[2].b0, zhi = q[2].b1;
    const bool ok = same(q[1].a0, x0) && same(q[1].a1, x1) && same(q[1].b0, y0) && same(q[1].b1, y1) &&
                    same(q[2].a0, x0) && same(q[2].a1, x1) && same(q[3].a0, x0) && same(q[3].a1, x1) &&
                    same(q[3].b0, zlo) && same(q[3].b1, zhi) && same(zlo, z0) && same(zhi, z1) &&
                    same(q[4].a0, y0) && same(q[4].a1, y1) && same(q[4].b0, z0) && same(q[4].b1, z1) &&
                    same(q[5].a0, y0) && same(q[5].a1, y1) && same(q[5].b0, z0) && same(q[5].b1, z1) &&
                    same(y1b, y1) && same(y0b, y0) && same(x1b, x1) && same(x0b, x0);
    if (!ok) return 0;
    DBox6 b{};
    b.lo[0] = x0, b.lo[1] = y0, b.lo[2] = z0;
    b.hi[0] = x1, b.hi[1] = y1, b.hi[2] = z1;
    b.first = first;
    L.box6.push_back(b);
    return (uint32_t)L.box6.size();
}

struct Converter {
    const rtow_scene& s;
    HostLayout& L;
    std::unordered_map<uint32_t, uint32_t> memo;
    std::string err;
    int depth = 0;

    bool boxOf(uint32_t hi, float* mn, float* mx) {
        // exact reference bounding boxes where the kernel may cull with them
        const rtow_hitable& h = s.hitables[hi];
        switch (h.kind) {
        case RTOW_HIT_BVH_NODE:
            for (int a = 0; a < 3; a++) {
                mn[a] = h.f[a];
                mx[a] = h.f[3 + a];
            }
            return true;
        case RTOW_HIT_SPHERE:
            for (int a = 0; a < 3; a++) {
                mn[a] = h.f[a] - h.f[3];
                mx[a] = h.f[a] + h.f[3];
            }
            return true;
        case RTOW_HIT_BOX:  // box.h:16-19: every side lies on it
            for (int a = 0; a < 3; a++) {
                mn[a] = h.f[a];
                mx[a] = h.f[3 + a];
            }
            return true;
        case RTOW_HIT_MOVING_SPHERE: {
            const float r = h.f[8];
            for (int a = 0; a < 3; a++) {
                // center(t0) = c0, center(t1) = c1 up to rounding; pad by the radius
                float lo = std::min(h.f[a], h.f[3 + a]), hi2 = std::max(h.f[a], h.f[3 + a]);
                mn[a] = lo - r;
                mx[a] = hi2 + r;
            }
            return true;
        }
        default:
            for (int a = 0; a < 3; a++) {
                mn[a] = -FLT_MAX;
                mx[a] = FLT_MAX;
            }
            return true;
        }
    }

    uint32_t conv(uint32_t hi, bool underBvh) {
        auto it = memo.find(hi);
        if (it != memo.end()) return it->second;
        if (hi >= s.n_hitables || ++depth > 4096) {
            err = "bad hitable index or cyclic scene";
            return mkref(DK_NONE, 0);
        }
        const rtow_hitable& h = s.hitables[hi];
        uint32_t ref = mkref(DK_NONE, 0);
        switch (h.kind) {
        case RTOW_HIT_SPHERE:
        case RTOW_HIT_MOVING_SPHERE: {
            // one leaf format for both classes (rtow_device_layout.h)
            DSphere d{};
            const bool moving = h.kind == RTOW_HIT_MOVING_SPHERE;
            for (int a = 0; a < 3; a++) {
                d.c0[a] = h.f[a];
                d.dc[a] = moving ? h.f[3 + a] - h.f[a] : 0.0f;  // (_center1 - _center0), sphere.h:130
            }
            d.t0 = moving ? h.f[6] : 0.0f;
            d.t1 = moving ? h.f[7] : 1.0f;
            d.r = moving ? h.f[8] : h.f[3];
            d.mat = h.a;
            d.moving = moving ? 1u : 0u;
            ref = mkref(DK_SPHERE, (uint32_t)L.sph.size());
            L.sph.push_back(d);
            break;
        }
        case RTOW_HIT_RECT_XY:
        case RTOW_HIT_RECT_XZ:
        case RTOW_HIT_RECT_YZ: {
            DRect d{};
            d.a0 = h.f[0];
            d.a1 = h.f[1];
            d.b0 = h.f[2];
            d.b1 = h.f[3];
            d.k = h.f[4];
            d.axis = h.kind == RTOW_HIT_RECT_XY ? 0u : (h.kind == RTOW_HIT_RECT_XZ ? 1u : 2u);
            d.mat = h.a;
            ref = mkref(DK_RECT, (uint32_t)L.rect.size());
            L.rect.push_back(d);
            break;
        }
        case RTOW_HIT_FLIP_NORMALS:
            if (s.hitables[h.a].kind >= RTOW_HIT_RECT_XY && s.hitables[h.a].kind <= RTOW_HIT_RECT_YZ) {
                // FlipNormals(rectangle): the flip folds into a copy of the leaf
                const uint32_t leaf = conv(h.a, underBvh);
                if ((leaf >> KIND_SHIFT) != DK_RECT) return mkref(DK_NONE, 0);
                DRect d = L.rect[leaf & INDEX_MASK];
                d.axis ^= RECT_FLIP;
                ref = mkref(DK_RECT, (uint32_t)L.rect.size());
                L.rect.push_back(d);
                break;
            }
            [[fallthrough]];
        case RTOW_HIT_TRANSLATE:
        case RTOW_HIT_ROTATE_Y: {
            uint32_t k = h.kind == RTOW_HIT_FLIP_NORMALS ? DK_FLIP : (h.kind == RTOW_HIT_TRANSLATE ? DK_TRANSLATE : DK_ROTY);
            uint32_t slot = (uint32_t)L.inst.size();
            L.inst.push_back(DInst{});
            ref = mkref(k, slot);
            memo[hi] = ref;
            uint32_t child = conv(h.a, underBvh);
            DInst d{};
            d.child = child;
            for (int a = 0; a < 6; a++) d.p[a] = (k == DK_ROTY && a >= 2) ? 0.0f : h.f[a];
            L.inst[slot] = d;
            break;
        }
        case RTOW_HIT_LIST: {
            uint32_t slot = (uint32_t)L.list.size();
            L.list.push_back(DList{});
            ref = mkref(DK_LIST, slot);
            memo[hi] = ref;
            uint32_t first = (uint32_t)L.refs.size();
            L.refs.resize(L.refs.size() + h.b + 1);
            L.refs[first + h.b] = mkref(DK_NONE, 0);  // end of this list's items (DK_LISTNEXT)
            bool rects = h.b > 0 && h.b <= 16;
            for (uint32_t i = 0; i < h.b; i++) {
                uint32_t c = conv(s.refs[h.a + i], underBvh);
                L.refs[first + i] = c;
                rects = rects && (c >> KIND_SHIFT) == DK_RECT;
            }
            L.list[slot] = DList{first, h.b, 0, 0};
            if (rects) {  // e.g. a Box's six sides: one fused loop over contiguous leaves
                const uint32_t r0 = (uint32_t)L.rect.size();
                for (uint32_t i = 0; i < h.b; i++) L.rect.push_back(L.rect[L.refs[first + i] & INDEX_MASK]);
                L.list[slot] = DList{r0, h.b, 0, 0};
                L.list[slot].box6 = detectBox6(L, r0, h.b);
                ref = mkref(DK_RECTS, slot);
            }
            break;
        }
        case RTOW_HIT_BOX:
            ref = conv(h.a, underBvh);
            break;
        case RTOW_HIT_BVH_NODE: {
            if (h.a == h.b) {  // n == 1 node: both children are the same leaf
                ref = conv(h.a, true);
                L.collapsed_of[ref] = (uint32_t)(L.collapsed_own.size() / 6);
                L.collapsed_own.insert(L.collapsed_own.end(), h.f, h.f + 6);
                break;
            }
            uint32_t slot = (uint32_t)L.bvh.size();
            L.bvh.push_back(DBvh{});
            L.bvh_own.resize(L.bvh.size() * 6, 0.0f);
            for (int q = 0; q < 6; q++) L.bvh_own[6 * (size_t)slot + q] = h.f[q];
            ref = mkref(DK_BVH, slot);
            memo[hi] = ref;
            uint32_t l = conv(h.a, true), r = conv(h.b, true);
            DBvh d{};
            float lmn[3], lmx[3], rmn[3], rmx[3];
            boxOf(h.a, lmn, lmx);
            boxOf(h.b, rmn, rmx);
            d.xs[0] = lmn[0]; d.xs[1] = lmx[0]; d.xs[2] = rmn[0]; d.xs[3] = rmx[0];
            d.ys[0] = lmn[1]; d.ys[1] = lmx[1]; d.ys[2] = rmn[1]; d.ys[3] = rmx[1];
            d.zs[0] = lmn[2]; d.zs[1] = lmx[2]; d.zs[2] = rmn[2]; d.zs[3] = rmx[2];
            d.left = l;
            d.right = r;
            L.bvh[slot] = d;
            break;
        }
        case RTOW_HIT_CONSTANT_MEDIUM: {
            (void)underBvh;  // below a BvhNode: replayed in the reference's visit order (ProgramBuilder)
            L.has_media = true;
            uint32_t slot = (uint32_t)L.med.size();
            L.med.push_back(DMedium{});
            ref = mkref(DK_MEDIUM, slot);
            memo[hi] = ref;
            uint32_t b = conv(h.a, underBvh);
            L.med[slot] = DMedium{b, h.b, 1.0f / h.f[0], 0};
            break;
        }
        default:
            err = "unknown hitable kind";
            return mkref(DK_NONE, 0);
        }
        memo[hi] = ref;
        depth--;
        return ref;
    }
};

// Upper bound on the traversal stack (entries) and instance nesting a ray
// can need below `ref`; media add their boundary's sub-traversal.
struct Bounds {
    const HostLayout& L;
    std::unordered_map<uint32_t, std::pair<uint32_t, uint32_t>> memo;
    bool mediaInBoundary = false;
    std::pair<uint32_t, uint32_t> need(uint32_t ref, bool inMedium) {
        auto it = memo.find(ref);
        if (it != memo.end() && !inMedium) return it->second;
        const uint32_t kind = ref >> KIND_SHIFT, idx = ref & INDEX_MASK;
        std::pair<uint32_t, uint32_t> r{0, 0};
        switch (kind) {
        case DK_BVH: {
            auto a = need(L.bvh[idx].left, inMedium), b = need(L.bvh[idx].right, inMedium);
            r = {1 + std::max(a.first, b.first), std::max(a.second, b.second)};
            break;
        }
        case DK_LIST: {
            const DList& l = L.list[idx];
            for (uint32_t i = 0; i < l.count; i++) {
                auto c = need(L.refs[l.first + i], inMedium);
                r.first = std::max(r.first, (i + 1 < l.count ? 1u : 0u) + c.first);  // one DK_LISTNEXT
                r.second = std::max(r.second, c.second);
            }
            break;
        }
        case DK_TRANSLATE:
        case DK_ROTY:
        case DK_FLIP: {
            auto c = need(L.inst[idx].child, inMedium);
            r = {1 + c.first, 1 + c.second};
            break;
        }
        case DK_MEDIUM: {
            if (inMedium) mediaInBoundary = true;
            auto c = need(L.med[idx].boundary, true);
            r = c;
            break;
        }
        case DK_PROG:  // every item (media too) runs below a two-entry continuation
            for (uint32_t p = idx; p < L.prog.size() && L.prog[p].op != PROG_END; p++) {
                if (L.prog[p].op != PROG_ITEM) continue;
                const uint32_t it = L.prog[p].arg;
                auto c = need(it, inMedium);
                // the kernel pushes (tin, DK_PROGNEXT) for every item, media included
                const uint32_t cont = 2u;
                r = {std::max(r.first, cont + c.first), std::max(r.second, c.second)};
            }
            break;
        default:
            break;
        }
        if (!inMedium) memo[ref] = r;
        return r;
    }
};

// For every rectangle, the own boxes of the reference BvhNodes above it in
// its frame (DevScene::rect_anc / abox; ref_reaches_rect), n == 1 nodes
// included (collapsed into their leaf here, still tested by AABB::hit there:
// a ray through the edge two adjacent Boxes share grazes such a node's box,
// which is the Box's own).  A Translate or RotateY starts a new frame (boxes above it see another ray: dropped, so
// those are not checked); FlipNormals keeps the ray.  Medium boundaries are
// queried with (-FLT_MAX, FLT_MAX) and sit below no BvhNode: not recorded.
void refAncestors(HostLayout& L, uint32_t ref, std::vector<uint32_t>& path, int depth = 0) {
    if (depth > 4096) return;
    const uint32_t kind = ref >> KIND_SHIFT, idx = ref & INDEX_MASK;
    // path entries: a BvhNode slot, or (bit 31) a collapsed n == 1 node's box
    const auto col = L.collapsed_of.find(ref);
    const bool collapsed = col != L.collapsed_of.end();
    if (collapsed) path.push_back(0x80000000u | col->second);
    auto record = [&](uint32_t rect) {
        if (path.empty() || path.size() > 255 || rect >= L.rect_anc.size()) return;
        const uint32_t off = (uint32_t)(L.abox.size() / 8);
        if (off >= (1u << 24)) return;
        for (uint32_t b : path) {
            const bool c = (b & 0x80000000u) != 0;
            const size_t at = 6 * (size_t)(b & 0x7fffffffu);
            if (at + 6 > (c ? L.collapsed_own.size() : L.bvh_own.size())) return;  // (not a reference node)
        }
        for (uint32_t b : path) {
            const float* o = (b & 0x80000000u) ? &L.collapsed_own[6 * (size_t)(b & 0x7fffffffu)]
                                               : &L.bvh_own[6 * (size_t)b];
            const float box[8] = {o[0], o[1], o[2], 0.0f, o[3], o[4], o[5], 0.0f};
            L.abox.insert(L.abox.end(), box, box + 8);
        }
        L.rect_anc[rect] = (off << 8) | (uint32_t)path.size();
    };
    switch (kind) {
    case DK_BVH:
        path.push_back(idx);
        refAncestors(L, L.bvh[idx].left, path, depth + 1);
        refAncestors(L, L.bvh[idx].right, path, depth + 1);
        path.pop_back();
        break;
    case DK_LIST:
        for (uint32_t j = 0; j < L.list[idx].count; j++) refAncestors(L, L.refs[L.list[idx].first + j], path, depth + 1);
        break;
    case DK_RECTS:
        for (uint32_t j = 0; j < L.list[idx].count; j++) record(L.list[idx].first + j);
        break;
    case DK_RECT:
        record(idx);
        break;
    case DK_FLIP:
        refAncestors(L, L.inst[idx].child, path, depth + 1);
        break;
    case DK_TRANSLATE:
    case DK_ROTY: {
        std::vector<uint32_t> fresh;
        refAncestors(L, L.inst[idx].child, fresh, depth + 1);
        break;
    }
    default:
        break;
    }
    if (collapsed) path.pop_back();
}

// BvhNode subtrees that hold media become DProg programs (DK_PROG): the
// reference's own BvhNode boxes (bvhNode.h:58; an n == 1 node's too) in
// depth-first order, each with how many entries its children take, the
// media as items called with the subtree's interval, every medium-free child
// as one item for the general traversal.  Run after the tie keys, the
// rectangles' ancestor boxes and the SAH rebuild (none of which touch a
// subtree with media) on the reference graph.
struct ProgramBuilder {
    HostLayout& L;
    std::string err;

    void box(const float* o, std::vector<DProg>& P) {
        DProg e{};
        for (int a = 0; a < 3; a++) {
            e.lo[a] = o[a];
            e.hi[a] = o[3 + a];
        }
        e.op = PROG_BOX;
        P.push_back(e);
    }
    void item(uint32_t ref, std::vector<DProg>& P) {
        DProg e{};
        e.op = PROG_ITEM;
        e.arg = ref;
        P.push_back(e);
    }
    // a child of a BvhNode with media (or a subtree root): an n == 1 node
    // (collapsed into its leaf by the converter) calls its leaf twice
    void child(uint32_t ref, std::vector<DProg>& P, int depth) {
        const auto col = L.collapsed_of.find(ref);
        if (col != L.collapsed_of.end() && refHasMedium(L, ref)) {
            const size_t at = P.size();
            box(&L.collapsed_own[6 * (size_t)col->second], P);
            node(ref, P, depth + 1);
            node(ref, P, depth + 1);
            P[at].arg = (uint32_t)(P.size() - at - 1);
            return;
        }
        node(ref, P, depth + 1);
    }
    void node(uint32_t ref, std::vector<DProg>& P, int depth) {
        if (depth > 512) {
            err = "BvhNode subtree with media too deep";
            return;
        }
        const uint32_t kind = ref >> KIND_SHIFT, idx = ref & INDEX_MASK;
        if (kind == DK_BVH && refHasMedium(L, ref)) {
            if (6 * (size_t)idx + 6 > L.bvh_own.size()) {
                err = "BvhNode with media without its own box";
                return;
            }
            const size_t at = P.size();
            box(&L.bvh_own[6 * (size_t)idx], P);
            child(L.bvh[idx].left, P, depth);
            child(L.bvh[idx].right, P, depth);
            P[at].arg = (uint32_t)(P.size() - at - 1);
        } else if (kind == DK_MEDIUM || !refHasMedium(L, ref)) {
            item(ref, P);
        } else {
            // an instance or list with media below a BvhNode would hand its
            // media the list's shrinking interval / its own frame: not replayed
            err = "ConstantMedium below a BvhNode behind an instance or a list";
        }
    }
    void patch(uint32_t& ref, int depth = 0) {
        if (depth > 512 || !err.empty()) return;
        const uint32_t kind = ref >> KIND_SHIFT, idx = ref & INDEX_MASK;
        const bool n1 = L.collapsed_of.count(ref) != 0;
        if ((kind == DK_BVH || n1) && refHasMedium(L, ref)) {
            const uint32_t start = (uint32_t)L.prog.size();
            std::vector<DProg> P;
            child(ref, P, 0);
            DProg end{};
            end.op = PROG_END;
            P.push_back(end);
            L.prog.insert(L.prog.end(), P.begin(), P.end());
            ref = mkref(DK_PROG, start);
            return;
        }
        switch (kind) {
        case DK_LIST: {
            const DList l = L.list[idx];
            for (uint32_t j = 0; j < l.count; j++) patch(L.refs[l.first + j], depth + 1);
            break;
        }
        case DK_TRANSLATE:
        case DK_ROTY:
        case DK_FLIP:
            patch(L.inst[idx].child, depth + 1);
            break;
        default:
            break;
        }
    }
};

// DTop descriptors of a general scene whose root, below its instances, is a
// list (empty otherwise)
void buildTop(HostLayout& L) {
    L.top.clear();
    // RTOW_DTREE=0: such trees go to the general traversal (TOP_GENERIC) instead (A/B)
    const char* dt = std::getenv("RTOW_DTREE");
    const bool dtree = !dt || std::atoi(dt) != 0;
    std::vector<uint32_t> path;
    uint32_t ref = L.root;
    for (int guard = 0; guard < 64; guard++) {
        const uint32_t k = ref >> KIND_SHIFT;
        if (k != DK_TRANSLATE && k != DK_ROTY && k != DK_FLIP) break;
        path.push_back(ref);
        ref = L.inst[ref & INDEX_MASK].child;
    }
    if ((ref >> KIND_SHIFT) != DK_LIST) return;
    uint32_t list_chain = ~0u;
    for (uint32_t c = 0; c < L.chains.size(); c++) {
        const DChain& C = L.chains[c];
        if (C.n != path.size()) continue;
        bool same = true;
        for (uint32_t k = 0; k < C.n; k++) same = same && C.ref[k] == path[k];
        if (same) {
            list_chain = c;
            break;
        }
    }
    if (list_chain == ~0u) return;
    const DList l = L.list[ref & INDEX_MASK];
    std::vector<uint32_t> items;
    for (uint32_t j = 0; j < l.count; j++) {
        const uint32_t item = L.refs[l.first + j];
        items.push_back(item);
        uint32_t leaf = item;
        for (int guard = 0; guard < 64; guard++) {
            const uint32_t k = leaf >> KIND_SHIFT;
            if (k != DK_TRANSLATE && k != DK_ROTY && k != DK_FLIP) break;
            leaf = L.inst[leaf & INDEX_MASK].child;
        }
        const uint32_t k = leaf >> KIND_SHIFT, i = leaf & INDEX_MASK;
        DTop t{TOP_GENERIC, item, 0, list_chain};
        if (k == DK_RECT) {
            t = DTop{TOP_RECTS, i, 1, L.rect[i].chain};
        } else if (k == DK_RECTS) {
            const DList& r = L.list[i];
            bool one = r.count > 0;
            for (uint32_t q = 1; q < r.count; q++) one = one && L.rect[r.first + q].chain == L.rect[r.first].chain;
            if (one) t = DTop{TOP_RECTS, r.first, r.count, L.rect[r.first].chain};
            if (one && r.box6) t = DTop{TOP_BOX6, r.box6 - 1, r.count, L.rect[r.first].chain};
        } else if (k == DK_SPHERE) {
            t = DTop{TOP_SPHERE, i, 0, L.sph[i].chain};
        } else if (k == DK_MEDIUM && L.med[i].bkind != MB_ANY) {
            t = DTop{TOP_MEDIUM, i, 0, L.med[i].chain};
        } else if (k == DK_BVH && leaf != item && GeneralSah{L, 0}.sphereInstance(item)) {
            uint32_t s0 = leaf;  // any leaf sphere gives the chain of the frame they share
            while ((s0 >> KIND_SHIFT) == DK_BVH) s0 = L.bvh[s0 & INDEX_MASK].left;
            t = DTop{TOP_SPHERES, i, 0, L.sph[s0 & INDEX_MASK].chain};
        } else if (k == DK_BVH && leaf == item && L.grid_of.count(item)) {
            const uint32_t g = L.grid_of[item];  // (the Boxes' frame: their sides' chain)
            t = DTop{TOP_GRID, g, 0, L.rect[L.box6[L.gcell[L.grid[g].cell0].box6].first].chain};
        } else if (k == DK_BVH && leaf == item && dtree && dtreeLeaves(L, item)) {
            t = DTop{TOP_DTREE, i, 0, list_chain};  // (the leaves sit in the list's frame: no instance below)
        }
        L.top.push_back(t);
    }
    // grids are walked by MODE 8 only, the MODE 5 kernel with grid_walk: in
    // worlds whose media (if any) are all TOP_MEDIUM items with sphere or Box
    // boundaries; elsewhere the grid's tree is traversed as before
    {
        bool other = L.media_any;
        std::vector<bool> topm(L.med.size(), false);
        for (const DTop& t : L.top)
            if (t.kind == TOP_MEDIUM) topm[t.a] = true;
        for (size_t q = 0; q < topm.size(); q++) other = other || !topm[q];
        L.grid_top = 0;
        for (size_t q = 0; q < L.top.size(); q++) {
            DTop& t = L.top[q];
            if (t.kind != TOP_GRID) continue;
            if (!other) {
                L.grid_top++;
                continue;
            }
            const uint32_t item = items[q];
            t = dtree && dtreeLeaves(L, item) ? DTop{TOP_DTREE, item & INDEX_MASK, 0, list_chain}
                                             : DTop{TOP_GENERIC, item, 0, list_chain};
        }
    }
    // in grid worlds (the MODE 8 kernels), runs of top-level spheres in one
    // frame become one item: the scan tests them in a loop over copies in
    // DevScene::tsph (the copy's `chain` holds the sphere's own index, for
    // the record and its tie key), one descriptor load and one dispatch for
    // the run instead of one per sphere.  (A/B, frames identical: final_ned
    // +2.8%; the loop in the MODE 5 kernel cost cornell / cornell_smoke 0.3 /
    // 0.8%, so those keep one item per sphere.)
    if (L.grid_top) {
        std::vector<DTop> merged;
        for (size_t q = 0; q < L.top.size();) {
            const DTop t = L.top[q];
            if (t.kind != TOP_SPHERE) {
                merged.push_back(t);
                q++;
                continue;
            }
            size_t e = q;
            while (e < L.top.size() && L.top[e].kind == TOP_SPHERE && L.top[e].chain == t.chain) e++;
            DTop m{TOP_SPHERE, (uint32_t)L.tsph.size(), (uint32_t)(e - q), t.chain};
            for (size_t k = q; k < e; k++) {
                DSphere c = L.sph[L.top[k].a];
                c.chain = L.top[k].a;
                L.tsph.push_back(c);
            }
            merged.push_back(m);
            q = e;
        }
        L.top = std::move(merged);
    }
    // where the scan's ray changes (traverse_top): a new frame, and a new
    // direction when the frames' rotations (their RotateY sines and cosines,
    // in chain order: translations leave the direction alone) differ.  Items
    // the general traversal runs (TOP_GENERIC) do not use the scan's ray, and
    // the first in-place item after one recomputes it.
    // the ray's frame: the chain's translations and rotations in order (a
    // FlipNormals leaves the ray alone), so items under chains that differ
    // only in flips share the scan's ray (cornell's walls: one ray for six)
    auto raySig = [&](uint32_t c) {
        std::vector<uint64_t> v;
        const DChain& C = L.chains[c];
        for (uint32_t k = 0; k < C.n; k++) {
            const uint32_t kind = C.ref[k] >> KIND_SHIFT;
            if (kind != DK_ROTY && kind != DK_TRANSLATE) continue;
            const DInst& I = L.inst[C.ref[k] & INDEX_MASK];
            uint32_t b[3];
            std::memcpy(b, I.p, 12);
            v.push_back((uint64_t)kind << 32 | b[0]);
            v.push_back((uint64_t)b[1] << 32 | b[2]);
        }
        return v;
    };
    auto dirSig = [&](uint32_t c) {
        std::vector<uint64_t> v;
        const DChain& C = L.chains[c];
        for (uint32_t k = 0; k < C.n; k++) {
            if ((C.ref[k] >> KIND_SHIFT) != DK_ROTY) continue;
            const DInst& I = L.inst[C.ref[k] & INDEX_MASK];
            uint32_t sb, cb;
            std::memcpy(&sb, &I.p[0], 4);
            std::memcpy(&cb, &I.p[1], 4);
            v.push_back((uint64_t)sb << 32 | cb);
        }
        return v;
    };
    uint32_t last = ~0u;
    std::vector<uint64_t> lastSig, lastRay;
    for (DTop& t : L.top) {
        if (t.kind == TOP_GENERIC) {  // (the kernel drops the scan's ray there)
            last = ~0u;
            continue;
        }
        if (t.chain == last) continue;
        std::vector<uint64_t> rs = raySig(t.chain);
        if (last != ~0u && rs == lastRay) {  // another chain, the same ray
            last = t.chain;
            continue;
        }
        std::vector<uint64_t> sig = dirSig(t.chain);
        t.kind |= TOP_NEWCHAIN;
        if (last == ~0u || sig != lastSig) t.kind |= TOP_NEWDIR;
        last = t.chain;
        lastSig = std::move(sig);
        lastRay = std::move(rs);
    }
}

// The DNode twin of every DBvh of a general scene (DevScene::gnode): sphere
// children with time0 = 0, time1 = 1 inline (center(time) = c0 + time * dc
// exactly, as sph_center computes it for them), other children as box slots
// (a non-inlined sphere as DK_MSPHERE, a Box as DK_BOX6: dnode_step scans its
// sides when its box is hit instead of visiting it); a lone sphere child goes
// to slot b, as in sahBuild.
void buildGeneralNodes(HostLayout& L) {
    L.node.assign(L.bvh.size(), DNode{});
    for (size_t i = 0; i < L.bvh.size(); i++) {
        const DBvh& b = L.bvh[i];
        uint32_t refs[2] = {b.left, b.right};
        float box[2][6];
        for (int k = 0; k < 2; k++) {
            box[k][0] = b.xs[2 * k], box[k][1] = b.ys[2 * k], box[k][2] = b.zs[2 * k];
            box[k][3] = b.xs[2 * k + 1], box[k][4] = b.ys[2 * k + 1], box[k][5] = b.zs[2 * k + 1];
        }
        bool inl[2];
        for (int k = 0; k < 2; k++) {
            inl[k] = false;
            if ((refs[k] >> KIND_SHIFT) == DK_SPHERE) {
                const DSphere& sp = L.sph[refs[k] & INDEX_MASK];
                inl[k] = sp.t0 == 0.0f && sp.t1 == 1.0f;
                if (!inl[k]) refs[k] = mkref(DK_MSPHERE, refs[k] & INDEX_MASK);
            } else if ((refs[k] >> KIND_SHIFT) == DK_RECTS && L.list[refs[k] & INDEX_MASK].box6) {
                refs[k] = mkref(DK_BOX6, L.list[refs[k] & INDEX_MASK].box6 - 1);  // scanned in the node step
            }
        }
        if (inl[0] && !inl[1]) {
            std::swap(refs[0], refs[1]);
            std::swap(inl[0], inl[1]);
            for (int q = 0; q < 6; q++) std::swap(box[0][q], box[1][q]);
        }
        DNode& d = L.node[i];
        for (int k = 0; k < 2; k++) {
            float* f = k == 0 ? d.a : d.b;
            (k == 0 ? d.ref_a : d.ref_b) = refs[k];
            if (inl[k]) {
                const DSphere& sp = L.sph[refs[k] & INDEX_MASK];
                f[0] = sp.c0[0], f[1] = sp.c0[1], f[2] = sp.c0[2], f[3] = sp.r * sp.r;
                f[4] = sp.dc[0], f[5] = sp.dc[1], f[6] = sp.dc[2];
            } else {
                for (int q = 0; q < 6; q++) f[q] = box[k][q];
                f[6] = 0.0f;
            }
        }
    }
    L.gnode = !L.bvh.empty();
}

bool textureNeedsUv(const rtow_scene& s, uint32_t ti, int guard = 0) {
    if (ti >= s.n_textures || guard > 32) return false;
    const rtow_texture& t = s.textures[ti];
    if (t.kind == RTOW_TEX_IMAGE) return true;
    if (t.kind == RTOW_TEX_CHECKER) return textureNeedsUv(s, t.a, guard + 1) || textureNeedsUv(s, t.b, guard + 1);
    return false;
}

}  // namespace

int buildLayout(const rtow_scene& s, HostLayout& L, int tree) {
    if (s.root >= s.n_hitables || !s.hitables || !s.materials || !s.textures || !s.perlin)
        return set_error(RTOW_E_INVALID, "incomplete scene");
    for (uint32_t i = 0; i < s.n_hitables; i++) {
        const rtow_hitable& h = s.hitables[i];
        if ((h.kind == RTOW_HIT_SPHERE || h.kind == RTOW_HIT_MOVING_SPHERE || h.kind == RTOW_HIT_RECT_XY ||
             h.kind == RTOW_HIT_RECT_XZ || h.kind == RTOW_HIT_RECT_YZ) &&
            h.a >= s.n_materials)
            return set_error(RTOW_E_INVALID, "material index out of range");
        if (h.kind == RTOW_HIT_LIST && (uint64_t)h.a + h.b > s.n_refs)
            return set_error(RTOW_E_INVALID, "list range out of range");
        if (h.kind == RTOW_HIT_CONSTANT_MEDIUM && h.b >= s.n_materials)
            return set_error(RTOW_E_INVALID, "phase material out of range");
    }
    Converter cv{s, L};
    L.root = cv.conv(s.root, false);
    if (!cv.err.empty()) return set_error(RTOW_E_UNSUPPORTED, cv.err);
    Bounds bd{L};
    auto nb = bd.need(L.root, false);
    L.stack_need = nb.first;
    L.chain_need = nb.second;
    if (L.chain_need > (uint32_t)MAXCHAIN)
        return set_error(RTOW_E_UNSUPPORTED, "instance nesting deeper than " + std::to_string(MAXCHAIN));
    for (const DSphere& sp : L.sph)
        if (sp.t0 != 0.0f || sp.t1 != 1.0f) L.unit_time = false;
    {
        uint32_t r = L.root;
        uint32_t n = 0;
        while (n < (uint32_t)ROOTCHAIN) {
            const uint32_t k = r >> KIND_SHIFT;
            if (k != DK_TRANSLATE && k != DK_ROTY && k != DK_FLIP) break;
            L.root_chain[n++] = r;
            r = L.inst[r & INDEX_MASK].child;
        }
        if (onlyBvhSpheres(L, r) && L.unit_time) {
            L.simple = true;
            L.root_chain_n = n;
            L.bvh_root = r;
            // DNode twin of every DBvh (same index): sphere children inline
            L.node.resize(L.bvh.size());
            for (size_t i = 0; i < L.bvh.size(); i++) {
                const DBvh& b = L.bvh[i];
                DNode& d = L.node[i];
                const uint32_t refs2[2] = {b.left, b.right};
                for (int k = 0; k < 2; k++) {
                    float* f = k == 0 ? d.a : d.b;
                    uint32_t& ref = k == 0 ? d.ref_a : d.ref_b;
                    ref = refs2[k];
                    if ((ref >> KIND_SHIFT) == DK_SPHERE) {
                        const DSphere& sp = L.sph[ref & INDEX_MASK];
                        f[0] = sp.c0[0]; f[1] = sp.c0[1]; f[2] = sp.c0[2]; f[3] = sp.r * sp.r;
                        f[4] = sp.dc[0]; f[5] = sp.dc[1]; f[6] = sp.dc[2];
                    } else {
                        f[0] = b.xs[2 * k]; f[1] = b.ys[2 * k]; f[2] = b.zs[2 * k];
                        f[3] = b.xs[2 * k + 1]; f[4] = b.ys[2 * k + 1]; f[5] = b.zs[2 * k + 1];
                        f[6] = 0.0f;
                    }
                }
            }
            if (tree == RTOW_TREE_SAH && (L.bvh_root >> KIND_SHIFT) == DK_BVH) rebuildSah(L);
            shiftBoxes(L);
            if (!checkSimpleNodes(L)) return set_error(RTOW_E_INVALID, "internal: simple-scene tree check failed");
        }
    }
    for (uint32_t i = 0; i < s.n_materials; i++) {
        const rtow_material& m = s.materials[i];
        DMat d{};
        d.kind = m.kind;
        d.tex = m.texture;
        d.param = m.param;
        d.inv_ri = (float)(1.0 / (double)m.param);
        for (int a = 0; a < 3; a++) d.albedo[a] = m.albedo[a];
        if ((m.kind == RTOW_MAT_LAMBERTIAN || m.kind == RTOW_MAT_DIFFUSE_LIGHT || m.kind == RTOW_MAT_ISOTROPIC) &&
            m.texture >= s.n_textures)
            return set_error(RTOW_E_INVALID, "texture index out of range");
        d.needs_uv = (m.kind == RTOW_MAT_METAL || m.kind == RTOW_MAT_DIELECTRIC) ? 0u
                                                                                 : (textureNeedsUv(s, m.texture) ? 1u : 0u);
        // a constant texture's colour inline (one record less to load per hit)
        if ((m.kind == RTOW_MAT_LAMBERTIAN || m.kind == RTOW_MAT_DIFFUSE_LIGHT || m.kind == RTOW_MAT_ISOTROPIC) &&
            s.textures[m.texture].kind == RTOW_TEX_CONSTANT) {
            d.tex = TEX_INLINE;
            for (int a = 0; a < 3; a++) d.albedo[a] = s.textures[m.texture].f[a];
        }
        L.mat.push_back(d);
    }
    for (uint32_t i = 0; i < s.n_textures; i++) {
        DTex d{};
        std::memcpy(&d, &s.textures[i], sizeof(rtow_texture));
        if (d.kind == RTOW_TEX_IMAGE && d.a >= s.n_images) return set_error(RTOW_E_INVALID, "image index out of range");
        if (d.kind == RTOW_TEX_CHECKER && (d.a >= s.n_textures || d.b >= s.n_textures))
            return set_error(RTOW_E_INVALID, "checker child out of range");
        // rtow_texture::c is unused for a checker (include/rtow.h): the device
        // reads DTex::c as the TEX_FLAT flag, so whatever the caller left there
        // must not reach it
        if (d.kind == RTOW_TEX_CHECKER) d.c = 0;
        L.tex.push_back(d);
    }
    // checkers of two constant textures: both colours inline (texture_at)
    for (DTex& d : L.tex) {
        if (d.kind != RTOW_TEX_CHECKER || s.textures[d.a].kind != RTOW_TEX_CONSTANT ||
            s.textures[d.b].kind != RTOW_TEX_CONSTANT)
            continue;
        d.c = TEX_FLAT;
        for (int a = 0; a < 3; a++) {
            d.f[a] = s.textures[d.a].f[a];
            d.g[a] = s.textures[d.b].f[a];
        }
    }
    L.ranvec.resize(256 * 4);
    L.perm.resize(256);
    for (int i = 0; i < 256; i++) {
        for (int a = 0; a < 3; a++) L.ranvec[4 * i + a] = s.perlin->ranvec[i][a];
        L.ranvec[4 * i + 3] = 0.0f;
        L.perm[i] = ((uint32_t)s.perlin->perm_x[i] & 255u) | (((uint32_t)s.perlin->perm_y[i] & 255u) << 8) |
                    (((uint32_t)s.perlin->perm_z[i] & 255u) << 16);
    }
    for (uint32_t i = 0; i < s.n_images; i++) {
        const rtow_image& im = s.images[i];
        if (im.channels != 3 || im.offset + (uint64_t)im.nx * im.ny * 3 > s.n_texel_bytes)
            return set_error(RTOW_E_INVALID, "image outside texel buffer (RGB8 expected)");
        L.img.push_back(DImage{im.nx, im.ny, im.offset});
    }
    if (s.n_texel_bytes) L.texels.assign(s.texels, s.texels + s.n_texel_bytes);
    // keep every array non-empty so each gets a valid device pointer
    if (L.bvh.empty()) L.bvh.push_back(DBvh{});
    {
        ChainAssigner ca(L);
        ca.walk(L.root);
        if (!ca.err.empty()) return set_error(RTOW_E_UNSUPPORTED, ca.err);
    }
    if (L.sph.size() > LEAF_MASK || L.rect.size() > LEAF_MASK || L.med.size() > LEAF_MASK)
        return set_error(RTOW_E_UNSUPPORTED, "more than 2^21 spheres, rectangles or media");
    L.sph_key.assign(L.sph.size(), 0ull);
    L.rect_key.assign(L.rect.size(), 0ull);
    L.med_key.assign(L.med.size(), 0ull);
    L.rect_lvl.assign(4 * L.rect.size(), 0u);
    L.rect_lmask.assign(L.rect.size(), 0ull);
    {
        std::vector<KeyComp> path;
        TieWalk tw;
        assignTieKeys(L, L.root, path, tw);
    }
    L.rect_anc.assign(L.rect.size(), 0u);
    if (!L.simple) {  // the reference BvhNodes above each rectangle (before the trees are rebuilt)
        std::vector<uint32_t> path;
        refAncestors(L, L.root, path);
    }
    // A medium inside a medium's boundary: the culled traversals cannot ask it
    // in the reference's order -- the world goes to the exact-order kernel
    bool exact = bd.mediaInBoundary;
    if (!exact && !L.simple && tree == RTOW_TREE_SAH) {  // after the tie keys: they come from the reference trees
        GeneralSah g{L, (uint32_t)L.bvh.size()};
        g.patch(L.root);
        Bounds bd2{L};
        L.stack_need = bd2.need(L.root, false).first;
    }
    if (!exact && !L.simple) {  // BvhNode subtrees with media: replayed programs (DK_PROG)
        ProgramBuilder pb{L};
        pb.patch(L.root);
        // a medium below a BvhNode behind an instance or inside a list: no
        // program replays it (a list hands it its own closest hit so far) --
        // the exact-order kernel does
        if (!pb.err.empty()) exact = true;
        if (!exact && !L.prog.empty()) {
            Bounds bd3{L};
            L.stack_need = bd3.need(L.root, false).first;
        }
    }
    // how each medium's boundary is queried (DMedium::bkind); REFERENCE mode
    // keeps the general traversal for all of them
    for (DMedium& M : L.med) {
        M.bkind = MB_ANY;
        if ((M.boundary >> KIND_SHIFT) == DK_SPHERE) {
            M.bkind = MB_SPHERE;
        } else if (tree == RTOW_TREE_SAH) {
            uint32_t ref = M.boundary;
            for (int guard = 0; guard < 64; guard++) {
                const uint32_t k = ref >> KIND_SHIFT;
                if (k != DK_TRANSLATE && k != DK_ROTY && k != DK_FLIP) break;
                ref = L.inst[ref & INDEX_MASK].child;
            }
            if ((ref >> KIND_SHIFT) == DK_RECTS) {
                const DList r = L.list[ref & INDEX_MASK];
                bool one = r.count > 0;
                for (uint32_t q = 1; q < r.count; q++) one = one && L.rect[r.first + q].chain == L.rect[r.first].chain;
                if (one) {
                    M.bkind = r.box6 ? MB_BOX6 : MB_RECTS;
                    M.bfirst = r.box6 ? r.box6 - 1 : r.first;
                    M.bcount = r.count;
                    M.bchain = L.rect[r.first].chain;
                }
            }
        }
        if (M.bkind == MB_ANY) L.media_any = true;
    }
    if (!exact && !L.simple) {
        if (tree == RTOW_TREE_SAH) buildTop(L);
        buildGeneralNodes(L);  // DNode twins of the SAH trees, or of the reference's own (RTOW_TREE_REFERENCE)
        // trace_dnodes (TOP_SPHERES) takes every non-sphere slot for an inner node
        for (const DTop& t : L.top)
            if (((t.kind & TOP_KIND_MASK) == TOP_SPHERES && !sphereNodesOnly(L, t.a)) ||
                ((t.kind & TOP_KIND_MASK) == TOP_DTREE && !dtreeNodesOnly(L, t.a)))
                return set_error(RTOW_E_INVALID, "internal: TOP_SPHERES / TOP_DTREE tree with a slot its loop does not test");
    }
    if (exact) {
        const int rc = buildExact(s, L);
        if (rc) return rc;
    } else if (!L.simple) {
        // the raw graph, for the rays whose record only the reference's own
        // recursion settles (xhit after ref_skips_hit / tie_unsettled)
        std::vector<int> memo(s.n_hitables, 0);
        L.xdepth = rawDepth(s, s.root, memo);
        if (L.xdepth > (uint32_t)XDEPTH)
            return set_error(RTOW_E_UNSUPPORTED, "scene graph deeper than " + std::to_string(XDEPTH) + " calls (or cyclic)");
        L.xh.resize(s.n_hitables);
        std::memcpy(L.xh.data(), s.hitables, sizeof(XHit) * s.n_hitables);
        L.xrefs.assign(s.refs, s.refs + s.n_refs);
        L.xroot = s.root;
    }
    // media the top-level scan does not ask (TOP_MEDIUM) are asked inside the
    // general traversal
    {
        std::vector<bool> top_med(L.med.size(), false);
        for (const DTop& t : L.top)
            if ((t.kind & TOP_KIND_MASK) == TOP_MEDIUM) top_med[t.a] = true;
        for (size_t i = 0; i < L.med.size(); i++)
            if (!top_med[i]) L.media_nested = true;
    }
    // finalize's "needs uv" bits (general scenes: finalize<false> reads them
    // from the leaf's own record instead of loading its material)
    if (!L.simple) {
        for (DRect& q : L.rect)
            if (q.mat < L.mat.size() && L.mat[q.mat].needs_uv) q.axis |= RECT_UV;
        for (DSphere& q : L.sph)
            if (!q.moving && q.mat < L.mat.size() && L.mat[q.mat].needs_uv) q.moving |= SPH_UV;
    }
    if (L.sph_key.empty()) L.sph_key.push_back(0);
    if (L.rect_key.empty()) L.rect_key.push_back(0);
    if (L.med_key.empty()) L.med_key.push_back(0);
    if (L.node.empty()) L.node.push_back(DNode{});
    if (L.sph.empty()) L.sph.push_back(DSphere{});
    if (L.rect.empty()) L.rect.push_back(DRect{});
    if (L.inst.empty()) L.inst.push_back(DInst{});
    if (L.list.empty()) L.list.push_back(DList{});
    if (L.refs.empty()) L.refs.push_back(0);
    if (L.med.empty()) L.med.push_back(DMedium{});
    if (L.img.empty()) L.img.push_back(DImage{});
    if (L.texels.empty()) L.texels.push_back(0);
    return RTOW_OK;
}

}  // namespace rtow_layout

using namespace rtow_layout;

extern "C" {

int rtow_scene_check(const rtow_scene* s, uint32_t* stack_need, uint32_t* chain_need) {
    if (!s) return set_error(RTOW_E_INVALID, "NULL scene");
    HostLayout L;
    const char* tr = std::getenv("RTOW_BVH");  // (as rtow_context_create reads it)
    int rc = buildLayout(*s, L, tr && std::string(tr) == "ref" ? RTOW_TREE_REFERENCE : RTOW_TREE_SAH);
    if (rc) return rc;
    if (L.stack_need > 64) return set_error(RTOW_E_UNSUPPORTED, "scene needs a traversal stack deeper than 64 entries");
    if (std::getenv("RTOW_LAYOUT_INFO"))
        std::fprintf(stderr,
                     "rtow-layout: simple %d gnode %d nodes %zu bvh %zu spheres %zu rects %zu lists %zu insts %zu media %zu "
                     "top %zu stack_need %u chain_need %u media_nested %d media_any %d\n",
                     (int)L.simple, (int)L.gnode, L.node.size(), L.bvh.size(), L.sph.size(), L.rect.size(), L.list.size(),
                     L.inst.size(), L.med.size(), L.top.size(), L.stack_need, L.chain_need, (int)L.media_nested,
                     (int)L.media_any);
    if (std::getenv("RTOW_LAYOUT_INFO"))
        for (size_t j = 0; j < L.top.size(); j++)
            std::fprintf(stderr, "rtow-layout: top[%zu] kind %u flags %03x a %08x b %u chain %u\n", j,
                         L.top[j].kind & TOP_KIND_MASK, L.top[j].kind >> 8, L.top[j].a, L.top[j].b, L.top[j].chain);
    if (std::getenv("RTOW_LAYOUT_INFO"))
        for (const DGrid& g : L.grid)
            std::fprintf(stderr, "rtow-layout: grid %ux%u axes %02x u %g..%g v %g..%g cell %g x %g h %g..%g margin %g (top %u)\n",
                         g.nu, g.nv, g.axes, g.u0, g.u1, g.v0, g.v1, g.wu, g.wv, g.hlo, g.hhi, g.margin, L.grid_top);
    if (const char* path = std::getenv("RTOW_LAYOUT_DUMP")) {  // (tools: every array the upload would copy)
        if (FILE* f = std::fopen(path, "wb")) {
            auto put = [&](const void* p, size_t n) {
                const uint64_t k = n;
                std::fwrite(&k, 8, 1, f);
                if (n) std::fwrite(p, 1, n, f);
            };
            auto vec = [&](const auto& v) { put(v.data(), v.size() * sizeof(v[0])); };
            vec(L.bvh), vec(L.node), vec(L.sph), vec(L.rect), vec(L.inst), vec(L.list), vec(L.refs), vec(L.med);
            vec(L.mat), vec(L.tex), vec(L.ranvec), vec(L.perm), vec(L.img), vec(L.texels), vec(L.sph_key);
            vec(L.rect_key), vec(L.med_key), vec(L.chains), vec(L.top), vec(L.tsph), vec(L.rect_lvl), vec(L.rect_lmask);
            vec(L.rect_anc), vec(L.abox), vec(L.prog), vec(L.box6), vec(L.grid), vec(L.gcell), vec(L.gq), vec(L.xh);
            vec(L.xrefs);
            const uint32_t sc[] = {L.root, L.stack_need, L.chain_need, L.has_media, L.media_any, L.gnode,
                                   L.media_nested, L.simple, L.unit_time, L.root_chain_n, L.root_chain[0],
                                   L.root_chain[1], L.root_chain[2], L.root_chain[3], L.bvh_root, L.grid_top,
                                   L.exact, L.xroot, L.xdepth};
            put(sc, sizeof sc);
            put(L.tshift, sizeof L.tshift);
            std::fclose(f);
        }
    }
    if (stack_need) *stack_need = L.stack_need;
    if (chain_need) *chain_need = L.chain_need;
    return RTOW_OK;
}

}  // extern "C"
