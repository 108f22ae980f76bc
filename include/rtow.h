/*
 * rtow.h — C-ABI of the MI355X path tracer (librtow_hip.so).
 *
 * This is the drop-in boundary for the reference's per-pixel render loop,
 * raytraceWorkerProcedure main.cpp:932-996.  The reference has
 * no FFI; the seam is that loop body, whose inputs are RenderProperties
 * (common.h:10-15), a Camera* (camera.h:10), a Hitable* world and a
 * WorkerImageBuffer (common.h:17-21) it writes in place.  Here:
 *
 *   Hitable* world         -> rtow_scene   (the object graph, flattened 1:1)
 *   Camera*                -> rtow_camera  (the basis camera.h:315-342 builds)
 *   RenderProperties       -> rtow_params
 *   WorkerImageBuffer      -> bgra_out     (W*H*4 bytes, layout main.cpp:982-989)
 *
 * Plain C types only: pointers, sizes, PODs.  Every function returns 0 on
 * success or a negative RTOW_E* code (rtow_error_string()); HIP errors are
 * reported as RTOW_E_HIP and the HIP message is kept for rtow_last_error().
 *
 * Scene-graph flattening order (so two producers of the same world produce
 * byte-identical rtow_scene arrays): depth-first pre-order from the root,
 * memoised by object identity (a shared object is emitted once and referenced
 * by index).  A hitable gets its index before its children are visited.
 * Children order: BvhNode left, right; HitableList items in order (the list's
 * refs range is reserved before its items are visited); Box -> its 6-side list;
 * FlipNormals/Translate/RotateY -> child; ConstantMedium -> boundary, then the
 * phase material.  Materials and textures are numbered at first use, in that
 * same walk; a CheckerTexture visits odd, then even.  Unused fields are zero.
 */
#ifndef RTOW_H
#define RTOW_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTOW_ABI_VERSION 1

/* ---- error codes ---------------------------------------------------------- */
enum {
    RTOW_OK = 0,
    RTOW_E_INVALID = -1,      /* bad argument / inconsistent scene */
    RTOW_E_UNSUPPORTED = -2,  /* scene construct the device path does not handle */
    RTOW_E_HIP = -3,          /* a HIP runtime call failed */
    RTOW_E_NO_DEVICE = -4,    /* no GPU visible */
    RTOW_E_IO = -5,           /* file read/write failed */
    RTOW_E_NOMEM = -6,
    RTOW_E_RCCL = -7          /* an RCCL call failed (rtow_multi_*: the ncclResult and its text
                                 are kept for rtow_last_error()) */
};

/* ---- scene graph ---------------------------------------------------------- */

/* One record per reference Hitable object.  Field use per kind:
 *   SPHERE         sphere.h:7-18       f[0..2] center, f[3] radius, a material
 *   MOVING_SPHERE  sphere.h:76-91      f[0..2] center0, f[3..5] center1,
 *                                      f[6] time0, f[7] time1, f[8] radius, a material
 *   RECT_XY        xy_rect.h:7-20      f[0] x0 f[1] x1 f[2] y0 f[3] y1 f[4] k, a material
 *   RECT_XZ        xy_rect.h:42-55     f[0] x0 f[1] x1 f[2] z0 f[3] z1 f[4] k, a material
 *   RECT_YZ        xy_rect.h:77-90     f[0] y0 f[1] y1 f[2] z0 f[3] z1 f[4] k, a material
 *   FLIP_NORMALS   hitable.h:25-42     a child
 *   TRANSLATE      hitable.h:44-51     a child, f[0..2] offset
 *   ROTATE_Y       hitable.h:74-88     a child, b hasBox, f[0] sinTheta, f[1] cosTheta,
 *                                      f[2..4] box min, f[5..7] box max
 *   LIST           hitableList.h:7-18  a first index in refs[], b count
 *   BOX            box.h:10-23         a its 6-side LIST, f[0..2] pMin, f[3..5] pMax
 *   BVH_NODE       bvhNode.h:12-23     a left, b right, f[0..2] box min, f[3..5] box max
 *   CONSTANT_MEDIUM constantMedium.h:10-24  a boundary, b phase material (ISOTROPIC),
 *                                      f[0] density
 */
enum {
    RTOW_HIT_SPHERE = 1,
    RTOW_HIT_MOVING_SPHERE = 2,
    RTOW_HIT_RECT_XY = 3,
    RTOW_HIT_RECT_XZ = 4,
    RTOW_HIT_RECT_YZ = 5,
    RTOW_HIT_FLIP_NORMALS = 6,
    RTOW_HIT_TRANSLATE = 7,
    RTOW_HIT_ROTATE_Y = 8,
    RTOW_HIT_LIST = 9,
    RTOW_HIT_BOX = 10,
    RTOW_HIT_BVH_NODE = 11,
    RTOW_HIT_CONSTANT_MEDIUM = 12
};

typedef struct rtow_hitable {
    uint32_t kind, a, b, c;
    float f[12];
} rtow_hitable; /* 64 bytes */

/* material.h:43-148.  LAMBERTIAN/DIFFUSE_LIGHT/ISOTROPIC use `texture`;
 * METAL uses albedo[] and param (= fuzz, already clamped to <= 1 as the
 * constructor material.h:60 does); DIELECTRIC uses param (= refIndex). */
enum {
    RTOW_MAT_LAMBERTIAN = 1,
    RTOW_MAT_METAL = 2,
    RTOW_MAT_DIELECTRIC = 3,
    RTOW_MAT_DIFFUSE_LIGHT = 4,
    RTOW_MAT_ISOTROPIC = 5
};

typedef struct rtow_material {
    uint32_t kind, texture;
    float param;
    float albedo[3];
    uint32_t pad[2];
} rtow_material; /* 32 bytes */

/* texture.h:11-79.  CONSTANT f[0..2] color; CHECKER a odd, b even;
 * NOISE f[0] scale, a filter flag; IMAGE a image index. */
enum {
    RTOW_TEX_CONSTANT = 1,
    RTOW_TEX_CHECKER = 2,
    RTOW_TEX_NOISE = 3,
    RTOW_TEX_IMAGE = 4
};

typedef struct rtow_texture {
    uint32_t kind, a, b, c;
    float f[4];
} rtow_texture; /* 32 bytes */

/* An RGB8 image as stbi_load returns it (scenes.h:140): nx*ny*3 bytes, row 0
 * first, at texels + offset. */
typedef struct rtow_image {
    uint32_t nx, ny, channels, pad;
    uint64_t offset;
} rtow_image; /* 24 bytes */

/* The static Perlin tables (noise.h:51-55, generated at noise.h:112-116). */
typedef struct rtow_perlin {
    float ranfloat[256];
    float ranvec[256][3];
    int32_t perm_x[256];
    int32_t perm_y[256];
    int32_t perm_z[256];
} rtow_perlin;

typedef struct rtow_scene {
    uint32_t root;
    uint32_t n_hitables;
    const rtow_hitable* hitables;
    uint32_t n_refs;
    const uint32_t* refs;
    uint32_t n_materials;
    const rtow_material* materials;
    uint32_t n_textures;
    const rtow_texture* textures;
    const rtow_perlin* perlin;
    uint32_t n_images;
    const rtow_image* images;
    uint64_t n_texel_bytes;
    const uint8_t* texels;
} rtow_scene;

/* ---- camera ----------------------------------------------------------------
 * The state Camera::getRay (camera.h:123-135) reads, as
 * setCamera_QuaternionMatrix (camera.h:315-342) leaves it. */
typedef struct rtow_camera {
    float origin[3];
    float lower_left_corner[3];
    float horizontal[3];
    float vertical[3];
    float u[3], v[3], w[3];
    float lens_radius;
    float time0, time1;
} rtow_camera;

/* ---- render parameters -----------------------------------------------------
 * Defaults (rtow_params_default) reproduce defines.h:23-27:
 * GLOBAL_ILLUM_EN 1, SKY_ILLUM_GAIN 1.0, GLOBAL_ILLUM_GAIN 0.3,
 * DEPTH_RECURSION 50.  Pixels are grouped in 8x8 tiles (tile t covers
 * columns 8*(t % tiles_x) .. and rows counted from the TOP of the image);
 * rank r of `world` renders tiles r, r+world, r+2*world, ... (the reference's
 * column interleave main.cpp:936, done by tiles). */
enum {
    RTOW_FLAG_STATS = 1u << 0,      /* count segments (color() calls) on device */
    RTOW_FLAG_CAMERA_DOF = 1u << 1, /* CAMERA_DOF_EN 1 (defines.h:26; off in the reference's
                                       build): Camera::getRay's offset is _lensRadius *
                                       randomInUnitDisk() + randomInUnitSphere() (camera.h:124-126) */
    RTOW_FLAG_FRAME_PLAN = 1u << 2  /* automatic chunking (samples_per_chunk 0) plans for the whole
                                       frame -- as rank 0 of world 1 -- whatever p->rank / p->world:
                                       every rank cuts its pixels' samples into the chunks rtow_render
                                       cuts, so the chunks' float sums, and the assembled frame, equal
                                       rtow_render's bit for bit.  Without it a rank's share plans for
                                       its own pixel count (shorter chunks on more ranks: a shorter
                                       grid tail, but other float chunk sums, so the last bits of the
                                       frame depend on the world size).  rtow_multi_render sets it. */
};

typedef struct rtow_params {
    uint32_t width, height;
    uint32_t spp;               /* antiAliasingSamplesPerPixel */
    uint32_t max_depth;         /* DEPTH_RECURSION */
    uint32_t gi_enable;         /* GLOBAL_ILLUM_EN */
    float sky_gain;             /* SKY_ILLUM_GAIN */
    float gi_gain;              /* GLOBAL_ILLUM_GAIN */
    uint32_t samples_per_chunk; /* work granularity: a work item is one pixel's chunk of consecutive
                                    samples, summed in float in sample order (main.cpp:946) and added to
                                    the pixel's sum in 192-bit fixed point (order-independent, exact);
                                    0 = auto (128, 64, 32 or 16: the longest leaving >= 30 items per
                                    lane of the grid, or spp/200 if larger; the last spc..2spc samples
                                    cut into halving chunks) -- rtow_render_plan shows the choice */
    uint64_t seed;              /* render stream seed (rtow_rng.h) */
    uint32_t rank, world;       /* tile partition; world 0 is treated as 1 */
    uint32_t flags;
    uint32_t blocks_per_cu;     /* persistent-grid blocks per CU; 0 = auto (the kernel's occupancy).
                                    Capped at that occupancy: blocks that cannot be resident add
                                    nothing to a persistent grid, so a larger request silently gets
                                    the occupancy (no error) */
} rtow_params;

typedef struct rtow_stats {
    uint64_t segments;   /* ray segments traced = reference color() calls */
    uint64_t samples;    /* paths (pixel samples) traced */
    uint64_t pixels;     /* pixels this call produced */
    double kernel_ms;    /* trace kernel, HIP events on the render stream */
    double resolve_ms;   /* pixel-sum average + quantise kernel */
    double total_ms;     /* whole call, host wall clock */
} rtow_stats;

/* ---- library ---------------------------------------------------------------- */
int rtow_abi_version(void);
const char* rtow_error_string(int code);
const char* rtow_last_error(void);
void rtow_params_default(rtow_params* p, uint32_t width, uint32_t height, uint32_t spp);

/* Number of tiles of an image, and how many of them rank r of world renders. */
uint32_t rtow_tile_count(uint32_t width, uint32_t height);
uint32_t rtow_rank_tile_count(uint32_t width, uint32_t height, uint32_t rank, uint32_t world);

/* ---- host-side scene construction (replaces scenes.h + main.cpp:111-137) --- */
enum {
    RTOW_SCENE_THREE_SPHERE = 1,  /* config 1: three Lambertian spheres (composed) */
    RTOW_SCENE_RANDOM_NED = 2,    /* randomScene_NED scenes.h:122-218, n parameterised */
    RTOW_SCENE_CORNELL_NED = 3,   /* cornellBox_NED scenes.h:355-483 */
    RTOW_SCENE_CORNELL_SMOKE = 4, /* cornellBox_NED + smoke box of scenes.h:461-470 */
    RTOW_SCENE_FINAL_NED = 5,     /* config 5: book 2's final scene composed from the reference's
                                     classes in NED; root Translate (600,-278,278) */
    RTOW_SCENE_RANDOM = 6,        /* randomScene scenes.h:29-120 (not NED; no root Translate: main.cpp
                                     renders the NED builders), n parameterised; its image is
                                     input_images/earth1300x1300.jpg (scenes.h:47) */
    RTOW_SCENE_CORNELL = 7        /* cornellBox scenes.h:220-353 (not NED; no root Translate) */
};

enum {
    RTOW_IMAGE_NONE = 0,       /* stbi_load failed: the reference's glass fallback */
    RTOW_IMAGE_SYNTHETIC = 1,  /* rtow_synthetic_image(2048, 1024) */
    RTOW_IMAGE_RAW = 2,        /* RGB8 raw file image_path, image_nx * image_ny * 3 */
    RTOW_IMAGE_JPEG = 3        /* JPEG file image_path, decoded as stbi_load(path, .., 0) decodes it
                                  (rtow_image_load_jpeg; scenes.h:140 loads 1_earth_8k.jpg) */
};

typedef struct rtow_build_opts {
    uint64_t scene_seed;       /* rtow_scene_key(scene_seed) drives Perlin + scene draws */
    uint32_t n;                /* randomScene_NED's n (reference: 100) */
    uint32_t image_mode;
    const char* image_path;
    uint32_t image_nx, image_ny;
    uint32_t wrap_world;       /* 1: add main.cpp's root Translate (main.cpp:132/136) */
    uint32_t ground_side;      /* final_ned: the ground's Boxes per side over the same 2000 x 2000
                                  (0: the book's 20; tests use larger grids) */
} rtow_build_opts;

typedef struct rtow_scene_buf rtow_scene_buf; /* owns the arrays an rtow_scene views */

void rtow_build_opts_default(rtow_build_opts* o);
int rtow_build_scene(int scene_id, const rtow_build_opts* opts, rtow_scene_buf** out);
const rtow_scene* rtow_scene_view(const rtow_scene_buf* buf);
void rtow_scene_free(rtow_scene_buf* buf);
int rtow_scene_save(const rtow_scene* scene, const char* path);
int rtow_scene_load(const char* path, rtow_scene_buf** out);
/* Number of random-stream draws the last rtow_build_scene consumed (diagnostic). */
uint32_t rtow_scene_draws(const rtow_scene_buf* buf);

/* The camera main.cpp:111-125 constructs for a width x height frame. */
int rtow_camera_main(uint32_t width, uint32_t height, rtow_camera* out);
/* The main camera after the GUI frame loop moved it (main.cpp:476/554 and
 * 624-628): Camera::setOrientationMatrix with rows view (w), east (u), down
 * (v) -- rows[0..2], [3..5], [6..8] -- and Camera::setLookFromPoint; the basis
 * as setCamera_QuaternionMatrix (camera.h:315-342) forms it. */
int rtow_camera_oriented(uint32_t width, uint32_t height, const float look_from[3], const float rows[9],
                         rtow_camera* out);
/* Camera(lookFrom, lookAt, up, vFoV, aspect, aperture, focusDistance, t0, t1)
 * with the basis of setCamera_Euler (camera.h:271-313: w = unit(lookFrom -
 * lookAt), u = unit(cross(up, w)), v = cross(w, u)), the classic look-at
 * camera; the reference's setCamera() compiles it out in favour of the
 * quaternion form (camera.h:344-350), so main.cpp never sees it. */
int rtow_camera_look_at(const float look_from[3], const float look_at[3], const float up[3], float vfov_deg,
                        float aspect, float aperture, float focus_distance, float time0, float time1,
                        rtow_camera* out);
/* JPEG decoding as the reference's stb_image.h v2.22 does it (stbi_load with
 * req_comp 0, scenes.h:140): baseline and progressive Huffman, 8-bit, 1/3/4
 * components, any sampling, restart intervals; same bytes as stbi_load
 * (tests/test_jpeg.py).  *pixels: nx * ny * channels bytes, row 0 first,
 * channels 3 (or 1 for a grayscale file); free with rtow_image_free. */
int rtow_image_decode_jpeg(const uint8_t* data, size_t size, uint8_t** pixels, uint32_t* nx, uint32_t* ny,
                           uint32_t* channels);
int rtow_image_load_jpeg(const char* path, uint8_t** pixels, uint32_t* nx, uint32_t* ny, uint32_t* channels);
void rtow_image_free(uint8_t* pixels);

/* Fill an RGB8 image with the synthetic "earth" stand-in. */
void rtow_synthetic_image(uint32_t nx, uint32_t ny, uint8_t* rgb);

/* ---- frame output ------------------------------------------------------------ */
/* The reference's BMP file (WINDIBBitmap::writeBMPToFile, winDIBbitmap.cpp:
 * 20-168, as main.cpp:774 calls it with the BGRA frame and 32 bpp): 54-byte
 * header with a POSITIVE height, then the buffer rows in order, each padded
 * to 4 bytes, so viewers show the top-down frame flipped exactly as the
 * reference's test.bmp.  size_bytes must be width*height*bits_per_pixel/8. */
int rtow_write_bmp(const char* path, const uint8_t* pixels, uint64_t size_bytes, uint32_t width,
                   uint32_t height, uint32_t bits_per_pixel);
/* Binary PPM (P6, RGB, top row first) of a BGRA frame, for inspection. */
int rtow_write_ppm(const char* path, const uint8_t* bgra, uint32_t width, uint32_t height);

/* ---- device path ------------------------------------------------------------ */
typedef struct rtow_context rtow_context;

int rtow_device_count(int* count);
int rtow_context_create(int device, rtow_context** out);
int rtow_context_destroy(rtow_context* ctx);
/* Host-only check that the device path can render `scene` (the conversion
 * rtow_scene_upload performs, without a GPU).  stack_need / chain_need (may
 * be NULL) receive the traversal-stack entries and instance nesting a ray
 * needs (for a world the exact-order kernel renders: the deepest hit() call
 * chain).  Returns RTOW_E_UNSUPPORTED (reason in rtow_last_error) e.g. for a
 * graph whose hit() recursion is deeper than 48 calls. */
int rtow_scene_check(const rtow_scene* scene, uint32_t* stack_need, uint32_t* chain_need);
/* Convert the scene graph to the device layout and copy it to HBM. */
int rtow_scene_upload(rtow_context* ctx, const rtow_scene* scene);

/* How the device organises the world (taking effect at the next
 * rtow_scene_upload).  The closest hit does not depend on it: exact ties are
 * settled by the reference's own evaluation order (BvhNode::hit,
 * bvhNode.h:74-77; HitableList::hit, hitableList.h:20-38) either way, so both
 * give the same frame.  SAH (default): surface-area-heuristic trees rebuilt
 * over the leaves of every BvhNode subtree and over runs of list items that
 * hold a large aggregate, and the top-level list scanned item by item.
 * REFERENCE: the reference's own random-axis median-split trees
 * (bvhNode.h:25-59) and lists, traversed as the object graph nests them.
 * The environment variable RTOW_BVH=ref|sah overrides the default at context
 * creation. */
enum {
    RTOW_TREE_SAH = 0,
    RTOW_TREE_REFERENCE = 1
};
int rtow_context_set_tree(rtow_context* ctx, int tree);

/* How a render with `p` cuts its work (diagnostic; host only): the samples per
 * work item the automatic chunking picks for this device's grid (or
 * p->samples_per_chunk), the full chunks per pixel, and the halving tail of
 * the last tail_samples samples in n_tail chunks.  ctx NULL plans for a
 * 256-CU MI355X without the RTOW_AUTO_SPC override.  The bench's config-2
 * frame (1920x1080x1024, one rank) gives 128-sample items, n_big 7 and a
 * 128-sample tail in 8 chunks (64, 32, ..., 1, 1). */
typedef struct rtow_plan {
    uint32_t samples_per_chunk;
    uint32_t n_big;         /* full chunks per pixel */
    uint32_t tail_samples;  /* samples of the halving tail (0: none) */
    uint32_t n_tail;        /* chunks of the tail */
    uint32_t n_chunks;      /* n_big + n_tail */
    uint32_t n_local_px;    /* pixels of the rank's tile slab (padding included) */
    uint64_t n_items;       /* work items = n_chunks * n_local_px */
    uint32_t cus;           /* compute units the plan assumed */
    uint32_t pad;
} rtow_plan;
int rtow_render_plan(const rtow_context* ctx, const rtow_params* p, rtow_plan* out);

/* Drop-in for main.cpp:932-996 on one GPU: render every pixel, write the BGRA
 * frame (host memory, W*H*4, alpha 0) and, if linear_out is not NULL, the
 * averaged linear RGB before sqrt/quantise (W*H*3 floats, same pixel order).
 * Synchronous. */
int rtow_render(rtow_context* ctx, const rtow_camera* cam, const rtow_params* p,
                uint8_t* bgra_out, float* linear_out, rtow_stats* stats);

/* Progressive rendering: the reference's GUI frame loop re-renders the frame
 * every iteration (main.cpp:247-687, camera updated through
 * setOrientationMatrix camera.h:231-235 / setLookFromPoint); here each call
 * renders p->spp NEW samples per pixel -- sample indices continue after the
 * ones already accumulated, so the random streams never repeat -- adds them to
 * the context's running sums and writes the average of everything so far.
 * The sums restart when `reset` is set, a scene is uploaded, or the camera
 * or any parameter other than spp / samples_per_chunk / blocks_per_cu /
 * RTOW_FLAG_STATS changed (RTOW_FLAG_CAMERA_DOF restarts them).  total_spp
 * (may be NULL) receives the samples per pixel accumulated.  F frames of S
 * spp, each one chunk (samples_per_chunk = S, or automatic chunking with
 * S <= 16), give the frame of one rtow_render of F*S spp with
 * samples_per_chunk = S, bit for bit. */
int rtow_render_progressive(rtow_context* ctx, const rtow_camera* cam, const rtow_params* p, int reset,
                            uint8_t* bgra_out, float* linear_out, uint32_t* total_spp, rtow_stats* stats);

/* Render this rank's tiles (p->rank of p->world) into compact DEVICE slabs:
 * tile-slot s of the rank holds global tile rank + s*world, 64 pixels row-major
 * inside the tile; d_bgra_slab gets 4 bytes per pixel, d_linear_slab (may be
 * NULL) 3 floats.  Enqueued on `stream` (a hipStream_t, NULL = the context's
 * own); returns after the work completes. */
int rtow_render_tiles_device(rtow_context* ctx, const rtow_camera* cam, const rtow_params* p,
                             void* d_bgra_slab, void* d_linear_slab, void* stream,
                             rtow_stats* stats);

/* Progressive rendering over this rank's tiles (p->rank of p->world): the
 * multi-GPU form of rtow_render_progressive.  Each call adds p->spp new samples
 * per pixel of the rank's tiles to the context's running sums (restarted as
 * rtow_render_progressive's are, and also when rank or world change) and
 * writes the average so far into DEVICE slabs laid out as
 * rtow_render_tiles_device's, ready for one gather and rtow_assemble_device.
 * The assembled frame of every rank's call equals rtow_render_progressive's
 * frame of the same calls bit for bit (the RNG is keyed by global pixel).
 * Enqueued on `stream` (NULL = the context's own); returns after the work
 * completes. */
int rtow_render_progressive_tiles_device(rtow_context* ctx, const rtow_camera* cam, const rtow_params* p,
                                         int reset, void* d_bgra_slab, void* d_linear_slab, void* stream,
                                         uint32_t* total_spp, rtow_stats* stats);

/* Diagnostic: render the frame with the segment-recording kernel and return
 * the path of ONE sample (pixel x, y of the top-down frame, sample index):
 * per color() call RTOW_DEBUG_SEG_FLOATS floats {hit, depth, t, p.xyz (the
 * ray direction on a miss), n.xyz, material, random draws so far, 1}; the
 * oracle's rtow_oracle_trace_sample writes the same records. */
#define RTOW_DEBUG_SEG_FLOATS 12
int rtow_debug_trace_sample(rtow_context* ctx, const rtow_camera* cam, const rtow_params* p, uint32_t x,
                            uint32_t y, uint32_t sample, float* out, uint32_t max_segments,
                            uint32_t* n_segments);

/* Scatter the gathered slabs of all `world` ranks (rank-major, each
 * rtow_rank_tile_count(...) * 64 pixels; equal-size padding allowed via
 * slab_stride_px) into a device BGRA frame. */
int rtow_assemble_device(rtow_context* ctx, uint32_t width, uint32_t height, uint32_t world,
                         const void* d_slabs, uint32_t slab_stride_px, void* d_bgra_frame,
                         void* stream);
/* The same for gathered LINEAR slabs (3 floats per pixel) into a device
 * W*H*3 float frame. */
int rtow_assemble_linear_device(rtow_context* ctx, uint32_t width, uint32_t height, uint32_t world,
                                const void* d_slabs, uint32_t slab_stride_px, void* d_linear_frame,
                                void* stream);

/* ---- several GPUs from one process -------------------------------------------
 * The reference renders a frame with N std::threads over one shared buffer,
 * thread i taking columns i, i+N, ... (main.cpp:182-195, 936).  rtow_multi is
 * that split across GPUs, for a caller that is one process (main.cpp):
 *   - one rtow_context per device (its stream, scene copy and buffers);
 *   - device i renders rank i of world n: the 8x8 tiles i, i+n, ... into a
 *     compact slab (rtow_render_tiles_device), all devices at once;
 *   - one RCCL gather: communicators from ncclCommInitAll over `devices`, the
 *     slabs sent to device 0 with grouped ncclSend / ncclRecv over xGMI (RCCL
 *     has no gather primitive); device 0's slab goes through RCCL too;
 *   - device 0 assembles the BGRA frame (and the linear one) and copies it out.
 * The frame equals rtow_render's bit for bit for any n: the RNG is keyed by
 * global pixel and sample, and the pixel sums are exact.  HIP failures return
 * RTOW_E_HIP, RCCL failures RTOW_E_RCCL (ncclResult text in rtow_last_error).
 * `devices`: n HIP device indices; the first entry's device gathers.
 * A device may be listed more than once: it then holds that many ranks (each
 * its own context and stream on the device, rendering at once), and because
 * RCCL allows one rank per device the WHOLE gather then uses device copies
 * (hipMemcpyPeerAsync into the first entry's slots) instead of RCCL, for
 * every entry, distinct ones included.  The frame is the same; the render is
 * an oversubscribed one (meant for running the n-rank path on fewer GPUs),
 * so list each device once for a real multi-GPU render. */
typedef struct rtow_multi rtow_multi;
int rtow_multi_create(const int* devices, uint32_t n_devices, rtow_multi** out);
int rtow_multi_destroy(rtow_multi* m);
uint32_t rtow_multi_device_count(const rtow_multi* m);
/* rtow_context_set_tree on every device (before rtow_multi_upload). */
int rtow_multi_set_tree(rtow_multi* m, int tree);
/* rtow_scene_upload on every device (the scene is replicated: <= ~10 MB). */
int rtow_multi_upload(rtow_multi* m, const rtow_scene* scene);
/* One frame over all devices (p->rank / p->world are ignored: device i is rank
 * i of n).  bgra_out: host W*H*4 (may be NULL); linear_out: host W*H*3 floats
 * (may be NULL).  stats: whole call -- segments / samples / pixels summed,
 * kernel_ms and resolve_ms the slowest device's, total_ms the wall clock
 * including the gather and assembly.  device_stats (may be NULL): n entries,
 * each device's own. */
int rtow_multi_render(rtow_multi* m, const rtow_camera* cam, const rtow_params* p, uint8_t* bgra_out,
                      float* linear_out, rtow_stats* stats, rtow_stats* device_stats);
/* create + upload + render + destroy in one call. */
int rtow_render_devices(const int* devices, uint32_t n_devices, const rtow_scene* scene, const rtow_camera* cam,
                        const rtow_params* p, uint8_t* bgra_out, float* linear_out, rtow_stats* stats);

#ifdef __cplusplus
}
#endif

#endif /* RTOW_H */
