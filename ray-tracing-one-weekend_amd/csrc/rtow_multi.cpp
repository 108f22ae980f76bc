// rtow_multi.cpp — several GPUs from one process (include/rtow.h, rtow_multi_*).
//
// The reference renders one frame with N std::threads over a shared buffer,
// thread i taking columns i, i+N, ... (main.cpp:182-195 start them, main.cpp:936
// interleaves the columns).  Here entry i of the device list is rank i of world
// n: it renders the 8x8 tiles i, i+n, ... of the frame into a compact slab on
// its own stream (rtow_render_tiles_device), all ranks at once (one host thread
// each: a render call returns when its work is done), then ONE gather brings
// the slabs to the first device and that device assembles the frame
// (rtow_assemble_device / _linear_device):
//   - n distinct devices: RCCL over xGMI -- communicators from ncclCommInitAll,
//     the gather as grouped ncclSend / ncclRecv (RCCL has no gather primitive);
//   - a device listed more than once (its ranks share it: each its own context
//     and stream; RCCL allows one rank per device): device copies
//     (hipMemcpyPeerAsync) onto the first device's stream.
// Every rank plans its chunks as the whole frame (RTOW_FLAG_FRAME_PLAN), so the
// frame equals rtow_render's bit for bit for any n.
//
// RCCL is opened on the first rtow_multi_create that needs it (dlopen of
// librccl.so.1, then $(ROCM)/lib's), so a caller that never uses several GPUs
// loads librtow_hip.so without it; missing RCCL is RTOW_E_RCCL.
//
// Host code over the public C-ABI plus HIP streams and RCCL; the kernels are
// rtow_device.hip's.  Payload: config 2's BGRA frame is 8.3 MB (1 MB per rank
// at n = 8), config 5's 67 MB -- microseconds to milliseconds against seconds
// of rendering.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rtow.h"
#include "rtow_internal.h"

#ifndef RTOW_ROCM_LIB
#define RTOW_ROCM_LIB "/opt/rocm/lib"
#endif

struct rtow_multi {
    std::vector<int> devices;
    bool shared = false;  // a device listed more than once: gather by device copies, no RCCL
    std::vector<rtow_context*> ctx;
    std::vector<ncclComm_t> comms;
    std::vector<hipStream_t> streams;
    // per rank: its slab (BGRA + linear); the first device also the gathered slabs and the frame
    std::vector<void*> slab_bgra, slab_lin;
    size_t slab_px = 0;  // slab capacity in pixels (every rank the same)
    void* gather_bgra = nullptr;
    void* gather_lin = nullptr;
    void* frame_bgra = nullptr;
    void* frame_lin = nullptr;
    size_t frame_px = 0;
};

namespace {

// ---- RCCL, resolved at first use ---------------------------------------------
struct Rccl {
    decltype(&ncclCommInitAll) commInitAll = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclGroupStart) groupStart = nullptr;
    decltype(&ncclGroupEnd) groupEnd = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGetErrorString) errorString = nullptr;
    std::string error;  // why loading failed
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        // librccl.so.1 first: in a process that already holds an RCCL (torch's),
        // the dynamic linker returns that one rather than loading a second
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen(RTOW_ROCM_LIB "/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            const char* e = dlerror();
            r.error = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
            return;
        }
        bool ok = true;
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn) {
                ok = false;
                r.error += std::string(r.error.empty() ? "" : ", ") + "no symbol " + name;
            }
        };
        sym(r.commInitAll, "ncclCommInitAll");
        sym(r.commDestroy, "ncclCommDestroy");
        sym(r.groupStart, "ncclGroupStart");
        sym(r.groupEnd, "ncclGroupEnd");
        sym(r.send, "ncclSend");
        sym(r.recv, "ncclRecv");
        sym(r.errorString, "ncclGetErrorString");
        if (!ok) r.commInitAll = nullptr;  // unusable
    });
    return r;
}

int hip_fail(hipError_t e, const char* what) {
    return set_error(RTOW_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

int nccl_fail(ncclResult_t r, const char* what) {
    const Rccl& R = rccl();
    return set_error(RTOW_E_RCCL, std::string(what) + ": ncclResult " + std::to_string((int)r) + " (" +
                                      (R.errorString ? R.errorString(r) : "?") + ")");
}

#define MHIP(expr)                                         \
    do {                                                   \
        hipError_t _e = (expr);                            \
        if (_e != hipSuccess) return hip_fail(_e, #expr);  \
    } while (0)
#define MNCCL(expr)                                           \
    do {                                                      \
        ncclResult_t _r = (expr);                             \
        if (_r != ncclSuccess) return nccl_fail(_r, #expr);   \
    } while (0)

void release(rtow_multi* m) {
    for (size_t i = 0; i < m->devices.size(); i++) {
        (void)hipSetDevice(m->devices[i]);
        if (i < m->streams.size() && m->streams[i]) (void)hipStreamSynchronize(m->streams[i]);
        if (i < m->slab_bgra.size() && m->slab_bgra[i]) (void)hipFree(m->slab_bgra[i]);
        if (i < m->slab_lin.size() && m->slab_lin[i]) (void)hipFree(m->slab_lin[i]);
        m->slab_bgra[i] = m->slab_lin[i] = nullptr;
    }
    if (!m->devices.empty()) {
        (void)hipSetDevice(m->devices[0]);
        for (void* p : {m->gather_bgra, m->gather_lin, m->frame_bgra, m->frame_lin})
            if (p) (void)hipFree(p);
    }
    m->gather_bgra = m->gather_lin = m->frame_bgra = m->frame_lin = nullptr;
    m->slab_px = m->frame_px = 0;
    for (ncclComm_t c : m->comms)
        if (c) (void)rccl().commDestroy(c);
    m->comms.clear();
    for (size_t i = 0; i < m->streams.size(); i++) {
        if (!m->streams[i]) continue;
        (void)hipSetDevice(m->devices[i]);
        (void)hipStreamDestroy(m->streams[i]);
    }
    m->streams.clear();
    for (rtow_context* c : m->ctx)
        if (c) rtow_context_destroy(c);
    m->ctx.clear();
}

// (re)size the slabs for a W x H frame split over the ranks
int ensure_buffers(rtow_multi* m, uint32_t W, uint32_t H) {
    const uint32_t n = (uint32_t)m->devices.size();
    const size_t need_px = (size_t)rtow_rank_tile_count(W, H, 0, n) * 64;  // rank 0 holds the most tiles
    const size_t frame_px = (size_t)W * H;
    if (need_px > m->slab_px) {
        for (uint32_t i = 0; i < n; i++) {
            MHIP(hipSetDevice(m->devices[i]));
            if (m->slab_bgra[i]) MHIP(hipFree(m->slab_bgra[i]));
            if (m->slab_lin[i]) MHIP(hipFree(m->slab_lin[i]));
            m->slab_bgra[i] = m->slab_lin[i] = nullptr;
            MHIP(hipMalloc(&m->slab_bgra[i], need_px * 4));
            MHIP(hipMalloc(&m->slab_lin[i], need_px * 12));
        }
        MHIP(hipSetDevice(m->devices[0]));
        if (m->gather_bgra) MHIP(hipFree(m->gather_bgra));
        if (m->gather_lin) MHIP(hipFree(m->gather_lin));
        m->gather_bgra = m->gather_lin = nullptr;
        MHIP(hipMalloc(&m->gather_bgra, need_px * n * 4));
        MHIP(hipMalloc(&m->gather_lin, need_px * n * 12));
        m->slab_px = need_px;
    }
    if (frame_px > m->frame_px) {
        MHIP(hipSetDevice(m->devices[0]));
        if (m->frame_bgra) MHIP(hipFree(m->frame_bgra));
        if (m->frame_lin) MHIP(hipFree(m->frame_lin));
        m->frame_bgra = m->frame_lin = nullptr;
        MHIP(hipMalloc(&m->frame_bgra, frame_px * 4));
        MHIP(hipMalloc(&m->frame_lin, frame_px * 12));
        m->frame_px = frame_px;
    }
    return RTOW_OK;
}

// One gather of every rank's slab (BGRA, and linear when asked) to the first
// device: rank i's slab (its tile count x 64 pixels) into slot i of the
// gathered buffer (slab_px pixels per slot).
int gather(rtow_multi* m, uint32_t W, uint32_t H, bool linear) {
    const uint32_t n = (uint32_t)m->devices.size();
    if (m->shared) {  // ranks sharing a device: device copies on the first device's stream
        MHIP(hipSetDevice(m->devices[0]));
        for (uint32_t i = 0; i < n; i++) {
            const size_t px = (size_t)rtow_rank_tile_count(W, H, i, n) * 64;
            MHIP(hipMemcpyPeerAsync((uint8_t*)m->gather_bgra + (size_t)i * m->slab_px * 4, m->devices[0],
                                    m->slab_bgra[i], m->devices[i], px * 4, m->streams[0]));
            if (linear)
                MHIP(hipMemcpyPeerAsync((float*)m->gather_lin + (size_t)i * m->slab_px * 3, m->devices[0],
                                        m->slab_lin[i], m->devices[i], px * 12, m->streams[0]));
        }
        MHIP(hipStreamSynchronize(m->streams[0]));
        return RTOW_OK;
    }
    const Rccl& R = rccl();
    MNCCL(R.groupStart());
    for (uint32_t i = 0; i < n; i++) {
        const size_t px = (size_t)rtow_rank_tile_count(W, H, i, n) * 64;
        ncclResult_t r = R.send(m->slab_bgra[i], px * 4, ncclUint8, 0, m->comms[i], m->streams[i]);
        if (r == ncclSuccess && linear) r = R.send(m->slab_lin[i], px * 3, ncclFloat32, 0, m->comms[i], m->streams[i]);
        if (r == ncclSuccess)
            r = R.recv((uint8_t*)m->gather_bgra + (size_t)i * m->slab_px * 4, px * 4, ncclUint8, (int)i, m->comms[0],
                       m->streams[0]);
        if (r == ncclSuccess && linear)
            r = R.recv((float*)m->gather_lin + (size_t)i * m->slab_px * 3, px * 3, ncclFloat32, (int)i, m->comms[0],
                       m->streams[0]);
        if (r != ncclSuccess) {
            (void)R.groupEnd();
            return nccl_fail(r, "ncclSend/ncclRecv (slab gather)");
        }
    }
    MNCCL(R.groupEnd());
    for (uint32_t i = 0; i < n; i++) {
        MHIP(hipSetDevice(m->devices[i]));
        MHIP(hipStreamSynchronize(m->streams[i]));
    }
    return RTOW_OK;
}

}  // namespace

extern "C" {

int rtow_multi_create(const int* devices, uint32_t n, rtow_multi** out) {
    if (!out) return set_error(RTOW_E_INVALID, "NULL out");
    *out = nullptr;
    if (!devices || n == 0) return set_error(RTOW_E_INVALID, "no devices");
    bool shared = false;
    for (uint32_t i = 0; i < n; i++) {
        if (devices[i] < 0) return set_error(RTOW_E_INVALID, "negative device index");
        for (uint32_t j = 0; j < i; j++) shared |= devices[j] == devices[i];
    }
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        return set_error(RTOW_E_NO_DEVICE, "no HIP device visible");
    for (uint32_t i = 0; i < n; i++)
        if (devices[i] >= count) return set_error(RTOW_E_INVALID, "device out of range");
    if (!shared && !rccl().commInitAll) return set_error(RTOW_E_RCCL, rccl().error);
    auto* m = new rtow_multi;
    m->devices.assign(devices, devices + n);
    m->shared = shared;
    m->ctx.assign(n, nullptr);
    m->slab_bgra.assign(n, nullptr);
    m->slab_lin.assign(n, nullptr);
    auto fail = [&](int rc) {
        release(m);
        delete m;
        return rc;
    };
    for (uint32_t i = 0; i < n; i++) {
        const int rc = rtow_context_create(devices[i], &m->ctx[i]);
        if (rc) return fail(rc);
    }
    m->streams.assign(n, nullptr);
    for (uint32_t i = 0; i < n; i++) {
        hipError_t e = hipSetDevice(devices[i]);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&m->streams[i], hipStreamNonBlocking);
        if (e != hipSuccess) return fail(hip_fail(e, "hipStreamCreateWithFlags"));
    }
    if (!shared) {
        m->comms.assign(n, nullptr);
        const ncclResult_t r = rccl().commInitAll(m->comms.data(), (int)n, devices);
        if (r != ncclSuccess) {
            m->comms.assign(n, nullptr);
            return fail(nccl_fail(r, "ncclCommInitAll"));
        }
    }
    *out = m;
    return RTOW_OK;
}

int rtow_multi_destroy(rtow_multi* m) {
    if (!m) return RTOW_OK;
    release(m);
    delete m;
    return RTOW_OK;
}

uint32_t rtow_multi_device_count(const rtow_multi* m) { return m ? (uint32_t)m->devices.size() : 0u; }

int rtow_multi_set_tree(rtow_multi* m, int tree) {
    if (!m) return set_error(RTOW_E_INVALID, "NULL argument");
    for (rtow_context* c : m->ctx) {
        const int rc = rtow_context_set_tree(c, tree);
        if (rc) return rc;
    }
    return RTOW_OK;
}

int rtow_multi_upload(rtow_multi* m, const rtow_scene* scene) {
    if (!m || !scene) return set_error(RTOW_E_INVALID, "NULL argument");
    for (rtow_context* c : m->ctx) {
        const int rc = rtow_scene_upload(c, scene);
        if (rc) return rc;
    }
    return RTOW_OK;
}

int rtow_multi_render(rtow_multi* m, const rtow_camera* cam, const rtow_params* p, uint8_t* bgra_out,
                      float* linear_out, rtow_stats* stats, rtow_stats* device_stats) {
    const auto t0 = std::chrono::steady_clock::now();
    if (!m || !cam || !p) return set_error(RTOW_E_INVALID, "NULL argument");
    if (p->width == 0 || p->height == 0 || p->spp == 0) return set_error(RTOW_E_INVALID, "bad params");
    const uint32_t n = (uint32_t)m->devices.size(), W = p->width, H = p->height;
    int rc = ensure_buffers(m, W, H);
    if (rc) return rc;
    const bool linear = linear_out != nullptr;
    // every rank renders its tiles at once (a render call returns when its
    // work is done, so one host thread per rank)
    std::vector<int> rcs(n, RTOW_OK);
    std::vector<std::string> errs(n);
    std::vector<rtow_stats> st(n);
    std::vector<std::thread> workers;
    for (uint32_t i = 0; i < n; i++) {
        workers.emplace_back([&, i] {
            rtow_params q = *p;
            q.rank = i;
            q.world = n;
            q.flags |= RTOW_FLAG_FRAME_PLAN;  // rtow_render's chunks: the same frame for any n
            rcs[i] = rtow_render_tiles_device(m->ctx[i], cam, &q, m->slab_bgra[i], linear ? m->slab_lin[i] : nullptr,
                                              m->streams[i], &st[i]);
            if (rcs[i]) errs[i] = rtow_last_error();  // the message is thread-local
        });
    }
    for (auto& w : workers) w.join();
    for (uint32_t i = 0; i < n; i++)
        if (rcs[i]) return set_error(rcs[i], "rank " + std::to_string(i) + " (device " + std::to_string(m->devices[i]) +
                                                 "): " + errs[i]);
    rc = gather(m, W, H, linear);
    if (rc) return rc;
    rc = rtow_assemble_device(m->ctx[0], W, H, n, m->gather_bgra, (uint32_t)m->slab_px, m->frame_bgra, m->streams[0]);
    if (rc) return rc;
    if (linear) {
        rc = rtow_assemble_linear_device(m->ctx[0], W, H, n, m->gather_lin, (uint32_t)m->slab_px, m->frame_lin,
                                         m->streams[0]);
        if (rc) return rc;
    }
    MHIP(hipSetDevice(m->devices[0]));
    if (bgra_out) MHIP(hipMemcpy(bgra_out, m->frame_bgra, (size_t)W * H * 4, hipMemcpyDeviceToHost));
    if (linear_out) MHIP(hipMemcpy(linear_out, m->frame_lin, (size_t)W * H * 12, hipMemcpyDeviceToHost));
    if (device_stats)
        for (uint32_t i = 0; i < n; i++) device_stats[i] = st[i];
    if (stats) {
        std::memset(stats, 0, sizeof *stats);
        for (const rtow_stats& s : st) {
            stats->segments += s.segments;
            stats->samples += s.samples;
            stats->pixels += s.pixels;
            stats->kernel_ms = std::max(stats->kernel_ms, s.kernel_ms);
            stats->resolve_ms = std::max(stats->resolve_ms, s.resolve_ms);
        }
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return RTOW_OK;
}

int rtow_render_devices(const int* devices, uint32_t n, const rtow_scene* scene, const rtow_camera* cam,
                        const rtow_params* p, uint8_t* bgra_out, float* linear_out, rtow_stats* stats) {
    if (!scene || !cam || !p) return set_error(RTOW_E_INVALID, "NULL argument");
    rtow_multi* m = nullptr;
    int rc = rtow_multi_create(devices, n, &m);
    if (rc) return rc;
    rc = rtow_multi_upload(m, scene);
    if (!rc) rc = rtow_multi_render(m, cam, p, bgra_out, linear_out, stats, nullptr);
    if (rc) {
        const std::string e = rtow_last_error();
        rtow_multi_destroy(m);
        return set_error(rc, e);
    }
    return rtow_multi_destroy(m);
}

}  // extern "C"
