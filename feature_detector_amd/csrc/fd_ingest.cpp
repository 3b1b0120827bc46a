// Ingest pipeline: pinned host slots, uploads on a copy stream of their own,
// detection + feature copy-back on the context stream, so consecutive slots overlap PCIe and compute.
// Built on the public C ABI (fd_points_detect with device frames and device outputs).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "fd_hip.h"

struct fd_ingest_slot {
    uint8_t *host_frames = nullptr;  // pinned
    uint8_t *dev_frames = nullptr;
    float *dev_xy = nullptr;
    int32_t *dev_counts = nullptr;
    float *host_xy = nullptr;  // pinned
    int32_t *host_counts = nullptr;
    uint32_t *host_status = nullptr;  // pinned: fd_ctx_frame_status of the slot's selection
    hipEvent_t uploaded = nullptr, done = nullptr;
    bool pending = false;
};

struct fd_ingest {
    fd_ctx *ctx = nullptr;
    int kind = 0, batch = 0, rows = 0, cols = 0;
    uint32_t need = 0;
    int32_t out_stride = 0;
    hipStream_t copy = nullptr;
    std::vector<fd_ingest_slot> slots;
};

namespace {

void release(fd_ingest *g) {
    for (fd_ingest_slot &s : g->slots) {
        if (s.host_frames) (void)hipHostFree(s.host_frames);
        if (s.host_xy) (void)hipHostFree(s.host_xy);
        if (s.host_counts) (void)hipHostFree(s.host_counts);
        if (s.host_status) (void)hipHostFree(s.host_status);
        if (s.dev_frames) (void)hipFree(s.dev_frames);
        if (s.dev_xy) (void)hipFree(s.dev_xy);
        if (s.dev_counts) (void)hipFree(s.dev_counts);
        if (s.uploaded) (void)hipEventDestroy(s.uploaded);
        if (s.done) (void)hipEventDestroy(s.done);
    }
    if (g->copy) (void)hipStreamDestroy(g->copy);
}

}  // namespace

extern "C" int fd_ingest_create(fd_ctx *ctx, int kind, int batch, int rows, int cols, int depth, uint32_t need,
                                int32_t out_stride, fd_ingest **out) {
    if (!ctx || !out || batch < 1 || rows < 1 || cols < 1 || depth < 1 || depth > 64 || out_stride < 1 ||
        kind < FD_HARRIS || kind > FD_FAST)
        return FD_ERR_INVALID;
    *out = nullptr;
    fd_ingest *g = new fd_ingest();
    g->ctx = ctx;
    g->kind = kind;
    g->batch = batch;
    g->rows = rows;
    g->cols = cols;
    g->need = need;
    g->out_stride = out_stride;
    g->slots.resize(depth);
    const size_t fbytes = static_cast<size_t>(batch) * rows * cols;
    const size_t xbytes = sizeof(float) * 2 * static_cast<size_t>(out_stride) * batch;
    const size_t cbytes = sizeof(int32_t) * batch;
    bool ok = hipStreamCreateWithFlags(&g->copy, hipStreamNonBlocking) == hipSuccess;
    for (fd_ingest_slot &s : g->slots) {
        ok = ok && hipHostMalloc(reinterpret_cast<void **>(&s.host_frames), fbytes, hipHostMallocDefault) == hipSuccess;
        ok = ok && hipHostMalloc(reinterpret_cast<void **>(&s.host_xy), xbytes, hipHostMallocDefault) == hipSuccess;
        ok = ok && hipHostMalloc(reinterpret_cast<void **>(&s.host_counts), cbytes, hipHostMallocDefault) == hipSuccess;
        ok = ok && hipHostMalloc(reinterpret_cast<void **>(&s.host_status), cbytes, hipHostMallocDefault) == hipSuccess;
        ok = ok && hipMalloc(reinterpret_cast<void **>(&s.dev_frames), fbytes) == hipSuccess;
        ok = ok && hipMalloc(reinterpret_cast<void **>(&s.dev_xy), xbytes) == hipSuccess;
        ok = ok && hipMalloc(reinterpret_cast<void **>(&s.dev_counts), cbytes) == hipSuccess;
        ok = ok && hipEventCreateWithFlags(&s.uploaded, hipEventDisableTiming) == hipSuccess;
        ok = ok && hipEventCreateWithFlags(&s.done, hipEventDisableTiming) == hipSuccess;
    }
    // workspace for this shape up front: submits then allocate nothing (they only enqueue)
    ok = ok && fd_ctx_reserve(ctx, kind, batch, rows, cols, 0) == FD_OK;
    if (!ok) {
        release(g);
        delete g;
        return FD_ERR_HIP;
    }
    *out = g;
    return FD_OK;
}

extern "C" void fd_ingest_destroy(fd_ingest *g) {
    if (!g) return;
    (void)hipStreamSynchronize(g->copy);
    (void)fd_ctx_synchronize(g->ctx);
    release(g);
    delete g;
}

extern "C" uint8_t *fd_ingest_frames(fd_ingest *g, int slot) {
    if (!g || slot < 0 || slot >= static_cast<int>(g->slots.size())) return nullptr;
    return g->slots[slot].host_frames;
}

extern "C" int fd_ingest_submit(fd_ingest *g, int slot, const fd_point_opts *opts) {
    if (!g || !opts || slot < 0 || slot >= static_cast<int>(g->slots.size())) return FD_ERR_INVALID;
    fd_ingest_slot &s = g->slots[slot];
    if (s.pending) return FD_ERR_INVALID;  // collect it (fd_ingest_wait) before reusing the slot
    const size_t fbytes = static_cast<size_t>(g->batch) * g->rows * g->cols;
    hipStream_t cs = static_cast<hipStream_t>(fd_ctx_get_stream(g->ctx));
    if (hipMemcpyAsync(s.dev_frames, s.host_frames, fbytes, hipMemcpyHostToDevice, g->copy) != hipSuccess ||
        hipEventRecord(s.uploaded, g->copy) != hipSuccess || hipStreamWaitEvent(cs, s.uploaded, 0) != hipSuccess)
        return FD_ERR_HIP;
    const int rc = fd_points_detect(g->ctx, g->kind, s.dev_frames, 1, g->batch, g->rows, g->cols, opts, nullptr, nullptr,
                                    g->need, s.dev_xy, g->out_stride, s.dev_counts, 1);
    if (rc != FD_OK) return rc;
    const size_t xbytes = sizeof(float) * 2 * static_cast<size_t>(g->out_stride) * g->batch;
    if (hipMemcpyAsync(s.host_xy, s.dev_xy, xbytes, hipMemcpyDeviceToHost, cs) != hipSuccess ||
        hipMemcpyAsync(s.host_counts, s.dev_counts, sizeof(int32_t) * g->batch, hipMemcpyDeviceToHost, cs) != hipSuccess ||
        fd_ctx_frame_status(g->ctx, s.host_status, g->batch, 1) != FD_OK || hipEventRecord(s.done, cs) != hipSuccess)
        return FD_ERR_HIP;
    s.pending = true;
    return FD_OK;
}

extern "C" int fd_ingest_wait(fd_ingest *g, int slot, const float **xy, const int32_t **counts) {
    if (!g || slot < 0 || slot >= static_cast<int>(g->slots.size())) return FD_ERR_INVALID;
    fd_ingest_slot &s = g->slots[slot];
    if (!s.pending) return FD_ERR_INVALID;
    if (hipEventSynchronize(s.done) != hipSuccess) return FD_ERR_HIP;
    s.pending = false;
    // the selection's consistency guards (the slot's status words), as fd_points_detect checks them
    // for host outputs; and the capacity check
    for (int b = 0; b < g->batch; ++b) {
        if (s.host_status[b] & FD_FRAME_GUARD) return FD_ERR_HIP;
        if (s.host_counts[b] > g->out_stride) return FD_ERR_CAPACITY;
    }
    if (xy) *xy = s.host_xy;
    if (counts) *counts = s.host_counts;
    return FD_OK;
}
