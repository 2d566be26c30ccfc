// sketch_host.cpp -- host -> device staging of pageable caller buffers.
//
// The redis-py facade hands the library numpy arrays: pageable host memory
// (SKE_MEM_HOST).  hipMemcpyAsync from pageable memory stages through the
// runtime's own pinned buffers one CPU copy at a time (≈ 32 GB/s measured for
// a C3 batch).  Here a batch larger than kDirectMax is cut into chunks; a pool
// of host threads copies each chunk into one of two pinned buffers while the
// DMA engine moves the previous chunk to the device, so the CPU copy and the
// host link overlap.  An offsets array is checked (never decreasing) by the
// same threads while they copy it -- the check that keeps every K1 id read in
// bounds.  Pinned caller buffers (hipHostMalloc / registered) and streams
// being captured go straight to hipMemcpyAsync.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "sketch_internal.h"

namespace ske {

namespace {

// A fixed set of worker threads; one job at a time, split in equal slices.
class CopyPool {
  public:
    explicit CopyPool(int n) {
        try {
            for (int i = 0; i < n; i++) th_.emplace_back([this, i] { work(i); });
        } catch (...) {  // the threads already started are stopped before rethrowing
            stop();
            throw;
        }
    }
    ~CopyPool() { stop(); }
    // copy n bytes (dst nullptr: none); with `mono`, also check the u32
    // array never decreases (returns false if it does)
    bool copy(void *dst, const void *src, size_t n, bool mono) {
        std::unique_lock<std::mutex> g(m_);
        dst_ = static_cast<char *>(dst);
        src_ = static_cast<const char *>(src);
        n_ = n;
        mono_ = mono;
        bad_.store(false);
        pending_ = int(th_.size());
        gen_++;
        cv_.notify_all();
        done_.wait(g, [this] { return pending_ == 0; });
        if (mono && dst) {  // the slice boundaries, on the finished copy
            const size_t per = slice_bytes(n);
            const uint32_t *u = reinterpret_cast<const uint32_t *>(dst);
            for (size_t a = per; a < n; a += per)
                if (u[a / 4] < u[a / 4 - 1]) bad_.store(true);
        }
        return !bad_.load();
    }

  private:
    // each thread's slice: 64-B aligned (whole u32 elements for the check)
    size_t slice_bytes(size_t n) const {
        const size_t T = th_.size();
        return ((n + T - 1) / T + 63) & ~size_t(63);
    }
    void stop() {
        {
            std::lock_guard<std::mutex> g(m_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
        th_.clear();
    }
    void work(int i) {
        uint64_t seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> g(m_);
            cv_.wait(g, [&] { return quit_ || gen_ != seen; });
            if (quit_) return;
            seen = gen_;
            char *dst = dst_;
            const char *src = src_;
            const size_t n = n_;
            const bool mono = mono_;
            g.unlock();
            const size_t per = slice_bytes(n);
            const size_t a = std::min(n, per * size_t(i)), b = std::min(n, a + per);
            if (b > a) {
                if (dst) memcpy(dst + a, src + a, b - a);
                if (mono) {
                    // the copy that the DMA will move is the one checked
                    // (fresh in this thread's cache), not the caller's buffer
                    const uint32_t *u = reinterpret_cast<const uint32_t *>(dst ? static_cast<const char *>(dst) : src);
                    uint32_t bad = 0;
                    // inside the slice; with a destination the slice
                    // boundaries are compared once every slice is copied
                    // (the neighbour's elements may not be there yet)
                    const size_t k0 = dst ? a / 4 + 1 : std::max<size_t>(a / 4, 1);
                    for (size_t k = k0; k < b / 4; k++) bad |= uint32_t(u[k] < u[k - 1]);
                    if (bad) bad_.store(true);
                }
            }
            g.lock();
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    char *dst_ = nullptr;
    const char *src_ = nullptr;
    size_t n_ = 0;
    bool mono_ = false;
    std::atomic<bool> bad_{false};
    int pending_ = 0;
    uint64_t gen_ = 0;
    bool quit_ = false;
};

constexpr size_t kDirectMax = size_t(8) << 20;  // below this, hipMemcpyAsync as is
constexpr size_t kChunk = size_t(32) << 20;     // bytes per pinned buffer
constexpr int kThreads = 8;

}  // namespace

struct HostStager {
    CopyPool *pool = nullptr;
    bool no_pool = false;  // the threads could not be started: plain hipMemcpyAsync
    void *pin[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool busy[2] = {false, false};
    int next = 0;
};

HostStager *stager_new() { return new HostStager(); }

void stager_delete(HostStager *s) {
    if (!s) return;
    for (int k = 0; k < 2; k++) {
        if (s->busy[k]) (void)hipEventSynchronize(s->ev[k]);
        if (s->ev[k]) (void)hipEventDestroy(s->ev[k]);
        if (s->pin[k]) (void)hipHostFree(s->pin[k]);
    }
    delete s->pool;
    delete s;
}

// the copy threads, started on first use (nullptr if they cannot be)
static CopyPool *get_pool(HostStager *s) {
    if (!s->pool && !s->no_pool) {
        try {
            s->pool = new CopyPool(kThreads);
        } catch (...) {
            s->no_pool = true;
        }
    }
    return s->pool;
}

// memory HIP knows (pinned host, device, managed): copied by the DMA engine
// as it is; false for pageable memory
static bool hip_known(const void *p) {
    hipPointerAttribute_t a{};
    const hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: not an error of ours
        return false;
    }
    return a.type == hipMemoryTypeHost || a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

static bool u32_monotone(const uint32_t *u, size_t n) {
    uint32_t bad = 0;
    for (size_t k = 1; k < n; k++) bad |= uint32_t(u[k] < u[k - 1]);
    return bad == 0;
}

// Host -> device copy of `bytes` on `st` (enqueued; the caller's buffer may
// be reused once the stream has passed this copy, and must not be modified
// before: a pinned caller buffer is read by the DMA engine directly, and its
// offsets are checked while the DMA runs).  mono: the source is a u32
// array that must never decrease -> *ok = false otherwise (the copy is still
// made; the caller must not launch a kernel on it).
hipError_t stage_h2d(HostStager *s, void *dst, const void *src, size_t bytes, hipStream_t st, bool mono,
                     bool *ok) {
    if (ok) *ok = true;
    if (bytes == 0) return hipSuccess;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    hipError_t e = hipStreamIsCapturing(st, &cs);
    if (e != hipSuccess) return e;
    if (bytes < kDirectMax || cs != hipStreamCaptureStatusNone || hip_known(src)) {
        e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
        if (e != hipSuccess || !mono || !ok) return e;
        // checked while the DMA runs: by the pool when large (device memory
        // is not readable here: a device offsets array stays unchecked, as on
        // the SKE_MEM_DEVICE path)
        hipPointerAttribute_t pa{};
        if (hipPointerGetAttributes(&pa, src) == hipSuccess && pa.type == hipMemoryTypeDevice) return e;
        (void)hipGetLastError();
        CopyPool *pool = bytes < kDirectMax ? nullptr : get_pool(s);
        *ok = pool ? pool->copy(nullptr, src, bytes, true)
                   : u32_monotone(static_cast<const uint32_t *>(src), bytes / 4);
        return e;
    }
    CopyPool *pool = get_pool(s);
    if (!pool) {  // no threads: the runtime's own pageable path
        e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
        if (e == hipSuccess && mono && ok) *ok = u32_monotone(static_cast<const uint32_t *>(src), bytes / 4);
        return e;
    }
    for (int k = 0; k < 2; k++) {
        if (!s->pin[k] && (e = hipHostMalloc(&s->pin[k], kChunk, hipHostMallocDefault)) != hipSuccess) return e;
        if (!s->ev[k] && (e = hipEventCreateWithFlags(&s->ev[k], hipEventDisableTiming)) != hipSuccess) return e;
    }
    const char *src8 = static_cast<const char *>(src);
    char *dst8 = static_cast<char *>(dst);
    bool good = true;
    uint32_t prev_last = 0;
    for (size_t off = 0; off < bytes; off += kChunk) {
        const size_t len = std::min(kChunk, bytes - off);
        const int k = s->next;
        s->next ^= 1;
        if (s->busy[k] && (e = hipEventSynchronize(s->ev[k])) != hipSuccess) return e;
        s->busy[k] = false;
        good &= pool->copy(s->pin[k], src8 + off, len, mono);
        const char *pk = static_cast<const char *>(s->pin[k]);
        if (mono && off) {  // the chunk boundary (chunks hold whole u32 elements)
            good &= *reinterpret_cast<const uint32_t *>(pk) >= prev_last;
        }
        if (mono) prev_last = *reinterpret_cast<const uint32_t *>(pk + len - 4);
        if ((e = hipMemcpyAsync(dst8 + off, s->pin[k], len, hipMemcpyHostToDevice, st)) != hipSuccess) return e;
        if ((e = hipEventRecord(s->ev[k], st)) != hipSuccess) return e;
        s->busy[k] = true;
    }
    if (ok) *ok = good;
    return hipSuccess;
}

}  // namespace ske
