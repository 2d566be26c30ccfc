// sketch_api.cpp -- libsketch C-ABI (include/sketch.h): context, Bloom chains,
// HLL register slab, host/device staging and the order-exact drivers.
//
// Host arithmetic here is the RedisBloom / Redis bookkeeping that is not
// data-parallel: link geometry (deps/bloom/bloom.c bloom_init + calc_bpe),
// chain growth (src/sb.c SBChain_Add), and the PFCOUNT estimator's
// m*tau(.) / m*sigma(.) tables (src/hyperloglog.c hllTau / hllSigma) built
// with the same libm calls as Redis.  Compiled with -ffp-contract=off.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/sketch.h"
#include "sketch_common.h"
#include "sketch_internal.h"

namespace ske {
Scratch *scratch_new();
void scratch_delete(Scratch *s);
hipError_t launch_bf_count_cands(uint64_t n, const uint8_t *state, unsigned long long *counter,
                                 int cus, hipStream_t st);
}  // namespace ske

using namespace ske;

// pass kinds of ske_pass_times: 0 a single-kernel K1 (LDS / global /
// XCD-partitioned), 1-3 the partitioned K1's passes A, B, C
constexpr int kPassKinds = SKE_PASS_KINDS;

namespace {

struct Link {
    uint8_t *bf = nullptr;  // device
    uint64_t entries = 0, bytes = 0, bits = 0, size = 0;
    double error = 0, bpe = 0;
    int hashes = 0;
    Divisor div{};
};

struct Filter {
    bool exists = false;
    bool dev_ok = false;  // `dev` matches `links`
    ChainDev dev{};       // cached kernel view of the chain (rebuilt on growth)
    std::vector<Link> links;
    uint64_t size = 0;
    uint32_t growth = 2;
    bool nonscaling = false;
};

struct Staged {
    const uint8_t *bytes = nullptr;
    const uint32_t *offs = nullptr;
};

}  // namespace

// The last use of a group of context scratch slots: a use on another stream
// first waits for it (scratch_user_begin below).
struct ScratchUse {
    hipEvent_t done = nullptr;
    hipStream_t stream = nullptr;
    unsigned long long cap = 0;  // capture id of stream's last scratch use (0: none)
    bool pending = false;        // that use is not yet covered by done (recorded lazily)
};

struct ske_ctx {
    int device = 0;
    int cus = 256;
    hipStream_t own = nullptr;
    hipStream_t st = nullptr;
    std::vector<Filter> filters;
    uint8_t *regs = nullptr;  // nslots * 16384
    uint32_t nslots = 0;
    double *tau = nullptr, *sig = nullptr;  // device estimator tables (lazy)
    Scratch *scratch = nullptr;
    // staging buffers (grow on demand)
    void *stg[9] = {};  // staging buffers by use (8: the device slot-range check word)
    size_t stg_cap[9] = {};
    HostStager *hs = nullptr;  // pinned double buffer + copy threads for pageable inputs (lazy)
    unsigned int *err = nullptr;  // [0] sticky slot-error word; see check_call_err
    bool err_pending = false;     // taken from the device, not yet reported by ske_sync
    unsigned long long *stats = nullptr;
    int pb = 2;           // K1 tile: swipes per thread in flight (1, 2, 4, 8)
    int variant = -1;     // -1 auto, 0 global, 1 LDS, 2 XCD-partitioned, 3 partitioned
    uint32_t part_sub = 0;  // partitioned K1: swipes per sub-batch (0: default)
    SegOpts seg;            // partitioned K1: the segmented PFADD's options
    bool lds_ok = false;
    bool k1_ok = false;       // short-id LDS K1 (sketch_k1.hip) usable
    int k1_grid = 0;          // blocks of the short-id LDS K1 (0: one per CU)
    int k1_persistent = 1;    // ske_swipes_many_async: one LDS K1 launch over all batches
    uint8_t *zero16 = nullptr;  // 16 zero bytes on the device
    // the XCD-partitioned K1 keeps per-launch state in the context scratch:
    // a launch on another stream first waits for the previous one
    ScratchUse xr;  // K1 (and every scratch user but routing)
    ScratchUse rt;  // routing (slot 40 / 41 only): ordered among routing calls, not behind K1
    // executable graphs alive (recorded, not yet freed): they hold pointers to
    // the scratch and the register slab, so neither may be reallocated
    void *hook_arg = nullptr;  // launch_swipes_part's pass hook state
    int live_graphs = 0;
    bool capturing = false;
    // scratch users recorded into the graph being captured (bit 0: xr,
    // bit 1: rt), and per live graph the users its replays hold: a replay
    // records only their events, so a graph without routing does not order
    // the next routing call behind itself
    unsigned cap_users = 0;
    std::unordered_map<void *, unsigned> graph_users;
    // pass timing (option "pass_timing"): HIP event pairs around every K1
    // kernel, recorded on the stream the kernel runs on (never inside a
    // capture); ske_pass_times() sums them per pass
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    struct Mark { int pass; hipEvent_t a, b; bool own_a; };
    std::vector<Mark> marks;
    double pass_ms[kPassKinds] = {};
    uint64_t pass_n[kPassKinds] = {};
    // ske_swipes_many_async: side streams of the fork/join branches (lazy)
    hipStream_t many_st[SKE_MANY_MAX_BRANCHES - 1] = {};
    hipEvent_t many_join[SKE_MANY_MAX_BRANCHES - 1] = {};
    hipEvent_t many_fork = nullptr;
    int many_n = 0;
    // host-fed chunk pipeline (ske_swipes_fixed_bits): a copy stream and one
    // event per chunk in flight (lazy)
    hipStream_t copy_st = nullptr;
    std::vector<hipEvent_t> chunk_ev;
    // ingest key table (open addressing on the 128-bit key hash)
    uint64_t *kt_key = nullptr;  // 2 per entry, kh0 == 0: empty
    uint32_t *kt_slot = nullptr;
    uint64_t kt_cap = 0, kt_count = 0;
    std::string last_hip;
};

#define HIPCHK(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess) {                                                                   \
            (ctx)->last_hip = std::string(#expr) + ": " + hipGetErrorString(_e);                  \
            return SKE_EHIP;                                                                      \
        }                                                                                         \
    } while (0)

namespace {

void *stage_buf(ske_ctx *c, int slot, size_t bytes, int *rc) {
    if (bytes < 64) bytes = 64;
    if (c->stg_cap[slot] < bytes) {
        if (c->stg[slot]) (void)hipFree(c->stg[slot]);
        c->stg[slot] = nullptr;
        c->stg_cap[slot] = 0;
        size_t want = bytes + bytes / 4 + 256;
        hipError_t e = hipMalloc(&c->stg[slot], want);
        if (e != hipSuccess) {
            c->last_hip = std::string("hipMalloc(staging): ") + hipGetErrorString(e);
            *rc = SKE_ENOMEM;
            return nullptr;
        }
        c->stg_cap[slot] = want;
    }
    return c->stg[slot];
}

// Items to device.  SKE_MEM_DEVICE pointers are used in place; host items are
// copied as the byte range [offs[0], offs[n]) plus offsets, and the device
// bytes pointer is rebased so that offs[] index it unchanged.
int stage_items(ske_ctx *c, const uint8_t *bytes, const uint32_t *offs, uint64_t n, int mem,
                Staged *out, int slot_bytes = 0, int slot_offs = 1) {
    if (mem == SKE_MEM_DEVICE) {
        out->bytes = bytes;
        out->offs = offs;
        return SKE_OK;
    }
    if (!offs || (!bytes && offs[n] != offs[0]) || offs[n] < offs[0]) return SKE_EINVAL;
    const uint64_t b0 = offs[0], total = uint64_t(offs[n]) - b0;
    int rc = SKE_OK;
    uint8_t *db = (uint8_t *)stage_buf(c, slot_bytes, total + 16, &rc);
    uint32_t *dof = (uint32_t *)stage_buf(c, slot_offs, (n + 1) * 4, &rc);
    if (rc) return rc;
    if (!c->hs) c->hs = stager_new();
    // the offsets are checked (never decreasing) as they are copied; no
    // kernel reads them before this returns
    // (bytes first: a direct offsets copy is checked while both DMAs run)
    bool ok = true;
    if (total) HIPCHK(c, stage_h2d(c->hs, db, bytes + b0, total, c->st, false, nullptr));
    HIPCHK(c, stage_h2d(c->hs, dof, offs, (n + 1) * 4, c->st, true, &ok));
    if (!ok) {
        HIPCHK(c, hipStreamSynchronize(c->st));  // the copies may still read the caller's buffers
        return SKE_EINVAL;
    }
    out->bytes = db - b0;
    out->offs = dof;
    return SKE_OK;
}

int stage_u32(ske_ctx *c, const uint32_t *p, uint64_t n, int mem, int slot, const uint32_t **out) {
    if (mem == SKE_MEM_DEVICE || n == 0) {
        *out = p;
        return SKE_OK;
    }
    int rc = SKE_OK;
    uint32_t *d = (uint32_t *)stage_buf(c, slot, n * 4, &rc);
    if (rc) return rc;
    if (!c->hs) c->hs = stager_new();
    HIPCHK(c, stage_h2d(c->hs, d, p, n * 4, c->st, false, nullptr));
    *out = d;
    return SKE_OK;
}

// ---- pass timing
hipEvent_t ev_get(ske_ctx *c) {
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// an event pair for one kernel of pass `pass` (nullptrs when not timing)
struct PassMark {
    hipEvent_t a = nullptr, b = nullptr;
    hipStream_t st = nullptr;  // the stream the kernel runs on
};
// `start`: an end event just recorded on st with nothing enqueued since (the
// previous kernel's), reused as this kernel's start: one marker packet fewer
PassMark mark_begin(ske_ctx *c, int pass, hipStream_t st, hipEvent_t start = nullptr) {
    PassMark m;
    if (!c->timing || c->capturing) return m;
    m.a = start ? start : ev_get(c);
    m.b = ev_get(c);
    m.st = st;
    if (!m.a || !m.b || (!start && hipEventRecord(m.a, st) != hipSuccess)) return PassMark();
    c->marks.push_back({pass, m.a, m.b, start == nullptr});
    return m;
}
PassMark mark_begin(ske_ctx *c, int pass) { return mark_begin(c, pass, c->st); }
void mark_end(ske_ctx *c, const PassMark &m) {
    if (m.b) (void)hipEventRecord(m.b, m.st);
}

// deps/bloom/bloom.c calc_bpe() + bloom_init() with BLOOM_OPT_NOROUND |
// BLOOM_OPT_FORCE64, the options rebloom.c's bfCreateChain() passes.
int link_geometry(uint64_t entries, double error, Link *L) {
    if (entries < 1 || !(error > 0) || error >= 1.0) return SKE_EINVAL;
    const double denom = 0.480453013918201;  // ln(2)^2
    double bpe = -(log(error) / denom);
    if (bpe < 0) bpe = -bpe;
    uint64_t bits = (uint64_t)((double)entries * bpe);
    if (bits == 0) bits = 1;
    uint64_t bytes = (bits % 64) ? ((bits / 64) + 1) * 8 : bits / 8;
    L->entries = entries;
    L->error = error;
    L->bpe = bpe;
    L->bytes = bytes;
    L->bits = bytes * 8;
    L->hashes = (int)ceil(0.693147180559945 * bpe);
    L->size = 0;
    if (L->bits >= (uint64_t(1) << 62)) return SKE_ENOMEM;
    L->div = make_divisor(L->bits);
    return SKE_OK;
}

int add_link(ske_ctx *c, Filter &F, uint64_t entries, double error) {
    if ((int)F.links.size() >= SKE_MAX_LINKS) return SKE_ENOMEM;
    Link L;
    int rc = link_geometry(entries, error, &L);
    if (rc) return rc;
    // pad to 16 bytes so 4-byte atomics and 16-byte staging never leave it
    hipError_t e = hipMalloc(&L.bf, (L.bytes + 15) & ~uint64_t(15));
    if (e != hipSuccess) {
        c->last_hip = std::string("hipMalloc(bloom link): ") + hipGetErrorString(e);
        return SKE_ENOMEM;
    }
    e = hipMemsetAsync(L.bf, 0, (L.bytes + 15) & ~uint64_t(15), c->st);
    if (e != hipSuccess) {
        (void)hipFree(L.bf);
        c->last_hip = std::string("hipMemset(bloom link): ") + hipGetErrorString(e);
        return SKE_EHIP;
    }
    F.links.push_back(L);
    F.dev_ok = false;
    return SKE_OK;
}

void free_filter(Filter &F) {
    for (auto &L : F.links)
        if (L.bf) (void)hipFree(L.bf);
    F = Filter();
}

ChainDev chain_dev(const Filter &F, size_t first = 0, size_t count = SIZE_MAX) {
    ChainDev ch{};
    ch.nlinks = 0;
    uint32_t lds = 0;
    const size_t end = std::min(F.links.size(), first + std::min(count, F.links.size()));
    for (size_t i = first; i < end; i++) {
        const Link &L = F.links[i];
        LinkDev &D = ch.link[ch.nlinks++];
        D.bf = L.bf;
        D.div = L.div;
        D.k = uint32_t(L.hashes);
        D.lds_off = lds;
        D.rmul = uint32_t((uint64_t(kRegions) << 32) / L.bits);
        const uint64_t padded = (L.bytes + 15) & ~uint64_t(15);
        lds = (lds + padded > 0xffffffffu) ? 0xffffffffu : uint32_t(lds + padded);
    }
    ch.lds_bytes = lds;
    return ch;
}

const ChainDev &cached_chain(Filter &F) {
    if (!F.dev_ok) {
        F.dev = chain_dev(F);
        F.dev_ok = true;
    }
    return F.dev;
}

LinkDev link_dev(const Link &L) {
    LinkDev D{};
    D.bf = L.bf;
    D.div = L.div;
    D.k = uint32_t(L.hashes);
    D.lds_off = 0;
    D.rmul = uint32_t((uint64_t(kRegions) << 32) / L.bits);
    return D;
}

bool use_lds(const ske_ctx *c, const ChainDev &ch) {
    if (!c->lds_ok || ch.nlinks == 0) return false;
    if (c->variant == 0 || c->variant == 2 || c->variant == 3) return false;
    return ch.lds_bytes <= lds_bloom_max();
}

// K1 variant for a chain: 1 LDS image (fits 152 KiB); for larger chains
// (>= 8 MB, or when asked for) 3 partitioned (probes routed to LDS-resident
// slices; sketch_part.hip) or 2 XCD-partitioned (L2-resident slices;
// sketch_xr.hip) when the chain's shape does not fit the partitioned
// kernel; else 0 global.
constexpr uint64_t kXrMinBytes = 8ull << 20;
int k1_variant(const ske_ctx *c, const ChainDev &ch) {
    if (ch.nlinks == 0) return 0;
    if (use_lds(c, ch)) return 1;
    if (c->variant == 0) return 0;
    uint64_t total = 0;
    for (int l = 0; l < ch.nlinks; l++) total += ch.link[l].div.d >> 3;
    const bool big = total >= kXrMinBytes || c->variant == 2 || c->variant == 3;
    if (!big) return 0;
    if (c->variant != 2 && part_supported(ch)) return 3;
    if (xr_supported(ch)) return 2;
    return 0;
}

// The XCD-partitioned and partitioned K1 keep per-launch state in the
// context scratch: a launch on another stream first waits for the previous
// one.  The wait only links launches of the same capture (or of none): an
// event recorded outside a capture cannot be waited on inside it, nor the
// reverse (the caller synchronises before recording a graph, as
// engine.capture does; ske_graph_launch records the event after a replay).
//
// A ScratchUse's done event is recorded lazily: only when a use on another stream needs it (or
// ske_set_stream leaves the stream), not after every call -- a marker packet
// per call costs ~6 us of GPU time between back-to-back steps.  Recording it
// later on its stream still covers the last use (it covers everything enqueued
// there so far).  A stream whose capture state changed since that use needs
// no wait: recording a graph starts from a synchronised stream.
static unsigned long long capture_id(hipStream_t st, hipError_t *e) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    unsigned long long cid = 0;
    *e = hipStreamGetCaptureInfo(st, &cs, &cid);
    return cs == hipStreamCaptureStatusActive ? cid : 0;
}

// cover u.stream's last scratch use by u.done (false: no wait is needed)
static int xr_flush(ske_ctx *c, ScratchUse &u, bool *covered) {
    *covered = false;
    if (!u.stream) return SKE_OK;
    if (!u.pending) {
        *covered = true;
        return SKE_OK;
    }
    hipError_t e = hipSuccess;
    const unsigned long long now = capture_id(u.stream, &e);
    HIPCHK(c, e);
    u.pending = false;
    if (now != u.cap) {
        u.stream = nullptr;
        return SKE_OK;
    }
    HIPCHK(c, hipEventRecord(u.done, u.stream));
    *covered = true;
    return SKE_OK;
}

static int scratch_user_begin(ske_ctx *c, unsigned long long *cid_out, ScratchUse &u) {
    if (!u.done) HIPCHK(c, hipEventCreateWithFlags(&u.done, hipEventDisableTiming));
    hipError_t e = hipSuccess;
    const unsigned long long cid = capture_id(c->st, &e);
    HIPCHK(c, e);
    if (u.stream && u.stream != c->st && u.cap == cid) {
        bool covered = false;
        const int rc = xr_flush(c, u, &covered);
        if (rc) return rc;
        if (covered) HIPCHK(c, hipStreamWaitEvent(c->st, u.done, 0));
    }
    *cid_out = cid;
    return SKE_OK;
}

static int scratch_user_end(ske_ctx *c, unsigned long long cid, ScratchUse &u) {
    if (cid) c->cap_users |= &u == &c->rt ? 2u : 1u;
    u.stream = c->st;
    u.cap = cid;
    u.pending = true;
    return SKE_OK;
}

int scratch_user_begin(ske_ctx *c, unsigned long long *cid_out) { return scratch_user_begin(c, cid_out, c->xr); }
int scratch_user_end(ske_ctx *c, unsigned long long cid) { return scratch_user_end(c, cid, c->xr); }

// scratch that cannot grow (a graph is being recorded, or alive) -> SKE_EBUSY
int scratch_error(ske_ctx *c, hipError_t e) {
    if (e == hipErrorStreamCaptureUnsupported) {
        c->last_hip = "scratch too small while a graph is recorded or alive: run the same call "
                      "(same or larger batch) once before recording, or free the graphs";
        return SKE_EBUSY;
    }
    c->last_hip = hipGetErrorString(e);
    return SKE_ENOMEM;
}

Filter *get_filter(ske_ctx *c, uint32_t fid) {
    if (fid >= c->filters.size()) return nullptr;
    return &c->filters[fid];
}

// hllTau / hllSigma exactly as Redis src/hyperloglog.c (glibc sqrt, pow).
double redis_sigma(double x) {
    if (x == 1.) return INFINITY;
    double zPrime, y = 1, z = x;
    do {
        x *= x;
        zPrime = z;
        z += x * y;
        y += y;
    } while (zPrime != z);
    return z;
}
double redis_tau(double x) {
    if (x == 0. || x == 1.) return 0.;
    double zPrime, y = 1.0, z = 1 - x;
    do {
        x = sqrt(x);
        zPrime = z;
        y *= 0.5;
        z -= pow(1 - x, 2) * y;
    } while (zPrime != z);
    return z / 3;
}

int ensure_tables(ske_ctx *c) {
    if (c->tau) return SKE_OK;
    const int M = SKE_HLL_REGISTERS;
    std::vector<double> tau(M + 1), sig(M + 1);
    const double m = M;
    for (int j = 0; j <= M; j++) {
        tau[j] = m * redis_tau((m - j) / (double)m);  // z = m * hllTau((m-H[Q+1])/m)
        sig[j] = m * redis_sigma(j / (double)m);      // z += m * hllSigma(H[0]/m)
    }
    HIPCHK(c, hipMalloc(&c->tau, (M + 1) * sizeof(double)));
    HIPCHK(c, hipMalloc(&c->sig, (M + 1) * sizeof(double)));
    HIPCHK(c, hipMemcpy(c->tau, tau.data(), (M + 1) * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->sig, sig.data(), (M + 1) * sizeof(double), hipMemcpyHostToDevice));
    return SKE_OK;
}

// The device error word err[0] is sticky: kernels only ever set it (a valid
// swipe naming a slot outside the slab).  It is read and cleared only by
// device-side exchanges (atomicExch), so a flag set by a kernel on any stream
// is never lost between a read and a clear:
//   * a synchronous call (K1, PFADD, ingest) first takes what earlier
//     enqueue-only calls left into err[kErrPrior] (k_err_begin, OR-ed), and at
//     its end takes its own flag into the report word (k_err_end); the prior
//     flag is then held on the host (c->err_pending) for the next ske_sync /
//     ske_check_errors -- a synchronous call reports only its own slots;
//   * ske_sync / ske_check_errors report everything not yet reported.
constexpr int kErrPrior = 16, kErrOut = 32;  // word offsets in c->err (64 words)

__global__ void k_err_begin(unsigned int *err) {
    const unsigned int v = atomicExch(err, 0u);
    if (v) atomicOr(err + kErrPrior, v);
}
// out[0] = the prior word (then cleared), out[1] = the live word (then cleared)
__global__ void k_err_end(unsigned int *err) {
    err[kErrOut] = atomicExch(err + kErrPrior, 0u);
    err[kErrOut + 1] = atomicExch(err, 0u);
}

int err_begin(ske_ctx *c) {
    hipLaunchKernelGGL(k_err_begin, dim3(1), dim3(1), 0, c->st, c->err);
    HIPCHK(c, hipGetLastError());
    return SKE_OK;
}

// the two words after this call's work: {earlier enqueue-only calls, this call}
int err_end(ske_ctx *c, unsigned int h[2]) {
    hipLaunchKernelGGL(k_err_end, dim3(1), dim3(1), 0, c->st, c->err);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(h, c->err + kErrOut, 8, hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

// end of a synchronous call that did err_begin(): its own slot errors only
int check_call_err(ske_ctx *c) {
    unsigned int h[2] = {0, 0};
    const int rc = err_end(c, h);
    if (rc) return rc;
    if (h[0]) c->err_pending = true;
    return h[1] ? SKE_ERANGE : SKE_OK;
}

// ske_sync / ske_check_errors: everything not yet reported
int check_err_flag(ske_ctx *c, int code_if_set) {
    unsigned int h[2] = {0, 0};
    const int rc = err_end(c, h);
    if (rc) return rc;
    const bool set = h[0] || h[1] || c->err_pending;
    c->err_pending = false;
    return set ? code_if_set : SKE_OK;
}

// The short-id LDS kernel (sketch_k1.hip) when the chain, the batch and the
// options allow it; false: use the generic kernels.
bool k1_fast_args(ske_ctx *c, const ChainDev &ch, const uint8_t *bytes, const uint32_t *offs,
                  uint32_t fixed_w, const uint32_t *slot, uint64_t n, uint8_t *out, K1Args *A) {
    if (!c->k1_ok || !use_lds(c, ch)) return false;
    if (n >= (uint64_t(1) << 31)) return false;
    if (!offs && uint64_t(fixed_w) * n >= (uint64_t(1) << 32)) return false;
    if (!k1_lds_plan(ch, A)) return false;
    A->bytes = bytes;
    A->offs = offs;
    A->slot = slot;
    A->regs = c->regs;
    A->out = out;
    A->err = c->err;
    A->zero16 = c->zero16;
    A->n = uint32_t(n);
    A->nslots = c->nslots;
    A->fixed_w = fixed_w;
    return true;
}

// The partitioned K1 over nb batches, every pass on the context stream.
int launch_part(ske_ctx *c, const ChainDev &ch, const PartBatch *bt, uint32_t nb) {
    uint64_t nmax = 0;
    for (uint32_t j = 0; j < nb; j++) nmax = bt[j].n > nmax ? bt[j].n : nmax;
    if (nmax == 0) return SKE_OK;
    hipError_t e = part_reserve(ch, nmax, c->part_sub, c->nslots, c->seg, c->scratch);
    if (e != hipSuccess) return scratch_error(c, e);
    unsigned long long cid = 0;
    int rc = scratch_user_begin(c, &cid);
    if (rc) return rc;
    // one event pair per kernel and unit, bracketed on the kernel's stream;
    // back-to-back kernels on one stream share the event between them
    struct Hook {
        PassMark pm[5];
        PassMark last;  // the mark whose end event was recorded last, if nothing came after it
    } hs;
    auto hook = [](void *u, int pass, int end, hipStream_t st) {
        ske_ctx *cc = static_cast<ske_ctx *>(u);
        Hook *h = reinterpret_cast<Hook *>(cc->hook_arg);
        if (end) {
            mark_end(cc, h->pm[pass]);
            h->last = h->pm[pass];
        } else {
            const bool share = h->last.b && h->last.st == st;
            h->pm[pass] = mark_begin(cc, 1 + pass, st, share ? h->last.b : nullptr);
            h->last = PassMark();
        }
    };
    c->hook_arg = &hs;
    e = launch_swipes_part(ch, bt, nb, c->regs, c->nslots, c->scratch, c->err, c->cus, c->part_sub, c->seg, c->st,
                           c->timing && !c->capturing ? +hook : nullptr, c);
    if (e != hipSuccess) {
        c->last_hip = std::string("launch_swipes_part: ") + hipGetErrorString(e);
        scratch_user_end(c, cid);
        return SKE_EHIP;
    }
    return scratch_user_end(c, cid);
}

// Enqueue K1 (mode swipes) with the variant the chain selects.
int launch_k1(ske_ctx *c, const ChainDev &ch, const uint8_t *bytes, const uint32_t *offs,
              uint32_t fixed_w, const uint32_t *slot, uint64_t n, uint8_t *out) {
    if (n == 0) return SKE_OK;
    K1Args A;
    if (k1_fast_args(c, ch, bytes, offs, fixed_w, slot, n, out, &A)) {
        const PassMark m = mark_begin(c, 0);
        HIPCHK(c, launch_swipes_lds(A, true, c->pb, c->k1_grid ? c->k1_grid : c->cus, c->st));
        mark_end(c, m);
        return SKE_OK;
    }
    const int var = k1_variant(c, ch);
    if (var == 3) {
        const PartBatch pb{bytes, offs, fixed_w, slot, n, out};
        return launch_part(c, ch, &pb, 1);
    }
    if (var == 2) {
        hipError_t e = hipSuccess;
        void *scr = scratch_get(c->scratch, 16, xr_scratch_bytes(n, ch.nlinks), &e);
        if (e != hipSuccess) return scratch_error(c, e);
        unsigned long long cid = 0;
        int rc = scratch_user_begin(c, &cid);
        if (rc) return rc;
        const PassMark m = mark_begin(c, 0);
        HIPCHK(c, launch_swipes_xr(ch, bytes, offs, fixed_w, slot, n, c->regs, c->nslots, out,
                                   scr, c->err, c->cus, 2, 1, c->st));
        mark_end(c, m);
        return scratch_user_end(c, cid);
    }
    const PassMark m = mark_begin(c, 0);
    HIPCHK(c, launch_swipes(0, ch, use_lds(c, ch), c->pb, bytes, offs, fixed_w, slot, n, c->regs,
                            c->nslots, out, (unsigned long long *)c->err, c->cus, c->st));
    mark_end(c, m);
    return SKE_OK;
}

}  // namespace

extern "C" {

const char *ske_strerror(int code) {
    switch (code) {
    case SKE_OK: return "OK";
    case SKE_EINVAL: return "ERR invalid argument";
    case SKE_ENOMEM: return "ERR out of device memory";
    case SKE_EHIP: return "ERR HIP runtime error";
    case SKE_ENOFILTER: return "ERR not found";
    case SKE_EEXISTS: return "ERR item exists";
    case SKE_EFULL: return "ERR non scaling filter is full";
    case SKE_ERANGE: return "ERR HLL slot out of range";
    case SKE_EBADRATE: return "ERR (0 < error rate range < 1)";
    case SKE_EBADCAP: return "ERR (capacity should be larger than 0)";
    case SKE_EBADEXP: return "ERR expansion should be greater or equal to 1";
    case SKE_EBADHLL: return "INVALIDOBJ Corrupted HLL object detected";
    case SKE_ETOOLONG: return "ERR item too long";
    case SKE_EBUSY: return "ERR device buffers in use by a recorded graph";
    default: return "ERR unknown";
    }
}

const char *ske_last_hip_error(ske_ctx *c) { return c ? c->last_hip.c_str() : ""; }

int ske_open(int device, ske_ctx **out) {
    if (!out) return SKE_EINVAL;
    *out = nullptr;
    ske_ctx *c = new ske_ctx();
    c->device = device;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        delete c;
        return SKE_EHIP;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        c->cus = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return SKE_EHIP;
    }
    c->st = c->own;
    c->filters.resize(SKE_MAX_FILTERS);
    c->scratch = scratch_new();
    if (hipMalloc(&c->err, 256) != hipSuccess || hipMalloc(&c->stats, 64) != hipSuccess ||
        hipMemset(c->err, 0, 256) != hipSuccess) {
        ske_close(c);
        return SKE_ENOMEM;
    }
    c->lds_ok = lds_bloom_setup() == hipSuccess;
    c->k1_ok = c->lds_ok && k1_lds_setup() == hipSuccess;
    if (hipMalloc(&c->zero16, 64) != hipSuccess || hipMemset(c->zero16, 0, 64) != hipSuccess) {
        ske_close(c);
        return SKE_ENOMEM;
    }
    *out = c;
    return SKE_OK;
}

int ske_close(ske_ctx *c) {
    if (!c) return SKE_EINVAL;
    (void)hipSetDevice(c->device);
    if (c->st) (void)hipStreamSynchronize(c->st);
    for (auto &F : c->filters) free_filter(F);
    if (c->regs) (void)hipFree(c->regs);
    if (c->tau) (void)hipFree(c->tau);
    if (c->sig) (void)hipFree(c->sig);
    for (int i = 0; i < 9; i++)
        if (c->stg[i]) (void)hipFree(c->stg[i]);
    stager_delete(c->hs);
    if (c->err) (void)hipFree(c->err);
    if (c->zero16) (void)hipFree(c->zero16);
    if (c->xr.done) (void)hipEventDestroy(c->xr.done);
    if (c->rt.done) (void)hipEventDestroy(c->rt.done);
    for (auto &m : c->marks) {
        (void)hipEventDestroy(m.a);
        (void)hipEventDestroy(m.b);
    }
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    for (int i = 0; i < c->many_n; i++) {
        (void)hipStreamDestroy(c->many_st[i]);
        (void)hipEventDestroy(c->many_join[i]);
    }
    if (c->many_fork) (void)hipEventDestroy(c->many_fork);
    for (hipEvent_t e : c->chunk_ev) (void)hipEventDestroy(e);
    if (c->copy_st) (void)hipStreamDestroy(c->copy_st);
    if (c->kt_key) (void)hipFree(c->kt_key);
    if (c->kt_slot) (void)hipFree(c->kt_slot);
    if (c->stats) (void)hipFree(c->stats);
    if (c->scratch) scratch_delete(c->scratch);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
    return SKE_OK;
}

int ske_set_stream(ske_ctx *c, void *stream) {
    if (!c) return SKE_EINVAL;
    hipStream_t next = stream ? (hipStream_t)stream : c->own;
    // leaving the stream of the last scratch use: cover it now, while the
    // stream is known to be alive
    for (ScratchUse *u : {&c->xr, &c->rt})
        if (next != c->st && u->pending && u->stream == c->st) {
            bool covered = false;
            const int rc = xr_flush(c, *u, &covered);
            if (rc) return rc;
        }
    c->st = next;
    return SKE_OK;
}

int ske_get_stream(ske_ctx *c, void **stream) {
    if (!c || !stream) return SKE_EINVAL;
    *stream = c->st == c->own ? nullptr : (void *)c->st;
    return SKE_OK;
}

int ske_sync(ske_ctx *c) {
    if (!c) return SKE_EINVAL;
    HIPCHK(c, hipStreamSynchronize(c->st));
    return check_err_flag(c, SKE_ERANGE);
}

int ske_check_errors(ske_ctx *c) {
    if (!c) return SKE_EINVAL;
    return check_err_flag(c, SKE_ERANGE);
}

int ske_pass_times(ske_ctx *c, double *ms, uint64_t *count, int reset) {
    if (!c || !ms || !count) return SKE_EINVAL;
    if (!c->marks.empty()) {
        for (auto &m : c->marks) HIPCHK(c, hipEventSynchronize(m.b));
        for (auto &m : c->marks) {
            float t = 0;
            HIPCHK(c, hipEventElapsedTime(&t, m.a, m.b));
            c->pass_ms[m.pass] += t;
            c->pass_n[m.pass]++;
            if (m.own_a) c->ev_pool.push_back(m.a);
            c->ev_pool.push_back(m.b);
        }
        c->marks.clear();
    }
    for (int i = 0; i < kPassKinds; i++) {
        ms[i] = c->pass_ms[i];
        count[i] = c->pass_n[i];
        if (reset) {
            c->pass_ms[i] = 0;
            c->pass_n[i] = 0;
        }
    }
    return SKE_OK;
}

int ske_device_alloc(ske_ctx *c, uint64_t bytes, void **out) {
    if (!c || !out) return SKE_EINVAL;
    hipError_t e = hipMalloc(out, bytes ? bytes : 16);
    if (e != hipSuccess) {
        c->last_hip = std::string("hipMalloc: ") + hipGetErrorString(e);
        return SKE_ENOMEM;
    }
    return SKE_OK;
}

int ske_device_free(ske_ctx *c, void *p) {
    if (!c) return SKE_EINVAL;
    HIPCHK(c, hipFree(p));
    return SKE_OK;
}

int ske_memcpy(ske_ctx *c, void *dst, const void *src, uint64_t bytes, int kind) {
    if (!c) return SKE_EINVAL;
    if (!bytes) return SKE_OK;
    hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice
                      : kind == 1 ? hipMemcpyDeviceToHost
                                  : hipMemcpyDeviceToDevice;
    HIPCHK(c, hipMemcpyAsync(dst, src, bytes, k, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

int ske_set_option(ske_ctx *c, const char *name, int64_t value) {
    if (!c || !name) return SKE_EINVAL;
    if (!strcmp(name, "tile")) {
        if (value != 1 && value != 2 && value != 4 && value != 8) return SKE_EINVAL;
        c->pb = int(value);
        return SKE_OK;
    }
    if (!strcmp(name, "pass_timing")) {  // 1: bracket every K1 kernel with HIP events
        if (value < 0 || value > 1) return SKE_EINVAL;
        c->timing = value != 0;
        return SKE_OK;
    }
    if (!strcmp(name, "part_sub")) {  // partitioned K1 sub-batch (swipes; 0 = default)
        if (value < 0 || value > (int64_t(1) << 26)) return SKE_EINVAL;
        c->part_sub = uint32_t(value);
        return SKE_OK;
    }
    if (!strcmp(name, "hll_seg")) {  // segmented PFADD: -1 auto, 0 never, 1 when the chain and slab allow
        if (value < -1 || value > 1) return SKE_EINVAL;
        c->seg.mode = int(value);
        return SKE_OK;
    }
    if (!strcmp(name, "seg_density")) {  // auto threshold: swipes per slab line x100
        if (value < 0 || value > 1000000) return SKE_EINVAL;
        c->seg.density_x100 = uint32_t(value);
        return SKE_OK;
    }
    if (!strcmp(name, "seg_dense_min")) {  // records per window line x100 to stage a window in LDS
        if (value < 0 || value > 1000000) return SKE_EINVAL;
        c->seg.dense_min_x100 = uint32_t(value);
        return SKE_OK;
    }
    if (!strcmp(name, "seg_klog")) {  // keys per window 2^klog
        if (value < 0 || value > 3) return SKE_EINVAL;
        c->seg.klog = int(value);
        return SKE_OK;
    }
    if (!strcmp(name, "seg_b1")) {  // segmented PFADD: 2^b1 level-1 buckets, -1 auto
        if (value < -1 || value > 9) return SKE_EINVAL;
        c->seg.b1 = int(value);
        return SKE_OK;
    }
    if (!strcmp(name, "rec_groups")) {  // pass A's records in the group layout: -1 auto, 0 per-tile runs, 1 on
        if (value < -1 || value > 1) return SKE_EINVAL;
        c->seg.rec_groups = int(value);
        return SKE_OK;
    }
    if (!strcmp(name, "k1_grid")) {
        if (value < 0 || value > 65535) return SKE_EINVAL;
        c->k1_grid = int(value);
        return SKE_OK;
    }
    if (!strcmp(name, "k1_persistent")) {  // 0: many-batch calls launch K1 per batch
        if (value < 0 || value > 1) return SKE_EINVAL;
        c->k1_persistent = int(value);
        return SKE_OK;
    }
    if (!strcmp(name, "variant")) {
        if (value < -1 || value > 3) return SKE_EINVAL;
        c->variant = int(value);
        return SKE_OK;
    }
    return SKE_EINVAL;
}

// ------------------------------------------------------------------ Bloom
int ske_bf_reserve(ske_ctx *c, uint32_t fid, double error_rate, uint64_t capacity,
                   uint32_t expansion, int nonscaling) {
    if (!c) return SKE_EINVAL;
    Filter *F = get_filter(c, fid);
    if (!F) return SKE_EINVAL;
    if (!(error_rate > 0) || error_rate >= 1) return SKE_EBADRATE;
    if (capacity == 0) return SKE_EBADCAP;
    if (expansion < 1 && !nonscaling) return SKE_EBADEXP;
    if (F->exists) return SKE_EEXISTS;
    Filter nf;
    nf.growth = expansion;
    nf.nonscaling = nonscaling != 0;
    // SB_NewChain(): first link error * ERROR_TIGHTENING_RATIO unless NONSCALING
    const double tightening = nf.nonscaling ? 1.0 : 0.5;
    int rc = add_link(c, nf, capacity, error_rate * tightening);
    if (rc) {
        free_filter(nf);
        return rc;
    }
    nf.exists = true;
    *F = nf;
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

int ske_bf_exists_key(ske_ctx *c, uint32_t fid) {
    Filter *F = c ? get_filter(c, fid) : nullptr;
    return (F && F->exists) ? 1 : 0;
}

int ske_bf_free(ske_ctx *c, uint32_t fid) {
    Filter *F = c ? get_filter(c, fid) : nullptr;
    if (!F) return SKE_EINVAL;
    (void)hipStreamSynchronize(c->st);
    free_filter(*F);
    return SKE_OK;
}

int ske_bf_info(ske_ctx *c, uint32_t fid, ske_bf_info_t *out) {
    Filter *F = c ? get_filter(c, fid) : nullptr;
    if (!F || !out) return SKE_EINVAL;
    if (!F->exists) return SKE_ENOFILTER;
    memset(out, 0, sizeof(*out));
    // SBChain_MemUsage(): sizeof(SBChain) + nfilters*sizeof(SBLink) + bytes
    uint64_t mem = 32 + 64 * F->links.size();
    for (auto &L : F->links) {
        out->capacity += L.entries;
        mem += L.bytes;
    }
    out->size_bytes = mem;
    out->nfilters = uint32_t(F->links.size());
    out->expansion = F->growth;
    out->inserted = F->size;
    out->nonscaling = F->nonscaling;
    return SKE_OK;
}

int ske_bf_link_info(ske_ctx *c, uint32_t fid, uint32_t link, ske_bf_link_t *out) {
    Filter *F = c ? get_filter(c, fid) : nullptr;
    if (!F || !out) return SKE_EINVAL;
    if (!F->exists) return SKE_ENOFILTER;
    if (link >= F->links.size()) return SKE_EINVAL;
    const Link &L = F->links[link];
    memset(out, 0, sizeof(*out));
    out->entries = L.entries;
    out->bytes = L.bytes;
    out->bits = L.bits;
    out->size = L.size;
    out->error = L.error;
    out->bpe = L.bpe;
    out->hashes = L.hashes;
    return SKE_OK;
}

int ske_bf_export_link(ske_ctx *c, uint32_t fid, uint32_t link, uint8_t *out, uint64_t cap) {
    Filter *F = c ? get_filter(c, fid) : nullptr;
    if (!F || !out) return SKE_EINVAL;
    if (!F->exists) return SKE_ENOFILTER;
    if (link >= F->links.size()) return SKE_EINVAL;
    const Link &L = F->links[link];
    if (cap < L.bytes) return SKE_EINVAL;
    HIPCHK(c, hipMemcpyAsync(out, L.bf, L.bytes, hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

int ske_bf_import_link(ske_ctx *c, uint32_t fid, uint32_t link, const uint8_t *in,
                       uint64_t nbytes) {
    Filter *F = c ? get_filter(c, fid) : nullptr;
    if (!F || !in) return SKE_EINVAL;
    if (!F->exists) return SKE_ENOFILTER;
    if (link >= F->links.size() || nbytes != F->links[link].bytes) return SKE_EINVAL;
    HIPCHK(c, hipMemcpyAsync(F->links[link].bf, in, nbytes, hipMemcpyHostToDevice, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

int ske_bf_link_write(ske_ctx *c, uint32_t fid, uint32_t link, uint64_t offset, const uint8_t *in,
                      uint64_t nbytes) {
    Filter *F = c ? get_filter(c, fid) : nullptr;
    if (!F || (!in && nbytes)) return SKE_EINVAL;
    if (!F->exists) return SKE_ENOFILTER;
    if (link >= F->links.size()) return SKE_EINVAL;
    const Link &L = F->links[link];
    if (offset > L.bytes || nbytes > L.bytes - offset) return SKE_EINVAL;
    if (nbytes) {
        HIPCHK(c, hipMemcpyAsync(L.bf + offset, in, nbytes, hipMemcpyHostToDevice, c->st));
        HIPCHK(c, hipStreamSynchronize(c->st));
    }
    return SKE_OK;
}

int ske_bf_load_header(ske_ctx *c, uint32_t fid, const ske_bf_link_t *links, uint32_t nlinks,
                       uint64_t inserted, uint32_t expansion, int nonscaling) {
    Filter *F = c ? get_filter(c, fid) : nullptr;
    if (!F || (!links && nlinks)) return SKE_EINVAL;
    if (F->exists) return SKE_EEXISTS;
    if (nlinks == 0 || nlinks > SKE_MAX_LINKS) return SKE_EINVAL;
    Filter nf;
    nf.growth = expansion;
    nf.nonscaling = nonscaling != 0;
    for (uint32_t i = 0; i < nlinks; i++) {
        const ske_bf_link_t &H = links[i];
        if (H.bytes == 0 || H.bits != H.bytes * 8 || H.bits >= (uint64_t(1) << 62) || H.hashes < 1 ||
            H.hashes > 64) {
            free_filter(nf);
            return SKE_EINVAL;
        }
        Link L;
        L.entries = H.entries;
        L.bytes = H.bytes;
        L.bits = H.bits;
        L.size = H.size;
        L.error = H.error;
        L.bpe = H.bpe;
        L.hashes = H.hashes;
        L.div = make_divisor(L.bits);
        hipError_t e = hipMalloc(&L.bf, (L.bytes + 15) & ~uint64_t(15));
        if (e == hipSuccess) e = hipMemsetAsync(L.bf, 0, (L.bytes + 15) & ~uint64_t(15), c->st);
        if (e != hipSuccess) {
            if (L.bf) (void)hipFree(L.bf);
            free_filter(nf);
            c->last_hip = std::string("load header: ") + hipGetErrorString(e);
            return SKE_ENOMEM;
        }
        nf.links.push_back(L);
    }
    nf.size = inserted;
    nf.exists = true;
    *F = nf;
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

int ske_bf_mexists(ske_ctx *c, uint32_t fid, const uint8_t *bytes, const uint32_t *offs,
                   uint64_t n, uint8_t *out, int mem) {
    if (!c || !out) return SKE_EINVAL;
    Filter *F = get_filter(c, fid);
    if (!F) return SKE_EINVAL;
    if (n == 0) return SKE_OK;
    if (!F->exists) {  // BFCheck on a missing key answers 0
        if (mem == SKE_MEM_DEVICE) {
            HIPCHK(c, hipMemsetAsync(out, 0, n, c->st));
            HIPCHK(c, hipStreamSynchronize(c->st));
        } else {
            memset(out, 0, n);
        }
        return SKE_OK;
    }
    Staged s;
    int rc = stage_items(c, bytes, offs, n, mem, &s);
    if (rc) return rc;
    uint8_t *dout = out;
    if (mem != SKE_MEM_DEVICE) {
        dout = (uint8_t *)stage_buf(c, 3, n, &rc);
        if (rc) return rc;
    }
    const ChainDev ch = chain_dev(*F);
    K1Args A;
    if (k1_fast_args(c, ch, s.bytes, s.offs, 0, nullptr, n, dout, &A))
        HIPCHK(c, launch_swipes_lds(A, false, c->pb, c->cus, c->st));
    else
        HIPCHK(c, launch_swipes(1, ch, use_lds(c, ch), c->pb, s.bytes, s.offs, 0, nullptr, n, nullptr,
                                0, dout, nullptr, c->cus, c->st));
    if (mem != SKE_MEM_DEVICE) HIPCHK(c, hipMemcpyAsync(out, dout, n, hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

// BF.MADD with SBChain_Add's sequential semantics, in epochs: an epoch fills
// the current link up to its remaining capacity with the candidates in
// order ("first setter" per bit decides who is still absent when its turn
// comes), then the chain grows and the rest continue in the new link.
int ske_bf_madd(ske_ctx *c, uint32_t fid, const uint8_t *bytes, const uint32_t *offs, uint64_t n,
                int8_t *out, int mem) {
    if (!c) return SKE_EINVAL;
    Filter *F = get_filter(c, fid);
    if (!F) return SKE_EINVAL;
    if (n == 0) return SKE_OK;
    if (n >= 0xffffffffull) return SKE_EINVAL;
    if (!F->exists) {  // rebloom.c BF.ADD / BF.MADD auto-create: 0.01, 100, expansion 2
        int rc = ske_bf_reserve(c, fid, 0.01, 100, 2, 0);
        if (rc) return rc;
    }
    Staged s;
    int rc = stage_items(c, bytes, offs, n, mem, &s);
    if (rc) return rc;
    hipError_t e = hipSuccess;
    uint64_t *ha = (uint64_t *)scratch_get(c->scratch, 10, n * 8, &e);
    uint64_t *hb = (uint64_t *)scratch_get(c->scratch, 11, n * 8, &e);
    uint8_t *state = (uint8_t *)scratch_get(c->scratch, 12, n, &e);
    int8_t *res = (int8_t *)scratch_get(c->scratch, 13, n, &e);
    uint32_t *absent = (uint32_t *)scratch_get(c->scratch, 14, n * 4, &e);
    uint32_t *pos = (uint32_t *)scratch_get(c->scratch, 15, n * 4, &e);
    if (e != hipSuccess) {
        c->last_hip = hipGetErrorString(e);
        return SKE_ENOMEM;
    }
    HIPCHK(c, hipMemsetAsync(state, 0, n, c->st));
    HIPCHK(c, launch_bf_hash(s.bytes, s.offs, n, ha, hb, c->cus, c->st));
    HIPCHK(c, launch_bf_settle_present(chain_dev(*F), n, ha, hb, state, res, c->cus, c->st));
    for (int epoch = 0; epoch < 4 * SKE_MAX_LINKS + 4; epoch++) {
        Link *L = &F->links.back();
        uint64_t cap = L->size >= L->entries ? 0 : L->entries - L->size;
        if (cap == 0) {
            HIPCHK(c, hipMemsetAsync(c->stats, 0, 8, c->st));
            HIPCHK(c, launch_bf_count_cands(n, state, c->stats, c->cus, c->st));
            unsigned long long remaining = 0;
            HIPCHK(c, hipMemcpyAsync(&remaining, c->stats, 8, hipMemcpyDeviceToHost, c->st));
            HIPCHK(c, hipStreamSynchronize(c->st));
            if (remaining == 0) break;
            if (F->nonscaling) {
                HIPCHK(c, launch_bf_fill_rest(n, state, res, -2, c->cus, c->st));
                break;
            }
            // SBChain_Add(): next link entries * growth, error * 0.5
            rc = add_link(c, *F, L->entries * (uint64_t)F->growth, L->error * 0.5);
            if (rc) return rc;
            L = &F->links.back();
            cap = L->entries;
        }
        if (L->bits > 0xffffffffull * 4ull) return SKE_ENOMEM;
        uint32_t *first = (uint32_t *)scratch_get(c->scratch, 0, L->bits * 4, &e);
        if (e != hipSuccess) {
            c->last_hip = hipGetErrorString(e);
            return SKE_ENOMEM;
        }
        HIPCHK(c, hipMemsetAsync(first, 0xff, L->bits * 4, c->st));
        const LinkDev D = link_dev(*L);
        HIPCHK(c, launch_bf_first_setter(D, n, ha, hb, state, first, c->cus, c->st));
        HIPCHK(c, launch_bf_absent(D, n, ha, hb, state, first, absent, c->cus, c->st));
        HIPCHK(c, scan_inclusive_u32(c->scratch, absent, pos, n, c->st));
        uint32_t total_absent = 0;
        HIPCHK(c, hipMemcpyAsync(&total_absent, pos + (n - 1), 4, hipMemcpyDeviceToHost, c->st));
        HIPCHK(c, hipStreamSynchronize(c->st));
        const uint32_t cap32 = cap > 0xffffffffull ? 0xffffffffu : uint32_t(cap);
        HIPCHK(c, launch_bf_resolve(D, n, ha, hb, state, absent, pos, cap32, res, L->bf, c->cus,
                                    c->st));
        const uint64_t added = std::min<uint64_t>(cap, total_absent);
        L->size += added;
        F->size += added;
        if (total_absent < cap) break;  // every candidate resolved
        // the rest see this link as left by the resolved adds
        ChainDev one{};
        one.nlinks = 1;
        one.link[0] = D;
        HIPCHK(c, launch_bf_settle_present(one, n, ha, hb, state, res, c->cus, c->st));
    }
    if (out) {
        if (mem == SKE_MEM_DEVICE)
            HIPCHK(c, hipMemcpyAsync(out, res, n, hipMemcpyDeviceToDevice, c->st));
        else
            HIPCHK(c, hipMemcpyAsync(out, res, n, hipMemcpyDeviceToHost, c->st));
    }
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

// ------------------------------------------------------------------ HLL
int ske_hll_reserve(ske_ctx *c, uint32_t nslots) {
    if (!c) return SKE_EINVAL;
    if (nslots <= c->nslots) return SKE_OK;
    if (c->live_graphs > 0 || c->capturing) {
        c->last_hip = "the HLL slab cannot move while a recorded graph points to it";
        return SKE_EBUSY;
    }
    uint64_t want = std::max<uint64_t>(nslots, uint64_t(c->nslots) * 3 / 2);
    want = std::max<uint64_t>(want, 16);
    uint8_t *nr = nullptr;
    hipError_t e = hipMalloc(&nr, want * SKE_HLL_REGISTERS);
    if (e != hipSuccess) {
        c->last_hip = std::string("hipMalloc(hll slab): ") + hipGetErrorString(e);
        return SKE_ENOMEM;
    }
    HIPCHK(c, hipMemsetAsync(nr, 0, want * SKE_HLL_REGISTERS, c->st));
    if (c->regs) {
        HIPCHK(c, hipMemcpyAsync(nr, c->regs, uint64_t(c->nslots) * SKE_HLL_REGISTERS,
                                 hipMemcpyDeviceToDevice, c->st));
        HIPCHK(c, hipStreamSynchronize(c->st));
        (void)hipFree(c->regs);
    }
    HIPCHK(c, hipStreamSynchronize(c->st));
    c->regs = nr;
    c->nslots = uint32_t(want);
    return SKE_OK;
}

uint32_t ske_hll_capacity(ske_ctx *c) { return c ? c->nslots : 0; }

int ske_hll_clear(ske_ctx *c, uint32_t slot) {
    if (!c) return SKE_EINVAL;
    if (slot >= c->nslots) return SKE_ERANGE;
    HIPCHK(c, hipMemsetAsync(c->regs + uint64_t(slot) * SKE_HLL_REGISTERS, 0, SKE_HLL_REGISTERS,
                             c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

int ske_hll_pfadd(ske_ctx *c, const uint32_t *slot, const uint8_t *bytes, const uint32_t *offs,
                  uint64_t n, uint8_t *changed, int mem) {
    if (!c || !slot) return SKE_EINVAL;
    if (n == 0) return SKE_OK;
    if (const int erc = err_begin(c)) return erc;  // earlier enqueue-only calls' slot errors
    if (n >= 0xffffffffull) return SKE_EINVAL;
    Staged s;
    int rc = stage_items(c, bytes, offs, n, mem, &s);
    if (rc) return rc;
    const uint32_t *dslot;
    rc = stage_u32(c, slot, n, mem, 2, &dslot);
    if (rc) return rc;
    if (changed) {
        uint8_t *dch = changed;
        if (mem != SKE_MEM_DEVICE) {
            dch = (uint8_t *)stage_buf(c, 3, n, &rc);
            if (rc) return rc;
        }
        HIPCHK(c, pfadd_exact(c->scratch, dslot, s.bytes, s.offs, n, c->regs, c->nslots, dch,
                              c->err, c->cus, c->st));
        if (mem != SKE_MEM_DEVICE)
            HIPCHK(c, hipMemcpyAsync(changed, dch, n, hipMemcpyDeviceToHost, c->st));
    } else {
        HIPCHK(c, launch_pfadd(dslot, s.bytes, s.offs, n, c->regs, c->nslots, c->err, c->cus,
                               c->st));
    }
    return check_call_err(c);
}

int ske_swipes(ske_ctx *c, uint32_t fid, const uint32_t *slot, const uint8_t *bytes,
               const uint32_t *offs, uint64_t n, uint8_t *out_valid, int mem) {
    if (!c || !slot) return SKE_EINVAL;
    Filter *F = get_filter(c, fid);
    if (!F) return SKE_EINVAL;
    if (n == 0) return SKE_OK;
    if (const int erc = err_begin(c)) return erc;  // earlier enqueue-only calls' slot errors
    const bool fed = mem != SKE_MEM_DEVICE;  // pass kinds 6-8: the host-fed call's stages
    const PassMark mcall = fed ? mark_begin(c, 8) : PassMark();
    const PassMark mh2d = fed ? mark_begin(c, 6) : PassMark();
    Staged s;
    int rc = stage_items(c, bytes, offs, n, mem, &s);
    if (rc) return rc;
    const uint32_t *dslot;
    rc = stage_u32(c, slot, n, mem, 2, &dslot);
    if (rc) return rc;
    mark_end(c, mh2d);
    uint8_t *dout = out_valid;
    if (out_valid && fed) {
        dout = (uint8_t *)stage_buf(c, 3, n, &rc);
        if (rc) return rc;
    }
    static const ChainDev empty{};
    rc = launch_k1(c, F->exists ? cached_chain(*F) : empty, s.bytes, s.offs, 0, dslot, n, dout);
    if (rc) return rc;
    if (out_valid && fed) {
        const PassMark md2h = mark_begin(c, 7);
        HIPCHK(c, hipMemcpyAsync(out_valid, dout, n, hipMemcpyDeviceToHost, c->st));
        mark_end(c, md2h);
    }
    mark_end(c, mcall);
    return check_call_err(c);
}

int ske_swipes_async(ske_ctx *c, uint32_t fid, const uint32_t *slot, const uint8_t *bytes,
                     const uint32_t *offs, uint64_t n, uint8_t *out_valid) {
    if (!c || !slot) return SKE_EINVAL;
    Filter *F = get_filter(c, fid);
    if (!F) return SKE_EINVAL;
    static const ChainDev empty{};
    return launch_k1(c, F->exists ? cached_chain(*F) : empty, bytes, offs, 0, slot, n, out_valid);
}

// Several resident batches in one call: batch j on branch j mod B, each branch
// a side stream forked from and joined back into the context stream (so the
// call also records into a graph).  With B > 1 the short-id K1 runs on one
// block per two CUs unless "k1_grid" is set, so two launches share the chip
// and one launch's fixed cost overlaps the other's steady state.
static int swipes_many_body(ske_ctx *c, const ChainDev &ch, const ske_swipe_batch *b,
                            uint32_t nb, uint32_t br, hipStream_t home) {
    HIPCHK(c, hipEventRecord(c->many_fork, home));
    uint32_t forked = 0;
    int rc = SKE_OK;
    for (; forked + 1 < br; forked++) {
        hipError_t e = hipStreamWaitEvent(c->many_st[forked], c->many_fork, 0);
        if (e != hipSuccess) {
            c->last_hip = std::string("hipStreamWaitEvent(fork): ") + hipGetErrorString(e);
            rc = SKE_EHIP;
            break;
        }
    }
    for (uint32_t j = 0; j < nb && rc == SKE_OK; j++) {
        uint32_t k = j % br;
        c->st = k ? c->many_st[k - 1] : home;
        rc = launch_k1(c, ch, b[j].bytes, b[j].width ? nullptr : b[j].offs, b[j].width, b[j].slot, b[j].n,
                       b[j].out_valid);
    }
    c->st = home;
    // join every forked branch on every path (an unjoined side stream would
    // invalidate a capture, and outside one leave work the home stream does
    // not wait for); the first error is returned
    for (uint32_t i = 0; i < forked; i++) {
        hipError_t e = hipEventRecord(c->many_join[i], c->many_st[i]);
        if (e == hipSuccess) e = hipStreamWaitEvent(home, c->many_join[i], 0);
        if (e != hipSuccess && rc == SKE_OK) {
            c->last_hip = std::string("join: ") + hipGetErrorString(e);
            rc = SKE_EHIP;
        }
    }
    return rc;
}

static int swipes_many_persistent(ske_ctx *c, const K1Args &A, const ske_swipe_batch *b, uint32_t nb) {
    const uint32_t T = k1_many_tile(c->pb);
    for (uint32_t j0 = 0; j0 < nb; j0 += kK1ManyMax) {
        K1Many M{};
        M.nb = nb - j0 < kK1ManyMax ? nb - j0 : kK1ManyMax;
        M.tpre[0] = 0;
        for (uint32_t j = 0; j < M.nb; j++) {
            const ske_swipe_batch &B = b[j0 + j];
            M.b[j] = K1Batch{B.bytes, B.width ? nullptr : B.offs, B.slot, B.out_valid, uint32_t(B.n), B.width};
            const uint64_t tp = M.tpre[j] + (B.n + T - 1) / T;
            if (tp >= (uint64_t(1) << 31)) return SKE_EINVAL;
            M.tpre[j + 1] = uint32_t(tp);
        }
        const PassMark m = mark_begin(c, 0);
        HIPCHK(c, launch_swipes_lds_many(A, M, c->pb, c->k1_grid ? c->k1_grid : c->cus, c->st));
        mark_end(c, m);
    }
    return SKE_OK;
}

int ske_swipes_many_async(ske_ctx *c, uint32_t fid, const ske_swipe_batch *b, uint32_t nb,
                          uint32_t branches) {
    if (!c || (nb && !b) || branches > SKE_MANY_MAX_BRANCHES) return SKE_EINVAL;
    Filter *F = get_filter(c, fid);
    if (!F) return SKE_EINVAL;
    for (uint32_t j = 0; j < nb; j++)
        if (!b[j].slot || (b[j].width == 0 && !b[j].offs) || b[j].width > 4096) return SKE_EINVAL;
    static const ChainDev empty{};
    const ChainDev &ch = F->exists ? cached_chain(*F) : empty;
    // the short-id LDS K1: one persistent launch per kK1ManyMax batches, the
    // branches unused
    if (nb && c->k1_persistent) {
        K1Args A;
        bool ok = true;
        for (uint32_t j = 0; j < nb && ok; j++)
            ok = k1_fast_args(c, ch, b[j].bytes, b[j].width ? nullptr : b[j].offs, b[j].width, b[j].slot,
                              b[j].n, b[j].out_valid, &A);
        if (ok) return swipes_many_persistent(c, A, b, nb);
    }
    // the partitioned K1: one call over every batch, before any branch
    // streams are made (it uses none; creating them lazily here cost ms of
    // host time per new count)
    const int var = nb ? k1_variant(c, ch) : 0;
    if (var == 3) {
        std::vector<PartBatch> pb(nb);
        for (uint32_t j = 0; j < nb; j++)
            pb[j] = PartBatch{b[j].bytes, b[j].width ? nullptr : b[j].offs, b[j].width, b[j].slot, b[j].n,
                              b[j].out_valid};
        return launch_part(c, ch, pb.data(), nb);
    }
    uint32_t br = branches ? branches : SKE_MANY_DEFAULT_BRANCHES;
    if (nb && br > nb) br = nb;
    if (br > 1) {  // with nb == 0: only prepares the side streams (e.g. before capture)
        if (!c->many_fork) HIPCHK(c, hipEventCreateWithFlags(&c->many_fork, hipEventDisableTiming));
        while (c->many_n < int(br) - 1) {
            HIPCHK(c, hipStreamCreateWithFlags(&c->many_st[c->many_n], hipStreamNonBlocking));
            HIPCHK(c, hipEventCreateWithFlags(&c->many_join[c->many_n], hipEventDisableTiming));
            c->many_n++;
        }
    }
    if (nb == 0) return SKE_OK;
    // the scratch of the largest batch before the first launch: batches of
    // different sizes never reallocate it between recorded launches
    uint64_t nmax = 0;
    for (uint32_t j = 0; j < nb; j++) nmax = b[j].n > nmax ? b[j].n : nmax;
    if (var == 2 && nmax) {
        hipError_t e = hipSuccess;
        (void)scratch_get(c->scratch, 16, xr_scratch_bytes(nmax, ch.nlinks), &e);
        if (e != hipSuccess) return scratch_error(c, e);
    }
    if (br == 1) {
        for (uint32_t j = 0; j < nb; j++) {
            int rc = launch_k1(c, ch, b[j].bytes, b[j].width ? nullptr : b[j].offs, b[j].width, b[j].slot, b[j].n,
                               b[j].out_valid);
            if (rc) return rc;
        }
        return SKE_OK;
    }
    hipStream_t home = c->st;
    int grid0 = c->k1_grid;
    if (!grid0) c->k1_grid = c->cus / 2 > 0 ? c->cus / 2 : 1;
    int rc = swipes_many_body(c, ch, b, nb, br, home);
    c->st = home;
    c->k1_grid = grid0;
    return rc;
}

int ske_route_swipes(ske_ctx *c, const uint8_t *ids, uint32_t width, const uint32_t *gkey, uint64_t n,
                     uint32_t world, const uint32_t *key_owner, const uint32_t *key_local, uint32_t nkeys,
                     uint8_t *send_ids, uint32_t *send_slots, uint32_t *pos, uint64_t *counts) {
    if (!c || !counts || world == 0 || world > 64 || width == 0 || width > 4096 || n >= (uint64_t(1) << 32))
        return SKE_EINVAL;
    if (n && (!ids || !gkey || !send_ids || !send_slots || !pos)) return SKE_EINVAL;
    if (nkeys && (!key_owner || !key_local)) return SKE_EINVAL;
    hipError_t e = hipSuccess;
    uint32_t *hist = (uint32_t *)scratch_get(c->scratch, 40, route_hist_words(n, world) * 4 + 4, &e);
    uint32_t *tot = e == hipSuccess ? (uint32_t *)scratch_get(c->scratch, 41, size_t(world) * 4, &e) : nullptr;
    if (e != hipSuccess) return scratch_error(c, e);
    unsigned long long cid = 0;
    const int rc = scratch_user_begin(c, &cid, c->rt);  // an async routing call on another stream finishes first
    if (rc) return rc;
    scratch_user_end(c, cid, c->rt);
    HIPCHK(c, launch_route(ids, width, gkey, n, world, key_owner, key_local, nkeys, send_ids, send_slots, pos,
                           hist, tot, c->st));
    uint32_t h[64];
    HIPCHK(c, hipMemcpyAsync(h, tot, size_t(world) * 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    for (uint32_t o = 0; o < world; o++) counts[o] = h[o];
    return SKE_OK;
}

int ske_route_swipes_cap_async(ske_ctx *c, const uint8_t *ids, uint32_t width, const uint32_t *gkey, uint64_t n,
                               uint32_t world, const uint32_t *key_route, uint32_t nkeys, uint32_t cap,
                               const uint32_t *sink_slots, uint8_t *send_ids, uint32_t *send_slots, uint32_t *pos,
                               uint32_t *counts) {
    if (!c || !counts || !sink_slots || world == 0 || world > 64 || width == 0 || width > 4096 ||
        n >= (uint64_t(1) << 32) || cap == 0 || uint64_t(cap) * world >= (uint64_t(1) << 32))
        return SKE_EINVAL;
    if (!send_ids || !send_slots || (n && (!ids || !gkey || !pos))) return SKE_EINVAL;
    if (nkeys && !key_route) return SKE_EINVAL;
    hipError_t e = hipSuccess;
    uint32_t *hist = (uint32_t *)scratch_get(c->scratch, 40, route_hist_words(n, world) * 4 + 4, &e);
    if (e != hipSuccess) return scratch_error(c, e);
    // the histogram is context scratch (slot 40, no K1 uses it): a routing
    // call on another stream waits for this one's kernels, a K1 does not --
    // the next batch's routing runs beside this batch's K1
    // (distributed.SwipeExchange's pipelined form)
    unsigned long long cid = 0;
    const int rc = scratch_user_begin(c, &cid, c->rt);
    if (rc) return rc;
    const hipError_t le = launch_route_cap(ids, width, gkey, n, world, key_route, nkeys, cap, sink_slots, send_ids,
                                           send_slots, pos, hist, counts, c->cus, c->st);
    if (le != hipSuccess) {
        c->last_hip = std::string("launch_route_cap: ") + hipGetErrorString(le);
        scratch_user_end(c, cid, c->rt);
        return SKE_EHIP;
    }
    return scratch_user_end(c, cid, c->rt);
}

int ske_route_slots_async(ske_ctx *c, const uint32_t *gkey, uint64_t n, const uint32_t *key_route, uint32_t nkeys,
                          uint32_t world, uint32_t *out_slots) {
    if (!c || world == 0 || world > 64 || (n && (!gkey || !out_slots)) || (!key_route && world != 1) ||
        (!key_route && nkeys > 0x3ffffffu))
        return SKE_EINVAL;
    HIPCHK(c, launch_route_slots(gkey, n, key_route, nkeys, world, out_slots, c->cus, c->st));
    return SKE_OK;
}

int ske_route_return_async(ske_ctx *c, const uint8_t *answers, const uint32_t *pos, uint64_t n, uint8_t *out) {
    if (!c || (n && (!answers || !pos || !out))) return SKE_EINVAL;
    HIPCHK(c, launch_route_return(answers, pos, n, out, c->cus, c->st));
    return SKE_OK;
}

int ske_swipes_fixed_async(ske_ctx *c, uint32_t fid, const uint32_t *slot, const uint8_t *bytes,
                           uint32_t width, uint64_t n, uint8_t *out_valid) {
    if (!c || !slot || width == 0 || width > 4096) return SKE_EINVAL;
    Filter *F = get_filter(c, fid);
    if (!F) return SKE_EINVAL;
    static const ChainDev empty{};
    return launch_k1(c, F->exists ? cached_chain(*F) : empty, bytes, nullptr, width, slot, n,
                     out_valid);
}

int ske_swipes_fixed(ske_ctx *c, uint32_t fid, const uint32_t *slot, const uint8_t *bytes,
                     uint32_t width, uint64_t n, uint8_t *out_valid, int mem) {
    if (!c || !slot || width == 0 || width > 4096) return SKE_EINVAL;
    Filter *F = get_filter(c, fid);
    if (!F) return SKE_EINVAL;
    if (n == 0) return SKE_OK;
    if (const int erc = err_begin(c)) return erc;  // earlier enqueue-only calls' slot errors
    int rc = SKE_OK;
    const uint8_t *db = bytes;
    const uint32_t *dslot = slot;
    uint8_t *dout = out_valid;
    if (mem != SKE_MEM_DEVICE) {
        uint8_t *b = (uint8_t *)stage_buf(c, 0, n * width + 16, &rc);
        if (rc) return rc;
        HIPCHK(c, hipMemcpyAsync(b, bytes, n * width, hipMemcpyHostToDevice, c->st));
        db = b;
        rc = stage_u32(c, slot, n, mem, 2, &dslot);
        if (rc) return rc;
        if (out_valid) {
            dout = (uint8_t *)stage_buf(c, 3, n, &rc);
            if (rc) return rc;
        }
    }
    rc = ske_swipes_fixed_async(c, fid, dslot, db, width, n, dout);
    if (rc) return rc;
    if (out_valid && mem != SKE_MEM_DEVICE)
        HIPCHK(c, hipMemcpyAsync(out_valid, dout, n, hipMemcpyDeviceToHost, c->st));
    return check_call_err(c);
}

// Fixed-width swipes with bit-packed answers.  Host inputs are cut into
// chunks of kFeedChunk swipes: the chunk's ids and slots go host -> device on
// a copy stream (sketch_host.cpp's pinned double buffer for pageable memory)
// while K1 runs on the previous chunk on the context stream; each chunk's
// answers are packed to bits on the device and copied back (1 bit per swipe).
// Per swipe the host link carries width + 4 bytes in and 1/8 byte out.
constexpr uint64_t kFeedChunk = uint64_t(4) << 20;

int ske_swipes_fixed_bits(ske_ctx *c, uint32_t fid, const uint32_t *slot, const uint8_t *bytes, uint32_t width,
                          uint64_t n, uint8_t *out_bits, int mem) {
    if (!c || !slot || !bytes || width == 0 || width > 4096) return SKE_EINVAL;
    Filter *F = get_filter(c, fid);
    if (!F) return SKE_EINVAL;
    if (n == 0) return SKE_OK;
    if (const int erc = err_begin(c)) return erc;  // earlier enqueue-only calls' slot errors
    int rc = SKE_OK;
    // the answers (bytes, 8-B aligned for the packer) always on the device
    uint8_t *dans = (uint8_t *)stage_buf(c, 4, n + 16, &rc);
    if (rc) return rc;
    if (mem == SKE_MEM_DEVICE) {
        rc = ske_swipes_fixed_async(c, fid, slot, bytes, width, n, dans);
        if (rc) return rc;
        if (out_bits) HIPCHK(c, launch_pack_bits(dans, n, out_bits, c->cus, c->st));
        return check_call_err(c);
    }
    uint8_t *db = (uint8_t *)stage_buf(c, 0, n * width + 16, &rc);
    uint32_t *ds = rc ? nullptr : (uint32_t *)stage_buf(c, 2, n * 4 + 16, &rc);
    uint8_t *dbits = rc ? nullptr : (uint8_t *)stage_buf(c, 3, (n + 7) / 8 + 16, &rc);
    if (rc) return rc;
    if (!c->copy_st) HIPCHK(c, hipStreamCreateWithFlags(&c->copy_st, hipStreamNonBlocking));
    if (!c->hs) c->hs = stager_new();
    const uint64_t nchunks = (n + kFeedChunk - 1) / kFeedChunk;
    while (c->chunk_ev.size() < nchunks) {
        hipEvent_t e = nullptr;
        HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->chunk_ev.push_back(e);
    }
    // the copy stream starts behind everything already on the context stream
    // (earlier users of the staging buffers)
    const PassMark mcall = mark_begin(c, 8);  // pass kinds 6-8: this host-fed call's stages
    HIPCHK(c, hipEventRecord(c->chunk_ev[0], c->st));
    HIPCHK(c, hipStreamWaitEvent(c->copy_st, c->chunk_ev[0], 0));
    // once a copy is queued, every exit waits for the copy stream first: the
    // DMA may still read the caller's (pinned) buffers
    auto chunks = [&]() -> int {
        for (uint64_t j = 0; j < nchunks; j++) {
            const uint64_t s0 = j * kFeedChunk, m = n - s0 < kFeedChunk ? n - s0 : kFeedChunk;
            const PassMark mh2d = mark_begin(c, 6, c->copy_st);
            HIPCHK(c, stage_h2d(c->hs, db + s0 * width, bytes + s0 * width, m * width, c->copy_st, false, nullptr));
            HIPCHK(c, stage_h2d(c->hs, ds + s0, slot + s0, m * 4, c->copy_st, false, nullptr));
            mark_end(c, mh2d);
            HIPCHK(c, hipEventRecord(c->chunk_ev[j], c->copy_st));
            HIPCHK(c, hipStreamWaitEvent(c->st, c->chunk_ev[j], 0));
            const int r = ske_swipes_fixed_async(c, fid, ds + s0, db + s0 * width, width, m, dans + s0);
            if (r) return r;
            if (out_bits) {
                HIPCHK(c, launch_pack_bits(dans + s0, m, dbits + s0 / 8, c->cus, c->st));
                const PassMark md2h = mark_begin(c, 7);
                HIPCHK(c, hipMemcpyAsync(out_bits + s0 / 8, dbits + s0 / 8, (m + 7) / 8, hipMemcpyDeviceToHost, c->st));
                mark_end(c, md2h);
            }
        }
        return SKE_OK;
    };
    rc = chunks();
    mark_end(c, mcall);
    const hipError_t se = hipStreamSynchronize(c->copy_st);
    if (rc) return rc;
    HIPCHK(c, se);
    return check_call_err(c);
}

#ifdef SKE_STAMPS
// diagnostic build only: point the phase-stamp side buffer at dev_ptr
int ske_diag_set_stamp_buffer(ske_ctx *c, void *dev_ptr) {
    if (!c) return SKE_EINVAL;
    HIPCHK(c, ske::set_stamp_buffer(dev_ptr));
    return SKE_OK;
}
int ske_diag_set_pb_stamp_buffer(ske_ctx *c, void *dev_ptr) {
    if (!c) return SKE_EINVAL;
    HIPCHK(c, ske::set_pb_stamp_buffer(dev_ptr));
    return SKE_OK;
}
int ske_diag_set_k1_stamp_buffer(ske_ctx *c, void *dev_ptr) {
    if (!c) return SKE_EINVAL;
    HIPCHK(c, ske::set_k1_stamp_buffer(dev_ptr));
    return SKE_OK;
}
#endif
#ifdef SKE_SEG_STAMPS
int ske_diag_set_seg_stamp_buffer(ske_ctx *c, void *dev_ptr) {
    if (!c) return SKE_EINVAL;
    HIPCHK(c, ske::set_seg_stamp_buffer(dev_ptr));
    return SKE_OK;
}
#endif

int ske_swipes_stats(ske_ctx *c, uint32_t fid, const uint8_t *bytes, const uint32_t *offs,
                     uint64_t n, uint64_t *probes, uint64_t *nvalid) {
    if (!c || !probes || !nvalid) return SKE_EINVAL;
    Filter *F = get_filter(c, fid);
    if (!F) return SKE_EINVAL;
    const ChainDev ch = F->exists ? chain_dev(*F) : ChainDev{};
    HIPCHK(c, hipMemsetAsync(c->stats, 0, 16, c->st));
    // every tile size follows RedisBloom's per-swipe probe order, so the
    // count is the sequential one
    HIPCHK(c, launch_swipes(2, ch, use_lds(c, ch), c->pb, bytes, offs, 0, nullptr, n, nullptr, 0, nullptr,
                            c->stats, c->cus, c->st));
    unsigned long long h[2] = {0, 0};
    HIPCHK(c, hipMemcpyAsync(h, c->stats, 16, hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    *probes = h[0];
    *nvalid = h[1];
    return SKE_OK;
}

int ske_swipes_variant(ske_ctx *c, uint32_t fid) {
    Filter *F = c ? get_filter(c, fid) : nullptr;
    if (!F) return SKE_EINVAL;
    const ChainDev ch = F->exists ? chain_dev(*F) : ChainDev{};
    return k1_variant(c, ch);
}

static int pfcount_impl(ske_ctx *c, const uint8_t *regs, const uint32_t *slots,
                        const uint32_t *goffs, uint32_t ngroups, uint64_t *out, int mem) {
    int rc = ensure_tables(c);
    if (rc) return rc;
    uint64_t *dout = out;
    if (mem != SKE_MEM_DEVICE) {
        dout = (uint64_t *)stage_buf(c, 5, uint64_t(ngroups) * 8, &rc);
        if (rc) return rc;
    }
    HIPCHK(c, launch_pfcount(regs, slots, goffs, ngroups, c->tau, c->sig, dout, c->cus, c->st));
    if (mem != SKE_MEM_DEVICE)
        HIPCHK(c, hipMemcpyAsync(out, dout, uint64_t(ngroups) * 8, hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

static int check_slots_host(ske_ctx *c, const uint32_t *slots, uint64_t n) {
    for (uint64_t i = 0; i < n; i++)
        if (slots[i] >= c->nslots) return SKE_ERANGE;
    return SKE_OK;
}

// a device-resident slot list in range of the slab (one reduction kernel and
// a 4-byte read back): SKE_ERANGE before any kernel addresses the slab with it
static int check_slots_dev(ske_ctx *c, const uint32_t *slots, uint64_t n) {
    if (n == 0) return SKE_OK;
    int rc = SKE_OK;
    unsigned int *d = (unsigned int *)stage_buf(c, 8, 4, &rc);
    if (rc) return rc;
    unsigned int mx = 0;
    HIPCHK(c, launch_slots_max(slots, n, d, c->cus, c->st));
    HIPCHK(c, hipMemcpyAsync(&mx, d, 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return mx >= c->nslots ? SKE_ERANGE : SKE_OK;
}

int ske_hll_pfcount(ske_ctx *c, const uint32_t *slots, uint32_t nkeys, uint64_t *out) {
    if (!c || !slots || !out || nkeys == 0) return SKE_EINVAL;
    int rc = check_slots_host(c, slots, nkeys);
    if (rc) return rc;
    const uint32_t *ds;
    rc = stage_u32(c, slots, nkeys, SKE_MEM_HOST, 6, &ds);
    if (rc) return rc;
    const uint32_t go[2] = {0, nkeys};
    const uint32_t *dg;
    rc = stage_u32(c, go, 2, SKE_MEM_HOST, 7, &dg);
    if (rc) return rc;
    return pfcount_impl(c, c->regs, ds, dg, 1, out, SKE_MEM_HOST);
}

int ske_hll_pfcount_each(ske_ctx *c, const uint32_t *slots, uint32_t nkeys, uint64_t *out,
                         int mem) {
    if (!c || !out) return SKE_EINVAL;
    if (nkeys == 0) return SKE_OK;
    if (slots) {
        int rc = mem == SKE_MEM_DEVICE ? check_slots_dev(c, slots, nkeys) : check_slots_host(c, slots, nkeys);
        if (rc) return rc;
    }
    const uint32_t *ds = nullptr;
    if (slots) {
        int rc = stage_u32(c, slots, nkeys, mem, 6, &ds);
        if (rc) return rc;
    } else if (nkeys > c->nslots) {
        return SKE_ERANGE;
    }
    return pfcount_impl(c, c->regs, ds, nullptr, nkeys, out, mem);
}

int ske_hll_pfcount_groups(ske_ctx *c, const uint32_t *slots, const uint32_t *goffs,
                           uint32_t ngroups, uint64_t *out, int mem) {
    if (!c || !slots || !goffs || !out) return SKE_EINVAL;
    if (ngroups == 0) return SKE_OK;
    int rc;
    if (mem != SKE_MEM_DEVICE) {
        for (uint32_t g = 0; g < ngroups; g++)
            if (goffs[g + 1] < goffs[g]) return SKE_EINVAL;
        rc = check_slots_host(c, slots + goffs[0], goffs[ngroups] - goffs[0]);
        if (rc) return rc;
    }
    const uint32_t *ds, *dg;
    const uint64_t nslots_total = mem == SKE_MEM_DEVICE ? 0 : goffs[ngroups];
    if (mem == SKE_MEM_DEVICE) {
        ds = slots;
        dg = goffs;
    } else {
        rc = stage_u32(c, slots, nslots_total, mem, 6, &ds);
        if (rc) return rc;
        rc = stage_u32(c, goffs, uint64_t(ngroups) + 1, mem, 7, &dg);
        if (rc) return rc;
    }
    return pfcount_impl(c, c->regs, ds, dg, ngroups, out, mem);
}

int ske_hll_merge_groups_dev(ske_ctx *c, const uint32_t *slots, const uint32_t *goffs,
                             uint32_t ngroups, uint8_t *dst_dev) {
    if (!c || !goffs || !dst_dev) return SKE_EINVAL;
    if (ngroups == 0) return SKE_OK;
    for (uint32_t g = 0; g < ngroups; g++)
        if (goffs[g + 1] < goffs[g]) return SKE_EINVAL;
    const uint64_t total = goffs[ngroups];
    if (total && !slots) return SKE_EINVAL;
    int rc = check_slots_host(c, slots, total);
    if (rc) return rc;
    const uint32_t *ds, *dg;
    rc = stage_u32(c, slots, total, SKE_MEM_HOST, 6, &ds);
    if (rc) return rc;
    rc = stage_u32(c, goffs, uint64_t(ngroups) + 1, SKE_MEM_HOST, 7, &dg);
    if (rc) return rc;
    HIPCHK(c, launch_merge_groups(c->regs, ds, dg, ngroups, dst_dev, c->cus, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

int ske_hll_count_raw_dev(ske_ctx *c, const uint8_t *regs_dev, uint32_t nkeys, uint64_t *out) {
    if (!c || !regs_dev || !out) return SKE_EINVAL;
    if (nkeys == 0) return SKE_OK;
    return pfcount_impl(c, regs_dev, nullptr, nullptr, nkeys, out, SKE_MEM_HOST);
}

static int pfmerge_impl(ske_ctx *c, uint32_t dst, const uint32_t *srcs, uint32_t n, int mem) {
    if (!c || (n && !srcs)) return SKE_EINVAL;
    if (dst >= c->nslots) return SKE_ERANGE;
    int rc = mem == SKE_MEM_DEVICE ? check_slots_dev(c, srcs, n) : check_slots_host(c, srcs, n);
    if (rc) return rc;
    if (n == 0) return SKE_OK;
    const uint32_t *ds;
    rc = stage_u32(c, srcs, n, mem, 6, &ds);
    if (rc) return rc;
    if (n <= 256) {
        HIPCHK(c, launch_pfmerge(c->regs, dst, ds, n, c->st));
    } else {
        // campus-wide merges (C5: 1.8M day keys): a two-level parallel max
        uint32_t per = 0;
        const uint32_t P = pfmerge_partitions(n, c->cus, &per);
        hipError_t e = hipSuccess;
        uint8_t *partial = (uint8_t *)scratch_get(c->scratch, 17, size_t(P) * SKE_HLL_REGISTERS, &e);
        if (e != hipSuccess) {
            c->last_hip = hipGetErrorString(e);
            return SKE_ENOMEM;
        }
        HIPCHK(c, launch_pfmerge_wide(c->regs, dst, ds, n, partial, per, P, c->st));
    }
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

int ske_hll_pfmerge(ske_ctx *c, uint32_t dst, const uint32_t *srcs, uint32_t n) {
    return pfmerge_impl(c, dst, srcs, n, SKE_MEM_HOST);
}

int ske_hll_pfmerge_dev(ske_ctx *c, uint32_t dst, const uint32_t *srcs_dev, uint32_t n) {
    return pfmerge_impl(c, dst, srcs_dev, n, SKE_MEM_DEVICE);
}

int ske_hll_histogram(ske_ctx *c, uint32_t slot, uint32_t *out64) {
    if (!c || !out64) return SKE_EINVAL;
    if (slot >= c->nslots) return SKE_ERANGE;
    int rc = SKE_OK;
    uint32_t *d = (uint32_t *)stage_buf(c, 5, 256, &rc);
    if (rc) return rc;
    HIPCHK(c, launch_histogram(c->regs + uint64_t(slot) * SKE_HLL_REGISTERS, d, c->st));
    HIPCHK(c, hipMemcpyAsync(out64, d, 256, hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

int ske_hll_export_raw(ske_ctx *c, uint32_t slot, uint8_t *out) {
    if (!c || !out) return SKE_EINVAL;
    if (slot >= c->nslots) return SKE_ERANGE;
    HIPCHK(c, hipMemcpyAsync(out, c->regs + uint64_t(slot) * SKE_HLL_REGISTERS, SKE_HLL_REGISTERS,
                             hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

int ske_hll_export_dense(ske_ctx *c, uint32_t slot, uint8_t *out) {
    if (!c || !out) return SKE_EINVAL;
    if (slot >= c->nslots) return SKE_ERANGE;
    int rc = SKE_OK;
    uint8_t *d = (uint8_t *)stage_buf(c, 5, SKE_HLL_DENSE_BYTES, &rc);
    if (rc) return rc;
    HIPCHK(c, launch_dense(c->regs + uint64_t(slot) * SKE_HLL_REGISTERS, d, c->st));
    HIPCHK(c, hipMemcpyAsync(out, d, SKE_HLL_DENSE_BYTES, hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

int ske_hll_import_raw(ske_ctx *c, uint32_t slot, const uint8_t *in) {
    if (!c || !in) return SKE_EINVAL;
    if (slot >= c->nslots) return SKE_ERANGE;
    for (int i = 0; i < SKE_HLL_REGISTERS; i++)
        if (in[i] > 51) return SKE_EBADHLL;  // no register can exceed Q+1
    HIPCHK(c, hipMemcpyAsync(c->regs + uint64_t(slot) * SKE_HLL_REGISTERS, in, SKE_HLL_REGISTERS,
                             hipMemcpyHostToDevice, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

int ske_hll_slab(ske_ctx *c, void **p, uint64_t *bytes) {
    if (!c || !p || !bytes) return SKE_EINVAL;
    *p = c->regs;
    *bytes = uint64_t(c->nslots) * SKE_HLL_REGISTERS;
    return SKE_OK;
}

// ------------------------------------------------------------------ ingest
static IngestCols ingest_cols(const ske_ingest_cols_t *c) {
    IngestCols k;
    k.status = c->status;
    k.id_start = c->id_start;
    k.id_len = c->id_len;
    k.lec_start = c->lec_start;
    k.lec_len = c->lec_len;
    k.ts_start = c->ts_start;
    k.ts_len = c->ts_len;
    k.day = c->day;
    k.kh = c->kh;
    return k;
}

int ske_ingest_parse(ske_ctx *c, const uint8_t *msgs, const uint32_t *moffs, uint64_t n,
                     int day_form, const ske_ingest_cols_t *cols) {
    if (!c || !cols || (n && (!msgs || !moffs))) return SKE_EINVAL;
    HIPCHK(c, launch_ingest_parse(msgs, moffs, n, day_form, ingest_cols(cols), c->cus, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

static int keytab_lookup(ske_ctx *c, const ske_ingest_cols_t *cols, uint64_t n, uint32_t *slot,
                         uint32_t **flag, uint32_t **mlen) {
    hipError_t e = hipSuccess;
    *flag = (uint32_t *)scratch_get(c->scratch, 18, n * 4, &e);
    *mlen = (uint32_t *)scratch_get(c->scratch, 19, n * 4, &e);
    if (e != hipSuccess) {
        c->last_hip = hipGetErrorString(e);
        return SKE_ENOMEM;
    }
    HIPCHK(c, launch_keytab_lookup(c->kt_key, c->kt_slot, c->kt_cap ? c->kt_cap - 1 : 0, cols->kh,
                                   cols->status, cols->id_len, n, slot, *flag, *mlen, c->cus, c->st));
    return SKE_OK;
}

int ske_keytab_lookup(ske_ctx *c, const ske_ingest_cols_t *cols, uint64_t n, uint32_t *slot_dev,
                      uint64_t *nmiss) {
    if (!c || !cols || !slot_dev) return SKE_EINVAL;
    if (nmiss) *nmiss = 0;
    if (!n) return SKE_OK;
    uint32_t *flag, *mlen;
    int rc = keytab_lookup(c, cols, n, slot_dev, &flag, &mlen);
    if (rc) return rc;
    if (nmiss) {
        // decoded - found = misses (flag is 1 for found keys)
        hipError_t e = hipSuccess;
        uint32_t *incl = (uint32_t *)scratch_get(c->scratch, 20, n * 4, &e);
        if (!incl) {
            c->last_hip = hipGetErrorString(e);
            return SKE_ENOMEM;
        }
        HIPCHK(c, scan_inclusive_u32(c->scratch, flag, incl, n, c->st));
        uint32_t found = 0;
        HIPCHK(c, hipMemcpyAsync(&found, incl + (n - 1), 4, hipMemcpyDeviceToHost, c->st));
        std::vector<uint8_t> st(n);
        HIPCHK(c, hipMemcpyAsync(st.data(), cols->status, n, hipMemcpyDeviceToHost, c->st));
        HIPCHK(c, hipStreamSynchronize(c->st));
        uint64_t decoded = 0;
        for (uint64_t i = 0; i < n; i++) decoded += st[i] == 0;
        *nmiss = decoded - found;
    } else {
        HIPCHK(c, hipStreamSynchronize(c->st));
    }
    return SKE_OK;
}

static int keytab_grow(ske_ctx *c, uint64_t want) {
    uint64_t cap = 1024;
    while (cap < want * 2) cap <<= 1;
    if (cap <= c->kt_cap) return SKE_OK;
    uint64_t *nk = nullptr;
    uint32_t *ns = nullptr;
    hipError_t e = hipMalloc(&nk, cap * 16);
    if (e == hipSuccess) e = hipMalloc(&ns, cap * 4);
    if (e == hipSuccess) e = hipMemsetAsync(nk, 0, cap * 16, c->st);
    if (e != hipSuccess) {
        if (nk) (void)hipFree(nk);
        if (ns) (void)hipFree(ns);
        c->last_hip = std::string("key table: ") + hipGetErrorString(e);
        return SKE_ENOMEM;
    }
    if (c->kt_cap)  // rehash the old entries (empty ones are skipped)
        HIPCHK(c, launch_keytab_insert(nk, ns, cap - 1, c->kt_key, c->kt_slot, c->kt_cap, c->cus, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    if (c->kt_key) (void)hipFree(c->kt_key);
    if (c->kt_slot) (void)hipFree(c->kt_slot);
    c->kt_key = nk;
    c->kt_slot = ns;
    c->kt_cap = cap;
    return SKE_OK;
}

int ske_keytab_insert(ske_ctx *c, const uint64_t *kh_host, const uint32_t *slots_host, uint64_t n) {
    if (!c || (n && (!kh_host || !slots_host))) return SKE_EINVAL;
    if (!n) return SKE_OK;
    for (uint64_t i = 0; i < n; i++)
        if ((kh_host[2 * i] & 1) == 0) return SKE_EINVAL;  // kh0 is odd by construction
    int rc = keytab_grow(c, c->kt_count + n);
    if (rc) return rc;
    int r2 = SKE_OK;
    uint64_t *dk = (uint64_t *)stage_buf(c, 6, n * 16, &r2);
    uint32_t *ds = (uint32_t *)stage_buf(c, 7, n * 4, &r2);
    if (r2) return r2;
    HIPCHK(c, hipMemcpyAsync(dk, kh_host, n * 16, hipMemcpyHostToDevice, c->st));
    HIPCHK(c, hipMemcpyAsync(ds, slots_host, n * 4, hipMemcpyHostToDevice, c->st));
    HIPCHK(c, launch_keytab_insert(c->kt_key, c->kt_slot, c->kt_cap - 1, dk, ds, n, c->cus, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    c->kt_count += n;
    return SKE_OK;
}

int ske_keytab_clear(ske_ctx *c) {
    if (!c) return SKE_EINVAL;
    if (c->kt_cap) {
        HIPCHK(c, hipMemsetAsync(c->kt_key, 0, c->kt_cap * 16, c->st));
        HIPCHK(c, hipStreamSynchronize(c->st));
    }
    c->kt_count = 0;
    return SKE_OK;
}

int ske_ingest_swipes(ske_ctx *c, uint32_t fid, const uint8_t *msgs, const ske_ingest_cols_t *cols,
                      uint64_t n, uint8_t *valid_dev, uint64_t *ntaken) {
    if (!c || !cols || !valid_dev || (n && !msgs)) return SKE_EINVAL;
    Filter *F = get_filter(c, fid);
    if (!F) return SKE_EINVAL;
    if (ntaken) *ntaken = 0;
    if (!n) return SKE_OK;
    if (const int erc = err_begin(c)) return erc;  // earlier enqueue-only calls' slot errors
    if (n >= (uint64_t(1) << 31)) return SKE_EINVAL;
    hipError_t e = hipSuccess;
    uint32_t *slot = (uint32_t *)scratch_get(c->scratch, 21, n * 4, &e);
    uint32_t *flag_incl = (uint32_t *)scratch_get(c->scratch, 22, n * 4, &e);
    uint32_t *len_incl = (uint32_t *)scratch_get(c->scratch, 23, n * 4, &e);
    if (e != hipSuccess) {
        c->last_hip = hipGetErrorString(e);
        return SKE_ENOMEM;
    }
    uint32_t *flag, *mlen;
    int rc = keytab_lookup(c, cols, n, slot, &flag, &mlen);
    if (rc) return rc;
    HIPCHK(c, scan_inclusive_u32(c->scratch, flag, flag_incl, n, c->st));
    HIPCHK(c, scan_inclusive_u32(c->scratch, mlen, len_incl, n, c->st));
    uint32_t tot[2] = {0, 0};
    HIPCHK(c, hipMemcpyAsync(&tot[0], flag_incl + (n - 1), 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipMemcpyAsync(&tot[1], len_incl + (n - 1), 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    const uint32_t taken = tot[0], nbytes = tot[1];
    uint8_t *ids = (uint8_t *)scratch_get(c->scratch, 24, size_t(nbytes) + 16, &e);
    uint32_t *ids_offs = (uint32_t *)scratch_get(c->scratch, 25, (size_t(taken) + 1) * 4, &e);
    uint32_t *kslot = (uint32_t *)scratch_get(c->scratch, 26, size_t(taken) * 4 + 4, &e);
    uint8_t *kvalid = (uint8_t *)scratch_get(c->scratch, 27, size_t(taken) + 4, &e);
    if (e != hipSuccess) {
        c->last_hip = hipGetErrorString(e);
        return SKE_ENOMEM;
    }
    const IngestCols k = ingest_cols(cols);
    HIPCHK(c, launch_ingest_pack(msgs, k, slot, flag_incl, len_incl, n, ids, ids_offs, kslot, c->cus,
                                 c->st));
    HIPCHK(c, hipMemsetAsync(kvalid, 0, size_t(taken) + 4, c->st));
    if (taken && F->exists) {
        rc = launch_k1(c, cached_chain(*F), ids, ids_offs, 0, kslot, taken, kvalid);
        if (rc) return rc;
    }
    HIPCHK(c, launch_ingest_unpack(k, slot, flag_incl, kvalid, n, valid_dev, c->cus, c->st));
    if (ntaken) *ntaken = taken;
    return check_call_err(c);
}

// ------------------------------------------------------------------ graphs
int ske_capture_begin(ske_ctx *c) {
    if (!c) return SKE_EINVAL;
    HIPCHK(c, hipStreamBeginCapture(c->st, hipStreamCaptureModeThreadLocal));
    c->capturing = true;
    c->cap_users = 0;
    scratch_set_recording(c->scratch, true);
    return SKE_OK;
}

int ske_capture_end(ske_ctx *c, void **graph_out) {
    if (!c || !graph_out) return SKE_EINVAL;
    *graph_out = nullptr;
    hipGraph_t g = nullptr;
    c->capturing = false;
    scratch_set_recording(c->scratch, false);
    hipError_t e = hipStreamEndCapture(c->st, &g);
    hipGraphExec_t ge = nullptr;
    const char *what = "hipStreamEndCapture";
    if (e == hipSuccess) {
        what = "hipGraphInstantiate";
        e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
    }
    if (e == hipSuccess) {
        what = "hipGraphUpload";
        e = hipGraphUpload(ge, c->st);
        if (e == hipSuccess) e = hipStreamSynchronize(c->st);
        if (e != hipSuccess) (void)hipGraphExecDestroy(ge);
    }
    if (e != hipSuccess) {
        // no graph holds what this capture pinned
        if (c->live_graphs == 0) scratch_unpin(c->scratch);
        c->last_hip = std::string(what) + ": " + hipGetErrorString(e);
        return SKE_EHIP;
    }
    *graph_out = ge;
    c->graph_users[(void *)ge] = c->cap_users;
    c->live_graphs++;  // the slots it pinned stay pinned until every graph is freed
    return SKE_OK;
}

int ske_graph_launch(ske_ctx *c, void *graph) {
    if (!c || !graph) return SKE_EINVAL;
    // a direct scratch use on another stream before the replay
    for (ScratchUse *u : {&c->xr, &c->rt})
        if (u->done && u->stream && u->stream != c->st && u->cap == 0) {
            bool covered = false;
            const int rc = xr_flush(c, *u, &covered);
            if (rc) return rc;
            if (covered) HIPCHK(c, hipStreamWaitEvent(c->st, u->done, 0));
        }
    HIPCHK(c, hipGraphLaunch(hipGraphExec_t(graph), c->st));
    // a replay may hold scratch users (the partitioned / XCD-partitioned K1,
    // routing): a later direct launch on another stream waits for it.  Only
    // the users the graph recorded are marked (a graph of unknown origin:
    // both).  Two replays of graphs holding scratch users on different
    // streams are not ordered by this; replay such graphs on one stream.
    const auto gu = c->graph_users.find(graph);
    const unsigned users = gu == c->graph_users.end() ? 3u : gu->second;
    for (ScratchUse *u : {&c->xr, &c->rt})
        if (u->done && (users & (u == &c->rt ? 2u : 1u))) {
            HIPCHK(c, hipEventRecord(u->done, c->st));
            u->stream = c->st;
            u->cap = 0;
            u->pending = false;
        }
    return SKE_OK;
}

int ske_graph_free(ske_ctx *c, void *graph) {
    if (!c) return SKE_EINVAL;
    if (graph) {
        HIPCHK(c, hipGraphExecDestroy(hipGraphExec_t(graph)));
        c->graph_users.erase(graph);
        if (c->live_graphs > 0) c->live_graphs--;
        if (c->live_graphs == 0 && !c->capturing) scratch_unpin(c->scratch);
    }
    return SKE_OK;
}

// ------------------------------------------------------------------ generator
int ske_gen_id_width(const ske_gen_params_t *p) {
    if (!p || p->id_hi <= p->id_lo) return SKE_EINVAL;
    uint64_t x = p->id_hi - 1;
    int w = 1;
    while (x >= 10) {
        x /= 10;
        w++;
    }
    return w;
}

static int gen_dev(const ske_gen_params_t *p, GenDev *g) {
    const int w = ske_gen_id_width(p);
    if (w < 1 || w > 19) return SKE_EINVAL;
    uint64_t p10 = 1;
    for (int i = 0; i < 20; i++) {
        g->pow10[i] = p10;
        if (i < 19) p10 *= 10;
    }
    if (p->id_lo < g->pow10[w - 1]) return SKE_EINVAL;  // all IDs share the digit count
    const uint64_t R = p->id_hi - p->id_lo;
    if (R >= (uint64_t(1) << 32) || p->n_members == 0 || p->n_members > R) return SKE_EINVAL;
    if (p->perm_mul % R == 0 || (unsigned __int128)(p->perm_mul % R) * (p->perm_mul_inv % R) % R != 1 % R)
        return SKE_EINVAL;
    if (p->n_keys == 0) return SKE_EINVAL;
    g->seed = p->seed;
    g->lo = p->id_lo;
    g->R = R;
    g->N = p->n_members;
    g->mul = p->perm_mul % R;
    g->add = p->perm_add % R;
    g->inv = p->perm_mul_inv % R;
    g->inv_thr = p->invalid_thresh;
    g->near_thr = p->near_thresh;
    g->n_keys = p->n_keys;
    g->slot_base = p->slot_base;
    g->width = uint32_t(w);
    g->key_cdf = p->key_cdf;
    return SKE_OK;
}

int ske_gen_members(ske_ctx *c, const ske_gen_params_t *p, uint64_t start, uint64_t n,
                    uint8_t *bytes_dev, uint32_t *offs_dev) {
    if (!c || !p || !bytes_dev || !offs_dev) return SKE_EINVAL;
    GenDev g{};
    int rc = gen_dev(p, &g);
    if (rc) return rc;
    if (start + n > g.N || n * g.width >= 0xffffffffull) return SKE_EINVAL;
    HIPCHK(c, launch_gen_members(g, start, n, bytes_dev, offs_dev, c->cus, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

int ske_gen_swipes(ske_ctx *c, const ske_gen_params_t *p, uint64_t start, uint64_t n,
                   uint8_t *bytes_dev, uint32_t *offs_dev, uint32_t *slot_dev) {
    if (!c || !p || !bytes_dev || !offs_dev || !slot_dev) return SKE_EINVAL;
    GenDev g{};
    int rc = gen_dev(p, &g);
    if (rc) return rc;
    if (n * g.width >= 0xffffffffull) return SKE_EINVAL;
    HIPCHK(c, launch_gen_swipes(g, start, n, bytes_dev, offs_dev, slot_dev, c->cus, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return SKE_OK;
}

}  // extern "C"
