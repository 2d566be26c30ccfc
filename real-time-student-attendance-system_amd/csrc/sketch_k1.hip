// sketch_k1.hip -- K1 for Bloom chains that fit one CU's LDS (C1/C2/C4: the
// 137 848 B RESERVE 0.01 / 1e5 filter, the reference's 4-link default chain).
//
// Same answers as k_swipes (sketch_kernels.hip): per swipe, BF.EXISTS
// (SBChain_Check: links newest -> oldest, each "present" iff all k probe bits
// are set, probes in RedisBloom's order (a + i*b) mod 2^64 mod bits) and, if
// present, PFADD (hllPatLen -> register max) -- attendance_processor.py:109-113
// and :127-129.  What differs is how it is laid out for gfx950, measured on
// C2 (1M swipes per launch): the launch is VALU-issue bound at the margin and
// carries a fixed per-launch cost, so this variant
//   - issues the LDS image copy (LDS-DMA, one 1 KiB piece per wave-instruction,
//     a compile-time count per wave) right after the first tile's loads and
//     hashes that tile while the copy lands -- the hashing no longer waits for
//     the image;
//   - loads an id of at most 8 bytes branch-free: the one or two aligned
//     64-bit words that hold it (an empty id reads a 16-byte zero buffer), a
//     funnel shift and a length mask;
//   - hashes MurmurHash64A of a short id in closed form: h = ((seed ^ len*m) ^
//     t) * m then the finaliser, t = the id word (len < 8) or its mixed block
//     (len == 8, mixed once for all three hashes);
//   - walks the probes with the precomputed-increment 32-bit walk
//     (ProbeWalk32) and reads the image with ds_read_u8;
//   - keeps 32-bit swipe indices (n < 2^31; the host falls back otherwise).
// Ids longer than 8 bytes are hashed by the generic routines (murmur_item) on a
// wave-uniform branch that short-id batches never take.
#include "sketch_common.h"
#include "sketch_internal.h"

namespace ske {

// cache policy of the swipe streams (read or written once): SKE_K1_NT bits --
// 1 offsets and slots, 2 id words, 4 answers -- take `nt`.  Off: at C2 the
// persistent kernel was 1-4 % slower with bits 3 or 7 (A/B, two alternations)
#ifndef SKE_K1_NT
#define SKE_K1_NT 0
#endif
template <int BIT> __device__ __forceinline__ constexpr int k1_aux() { return (SKE_K1_NT & BIT) ? 2 : 0; }
// SKE_K1_ABLATE (diagnostic builds only, registers may be wrong): 1 a raise is a
// plain byte store instead of the CAS (prices the atomics' round trips), 2 the
// CAS issued without using its return value (no settle)
#ifndef SKE_K1_ABLATE
#define SKE_K1_ABLATE 0
#endif

constexpr uint32_t kK1Block = 1024;     // threads per block, one block per CU
constexpr uint32_t kK1Waves = kK1Block / 64;
constexpr int kK1MaxPieces = 10;        // 1 KiB LDS pieces per wave (152 KiB / 16 waves)

typedef __attribute__((address_space(3))) uint8_t lds_u8;  // an LDS byte

// Diagnostic phase stamps (tools/stamps, built only with -DSKE_STAMPS; the
// product library has none): lane 0 of every wave records s_memtime at fixed
// points of its first two tiles into a side buffer no output depends on.
#ifdef SKE_STAMPS
__device__ unsigned long long *ske_k1_stamp_buf;
hipError_t set_k1_stamp_buffer(void *p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(ske_k1_stamp_buf), &p, sizeof(void *));
}
#define K1_STAMP(k)                                                                                \
    do {                                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                                         \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                \
        __builtin_amdgcn_sched_barrier(0);                                                         \
        if ((threadIdx.x & 63) == 0 && (k) < 16)                                                   \
            ske_k1_stamp_buf[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 16 + (k)] = t_;              \
    } while (0)
#else
#define K1_STAMP(k) \
    do {            \
    } while (0)
#endif

__device__ __forceinline__ uint64_t mul_m(uint64_t x) { return x * kMurmurM; }

// Copy this wave's P pieces of the LDS image: piece p of the flat piece list
// (links newest first, each padded to whole 1 KiB pieces) lands at img + p*1024.
// Pieces past the end repeat the last one (same bytes, same place), so every
// wave issues exactly P LDS-DMA instructions and the compiler can wait for the
// tile's own loads with vmcnt(P) while the image is still in flight.  Bytes past
// a link's 16-byte-padded end read as zero (buffer range check).
template <int P>
__device__ __forceinline__ void k1_stage(const K1Args &A, lds_u8 *img, uint32_t wave, uint32_t lane,
                                         const __amdgpu_buffer_rsrc_t &r0) {
    if (A.nlinks == 1) {
        // one link (every RESERVEd filter that has not grown): r0, set up at
        // kernel entry, covers every piece -- no per-piece descriptor loads
#pragma unroll
        for (int j = 0; j < P; j++) {
            uint32_t p = wave + kK1Waves * uint32_t(j);
            p = p < A.npieces ? p : A.npieces - 1;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                r0, (__attribute__((address_space(3))) void *)(img + p * 1024), 16,
                int(p * 1024 + lane * 16), 0, 0, 0);
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < P; j++) {
        uint32_t p = wave + kK1Waves * uint32_t(j);
        p = p < A.npieces ? p : A.npieces - 1;
        uint32_t l = A.nlinks - 1;  // pieces run newest link first
        while (l > 0 && p >= A.link[l - 1].piece0) l--;
        const K1Link &L = A.link[l];
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(L.bf), 0, int(L.nbytes16), 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            r, (__attribute__((address_space(3))) void *)(img + p * 1024), 16,
            int((p - L.piece0) * 1024 + lane * 16), 0, 0, 0);
    }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t k1_rsrc(const void *p, uint32_t nbytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, int(nbytes), 0x00020000);
}

// Probe rounds of one link for U swipes in lock step.  Every swipe keeps
// RedisBloom's sequential order: `alive` drops at its first unset bit and a
// dead swipe's later probes are ignored (the bit array is read-only, so the
// answer and the register updates are exactly the sequential ones).  The
// rounds carry no wave-level exit: at 90 % members nearly every wave needs
// all k rounds, and the exit test costs more than the rounds it saves.
// kTop: the newest link, placed at LDS offset 0.
template <int U, bool kTop>
__device__ __forceinline__ void k1_probe_link(const K1Link &L, const lds_u8 *img, ProbeWalk32 *wk,
                                              uint32_t *alive) {
    const lds_u8 *limg = kTop ? img : img + L.piece0 * 1024;
    const uint32_t d = L.d;
#pragma unroll 4
    for (uint32_t j = 0; j < L.k; j++) {
        uint32_t byte[U];
#pragma unroll
        for (int u = 0; u < U; u++) byte[u] = limg[wk[u].x >> 3];
#pragma unroll
        for (int u = 0; u < U; u++) {
            alive[u] &= __builtin_amdgcn_ubfe(byte[u], wk[u].x & 7, 1);
            // x_{j+1}: the 64-bit running sum's carry selects the increment
            unsigned c1, c2;
            const uint32_t lo = __builtin_addc(uint32_t(wk[u].v), uint32_t(wk[u].b), 0u, &c1);
            const uint32_t hi = __builtin_addc(uint32_t(wk[u].v >> 32), uint32_t(wk[u].b >> 32), c1, &c2);
            wk[u].v = (uint64_t(hi) << 32) | lo;
            const uint32_t xn = wk[u].x + (c2 ? wk[u].inc1 : wk[u].inc0);
            wk[u].x = umin32(xn, xn - d);
        }
    }
}

// A tile: U swipes per thread (swipe base + u*1024 + tid).  The block runs
// its tiles as a two-stage software pipeline: the next tile's offsets and key
// slots are loaded while the current tile probes, its id words while the
// current tile updates registers, so no tile but the first waits for HBM.
// Loads of a tile past the block's chunk are still issued (clamped to the last
// swipe: one cache line) so that the number of memory operations in flight
// does not depend on the branch taken, and the compiler's waits stay exact.
template <int U>
struct K1In {  // a tile's loads in flight
    uint32_t idx[U], b[U], e[U], sl[U];
    bool act[U];
    uint64_t w0[U], w1[U];
};

template <int U>
struct K1Hot {  // a hashed tile
    uint32_t idx[U], sl[U], rank[U], cur[U], sh[U];
    bool act[U];
    uint64_t ha[U], hb[U];
    uint32_t *w[U];  // the aligned word holding the swipe's register
    ProbeWalk32 wk[U];
};

template <int U>
struct K1Pend {  // a committed tile's register CASes, settled one tile later
    uint32_t *w[U];
    uint32_t exp[U], prev[U], rank[U], sh[U];
    bool on[U];
};

// One batch as the tile loop sees it: 32-bit offsets into its buffers
// (u32 offsets keep the ids below 4 GiB) and its answer array.
struct K1View {
    __amdgpu_buffer_rsrc_t offs, slot, bytes;
    const uint8_t *bytes_p;
    const uint32_t *offs_p;  // nullptr: fixed-width ids
    uint8_t *out;            // may be nullptr
    uint32_t n, fixed_w;
};

__device__ __forceinline__ K1View k1_view(const uint8_t *bytes, const uint32_t *offs, const uint32_t *slot,
                                          uint8_t *out, uint32_t n, uint32_t fixed_w) {
    K1View V;
    V.offs = k1_rsrc(offs, 0xfffffff0u);
    V.slot = k1_rsrc(slot, 0xfffffff0u);
    V.bytes = k1_rsrc(bytes, 0xfffffff0u);
    V.bytes_p = bytes;
    V.offs_p = offs;
    V.out = out;
    V.n = n;
    V.fixed_w = fixed_w;
    return V;
}

template <bool kHll, int U>
__device__ __forceinline__ void k1_issue_a(const K1View &V, uint32_t base, uint32_t c1, K1In<U> &in) {
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint32_t i = base + uint32_t(u) * kK1Block + threadIdx.x;
        in.act[u] = i < c1;
        in.idx[u] = i;
        const uint32_t ic = in.act[u] ? i : V.n - 1;  // clamped: every load stays in bounds
        if (V.offs_p) {
            in.b[u] = __builtin_amdgcn_raw_buffer_load_b32(V.offs, ic * 4, 0, k1_aux<1>());
            in.e[u] = __builtin_amdgcn_raw_buffer_load_b32(V.offs, ic * 4 + 4, 0, k1_aux<1>());
        } else {
            in.b[u] = ic * V.fixed_w;
            in.e[u] = in.b[u] + V.fixed_w;
        }
        in.sl[u] = kHll ? __builtin_amdgcn_raw_buffer_load_b32(V.slot, ic * 4, 0, k1_aux<1>()) : 0u;
    }
}

template <int U>
__device__ __forceinline__ void k1_issue_b(const K1View &R, K1In<U> &in) {
#pragma unroll
    for (int u = 0; u < U; u++) {
        // an empty id reads past the range (zero); a second word only when the
        // id crosses an 8-byte boundary (else the first word again)
        const uint32_t len = in.e[u] - in.b[u], s8 = in.b[u] & 7;
        const uint32_t o0 = len ? (in.b[u] & ~7u) : 0xfffffff8u;
        const uint32_t o1 = (s8 + len > 8 && len <= 8) ? o0 + 8 : o0;
        in.w0[u] = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(R.bytes, o0, 0, k1_aux<2>()));
        in.w1[u] = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(R.bytes, o1, 0, k1_aux<2>()));
    }
}

// hashes (a = H(x, bloom seed), b = H(x, a), h = H(x, hll seed)), the HLL
// register and rank with its pre-check load, and the newest link's walk
template <bool kHll, int U>
__device__ __forceinline__ void k1_hash(const K1Args &A, const K1View &V, const K1In<U> &in, K1Hot<U> &h) {
    uint32_t len[U];
    uint64_t hh[U];
    bool long_ids = false;
#pragma unroll
    for (int u = 0; u < U; u++) {
        len[u] = in.e[u] - in.b[u];
        h.idx[u] = in.idx[u];
        h.act[u] = in.act[u];
        h.sl[u] = in.sl[u];
        long_ids |= in.act[u] && len[u] > 8;
    }
    if (__any(long_ids)) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = in.act[u] ? in.idx[u] : V.n - 1;
            const uint32_t b = V.offs_p ? V.offs_p[i] : i * V.fixed_w;
            const Item it = load_item(V.bytes_p, b, b + len[u]);
            h.ha[u] = murmur_item(it, kBloomSeed);
            h.hb[u] = murmur_item(it, h.ha[u]);
            hh[u] = kHll ? murmur_item(it, kHllSeed) : 0;
        }
    } else {
        uint64_t tw[U];
        bool any8 = false;
#pragma unroll
        for (int u = 0; u < U; u++) {
            // bytes s8 .. s8+len-1 of w1:w0, then only the low len bytes kept
            // (len == 0 never reads t below)
            const uint32_t sh = (in.b[u] & 7) * 8;
            const bool hi = sh >= 32;
            const uint32_t a = hi ? uint32_t(in.w0[u] >> 32) : uint32_t(in.w0[u]);
            const uint32_t bb = hi ? uint32_t(in.w1[u]) : uint32_t(in.w0[u] >> 32);
            const uint32_t c = hi ? uint32_t(in.w1[u] >> 32) : uint32_t(in.w1[u]);
            const uint64_t v = (uint64_t(__builtin_amdgcn_alignbit(c, bb, sh & 31)) << 32) |
                               __builtin_amdgcn_alignbit(bb, a, sh & 31);
            const uint32_t drop = (64 - len[u] * 8) & 63;
            tw[u] = (v << drop) >> drop;
            any8 |= len[u] == 8;
        }
        if (__any(any8)) {
#pragma unroll
            for (int u = 0; u < U; u++) {
                uint64_t k = mul_m(tw[u]);
                k ^= k >> 47;
                k = mul_m(k);
                tw[u] = len[u] == 8 ? k : tw[u];
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t t = tw[u] ^ (uint64_t(len[u]) * kMurmurM);
            const bool nz = len[u] != 0;
            h.ha[u] = mm_final(nz ? mul_m(kBloomSeed ^ t) : kBloomSeed);
            h.hb[u] = mm_final(nz ? mul_m(h.ha[u] ^ t) : h.ha[u]);
            if (kHll) hh[u] = mm_final(nz ? mul_m(kHllSeed ^ t) : kHllSeed);
        }
    }
    if constexpr (kHll) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            uint32_t ridx;
            hll_patlen(hh[u], ridx, h.rank[u]);
            const bool ok = in.act[u] && in.sl[u] < A.nslots;
            uint8_t *reg = ok ? A.regs + (uint64_t(in.sl[u]) << kHllP) + (ridx & ~3u)
                              : const_cast<uint8_t *>(A.zero16);
            h.w[u] = reinterpret_cast<uint32_t *>(reg);
            h.sh[u] = (ridx & 3) * 8;
        }
        // the pre-check load of the register's word flies over the probes; it
        // is also the expected value of the CAS that raises the register
#pragma unroll
        for (int u = 0; u < U; u++) h.cur[u] = *h.w[u];
    }
    const K1Link &L = A.link[A.nlinks - 1];
    const Divisor D{L.d, L.m, L.t, L.sh, 0};
#pragma unroll
    for (int u = 0; u < U; u++) h.wk[u].init(h.ha[u], h.hb[u], D);
}

// Bloom: newest link first, stop at the first link that has the id
template <int U>
__device__ __forceinline__ void k1_probe(const K1Args &A, const lds_u8 *img, K1Hot<U> &h,
                                         uint32_t *valid) {
    const int top = int(A.nlinks) - 1;
    uint32_t alive[U];
#pragma unroll
    for (int u = 0; u < U; u++) alive[u] = h.act[u];
    k1_probe_link<U, true>(A.link[top], img, h.wk, alive);
#pragma unroll
    for (int u = 0; u < U; u++) valid[u] = alive[u];
    for (int l = top - 1; l >= 0; --l) {
        bool any = false;
#pragma unroll
        for (int u = 0; u < U; u++) {
            alive[u] = h.act[u] && !valid[u];
            any |= alive[u] != 0;
        }
        if (!__any(any)) break;
        const K1Link &L = A.link[l];
        const Divisor D{L.d, L.m, L.t, L.sh, 0};
#pragma unroll
        for (int u = 0; u < U; u++) h.wk[u].init(h.ha[u], h.hb[u], D);
        k1_probe_link<U, false>(L, img, h.wk, alive);
#pragma unroll
        for (int u = 0; u < U; u++) valid[u] |= alive[u];
    }
}

// PFADD of the valid swipes, answers.  A register below the swipe's rank is
// raised by one CAS whose expected value is the pre-check word: it is issued
// here and its result is looked at one tile later (k1_settle), after the next
// tile's hash and probes, so the atomic's round trip to memory is hidden.
// The pre-check may be stale, never too high (registers only grow): a stale
// word makes the CAS fail, and k1_settle finishes the byte max in a loop.
template <bool kHll, int U>
__device__ __forceinline__ void k1_commit(const K1Args &A, const K1View &V, const K1Hot<U> &h,
                                          const uint32_t *valid, K1Pend<U> &pd) {
    if constexpr (kHll) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const bool slot_ok = h.sl[u] < A.nslots;
            if (valid[u] && !slot_ok) atomicOr(A.err, 1u);
            const bool need = valid[u] && slot_ok && ((h.cur[u] >> h.sh[u]) & 0xffu) < h.rank[u];
            pd.on[u] = need;
            pd.w[u] = h.w[u];
            pd.exp[u] = h.cur[u];
            pd.prev[u] = h.cur[u];
            pd.rank[u] = h.rank[u];
            pd.sh[u] = h.sh[u];
            if constexpr ((SKE_K1_ABLATE & 1) != 0) {
                if (need) reinterpret_cast<uint8_t *>(h.w[u])[h.sh[u] >> 3] = uint8_t(h.rank[u]);
            } else if constexpr ((SKE_K1_ABLATE & 2) != 0) {  // the CAS without its return (no settle)
                if (need) (void)atomicCAS(h.w[u], h.cur[u], (h.cur[u] & ~(0xffu << h.sh[u])) | (h.rank[u] << h.sh[u]));
            } else if (need) {
                pd.prev[u] = atomicCAS(h.w[u], h.cur[u],
                                       (h.cur[u] & ~(0xffu << h.sh[u])) | (h.rank[u] << h.sh[u]));
            }
        }
    }
    if (V.out) {
        const __amdgpu_buffer_rsrc_t r_out = k1_rsrc(V.out, V.n);
#pragma unroll
        for (int u = 0; u < U; u++)  // lanes past the chunk store out of range (dropped)
            __builtin_amdgcn_raw_buffer_store_b8(uint8_t(valid[u]), r_out, h.act[u] ? h.idx[u] : 0xffffffffu,
                                                 0, k1_aux<4>());
    }
}

template <bool kHll, int U>
__device__ __forceinline__ void k1_settle(K1Pend<U> &pd) {
    if constexpr (kHll) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (!pd.on[u] || pd.prev[u] == pd.exp[u]) continue;
            const uint32_t sh = pd.sh[u], rank = pd.rank[u];
            uint32_t old = pd.prev[u];
            while (((old >> sh) & 0xffu) < rank) {
                const uint32_t p = atomicCAS(pd.w[u], old, (old & ~(0xffu << sh)) | (rank << sh));
                if (p == old) break;
                old = p;
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) pd.on[u] = false;
    }
}

// Each block owns one contiguous chunk of the batch.  Its first tile is
// loaded, the LDS image copy issued behind it (P LDS-DMA pieces per wave) and
// the tile hashed while the copy lands; then the pipelined tile loop.  A block
// without swipes still stages and joins the barrier.
template <bool kHll, int U, int P>
__global__ void __launch_bounds__(kK1Block) k_swipes_lds(const K1Args A) {
    // a static image (not dynamic LDS): its address folds to 0 in the probe
    // address arithmetic (one VALU op per probe less)
    __shared__ __attribute__((aligned(16))) uint8_t img_[kLdsBloomMaxBytes];
    lds_u8 *img = (lds_u8 *)img_;
    const uint32_t per_block = (A.n + gridDim.x - 1) / gridDim.x;
    const uint32_t c0 = blockIdx.x * per_block;
    const uint32_t c1 = c0 + per_block < A.n ? c0 + per_block : A.n;
    const K1View V = k1_view(A.bytes, A.offs, A.slot, A.out, A.n, A.fixed_w);
    K1In<U> in;
    K1Hot<U> hot;
    K1_STAMP(0);
    // the tile's offset / slot loads first, then the image copy behind them,
    // then the id-word loads (which need the offsets): the id loads and the
    // hash wait for their own loads only (vmcnt(P)) while the P pieces land.
    // (Copy first, loads behind: measured 3 % slower at 524k swipes.)
    const K1Link &L0 = A.link[A.nlinks - 1];  // the newest link: LDS offset 0
    const __amdgpu_buffer_rsrc_t r0 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(L0.bf), 0, int(L0.nbytes16), 0x00020000);
    k1_issue_a<kHll, U>(V, c0, c1, in);
    __builtin_amdgcn_sched_barrier(0);
    k1_stage<P>(A, img, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), threadIdx.x & 63, r0);
    __builtin_amdgcn_sched_barrier(0);
    k1_issue_b<U>(V, in);  // waits for the offsets only (vmcnt(P): the copy is younger)
    K1_STAMP(1);
    k1_hash<kHll, U>(A, V, in, hot);
    K1_STAMP(2);
    __syncthreads();  // the image has landed
    K1_STAMP(3);
    [[maybe_unused]] int it = 0;  // stamp index only
    K1Pend<U> pend;
#pragma unroll
    for (int u = 0; u < U; u++) pend.on[u] = false;
    for (uint32_t base = c0;; it++) {
        const uint32_t next = base + kK1Block * U;
        const bool more = next < c1;  // block-uniform
        k1_issue_a<kHll, U>(V, next, c1, in);
        uint32_t valid[U];
        k1_probe<U>(A, img, hot, valid);
        K1_STAMP(4 + 3 * it);
        k1_issue_b<U>(V, in);
        k1_settle<kHll, U>(pend);  // the previous tile's CASes (landed during this tile)
        k1_commit<kHll, U>(A, V, hot, valid, pend);
        K1_STAMP(5 + 3 * it);
        if (!more) break;
        k1_hash<kHll, U>(A, V, in, hot);
        K1_STAMP(6 + 3 * it);
        base = next;
    }
    k1_settle<kHll, U>(pend);
    K1_STAMP(15);
}

// Many batches in one launch (ske_swipes_many_async): the batches are cut into
// tiles of 1024*U swipes (a batch's last tile is partial; no tile spans two
// batches), the concatenated tile list is dealt to the blocks in contiguous
// equal shares, and each block stages the LDS image once and runs the same
// pipelined tile loop across its share, switching batch views (wave-uniform,
// from the kernel arguments) at batch boundaries.  One launch per call: the
// per-launch fixed cost -- the image copy, the first tile's loads, the grid
// ramp and drain -- is paid once for all the call's batches.
template <bool kHll, int U, int P>
__global__ void __launch_bounds__(kK1Block) k_swipes_lds_many(const K1Args A, const K1Many M) {
    __shared__ __attribute__((aligned(16))) uint8_t img_[kLdsBloomMaxBytes];
    lds_u8 *img = (lds_u8 *)img_;
    constexpr uint32_t T = kK1Block * U;
    const uint32_t ntiles = M.tpre[M.nb];
    uint32_t t = uint32_t(uint64_t(ntiles) * blockIdx.x / gridDim.x);
    const uint32_t tend = uint32_t(uint64_t(ntiles) * (blockIdx.x + 1) / gridDim.x);
    // batch of tile t (the block's tiles only move forward)
    uint32_t j = 0;
    while (j + 1 < M.nb && t >= M.tpre[j + 1]) j++;
    auto view = [&](uint32_t jj) {
        const K1Batch &B = M.b[jj];
        return k1_view(B.bytes, B.offs, B.slot, B.out, B.n, B.fixed_w);
    };
    K1View Vn = view(j);
    K1In<U> in;
    K1Hot<U> hot;
    const K1Link &L0 = A.link[A.nlinks - 1];
    const __amdgpu_buffer_rsrc_t r0 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(L0.bf), 0, int(L0.nbytes16), 0x00020000);
    const bool any = t < tend;  // block-uniform
    if (any) k1_issue_a<kHll, U>(Vn, (t - M.tpre[j]) * T, Vn.n, in);
    __builtin_amdgcn_sched_barrier(0);
    k1_stage<P>(A, img, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), threadIdx.x & 63, r0);
    __builtin_amdgcn_sched_barrier(0);
    if (any) {
        k1_issue_b<U>(Vn, in);
        k1_hash<kHll, U>(A, Vn, in, hot);
    }
    __syncthreads();  // the image has landed
    if (!any) return;
    K1Pend<U> pend;
#pragma unroll
    for (int u = 0; u < U; u++) pend.on[u] = false;
    K1View Vh = Vn;
    for (;;) {
        const bool more = t + 1 < tend;  // block-uniform
        if (more) {
            t++;
            if (t >= M.tpre[j + 1]) {
                while (t >= M.tpre[j + 1]) j++;  // (skips empty batches)
                Vn = view(j);
            }
            k1_issue_a<kHll, U>(Vn, (t - M.tpre[j]) * T, Vn.n, in);
        }
        uint32_t valid[U];
        k1_probe<U>(A, img, hot, valid);
        if (more) k1_issue_b<U>(Vn, in);
        k1_settle<kHll, U>(pend);
        k1_commit<kHll, U>(A, Vh, hot, valid, pend);
        if (!more) break;
        k1_hash<kHll, U>(A, Vn, in, hot);
        Vh = Vn;
    }
    k1_settle<kHll, U>(pend);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
bool k1_lds_plan(const ChainDev &ch, K1Args *A) {
    if (ch.nlinks < 1 || ch.nlinks > kK1MaxLinks) return false;
    uint32_t pieces = 0;
    for (int l = ch.nlinks - 1; l >= 0; l--) {  // the newest link (probed first) at LDS offset 0
        const LinkDev &L = ch.link[l];
        if (L.div.d > (uint64_t(1) << 31) || L.div.d < 64) return false;
        const uint64_t nb16 = (((L.div.d >> 3) + 15) >> 4) << 4;
        K1Link &K = A->link[l];
        K.bf = L.bf;
        K.m = L.div.m;
        K.d = uint32_t(L.div.d);
        K.t = uint32_t(L.div.t);
        K.sh = L.div.sh;
        K.k = L.k;
        K.nbytes16 = uint32_t(nb16);
        K.piece0 = pieces;
        pieces += uint32_t((nb16 + 1023) / 1024);
    }
    if (pieces * 1024 > lds_bloom_max() || pieces > kK1Waves * kK1MaxPieces) return false;
    A->nlinks = uint32_t(ch.nlinks);
    A->npieces = pieces;
    return true;
}

template <bool kHll, int U>
static hipError_t k1_launch_p(const K1Args &A, unsigned grid, hipStream_t st) {
    const int P = int((A.npieces + kK1Waves - 1) / kK1Waves);
#define SKE_P(PP)                                                                                  \
    case PP:                                                                                       \
        hipLaunchKernelGGL((k_swipes_lds<kHll, U, PP>), dim3(grid), dim3(kK1Block), 0, st, A);     \
        break;
    switch (P) {
        SKE_P(1) SKE_P(2) SKE_P(3) SKE_P(4) SKE_P(5) SKE_P(6) SKE_P(7) SKE_P(8) SKE_P(9) SKE_P(10)
    default: return hipErrorInvalidValue;
    }
#undef SKE_P
    return hipGetLastError();
}

hipError_t launch_swipes_lds(const K1Args &A, bool hll, int tile, int cus, hipStream_t st) {
    if (A.n == 0) return hipSuccess;
    const int U = tile >= 4 ? 4 : (tile >= 2 ? 2 : 1);
    uint64_t g = (uint64_t(A.n) + uint64_t(kK1Block) * U - 1) / (uint64_t(kK1Block) * U);
    const unsigned grid = unsigned(g < uint64_t(cus) ? (g ? g : 1) : uint64_t(cus));
    if (hll) {
        if (U == 4) return k1_launch_p<true, 4>(A, grid, st);
        if (U == 2) return k1_launch_p<true, 2>(A, grid, st);
        return k1_launch_p<true, 1>(A, grid, st);
    }
    if (U == 4) return k1_launch_p<false, 4>(A, grid, st);
    if (U == 2) return k1_launch_p<false, 2>(A, grid, st);
    return k1_launch_p<false, 1>(A, grid, st);
}

template <bool kHll, int U>
static hipError_t k1_launch_many_p(const K1Args &A, const K1Many &M, unsigned grid, hipStream_t st) {
    const int P = int((A.npieces + kK1Waves - 1) / kK1Waves);
#define SKE_P(PP)                                                                                   \
    case PP:                                                                                        \
        hipLaunchKernelGGL((k_swipes_lds_many<kHll, U, PP>), dim3(grid), dim3(kK1Block), 0, st, A, M); \
        break;
    switch (P) {
        SKE_P(1) SKE_P(2) SKE_P(3) SKE_P(4) SKE_P(5) SKE_P(6) SKE_P(7) SKE_P(8) SKE_P(9) SKE_P(10)
    default: return hipErrorInvalidValue;
    }
#undef SKE_P
    return hipGetLastError();
}

uint32_t k1_many_tile(int tile) { return kK1Block * uint32_t(tile >= 4 ? 4 : (tile >= 2 ? 2 : 1)); }

hipError_t launch_swipes_lds_many(const K1Args &A, const K1Many &M, int tile, int cus, hipStream_t st) {
    if (M.nb == 0 || M.tpre[M.nb] == 0) return hipSuccess;
    const int U = tile >= 4 ? 4 : (tile >= 2 ? 2 : 1);
    const uint32_t nt = M.tpre[M.nb];
    const unsigned grid = unsigned(nt < uint32_t(cus) ? nt : uint32_t(cus));
    if (U == 4) return k1_launch_many_p<true, 4>(A, M, grid, st);
    if (U == 2) return k1_launch_many_p<true, 2>(A, M, grid, st);
    return k1_launch_many_p<true, 1>(A, M, grid, st);
}

hipError_t k1_lds_setup() { return hipSuccess; }  // static LDS: nothing to raise

}  // namespace ske
