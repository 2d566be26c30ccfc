// sketch_kernels.hip -- gfx950 kernels of the validate-and-count hot path.
//
//  K1  k_swipes      fused BF.EXISTS (SBChain_Check newest->oldest) + valid-gated
//                    PFADD (hllPatLen + register max) per swipe
//                    (attendance_processor.py:109-113 + :127-129)
//  K1e k_swipes<Exists>   BF.MEXISTS only (attendance_processor.py:109, :78)
//  K1s k_swipes<Stats>    probe statistics for the roofline (untimed)
//      k_pfadd       PFADD of (slot, element) pairs without reply flags
//  K2  k_pfcount     per-group register max-merge + 64-bin histogram + Ertl
//                    estimator (hllCount) on device (attendance_processor.py:152)
//  K3  k_pfmerge     PFMERGE register max
//      k_dense       HLL_DENSE_SET_REGISTER packing for export
//      k_gen_*       counter-based synthetic stream (DESIGN.md "Synthetic workload")
//
// Data layout in HBM: Bloom links are RedisBloom's own LSB-first bit arrays
// (bit x at byte x>>3, mask 1<<(x&7)); HLL keys are 16384-byte slabs, one
// byte per register (Redis HLL_RAW view), key s at regs + s*16384.
#include "sketch_common.h"
#include "sketch_internal.h"

namespace ske {

// Byte max into a register slab.  There is no byte atomic max, so the byte's
// aligned 32-bit word is updated with a CAS loop; the loop starts from a
// plain load, which may be stale but never too high (registers only grow).
__device__ __forceinline__ bool reg_max(uint8_t *reg, uint32_t rank) {
    const uint32_t b = uint32_t(reinterpret_cast<uintptr_t>(reg) & 3);
    uint32_t *w = reinterpret_cast<uint32_t *>(reg - b);
    const uint32_t sh = b * 8;
    uint32_t old = *w;
    bool changed = false;
    while (((old >> sh) & 0xffu) < rank) {
        uint32_t nw = (old & ~(0xffu << sh)) | (rank << sh);
        uint32_t prev = atomicCAS(w, old, nw);
        if (prev == old) {
            changed = true;
            break;
        }
        old = prev;
    }
    return changed;
}

enum SwipeMode { kModeSwipes = 0, kModeExists = 1, kModeStats = 2 };

// Diagnostic phase stamps (tools/stamps: built only with -DSKE_STAMPS; the
// product library has none).  Lane 0 of every wave records s_memtime at the
// phase boundaries of its first two tiles into a side buffer that no output
// depends on.
#ifdef SKE_STAMPS
__device__ unsigned long long *ske_stamp_buf;
hipError_t set_stamp_buffer(void *p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(ske_stamp_buf), &p, sizeof(void *));
}
#define SKE_STAMP(tile, k)                                                                         \
    do {                                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                                         \
        unsigned long long t_;                                                                     \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
        __builtin_amdgcn_sched_barrier(0);                                                         \
        if ((threadIdx.x & 63) == 0 && (tile) < 2)                                                 \
            ske_stamp_buf[((blockIdx.x * 16 + (threadIdx.x >> 6)) * 2 + (tile)) * 8 + (k)] = t_;   \
    } while (0)
#else
#define SKE_STAMP(tile, k) \
    do {                   \
    } while (0)
#endif

constexpr int kLdsBloomMax = kLdsBloomMaxBytes;

// Copy every link's bit array into the LDS image by LDS-DMA
// (global_load_lds_dwordx4: one wave-instruction moves 1 KiB straight into
// LDS, no VGPR round trip), every piece of the block in flight at once; the
// caller's __syncthreads() waits for them (vmcnt(0) + barrier).
__device__ __forceinline__ void stage_bloom(const ChainDev &ch, uint8_t *lds) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
    for (int l = 0; l < ch.nlinks; l++) {
        const LinkDev &L = ch.link[l];
        const uint32_t nbytes = uint32_t((((L.div.d >> 3) + 15) >> 4) << 4);  // 16-B padded link
        for (uint32_t piece = wave; piece * 1024 < nbytes; piece += nwaves) {
            const uint32_t off = piece * 1024 + lane * 16;
            if (off < nbytes)
                __builtin_amdgcn_global_load_lds(L.bf + off, lds + L.lds_off + piece * 1024, 16, 0, 0);
        }
    }
}

// Membership of U swipes in one link, advanced in lock step (round j issues
// the j-th probe of every swipe still undecided); Cursor is ProbeCursor32
// when bits <= 2^31, else the 64-bit ProbeCursor.
// LDS image, bits <= 2^31: branch-free rounds.  Every swipe of the tile reads
// its byte each round (a decided swipe re-reads a valid address and ignores
// it); the loop exit is wave-uniform (no lane has an undecided swipe left).
template <int U>
__device__ __forceinline__ void link_probe_lds32(const LinkDev &L, const uint8_t *lds,
                                                 const uint64_t *ha, const uint64_t *hb,
                                                 const bool *act, bool *valid, uint32_t &probes) {
    const uint32_t d = uint32_t(L.div.d);
    const uint8_t *img = lds + L.lds_off;
    ProbeWalk32 c[U];
    bool alive[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        alive[u] = act[u] && !valid[u];
        c[u].init(ha[u], hb[u], L.div);
    }
    for (uint32_t j = 0; j < L.k; j++) {
        uint32_t byte[U];
#pragma unroll
        for (int u = 0; u < U; u++) byte[u] = img[c[u].x >> 3];
        bool any = false;
#pragma unroll
        for (int u = 0; u < U; u++) {
            probes += alive[u];
            alive[u] = alive[u] && ((byte[u] >> (c[u].x & 7)) & 1);
            any |= alive[u];
            c[u].step(d);
        }
        if (!__any(any)) break;
    }
#pragma unroll
    for (int u = 0; u < U; u++) valid[u] |= alive[u];
}

template <bool kLds, int U, typename Cursor>
__device__ __forceinline__ void link_probe(const LinkDev &L, const uint8_t *lds, const uint64_t *ha,
                                           const uint64_t *hb, const bool *act, bool *valid,
                                           uint32_t &probes) {
    Cursor c[U];
    bool alive[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        alive[u] = act[u] && !valid[u];
        c[u].init(ha[u], hb[u], L.div);
    }
    for (uint32_t j = 0; j < L.k; j++) {
        uint8_t byte[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t x = c[u].x;
            byte[u] = alive[u] ? (kLds ? lds[L.lds_off + uint32_t(x >> 3)] : L.bf[x >> 3]) : uint8_t(0);
        }
        bool any = false;
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (alive[u]) {
                probes++;
                alive[u] = (byte[u] >> (c[u].x & 7)) & 1;
                c[u].step(L.div);
                any |= alive[u];
            }
        }
        if (!any) break;
    }
#pragma unroll
    for (int u = 0; u < U; u++) valid[u] |= alive[u];
}

// K1, tiled: every thread owns U swipes of a tile (swipe base + u*T + tid,
// so a wave's 64 lanes read 64 consecutive offsets / ids).  All loads of a
// tile are issued before any is consumed, and the Bloom test advances the U
// swipes in lock step -- round j issues the j-th probe of every swipe still
// undecided -- so each thread keeps U probe loads in flight while every swipe
// still follows RedisBloom's sequential order (newest link first, stop at the
// first unset bit; the probe count equals the CPU oracle's).  Each block
// works on one contiguous chunk of the batch.  LDS variant: the Bloom image
// is staged while the first tile's loads are in flight.
template <int kMode, bool kLds, int U>
__global__ void __launch_bounds__(kLds ? 1024 : 256)
    k_swipes(const ChainDev ch, const uint8_t *__restrict__ bytes,
             const uint32_t *__restrict__ offs, uint32_t fixed_w,
             const uint32_t *__restrict__ slot, uint64_t n, uint8_t *__restrict__ regs,
             uint32_t nslots, uint8_t *__restrict__ out, unsigned long long *__restrict__ stats) {
    // fixed_w > 0: ids are packed at a fixed width (id i at bytes + i*fixed_w,
    // offs unused) -- the id load then needs no offset load first
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_img[];
    const uint32_t T = blockDim.x, tid = threadIdx.x;
    const uint64_t per_block = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t c0 = uint64_t(blockIdx.x) * per_block;
    const uint64_t c1 = c0 + per_block < n ? c0 + per_block : n;
    bool staged = !kLds;
    uint32_t probes = 0, nvalid = 0;
    // a block with no work still joins the staging barrier below
    int tile_no = 0;
    SKE_STAMP(0, 0);
    for (uint64_t base = c0; base < c1 || !staged; base += uint64_t(T) * U, tile_no++) {
        SKE_STAMP(tile_no, 1);
        Item it[U];
        uint32_t sl[U];
        bool act[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t i = base + uint64_t(u) * T + tid;
            act[u] = i < c1;
            it[u].len = 0;
            sl[u] = 0;
            if (act[u]) {
                const uint64_t b = fixed_w ? i * fixed_w : offs[i];
                const uint64_t e = fixed_w ? b + fixed_w : offs[i + 1];
                it[u] = load_item(bytes, b, e);
                if (kMode == kModeSwipes) sl[u] = slot[i];
            }
        }
        if (!staged) {
            stage_bloom(ch, lds_img);
            __syncthreads();
            staged = true;
        }
        SKE_STAMP(tile_no, 2);
        // ids of at most 8 bytes (every config's decimal student id) take the
        // short MurmurHash64A path, chosen per wave
        bool short_ids = true;
#pragma unroll
        for (int u = 0; u < U; u++) short_ids &= it[u].len <= 8;
        short_ids = __all(short_ids);
        uint64_t ha[U], hb[U], hh[U];
        if (short_ids) {
#pragma unroll
            for (int u = 0; u < U; u++) {
                ha[u] = murmur_short(it[u].w0, it[u].len, kBloomSeed);
                hh[u] = murmur_short(it[u].w0, it[u].len, kHllSeed);
                hb[u] = murmur_short(it[u].w0, it[u].len, ha[u]);
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; u++) {
                ha[u] = murmur_item(it[u], kBloomSeed);
                hh[u] = murmur_item(it[u], kHllSeed);
                hb[u] = murmur_item(it[u], ha[u]);
            }
        }
        // HLL half, issued before the probes so its register pre-check loads
        // fly while the Bloom is tested (a swipe found invalid later simply
        // discards them).  hllPatLen -> (register, rank).
        uint8_t *reg[U];
        uint32_t rank[U], cur[U];
        if constexpr (kMode == kModeSwipes) {
#pragma unroll
            for (int u = 0; u < U; u++) {
                reg[u] = nullptr;
                rank[u] = 0;
                cur[u] = 0xffu;
                if (act[u] && sl[u] < nslots) {
                    uint32_t idx;
                    hll_patlen(hh[u], idx, rank[u]);
                    reg[u] = regs + size_t(sl[u]) * kHllRegs + idx;
                }
            }
#pragma unroll
            for (int u = 0; u < U; u++) cur[u] = reg[u] ? *reg[u] : 0xffu;
        }
        SKE_STAMP(tile_no, 3);
        bool valid[U];
#pragma unroll
        for (int u = 0; u < U; u++) valid[u] = false;
        for (int l = ch.nlinks - 1; l >= 0; --l) {
            const LinkDev &L = ch.link[l];
            if (kLds && L.div.d <= (uint64_t(1) << 31))
                link_probe_lds32<U>(L, lds_img, ha, hb, act, valid, probes);
            else if (L.div.d <= (uint64_t(1) << 31))
                link_probe<kLds, U, ProbeCursor32>(L, lds_img, ha, hb, act, valid, probes);
            else
                link_probe<kLds, U, ProbeCursor>(L, lds_img, ha, hb, act, valid, probes);
        }
        SKE_STAMP(tile_no, 4);
        if constexpr (kMode == kModeSwipes) {
#pragma unroll
            for (int u = 0; u < U; u++) {
                if (!valid[u]) continue;
                if (sl[u] >= nslots) {
                    atomicOr(reinterpret_cast<unsigned int *>(stats), 1u);
                } else if (cur[u] < rank[u]) {
                    reg_max(reg[u], rank[u]);  // the pre-check may be stale but is never too high
                }
            }
            SKE_STAMP(tile_no, 5);
            if (out) {
#pragma unroll
                for (int u = 0; u < U; u++)
                    if (act[u]) out[base + uint64_t(u) * T + tid] = valid[u];
            }
        } else if constexpr (kMode == kModeExists) {
#pragma unroll
            for (int u = 0; u < U; u++)
                if (act[u]) out[base + uint64_t(u) * T + tid] = valid[u];
        } else {
#pragma unroll
            for (int u = 0; u < U; u++) nvalid += valid[u];
        }
    }
    if constexpr (kMode == kModeStats) {
        atomicAdd(&stats[0], (unsigned long long)probes);
        atomicAdd(&stats[1], (unsigned long long)nvalid);
    }
}

__global__ void __launch_bounds__(256)
    k_pfadd(const uint32_t *__restrict__ slot, const uint8_t *__restrict__ bytes,
            const uint32_t *__restrict__ offs, uint64_t n, uint8_t *__restrict__ regs,
            uint32_t nslots, unsigned int *__restrict__ err) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t s = slot[i];
        if (s >= nslots) {
            atomicOr(err, 1u);
            continue;
        }
        const Item it = load_item(bytes, offs[i], offs[i + 1]);
        uint32_t idx, rank;
        hll_patlen(murmur_item(it, kHllSeed), idx, rank);
        reg_max(regs + size_t(s) * kHllRegs + idx, rank);
    }
}

// ---------------------------------------------------------------------------
// K2: PFCOUNT.  One 256-thread block per group; each thread owns 4 x 16-byte
// chunks (64 registers), max-merges them across the group's keys, and bins
// them into a per-wave LDS histogram.  Thread 0 then runs hllCount()'s
// estimator with the Redis operation order; m*tau(.) and m*sigma(.) come from
// host tables built with the same libm calls as Redis (tau_tab[H51],
// sig_tab[H0]) so only IEEE add / mul / div (correctly rounded) run here.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint4 max_u8x16(uint4 a, uint4 b) {
    uint32_t av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int q = 0; q < 4; q++) {
        uint32_t r = 0;
#pragma unroll
        for (int s = 0; s < 32; s += 8) {
            uint32_t x = (av[q] >> s) & 0xff, y = (bv[q] >> s) & 0xff;
            r |= (x > y ? x : y) << s;
        }
        av[q] = r;
    }
    return make_uint4(av[0], av[1], av[2], av[3]);
}

// Max over the 16-B chunk `chunk` of the keys srcs[s0..s1) (slots index the
// slab; srcs == nullptr: keys s0..s1), four loads in flight per step.
// One 16-B chunk of a key's registers.  The rollups (K2, K3) stream the slab
// once, with the non-temporal policy: C5 per-lecture unions 4.94 -> 4.67 ms
// (6.05 -> 6.40 TB/s), PFCOUNT-each 5.24 -> 5.20 ms, PFMERGE unchanged
// (tools/bench_rollup.py A/B, two alternations).
#ifndef SKE_K2_NT
#define SKE_K2_NT 1
#endif
__device__ __forceinline__ uint4 ld_regs16(const uint8_t *p) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    if constexpr (SKE_K2_NT != 0) {
        const v4 x = __builtin_nontemporal_load(reinterpret_cast<const v4 *>(p));
        return make_uint4(x[0], x[1], x[2], x[3]);
    } else {
        return *reinterpret_cast<const uint4 *>(p);
    }
}

__device__ __forceinline__ uint4 max_keys(const uint8_t *__restrict__ regs, const uint32_t *srcs,
                                          uint32_t s0, uint32_t s1, uint32_t chunk, uint4 v) {
    uint32_t s = s0;
#ifndef SKE_MK_UNROLL
#define SKE_MK_UNROLL 8
#endif
    // keys whose chunk loads are in flight together (C5 A/B: 4 / 8 / 16 within 1 %;
    // campus PFMERGE 5.22 -> 5.16 ms with 8)
    constexpr int kU = SKE_MK_UNROLL;
    for (; s + kU <= s1; s += kU) {
        uint4 r[kU];
#pragma unroll
        for (int q = 0; q < kU; q++) {
            const uint32_t key = srcs ? srcs[s + q] : s + q;
            r[q] = ld_regs16(regs + size_t(key) * kHllRegs + size_t(chunk) * 16);
        }
#pragma unroll
        for (int q = 0; q < kU; q++) v = max_u8x16(v, r[q]);
    }
    for (; s < s1; s++) {
        const uint32_t key = srcs ? srcs[s] : s;
        v = max_u8x16(v, ld_regs16(regs + size_t(key) * kHllRegs + size_t(chunk) * 16));
    }
    return v;
}

__device__ __forceinline__ uint64_t hll_estimate_dev(const uint32_t *h, const double *tau_tab,
                                                     const double *sig_tab) {
    double z = tau_tab[h[kHllQ + 1]];
    for (int j = kHllQ; j >= 1; --j) {
        z = __dadd_rn(z, double(h[j]));
        z = __dmul_rn(z, 0.5);
    }
    z = __dadd_rn(z, sig_tab[h[0]]);
    // HLL_ALPHA_INF * m * m, exact (m = 2^14)
    const double num = 0.721347520444481703680 * 16384.0 * 16384.0;
    const double q = num / z;
    // Redis: E = llroundl(q); return (uint64_t)E.  When q is +inf (every
    // register 51) or >= 2^63, x86-64 llroundl yields LLONG_MIN and the
    // double -> uint64 conversion of -2^63 gives 2^63; reproduce that.
    if (!(q < 9223372036854775808.0)) return uint64_t(1) << 63;
    return uint64_t(double(llround(q)));
}

__global__ void __launch_bounds__(256)
    k_pfcount(const uint8_t *__restrict__ regs, const uint32_t *__restrict__ slots,
              const uint32_t *__restrict__ goffs, uint32_t ngroups,
              const double *__restrict__ tau_tab, const double *__restrict__ sig_tab,
              uint64_t *__restrict__ out) {
    __shared__ uint32_t hist[4][64];
    const int tid = threadIdx.x, wave = tid >> 6;
    for (uint32_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
        for (int q = tid; q < 4 * 64; q += 256) (&hist[0][0])[q] = 0;
        __syncthreads();
        const uint32_t s0 = goffs ? goffs[g] : g, s1 = goffs ? goffs[g + 1] : g + 1;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t chunk = c * 256 + tid;  // 1024 chunks of 16 B
            const uint4 v = max_keys(regs, slots, s0, s1, chunk, make_uint4(0, 0, 0, 0));
            const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; q++)
#pragma unroll
                for (int sft = 0; sft < 32; sft += 8) atomicAdd(&hist[wave][(vv[q] >> sft) & 63], 1u);
        }
        __syncthreads();
        if (tid < 64) hist[0][tid] += hist[1][tid] + hist[2][tid] + hist[3][tid];
        __syncthreads();
        if (tid == 0) out[g] = (s1 > s0) ? hll_estimate_dev(hist[0], tau_tab, sig_tab) : 0;
        __syncthreads();
    }
}

// K2 for one key per group (PFCOUNT of every lecture-day key, the C5
// rankings): one wave per key, four waves per block.  Each lane bins its 256
// registers into a lane-private column of 64 counters in LDS (bin r of lane l
// at wave base + r*256 + l*4: every lane a different bank, no contention even
// when all registers share a value, which the block-per-group kernel's shared
// bins serialise on), so a register costs one bit-field extract, one OR and
// one ds_add.  The columns are never cleared: they keep running totals over
// the wave's keys, lane r keeps the previous sum of bin r over the 64 columns,
// and a key's bin r is the difference.  The sums read the columns in a
// lane-rotated order (bank-conflict free), and the next key's registers are
// loaded while this key is binned.  hllCount()'s 50-step dependent chain runs
// for kK2Batch keys side by side, one lane each, once their histograms are
// in (run per key on lane 0 it cost 0.8 ms of the 6 ms C5 pass).  A wave's LDS
// operations complete in order; wave_sync() keeps the compiler from
// reordering across the cross-lane hand-offs and drains lgkmcnt.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int kK2Waves = 4;
constexpr int kK2Batch = 8;  // keys whose estimates a wave runs side by side
__global__ void __launch_bounds__(64 * kK2Waves)
    k_pfcount_wave(const uint8_t *__restrict__ regs, const uint32_t *__restrict__ slots,
                   uint32_t nkeys, const double *__restrict__ tau_tab,
                   const double *__restrict__ sig_tab, uint64_t *__restrict__ out) {
    __shared__ uint32_t cols[kK2Waves * 64 * 64];  // [wave][bin][lane]
    __shared__ uint32_t hist[kK2Waves][kK2Batch][64];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // byte address of this lane's bin 0; bits 8..13 stay free for the bin
    const uint32_t base = wave * 16384 + lane * 4;
    char *lds = reinterpret_cast<char *>(cols);
#pragma unroll
    for (int r = 0; r < 64; r++) *(uint32_t *)(lds + base + r * 256) = 0;
    uint32_t prev = 0;  // lane r: sum of bin r over the columns after the last key
    const uint32_t stride = gridDim.x * kK2Waves;
    uint32_t g = blockIdx.x * kK2Waves + wave;
    uint4 v[16];
    if (g < nkeys) {
        const uint8_t *src = regs + size_t(slots ? slots[g] : g) * kHllRegs;
#pragma unroll
        for (int q = 0; q < 16; q++) v[q] = ld_regs16(src + (q * 64 + lane) * 16);  // coalesced 1 KiB per step
    }
    wave_sync();
    uint32_t e = 0;  // histograms waiting for their estimate
    for (; g < nkeys; g += stride) {
        const uint32_t gn = g + stride;
        uint4 nv[16];
        if (gn < nkeys) {  // the next key's registers fly while this one is binned
            const uint8_t *src = regs + size_t(slots ? slots[gn] : gn) * kHllRegs;
#pragma unroll
            for (int q = 0; q < 16; q++) nv[q] = ld_regs16(src + (q * 64 + lane) * 16);
        }
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const uint32_t wd[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
            for (int e4 = 0; e4 < 4; e4++)
#pragma unroll
                for (int b = 0; b < 32; b += 8) {
                    const uint32_t r = __builtin_amdgcn_ubfe(wd[e4], b, 6);
                    __hip_atomic_fetch_add((uint32_t *)(lds + ((r << 8) | base)), 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                }
        }
        wave_sync();
        const char *bin = lds + wave * 16384 + lane * 256;  // lane r sums bin r
        uint32_t sum = 0;
#pragma unroll 8
        for (int l = 0; l < 64; l++) sum += *(const uint32_t *)(bin + (((l + lane) & 63) << 2));
        hist[wave][e][lane] = sum - prev;
        prev = sum;
        // hllCount() of the batch: lane j < kK2Batch estimates the key
        // binned j keys after the batch's first (g - (e - j) * stride)
        if (++e == kK2Batch || gn >= nkeys) {
            wave_sync();
            if (lane < e) out[g - (e - 1 - lane) * stride] = hll_estimate_dev(hist[wave][lane], tau_tab, sig_tab);
            e = 0;
        }
        wave_sync();
#pragma unroll
        for (int q = 0; q < 16; q++) v[q] = nv[q];
    }
}

// Register histogram of one key (for the oracle cross-check of K2's bins).
__global__ void __launch_bounds__(256)
    k_histogram(const uint8_t *__restrict__ regs, uint32_t *__restrict__ out64) {
    __shared__ uint32_t hist[64];
    if (threadIdx.x < 64) hist[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < kHllRegs; r += blockDim.x) atomicAdd(&hist[regs[r] & 63], 1u);
    __syncthreads();
    if (threadIdx.x < 64) out64[threadIdx.x] = hist[threadIdx.x];
}

// K3 for many sources, pass 1: partition p of the sources (`per` consecutive
// entries of srcs) max-merged into partial row p; block = (partition, quarter
// of the 1024 chunks).
__global__ void __launch_bounds__(256)
    k_pfmerge_part(const uint8_t *__restrict__ regs, const uint32_t *__restrict__ srcs, uint32_t n,
                   uint32_t per, uint8_t *__restrict__ partial) {
    const uint32_t chunk = threadIdx.x + (blockIdx.x & 3) * 256;
    const uint32_t p = blockIdx.x >> 2;
    const uint32_t s0 = p * per, s1 = s0 + per < n ? s0 + per : n;
    const uint4 v = max_keys(regs, srcs, s0, s1, chunk, make_uint4(0, 0, 0, 0));
    reinterpret_cast<uint4 *>(partial + size_t(p) * kHllRegs)[chunk] = v;
}

// pass 2: dst = max(dst, partial rows 0..P)
__global__ void __launch_bounds__(256)
    k_pfmerge_rows(uint8_t *__restrict__ regs, uint32_t dst, const uint8_t *__restrict__ partial,
                   uint32_t P) {
    const uint32_t chunk = blockIdx.x * blockDim.x + threadIdx.x;
    if (chunk >= kHllRegs / 16) return;
    uint4 *d = reinterpret_cast<uint4 *>(regs + size_t(dst) * kHllRegs) + chunk;
    *d = max_keys(partial, nullptr, 0, P, chunk, *d);
}

// K3: PFMERGE dst = max(dst, srcs...)
__global__ void __launch_bounds__(256)
    k_pfmerge(uint8_t *__restrict__ regs, uint32_t dst, const uint32_t *__restrict__ srcs,
              uint32_t n) {
    const uint32_t chunk = blockIdx.x * blockDim.x + threadIdx.x;
    if (chunk >= kHllRegs / 16) return;
    uint4 *d = reinterpret_cast<uint4 *>(regs + size_t(dst) * kHllRegs) + chunk;
    *d = max_keys(regs, srcs, 0, n, chunk, *d);
}

// K3 into an external buffer: dst[g] = max over the group's slots
__global__ void __launch_bounds__(256)
    k_merge_groups(const uint8_t *__restrict__ regs, const uint32_t *__restrict__ slots,
                   const uint32_t *__restrict__ goffs, uint32_t ngroups, uint8_t *__restrict__ dst) {
    const uint32_t chunk = threadIdx.x + (blockIdx.x & 3) * 256;  // 1024 x 16 B per key
    for (uint32_t g = blockIdx.x >> 2; g < ngroups; g += gridDim.x >> 2) {
        const uint4 v = max_keys(regs, slots, goffs[g], goffs[g + 1], chunk, make_uint4(0, 0, 0, 0));
        reinterpret_cast<uint4 *>(dst + size_t(g) * kHllRegs)[chunk] = v;
    }
}

hipError_t launch_merge_groups(const uint8_t *regs, const uint32_t *slots, const uint32_t *goffs,
                               uint32_t ngroups, uint8_t *dst, int cus, hipStream_t st) {
    if (ngroups == 0) return hipSuccess;
    const unsigned g = ngroups < unsigned(cus) * 4 ? ngroups : unsigned(cus) * 4;
    hipLaunchKernelGGL(k_merge_groups, dim3(g * 4), dim3(256), 0, st, regs, slots, goffs, ngroups, dst);
    return hipGetLastError();
}

// HLL_DENSE_SET_REGISTER packing: registers 4j..4j+3 -> bytes 3j..3j+2
__global__ void __launch_bounds__(256)
    k_dense(const uint8_t *__restrict__ regs, uint8_t *__restrict__ dense) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= kHllRegs / 4) return;
    const uint32_t w = reinterpret_cast<const uint32_t *>(regs)[j];
    const uint32_t r0 = w & 63, r1 = (w >> 8) & 63, r2 = (w >> 16) & 63, r3 = (w >> 24) & 63;
    const uint32_t bits = r0 | (r1 << 6) | (r2 << 12) | (r3 << 18);
    dense[3 * j + 0] = uint8_t(bits);
    dense[3 * j + 1] = uint8_t(bits >> 8);
    dense[3 * j + 2] = uint8_t(bits >> 16);
}

// ---------------------------------------------------------------------------
// Synthetic stream
// ---------------------------------------------------------------------------
__device__ __forceinline__ void write_decimal(uint8_t *dst, uint64_t x, uint32_t width) {
    for (int d = int(width) - 1; d >= 0; --d) {
        dst[d] = uint8_t('0' + x % 10);
        x /= 10;
    }
}

__device__ uint64_t gen_swipe_id(const GenDev &g, uint64_t i) {
    const uint64_t u0 = mix(g.seed, i, 0);
    if (uint32_t(u0 >> 32) >= g.inv_thr) return gen_member(g, mix(g.seed, i, 1) % g.N);
    if (g.near_thr && uint32_t(mix(g.seed, i, 1) >> 32) < g.near_thr) {
        const uint64_t base = gen_member(g, mix(g.seed, i, 2) % g.N);
        const uint64_t u = mix(g.seed, i, 3);
        int64_t cand;
        if ((u & 1) == 0) {
            cand = ((u >> 1) & 1) ? int64_t(base) + 1 : int64_t(base) - 1;
        } else {
            const uint32_t pos = uint32_t((u >> 8) % g.width);
            const int64_t p10 = int64_t(g.pow10[pos]);
            const int64_t dold = int64_t(base / uint64_t(p10)) % 10;
            const int64_t dnew = (dold + 1 + int64_t((u >> 16) % 9)) % 10;
            cand = int64_t(base) + (dnew - dold) * p10;
        }
        if (cand >= int64_t(g.lo) && cand < int64_t(g.lo + g.R) && !gen_is_member(g, uint64_t(cand)))
            return uint64_t(cand);
    }
    uint64_t x = 0;
    for (uint32_t t = 0; t < 64; t++) {
        x = g.lo + mix(g.seed, i, 4 + t) % g.R;
        if (!gen_is_member(g, x)) break;
    }
    return x;
}

__global__ void __launch_bounds__(256)
    k_gen_swipes(const GenDev g, uint64_t start, uint64_t n, uint8_t *__restrict__ bytes,
                 uint32_t *__restrict__ offs, uint32_t *__restrict__ slot) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < n; t += stride) {
        const uint64_t i = start + t;
        write_decimal(bytes + t * g.width, gen_swipe_id(g, i), g.width);
        offs[t] = uint32_t(t * g.width);
        if (t == n - 1) offs[n] = uint32_t(n * g.width);
        uint32_t s;
        if (g.key_cdf) {
            const uint32_t u = uint32_t(mix(g.seed, i, 200) >> 32);
            uint32_t lo = 0, hi = g.n_keys - 1;  // first j with cdf[j] > u; last key absorbs
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (g.key_cdf[mid] > u) hi = mid; else lo = mid + 1;
            }
            s = lo;
        } else {
            s = uint32_t(mix(g.seed, i, 200) % g.n_keys);
        }
        slot[t] = g.slot_base + s;
    }
}

__global__ void __launch_bounds__(256)
    k_gen_members(const GenDev g, uint64_t start, uint64_t n, uint8_t *__restrict__ bytes,
                  uint32_t *__restrict__ offs) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < n; t += stride) {
        write_decimal(bytes + t * g.width, gen_member(g, start + t), g.width);
        offs[t] = uint32_t(t * g.width);
        if (t == n - 1) offs[n] = uint32_t(n * g.width);
    }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static inline unsigned grid_for(uint64_t n, unsigned block, unsigned cap) {
    uint64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    return unsigned(g < cap ? g : cap);
}

template <int kMode, int U>
static hipError_t launch_swipes_u(const ChainDev &ch, bool lds, const uint8_t *bytes,
                                  const uint32_t *offs, uint32_t fixed_w, const uint32_t *slot, uint64_t n,
                                  uint8_t *regs, uint32_t nslots, uint8_t *out,
                                  unsigned long long *stats, int cus, hipStream_t st) {
    if (lds) {
        // one 1024-thread block per CU (the LDS image caps residency at one)
        const unsigned grid = grid_for(n, 1024 * U, unsigned(cus));
        hipLaunchKernelGGL((k_swipes<kMode, true, U>), dim3(grid), dim3(1024), ch.lds_bytes, st, ch,
                           bytes, offs, fixed_w, slot, n, regs, nslots, out, stats);
    } else {
        const unsigned grid = grid_for(n, 256 * U, unsigned(cus) * 8);
        hipLaunchKernelGGL((k_swipes<kMode, false, U>), dim3(grid), dim3(256), 0, st, ch, bytes,
                           offs, fixed_w, slot, n, regs, nslots, out, stats);
    }
    return hipGetLastError();
}

hipError_t launch_swipes(int mode, const ChainDev &ch, bool lds, int tile, const uint8_t *bytes,
                         const uint32_t *offs, uint32_t fixed_w, const uint32_t *slot, uint64_t n, uint8_t *regs,
                         uint32_t nslots, uint8_t *out, unsigned long long *stats, int cus,
                         hipStream_t st) {
    if (n == 0) return hipSuccess;
#define SKE_U(UU)                                                                                  \
    if (mode == kModeSwipes)                                                                       \
        return launch_swipes_u<kModeSwipes, UU>(ch, lds, bytes, offs, fixed_w, slot, n, regs, nslots, out,  \
                                                stats, cus, st);                                   \
    if (mode == kModeExists)                                                                       \
        return launch_swipes_u<kModeExists, UU>(ch, lds, bytes, offs, fixed_w, slot, n, regs, nslots, out,  \
                                                stats, cus, st);                                   \
    return launch_swipes_u<kModeStats, UU>(ch, lds, bytes, offs, fixed_w, slot, n, regs, nslots, out,       \
                                           stats, cus, st);
    if (tile >= 8) {
        SKE_U(8)
    } else if (tile >= 4) {
        SKE_U(4)
    } else if (tile >= 2) {
        SKE_U(2)
    } else {
        SKE_U(1)
    }
#undef SKE_U
}

hipError_t lds_bloom_setup() {
    // allow the LDS-staged variant to declare up to kLdsBloomMax bytes
    hipError_t e = hipSuccess;
#define SKE_ATTR(M, UU)                                                                            \
    e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_swipes<M, true, UU>),                \
                            hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBloomMax);             \
    if (e != hipSuccess) return e;
    SKE_ATTR(kModeSwipes, 1) SKE_ATTR(kModeSwipes, 2) SKE_ATTR(kModeSwipes, 4) SKE_ATTR(kModeSwipes, 8)
    SKE_ATTR(kModeExists, 1) SKE_ATTR(kModeExists, 2) SKE_ATTR(kModeExists, 4) SKE_ATTR(kModeExists, 8)
    SKE_ATTR(kModeStats, 1) SKE_ATTR(kModeStats, 2) SKE_ATTR(kModeStats, 4) SKE_ATTR(kModeStats, 8)
#undef SKE_ATTR
    return e;
}

uint32_t lds_bloom_max() { return kLdsBloomMax; }

hipError_t launch_pfadd(const uint32_t *slot, const uint8_t *bytes, const uint32_t *offs,
                        uint64_t n, uint8_t *regs, uint32_t nslots, unsigned int *err, int cus,
                        hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pfadd, dim3(grid_for(n, 256, cus * 16)), dim3(256), 0, st, slot, bytes,
                       offs, n, regs, nslots, err);
    return hipGetLastError();
}

hipError_t launch_pfcount(const uint8_t *regs, const uint32_t *slots, const uint32_t *goffs,
                          uint32_t ngroups, const double *tau, const double *sig, uint64_t *out,
                          int cus, hipStream_t st) {
    if (ngroups == 0) return hipSuccess;
    if (!goffs) {  // one key per group
        const unsigned want = (ngroups + kK2Waves - 1) / kK2Waves, cap = unsigned(cus) * 2;
        hipLaunchKernelGGL(k_pfcount_wave, dim3(want < cap ? want : cap), dim3(64 * kK2Waves), 0, st, regs,
                           slots, ngroups, tau, sig, out);
        return hipGetLastError();
    }
    const unsigned grid = ngroups < unsigned(cus) * 8 ? ngroups : unsigned(cus) * 8;
    hipLaunchKernelGGL(k_pfcount, dim3(grid), dim3(256), 0, st, regs, slots, goffs, ngroups, tau,
                       sig, out);
    return hipGetLastError();
}

hipError_t launch_histogram(const uint8_t *regs, uint32_t *out64, hipStream_t st) {
    hipLaunchKernelGGL(k_histogram, dim3(1), dim3(256), 0, st, regs, out64);
    return hipGetLastError();
}

hipError_t launch_pfmerge(uint8_t *regs, uint32_t dst, const uint32_t *srcs, uint32_t n,
                          hipStream_t st) {
    hipLaunchKernelGGL(k_pfmerge, dim3(kHllRegs / 16 / 256), dim3(256), 0, st, regs, dst, srcs, n);
    return hipGetLastError();
}

// PFMERGE of many sources: partitions of `per` sources reduced in parallel
// into partial rows (P <= 4 per CU), then one pass over the rows.
uint32_t pfmerge_partitions(uint32_t n, int cus, uint32_t *per) {
    const uint32_t maxp = uint32_t(cus) * 4;
    uint32_t pp = (n + maxp - 1) / maxp;
    *per = pp < 16 ? 16 : pp;
    return (n + *per - 1) / *per;
}

hipError_t launch_pfmerge_wide(uint8_t *regs, uint32_t dst, const uint32_t *srcs, uint32_t n,
                               uint8_t *partial, uint32_t per, uint32_t P, hipStream_t st) {
    hipLaunchKernelGGL(k_pfmerge_part, dim3(P * 4), dim3(256), 0, st, regs, srcs, n, per, partial);
    hipLaunchKernelGGL(k_pfmerge_rows, dim3(kHllRegs / 16 / 256), dim3(256), 0, st, regs, dst,
                       partial, P);
    return hipGetLastError();
}

// the largest of n device slots, into *out (zeroed by the caller): the range
// check of a device-resident slot list (ske_hll_pfmerge_dev, ske_hll_pfcount_each
// with SKE_MEM_DEVICE) before any kernel addresses the slab with it
__global__ void __launch_bounds__(256) k_slots_max(const uint32_t *__restrict__ s, uint64_t n, unsigned int *out) {
    uint32_t m = 0;
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256)
        m = s[i] > m ? s[i] : m;
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t y = __shfl_xor(m, o, 64);
        m = y > m ? y : m;
    }
    if ((threadIdx.x & 63) == 0 && m) atomicMax(out, m);
}

hipError_t launch_slots_max(const uint32_t *slots, uint64_t n, unsigned int *out, int cus, hipStream_t st) {
    hipError_t e = hipMemsetAsync(out, 0, 4, st);
    if (e != hipSuccess || n == 0) return e;
    hipLaunchKernelGGL(k_slots_max, dim3(grid_for(n, 256, cus * 4)), dim3(256), 0, st, slots, n, out);
    return hipGetLastError();
}

hipError_t launch_dense(const uint8_t *regs, uint8_t *dense, hipStream_t st) {
    hipLaunchKernelGGL(k_dense, dim3(kHllRegs / 4 / 256), dim3(256), 0, st, regs, dense);
    return hipGetLastError();
}

hipError_t launch_gen_swipes(const GenDev &g, uint64_t start, uint64_t n, uint8_t *bytes,
                             uint32_t *offs, uint32_t *slot, int cus, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_swipes, dim3(grid_for(n, 256, cus * 16)), dim3(256), 0, st, g, start,
                       n, bytes, offs, slot);
    return hipGetLastError();
}

hipError_t launch_gen_members(const GenDev &g, uint64_t start, uint64_t n, uint8_t *bytes,
                              uint32_t *offs, int cus, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_members, dim3(grid_for(n, 256, cus * 16)), dim3(256), 0, st, g, start,
                       n, bytes, offs);
    return hipGetLastError();
}

}  // namespace ske
