// sketch_part.hip -- K1 for Bloom chains too large for one CU's LDS (C3/C5:
// the 19.8 MB RESERVE 0.001 / 1e7 filter), partitioned: every probe is tested
// against an LDS-resident 64 KiB slice of its link.
//
// Same answers as every K1 variant: per swipe BF.EXISTS (SBChain_Check: a link
// says "present" iff all k probe bits (a + i*b) mod 2^64 mod bits are set, the
// chain iff any link does -- attendance_processor.py:109-113) and, if present,
// PFADD (hllPatLen -> register max, :127-129).
//
// Why partitioned.  A random probe into a 19.8 MB bit array is a random line
// request: 55 G/s chip-wide from the Infinity Cache or HBM, 252 G/s from a
// slice kept L2-resident per XCD (tools/randbench.hip).  176 M probes per
// 16 M-swipe step are then 0.7 ms even at the L2 rate.  A random ds_read_u8
// from LDS runs at 4.6 T/s.  The whole filter (19.8 MB) fits in the chip's
// aggregate LDS (256 x 160 KiB), so the probes are routed to the CU holding
// their slice instead -- a radix partition of 4-byte probe records, streamed
// through HBM in whole lines:
//
//   pass A (k_part_a)  one tile of T = 1024*U swipes per iteration: hash each
//                      id (MurmurHash64A a, b, and the HLL hash), walk every
//                      link's k probes, and emit one record per probe,
//                      (bit offset in its slice) | (swipe index in tile) << 19,
//                      counting-sorted by slice in LDS and written out as one
//                      contiguous run per tile; off[tile][slice] holds the run
//                      boundaries.  Also the HLL word (register | rank << 16)
//                      and a cleared fail byte per swipe and link.
//   pass B (k_part_b)  one slice per block, staged into LDS; the block reads
//                      its slice's run of every tile in its range and stores
//                      fail[link][swipe] = 1 for every probe whose bit is 0.
//   pass C (k_part_c)  per swipe: valid = some link without a failed probe;
//                      register max (pre-check load, CAS) and the answer.
//
// Placement of blocks on XCDs is a speed matter only; every (tile, slice) run
// is read by exactly one block, and fail bytes are only ever set to 1.
#include <algorithm>

#include "sketch_common.h"
#include "sketch_internal.h"

namespace ske {

constexpr uint32_t kPaBlock = 1024;
constexpr uint32_t kPbBlock = 1024;
constexpr uint32_t kPcBlock = 256;
constexpr uint32_t kPSliceMask = kPSliceBits - 1;
constexpr uint32_t kPSliceBytes = kPSliceBits / 8;  // 64 KiB
constexpr uint32_t kPSub = 1u << 24;                // swipes per sub-batch (passes A-B-C)
constexpr uint32_t kPbGroup = 8;                    // tiles a pass-B wave reads at once
constexpr uint32_t kPbLanes = 64 / kPbGroup;        // lanes per tile run
constexpr uint32_t kPcErr = 0xffffffffu;            // pre: an HLL word whose slot is outside the slab

struct PartLink {
    const uint8_t *bf;
    uint64_t m;          // Granlund-Montgomery magic of d
    uint32_t d;          // bloom->bits (<= 2^31)
    uint32_t t;          // 2^64 mod d
    uint32_t sh;         // l - 1 of the magic
    uint32_t k;          // bloom->hashes
    uint32_t slice0;     // first global slice of this link
    uint32_t nbytes16;   // bit-array bytes rounded up to 16 (readable)
};

struct PartArgs {
    const uint8_t *bytes;
    const uint32_t *offs;  // nullptr: fixed-width ids
    const uint32_t *slot;
    uint8_t *regs;
    uint8_t *out;          // may be nullptr
    unsigned int *err;
    uint32_t *rec;         // [ntiles][stride] probe records
    uint32_t *off;         // [nslices + 1][off_stride] run boundaries (slice-major)
    uint8_t *fail;         // [nlinks][fail_stride]
    uint32_t *hllw;        // [n] register | rank << 16 (pre: rank 0 = no raise, kPcErr = slot out of range)
    uint32_t *oldw;        // [n] pre: the register's aligned word as pass A read it (pass C's CAS expectation)
    uint32_t fixed_w, n, stride, ntiles, nslices, nlinks, ksum, nslots, fail_stride, off_stride;
    uint32_t pre;          // pass A pre-checks the register (k_part_a2, CAS pass C only)
    uint16_t *flist;       // [nunits][fl_stride][kPbLanes] fail lists (pass B -> pass C), or nullptr
    uint32_t nunits, fl_stride;
    uint32_t tile_log;     // swipes per tile = 1 << tile_log (10, or 11 for k_part_a2<11, 1024>)
    PartLink link[kPMaxLinks];
};

__device__ __forceinline__ Divisor part_div(const PartLink &L) { return Divisor{L.d, L.m, L.t, L.sh, 0}; }

// A workgroup barrier for hand-offs through LDS only: it waits for this
// wave's LDS operations (lgkmcnt(0)) and not for its global loads and stores
// in flight, which __syncthreads() drains too (vmcnt(0)).  The partitioned
// passes share nothing through global memory inside a block, so the next
// tile's prefetched ids (pass A), the next round's records (pass B) and the
// register CASes (pass C) stay in flight across their barriers.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Tiles are dealt to kPGroups contiguous groups, and every pass gives the
// blocks b with b % kPGroups == x the tiles of group x.  Blocks are dealt
// round-robin over the 8 XCDs, so a group's fail bytes (2 MB at C3) are
// written by pass A, set by pass B and read by pass C in one XCD's L2.  This
// is placement for speed only: every tile of a group is handled by exactly one
// block of the group, whichever XCD it runs on.
constexpr uint32_t kPGroups = 8;
__device__ __forceinline__ void part_group(uint32_t ntiles, uint32_t x, uint32_t &t0, uint32_t &t1) {
    t0 = uint32_t(uint64_t(ntiles) * x / kPGroups);
    t1 = uint32_t(uint64_t(ntiles) * (x + 1) / kPGroups);
}

// ---------------------------------------------------------------------------
// ids of at most 8 bytes (every config's student ids), read and hashed the way
// the LDS K1 does (sketch_k1.hip): the one or two aligned 64-bit words holding
// the id (an empty or long id reads zeros past the range), a funnel shift and
// a length mask, MurmurHash64A in closed form h = ((seed ^ len*m) ^ t) * m then
// the finaliser, t the id word or (len 8) its mixed block, mixed once for the
// three hashes.  A wave holding a longer id takes the generic routines.
// ---------------------------------------------------------------------------
__device__ __forceinline__ __amdgpu_buffer_rsrc_t part_rsrc(const void *p, uint32_t nbytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, int(nbytes), 0x00020000);
}

// Streams read or written once take the non-temporal policy (`nt`): pass B's
// probe records always; SKE_NT bits select the rest -- 1 pass B's run
// boundaries, 2 pass A's ids and offsets, 4 pass A's record copy-out, 8 pass
// A's HLL words and fail bytes, 16 pass C's streams (fail bytes, slots, HLL
// words, answers), 32 pass C's register pre-check loads.  Measured at C3 (A/B,
// two alternations): records nt: pass B 0.276 -> 0.260 ms; + bits 1|2|4:
// 0.25 ms; bits 8 and 16 neutral to slightly slower; bit 32 makes pass C
// 0.39 -> 0.59 ms (the raising CAS no longer finds its line near).  Default 7.
#ifndef SKE_NT
#define SKE_NT 7
#endif
typedef uint32_t part_u32x4 __attribute__((ext_vector_type(4)));
template <int BIT, class T> __device__ __forceinline__ T nt_ld(const T *p) {
    if constexpr ((SKE_NT & BIT) != 0) return __builtin_nontemporal_load(p);
    else return *p;
}
template <int BIT, class T> __device__ __forceinline__ void nt_st(T *p, T v) {
    if constexpr ((SKE_NT & BIT) != 0) __builtin_nontemporal_store(v, p);
    else *p = v;
}
template <int BIT> __device__ __forceinline__ constexpr int nt_aux() { return (SKE_NT & BIT) ? 2 : 0; }

struct PartId {
    uint32_t b, len;
    uint64_t w0, w1;
};

__device__ __forceinline__ void part_id_load(const __amdgpu_buffer_rsrc_t &rb, uint32_t b, uint32_t e,
                                             PartId &d) {
    d.b = b;
    d.len = e - b;
    const uint32_t s8 = b & 7;
    const bool sh = d.len && d.len <= 8;
    const uint32_t o0 = sh ? (b & ~7u) : 0xfffffff8u;
    const uint32_t o1 = (sh && s8 + d.len > 8) ? o0 + 8 : o0;
    d.w0 = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(rb, o0, 0, nt_aux<2>()));
    d.w1 = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(rb, o1, 0, nt_aux<2>()));
}

__device__ __forceinline__ void part_hash3(const uint8_t *bytes, const PartId &d, uint64_t &ha, uint64_t &hb,
                                           uint64_t &hh) {
    if (__any(d.len > 8)) {
        const Item it = load_item(bytes, d.b, d.b + d.len);
        ha = murmur_item(it, kBloomSeed);
        hb = murmur_item(it, ha);
        hh = murmur_item(it, kHllSeed);
        return;
    }
    const uint32_t sh = (d.b & 7) * 8;
    const bool hi = sh >= 32;
    const uint32_t a = hi ? uint32_t(d.w0 >> 32) : uint32_t(d.w0);
    const uint32_t bb = hi ? uint32_t(d.w1) : uint32_t(d.w0 >> 32);
    const uint32_t c = hi ? uint32_t(d.w1 >> 32) : uint32_t(d.w1);
    const uint64_t v = (uint64_t(__builtin_amdgcn_alignbit(c, bb, sh & 31)) << 32) |
                       __builtin_amdgcn_alignbit(bb, a, sh & 31);
    const uint32_t drop = (64 - d.len * 8) & 63;
    uint64_t tw = (v << drop) >> drop;
    if (__any(d.len == 8)) {
        uint64_t k = tw * kMurmurM;
        k ^= k >> 47;
        k *= kMurmurM;
        tw = d.len == 8 ? k : tw;
    }
    const uint64_t t = tw ^ (uint64_t(d.len) * kMurmurM);
    const bool nz = d.len != 0;
    ha = mm_final(nz ? (kBloomSeed ^ t) * kMurmurM : kBloomSeed);
    hb = mm_final(nz ? (ha ^ t) * kMurmurM : ha);
    hh = mm_final(nz ? (kHllSeed ^ t) * kMurmurM : kHllSeed);
}

// ---------------------------------------------------------------------------
// pass A: hash, probe records, counting sort by slice
// ---------------------------------------------------------------------------
// One tile = 1024 swipes, one per thread.  KM: the most probes per swipe the
// instantiation holds (every link's k summed); records of a tile live in LDS
// (KM = 11: 44 KiB, two blocks per CU, so one block's hashing overlaps the
// other's sort and copy-out).  One-link chains of k = 11 (C3/C5) take
// k_part_a2 below.
template <int KM>
__global__ void __launch_bounds__(kPaBlock, KM <= 11 ? 8 : 4) k_part_a(const PartArgs A) {
    __shared__ __attribute__((aligned(16))) uint32_t srec[kPaBlock * KM];
    // slice histogram, then run starts; two buffers used by alternate tiles,
    // so the one the next tile counts into is cleared while this tile still
    // reads its own (four barriers per tile)
    __shared__ uint32_t scnt2[2][kPMaxSlices + 1];
    __shared__ uint32_t swsum[kPaBlock / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t S = A.nslices;
    for (uint32_t g = tid; g <= kPMaxSlices; g += kPaBlock) scnt2[0][g] = scnt2[1][g] = 0;
    __syncthreads();
    // the next tile's ids are loaded while this tile sorts: its offsets at the
    // top of the iteration, its id words after the scan
    auto offsets = [&](uint32_t t, uint32_t &b, uint32_t &e) {
        const uint32_t i = t * kPaBlock + tid;
        const uint32_t ic = i < A.n ? i : A.n - 1;
        b = A.offs ? A.offs[ic] : ic * A.fixed_w;
        e = A.offs ? A.offs[ic + 1] : b + A.fixed_w;
    };
    uint32_t gt0, gt1;
    part_group(A.ntiles, blockIdx.x % kPGroups, gt0, gt1);
    const uint32_t tstep = gridDim.x / kPGroups;
    const __amdgpu_buffer_rsrc_t rbytes = part_rsrc(A.bytes, 0xfffffff0u);
    uint32_t par = 0, nb_ = 0, ne_ = 0;
    PartId it;
    {
        const uint32_t t = gt0 + blockIdx.x / kPGroups;
        offsets(t < gt1 ? t : gt0, nb_, ne_);
        part_id_load(rbytes, nb_, ne_, it);
    }
    for (uint32_t t = gt0 + blockIdx.x / kPGroups; t < gt1; t += tstep, par ^= 1) {
        uint32_t *scnt = scnt2[par];
        uint32_t rv[KM], rp[KM];
        const uint32_t tn = t + tstep < gt1 ? t + tstep : t;
        offsets(tn, nb_, ne_);
        {
            const uint32_t i = t * kPaBlock + tid;
            const bool act = i < A.n;
            uint64_t ha, hb, hh;
            part_hash3(A.bytes, it, ha, hb, hh);
            if (act) {
                uint32_t idx, rank;
                hll_patlen(hh, idx, rank);
                A.hllw[i] = idx | (rank << 16);
                for (uint32_t l = 0; l < A.nlinks; l++) A.fail[size_t(l) * A.fail_stride + i] = 0;
            }
            // every link's k probes in RedisBloom's order, newest link first
            // (the order is immaterial to the answer; records carry no link:
            // a slice belongs to one link)
            // bit 29 of a record: its slice's parity (pass B's slice pairs)
            const uint32_t rbase = (tid << kPSliceLog) | 0x80000000u;
            {
                uint32_t l = A.nlinks - 1, jl = 0;
                ProbeWalk32 wk;
                wk.init(ha, hb, part_div(A.link[l]));
#pragma unroll
                for (int q = 0; q < KM; q++) {
                    rp[q] = 0xffffffffu;
                    rv[q] = 0;
                    if (uint32_t(q) < A.ksum) {  // block-uniform
                        if (jl == A.link[l].k) {
                            l--;
                            jl = 0;
                            wk.init(ha, hb, part_div(A.link[l]));
                        }
                        const uint32_t x = wk.x;
                        const uint32_t g = A.link[l].slice0 + (x >> kPSliceLog);
                        rv[q] = (x & kPSliceMask) | ((g & 1u) << 29) | rbase;
                        if (act) rp[q] = (g << 16) | atomicAdd(&scnt[g], 1u);
                        wk.step(A.link[l].d);
                        jl++;
                    }
                }
            }
        }
        __syncthreads();
        part_id_load(rbytes, nb_, ne_, it);  // the next tile's ids
        // exclusive scan of scnt[0..S] (scnt[S] == 0 becomes the tile's total)
        constexpr int kPer = (kPMaxSlices + 1) / kPaBlock;
        uint32_t v[kPer], s = 0;
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            v[j] = scnt[tid * kPer + j];
            s += v[j];
        }
        uint32_t incl = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= uint32_t(o)) incl += y;
        }
        if (lane == 63) swsum[wave] = incl;
        __syncthreads();
        uint32_t run = incl - s;
        for (uint32_t w = 0; w < wave; w++) run += swsum[w];
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            scnt[tid * kPer + j] = run;
            run += v[j];
        }
        __syncthreads();
        // run boundaries, slice-major: off[g][t] (a pass-B wave reads the
        // boundaries of consecutive tiles of its slice as two short rows)
        for (uint32_t g = tid; g <= S; g += kPaBlock) A.off[size_t(g) * A.off_stride + t] = scnt[g];
#pragma unroll
        for (int q = 0; q < KM; q++)
            if (rp[q] != 0xffffffffu) srec[scnt[rp[q] >> 16] + (rp[q] & 0xffffu)] = rv[q];
        // the next tile's histogram (its previous readers passed two barriers ago)
        for (uint32_t g = tid; g <= S; g += kPaBlock) scnt2[par ^ 1][g] = 0;
        __syncthreads();
        // copy-out; the next tile places records only after three more barriers
        const uint32_t total = scnt[S];
        uint4 *dst = reinterpret_cast<uint4 *>(A.rec + size_t(t) * A.stride);
        const uint4 *src = reinterpret_cast<const uint4 *>(srec);
        for (uint32_t j = tid; j * 4 < total; j += kPaBlock) dst[j] = src[j];
    }
}

// The same pass A for one-link chains of exactly KM probes with half the
// threads: a 512-thread block owns the 1024-swipe tile, two swipes per
// thread (swipes tid and tid + 512 of the tile, the same record layout), so a
// thread has twice the independent work between barriers and 128 VGPRs
// (two blocks per CU, 16 waves) instead of 64 -- no spills, half the barrier
// width.  C3: 0.315 -> 0.273 ms per 16M swipes (A/B on one box); 256 threads x
// 4 swipes (208 VGPRs, 8 waves per CU) was slower again, 0.323 ms.
constexpr uint32_t kA2Threads = 512;
template <int KM, uint32_t kA2Threads = kA2Threads, uint32_t kA2U = 2, bool kPre = false>
__global__ void __launch_bounds__(kA2Threads, kA2Threads == 1024 ? 1 : 2) k_part_a2(const PartArgs A) {
    constexpr uint32_t kTile = kA2Threads * kA2U;  // swipes per tile (1 << A.tile_log)
    constexpr uint32_t kTileLog = kTile == 2048 ? 11 : 10;
    static_assert(kTile == 1024 || kTile == 2048, "tile");
    __shared__ __attribute__((aligned(16))) uint32_t srec[kTile * KM];
    __shared__ uint32_t scnt2[2][kPMaxSlices + 1];
    __shared__ uint32_t swsum[kA2Threads / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t S = A.nslices;
    // a slice counter starts at g << 16, so an LDS atomic's return value is
    // already the record's (slice, rank) pair
    for (uint32_t g = tid; g <= kPMaxSlices; g += kA2Threads) scnt2[0][g] = scnt2[1][g] = g << 16;
    __syncthreads();
    auto offsets = [&](uint32_t t, uint32_t u, uint32_t &b, uint32_t &e, uint32_t &sl) {
        const uint32_t i = t * kTile + u * kA2Threads + tid;
        const uint32_t ic = i < A.n ? i : A.n - 1;
        b = A.offs ? nt_ld<2>(A.offs + ic) : ic * A.fixed_w;
        e = A.offs ? nt_ld<2>(A.offs + ic + 1) : b + A.fixed_w;
        sl = kPre ? A.slot[ic] : 0;
    };
    uint32_t gt0, gt1;
    part_group(A.ntiles, blockIdx.x % kPGroups, gt0, gt1);
    const uint32_t tstep = gridDim.x / kPGroups;
    const __amdgpu_buffer_rsrc_t rbytes = part_rsrc(A.bytes, 0xfffffff0u);
    const PartLink &L = A.link[0];
    uint32_t par = 0, nb_[kA2U], ne_[kA2U], sl_[kA2U];
    PartId it[kA2U];
    {
        const uint32_t t = gt0 + blockIdx.x / kPGroups;
#pragma unroll
        for (uint32_t u = 0; u < kA2U; u++) {
            offsets(t < gt1 ? t : gt0, u, nb_[u], ne_[u], sl_[u]);
            part_id_load(rbytes, nb_[u], ne_[u], it[u]);
        }
    }
    for (uint32_t t = gt0 + blockIdx.x / kPGroups; t < gt1; t += tstep, par ^= 1) {
        uint32_t *scnt = scnt2[par];
        uint32_t rv[kA2U][KM], rp[kA2U][KM];
        bool act[kA2U];
        // pre: this tile's register words, loaded after hashing and examined
        // after the scan (their latency hidden by the probes and the sort)
        uint32_t hv[kA2U], wv[kA2U];
        const uint32_t tn = t + tstep < gt1 ? t + tstep : t;
        uint32_t slc[kA2U];
#pragma unroll
        for (uint32_t u = 0; u < kA2U; u++) {
            slc[u] = sl_[u];
            offsets(tn, u, nb_[u], ne_[u], sl_[u]);
        }
#pragma unroll
        for (uint32_t u = 0; u < kA2U; u++) {
            const uint32_t lu = u * kA2Threads + tid;
            const uint32_t i = t * kTile + lu;
            act[u] = i < A.n;
            uint64_t ha, hb, hh;
            part_hash3(A.bytes, it[u], ha, hb, hh);
            hv[u] = kPcErr;
            wv[u] = 0;
            if (act[u]) {
                uint32_t idx, rank;
                hll_patlen(hh, idx, rank);
                if (!kPre) {
                    nt_st<8>(A.hllw + i, idx | (rank << 16));
                } else if (slc[u] < A.nslots) {
                    hv[u] = idx | (rank << 16);
                    wv[u] = *reinterpret_cast<const uint32_t *>(A.regs + (uint64_t(slc[u]) << kHllP) +
                                                                (idx & ~3u));
                }
                nt_st<8>(A.fail + i, uint8_t(0));
            }
            // bit 19 + tile_log of a record: its slice's parity (pass B's pairs)
            const uint32_t rbase = (lu << kPSliceLog) | 0x80000000u;
            ProbeWalk32 wk;
            wk.init(ha, hb, part_div(L));
#pragma unroll
            for (int q = 0; q < KM; q++) {
                const uint32_t x = wk.x;
                const uint32_t g = x >> kPSliceLog;
                rv[u][q] = (x & kPSliceMask) | ((g & 1u) << (kPSliceLog + kTileLog)) | rbase;
                // no branch: a lane past the batch counts into scnt[S], which
                // the exclusive scan leaves out (it becomes the tile's total),
                // so its records land past the tile's end, never copied out;
                // the swipe's 11 returning atomics are in flight together
                rp[u][q] = atomicAdd(&scnt[act[u] ? g : S], 1u);
                if (q + 1 < KM) wk.step(L.d);
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this swipe's 11 atomics, once
        }
        __syncthreads();
#pragma unroll
        for (uint32_t u = 0; u < kA2U; u++) part_id_load(rbytes, nb_[u], ne_[u], it[u]);  // the next tile's ids
        // exclusive scan of the counts in scnt[0..S] (scnt[S] becomes the tile's total)
        constexpr int kPer = (kPMaxSlices + 1) / kA2Threads;
        uint32_t v[kPer], s = 0;
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            v[j] = scnt[tid * kPer + j] - ((tid * kPer + j) << 16);
            s += v[j];
        }
        uint32_t incl = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= uint32_t(o)) incl += y;
        }
        if (lane == 63) swsum[wave] = incl;
        __syncthreads();
        uint32_t run = incl - s;
        for (uint32_t w = 0; w < wave; w++) run += swsum[w];
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            scnt[tid * kPer + j] = run;
            run += v[j];
        }
        __syncthreads();
        if (kPre) {
            // rank 0: the register already holds at least this rank (registers
            // only grow, so pass C may skip it); else pass C's CAS starts from
            // the word read here
#pragma unroll
            for (uint32_t u = 0; u < kA2U; u++) {
                const uint32_t i = t * kTile + u * kA2Threads + tid;
                if (act[u]) {
                    uint32_t h = hv[u];
                    if (h != kPcErr && ((wv[u] >> ((h & 3u) * 8)) & 0xffu) >= (h >> 16)) h &= 0xffffu;
                    A.hllw[i] = h;
                    A.oldw[i] = wv[u];
                }
            }
        }
        for (uint32_t g = tid; g <= S; g += kA2Threads) A.off[size_t(g) * A.off_stride + t] = scnt[g];
#pragma unroll
        for (uint32_t u = 0; u < kA2U; u++)
#pragma unroll
            for (int q = 0; q < KM; q++)
                srec[scnt[rp[u][q] >> 16] + (rp[u][q] & 0xffffu)] = rv[u][q];
        for (uint32_t g = tid; g <= S; g += kA2Threads) scnt2[par ^ 1][g] = g << 16;
        __syncthreads();
        const uint32_t total = scnt[S];
        part_u32x4 *dst = reinterpret_cast<part_u32x4 *>(A.rec + size_t(t) * A.stride);
        const part_u32x4 *src = reinterpret_cast<const part_u32x4 *>(srec);
        for (uint32_t j = tid; j * 4 < total; j += kA2Threads) nt_st<4>(dst + j, src[j]);
    }
}

// Pass A of the fail-list path (one link, k = KM, slice pairs, 1024-swipe
// tiles, 512 threads x 2 swipes): the same hashing, probes and counting sort
// as k_part_a2 with fewer instructions per probe record (VALU issue bounds
// pass A: 93 M wave-instructions per C3 step, PMC r02):
//   * records are (bit offset in the slice PAIR: 20 bits) | swipe << 20,
//     one v_and_or per probe (pass B of the pair reads the offset as is);
//   * a counter counts in 4s from a bias of (its LDS word index) << 18, so an
//     atomic's return value >> 16 is its own byte offset in the counter
//     array; after the scan the counter holds 4 * start - bias, so a
//     record's byte offset in the tile's LDS record array is the atomic's
//     return value plus that word: one shift and one add per record;
//   * full tiles take a probe loop without the past-the-batch select.
// Counters of the two tile parities are one array (bias index par*2048 + g).
// SKE_A3_ABLATE (diagnostic builds only, answers wrong): 1 no record copy-out,
// 2 no placement / copy-out, 4 counting by plain LDS reads, 8 counting atomics at
// bank-conflict-free addresses, 16 placement base reads at bank-conflict-free addresses
#ifndef SKE_A3_ABLATE
#define SKE_A3_ABLATE 0
#endif
constexpr uint32_t kOORa = 0x80000000u;  // a buffer offset past every range: load 0, store dropped
template <int KM, uint32_t kT = 512, uint32_t kCnt = kPMaxSlices + 1, int kMinBlocks = 2>
__global__ void __launch_bounds__(kT, kMinBlocks * kT / 256) k_part_a3(const PartArgs A) {  // waves per SIMD
    // kCnt: counters per tile parity (slices + the past-the-batch sink); 512
    // for chains of <= 511 slices (C3/C5: 303) shrinks the block's LDS to
    // 49 KiB, so three blocks fit a CU
    constexpr uint32_t kU = 1024 / kT, kTile = 1024;
    constexpr int kPer = kCnt / kT;
    static_assert(kCnt % kT == 0 && 4u * kTile * KM < 65536u, "a rank * 4 stays below bit 16");
    __shared__ __attribute__((aligned(16))) uint32_t srec[kTile * KM];
    __shared__ uint32_t cnt[2 * kCnt];
    __shared__ uint32_t swsum[kT / 64];
    __shared__ uint32_t stot;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t S = A.nslices;
    for (uint32_t c = tid; c < 2 * kCnt; c += kT) cnt[c] = c << 18;
    lds_barrier();
    // Every global load and store below is issued by every wave the same
    // number of times (buffer operations; a lane or a whole call with nothing
    // to move gives an offset past the range): vmcnt counts in issue order and
    // the compiler counts only what every path issues, so with a conditional
    // store between a load and its use the wait for the load also waited for
    // the stores (the copy-out's memory round trip, once per tile).
    const __amdgpu_buffer_rsrc_t roffs = part_rsrc(A.offs, A.offs ? (A.n + 1) * 4 : 0u);
    const __amdgpu_buffer_rsrc_t rhllw = part_rsrc(A.hllw, A.n * 4);
    const __amdgpu_buffer_rsrc_t rfail0 = part_rsrc(A.fail, A.n);
    const __amdgpu_buffer_rsrc_t roff = part_rsrc(A.off, (A.nslices + 1) * A.off_stride * 4);
    auto offsets = [&](uint32_t t, uint32_t u, uint32_t &b, uint32_t &e) {
        const uint32_t i = t * kTile + u * kT + tid;
        const uint32_t ic = i < A.n ? i : A.n - 1;
        const uint32_t lb = __builtin_amdgcn_raw_buffer_load_b32(roffs, ic * 4, 0, nt_aux<2>());
        const uint32_t le = __builtin_amdgcn_raw_buffer_load_b32(roffs, ic * 4 + 4, 0, nt_aux<2>());
        b = A.offs ? lb : ic * A.fixed_w;
        e = A.offs ? le : b + A.fixed_w;
    };
    uint32_t gt0, gt1;
    part_group(A.ntiles, blockIdx.x % kPGroups, gt0, gt1);
    const uint32_t tstep = gridDim.x / kPGroups;
    const __amdgpu_buffer_rsrc_t rbytes = part_rsrc(A.bytes, 0xfffffff0u);
    const PartLink &L = A.link[0];
    uint32_t par = 0, nb_[kU], ne_[kU];
    PartId it[kU];
    {
        const uint32_t t = gt0 + blockIdx.x / kPGroups;
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
            offsets(t < gt1 ? t : gt0, u, nb_[u], ne_[u]);
            part_id_load(rbytes, nb_[u], ne_[u], it[u]);
        }
    }
    const uint8_t *cntb = reinterpret_cast<const uint8_t *>(cnt);
    uint8_t *srecb = reinterpret_cast<uint8_t *>(srec);
    for (uint32_t t = gt0 + blockIdx.x / kPGroups; t < gt1; t += tstep, par ^= 1) {
        const uint32_t cb = par * kCnt;
        uint32_t *cp = cnt + cb;
        uint32_t rv[kU][KM], rp[kU][KM];
        const uint32_t tn = t + tstep < gt1 ? t + tstep : t;
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) offsets(tn, u, nb_[u], ne_[u]);
        const bool full = (t + 1) * kTile <= A.n;  // block-uniform
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
            const uint32_t lu = u * kT + tid;
            const uint32_t i = t * kTile + lu;
            const bool act = i < A.n;
            uint64_t ha, hb, hh;
            part_hash3(A.bytes, it[u], ha, hb, hh);
            {
                uint32_t idx, rank;
                hll_patlen(hh, idx, rank);
                __builtin_amdgcn_raw_buffer_store_b32(idx | (rank << 16), rhllw, act ? i * 4 : kOORa, 0, nt_aux<8>());
                __builtin_amdgcn_raw_buffer_store_b8(uint8_t(0), rfail0, act ? i : kOORa, 0, nt_aux<8>());
            }
            const uint32_t lu20 = lu << 20;
            ProbeWalk32 wk;
            wk.init(ha, hb, part_div(L));
            if (full) {
#pragma unroll
                for (int q = 0; q < KM; q++) {
                    const uint32_t x = wk.x;
                    rv[u][q] = (x & 0xfffffu) | lu20;
                    if constexpr ((SKE_A3_ABLATE & 4) != 0) {
                        rp[u][q] = cp[__builtin_amdgcn_ubfe(x, kPSliceLog, 12)];
                    } else if constexpr ((SKE_A3_ABLATE & 8) != 0) {  // bank-conflict-free atomics
                        rp[u][q] = atomicAdd(&cp[(lane & 31) | ((__builtin_amdgcn_ubfe(x, kPSliceLog, 12) & 7) << 5)], 4u);
                    } else {
                        rp[u][q] = atomicAdd(&cp[__builtin_amdgcn_ubfe(x, kPSliceLog, 12)], 4u);
                    }
                    if (q + 1 < KM) wk.step(L.d);
                }
            } else {
                // a lane past the batch counts into slice S, left out of the
                // scan: its records land past the tile's total, never copied
#pragma unroll
                for (int q = 0; q < KM; q++) {
                    const uint32_t x = wk.x;
                    rv[u][q] = (x & 0xfffffu) | lu20;
                    rp[u][q] = atomicAdd(&cp[act ? __builtin_amdgcn_ubfe(x, kPSliceLog, 12) : S], 4u);
                    if (q + 1 < KM) wk.step(L.d);
                }
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this swipe's atomics, once
        }
        lds_barrier();
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) part_id_load(rbytes, nb_[u], ne_[u], it[u]);  // the next tile's ids
        // exclusive scan of the counts of slices 0..S
        uint32_t v[kPer], s = 0;
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            const uint32_t c = cb + tid * kPer + j;
            v[j] = (cnt[c] - (c << 18)) >> 2;
            s += v[j];
        }
        uint32_t incl = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= uint32_t(o)) incl += y;
        }
        if (lane == 63) swsum[wave] = incl;
        lds_barrier();
        uint32_t run = incl - s;
        for (uint32_t w = 0; w < wave; w++) run += swsum[w];
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            const uint32_t g = tid * kPer + j, c = cb + g;
            __builtin_amdgcn_raw_buffer_store_b32(run, roff, g <= S ? (g * A.off_stride + t) * 4 : kOORa, 0,
                                                  0);  // run starts (pass B)
            if (g == S) stot = run;
            cnt[c] = 4 * run - (c << 18);
            run += v[j];
        }
        lds_barrier();
        if constexpr ((SKE_A3_ABLATE & 2) == 0) {
#pragma unroll
            for (uint32_t u = 0; u < kU; u++)
#pragma unroll
                for (int q = 0; q < KM; q++) {
                    const uint32_t r = rp[u][q];
                    if constexpr ((SKE_A3_ABLATE & 16) != 0)  // bank-conflict-free base reads
                        *reinterpret_cast<uint32_t *>(srecb + ((r + cnt[(lane & 31) | ((r >> 18) & 0x3e0u)]) & 0x7ffcu)) = rv[u][q];
                    else if constexpr ((SKE_A3_ABLATE & 8) != 0)
                        *reinterpret_cast<uint32_t *>(
                            srecb + ((r + *reinterpret_cast<const uint32_t *>(cntb + (r >> 16))) & 0x7ffcu)) = rv[u][q];
                    else
                        *reinterpret_cast<uint32_t *>(srecb + (r + *reinterpret_cast<const uint32_t *>(cntb + (r >> 16)))) =
                            rv[u][q];
                }
        } else {
            uint32_t x = 0;
#pragma unroll
            for (uint32_t u = 0; u < kU; u++)
#pragma unroll
                for (int q = 0; q < KM; q++) x ^= rp[u][q] ^ rv[u][q];
            if (x == 0x12345678u) srec[tid] = x;  // keep the values live
        }
        const uint32_t nb = (cb ^ kCnt);
        for (uint32_t g = tid; g <= S; g += kT) cnt[nb + g] = (nb + g) << 18;
        lds_barrier();
        const uint32_t total = (SKE_A3_ABLATE & 3) ? 0u : (SKE_A3_ABLATE & 24) ? min(stot, kTile * KM) : stot;
        // a fixed number of 16-B pieces per thread (the last ones past the
        // tile's total go out of range); the LDS reads past the records stay
        // inside the block's allocation (the counter table follows srec)
        const __amdgpu_buffer_rsrc_t rdst = part_rsrc(A.rec + size_t(t) * A.stride, A.stride * 4);
        const part_u32x4 *src = reinterpret_cast<const part_u32x4 *>(srec);
        constexpr uint32_t kCo = (kTile * KM / 4 + kT - 1) / kT;
        static_assert(kCo * kT * 16 <= sizeof(srec) + sizeof(cnt), "copy-out reads stay in the block's LDS");
#pragma unroll
        for (uint32_t c = 0; c < kCo; c++) {
            const uint32_t j = c * kT + tid;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, src[j]),
                                                   rdst, j * 4 < total ? j * 16 : kOORa, 0, nt_aux<4>());
        }
    }
}

// k_part_a4: k_part_a3 with the slice counters spread over kCp = 16 copies,
// counter (slice s, copy lane & 15) at word s * 16 + (lane & 15).  A counting
// atomic or a placement read of 32 lanes then meets at most 2 distinct words
// per bank (lanes l and l + 16 share a copy; banks are (word mod 32) for
// ds_add / ds_read_b32, MI355X_MICROARCH.md §LDS) instead of the ~3.5 of 32
// random counters; the run of slice s is the copies' runs in copy order, so
// the scan runs over slices * 16 words (10 per thread, read as 8-byte pairs:
// lane t's pair starts at bank 10t mod 64, all distinct).  One counter table
// (20 KiB for <= 319 slices) keeps two blocks per CU: it is reset to its bias
// after placement, behind one more barrier per tile.
template <int KM, uint32_t kT = 512, uint32_t kSl = 320>
__global__ void __launch_bounds__(kT, 2 * kT / 256) k_part_a4(const PartArgs A) {
    constexpr uint32_t kU = 1024 / kT, kTile = 1024, kCp = 16, kW = kSl * kCp;
    constexpr uint32_t kPer = kW / kT;
    static_assert(kW % kT == 0 && kPer % 2 == 0 && kPer < kCp && 4u * kTile * KM < 65536u && kW < 16384u,
                  "bias << 18 stays in 32 bits; a rank * 4 below bit 16; at most one slice start per thread");
    __shared__ __attribute__((aligned(16))) uint32_t srec[kTile * KM];
    __shared__ __attribute__((aligned(16))) uint32_t cnt[kW];
    __shared__ uint32_t swsum[kT / 64];
    __shared__ uint32_t stot;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t S = A.nslices;
    const uint32_t cpy = (lane & (kCp - 1)) << 2;  // this lane's copy, in bytes
    const uint32_t w0 = tid * kPer;                // the scan's words of this thread
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) cnt[w0 + j] = (w0 + j) << 18;
    lds_barrier();
    auto offsets = [&](uint32_t t, uint32_t u, uint32_t &b, uint32_t &e) {
        const uint32_t i = t * kTile + u * kT + tid;
        const uint32_t ic = i < A.n ? i : A.n - 1;
        b = A.offs ? nt_ld<2>(A.offs + ic) : ic * A.fixed_w;
        e = A.offs ? nt_ld<2>(A.offs + ic + 1) : b + A.fixed_w;
    };
    uint32_t gt0, gt1;
    part_group(A.ntiles, blockIdx.x % kPGroups, gt0, gt1);
    const uint32_t tstep = gridDim.x / kPGroups;
    const __amdgpu_buffer_rsrc_t rbytes = part_rsrc(A.bytes, 0xfffffff0u);
    const PartLink &L = A.link[0];
    uint32_t nb_[kU], ne_[kU];
    PartId it[kU];
    {
        const uint32_t t = gt0 + blockIdx.x / kPGroups;
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
            offsets(t < gt1 ? t : gt0, u, nb_[u], ne_[u]);
            part_id_load(rbytes, nb_[u], ne_[u], it[u]);
        }
    }
    uint8_t *cntb = reinterpret_cast<uint8_t *>(cnt);
    uint8_t *srecb = reinterpret_cast<uint8_t *>(srec);
    for (uint32_t t = gt0 + blockIdx.x / kPGroups; t < gt1; t += tstep) {
        uint32_t rv[kU][KM], rp[kU][KM];
        const uint32_t tn = t + tstep < gt1 ? t + tstep : t;
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) offsets(tn, u, nb_[u], ne_[u]);
        const bool full = (t + 1) * kTile <= A.n;  // block-uniform
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
            const uint32_t lu = u * kT + tid;
            const uint32_t i = t * kTile + lu;
            const bool act = i < A.n;
            uint64_t ha, hb, hh;
            part_hash3(A.bytes, it[u], ha, hb, hh);
            if (act) {
                uint32_t idx, rank;
                hll_patlen(hh, idx, rank);
                nt_st<8>(A.hllw + i, idx | (rank << 16));
                nt_st<8>(A.fail + i, uint8_t(0));
            }
            const uint32_t lu20 = lu << 20;
            ProbeWalk32 wk;
            wk.init(ha, hb, part_div(L));
            if (full) {
#pragma unroll
                for (int q = 0; q < KM; q++) {
                    const uint32_t x = wk.x;
                    rv[u][q] = (x & 0xfffffu) | lu20;
                    rp[u][q] = atomicAdd(reinterpret_cast<uint32_t *>(
                                             cntb + ((__builtin_amdgcn_ubfe(x, kPSliceLog, 12) << 6) | cpy)), 4u);
                    if (q + 1 < KM) wk.step(L.d);
                }
            } else {
                // a lane past the batch counts into slice S, left out of the
                // scan's total: its records land past it, never copied
#pragma unroll
                for (int q = 0; q < KM; q++) {
                    const uint32_t x = wk.x;
                    rv[u][q] = (x & 0xfffffu) | lu20;
                    const uint32_t s = act ? __builtin_amdgcn_ubfe(x, kPSliceLog, 12) : S;
                    rp[u][q] = atomicAdd(reinterpret_cast<uint32_t *>(cntb + ((s << 6) | cpy)), 4u);
                    if (q + 1 < KM) wk.step(L.d);
                }
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this swipe's atomics, once
        }
        lds_barrier();
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) part_id_load(rbytes, nb_[u], ne_[u], it[u]);  // the next tile's ids
        // exclusive scan of the counts of words (slice, copy) 0 .. (S + 1) * 16
        uint32_t v[kPer], s = 0;
#pragma unroll
        for (uint32_t j = 0; j < kPer; j += 2) {
            const uint2 c2 = *reinterpret_cast<const uint2 *>(cnt + w0 + j);
            v[j] = (c2.x - ((w0 + j) << 18)) >> 2;
            v[j + 1] = (c2.y - ((w0 + j + 1) << 18)) >> 2;
            s += v[j] + v[j + 1];
        }
        uint32_t incl = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= uint32_t(o)) incl += y;
        }
        if (lane == 63) swsum[wave] = incl;
        lds_barrier();
        uint32_t run = incl - s;
        for (uint32_t w = 0; w < wave; w++) run += swsum[w];
#pragma unroll
        for (uint32_t j = 0; j < kPer; j += 2) {
            uint2 b2;
            const uint32_t wa = w0 + j, wb = wa + 1;
            if ((wa & (kCp - 1)) == 0 && (wa >> 4) <= S) A.off[size_t(wa >> 4) * A.off_stride + t] = run;
            if (wa == S * kCp) stot = run;
            b2.x = 4 * run - (wa << 18);
            run += v[j];
            if ((wb & (kCp - 1)) == 0 && (wb >> 4) <= S) A.off[size_t(wb >> 4) * A.off_stride + t] = run;
            if (wb == S * kCp) stot = run;
            b2.y = 4 * run - (wb << 18);
            run += v[j + 1];
            *reinterpret_cast<uint2 *>(cnt + wa) = b2;
        }
        lds_barrier();
#pragma unroll
        for (uint32_t u = 0; u < kU; u++)
#pragma unroll
            for (int q = 0; q < KM; q++) {
                const uint32_t r = rp[u][q];
                *reinterpret_cast<uint32_t *>(srecb + (r + *reinterpret_cast<const uint32_t *>(cntb + (r >> 16)))) =
                    rv[u][q];
            }
        lds_barrier();
        const uint32_t total = stot;
#pragma unroll
        for (uint32_t j = 0; j < kPer; j += 2)
            *reinterpret_cast<uint2 *>(cnt + w0 + j) = make_uint2((w0 + j) << 18, (w0 + j + 1) << 18);
        part_u32x4 *dst = reinterpret_cast<part_u32x4 *>(A.rec + size_t(t) * A.stride);
        const part_u32x4 *src = reinterpret_cast<const part_u32x4 *>(srec);
        for (uint32_t j = tid; j * 4 < total; j += kT) nt_st<4>(dst + j, src[j]);
        lds_barrier();  // the counters are reset before the next tile counts
    }
}

// ---------------------------------------------------------------------------
// pass B: LDS-resident slices, probe their runs
// ---------------------------------------------------------------------------
constexpr uint32_t kOOR = 0x80000000u;  // a buffer offset past every range: load 0, store dropped

// The (slice, tile) space is cut into gridDim.x equal contiguous ranges, slice
// major: a block probes one or two slices (restaging the LDS image once) over
// a range of tiles, so the resident grid is balanced to the tile and no block
// waits for a tail.
//
// Memory instructions are what this pass is made of (PMC: the address unit
// busy 84 % of the time, stalled behind L1 misses, when lanes read 4-byte
// pieces), so each one is made to move whole lines: within a slice (or slice
// pair) a wave takes kPbGroup consecutive tiles at a time, 8 lanes per tile
// run, and a lane loads 16 bytes (4 records) -- one instruction reads one
// whole 128-B line of each of 8 runs (pieces start at the line holding the
// run's first record).  2*SP such pieces cover a run of up to 64*SP records
// from its line (37 / 74 at C3 for single slices / pairs); longer runs finish
// in a tail loop.  The few failing
// probes (a member never fails; a non-member's probes fail about half the
// time) are compacted through LDS so a group ends in one fail-byte store
// instruction.  Loads and stores are buffer operations whose out-of-range
// lanes read 0 / are dropped, so every wave issues a fixed number per group
// and the pipeline keeps exact waits: the run boundaries of the group after
// next and the records of the next group are in flight while a group is
// tested.
constexpr uint32_t kPbQueue = 64;  // compacted fail stores per wave and group

// Fail lists (FL, one-link chains in slice pairs, 1024-swipe tiles): instead
// of one byte store per failing probe -- gfx950's L2 passes every store on to
// memory, so 8.8 M scattered byte stores per C3 step were 8.8 M partial-line
// fabric writes (WRITE_SIZE 251 MB for a 16 MB fail array, PMC r02) -- the
// failing swipes of each (slice unit, tile) go to a fixed list of kPbLanes
// u16 swipe indices, flist[unit][tile][], 0xffff = none.  A wave's round
// covers kPbGroup consecutive tiles of one unit, so its lists are one
// 128-byte span, written by one 2-byte-per-lane store instruction.  The
// failures past a list's kPbLanes entries (Poisson(3.7) at C3: ~2 % of the
// lists overflow) and those of the rare long runs keep the byte store; pass C
// (k_part_c_fl) folds the lists of a tile into LDS flags.
// Diagnostic block stamps of pass B (tools/stamps/run_pb_stamps.py; built only
// with -DSKE_STAMPS, the product library has none): thread 0 of every block
// records s_memrealtime (100 MHz) at entry and exit and the block's XCD into a
// side buffer no output depends on.
#ifdef SKE_STAMPS
__device__ unsigned long long *ske_pb_stamp_buf;
hipError_t set_pb_stamp_buffer(void *p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(ske_pb_stamp_buf), &p, sizeof(void *));
}
#define PB_STAMP(k)                                                                                    \
    do {                                                                                               \
        if ((k) == 1) __syncthreads();                                                                 \
        __builtin_amdgcn_sched_barrier(0);                                                             \
        unsigned long long t_;                                                                         \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                \
        __builtin_amdgcn_sched_barrier(0);                                                             \
        if (threadIdx.x == 0 && ske_pb_stamp_buf) {                                                    \
            ske_pb_stamp_buf[blockIdx.x * 4 + (k)] = t_;                                               \
            ske_pb_stamp_buf[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_getreg((3 << 11) | 20);         \
        }                                                                                              \
    } while (0)
#else
#define PB_STAMP(k) \
    do {            \
    } while (0)
#endif
#ifndef SKE_PB_ABLATE
#define SKE_PB_ABLATE 0  // diagnostic builds only: 1 = one slice image per block
#endif
#ifndef SKE_PB_IMG_BATCH
#define SKE_PB_IMG_BATCH 1  // pass B's slice-pair image copy as one batch of loads (0.195 -> 0.190 ms, r03_ab_pass_a_vmcnt.txt)
#endif
// SKE_PB_DPP 1 (default): the fail-list pass B's 8-lane prefix by DPP row
// shifts instead of three ds_bpermute rounds and a broadcast (pass B 0.1966 ->
// 0.1946 ms, three alternations, profiles/r03_ab_pass_a_vmcnt.txt)
#ifndef SKE_PB_DPP
#define SKE_PB_DPP 1
#endif
template <int SP, int R = 2 * SP, bool FL = false>  // R: 16-byte pieces per lane and run (runs of SP slices)
__global__ void __launch_bounds__(kPbBlock, SP == 1 ? 8 : 4) k_part_b(const PartArgs A) {
    PB_STAMP(0);
    const uint32_t tmask = (1u << A.tile_log) - 1;
    __shared__ __attribute__((aligned(16))) uint8_t img[kPSliceBytes * SP];
    __shared__ uint32_t fq[kPbBlock / 64][kPbQueue];
    // this block's share of its group's (slice, tile) space, slice major
    uint32_t gt0, gt1;
    part_group(A.ntiles, blockIdx.x % kPGroups, gt0, gt1);
    const uint32_t gn = gt1 - gt0, nblk = gridDim.x / kPGroups, bi = blockIdx.x / kPGroups;
    const uint32_t nunits = (A.nslices + SP - 1) / SP;
    const uint32_t total = nunits * gn;
    uint32_t w = uint32_t(uint64_t(total) * bi / nblk);
    const uint32_t wend = uint32_t(uint64_t(total) * (bi + 1) / nblk);
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t k = lane / kPbLanes, qq = lane % kPbLanes;
    constexpr uint32_t kWaves = kPbBlock / 64, kStep = kWaves * kPbGroup;
    const __amdgpu_buffer_rsrc_t rrec = part_rsrc(A.rec, A.ntiles * A.stride * 4);
    const __amdgpu_buffer_rsrc_t roff = part_rsrc(A.off, (A.nslices + 1) * A.off_stride * 4);
    const __amdgpu_buffer_rsrc_t rfl = part_rsrc(A.flist, FL ? A.nunits * A.fl_stride * kPbLanes * 2 : 0);
    uint32_t *q = fq[wave];
#if SKE_PB_ABLATE & 1
    bool pb_loaded = false;
#endif
    while (w < wend) {
        // slices g .. g + SP - 1 (SP = 2: one link only, host-checked), so
        // one run per tile covers them all
        const uint32_t unit = w / gn, g = unit * SP, ta = gt0 + w % gn;
        const uint32_t tb = gt1 - ta < wend - w ? gt1 : ta + (wend - w);
        const uint32_t ge = g + SP < A.nslices ? g + SP : A.nslices;
        w += tb - ta;
        uint32_t l = 0;
        while (l + 1 < A.nlinks && g >= A.link[l + 1].slice0) l++;
        const PartLink &L = A.link[l];
        const uint32_t b0 = (g - L.slice0) * kPSliceBytes;
        const uint32_t nb = L.nbytes16 - b0 < kPSliceBytes * SP ? L.nbytes16 - b0 : kPSliceBytes * SP;
#if SKE_PB_ABLATE & 1
        // diagnostic (answers wrong): the image of the block's first unit only
        if (!pb_loaded) {
            pb_loaded = true;
#endif
        lds_barrier();  // every wave is done with the previous slice
#if SKE_PB_IMG_BATCH
        {
            // the pair image in one batch of fixed-count buffer loads (past nb
            // the range check returns zeros, which no record addresses): one
            // memory round trip per unit instead of one per 16 KiB piece
            constexpr uint32_t kCp = kPSliceBytes * SP / (kPbBlock * 16);
            static_assert(kCp * kPbBlock * 16 == kPSliceBytes * SP, "image pieces");
            const __amdgpu_buffer_rsrc_t rimg = part_rsrc(L.bf + b0, nb);
            uint4 piece[kCp];
#pragma unroll
            for (uint32_t c = 0; c < kCp; c++)
                piece[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                         rimg, (c * kPbBlock + threadIdx.x) * 16, 0, 0));
#pragma unroll
            for (uint32_t c = 0; c < kCp; c++)
                *reinterpret_cast<uint4 *>(img + (c * kPbBlock + threadIdx.x) * 16) = piece[c];
        }
#else
        for (uint32_t o = threadIdx.x * 16; o < nb; o += kPbBlock * 16)
            *reinterpret_cast<uint4 *>(img + o) = *reinterpret_cast<const uint4 *>(L.bf + b0 + o);
#endif
        lds_barrier();
#if SKE_PB_ABLATE & 1
        }
#endif
        const __amdgpu_buffer_rsrc_t rfail = part_rsrc(A.fail + size_t(l) * A.fail_stride, A.fail_stride);
        const uint32_t orow = g * A.off_stride, erow = ge * A.off_stride;
        // run boundaries of 8 rounds at once: lane L holds those of tile
        // tg0 + (L / 8) * kStep + L % 8 (0, 0 past tb); a round's lanes take
        // theirs from it with a cross-lane read, so boundary loads are one
        // instruction pair per 8 rounds
        auto load_be8 = [&](uint32_t tg0, uint32_t &B, uint32_t &E) {
            const uint32_t t = tg0 + (lane / kPbGroup) * kStep + lane % kPbGroup;
            const bool in = t < tb;
            B = __builtin_amdgcn_raw_buffer_load_b32(roff, in ? (orow + t) * 4 : kOOR, 0, nt_aux<1>());
            E = __builtin_amdgcn_raw_buffer_load_b32(roff, in ? (erow + t) * 4 : kOOR, 0, nt_aux<1>());
        };
        // 16-byte pieces qq, qq + 8, ... of the run from the 128-B line holding
        // its start: every piece is one whole line (one request, not two)
        auto load_recs = [&](uint32_t tg, uint32_t b, uint32_t e, uint4 (&r)[R]) {
            const uint32_t base = (tg + k) * A.stride, s0 = b & ~31u;
#pragma unroll
            for (uint32_t c = 0; c < R; c++) {
                const uint32_t i = s0 + c * 32 + qq * 4;
                r[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     rrec, i < e ? (base + i) * 4 : kOOR, 0, 2));
            }
        };
        uint32_t tg = ta + wave * kPbGroup;
        uint32_t Bc, Ec, Bn, En;  // boundaries of rounds [8q, 8q + 8) and of the 8 after
        load_be8(tg, Bc, Ec);
        load_be8(tg + kPbGroup * kStep, Bn, En);
        uint32_t bc = __shfl(Bc, k, 64), ec = __shfl(Ec, k, 64);
        uint4 r[R];
        load_recs(tg, bc, ec, r);
        for (uint32_t rr = 0; tg < tb; tg += kStep, rr++) {
            const uint32_t nr = (rr + 1) % kPbGroup;
            if (nr == 0) {  // wave-uniform
                Bc = Bn;
                Ec = En;
                load_be8(tg + (kPbGroup + 1) * kStep, Bn, En);
            }
            const uint32_t b1 = __shfl(Bc, nr * kPbGroup + k, 64), e1 = __shfl(Ec, nr * kPbGroup + k, 64);
            uint4 rn[R];
            load_recs(tg + kStep, b1, e1, rn);
            // the (up to) 4R records of this lane: piece c starts at record
            // lo_c = s0 + c*32 + qq*4; bit j of vm: record j in [bc, ec)
            const uint32_t s0 = bc & ~31u;
            uint32_t rec[4 * R];
#pragma unroll
            for (uint32_t c = 0; c < R; c++) {
                rec[4 * c] = r[c].x;
                rec[4 * c + 1] = r[c].y;
                rec[4 * c + 2] = r[c].z;
                rec[4 * c + 3] = r[c].w;
            }
            auto in_run = [&](uint32_t lo) {  // 4-bit mask of lo + j in [bc, ec), j < 4
                const int32_t hi = int32_t(ec) - int32_t(lo), lw = int32_t(bc) - int32_t(lo);
                const uint32_t nh = uint32_t(hi < 0 ? 0 : (hi > 4 ? 4 : hi));
                const uint32_t nl = uint32_t(lw < 0 ? 0 : (lw > 4 ? 4 : lw));
                return ((1u << nh) - 1u) & ~((1u << nl) - 1u);
            };
            const uint32_t lo0 = s0 + qq * 4;
            uint32_t vm = 0;
#pragma unroll
            for (uint32_t c = 0; c < R; c++) vm |= in_run(lo0 + c * 32) << (4 * c);
            // bit set in the image: its 32-bit word, bit (offset & 31); with
            // slice pairs the record's parity bit selects the image half
            const uint32_t *img32 = reinterpret_cast<const uint32_t *>(img);
            uint32_t okm = 0;
#pragma unroll
            for (uint32_t j = 0; j < 4 * R; j++) {
                const uint32_t rr = rec[j];
                const uint32_t o = FL ? (rr & 0xfffffu)  // k_part_a3: the offset in the pair
                                      : SP == 1 ? (rr & kPSliceMask)
                                                : ((rr & kPSliceMask) | ((rr >> A.tile_log) & kPSliceBits));
                okm |= __builtin_amdgcn_ubfe(img32[o >> 5], rr & 31, 1) << j;
            }
            uint32_t fm = vm & ~okm;
            const uint32_t tbase = (tg + k) << A.tile_log;
            const uint32_t cnt = __builtin_popcount(fm);
            // the record a lane's next failing probe sits in, by a select
            // tree on its index bits (no compare chain)
            auto pick = [&](uint32_t j) {
                constexpr uint32_t kNR = 4 * R, kL = kNR <= 8 ? 3 : (kNR <= 16 ? 4 : 5);
                uint32_t tt[1u << kL];
#pragma unroll
                for (uint32_t i = 0; i < (1u << kL); i++) tt[i] = rec[i < kNR ? i : 0];
#pragma unroll
                for (uint32_t l = 0; l < kL; l++) {
                    const bool bit = (j >> l) & 1u;
#pragma unroll
                    for (uint32_t i = 0; i < ((1u << kL) >> (l + 1)); i++) tt[i] = bit ? tt[2 * i + 1] : tt[2 * i];
                }
                return tt[0];
            };
            if constexpr (FL) {
                // this tile's failures (its kPbLanes lanes): positions by a
                // segment prefix; the first kPbLanes go to the tile's list
                uint32_t incl = cnt;
#if SKE_PB_DPP
                // 8-lane segment prefix by DPP row shifts (VALU, no LDS round
                // trip); the list slots start as 0xffff and get the failures
                q[lane] = 0xffffu;
                __builtin_amdgcn_wave_barrier();
                {
                    uint32_t y = __builtin_amdgcn_update_dpp(0u, incl, 0x111, 0xf, 0xf, true);  // row_shr:1
                    incl += qq >= 1 ? y : 0u;
                    y = __builtin_amdgcn_update_dpp(0u, incl, 0x112, 0xf, 0xf, true);  // row_shr:2
                    incl += qq >= 2 ? y : 0u;
                    y = __builtin_amdgcn_update_dpp(0u, incl, 0x114, 0xf, 0xf, true);  // row_shr:4
                    incl += qq >= 4 ? y : 0u;
                }
#else
#pragma unroll
                for (uint32_t o = 1; o < kPbLanes; o <<= 1) {
                    const uint32_t y = __shfl_up(incl, o, 64);
                    if (qq >= o) incl += y;
                }
                const uint32_t tot = __shfl(incl, k * kPbLanes + kPbLanes - 1, 64);
#endif
                uint32_t pos = incl - cnt;
                while (fm) {
                    const uint32_t j = __builtin_ctz(fm);
                    fm &= fm - 1;
                    const uint32_t at = (pick(j) >> 20) & tmask;  // k_part_a3's swipe field
                    if (pos < kPbLanes) q[k * kPbLanes + pos] = at;
                    else __builtin_amdgcn_raw_buffer_store_b8(uint8_t(1), rfail, tbase + at, 0, 0);  // overflow
                    pos++;
                }
                __builtin_amdgcn_wave_barrier();
                // lane (k, qq) writes entry qq of tile tg + k's list (tiles past
                // this block's range belong to another wave: not written)
#if SKE_PB_DPP
                const uint32_t v = q[lane];
#else
                const uint32_t v = qq < tot ? q[lane] : 0xffffu;
#endif
                const uint32_t fo = ((unit * A.fl_stride + tg + k) * kPbLanes + qq) * 2;
                __builtin_amdgcn_raw_buffer_store_b16(uint16_t(v), rfl, tg + k < tb ? fo : kOOR, 0, 0);
                __builtin_amdgcn_wave_barrier();
            } else {
                // compact the failing swipes of the wave: this lane's count, the
                // wave's exclusive prefix, one store instruction per 64 of them
                uint32_t incl = cnt;
#pragma unroll
                for (uint32_t o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_up(incl, o, 64);
                    if (lane >= o) incl += y;
                }
                const uint32_t nq = __shfl(incl, 63, 64);
                uint32_t pos = incl - cnt;
                while (fm) {
                    const uint32_t j = __builtin_ctz(fm);
                    fm &= fm - 1;
                    const uint32_t at = tbase + ((pick(j) >> kPSliceLog) & tmask);
                    if (pos < kPbQueue) q[pos] = at;
                    else __builtin_amdgcn_raw_buffer_store_b8(uint8_t(1), rfail, at, 0, 0);  // overflow
                    pos++;
                }
                __builtin_amdgcn_wave_barrier();
                if (nq) {
                    const uint32_t at = q[lane];
                    __builtin_amdgcn_raw_buffer_store_b8(uint8_t(1), rfail, lane < nq ? at : kOOR, 0, 0);
                }
                __builtin_amdgcn_wave_barrier();
            }
            if (ec - s0 > 32 * R) {  // rare: a long run
                const uint32_t base = (tg + k) * A.stride;
                for (uint32_t i = s0 + 32 * R + qq; i < ec; i += kPbLanes) {
                    const uint32_t rr = __builtin_amdgcn_raw_buffer_load_b32(rrec, (base + i) * 4, 0, 0);
                    const uint32_t o = FL ? (rr & 0xfffffu)
                                          : SP == 1 ? (rr & kPSliceMask)
                                                    : ((rr & kPSliceMask) | ((rr >> A.tile_log) & kPSliceBits));
                    if (!((img[o >> 3] >> (o & 7)) & 1))
                        __builtin_amdgcn_raw_buffer_store_b8(uint8_t(1), rfail,
                                                             tbase + ((rr >> (FL ? 20 : kPSliceLog)) & tmask), 0, 0);
                }
            }
#pragma unroll
            for (uint32_t c = 0; c < R; c++) r[c] = rn[c];
            bc = b1;
            ec = e1;
        }
    }
    PB_STAMP(1);
}

// ---------------------------------------------------------------------------
// pass C: answers and register max
// ---------------------------------------------------------------------------
__device__ __forceinline__ void part_reg_max(uint32_t *w, uint32_t sh, uint32_t rank, uint32_t old) {
    while (((old >> sh) & 0xffu) < rank) {
        const uint32_t prev = atomicCAS(w, old, (old & ~(0xffu << sh)) | (rank << sh));
        if (prev == old) return;
        old = prev;
    }
}

template <int U>
__global__ void __launch_bounds__(kPcBlock) k_part_c(const PartArgs A) {
    const uint32_t T = kPcBlock, tid = threadIdx.x;
    uint32_t gt0, gt1;
    part_group(A.ntiles, blockIdx.x % kPGroups, gt0, gt1);
    const uint64_t tile = uint64_t(1) << A.tile_log;
    const uint64_t end = uint64_t(gt1) * tile < A.n ? uint64_t(gt1) * tile : A.n;
    const uint64_t stride = uint64_t(gridDim.x / kPGroups) * T * U;
    for (uint64_t base = uint64_t(gt0) * tile + uint64_t(blockIdx.x / kPGroups) * T * U; base < end;
         base += stride) {
        bool valid[U];
        uint32_t *w[U];
        uint32_t rank[U], sh[U], cur[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t i = base + uint64_t(u) * T + tid;
            valid[u] = false;
            w[u] = nullptr;
            rank[u] = 0;
            sh[u] = 0;
            cur[u] = 0;
            if (i < end) {
                for (uint32_t l = 0; l < A.nlinks; l++) valid[u] |= nt_ld<16>(A.fail + size_t(l) * A.fail_stride + i) == 0;
                if (valid[u] && A.pre) {
                    // pass A read the register: only raises remain, from its word
                    const uint32_t hv = A.hllw[i];
                    if (hv == kPcErr) {
                        atomicOr(A.err, 1u);
                    } else if (hv >> 16) {
                        const uint32_t s = A.slot[i];
                        w[u] = reinterpret_cast<uint32_t *>(A.regs + (uint64_t(s) << kHllP) + (hv & 0xfffcu));
                        sh[u] = (hv & 3) * 8;
                        rank[u] = hv >> 16;
                        cur[u] = A.oldw[i];
                    }
                } else if (valid[u]) {
                    const uint32_t s = nt_ld<16>(A.slot + i);
                    if (s >= A.nslots) {
                        atomicOr(A.err, 1u);
                    } else {
                        const uint32_t hv = nt_ld<16>(A.hllw + i);
                        const uint32_t ridx = hv & 0xffffu;
                        w[u] = reinterpret_cast<uint32_t *>(A.regs + (uint64_t(s) << kHllP) + (ridx & ~3u));
                        sh[u] = (ridx & 3) * 8;
                        rank[u] = hv >> 16;
                    }
                }
            }
        }
        if (!A.pre) {
#pragma unroll
            for (int u = 0; u < U; u++) cur[u] = w[u] ? nt_ld<32>(w[u]) : 0xffffffffu;
        }
#pragma unroll
        for (int u = 0; u < U; u++)
            if (w[u]) part_reg_max(w[u], sh[u], rank[u], cur[u]);
        if (A.out) {
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint64_t i = base + uint64_t(u) * T + tid;
                if (i < end) nt_st<16>(A.out + i, uint8_t(valid[u]));
            }
        }
    }
}

// Pass C over pass B's fail lists (one-link chains, 1024-swipe tiles): a
// block takes runs of kPbGroup consecutive tiles of its XCD group (the span
// one pass-B round writes, so a unit's lists for the run are one 128-byte
// line, loaded by 8 lanes together), marks the listed swipes in LDS, and
// after one barrier runs k_part_c's per-swipe answer and register max over
// the run's tiles -- the next tile's fail bytes (list overflows), slots and
// HLL words in flight while a tile's CASes are, every CAS of a tile issued
// before any is settled.  Marks carry the run's index: nothing is cleared.
// SKE_PC_FIXED 1: pass C's loads and stores at a fixed count per tile (as pass
// A's); measured equal at C3 (0.408 vs 0.409 ms, three alternations,
// profiles/r03_ab_pass_a_vmcnt.txt): pass C is bound by the memory side's
// random requests, not by its waves' waits.  Default 0.
#ifndef SKE_PC_FIXED
#define SKE_PC_FIXED 0
#endif
template <int U>
__global__ void __launch_bounds__(kPcBlock) k_part_c_fl(const PartArgs A) {
    static_assert(kPcBlock * U == 1024, "one 1024-swipe tile per sub-step");
    constexpr uint32_t kRun = kPbGroup;  // tiles per block iteration
    __shared__ uint16_t mark[kRun * 1024];
    const uint32_t tid = threadIdx.x;
    for (uint32_t j = tid; j < kRun * 1024; j += kPcBlock) mark[j] = 0;
    uint32_t gt0, gt1;
    part_group(A.ntiles, blockIdx.x % kPGroups, gt0, gt1);
    const uint32_t nblk = gridDim.x / kPGroups;
    const uint32_t npieces = A.nunits * kRun;  // 16-B lists of one run
    const __amdgpu_buffer_rsrc_t rfl = part_rsrc(A.flist, A.nunits * A.fl_stride * kPbLanes * 2);
    struct In {
        uint32_t fb[U], sl[U], hv[U];
    };
#if SKE_PC_FIXED
    // every global load and store of a tile is issued a fixed number of times
    // (buffer operations out of range for lanes with nothing to move; the
    // pre-check load of a lane without a register reads the slab's first
    // word), so the wait for the next tile's streams does not also wait for
    // this tile's answer stores (see k_part_a3)
    const __amdgpu_buffer_rsrc_t rfb = part_rsrc(A.fail, A.n), rsl = part_rsrc(A.slot, A.n * 4),
                                 rhv = part_rsrc(A.hllw, A.n * 4), rout = part_rsrc(A.out, A.out ? A.n : 0u);
    auto load = [&](uint32_t t, uint32_t tend, In &in) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = t * 1024 + uint32_t(u) * kPcBlock + tid;
            const uint32_t oor = uint32_t(!(t < tend && i < A.n)) << 31;
            const uint32_t fb = __builtin_amdgcn_raw_buffer_load_b8(rfb, i | oor, 0, nt_aux<16>());
            in.fb[u] = oor ? 1u : fb;
            in.sl[u] = __builtin_amdgcn_raw_buffer_load_b32(rsl, (i * 4) | oor, 0, nt_aux<16>());
            in.hv[u] = __builtin_amdgcn_raw_buffer_load_b32(rhv, (i * 4) | oor, 0, nt_aux<16>());
        }
    };
#else
    auto load = [&](uint32_t t, uint32_t tend, In &in) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = t * 1024 + uint32_t(u) * kPcBlock + tid;
            const bool act = t < tend && i < A.n;
            in.fb[u] = act ? nt_ld<16>(A.fail + i) : 1u;
            in.sl[u] = act ? nt_ld<16>(A.slot + i) : 0u;
            in.hv[u] = act ? nt_ld<16>(A.hllw + i) : 0u;
        }
    };
#endif
    lds_barrier();
    for (uint32_t r0 = gt0 + (blockIdx.x / kPGroups) * kRun; r0 < gt1; r0 += nblk * kRun) {
        const uint32_t r1 = r0 + kRun < gt1 ? r0 + kRun : gt1;
        const uint16_t ep = uint16_t(r0 / kRun + 1);  // < 2^16: sub-batches hold <= 16384 tiles
        In cur;
        load(r0, r1, cur);
        // the run's lists: piece p = (unit p / kRun, tile r0 + p % kRun)
        for (uint32_t p0 = 0; p0 < npieces; p0 += 4 * kPcBlock) {
            part_u32x4 e[4];
            bool ok[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t p = p0 + uint32_t(j) * kPcBlock + tid;
                const uint32_t un = p / kRun, tt = r0 + p % kRun;
                ok[j] = p < npieces && tt < r1;
                e[j] = __builtin_bit_cast(part_u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                         rfl, ok[j] ? (un * A.fl_stride + tt) * kPbLanes * 2 : kOOR, 0, 0));
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t base = ((p0 + uint32_t(j) * kPcBlock + tid) % kRun) * 1024;
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const uint32_t lo = e[j][c] & 0xffffu, hi = e[j][c] >> 16;
                    if (ok[j] && lo != 0xffffu) mark[base + (lo & 1023u)] = ep;
                    if (ok[j] && hi != 0xffffu) mark[base + (hi & 1023u)] = ep;
                }
            }
        }
        lds_barrier();
        for (uint32_t t = r0; t < r1; t++) {
            In nxt;
            load(t + 1, r1, nxt);
            const uint16_t *mk = mark + (t - r0) * 1024;
            bool valid[U];
            uint32_t *w[U];
            uint32_t rank[U], sh[U], cw[U], seen[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t i = t * 1024 + uint32_t(u) * kPcBlock + tid;
                valid[u] = i < A.n && cur.fb[u] == 0 && mk[uint32_t(u) * kPcBlock + tid] != ep;
                w[u] = nullptr;
                rank[u] = sh[u] = 0;
                if (valid[u]) {
                    if (cur.sl[u] >= A.nslots) {
                        atomicOr(A.err, 1u);
                    } else {
                        const uint32_t ridx = cur.hv[u] & 0xffffu;
                        w[u] = reinterpret_cast<uint32_t *>(A.regs + (uint64_t(cur.sl[u]) << kHllP) + (ridx & ~3u));
                        sh[u] = (ridx & 3) * 8;
                        rank[u] = cur.hv[u] >> 16;
                    }
                }
            }
#if SKE_PC_FIXED
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t x = nt_ld<32>(w[u] ? w[u] : reinterpret_cast<uint32_t *>(A.regs));
                cw[u] = w[u] ? x : 0xffffffffu;
            }
#else
#pragma unroll
            for (int u = 0; u < U; u++) cw[u] = w[u] ? nt_ld<32>(w[u]) : 0xffffffffu;
#endif
            // every raising CAS of the tile in flight at once, then settled
            // (a lost race retries from the word the CAS returned)
#pragma unroll
            for (int u = 0; u < U; u++) {
                seen[u] = cw[u];
                if (w[u] && ((cw[u] >> sh[u]) & 0xffu) < rank[u])
                    seen[u] = atomicCAS(w[u], cw[u], (cw[u] & ~(0xffu << sh[u])) | (rank[u] << sh[u]));
            }
#if SKE_PC_FIXED
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t i = t * 1024 + uint32_t(u) * kPcBlock + tid;
                __builtin_amdgcn_raw_buffer_store_b8(uint8_t(valid[u]), rout, i < A.n ? i : kOOR, 0, nt_aux<16>());
            }
#else
            if (A.out) {
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const uint32_t i = t * 1024 + uint32_t(u) * kPcBlock + tid;
                    if (i < A.n) nt_st<16>(A.out + i, uint8_t(valid[u]));
                }
            }
#endif
#pragma unroll
            for (int u = 0; u < U; u++)
                if (w[u] && seen[u] != cw[u]) part_reg_max(w[u], sh[u], rank[u], seen[u]);
            cur = nxt;
        }
        lds_barrier();  // the marks are rewritten by the next run
    }
}

// ---------------------------------------------------------------------------
// PFADD by owned register lines (passes C2, D, E): the valid swipes' register
// updates are partitioned by register line, each line is owned by one block,
// gathered once into LDS, raised there and written back whole.  No global
// atomics: at C3 the CAS form above issues ~8.6M memory-side atomics and
// 14.4M one-sector pre-checks per 16M-swipe step, while the step touches only
// ~3.9M distinct 128-B lines.
//
//   C2 (k_part_c2)  per group of 8 tiles (8192 swipes): answers, and one 8-B
//                   record (line | reg-in-line, rank) per valid swipe,
//                   counting-sorted by level-1 bucket h1 = hash(line) >> 25
//                   (128 buckets) into the group's region; run starts per
//                   (bucket, group), bucket major.
//   S  (k_part_hscan) per bucket: exclusive prefix of its runs over groups.
//   D  (k_part_hd)  per chunk of kHChunk records of one bucket's stream:
//                   counting sort by level-2 sub-bucket (64 per bucket).
//   E  (k_part_he)  per sub-bucket (8192 in all): the distinct lines of its
//                   records into an LDS table, those lines gathered into LDS
//                   (kHLines at a time), every record's byte max in LDS
//                   (ds CAS), the lines that changed stored back whole.  A
//                   line that does not fit the table takes the CAS path.
// Every register of a line is updated by the one block owning the line, so
// the order of updates is free (max is commutative) and the result equals
// the sequential hllAdd()s of attendance_processor.py:127-129.
constexpr uint32_t kHGroupTiles = 8;
constexpr uint32_t kHGroup = kHGroupTiles * kPaBlock;  // swipes per level-1 group
constexpr uint32_t kH1 = 128;                          // level-1 buckets
constexpr uint32_t kH2 = 64;                           // level-2 sub-buckets per bucket
constexpr uint32_t kHChunk = 8192;                     // records per level-2 chunk
constexpr uint32_t kHTab = 2048;                       // level-3 line table entries
constexpr uint32_t kHLines = 384;                      // lines gathered per round (48 KiB)
constexpr uint32_t kHeBlock = 512;
constexpr uint32_t kHProbe = 32;                       // longest probe chain of the line table

struct HllArgs {
    uint32_t *r1;      // [ngroups][kHGroup] x 2 u32: (line, reg-in-line | rank << 8)
    uint32_t *o1;      // [kH1 + 1][o_stride] run starts per group, bucket major
    uint32_t *p1;      // [kH1][o_stride] exclusive prefix over groups; [h][ngroups] = total
    uint32_t *r2;      // [maxchunks][kHChunk] x 2 u32
    uint32_t *o2;      // [maxchunks][kH2 + 1]
    uint32_t *cst;     // [kH1][c_stride] group holding the first record of each chunk
    uint32_t ngroups, o_stride, maxchunks, c_stride;
};

__device__ __forceinline__ uint32_t hline_mix(uint32_t line) {
    uint32_t x = line * 0x9E3779B1u;
    x ^= x >> 15;
    x *= 0x85EBCA77u;
    x ^= x >> 13;
    return x;
}
__device__ __forceinline__ uint32_t hl_b1(uint32_t m) { return m >> 25; }          // 7 bits
__device__ __forceinline__ uint32_t hl_b2(uint32_t m) { return (m >> 19) & 63u; }  // 6 bits
__device__ __forceinline__ uint32_t hl_slot(uint32_t m) { return m & (kHTab - 1); }

// exclusive scan of cnt[0..n) in place by one block (n <= 4 * blockDim.x);
// returns the total; `tmp` holds blockDim.x / 64 words
__device__ uint32_t block_excl_scan(uint32_t *cnt, uint32_t n, uint32_t *tmp) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x / 64;
    uint32_t v[4], s = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t i = tid * 4 + j;
        v[j] = i < n ? cnt[i] : 0;
        s += v[j];
    }
    uint32_t incl = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= uint32_t(o)) incl += y;
    }
    __syncthreads();
    if (lane == 63) tmp[wave] = incl;
    __syncthreads();
    uint32_t run = incl - s, total = 0;
    for (uint32_t w = 0; w < nw; w++) {
        if (w < wave) run += tmp[w];
        total += tmp[w];
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t i = tid * 4 + j;
        if (i < n) cnt[i] = run;
        run += v[j];
    }
    __syncthreads();
    return total;
}

__global__ void __launch_bounds__(kPaBlock) k_part_c2(const PartArgs A, const HllArgs H) {
    __shared__ __attribute__((aligned(16))) uint2 srec[kHGroup];  // 64 KiB
    __shared__ uint32_t hcnt[kH1 + 1];
    __shared__ uint32_t tmp[kPaBlock / 64];
    const uint32_t tid = threadIdx.x;
    // groups of this block's XCD group (see part_group), round robin
    const uint32_t x = blockIdx.x % kPGroups, nbk = gridDim.x / kPGroups;
    const uint32_t g0 = uint32_t(uint64_t(H.ngroups) * x / kPGroups);
    const uint32_t g1 = uint32_t(uint64_t(H.ngroups) * (x + 1) / kPGroups);
    for (uint32_t gg = g0 + blockIdx.x / kPGroups; gg < g1; gg += nbk) {
        if (tid <= kH1) hcnt[tid] = 0;
        __syncthreads();
        uint32_t line[kHGroupTiles], rr[kHGroupTiles], hp[kHGroupTiles];
#pragma unroll
        for (uint32_t u = 0; u < kHGroupTiles; u++) {
            const uint32_t i = gg * kHGroup + u * kPaBlock + tid;
            hp[u] = 0xffffffffu;
            if (i >= A.n) continue;
            bool valid = false;
            for (uint32_t l = 0; l < A.nlinks; l++) valid |= A.fail[size_t(l) * A.fail_stride + i] == 0;
            if (A.out) A.out[i] = valid;
            if (!valid) continue;
            const uint32_t sl = A.slot[i];
            if (sl >= A.nslots) {
                atomicOr(A.err, 1u);
                continue;
            }
            const uint32_t hv = A.hllw[i], reg = hv & 0xffffu;
            line[u] = sl * (kHllRegs / 128) + (reg >> 7);
            rr[u] = (reg & 127u) | ((hv >> 16) << 8);
            const uint32_t h = hl_b1(hline_mix(line[u]));
            hp[u] = (h << 16) | atomicAdd(&hcnt[h], 1u);
        }
        __syncthreads();
        const uint32_t total = block_excl_scan(hcnt, kH1 + 1, tmp);  // hcnt[kH1] == 0 -> total
        (void)total;
        if (tid <= kH1) H.o1[size_t(tid) * H.o_stride + gg] = hcnt[tid];
#pragma unroll
        for (uint32_t u = 0; u < kHGroupTiles; u++)
            if (hp[u] != 0xffffffffu) srec[hcnt[hp[u] >> 16] + (hp[u] & 0xffffu)] = make_uint2(line[u], rr[u]);
        __syncthreads();
        const uint32_t cnt = hcnt[kH1];
        uint4 *dst = reinterpret_cast<uint4 *>(H.r1 + size_t(gg) * kHGroup * 2);
        const uint4 *src = reinterpret_cast<const uint4 *>(srec);
        for (uint32_t j = tid; j * 2 < cnt; j += kPaBlock) dst[j] = src[j];
        __syncthreads();
    }
}

// per bucket: exclusive prefix of its run lengths over groups (p1[h][ngroups]
// = total), and the group holding the first record of each of its level-2
// chunks (cst[h][c], c < ceil(total / kHChunk))
__global__ void __launch_bounds__(1024) k_part_hscan(const HllArgs H) {
    __shared__ uint32_t tmp[16];
    __shared__ uint32_t carry;
    __shared__ uint32_t buf[4096];
    const uint32_t h = blockIdx.x, tid = threadIdx.x;
    const uint32_t *ob = H.o1 + size_t(h) * H.o_stride, *oe = ob + H.o_stride;
    uint32_t *pp = H.p1 + size_t(h) * H.o_stride;
    uint32_t *cst = H.cst + size_t(h) * H.c_stride;
    if (tid == 0) carry = 0;
    for (uint32_t g0 = 0; g0 < H.ngroups; g0 += 4096) {
        const uint32_t m = H.ngroups - g0 < 4096 ? H.ngroups - g0 : 4096;
        for (uint32_t j = tid; j < m; j += 1024) buf[j] = oe[g0 + j] - ob[g0 + j];
        __syncthreads();
        const uint32_t tot = block_excl_scan(buf, m, tmp);
        const uint32_t c = carry;
        for (uint32_t j = tid; j < m; j += 1024) {
            const uint32_t a = c + buf[j], len = oe[g0 + j] - ob[g0 + j];
            pp[g0 + j] = a;
            // chunks whose first position falls inside this group's run
            for (uint32_t q = (a + kHChunk - 1) / kHChunk; q * kHChunk < a + len; q++) cst[q] = g0 + j;
        }
        __syncthreads();
        if (tid == 0) carry = c + tot;
        __syncthreads();
    }
    if (tid == 0) pp[H.ngroups] = carry;
}

// chunk bases of the buckets: nch[h] = ceil(total[h] / kHChunk), cb = prefix
__device__ void hll_chunks(const HllArgs &H, uint32_t *tot, uint32_t *cb, uint32_t *tmp) {
    const uint32_t tid = threadIdx.x;
    if (tid < kH1) {
        tot[tid] = H.p1[size_t(tid) * H.o_stride + H.ngroups];
        cb[tid] = (tot[tid] + kHChunk - 1) / kHChunk;
    }
    if (tid == kH1) cb[kH1] = 0;
    __syncthreads();
    block_excl_scan(cb, kH1 + 1, tmp);  // cb[kH1] = number of chunks
}

// index of the last entry of a[0..n) (ascending) that is <= v (a[0] <= v)
__device__ __forceinline__ uint32_t lds_last_le(const uint32_t *a, uint32_t n, uint32_t v) {
    uint32_t lo = 0, len = n;
    while (len > 1) {
        const uint32_t half = len / 2;
        if (a[lo + half] <= v) lo += half;
        len -= half;
    }
    return lo;
}

// Level 2: one chunk (kHChunk consecutive records of a bucket's stream) per
// iteration.  Its groups' run starts are staged in LDS; every thread reads 8
// records of the window at once (a binary search in LDS finds each one's
// group), counts their sub-buckets, and after the scan places them from its
// registers.  A window spread over more than kHdGroups groups (only with
// adversarial key skew) reads group by group.
constexpr uint32_t kHdGroups = 1536;
__global__ void __launch_bounds__(1024, 8) k_part_hd(const HllArgs H) {
    __shared__ __attribute__((aligned(16))) uint2 sb[kHChunk];  // sorted by sub-bucket
    __shared__ uint32_t spp[kHdGroups + 1], sob[kHdGroups];
    __shared__ uint32_t tot[kH1], cb[kH1 + 1], tmp[16], c2[kH2 + 1];
    const uint32_t tid = threadIdx.x;
    constexpr uint32_t R = kHChunk / 1024;
    hll_chunks(H, tot, cb, tmp);
    for (uint32_t q = blockIdx.x; q < cb[kH1]; q += gridDim.x) {
        uint32_t h = 0;
        while (h + 1 < kH1 && cb[h + 1] <= q) h++;
        const uint32_t c = q - cb[h], w0 = c * kHChunk;
        const uint32_t w1 = tot[h] - w0 < kHChunk ? tot[h] : w0 + kHChunk;
        const uint32_t *pp = H.p1 + size_t(h) * H.o_stride;
        const uint32_t *ob = H.o1 + size_t(h) * H.o_stride;
        const uint32_t *cst = H.cst + size_t(h) * H.c_stride;
        const uint32_t ga = cst[c];
        const uint32_t gb = w1 < tot[h] ? cst[c + 1] + 1 : H.ngroups;  // groups [ga, gb)
        const uint32_t ng = gb - ga;
        const bool staged = ng <= kHdGroups;  // block-uniform
        if (staged)
            for (uint32_t j = tid; j <= ng; j += 1024) {
                spp[j] = pp[ga + j];
                if (j < ng) sob[j] = ob[ga + j];
            }
        if (tid <= kH2) c2[tid] = 0;
        __syncthreads();
        uint2 r[R];
        uint32_t bp[R];
        const uint2 *r1 = reinterpret_cast<const uint2 *>(H.r1);
#pragma unroll
        for (uint32_t j = 0; j < R; j++) {
            const uint32_t p = w0 + j * 1024 + tid;
            bp[j] = 0xffffffffu;
            if (p >= w1) continue;
            uint32_t g, a, o;
            if (staged) {
                const uint32_t k = lds_last_le(spp, ng, p);
                g = ga + k;
                a = spp[k];
                o = sob[k];
            } else {
                uint32_t lo = ga, hi = gb - 1;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi + 1) / 2;
                    if (pp[mid] <= p) lo = mid; else hi = mid - 1;
                }
                g = lo;
                a = pp[g];
                o = ob[g];
            }
            r[j] = r1[size_t(g) * kHGroup + o + (p - a)];
        }
#pragma unroll
        for (uint32_t j = 0; j < R; j++)
            if (w0 + j * 1024 + tid < w1) {
                const uint32_t b2 = hl_b2(hline_mix(r[j].x));
                bp[j] = (b2 << 16) | atomicAdd(&c2[b2], 1u);
            }
        __syncthreads();
        block_excl_scan(c2, kH2 + 1, tmp);
        uint32_t *o2 = H.o2 + size_t(q) * (kH2 + 1);
        if (tid <= kH2) o2[tid] = c2[tid];
#pragma unroll
        for (uint32_t j = 0; j < R; j++)
            if (bp[j] != 0xffffffffu) sb[c2[bp[j] >> 16] + (bp[j] & 0xffffu)] = r[j];
        __syncthreads();
        const uint32_t cnt = w1 - w0;
        uint4 *dst = reinterpret_cast<uint4 *>(H.r2 + size_t(q) * kHChunk * 2);
        const uint4 *src = reinterpret_cast<const uint4 *>(sb);
        for (uint32_t j = tid; j * 2 < cnt; j += 1024) dst[j] = src[j];
        __syncthreads();
    }
}

__device__ __forceinline__ void lds_byte_max(uint32_t *w, uint32_t sh, uint32_t rank, bool *raised) {
    uint32_t old = *w;
    while (((old >> sh) & 0xffu) < rank) {
        const uint32_t prev = atomicCAS(w, old, (old & ~(0xffu << sh)) | (rank << sh));
        if (prev == old) {
            *raised = true;
            return;
        }
        old = prev;
    }
}

// Level 3: one sub-bucket per iteration.  Its records -- the sub-bucket's run
// of each chunk of the bucket -- are read kHeRec at a time (kHeR per thread,
// all in flight; a binary search over the runs' prefix in LDS finds each
// record) and kept in registers.  For every window: its distinct lines into
// the LDS table, compacted; the lines gathered into LDS kHLines at a time
// (L1-bypassing loads: a line this block stored for an earlier window is read
// back from L2), every record's byte max in LDS, the changed lines stored
// back whole.  A line that misses the full table takes the CAS path.
constexpr uint32_t kHeR = 8;
constexpr uint32_t kHeRec = kHeBlock * kHeR;
constexpr uint32_t kHeRuns = 1024;
__global__ void __launch_bounds__(kHeBlock, 4) k_part_he(const PartArgs A, const HllArgs H) {
    __shared__ uint32_t key[kHTab];      // line + 1, 0 = empty
    __shared__ uint16_t idx[kHTab];      // compact index of an occupied entry
    __shared__ __attribute__((aligned(16))) uint32_t lines[kHLines * 32];
    __shared__ uint8_t dirty[kHLines];
    __shared__ uint32_t lof[kHLines];   // lines of the current round
    __shared__ uint32_t rpre[kHeRuns + 1], rbase[kHeRuns];
    __shared__ uint32_t tot[kH1], cb[kH1 + 1], tmp[kHeBlock / 64], nl;
    const uint32_t tid = threadIdx.x;
    const uint2 *r2 = reinterpret_cast<const uint2 *>(H.r2);
    hll_chunks(H, tot, cb, tmp);
    for (uint32_t sbk = blockIdx.x; sbk < kH1 * kH2; sbk += gridDim.x) {
        const uint32_t h = sbk / kH2, h2 = sbk % kH2;
        const uint32_t q0 = cb[h], q1 = cb[h + 1];
        if (q0 == q1) continue;  // block-uniform
        // the runs of this sub-bucket, kHeRuns chunks at a time
        for (uint32_t qa = q0; qa < q1; qa += kHeRuns) {
            const uint32_t nq = q1 - qa < kHeRuns ? q1 - qa : kHeRuns;
            __syncthreads();
            for (uint32_t j = tid; j < nq; j += kHeBlock) {
                const uint32_t *o2 = H.o2 + size_t(qa + j) * (kH2 + 1);
                const uint32_t b = o2[h2], e = o2[h2 + 1];
                rpre[j] = e - b;
                rbase[j] = (qa + j) * kHChunk + b;
            }
            if (tid == 0) rpre[nq] = 0;
            __syncthreads();
            const uint32_t nrec = block_excl_scan(rpre, nq + 1, tmp);
            for (uint32_t w0 = 0; w0 < nrec; w0 += kHeRec) {
                uint2 r[kHeR];
#pragma unroll
                for (uint32_t j = 0; j < kHeR; j++) {
                    const uint32_t p = w0 + j * kHeBlock + tid;
                    r[j] = make_uint2(0xffffffffu, 0);
                    if (p < nrec) {
                        const uint32_t k = lds_last_le(rpre, nq, p);
                        r[j] = r2[rbase[k] + (p - rpre[k])];
                    }
                }
                for (uint32_t j = tid; j < kHTab; j += kHeBlock) key[j] = 0;
                __syncthreads();
                // 1. distinct lines into the table (linear probing; a full
                //    table leaves the line out: its records take the CAS path)
#pragma unroll
                for (uint32_t j = 0; j < kHeR; j++) {
                    if (r[j].x == 0xffffffffu) continue;
                    uint32_t sl = hl_slot(hline_mix(r[j].x));
                    for (uint32_t probe = 0; probe < kHProbe; probe++) {
                        const uint32_t prev = atomicCAS(&key[sl], 0u, r[j].x + 1);
                        if (prev == 0 || prev == r[j].x + 1) break;
                        sl = (sl + 1) & (kHTab - 1);
                    }
                }
                __syncthreads();
                // 2. compact indices of the occupied entries
                {
                    uint32_t *cidx = lines;  // scratch: kHTab words
                    for (uint32_t j = tid; j < kHTab; j += kHeBlock) cidx[j] = key[j] != 0;
                    __syncthreads();
                    const uint32_t n = block_excl_scan(cidx, kHTab, tmp);
                    for (uint32_t j = tid; j < kHTab; j += kHeBlock)
                        if (key[j]) idx[j] = uint16_t(cidx[j]);
                    if (tid == 0) nl = n;
                    __syncthreads();
                }
                const uint32_t nlines = nl;
                // each record's compact line index (or none)
                uint32_t at[kHeR];
#pragma unroll
                for (uint32_t j = 0; j < kHeR; j++) {
                    at[j] = 0xffffffffu;
                    if (r[j].x == 0xffffffffu) continue;
                    uint32_t sl = hl_slot(hline_mix(r[j].x));
                    for (uint32_t probe = 0; probe < kHProbe; probe++) {
                        const uint32_t k = key[sl];
                        if (k == r[j].x + 1) {
                            at[j] = idx[sl];
                            break;
                        }
                        if (k == 0) break;
                        sl = (sl + 1) & (kHTab - 1);
                    }
                    if (at[j] == 0xffffffffu) {  // not in the table: CAS on the slab
                        const uint32_t reg = r[j].y & 127u;
                        uint32_t *w = reinterpret_cast<uint32_t *>(A.regs + size_t(r[j].x) * 128 + (reg & ~3u));
                        part_reg_max(w, (reg & 3) * 8, r[j].y >> 8,
                                     __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                    }
                }
                // 3. rounds of kHLines lines: the round's line list, the
                //    lines gathered 8 lanes x 16 B each, byte maxes in LDS,
                //    the changed lines stored back whole (plain loads: a line
                //    stored by this block for an earlier window is seen after
                //    the barrier, no other block owns it)
                for (uint32_t r0 = 0; r0 < nlines; r0 += kHLines) {
                    const uint32_t rn = nlines - r0 < kHLines ? nlines - r0 : kHLines;
                    for (uint32_t j = tid; j < kHTab; j += kHeBlock) {
                        const uint32_t k = key[j];
                        if (k && idx[j] >= r0 && idx[j] < r0 + rn) lof[idx[j] - r0] = k - 1;
                    }
                    for (uint32_t j = tid; j < rn; j += kHeBlock) dirty[j] = 0;
                    __syncthreads();
                    const uint4 *src = reinterpret_cast<const uint4 *>(A.regs);
                    for (uint32_t j = tid; j < rn * 8; j += kHeBlock)
                        *reinterpret_cast<uint4 *>(&lines[j * 4]) = src[size_t(lof[j / 8]) * 8 + (j % 8)];
                    __syncthreads();
#pragma unroll
                    for (uint32_t j = 0; j < kHeR; j++) {
                        if (at[j] < r0 || at[j] >= r0 + rn) continue;
                        const uint32_t reg = r[j].y & 127u;
                        bool raised = false;
                        lds_byte_max(&lines[(at[j] - r0) * 32 + reg / 4], (reg & 3) * 8, r[j].y >> 8, &raised);
                        if (raised) dirty[at[j] - r0] = 1;
                    }
                    __syncthreads();
                    uint4 *dst = reinterpret_cast<uint4 *>(A.regs);
                    for (uint32_t j = tid; j < rn * 8; j += kHeBlock)
                        if (dirty[j / 8])
                            dst[size_t(lof[j / 8]) * 8 + (j % 8)] = *reinterpret_cast<const uint4 *>(&lines[j * 4]);
                    __syncthreads();
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static inline unsigned part_grid(uint64_t n, unsigned block, unsigned cap) {
    uint64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    return unsigned(g < cap ? g : cap);
}

// probes per swipe an instantiation of pass A holds: 11 (C3/C5's k = 11
// filter; two blocks per CU) or 22; 0: the chain is not supported
static uint32_t part_km(uint32_t ksum) {
    if (ksum == 0) return 0;
    if (ksum <= 11) return 11;
    if (ksum <= 22) return 22;
    return 0;
}

// records per tile, rounded so tiles start on 128-B lines
static uint32_t part_stride(uint32_t ksum, uint32_t tile_log) { return ((ksum << tile_log) + 31) & ~31u; }

static bool part_plan(const ChainDev &ch, PartArgs *A) {
    if (ch.nlinks < 1 || ch.nlinks > kPMaxLinks) return false;
    uint32_t slices = 0, ksum = 0;
    for (int l = 0; l < ch.nlinks; l++) {
        const LinkDev &L = ch.link[l];
        if (L.div.d > (uint64_t(1) << 31) || L.div.d < 64 || L.k == 0 || L.k > 64) return false;
        PartLink &P = A->link[l];
        P.bf = L.bf;
        P.m = L.div.m;
        P.d = uint32_t(L.div.d);
        P.t = uint32_t(L.div.t);
        P.sh = L.div.sh;
        P.k = L.k;
        P.slice0 = slices;
        P.nbytes16 = uint32_t((((L.div.d >> 3) + 15) >> 4) << 4);
        slices += uint32_t((L.div.d + kPSliceBits - 1) / kPSliceBits);
        ksum += L.k;
    }
    if (slices > kPMaxSlices || part_km(ksum) == 0) return false;
    A->nlinks = uint32_t(ch.nlinks);
    A->nslices = slices;
    A->ksum = ksum;
    A->tile_log = 10;
    A->stride = part_stride(ksum, 10);
    return true;
}

bool part_supported(const ChainDev &ch) {
    PartArgs A{};
    return part_plan(ch, &A);
}

// the scratch of a sub-batch of up to `sub` swipes (slots 28-31 of the context
// scratch: probe records, run boundaries, fail bytes, HLL words)
// the line-owned PFADD's scratch (slots 32-35): level-1 and level-2 records and run tables
static hipError_t hll_scratch(HllArgs *H, uint32_t m, Scratch *scr) {
    H->ngroups = (m + kHGroup - 1) / kHGroup;
    H->o_stride = (H->ngroups + 1 + 15) & ~15u;
    H->maxchunks = (m + kHChunk - 1) / kHChunk + kH1;
    hipError_t e = hipSuccess;
    H->r1 = (uint32_t *)scratch_get(scr, 32, size_t(H->ngroups) * kHGroup * 8, &e);
    if (e == hipSuccess) H->o1 = (uint32_t *)scratch_get(scr, 33, size_t(kH1 + 1) * H->o_stride * 4, &e);
    if (e == hipSuccess) H->p1 = (uint32_t *)scratch_get(scr, 34, size_t(kH1) * H->o_stride * 4, &e);
    if (e == hipSuccess) H->r2 = (uint32_t *)scratch_get(scr, 35, size_t(H->maxchunks) * kHChunk * 8, &e);
    if (e == hipSuccess) H->o2 = (uint32_t *)scratch_get(scr, 36, size_t(H->maxchunks) * (kH2 + 1) * 4, &e);
    H->c_stride = (m + kHChunk - 1) / kHChunk + 2;
    if (e == hipSuccess) H->cst = (uint32_t *)scratch_get(scr, 37, size_t(kH1) * H->c_stride * 4, &e);
    return e;
}

static hipError_t part_scratch(PartArgs *A, uint64_t n, uint32_t sub, Scratch *scr) {
    const uint32_t m = n < sub ? uint32_t(n) : sub;
    // sized for either tile size (1024 or 2048 swipes; the launcher picks)
    const uint32_t ntiles_max = (m + kPaBlock - 1) / kPaBlock;
    const uint64_t rec_words = std::max<uint64_t>(uint64_t(ntiles_max) * part_stride(A->ksum, 10),
                                                  uint64_t((m + 2047) / 2048) * part_stride(A->ksum, 11));
    const uint32_t fstride = (m + 255) & ~255u;
    A->off_stride = (ntiles_max + 15) & ~15u;
    hipError_t e = hipSuccess;
    A->rec = (uint32_t *)scratch_get(scr, 28, size_t(rec_words) * 4, &e);
    if (e == hipSuccess) A->off = (uint32_t *)scratch_get(scr, 29, size_t(A->off_stride) * (A->nslices + 1) * 4, &e);
    if (e == hipSuccess) A->fail = (uint8_t *)scratch_get(scr, 30, size_t(fstride) * A->nlinks, &e);
    if (e == hipSuccess) A->hllw = (uint32_t *)scratch_get(scr, 31, size_t(m) * 4, &e);
    if (e == hipSuccess) A->oldw = (uint32_t *)scratch_get(scr, 42, size_t(m) * 4, &e);
    A->fail_stride = fstride;
    // pass B -> C fail lists of slice pairs (one-link chains)
    A->nunits = (A->nslices + 1) / 2;
    A->fl_stride = A->off_stride;
    if (e == hipSuccess && A->nlinks == 1)
        A->flist = (uint16_t *)scratch_get(scr, 44, size_t(A->nunits) * A->fl_stride * kPbLanes * 2, &e);
    if (e == hipSuccess) {
        HllArgs H{};
        e = hll_scratch(&H, m, scr);
    }
    return e;
}

static uint32_t part_sub(uint32_t sub_opt) {
    uint32_t sub = sub_opt ? sub_opt : kPSub;
    sub = (sub + kPaBlock - 1) / kPaBlock * kPaBlock;
    return sub < kPaBlock ? kPaBlock : (sub > kPSub ? kPSub : sub);
}



// The fail bytes, HLL words and register words pass C reads: two sets, so
// that with pass C on a side stream the next unit's pass A (which writes them)
// does not wait for it (set 1: slots 38, 39, 43; set 0 holds its register words in slot 42)
static hipError_t part_scratch_c(PartArgs *A, uint32_t m, int set, Scratch *scr) {
    if (set == 0) return hipSuccess;  // part_scratch's slots 30, 31
    hipError_t e = hipSuccess;
    A->fail = (uint8_t *)scratch_get(scr, 38, size_t(A->fail_stride) * A->nlinks, &e);
    if (e == hipSuccess) A->hllw = (uint32_t *)scratch_get(scr, 39, size_t(m) * 4, &e);
    if (e == hipSuccess) A->oldw = (uint32_t *)scratch_get(scr, 43, size_t(m) * 4, &e);
    if (e == hipSuccess && A->nlinks == 1)
        A->flist = (uint16_t *)scratch_get(scr, 45, size_t(A->nunits) * A->fl_stride * kPbLanes * 2, &e);
    return e;
}

// both scratch sets, so a graph recorded after a single-batch warm-up can hold
// pipelined many-batch calls too
hipError_t part_reserve(const ChainDev &ch, uint64_t n, uint32_t sub_opt, Scratch *scr) {
    PartArgs A{};
    if (!part_plan(ch, &A)) return hipErrorInvalidValue;
    const uint32_t sub = part_sub(sub_opt);
    hipError_t e = part_scratch(&A, n ? n : 1, sub, scr);
    if (e == hipSuccess) e = part_scratch_c(&A, uint32_t(n < sub ? (n ? n : 1) : sub), 1, scr);
    return e;
}

// Units = (batch, sub-batch of at most `sub` swipes), in order.  Without a
// side stream every pass runs on st.  With one (`side`, events ev[0..3]):
// passes A and B of unit u on st, its pass C on `side` once pass A of unit
// u + 1 is done (ovl 1, event ev[(u + 1) & 1]: pass C of one unit, memory-side
// register atomics, beside pass B of the next, slice probes) or once its own
// pass B is done (ovl 2, event ev[u & 1]: beside pass A of the next, hashing
// and LDS sorting); unit u's pass A first waits for pass C of unit u - 2
// (event ev[2 + (u & 1)]), the last reader of the scratch set it writes; st
// joins `side` at the end.  Results equal the serial order: units touch
// disjoint answers and PFADD is a max.
hipError_t launch_swipes_part(const ChainDev &ch, const PartBatch *bt, uint32_t nb, uint8_t *regs,
                              uint32_t nslots, Scratch *scr, unsigned int *err, int cus, uint32_t sub_opt,
                              int hll_mode, int pb_pairs, int tile_opt, int pre_opt, int ovl, int a_grid, hipStream_t st, hipStream_t side,
                              hipEvent_t *ev, PassHook hook, void *hook_user, int a3_threads,
                              hipStream_t side_a, int c_cus) {
    PartArgs A{};
    if (!part_plan(ch, &A)) return hipErrorInvalidValue;
    const uint32_t sub = part_sub(sub_opt);
    uint64_t nmax = 0;
    for (uint32_t j = 0; j < nb; j++) nmax = bt[j].n > nmax ? bt[j].n : nmax;
    if (nmax == 0) return hipSuccess;
    hipError_t e = part_scratch(&A, nmax, sub, scr);
    if (e != hipSuccess) return e;
    // (set 1 too, even when not pipelined: see part_reserve)
    uint8_t *fail0 = A.fail;
    uint32_t *hllw0 = A.hllw, *oldw0 = A.oldw;
    uint16_t *flist0 = A.flist;
    e = part_scratch_c(&A, uint32_t(nmax < sub ? nmax : sub), 1, scr);
    if (e != hipSuccess) return e;
    uint8_t *fail1 = A.fail;
    uint32_t *hllw1 = A.hllw, *oldw1 = A.oldw;
    uint16_t *flist1 = A.flist;
    A.flist = flist0;
    // ovl 3: pass A of unit u + 1 on side_a (the CUs pass C does not use)
    // beside pass C of unit u on side (c_cus CUs); pass B on st, alone
    const bool split = side && side_a && ovl == 3 && c_cus > 0 && c_cus < cus;
    A.regs = regs;
    A.nslots = nslots;
    A.err = err;
    const uint32_t km = part_km(A.ksum);
    // tiles of 1024 swipes; tile_opt 11: 2048 for a one-link k = 11 chain
    // (k_part_a2<11, 1024>, one block per CU): pass B's runs twice as long
    // (0.287 -> 0.26 ms at C3) but pass A slower (0.276 -> 0.315 ms), no net gain
    const bool one11 = A.nlinks == 1 && A.ksum == 11;
    A.tile_log = (one11 && tile_opt == 11) ? 11 : 10;
    A.stride = part_stride(A.ksum, A.tile_log);
    // the register pre-check moves pass C's random register loads into pass A
    // (VALU / LDS bound, its memory path has room), so pass C touches only the
    // registers that rise (k_part_a2 of 1024-swipe tiles, CAS PFADD)
    A.pre = (pre_opt && hll_mode == 0 && one11 && A.tile_log == 10) ? 1u : 0u;
    // pass B -> C through fail lists (pb_pairs 2): one-link chains probed in
    // slice pairs over 1024-swipe tiles, PFADD by CAS from pass C's own
    // pre-check, passes in stream order (the lists are one buffer)
    const bool flist = pb_pairs == 2 && one11 && A.tile_log == 10 && hll_mode == 0 && !A.pre && (!side || split) &&
                       A.flist != nullptr && (!split || flist1 != nullptr);
    const uint32_t tile = 1u << A.tile_log;
#define SKE_CK(x)                        \
    do {                                 \
        hipError_t e_ = (x);             \
        if (e_ != hipSuccess) return e_; \
    } while (0)
    // pass C of unit u - 1 (with its arguments) waits for pass A of unit u:
    // it then runs beside pass B of unit u (slice probes, one block per CU)
    // and not beside pass A (whose two blocks per CU fill the register file)
    PartArgs prev{};
    uint32_t prev_ms = 0;
    bool have_prev = false;
    auto launch_c = [&](const PartArgs &P, uint32_t ms, hipStream_t sc) -> hipError_t {
        if (hook) hook(hook_user, 2, 0, sc);
        if (hll_mode == 1) {
            // PFADD by owned register lines: C2, S, D, E (timed together as pass C)
            HllArgs H{};
            hipError_t e2 = hll_scratch(&H, ms, scr);
            if (e2 != hipSuccess) return e2;
            hipLaunchKernelGGL(k_part_c2, dim3(unsigned(cus) * 2 / kPGroups * kPGroups), dim3(kPaBlock), 0,
                               sc, P, H);
            hipLaunchKernelGGL(k_part_hscan, dim3(kH1), dim3(1024), 0, sc, H);
            hipLaunchKernelGGL(k_part_hd, dim3(unsigned(cus) * 2), dim3(1024), 0, sc, H);
            hipLaunchKernelGGL(k_part_he, dim3(unsigned(cus) * 2), dim3(kHeBlock), 0, sc, P, H);
        } else if (flist) {
            const unsigned gc = (part_grid(ms, 1024 * kPbGroup, (split ? c_cus : cus) * 8) + kPGroups - 1) / kPGroups *
                                kPGroups;
            hipLaunchKernelGGL(k_part_c_fl<4>, dim3(gc), dim3(kPcBlock), 0, sc, P);
        } else {
            const unsigned gc = (part_grid(ms, kPcBlock * 2, cus * 8) + kPGroups - 1) / kPGroups * kPGroups;
            hipLaunchKernelGGL(k_part_c<2>, dim3(gc), dim3(kPcBlock), 0, sc, P);
        }
        if (hook) hook(hook_user, 2, 1, sc);
        return hipGetLastError();
    };
    uint32_t u = 0;
    for (uint32_t j = 0; j < nb; j++) {
        const PartBatch &B = bt[j];
        // fixed-width ids: a sub-batch's byte offsets (swipe * width) stay 32-bit
        uint32_t subj = sub;
        if (!B.offs && B.fixed_w) {
            const uint64_t cap = (0xffffff00ull / B.fixed_w) / kPaBlock * kPaBlock;
            subj = cap < sub ? uint32_t(cap < kPaBlock ? kPaBlock : cap) : sub;
        }
        for (uint64_t s0 = 0; s0 < B.n; s0 += subj, u++) {
            const uint32_t ms = B.n - s0 < subj ? uint32_t(B.n - s0) : subj;
            const int set = side ? int(u & 1) : 0;
            A.fail = set ? fail1 : fail0;
            A.hllw = set ? hllw1 : hllw0;
            A.oldw = set ? oldw1 : oldw0;
            if (split) A.flist = set ? flist1 : flist0;
            A.fixed_w = B.fixed_w;
            A.n = ms;
            A.ntiles = (ms + tile - 1) / tile;
            A.bytes = B.offs ? B.bytes : B.bytes + s0 * B.fixed_w;
            A.offs = B.offs ? B.offs + s0 : nullptr;
            A.slot = B.slot + s0;
            A.out = B.out ? B.out + s0 : nullptr;
            // pass C of unit u - 2 was the last reader of this scratch set
            hipStream_t sa = st;  // pass A's stream
            if (split) {
                // after the work before this call (u = 0) or pass B of unit u - 1
                // (the probe records and run table), and pass C of unit u - 2
                sa = side_a;
                if (u == 0) SKE_CK(hipEventRecord(ev[1], st));
                SKE_CK(hipStreamWaitEvent(sa, ev[1], 0));
                if (u >= 2) SKE_CK(hipStreamWaitEvent(sa, ev[2 + set], 0));
            } else if (side && u >= 2) {
                SKE_CK(hipStreamWaitEvent(st, ev[2 + set], 0));
            }
            const unsigned acus = unsigned(split ? cus - c_cus : cus);
            const unsigned per_cu = km <= 11 ? (a_grid ? unsigned(a_grid) : 2u) : 1;
            const unsigned ga = unsigned(cus) * per_cu / kPGroups * kPGroups;  // blocks past a group's tiles exit
            if (hook) hook(hook_user, 0, 0, sa);
            if (flist && a3_threads == 1024)  // the fail-list path's own record format (k_part_a3 -> k_part_b<2, 4, true>)
                hipLaunchKernelGGL((k_part_a3<11, 1024>), dim3(acus * 2 / kPGroups * kPGroups), dim3(1024), 0, sa, A);
            else if (flist && A.nslices < 320 && a_grid == 5)  // slice counters in 16 copies
                hipLaunchKernelGGL((k_part_a4<11, 512, 320>), dim3(acus * 2 / kPGroups * kPGroups), dim3(512), 0, sa, A);
            else if (flist && A.nslices < 512 && a_grid == 3)  // small counter table: three blocks per CU
                hipLaunchKernelGGL((k_part_a3<11, 512, 512, 3>), dim3(acus * 3 / kPGroups * kPGroups), dim3(512), 0, sa,
                                   A);
            else if (flist && A.nslices < 512 && (a_grid == 0 || a_grid == 4))  // small counter table, two blocks per CU
                hipLaunchKernelGGL((k_part_a3<11, 512, 512, 2>), dim3(acus * 2 / kPGroups * kPGroups), dim3(512), 0, sa,
                                   A);
            else if (flist)
                hipLaunchKernelGGL((k_part_a3<11, 512>), dim3(acus * 2 / kPGroups * kPGroups), dim3(512), 0, sa, A);
            else if (one11 && A.tile_log == 11)  // RESERVE 0.001 (C3/C5): one link, k = 11
                hipLaunchKernelGGL((k_part_a2<11, 1024>), dim3(unsigned(cus) / kPGroups * kPGroups), dim3(1024),
                                   0, sa, A);
            else if (one11 && A.pre)
                hipLaunchKernelGGL((k_part_a2<11, kA2Threads, 2, true>),
                                   dim3(unsigned(cus) * per_cu / kPGroups * kPGroups), dim3(kA2Threads), 0, sa, A);
            else if (one11)
                hipLaunchKernelGGL((k_part_a2<11>), dim3(unsigned(cus) * per_cu / kPGroups * kPGroups),
                                   dim3(kA2Threads), 0, sa, A);
            else if (km <= 11)
                hipLaunchKernelGGL(k_part_a<11>, dim3(ga), dim3(kPaBlock), 0, sa, A);
            else
                hipLaunchKernelGGL(k_part_a<22>, dim3(ga), dim3(kPaBlock), 0, sa, A);
            if (hook) hook(hook_user, 0, 1, sa);
            if (split) {  // pass B behind pass A
                SKE_CK(hipEventRecord(ev[0], sa));
                SKE_CK(hipStreamWaitEvent(st, ev[0], 0));
            }
            if (side && ovl == 1 && have_prev) {  // C(u - 1) behind A(u) (and so behind B(u - 1))
                SKE_CK(hipEventRecord(ev[set], st));
                SKE_CK(hipStreamWaitEvent(side, ev[set], 0));
                SKE_CK(launch_c(prev, prev_ms, side));
                SKE_CK(hipEventRecord(ev[2 + (set ^ 1)], side));
            }
            // all blocks resident, each an equal share of (slice unit, tile); a
            // one-link chain is probed in slice pairs (128 KiB images, one block
            // per CU): runs twice as long per tile
            const bool pairs = A.nlinks == 1 && pb_pairs;
            const unsigned gb = unsigned(cus) * (pairs ? 1 : 2) / kPGroups * kPGroups;
            if (hook) hook(hook_user, 1, 0, st);
            if (pairs && A.tile_log == 11)  // runs of ~148 records
                hipLaunchKernelGGL((k_part_b<2, 6>), dim3(gb), dim3(kPbBlock), 0, st, A);
            else if (flist)
                hipLaunchKernelGGL((k_part_b<2, 4, true>), dim3(gb), dim3(kPbBlock), 0, st, A);
            else if (pairs)
                hipLaunchKernelGGL(k_part_b<2>, dim3(gb), dim3(kPbBlock), 0, st, A);
            else
                hipLaunchKernelGGL(k_part_b<1>, dim3(gb), dim3(kPbBlock), 0, st, A);
            if (hook) hook(hook_user, 1, 1, st);
            if (split) {  // C(u) behind B(u), beside A(u + 1) on the other CUs
                SKE_CK(hipEventRecord(ev[1], st));
                SKE_CK(hipStreamWaitEvent(side, ev[1], 0));
                SKE_CK(launch_c(A, ms, side));
                SKE_CK(hipEventRecord(ev[2 + set], side));
                have_prev = true;
            } else if (side && ovl == 2) {  // C(u) behind B(u), beside A(u + 1)
                SKE_CK(hipEventRecord(ev[set], st));
                SKE_CK(hipStreamWaitEvent(side, ev[set], 0));
                SKE_CK(launch_c(A, ms, side));
                SKE_CK(hipEventRecord(ev[2 + set], side));
                have_prev = true;
            } else if (side) {
                prev = A;
                prev_ms = ms;
                have_prev = true;
            } else {
                SKE_CK(launch_c(A, ms, st));
            }
            SKE_CK(hipGetLastError());
        }
    }
    if (split && have_prev) {  // join the last unit's pass C (and so every pass before it)
        SKE_CK(hipStreamWaitEvent(st, ev[2 + int((u - 1) & 1)], 0));
    } else if (side && ovl == 2 && have_prev) {  // join the last unit's pass C
        SKE_CK(hipStreamWaitEvent(st, ev[2 + int((u - 1) & 1)], 0));
    } else if (side && have_prev) {  // the last unit's pass C behind its pass B, then join
        const int set = int((u - 1) & 1);
        SKE_CK(hipEventRecord(ev[set], st));
        SKE_CK(hipStreamWaitEvent(side, ev[set], 0));
        SKE_CK(launch_c(prev, prev_ms, side));
        SKE_CK(hipEventRecord(ev[2 + set], side));
        SKE_CK(hipStreamWaitEvent(st, ev[2 + set], 0));
    }
#undef SKE_CK
    return hipGetLastError();
}

}  // namespace ske
