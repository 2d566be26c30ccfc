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
//   pass A             per tile of 1024 swipes: hash each id (MurmurHash64A
//                      a, b, and the HLL hash), walk every link's k probes,
//                      and emit one 4-byte record per probe (its bit offset in
//                      the slice unit | the swipe's index in the tile),
//                      counting-sorted by slice in LDS and written out as one
//                      contiguous run per (tile, slice unit); off[slice][tile]
//                      holds the run boundaries.  Also the HLL word (register
//                      | rank << 16; one-link k = 11 chains: its top byte is
//                      the swipe's overflow flag) and, for other chains, a
//                      cleared fail byte per swipe.
//   pass B             per slice unit (one slice, or a pair of a one-link
//                      chain's adjacent slices), staged into LDS: the unit's
//                      run of every tile in the block's range; a failing
//                      probe's swipe goes to the tile's fail list (one-link
//                      k = 11 chains; a full list's overflow sets the HLL
//                      word's top byte) or sets its fail byte.
//   pass C             per swipe: valid = no failed probe in some link; the
//                      answer; register max (pre-check load, CAS).
//
// Two instantiations of the passes, picked by the host per chain:
//   * one link of k = 11 (C3/C5's RESERVE 0.001 / 1e7 filter, the headline):
//     k_part_a3 -> k_part_b<2, 4, true> -> k_part_c_fl (slice pairs, dense
//     pair runs, fail lists);
//   * any other chain the slice plan takes (several links, or k != 11; up to
//     22 probes per swipe): k_part_a -> k_part_b<1 or 2> -> k_part_c (fail
//     bytes).
// Variants measured slower were removed in round 4 (DESIGN.md §3 keeps their
// numbers): 512-thread pass A without fail lists, 2048-swipe tiles, the
// 16-copy counter table, pass A at three blocks per CU, the register
// pre-check in pass A, PFADD by owned register lines, pass C on a side or
// CU-masked stream; in round 4 also pair runs padded to 128-B lines, the
// tile parity unrolled, and a two-phase pass C.
//
// Placement of blocks on XCDs is a speed matter only; every (tile, slice) run
// is read by exactly one block, and fail marks are only ever set.
#include <algorithm>
#include <cmath>
#include <type_traits>

#include "sketch_common.h"
#include "sketch_internal.h"

namespace ske {

constexpr uint32_t kPaBlock = 1024;
constexpr uint32_t kPbBlock = 1024;
// pass C's block: 1024 threads x 1 swipe per tile (round 4 A/B, three
// alternations: 0.406-0.407 ms at 256 x 4, 0.402 at 512 x 2, 0.400 at 1024 x 1)
#ifndef SKE_PC_BLOCK
#define SKE_PC_BLOCK 1024
#endif
#ifndef SKE_PC_BLOCKS_PER_CU
#define SKE_PC_BLOCKS_PER_CU 8
#endif
constexpr uint32_t kPcBlock = 256;            // k_part_c (fail bytes)
constexpr uint32_t kPSliceMask = kPSliceBits - 1;
constexpr uint32_t kPSliceBytes = kPSliceBits / 8;  // 64 KiB
constexpr uint32_t kPSub = 1u << 26;                // swipes per sub-batch (passes A-B-C), at most
constexpr uint32_t kPbGroup = 8;                    // tiles a pass-B wave reads at once
constexpr uint32_t kPbLanes = 64 / kPbGroup;        // lanes per tile run
constexpr uint32_t kPTileLog = 10;                  // swipes per tile = 1 << kPTileLog
// swipes per tile of the fail-list chains (one link, k = 11: C3 / C5's
// filter): 1024, or 1536 (longer (pair, tile) runs for pass B)
#ifndef SKE_TILE_FL
#define SKE_TILE_FL 1024
#endif
constexpr uint32_t kTileFl = SKE_TILE_FL;
static_assert(kTileFl == 1024 || kTileFl == 1536, "fail-list tiles of 1024 or 1536 swipes");
// pass B's 16-B pieces per lane and run of the fail-list chains: a (pair,
// tile) run of ~74 records (1024-swipe tiles) or ~111 (1536) from the line
// holding its start (runs longer than 32 R - 31 records finish in a tail loop)
constexpr int kPbRFl = kTileFl == 1024 ? 4 : 6;
// pass C (fail lists): threads per block, kTileFl / kPcFlT swipes each per tile
constexpr uint32_t kPcFlT = kTileFl == 1024 ? SKE_PC_BLOCK : 768;

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
    uint32_t *hllw;        // [n] register | rank << 16
    uint32_t fixed_w, n, stride, ntiles, nslices, nlinks, ksum, nslots, fail_stride, off_stride;
    uint16_t *flist;       // [nunits][fl_stride][kPbLanes] fail lists (pass B -> pass C), or nullptr
    uint32_t nunits, fl_stride;
    // group layout (gcap != 0; k_part_a3 / k_part_b<2, 4, true, true>): the
    // runs of a unit over a group of 8 tiles adjacent in rec[group][unit][gcap],
    // a run that does not fit at its tile's place in rec[govf + tile * stride]
    uint32_t gcap, govf;
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
// (group edges on multiples of 8 tiles: pass B's rounds and the group layout's
// 8-tile groups never straddle two XCD groups)
__device__ __forceinline__ void part_group(uint32_t ntiles, uint32_t x, uint32_t &t0, uint32_t &t1) {
    t0 = uint32_t(uint64_t(ntiles) * x / kPGroups) & ~7u;
    t1 = x + 1 == kPGroups ? ntiles : uint32_t(uint64_t(ntiles) * (x + 1) / kPGroups) & ~7u;
}

// Bit (pos & 31) of w: v_bfe_u32 reads only its offset operand's low 5 bits,
// so pos goes in as it is (the compiler's ubfe masks it first: one VALU per
// probe record in pass B)
__device__ __forceinline__ uint32_t part_bit(uint32_t w, uint32_t pos) {
    uint32_t r;
    asm("v_bfe_u32 %0, %1, %2, 1" : "=v"(r) : "v"(w), "v"(pos));
    return r;
}

// ((1 << width) - 1) << offset (width, offset < 32) as one v_bfm_b32
__device__ __forceinline__ uint32_t part_bfm(uint32_t width, uint32_t offset) {
    uint32_t r;
    asm("v_bfm_b32 %0, %1, %2" : "=v"(r) : "v"(width), "s"(offset));
    return r;
}

// Inclusive prefix sum over a wave's 64 lanes on DPP: row shifts 1, 2, 4, 8
// inside 16-lane rows, then row_bcast:15 / row_bcast:31 across rows (gfx9);
// a lane whose source is outside its row adds the identity.  VALU only.
__device__ __forceinline__ uint32_t part_wave_scan(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 into rows 1, 3
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 into rows 2, 3
    return v;
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

// Streams read or written once take the non-temporal policy (`nt`); SKE_NT
// bits select them -- 1 pass B's run boundaries, 2 pass A's ids and offsets,
// 4 pass A's record copy-out, 8 pass A's HLL words and fail bytes, 16 pass
// C's streams (fail bytes, slots, HLL words, answers), 32 pass C's register
// pre-check loads, 64 pass B's probe records.  Measured at C3 (A/B,
// two alternations): records nt: pass B 0.276 -> 0.260 ms; + bits 1|2|4:
// 0.25 ms; bits 8 and 16 neutral to slightly slower; bit 32 makes pass C
// 0.39 -> 0.59 ms (the raising CAS no longer finds its line near).  Default 7.
// (Round 4, final kernels: 15 and 23 within 0.1 % of 7, profiles/r04_ab_nt.txt.)
// Bit 64 (pass B's records) was always on before round 5 (default 71).
// Round 6, the segmented PFADD at 2^28-swipe steps (profiles/r06_ab_nt.txt,
// three sessions, N = 1 and the 8-way shard): pass B's record loads without
// `nt` and the copy-out with it -- pass B 0.39 -> 0.37 ms per 2^25 sub-batch --
// and C1's streams (bit 16) with it -- C1 0.116 -> 0.099 -- and pass A's HLL
// words (bit 8) with it (pass B 0.370 -> 0.364): default 29 (1 | 4 | 8 | 16),
// step 9.2 -> 8.85-8.9 ms; without bit 4, or with bit 64, pass B is back at
// 0.38+; bit 2 (pass A's ids) costs pass B 0.01.
#ifndef SKE_NT
#define SKE_NT 29
#endif
// pass A3's id prefetch distance: 1 -- a tile's ids load after the previous
// tile's atomics (from offsets loaded at that tile's start); 2 -- at the
// previous tile's start, from offsets loaded a tile earlier
#ifndef SKE_PA_AHEAD
#define SKE_PA_AHEAD (kTileFl == 1024 ? 2 : 1)  // (1536-swipe tiles: 2 would spill)
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
// The segmented PFADD's streams (SKE_NT2 bits): 1 C1's level-1 record
// copy-out, 2 D's level-1 record loads, 4 D's level-2 record copy-out, 8 the
// window pass's record loads, 16 its register-image loads (LDS-DMA), 32 its
// line write-back.  Default 0 (round 5's policies).
#ifndef SKE_NT2
#define SKE_NT2 0
#endif
template <int BIT> __device__ __forceinline__ constexpr int nt2_aux() { return (SKE_NT2 & BIT) ? 2 : 0; }
template <int BIT, class T> __device__ __forceinline__ void nt2_st(T *p, T v) {
    if constexpr ((SKE_NT2 & BIT) != 0) __builtin_nontemporal_store(v, p);
    else *p = v;
}

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
    // (an id inside one aligned word needs no second word: its load goes
    // past the range, no memory access; the hash masks those bytes off)
    const uint32_t o1 = (sh && s8 + d.len > 8) ? o0 + 8 : 0xfffffff8u;
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

// Pass A of the fail-list path (one link, k = KM, slice pairs, 1024-swipe
// tiles, 512 threads x 2 swipes: a thread has 128 VGPRs and twice the
// independent work between barriers of a 1024 x 1 block; C3 0.315 -> 0.273
// ms, round 2):
//   * records are (bit offset in the slice PAIR: 20 bits) | swipe << 20,
//     one v_and_or per probe (pass B of the pair reads the offset as is);
//   * a counter counts in 4s from a bias of (its LDS word index) << 18, so an
//     atomic's return value >> 16 is its own byte offset in the counter
//     array; after the scan the counter holds 4 * start - bias, so a
//     record's byte offset in the tile's LDS record array is the atomic's
//     return value plus that word: one shift and one add per record;
//   * full tiles take a probe loop without the past-the-batch select;
//   * the two slices of a pair are counted apart but their runs are
//     adjacent with no gap (dense pair runs, round 4): pass B reads one word
//     per (pair, tile), off[pair][tile] = start | count << 16.  Runs padded
//     to 128-B lines made pass B read 12 % fewer lines but pass A write 21 %
//     more bytes, a net loss (A/B in DESIGN.md section 3);
//   * the counter scan's wave prefix is DPP (part_wave_scan) and a probe's
//     counter address is v_bfe + v_lshl_add (0.238 -> 0.222 ms, round 4).
// Counters of the two tile parities are one array (bias index par*kCnt + g);
// lanes past the batch count into the first pair past the chain (the sink),
// whose records land past the copy-out.  kCnt: 1024 (two counters per
// thread) for chains of < 512 pairs (C3/C5: 152), else 2048.
constexpr uint32_t kOORa = 0x80000000u;  // a buffer offset past every range: load 0, store dropped
#ifndef SKE_PA_WAIT_LAST
#define SKE_PA_WAIT_LAST 1  // round 4 A/B: pass A 0.226-0.230 -> 0.225 ms
#endif
// GL: the group layout (PartArgs::gcap).  A block takes whole groups of 8
// consecutive tiles, one tile after the other, and keeps each of its units'
// place in the group's region in a register; every run starts on a 16-B
// piece (padded to 4 records in LDS and in the region), so the copy-out stays
// one 16-B store per piece, to the place an LDS map gives the piece's unit.
template <int KM, uint32_t kCnt, bool GL = false, uint32_t TILE = 1024>
__global__ void __launch_bounds__(512, 4) k_part_a3(const PartArgs A) {  // two blocks per CU
    constexpr uint32_t kT = 512;
    constexpr uint32_t kU = TILE / kT, kTile = TILE;
    constexpr uint32_t kPer = kCnt / kT;  // counters per thread: kPer / 2 whole pairs
    // (the sink's records land past the copy-out; GL: a unit's run padded to 4)
    constexpr uint32_t kRecWords = kTile * KM + (GL ? 4 * (kCnt / 2) : 0);
    constexpr uint32_t kCo = (kRecWords / 4 + kT - 1) / kT;  // 16-B copy-out pieces per thread
    constexpr uint32_t kMap = GL ? kRecWords / 4 : 1;        // GL: a piece's place - its LDS place
    // counter bias: counter c starts at c << kSB, so an atomic's return value
    // >> kRS (= kSB - 2) is its byte offset 4 c as long as 4 * rank stays below
    // bit kRS (1024-swipe tiles: 18 / 16; 1536: 19 / 17)
    constexpr uint32_t kSB = 4u * kRecWords < 65536u ? 18 : 19, kRS = kSB - 2;
    static_assert(kCnt % (2 * kT) == 0 && 4u * kRecWords < (1u << kRS) && kRecWords < 65536u &&
                      (2 * kCnt - 1) < (1u << (32 - kSB)) && kTile % kT == 0 && kTile <= 2048,
                  "whole pairs per thread; a rank * 4 below bit kRS; starts fit 16 bits; 11-bit swipe field");
    // one LDS object, counters first: it sits at LDS address 0, so a probe's
    // counter address is its slice field shifted and added to the parity's
    // base (v_bfe + v_lshl_add: two VALU per probe)
    struct __attribute__((aligned(16))) Lds {
        uint32_t cnt[2 * kCnt];
        uint32_t srec[kRecWords];
        uint32_t dmap[kMap];
        uint32_t swsum[kT / 64];
        uint32_t stot;
    };
    __shared__ Lds lds;
    uint32_t *const cnt = lds.cnt, *const srec = lds.srec, *const swsum = lds.swsum;
    uint32_t &stot = lds.stot;
    static_assert((kCnt & (kCnt - 1)) == 0, "parity base above the counter index bits");
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t nunits = A.nunits;
    const uint32_t sink = 2 * nunits;  // the sink pair's first slice
    for (uint32_t c = tid; c < 2 * kCnt; c += kT) cnt[c] = c << kSB;
    lds_barrier();
    // Every global load and store below is issued by every wave the same
    // number of times (buffer operations; a lane or a whole call with nothing
    // to move gives an offset past the range): vmcnt counts in issue order and
    // the compiler counts only what every path issues, so with a conditional
    // store between a load and its use the wait for the load also waited for
    // the stores (the copy-out's memory round trip, once per tile).
    const __amdgpu_buffer_rsrc_t roffs = part_rsrc(A.offs, A.offs ? (A.n + 1) * 4 : 0u);
    const __amdgpu_buffer_rsrc_t rhllw = part_rsrc(A.hllw, A.n * 4);
    const __amdgpu_buffer_rsrc_t roff = part_rsrc(A.off, nunits * A.off_stride * 4);
    auto offsets = [&](uint32_t t, uint32_t u, uint32_t &b, uint32_t &e) {
        const uint32_t i = t * kTile + u * kT + tid;
        const uint32_t ic = i < A.n ? i : A.n - 1;
        // the swipe's two offsets in one 8-B load
        const uint2 lbe = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(roffs, ic * 4, 0, nt_aux<2>()));
        b = A.offs ? lbe.x : ic * A.fixed_w;
        e = A.offs ? lbe.y : b + A.fixed_w;
    };
    uint32_t gt0, gt1;
    part_group(A.ntiles, blockIdx.x % kPGroups, gt0, gt1);
    const uint32_t tstep = gridDim.x / kPGroups;
    // this block's tiles: every tstep-th of its group's (GL: every tstep-th
    // group of 8 tiles, its tiles in order; gt0 is a multiple of 8)
    const uint32_t tfirst = GL ? gt0 + 8 * (blockIdx.x / kPGroups) : gt0 + blockIdx.x / kPGroups;
    auto tnext = [&](uint32_t t) {
        if constexpr (GL) return (t & 7u) != 7u && t + 1 < gt1 ? t + 1 : (t & ~7u) + 8 * tstep;
        else return t + tstep;
    };
    const __amdgpu_buffer_rsrc_t rbytes = part_rsrc(A.bytes, 0xfffffff0u);
    const PartLink &L = A.link[0];
    uint32_t nb_[kU], ne_[kU];
    PartId it[kU];
    uint32_t gofs[kPer / 2] = {};  // GL: this thread's units' places in the current group
    {
        // the first tile's ids, then the second tile's offsets (SKE_PA_AHEAD
        // 2: a tile's ids load at the start of the tile before it, from
        // offsets loaded one tile earlier still)
        const uint32_t t = tfirst;
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
            offsets(t < gt1 ? t : gt0, u, nb_[u], ne_[u]);
            part_id_load(rbytes, nb_[u], ne_[u], it[u]);
        }
        if (SKE_PA_AHEAD == 2) {
            const uint32_t t1 = t < gt1 && tnext(t) < gt1 ? tnext(t) : (t < gt1 ? t : gt0);
#pragma unroll
            for (uint32_t u = 0; u < kU; u++) offsets(t1, u, nb_[u], ne_[u]);
        }
    }
    const uint8_t *cntb = reinterpret_cast<const uint8_t *>(cnt);
    uint8_t *srecb = reinterpret_cast<uint8_t *>(srec);
    uint8_t *const cntw = reinterpret_cast<uint8_t *>(cnt);
    // a probe's slice (kCnt - 1 masks it: slices < kCnt), as one v_bfe the
    // compiler cannot fold into a shift and mask of the address
    auto part_slice = [](uint32_t x) {
        constexpr uint32_t kW = __builtin_ctz(kCnt);
        uint32_t r;
        asm("v_bfe_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "i"(kPSliceLog), "i"(kW));
        return r;
    };
    auto tile = [&](const uint32_t t, const uint32_t par) {
        const uint32_t cb = par * kCnt;
        const uint32_t pb = cb * 4;  // the parity's byte base, above (kCnt - 1) * 4
        uint32_t rv[kU][KM], rp[kU][KM];
        const uint32_t tn = tnext(t) < gt1 ? tnext(t) : t;
        PartId itn[kU];
        if (SKE_PA_AHEAD == 2) {
            // the next tile's ids (nb_ / ne_ hold its offsets), then the
            // offsets of the tile after it
            const uint32_t tn2 = tnext(tn) < gt1 ? tnext(tn) : tn;
#pragma unroll
            for (uint32_t u = 0; u < kU; u++) part_id_load(rbytes, nb_[u], ne_[u], itn[u]);
#pragma unroll
            for (uint32_t u = 0; u < kU; u++) offsets(tn2, u, nb_[u], ne_[u]);
        } else {
#pragma unroll
            for (uint32_t u = 0; u < kU; u++) offsets(tn, u, nb_[u], ne_[u]);
        }
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
                // (its top byte is the swipe's overflow flag, set by pass B)
                __builtin_amdgcn_raw_buffer_store_b32(idx | (rank << 16), rhllw, act ? i * 4 : kOORa, 0, nt_aux<8>());
            }
            const uint32_t lu20 = lu << 20;
            ProbeWalk32 wk;
            wk.init(ha, hb, part_div(L));
            if (full) {
#pragma unroll
                for (int q = 0; q < KM; q++) {
                    const uint32_t x = wk.x;
                    rv[u][q] = (x & 0xfffffu) | lu20;
                    rp[u][q] = atomicAdd(reinterpret_cast<uint32_t *>(cntw + part_slice(x) * 4 + pb), 4u);
                    if (q + 1 < KM) wk.step(L.d);
                }
            } else {
#pragma unroll
                for (int q = 0; q < KM; q++) {
                    const uint32_t x = wk.x;
                    rv[u][q] = (x & 0xfffffu) | lu20;
                    rp[u][q] = atomicAdd(reinterpret_cast<uint32_t *>(cntw + (act ? part_slice(x) : sink) * 4 + pb), 4u);
                    if (q + 1 < KM) wk.step(L.d);
                }
            }
            // lgkmcnt(0): this swipe's atomics, once (SKE_PA_WAIT_LAST: only
            // after the last swipe, so the first one's atomics overlap the
            // second one's hash)
            if (!SKE_PA_WAIT_LAST || u + 1 == kU) __builtin_amdgcn_s_waitcnt(0xc07f);
        }
        lds_barrier();
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {  // the next tile's ids
            if (SKE_PA_AHEAD == 2) it[u] = itn[u];
            else part_id_load(rbytes, nb_[u], ne_[u], it[u]);
        }
        // exclusive scan over pairs of their two slices' counts
        uint32_t v[kPer], s = 0;
#pragma unroll
        for (uint32_t j = 0; j < kPer; j++) {
            const uint32_t c = cb + tid * kPer + j;
            v[j] = (cnt[c] - (c << kSB)) >> 2;
        }
#pragma unroll
        for (uint32_t j = 0; j < kPer; j += 2) s += GL ? (v[j] + v[j + 1] + 3) & ~3u : v[j] + v[j + 1];
        const uint32_t incl = part_wave_scan(s);
        if (lane == 63) swsum[wave] = incl;
        lds_barrier();
        uint32_t run = incl - s;
        for (uint32_t w = 0; w < wave; w++) run += swsum[w];
#pragma unroll
        for (uint32_t j = 0; j < kPer; j += 2) {
            const uint32_t g = tid * kPer + j, c = cb + g, un = g / 2, n2 = v[j] + v[j + 1];
            uint32_t W = run | (n2 << 16);  // pass B's run: start | count << 16
            if constexpr (GL) {
                // the unit's next place in the group's region, or (it does not
                // fit) its LDS place in the tile's overflow row: bit 31
                const uint32_t p4 = (n2 + 3) & ~3u;
                if ((t & 7u) == 0) gofs[j / 2] = 0;
                const bool fits = gofs[j / 2] + p4 <= A.gcap;
                const uint32_t dst = fits ? ((t >> 3) * nunits + un) * A.gcap + gofs[j / 2] : A.govf + t * A.stride + run;
                W = fits ? gofs[j / 2] | (n2 << 16) : W | 0x80000000u;
                if (fits) gofs[j / 2] += p4;
                if (un < nunits)
                    for (uint32_t p = run / 4; p < (run + p4) / 4; p++) lds.dmap[p] = dst - run;
            }
            __builtin_amdgcn_raw_buffer_store_b32(W, roff, un < nunits ? (un * A.off_stride + t) * 4 : kOORa, 0, 0);
            if (g == sink) stot = run;
            cnt[c] = 4 * run - (c << kSB);
            cnt[c + 1] = 4 * (run + v[j]) - ((c + 1) << kSB);
            run += GL ? (n2 + 3) & ~3u : n2;
        }
        lds_barrier();
#pragma unroll
        for (uint32_t u = 0; u < kU; u++)
#pragma unroll
            for (int q = 0; q < KM; q++) {
                const uint32_t r = rp[u][q];
                *reinterpret_cast<uint32_t *>(srecb + (r + *reinterpret_cast<const uint32_t *>(cntb + (r >> kRS)))) =
                    rv[u][q];
            }
        const uint32_t nb = (cb ^ kCnt);
        for (uint32_t g = tid; g <= sink + 1; g += kT) cnt[nb + g] = (nb + g) << kSB;
        lds_barrier();
        const uint32_t total = stot;
        // a fixed number of 16-B pieces per thread (those past the tile's
        // total go out of range)
        const __amdgpu_buffer_rsrc_t rdst =
            GL ? part_rsrc(A.rec, (A.govf + A.ntiles * A.stride) * 4) : part_rsrc(A.rec + size_t(t) * A.stride, A.stride * 4);
        // (a piece past the records reads the last piece instead: an LDS read
        // past srec would be undefined behaviour, from which the compiler may
        // infer a bound on tid for the rest of the kernel -- round 4 had one:
        // the unclamped index read past srec for the last pieces, and the
        // partitioned-K1 answers of some A/B builds were wrong; the
        // 2048-counter case of tests/test_k1_partitioned.py pins the fix)
        const part_u32x4 *src = reinterpret_cast<const part_u32x4 *>(srec);
        constexpr uint32_t kLast = kRecWords / 4 - 1;
        static_assert(kRecWords % 4 == 0 && kCo * kT >= kLast + 1, "the copy-out covers srec in 16-B pieces");
        static_assert([] {  // every piece index the copy-out reads is inside srec
            for (uint32_t c = 0; c < kCo; c++)
                for (uint32_t t = 0; t < kT; t++) {
                    const uint32_t j = c * kT + t;
                    if (((c + 1) * kT <= kLast + 1 ? j : (j < kLast ? j : kLast)) > kLast) return false;
                }
            return true;
        }(), "copy-out LDS index bound");
#pragma unroll
        for (uint32_t c = 0; c < kCo; c++) {
            const uint32_t j = c * kT + tid;
            const uint32_t jr = (c + 1) * kT <= kLast + 1 ? j : (j < kLast ? j : kLast);
            const uint32_t at = GL ? (j * 4 + lds.dmap[jr]) * 4 : j * 16;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, src[jr]),
                                                   rdst, j * 4 < total ? at : kOORa, 0, nt_aux<4>());
        }
    };
    uint32_t par = 0;
    for (uint32_t t = tfirst; t < gt1; t = tnext(t), par ^= 1) tile(t, par);
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
// The fail-list pass B's 8-lane prefix runs on DPP row shifts instead of three
// ds_bpermute rounds and a broadcast (0.1966 -> 0.1946 ms, round 3); the
// slice-pair image is copied as one batch of buffer loads (0.195 -> 0.190 ms).
// SKE_PB_SPLIT: how pass B's blocks share the (slice unit, tile) space.
// 0: per XCD tile group, unit major (round 3); 1: all tiles, unit major (a
// block restages its image once or twice: pass B 0.189 -> 0.183 ms);
// 2: XCD x takes tile group x and its 32 blocks take units round
// robin, so adjacent units' runs, which share their boundary lines, are read
// by neighbouring CUs of one XCD at about the same time (round 4, A/B of
// three alternations on one box: 0.211 -> 0.200 ms; 128-B read requests
// 8.34 -> 8.06 M, L2 hits 0.65 -> 1.84 M per dispatch); 3 (default, round 5):
// as 2 while every block gets a whole unit (4 rounds of 32 of C3's 152), then
// the remaining units' (unit, 8-tile group) space in equal contiguous shares,
// so no block runs a fifth unit while the others wait (pass B 0.368 -> 0.362
// ms per 2^25 sub-batch, three alternations; profiles/r05_ab_pass_b_split.txt)
#ifndef SKE_PB_SPLIT
#define SKE_PB_SPLIT 3
#endif
// GL (FL only): the group layout -- a run's start is its place in the (tile
// group, unit) region, or (bit 31 of its run word) in the tile's overflow row
// TILE: swipes per tile (FL: kTileFl; the others 1024); a k_part_a3 record's
// swipe field is its bits 20..30
template <int SP, int R = 2 * SP, bool FL = false, bool GL = false, uint32_t TILE = 1024>  // R: 16-byte pieces per lane and run (runs of SP slices)
__global__ void __launch_bounds__(kPbBlock, SP == 1 ? 8 : 4) k_part_b(const PartArgs A) {
    static_assert(FL || TILE == 1024, "tiles of other than 1024 swipes are the fail-list chains'");
    static_assert(!GL || FL, "the group layout is pass A3's");
    PB_STAMP(0);
    const uint32_t tmask = (1u << kPTileLog) - 1;
    __shared__ __attribute__((aligned(16))) uint8_t img[kPSliceBytes * SP];
    __shared__ uint32_t fq[kPbBlock / 64][kPbQueue];
    // this block's share of the (slice unit, tile) space, unit major: of its
    // XCD group's tiles (SKE_PB_SPLIT 0), or of all tiles (1: every block
    // restages its images once or twice instead of ~6 times)
    // SKE_PB_SPLIT 2: XCD x (blocks b % 8 == x) takes tile group x, and its
    // blocks take whole units round robin (block j: units j, j + 32, ...),
    // so the 32 CUs of an XCD sweep the same tiles of 32 ADJACENT units at
    // about the same pace: a line two neighbouring runs share is read while
    // the other block's read of it is still in the XCD's L2
    uint32_t gt0 = 0, gt1 = A.ntiles, nblk = gridDim.x, bi = blockIdx.x;
    if (SKE_PB_SPLIT != 1) {
        part_group(A.ntiles, blockIdx.x % kPGroups, gt0, gt1);
        nblk = gridDim.x / kPGroups;
        bi = blockIdx.x / kPGroups;
    }
    const uint32_t gn = gt1 - gt0;
    // (an empty XCD tile group -- a sub-batch of fewer than 64 tiles: the
    // whole block leaves before the split arithmetic divides by gn8 = 0)
    if (gn == 0) return;
    const uint32_t nunits = (A.nslices + SP - 1) / SP;
    const uint32_t total = nunits * gn;
    uint32_t w = uint32_t(uint64_t(total) * bi / nblk);
    uint32_t wend = uint32_t(uint64_t(total) * (bi + 1) / nblk);
    uint32_t su = bi;  // SKE_PB_SPLIT 2 / 3: this block's current unit
    // SKE_PB_SPLIT 3: units round robin while every block gets a whole one,
    // then the remaining units' (unit, 8-tile group) space in equal
    // contiguous shares, so no block waits with a fifth unit while others idle
    const uint32_t full = SKE_PB_SPLIT == 3 ? nunits / nblk * nblk : nunits;
    const uint32_t gn8 = (gn + 7) / 8;
    auto lin = [&](uint32_t c) {  // the remaining space's 8-tile group c as a (unit, tile) index
        const uint32_t t8 = (c % gn8) * 8;
        return (full + c / gn8) * gn + (t8 < gn ? t8 : gn);
    };
    bool rest = false;
    auto take_rest = [&]() {
        const uint32_t space = (nunits - full) * gn8;
        w = lin(uint32_t(uint64_t(space) * bi / nblk));
        wend = lin(uint32_t(uint64_t(space) * (bi + 1) / nblk));
        rest = true;
    };
    if (SKE_PB_SPLIT == 2 || SKE_PB_SPLIT == 3) {
        w = su < full ? su * gn : total;
        wend = su < full ? w + gn : total;
        if (SKE_PB_SPLIT == 3 && su >= full) take_rest();
    }
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t k = lane / kPbLanes, qq = lane % kPbLanes;
    constexpr uint32_t kWaves = kPbBlock / 64, kStep = kWaves * kPbGroup;
    // the records of this block's tile group (per-tile layout; offsets from
    // its first tile, so a 2^26-swipe sub-batch's 2.95 GB stay 32-bit), or
    // of every group (the group layout: regions and overflow rows)
    const size_t rbase = GL ? 0 : size_t(gt0) * A.stride;
    const __amdgpu_buffer_rsrc_t rrec =
        GL ? part_rsrc(A.rec, (A.govf + A.ntiles * A.stride) * 4) : part_rsrc(A.rec + rbase, (gt1 - gt0) * A.stride * 4);
    const __amdgpu_buffer_rsrc_t roff = part_rsrc(A.off, (A.nslices + 1) * A.off_stride * 4);
    const __amdgpu_buffer_rsrc_t rfl = part_rsrc(A.flist, FL ? A.nunits * A.fl_stride * kPbLanes * 2 : 0);
    uint32_t *q = fq[wave];
    while (true) {
        if (w >= wend) {
            if (SKE_PB_SPLIT != 2 && SKE_PB_SPLIT != 3) break;
            if (rest) break;
            su += nblk;  // block-uniform
            if (su < full) {
                w = su * gn;
                wend = w + gn;
            } else {
                if (SKE_PB_SPLIT == 2) break;
                take_rest();
                if (w >= wend) break;
            }
        }
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
        lds_barrier();  // every wave is done with the previous slice
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
        lds_barrier();
        // failures that do not fit a fail list: a byte store of 1 (FL: into
        // the top byte of the swipe's HLL word -- byte 4 i + 3, which pass A
        // wrote 0 -- so pass A writes no fail bytes and C reads none)
        const __amdgpu_buffer_rsrc_t rfail =
            FL ? part_rsrc(A.hllw, A.n * 4) : part_rsrc(A.fail + size_t(l) * A.fail_stride, A.fail_stride);
        auto fail_at = [](uint32_t i) { return FL ? i * 4 + 3 : i; };
        const uint32_t orow = (FL ? unit : g) * A.off_stride, erow = ge * A.off_stride;
        // run boundaries of 8 rounds at once: lane L holds those of tile
        // tg0 + (L / 8) * kStep + L % 8 (0, 0 past tb); a round's lanes take
        // theirs from it with a cross-lane read, so boundary loads are one
        // instruction (FL: start | count << 16 per pair run) or one pair per
        // 8 rounds
        auto load_be8 = [&](uint32_t tg0, uint32_t &B, uint32_t &E) {
            const uint32_t t = tg0 + (lane / kPbGroup) * kStep + lane % kPbGroup;
            const bool in = t < tb;
            if constexpr (GL) {  // B keeps the overflow bit 31
                const uint32_t W = __builtin_amdgcn_raw_buffer_load_b32(roff, in ? (orow + t) * 4 : kOOR, 0, nt_aux<1>());
                B = W & 0x8000ffffu;
                E = (W & 0xffffu) + ((W >> 16) & 0x7fffu);
            } else if constexpr (FL) {
                const uint32_t W = __builtin_amdgcn_raw_buffer_load_b32(roff, in ? (orow + t) * 4 : kOOR, 0, nt_aux<1>());
                B = W & 0xffffu;
                E = B + (W >> 16);
            } else {
                B = __builtin_amdgcn_raw_buffer_load_b32(roff, in ? (orow + t) * 4 : kOOR, 0, nt_aux<1>());
                E = __builtin_amdgcn_raw_buffer_load_b32(roff, in ? (erow + t) * 4 : kOOR, 0, nt_aux<1>());
            }
        };
        // 16-byte pieces qq, qq + 8, ... of the run from the 128-B line holding
        // its start: every piece is one whole line (one request, not two)
        // (one byte offset per lane; piece c adds 128 c, an immediate of the
        // load; a piece past the run's end goes out of range)
        // the word where tile t's run of this unit is placed from (GL: its
        // group region, or with bit 31 of b its overflow row)
        auto row = [&](uint32_t t, uint32_t b) {
            if constexpr (GL) return (b >> 31) ? A.govf + t * A.stride : ((t >> 3) * A.nunits + unit) * A.gcap;
            else return (t - gt0) * A.stride;
        };
        auto load_recs = [&](uint32_t tg, uint32_t b, uint32_t e, uint4 (&r)[R]) {
            const uint32_t i0 = (b & (GL ? 0xffe0u : ~31u)) + qq * 4;
            const uint32_t v0 = (row(tg + k, b) + i0) * 4;
            const int32_t left = int32_t(e) - int32_t(i0);
#pragma unroll
            for (uint32_t c = 0; c < R; c++)
                r[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     rrec, (left > int32_t(32 * c) ? v0 : kOOR) + 128 * c, 0, nt_aux<64>()));
        };
        uint32_t tg = ta + wave * kPbGroup;
        uint32_t Bc, Ec, Bn, En;  // boundaries of rounds [8q, 8q + 8) and of the 8 after
        load_be8(tg, Bc, Ec);
        load_be8(tg + kPbGroup * kStep, Bn, En);
        uint32_t bc = __shfl(Bc, k, 64), ec = __shfl(Ec, k, 64);
        // one round = kPbGroup tiles' runs of this unit; the next round's
        // records load while this one is tested.  Two rounds per loop
        // iteration with the record buffers in turn (no register copies).
        uint32_t rr = 0;
        auto round = [&](const uint4 (&r)[R], uint4 (&rn)[R]) {
            const uint32_t nr = (rr + 1) % kPbGroup;
            if (nr == 0) {  // wave-uniform
                Bc = Bn;
                Ec = En;
                load_be8(tg + (kPbGroup + 1) * kStep, Bn, En);
            }
            const uint32_t b1 = __shfl(Bc, nr * kPbGroup + k, 64), e1 = __shfl(Ec, nr * kPbGroup + k, 64);
            load_recs(tg + kStep, b1, e1, rn);
            // the (up to) 4R records of this lane: piece c starts at record
            // lo_c = s0 + c*32 + qq*4; bit j of vm: record j in [bc, ec)
            const uint32_t bw = GL ? bc & 0xffffu : bc;  // (GL: without the overflow bit)
            const uint32_t s0 = bw & ~31u;
            uint32_t rec[4 * R];
#pragma unroll
            for (uint32_t c = 0; c < R; c++) {
                rec[4 * c] = r[c].x;
                rec[4 * c + 1] = r[c].y;
                rec[4 * c + 2] = r[c].z;
                rec[4 * c + 3] = r[c].w;
            }
            // bit 4c + j: record lo0 + 32c + j lies in [bc, ec).  Only piece 0
            // can start before bc (s0 = bc & ~31), so the lower bound masks
            // piece 0 alone; the upper bound clamps every piece.
            // (v_bfm: ((1 << width) - 1) << offset in one VALU)
            auto clamp4 = [](int32_t v) { return uint32_t(v < 0 ? 0 : (v > 4 ? 4 : v)); };
            const uint32_t lo0 = s0 + qq * 4;
            const int32_t dh = int32_t(ec) - int32_t(lo0);
            uint32_t vm = 0;
#pragma unroll
            for (uint32_t c = 0; c < R; c++) vm |= part_bfm(clamp4(dh - int32_t(32 * c)), 4 * c);
            vm &= ~part_bfm(clamp4(int32_t(bw) - int32_t(lo0)), 0);
            // bit set in the image: its 32-bit word, bit (offset & 31); with
            // slice pairs the record's parity bit selects the image half
            const uint32_t *img32 = reinterpret_cast<const uint32_t *>(img);
            uint32_t okm = 0;
#pragma unroll
            for (uint32_t j = 0; j < 4 * R; j++) {
                const uint32_t rr = rec[j];
                const uint32_t o = FL ? (rr & 0xfffffu)  // k_part_a3: the offset in the pair
                                      : SP == 1 ? (rr & kPSliceMask)
                                                : ((rr & kPSliceMask) | ((rr >> kPTileLog) & kPSliceBits));
                okm |= part_bit(img32[o >> 5], rr) << j;
            }
            uint32_t fm = vm & ~okm;
            const uint32_t tbase = (tg + k) * TILE;
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
                uint32_t pos = incl - cnt;
                while (fm) {
                    const uint32_t j = __builtin_ctz(fm);
                    fm &= fm - 1;
                    const uint32_t at = (pick(j) >> 20) & 0x7ffu;  // k_part_a3's swipe field
                    if (pos < kPbLanes) q[k * kPbLanes + pos] = at;
                    else __builtin_amdgcn_raw_buffer_store_b8(uint8_t(1), rfail, fail_at(tbase + at), 0, 0);  // overflow
                    pos++;
                }
                __builtin_amdgcn_wave_barrier();
                // lane (k, qq) writes entry qq of tile tg + k's list (tiles past
                // this block's range belong to another wave: not written)
                const uint32_t v = q[lane];
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
                const uint32_t base = row(tg + k, bc);
                for (uint32_t i = s0 + 32 * R + qq; i < ec; i += kPbLanes) {
                    const uint32_t rr = __builtin_amdgcn_raw_buffer_load_b32(rrec, (base + i) * 4, 0, 0);
                    const uint32_t o = FL ? (rr & 0xfffffu)
                                          : SP == 1 ? (rr & kPSliceMask)
                                                    : ((rr & kPSliceMask) | ((rr >> kPTileLog) & kPSliceBits));
                    if (!((img[o >> 3] >> (o & 7)) & 1))
                        __builtin_amdgcn_raw_buffer_store_b8(uint8_t(1), rfail,
                                                             fail_at(tbase + (FL ? (rr >> 20) & 0x7ffu : (rr >> kPSliceLog) & tmask)), 0, 0);
                }
            }
            bc = b1;
            ec = e1;
            tg += kStep;
            rr++;
        };
        uint4 ra[R], rb[R];
        load_recs(tg, bc, ec, ra);
        while (tg < tb) {
            round(ra, rb);
            if (tg >= tb) break;  // wave-uniform
            round(rb, ra);
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
    const uint64_t tile = uint64_t(1) << kPTileLog;
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
                if (valid[u]) {
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
#pragma unroll
        for (int u = 0; u < U; u++) cur[u] = w[u] ? nt_ld<32>(w[u]) : 0xffffffffu;
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
// (Its loads and stores at a fixed count per tile, as pass A's, measured
// equal, 0.408 vs 0.409 ms: pass C is bound by the memory side's random
// requests, not by its waves' waits.)
// (A two-phase form -- the answers and the rank-1 raises as plain byte
// stores first, the rank >= 2 raises by CAS in a second kernel -- measured
// slower, 0.409 -> 0.436 ms, round 4: the line traffic, not the CAS count,
// holds this pass.)  U swipes per thread per tile, kPcFlBlock * U = 1024
// (1024 x 1 since round 4; see SKE_PC_BLOCK).
template <uint32_t BT, int U, uint32_t TILE>
__global__ void __launch_bounds__(BT) k_part_c_fl(const PartArgs A) {
    static_assert(BT * U == TILE, "one tile per sub-step");
    constexpr uint32_t kPcFlBlock = BT;
    constexpr uint32_t kRun = kPbGroup;  // tiles per block iteration
    __shared__ uint16_t mark[kRun * TILE];
    const uint32_t tid = threadIdx.x;
    for (uint32_t j = tid; j < kRun * TILE; j += kPcFlBlock) mark[j] = 0;
    uint32_t gt0, gt1;
    part_group(A.ntiles, blockIdx.x % kPGroups, gt0, gt1);
    const uint32_t nblk = gridDim.x / kPGroups;
    const uint32_t npieces = A.nunits * kRun;  // 16-B lists of one run
    const __amdgpu_buffer_rsrc_t rfl = part_rsrc(A.flist, A.nunits * A.fl_stride * kPbLanes * 2);
    struct In {
        uint32_t fb[U], sl[U], hv[U];
    };
    auto load = [&](uint32_t t, uint32_t tend, In &in) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = t * TILE + uint32_t(u) * kPcFlBlock + tid;
            const bool act = t < tend && i < A.n;
            in.sl[u] = act ? nt_ld<16>(A.slot + i) : 0u;
            in.hv[u] = act ? nt_ld<16>(A.hllw + i) : 0xff000000u;  // (top byte: pass B's overflow flag)
            in.fb[u] = in.hv[u] >> 24;
        }
    };
    lds_barrier();
    for (uint32_t r0 = gt0 + (blockIdx.x / kPGroups) * kRun; r0 < gt1; r0 += nblk * kRun) {
        const uint32_t r1 = r0 + kRun < gt1 ? r0 + kRun : gt1;
        const uint16_t ep = uint16_t(r0 / kRun + 1);  // < 2^16: sub-batches hold <= 16384 tiles
        In cur;
        load(r0, r1, cur);
        // the run's lists: piece p = (unit p / kRun, tile r0 + p % kRun)
        for (uint32_t p0 = 0; p0 < npieces; p0 += 4 * kPcFlBlock) {
            part_u32x4 e[4];
            bool ok[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t p = p0 + uint32_t(j) * kPcFlBlock + tid;
                const uint32_t un = p / kRun, tt = r0 + p % kRun;
                ok[j] = p < npieces && tt < r1;
                e[j] = __builtin_bit_cast(part_u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                         rfl, ok[j] ? (un * A.fl_stride + tt) * kPbLanes * 2 : kOOR, 0, 0));
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t base = ((p0 + uint32_t(j) * kPcFlBlock + tid) % kRun) * TILE;
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const uint32_t lo = e[j][c] & 0xffffu, hi = e[j][c] >> 16;
                    if (ok[j] && lo < TILE) mark[base + lo] = ep;  // (0xffff: no entry)
                    if (ok[j] && hi < TILE) mark[base + hi] = ep;
                }
            }
        }
        lds_barrier();
        for (uint32_t t = r0; t < r1; t++) {
            In nxt;
            load(t + 1, r1, nxt);
            const uint16_t *mk = mark + (t - r0) * TILE;
            bool valid[U];
            uint32_t *w[U];
            uint32_t rank[U], sh[U], cw[U], seen[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t i = t * TILE + uint32_t(u) * kPcFlBlock + tid;
                valid[u] = i < A.n && cur.fb[u] == 0 && mk[uint32_t(u) * kPcFlBlock + tid] != ep;
                w[u] = nullptr;
                rank[u] = sh[u] = 0;
                if (valid[u]) {
                    const uint32_t rk = (cur.hv[u] >> 16) & 0xffu;
                    if (cur.sl[u] >= A.nslots) {
                        atomicOr(A.err, 1u);
                    } else {
                        const uint32_t ridx = cur.hv[u] & 0xffffu;
                        w[u] = reinterpret_cast<uint32_t *>(A.regs + (uint64_t(cur.sl[u]) << kHllP) + (ridx & ~3u));
                        sh[u] = (ridx & 3) * 8;
                        rank[u] = rk;
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < U; u++) cw[u] = w[u] ? nt_ld<32>(w[u]) : 0xffffffffu;
            // every raising CAS of the tile in flight at once, then settled
            // (a lost race retries from the word the CAS returned)
#pragma unroll
            for (int u = 0; u < U; u++) {
                seen[u] = cw[u];
                if (w[u] && ((cw[u] >> sh[u]) & 0xffu) < rank[u])
                    seen[u] = atomicCAS(w[u], cw[u], (cw[u] & ~(0xffu << sh[u])) | (rank[u] << sh[u]));
            }
            if (A.out) {
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const uint32_t i = t * TILE + uint32_t(u) * kPcFlBlock + tid;
                    if (i < A.n) nt_st<16>(A.out + i, uint8_t(valid[u]));
                }
            }
#pragma unroll
            for (int u = 0; u < U; u++)
                if (w[u] && seen[u] != cw[u]) part_reg_max(w[u], sh[u], rank[u], seen[u]);
            cur = nxt;
        }
        lds_barrier();  // the marks are rewritten by the next run
    }
}

// ---------------------------------------------------------------------------
// Segmented PFADD (north_star's HLL kernel form): pass C of the one-link
// partitioned K1 when the call's register updates are dense in the slab --
// the batch is segmented by key, each key window's registers are staged in
// LDS, raised there, and flushed to HBM as whole lines.  Same result as
// k_part_c_fl (hllAdd's register max, attendance_processor.py:127-129; max is
// commutative, so the order of updates is free).
//
// Why.  k_part_c_fl costs one random 128-B line read per valid swipe (its
// register's pre-check) plus one memory-side CAS per raise: 14.4 M + 7 M
// random requests per 16 M-swipe C3 step.  When a call's updates are dense
// in the slab -- an 8-way shard (12.5 k keys, 205 MB, ~9 updates per 128-B
// line per 16 M swipes) or a large batch -- reading every line of the slab
// once and writing back the lines that rose costs fewer bytes than the
// random requests, and no atomics reach memory.
//
//   C1 (k_seg_c1)   per run of 8 tiles (8192 swipes; pass B's fail lists of a
//                   run are one line per unit): the answers as k_part_c_fl,
//                   and for each valid swipe one 4-byte record
//                   (slot-in-bucket << 20 | register << 6 | rank),
//                   counting-sorted in LDS by level-1 bucket (slot >> s1,
//                   <= 512 buckets).  Arena form (default): each bucket's
//                   records of the run reserved in the bucket's contiguous
//                   sequence of the sub-batch (one atomic add) and stored
//                   into its 8192-record chunk slots.  Run-table form
//                   (SKE_SEG_ARENA 0): written as the run's block of
//                   records; o1[bucket][run] = the bucket's start in it.
//   S  (k_seg_scan) run-table form only: per bucket, prefix of its run
//                   lengths over the runs, and the run holding the first
//                   record of each of its 8192-record level-2 chunks.
//   D  (k_seg_da /  per chunk: its records (arena: read whole; run-table
//       k_seg_d)    form: gathered from the runs), counting-sorted in LDS
//                   by window (2^klog keys) within the bucket;
//                   o2[chunk][window] = the window's start.
//   E  (k_seg_e)    per window, once per call (after every sub-batch's C1,
//                   S, D): its records' runs over every chunk of its bucket;
//                   with at least dense_min records the window's registers
//                   (2^klog x 16 KiB) are loaded into LDS in whole lines,
//                   raised there (LDS CAS; registers only grow), and the
//                   lines that rose are stored back; a sparse window raises
//                   its records in place (pre-check load + CAS, as pass C).
// ---------------------------------------------------------------------------
constexpr uint32_t kSegRunTiles = kPbGroup;                 // tiles per level-1 run
constexpr uint32_t kSegRunSw = kSegRunTiles * kTileFl;    // 8192 swipes (12 288 with 1536-swipe tiles)
constexpr uint32_t kSegMaxB1 = 512;                         // level-1 buckets
constexpr uint32_t kSegMaxWpb = 512;                        // windows per bucket
constexpr uint32_t kSegChunk = 8192;                        // records per level-2 chunk
constexpr uint32_t kSegMaxRuns = kPSub / kSegRunSw;         // 8192 runs per sub-batch
constexpr uint32_t kSegDStage = 2048;                       // D: runs of a chunk staged in LDS
constexpr uint32_t kSegRecShift = 20;                       // record: slot-in-bucket above bit 20
static_assert(kSegMaxRuns < 65536, "k_seg_c1's uint16 mark epochs (run + 1) would wrap");

struct SegArgs {
    uint32_t *r1;     // [nruns][kSegRunSw] level-1 records of a sub-batch, bucket-sorted per run
    uint32_t *o1;     // [nb1 + 1][kSegMaxRuns] bucket h's start in run r; [nb1][r] = the run's total
    uint32_t *p1;     // [nb1][kSegMaxRuns + 1] prefix over runs of bucket h's lengths; [h][nruns] = total
    uint32_t *cst;    // [nb1][kSegMaxRuns + 1] run holding chunk c's first record
    uint32_t *r2;     // [nsub][maxch][kSegChunk] level-2 records, window-sorted per chunk
    uint32_t *o2;     // [nsub][maxch][wpb + 1] window w's start in chunk q
    uint32_t *cb;     // [nsub][nb1 + 1] first chunk of bucket h in sub-batch s (prefix)
    uint32_t nruns;   // level-1 runs of this sub-batch
    uint32_t nb1;     // level-1 buckets: 2^b1, window W = slot >> klog in bucket W & (nb1 - 1)
    uint32_t b1;      // log2(nb1)
    uint32_t s1;      // bits of a record's slot-in-bucket: (W >> b1) << klog | slot & (2^klog - 1) (<= 12)
    uint32_t wlog;    // windows per bucket = 1 << wlog
    uint32_t klog;    // keys per window = 1 << klog
    uint32_t s;       // this sub-batch's index in the call
    uint32_t nsub;    // sub-batches of the call
    uint32_t maxch;   // level-2 chunk slots per sub-batch
    uint32_t nwin;    // windows of the slab (E)
    uint32_t dense_min;  // E: records at which a window is staged in LDS
    uint32_t *q;      // window pass queue header: [0] queued slices, [1] copies, [2] cut windows, [5] E2 items
                      // and [8 + x] XCD x's E1 items claimed past the first gridDim.x (zeroed per window pass)
    uint4 *qitems;    // queued slices (window, slice, copy)
    uint4 *mlist;     // cut windows (window, first copy, slices)
    uint8_t *copies;  // [ccap][window bytes] LDS copies of cut windows' slices
    uint32_t ccap;    // copies (and queue entries) available
    // the arena form (SKE_SEG_ARENA): level-1 records in chunk slots of r1
    uint32_t *fill;   // [nsub][nb1 + 1] (x kSegFillStride words) records reserved per bucket; [s][nb1] =
                      // counted chunk slots taken
    uint32_t *ctab;   // [nb1][kmaxc] chunk c of bucket h: its slot + 1 (0: not yet placed)
    uint32_t kmaxc;   // chunks a bucket can have in a sub-batch
    uint32_t kstat;   // chunk c < kstat of bucket h sits in slot h * kstat + c; later chunks take
                      // slots nb1 * kstat + (counter), named in ctab
};

// The arena form of C1 -> D (SKE_SEG_ARENA 1).  C1 reserves each bucket's
// records of a run with one atomic add on the bucket's fill count (issued
// before the run's scan and placement, which hide its latency), so a
// bucket's records are one contiguous sequence of the sub-batch; the sequence
// lives in 8 192-record chunks.  The first kstat chunks of bucket h have the
// fixed slots h * kstat + c of r1 (about twice a bucket's mean); a later
// chunk of a heavy bucket takes a slot from a counter, claimed by the run
// whose reservation holds the chunk's first record, which publishes it in
// ctab before it waits for any other.  D then reads whole chunks: no scan
// pass S, no run tables, no gather.
// Measured at the 2^28 default step (profiles/r06_ab_seg_arena.txt): C1 +
// D 0.195 -> 0.169 ms per 2^25 sub-batch at N = 1 (C1 0.100 -> 0.110, S + D
// 0.095 -> 0.059), 0.193 -> 0.172 at the 8-way shard; step 8.87 -> 8.63 ms.
// 0: round 6's run-table form (k_seg_scan + k_seg_d).
#ifndef SKE_SEG_ARENA
#define SKE_SEG_ARENA 1
#endif

// Exclusive prefix of one value per thread over the block (blockDim a
// multiple of 64); every thread also gets the total.  `ws`: blockDim / 64
// words of LDS.  LDS-only barriers (global loads and stores stay in flight).
__device__ __forceinline__ uint32_t seg_scan(uint32_t v, uint32_t *ws, uint32_t &total) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    const uint32_t inc = part_wave_scan(v);
    lds_barrier();  // the previous scan's readers of ws are done
    if (lane == 63) ws[wave] = inc;
    lds_barrier();
    uint32_t pre = 0, tot = 0;
    for (uint32_t w = 0; w < nw; w++) {
        const uint32_t x = ws[w];
        pre += w < wave ? x : 0;
        tot += x;
    }
    total = tot;
    return pre + inc - v;
}

// index of the last entry of a[0..n) that is <= v (a ascending, a[0] <= v)
__device__ __forceinline__ uint32_t seg_last_le(const uint32_t *a, uint32_t n, uint32_t v) {
    uint32_t lo = 0, len = n;
    while (len > 1) {
        const uint32_t half = len >> 1;
        if (a[lo + half] <= v) lo += half;
        len -= half;
    }
    return lo;
}

// Arena: the slots of the (at most two) chunks that bucket h's cv records
// of a run, from sequence index base on, fall in, packed as slot0 | slot1 <<
// 14 | (chunk0 & 1) << 28.  A fixed chunk (c < kstat) needs nothing; a
// counted chunk whose first record is in this reservation takes its slot
// here and publishes it; one begun by an earlier reservation is waited for
// (its owner took its fill index before this one did, so it is resident and
// publishes without waiting on anything).  A wait that never ends sets error
// bit 4 (reported as the call's error) after ~1 s.
static_assert(kSegChunk == 8192, "the arena's chunk arithmetic");
// fill counts 256 B apart: every run adds to every bucket's, and counters
// packed in a few lines would queue on the few memory channels holding them
#ifndef SKE_SEG_FILL_STRIDE
#define SKE_SEG_FILL_STRIDE 64
#endif
constexpr uint32_t kSegFillStride = SKE_SEG_FILL_STRIDE;
__device__ __forceinline__ uint32_t seg_fill_at(const SegArgs &S, uint32_t h) {
    return (S.s * (S.nb1 + 1) + h) * kSegFillStride;
}
__device__ __forceinline__ uint32_t seg_arena_slot(const SegArgs &S, unsigned int *err, uint32_t h, uint32_t c,
                                                   bool own) {
    if (c < S.kstat) return h * S.kstat + c;
    uint32_t *ct = S.ctab + size_t(h) * S.kmaxc + c;
    if (own) {
        const uint32_t d = atomicAdd(S.fill + seg_fill_at(S, S.nb1), 1u);
        __hip_atomic_store(ct, d + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return S.nb1 * S.kstat + d;
    }
    uint32_t v = 0;
    for (uint32_t it = 0; it < (1u << 22); it++) {
        v = __hip_atomic_load(ct, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v) break;
        __builtin_amdgcn_s_sleep(8);
    }
    if (!v) {
        atomicOr(err, 4u);
        v = 1;
    }
    return S.nb1 * S.kstat + v - 1;
}
__device__ __forceinline__ uint32_t seg_arena_slots(const SegArgs &S, unsigned int *err, uint32_t h, uint32_t cv,
                                                    uint32_t base) {
    const uint32_t c0 = base >> 13, c1 = (base + cv - 1) >> 13;  // cv <= 8192: c1 <= c0 + 1
    // (chunk c1 > c0 starts inside this reservation: it is ours, published
    // before we wait for c0)
    const uint32_t s1 = c1 != c0 ? seg_arena_slot(S, err, h, c1, true) : 0u;
    __asm__ volatile("" ::: "memory");
    const uint32_t s0 = seg_arena_slot(S, err, h, c0, (base & (kSegChunk - 1)) == 0);
    return s0 | ((c1 != c0 ? s1 : s0) << 14) | ((c0 & 1u) << 28);
}

// C1's block: T threads, U = kSegRunSw / T swipes of a run each (1024 x 8 at
// two blocks per CU, or 512 x 16 at three: three runs in flight per CU; with
// 1536-swipe tiles 768 x 16 at two)
#ifndef SKE_SEG_C1T
#define SKE_SEG_C1T (kTileFl == 1024 ? 512 : 768)
#endif
template <uint32_t T> struct SegC1 {
    static constexpr uint32_t U = kSegRunSw / T;       // swipes per thread per run
    static constexpr uint32_t PT = kTileFl / T;        // swipes per thread per tile
    static constexpr uint32_t BPC = T == 512 ? 3 : 2;  // blocks per CU
    static constexpr uint32_t WPE = BPC * (T / 64) / 4;
    static_assert(kTileFl % T == 0, "whole tile slices per thread");
};
template <uint32_t T>
__global__ void __launch_bounds__(T, SegC1<T>::WPE) k_seg_c1(const PartArgs A, const SegArgs S) {
    constexpr uint32_t U = SegC1<T>::U, PT = SegC1<T>::PT;
    __shared__ __attribute__((aligned(16))) uint16_t mark[kSegRunSw];
    __shared__ __attribute__((aligned(16))) uint32_t srec[kSegRunSw];
    __shared__ uint32_t cnt[kSegMaxB1 + 1];
    __shared__ uint32_t slt[SKE_SEG_ARENA ? kSegMaxB1 : 1];
    __shared__ uint32_t ws[T / 64];
    const uint32_t tid = threadIdx.x;
    for (uint32_t j = tid; j < kSegRunSw; j += T) mark[j] = 0;
    const uint32_t npieces = A.nunits * kSegRunTiles;  // 16-B lists of one run
    const __amdgpu_buffer_rsrc_t rfl = part_rsrc(A.flist, A.nunits * A.fl_stride * kPbLanes * 2);
    const uint32_t kmask = (1u << S.klog) - 1, bmask = S.nb1 - 1;
    lds_barrier();  // marks cleared before any run sets one
    for (uint32_t r = blockIdx.x; r < S.nruns; r += gridDim.x) {
        const uint32_t t0 = r * kSegRunTiles;
        const uint32_t t1 = t0 + kSegRunTiles < A.ntiles ? t0 + kSegRunTiles : A.ntiles;
        const uint16_t ep = uint16_t(r + 1);  // <= kSegMaxRuns (8192) < 2^16: marks are never cleared
        // the run's streams, every tile's in flight together (the HLL
        // word's top byte is pass B's overflow flag)
        uint32_t sl[U], hv[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {  // swipe u: tile u / PT, its (u % PT)-th T-thread slice
            const uint32_t i = (t0 + u / PT) * kTileFl + (u % PT) * T + tid;
            const bool act = t0 + u / PT < t1 && i < A.n;
            sl[u] = act ? nt_ld<16>(A.slot + i) : 0u;
            hv[u] = act ? nt_ld<16>(A.hllw + i) : 0xff000000u;
        }
        for (uint32_t j = tid; j <= S.nb1; j += T) cnt[j] = 0;
        // the run's fail lists -> marks (piece p = unit p / 8, tile t0 + p % 8)
        for (uint32_t p0 = 0; p0 < npieces; p0 += 4 * T) {
            part_u32x4 e[4];
            bool ok[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t p = p0 + uint32_t(j) * T + tid;
                const uint32_t un = p / kSegRunTiles, tt = t0 + p % kSegRunTiles;
                ok[j] = p < npieces && tt < t1;
                e[j] = __builtin_bit_cast(part_u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                         rfl, ok[j] ? (un * A.fl_stride + tt) * kPbLanes * 2 : kOOR, 0, 0));
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t base = ((p0 + uint32_t(j) * T + tid) % kSegRunTiles) * kTileFl;
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const uint32_t lo = e[j][c] & 0xffffu, hi = e[j][c] >> 16;
                    if (ok[j] && lo < kTileFl) mark[base + lo] = ep;  // (0xffff: no entry)
                    if (ok[j] && hi < kTileFl) mark[base + hi] = ep;
                }
            }
        }
        lds_barrier();
        uint32_t rec[U], pos[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t lt = (u / PT) * kTileFl + (u % PT) * T + tid;  // the swipe's place in the run
            const uint32_t i = t0 * kTileFl + lt;
            const bool act = t0 + u / PT < t1 && i < A.n;
            const bool valid = act && (hv[u] >> 24) == 0 && mark[lt] != ep;
            if (A.out && act) nt_st<16>(A.out + i, uint8_t(valid));
            pos[u] = 0xffffffffu;
            rec[u] = 0;
            if (valid) {
                if (sl[u] >= A.nslots) {
                    atomicOr(A.err, 1u);
                } else {
                    const uint32_t w = sl[u] >> S.klog, b = w & bmask;
                    const uint32_t sib = ((w >> S.b1) << S.klog) | (sl[u] & kmask);
                    rec[u] = (sib << kSegRecShift) | ((hv[u] & 0x3fffu) << 6) | (hv[u] >> 16);
                    pos[u] = (b << 16) | atomicAdd(&cnt[b], 1u);
                }
            }
        }
        lds_barrier();
        uint32_t total;
        const uint32_t cv = tid < S.nb1 ? cnt[tid] : 0u;
        // Arena: each bucket's reservation is rounded up to 4 records, so every
        // reservation starts 16-B aligned; the pad holds records of rank 0 (a
        // real record's rank is >= 1), which D skips.  The reservation is a
        // buffer atomic issued here and first waited for after the placement
        // (its address is one VGPR rebuilt from tid: no 64-bit pointer is kept
        // live -- and spilled -- across the run).
        const uint32_t cvp = SKE_SEG_ARENA ? (cv + 3) & ~3u : cv;
        uint32_t abase = 0;
        if (SKE_SEG_ARENA && cv)
            abase = uint32_t(__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(
                int(cvp), part_rsrc(S.fill, S.nsub * (S.nb1 + 1) * kSegFillStride * 4), int(seg_fill_at(S, tid) * 4), 0,
                0));
        // one scan for both run layouts (arena: the padded prefix in the high
        // half; both totals stay below 2^16)
        uint32_t tot2;
        const uint32_t ex2 = seg_scan(SKE_SEG_ARENA ? (cvp << 16) | cv : cv, ws, tot2);
        const uint32_t ex = SKE_SEG_ARENA ? ex2 & 0xffffu : ex2, exp = ex2 >> 16;
        total = SKE_SEG_ARENA ? tot2 & 0xffffu : tot2;
        // (the padded layout when it fits the run's LDS, else the unpadded one:
        // block-uniform)
        const bool padded = SKE_SEG_ARENA && (tot2 >> 16) <= kSegRunSw;
        if (tid < S.nb1) {
            cnt[tid] = padded ? exp : ex;
            if (!SKE_SEG_ARENA) S.o1[size_t(tid) * kSegMaxRuns + r] = ex;
            if (padded)
                for (uint32_t k = cv; k < cvp; k++) srec[exp + k] = 0u;
        }
        if (!SKE_SEG_ARENA && tid == 0) S.o1[size_t(S.nb1) * kSegMaxRuns + r] = total;  // [nb1] = the run's total
        lds_barrier();
#pragma unroll
        for (uint32_t u = 0; u < U; u++)
            if (pos[u] != 0xffffffffu) {
                const uint32_t b = pos[u] >> 16, at = cnt[b] + (pos[u] & 0xffffu);
                srec[at] = rec[u];
                // (arena: the record's bucket, tagged so that no run's epoch
                // (<= kSegMaxRuns < 0x8000) ever equals it; the padded layout
                // reads it at group starts only)
                if (SKE_SEG_ARENA && (!padded || (at & 3u) == 0)) mark[at] = uint16_t(0x8000u | b);
            }
        if (SKE_SEG_ARENA) {
            // the run's chunk slots (after the placement, so that no record
            // registers are live across them); record j of the run (bucket h)
            // is then the bucket's sequence index i = j + (base - start of h
            // in the run), in the bucket's first or second chunk of this
            // reservation (told apart by i's chunk parity)
            const uint32_t aslot = cv ? seg_arena_slots(S, A.err, tid, cvp, abase) : 0u;
            lds_barrier();  // the placement's reads of cnt are done
            if (tid < S.nb1) {
                cnt[tid] = abase - (padded ? exp : ex);
                slt[tid] = aslot;
            }
            lds_barrier();
            auto slot_of = [](uint32_t i, uint32_t v) {
                return ((i >> 13) & 1u) == (v >> 28) ? (v & 0x3fffu) : ((v >> 14) & 0x3fffu);
            };
            if (padded) {
                // every 4-record group lies in one bucket and one chunk, 16-B
                // aligned at both ends (a group's first record is never a pad)
                const uint32_t ng = (tot2 >> 16) / 4;
                for (uint32_t g = tid; g < ng; g += T) {
                    const uint32_t h = mark[4 * g] & (kSegMaxB1 - 1), i = 4 * g + cnt[h];
                    nt2_st<1>(reinterpret_cast<part_u32x4 *>(S.r1 + size_t(slot_of(i, slt[h])) * kSegChunk +
                                                             (i & (kSegChunk - 1))),
                              reinterpret_cast<const part_u32x4 *>(srec)[g]);
                }
            } else {
                // (a run too full for its pads in LDS) four records per
                // thread: one 16-B store when they share a bucket and a chunk,
                // else one store each; each bucket's pad stored by its thread
                typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
                for (uint32_t g = tid; g * 4 < total; g += T) {
                    const uint32_t j = g * 4;
                    const part_u32x4 v = reinterpret_cast<const part_u32x4 *>(srec)[g];
                    const uint2 mk = reinterpret_cast<const uint2 *>(mark)[g];
                    const uint32_t m[4] = {mk.x & 0xffffu, mk.x >> 16, mk.y & 0xffffu, mk.y >> 16};
                    const uint32_t h0 = m[0] & (kSegMaxB1 - 1), i0 = j + cnt[h0];
                    if (j + 4 <= total && m[3] == m[0] && (i0 & (kSegChunk - 1)) <= kSegChunk - 4) {
                        *reinterpret_cast<u32x4a *>(S.r1 + size_t(slot_of(i0, slt[h0])) * kSegChunk +
                                                    (i0 & (kSegChunk - 1))) = u32x4a{v.x, v.y, v.z, v.w};
                    } else {
#pragma unroll
                        for (uint32_t e = 0; e < 4; e++) {
                            if (j + e >= total) break;
                            const uint32_t h = m[e] & (kSegMaxB1 - 1), i = j + e + cnt[h];
                            S.r1[size_t(slot_of(i, slt[h])) * kSegChunk + (i & (kSegChunk - 1))] = v[e];
                        }
                    }
                }
                if (tid < S.nb1)
                    for (uint32_t k = cv; k < cvp; k++)
                        S.r1[size_t(slot_of(abase + k, aslot)) * kSegChunk + ((abase + k) & (kSegChunk - 1))] = 0u;
            }
            lds_barrier();  // cnt, slt and marks are rewritten by the next run
        } else {
            lds_barrier();
            part_u32x4 *dst = reinterpret_cast<part_u32x4 *>(S.r1 + size_t(r) * kSegRunSw);
            const part_u32x4 *src = reinterpret_cast<const part_u32x4 *>(srec);
            for (uint32_t j = tid; j * 4 < total; j += T) nt2_st<1>(dst + j, src[j]);
        }
        // (the next run rewrites cnt, marks and srec only behind barriers
        // that every reader of this run's values has passed)
    }
}

// C1 with the next run's streams in flight (chains whose fail lists of a run
// fit NP 16-B pieces per thread: C3/C5's 152 slice pairs take 1216 of 2048).
// The run's slots, HLL words and fail lists are loaded into registers while
// the previous run is sorted and copied out; every memory operation after
// those loads is a buffer operation issued a fixed number of times (offsets
// past a range for lanes with nothing to do), so the wait for them is exact
// and does not wait for the copy-out's stores.  Same output as k_seg_c1.
__global__ void __launch_bounds__(1024) k_seg_scan(const SegArgs S) {

    __shared__ uint32_t ws[16];
    const uint32_t h = blockIdx.x, tid = threadIdx.x;
    const uint32_t *oa = S.o1 + size_t(h) * kSegMaxRuns, *ob = oa + kSegMaxRuns;
    uint32_t *pp = S.p1 + size_t(h) * (kSegMaxRuns + 1);
    uint32_t *cs = S.cst + size_t(h) * (kSegMaxRuns + 1);
    constexpr uint32_t kPer = kSegMaxRuns / 1024;  // runs per thread (nruns <= kSegMaxRuns)
    uint32_t c[kPer], sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
        const uint32_t r = kPer * tid + j;
        c[j] = r < S.nruns ? ob[r] - oa[r] : 0u;
        sum += c[j];
    }
    uint32_t total;
    uint32_t a = seg_scan(sum, ws, total);
    if (tid == 0) pp[S.nruns] = total;
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
        const uint32_t r = kPer * tid + j;
        if (r < S.nruns) pp[r] = a;
        // a run holds <= 8192 records: at most one chunk starts inside it
        for (uint32_t q = (a + kSegChunk - 1) / kSegChunk; q * kSegChunk < a + c[j]; q++) cs[q] = r;
        a += c[j];
    }
}

// D: per chunk of 8 192 records of one bucket, the records gathered from
// the level-1 runs that hold them and counting-sorted by window within the
// bucket.  A staged chunk (every chunk but a sparse bucket's: fewer than
// kSegDStage runs) keeps its runs' record prefix and, per run, the offset
// that turns a record index into its word in r1 (run * 8192 + start in run
// - prefix) in LDS, read through LDS pointers only (round 5 read them
// through a pointer that could be LDS or global: every table read a flat
// load); records are lane-interleaved (one buffer load covers 64
// consecutive records), each lane's run found by its own binary search, 8
// searches side by side (S + D 0.122 -> 0.100 ms per 2^25 sub-batch,
// profiles/r06_ab_seg_d.txt).  Not kept (profiles/r06_ab_seg_c1d.txt): the
// next chunk's run-table words loaded during this chunk's sort
// (SKE_SEG_D_PIPE 1: 0.101 -> 0.106 ms, 64 VGPRs with spills), and C1 with
// the next run's streams loaded during this run's sort (0.120 -> 0.163 ms,
// spills) or copy-out (0.122).
#ifndef SKE_SEG_D_PIPE
#define SKE_SEG_D_PIPE 0
#endif
// D's block: T threads, R = 8192 / T records each, BPC blocks per CU (1024 x
// 8 at 2 per CU, or 512 x 16 at 3 per CU: three chunks in flight per CU)
#ifndef SKE_SEG_DT
#define SKE_SEG_DT 512
#endif
template <uint32_t T> struct SegD {
    static constexpr uint32_t R = kSegChunk / T;                 // records per thread
    static constexpr uint32_t BPC = T == 1024 ? 2 : 3;           // blocks per CU
    static constexpr uint32_t STAGE = T == 1024 ? 2048 : 1536;   // runs of a chunk staged in LDS
    static constexpr uint32_t SPT = STAGE / T;                   // table words per thread
    static constexpr uint32_t WPE = BPC * (T / 64) / 4;          // waves per SIMD (launch bounds)
};
template <uint32_t T>
__global__ void __launch_bounds__(T, SegD<T>::WPE) k_seg_d(const SegArgs S) {
    using DC = SegD<T>;
    constexpr uint32_t R = DC::R, STAGE = DC::STAGE, SPT = DC::SPT;
    static_assert(STAGE % T == 0 && kSegChunk % T == 0 && STAGE <= kSegDStage && kSegMaxWpb <= T && kSegMaxB1 <= T,
                  "D geometry: whole table words and records per thread; a thread per window and per bucket");
    __shared__ uint32_t tot[kSegMaxB1], cbl[kSegMaxB1 + 1];
    // the chunk's runs' prefix and r1 offsets, staged when fewer than STAGE
    // runs hold it (a chunk of a sparse bucket spanning more reads them in place)
    __shared__ uint32_t spp[STAGE + 1], sob[STAGE];
    __shared__ uint32_t c2[kSegMaxWpb + 1];
    __shared__ __attribute__((aligned(16))) uint32_t sb[kSegChunk];
    __shared__ uint32_t ws[T / 64];
    const uint32_t tid = threadIdx.x, wpb = 1u << S.wlog;
    // the buckets' chunk bases (every block; block 0 keeps them for E)
    uint32_t t = 0;
    if (tid < S.nb1) {
        t = S.p1[size_t(tid) * (kSegMaxRuns + 1) + S.nruns];
        tot[tid] = t;
    }
    uint32_t nq;
    const uint32_t cbase = seg_scan(tid < S.nb1 ? (t + kSegChunk - 1) / kSegChunk : 0u, ws, nq);
    if (tid < S.nb1) {
        cbl[tid] = cbase;
        if (blockIdx.x == 0) S.cb[size_t(S.s) * (S.nb1 + 1) + tid] = cbase;
    }
    if (tid == 0) {
        cbl[S.nb1] = nq;
        if (blockIdx.x == 0) S.cb[size_t(S.s) * (S.nb1 + 1) + S.nb1] = nq;
    }
    lds_barrier();
    uint32_t *r2 = S.r2 + size_t(S.s) * S.maxch * kSegChunk;
    uint32_t *o2 = S.o2 + size_t(S.s) * S.maxch * (wpb + 1);
    const __amdgpu_buffer_rsrc_t rr1 = part_rsrc(S.r1, S.nruns * kSegRunSw * 4);
    const __amdgpu_buffer_rsrc_t rp1 = part_rsrc(S.p1, S.nb1 * (kSegMaxRuns + 1) * 4);
    const __amdgpu_buffer_rsrc_t ro1 = part_rsrc(S.o1, S.nb1 * kSegMaxRuns * 4);
    // chunk q: bucket h (block-uniform, in a scalar register, so its run
    // table's chunk starts are scalar loads), records [w0, w1) of the bucket,
    // held by runs [ga, ga + ng)
    struct Chunk {
        uint32_t h, w0, w1, ga, ng;
    };
    auto desc = [&](uint32_t q) {
        Chunk d;
        d.h = __builtin_amdgcn_readfirstlane(seg_last_le(cbl, S.nb1, q));  // buckets without chunks share the next one's base
        const uint32_t c = __builtin_amdgcn_readfirstlane(q - cbl[d.h]), th = __builtin_amdgcn_readfirstlane(tot[d.h]);
        d.w0 = c * kSegChunk;
        d.w1 = th - d.w0 < kSegChunk ? th : d.w0 + kSegChunk;
        const uint32_t *cs = S.cst + size_t(d.h) * (kSegMaxRuns + 1);
        d.ga = cs[c];
        const uint32_t gb = d.w1 < th ? cs[c + 1] + 1 : S.nruns;
        d.ng = gb - d.ga;
        return d;
    };
    // a staged chunk's table words j = tid + i T: prefix (j <= ng) and start
    // in run (j < ng); always the same loads (offsets past the range read
    // nothing), so the wait for the records before them is exact
    uint32_t ta[SPT], tb[SPT];
    auto tload = [&](const Chunk &d, bool on) {
#pragma unroll
        for (uint32_t i = 0; i < SPT; i++) {
            const uint32_t j = tid + i * T;
            const bool st = on && d.ng < STAGE;
            ta[i] = __builtin_amdgcn_raw_buffer_load_b32(
                rp1, st && j <= d.ng ? (d.h * (kSegMaxRuns + 1) + d.ga + j) * 4 : kOOR, 0, 0);
            tb[i] = __builtin_amdgcn_raw_buffer_load_b32(
                ro1, st && j < d.ng ? (d.h * kSegMaxRuns + d.ga + j) * 4 : kOOR, 0, 0);
        }
    };
    uint32_t q = blockIdx.x;
    Chunk cur{};
    if (q < nq) {
        cur = desc(q);
        tload(cur, true);
    }
    while (q < nq) {
        const bool staged = cur.ng < STAGE;  // block-uniform
        const uint32_t w0 = cur.w0, w1 = cur.w1, ga = cur.ga, ng = cur.ng;
        if (staged) {
#pragma unroll
            for (uint32_t i = 0; i < SPT; i++) {
                const uint32_t j = tid + i * T;
                if (j <= ng) spp[j] = ta[i];
                if (j < ng) sob[j] = (ga + j) * kSegRunSw + tb[i] - ta[i];
            }
        }
        for (uint32_t j = tid; j <= wpb; j += T) c2[j] = 0;
        lds_barrier();
        const uint32_t qn = q + gridDim.x;
        Chunk nx{};
        if (SKE_SEG_D_PIPE && qn < nq) nx = desc(qn);
        uint32_t rec[R], pos[R];
        if (staged) {
            uint32_t k[R];
#pragma unroll
            for (uint32_t j = 0; j < R; j++) k[j] = 0;
            for (uint32_t len = ng; len > 1;) {
                const uint32_t half = len >> 1;
#pragma unroll
                for (uint32_t j = 0; j < R; j++) {
                    const uint32_t p = w0 + j * T + tid;
                    k[j] = spp[k[j] + half] <= p ? k[j] + half : k[j];
                }
                len -= half;
            }
#pragma unroll
            for (uint32_t j = 0; j < R; j++) {
                const uint32_t p = w0 + j * T + tid;
                rec[j] = __builtin_amdgcn_raw_buffer_load_b32(rr1, p < w1 ? (sob[k[j]] + p) * 4 : kOOR, 0, nt2_aux<2>());
            }
        } else {
            // (a sparse bucket's chunk over more runs than LDS stages: the
            // run tables read in place, one search per thread, then a walk)
            const uint32_t *gpp = S.p1 + size_t(cur.h) * (kSegMaxRuns + 1) + ga;
            const uint32_t *gob = S.o1 + size_t(cur.h) * kSegMaxRuns + ga;
            const uint32_t p0 = w0 + tid * R;
            uint32_t k = p0 < w1 ? seg_last_le(gpp, ng, p0) : 0u;
#pragma unroll
            for (uint32_t j = 0; j < R; j++) {
                const uint32_t p = p0 + j;
                rec[j] = 0;
                if (p < w1) {
                    while (gpp[k + 1] <= p) k++;
                    rec[j] = S.r1[size_t(ga + k) * kSegRunSw + gob[k] + (p - gpp[k])];
                }
            }
        }
        // the next chunk's run table, in flight during this chunk's sort
        if (SKE_SEG_D_PIPE) tload(nx, qn < nq);
#pragma unroll
        for (uint32_t j = 0; j < R; j++) {
            pos[j] = 0xffffffffu;
            const uint32_t p = staged ? w0 + j * T + tid : w0 + tid * R + j;
            if (p < w1) {
                const uint32_t w2 = (rec[j] >> (kSegRecShift + S.klog)) & (wpb - 1);
                pos[j] = (w2 << 16) | atomicAdd(&c2[w2], 1u);
            }
        }
        lds_barrier();
        uint32_t total;
        const uint32_t ex = seg_scan(tid < wpb ? c2[tid] : 0u, ws, total);
        if (tid < wpb) {
            c2[tid] = ex;
            o2[size_t(q) * (wpb + 1) + tid] = ex;
        }
        if (tid == 0) o2[size_t(q) * (wpb + 1) + wpb] = total;
        lds_barrier();
#pragma unroll
        for (uint32_t j = 0; j < R; j++)
            if (pos[j] != 0xffffffffu) sb[c2[pos[j] >> 16] + (pos[j] & 0xffffu)] = rec[j];
        lds_barrier();
        part_u32x4 *dst = reinterpret_cast<part_u32x4 *>(r2 + size_t(q) * kSegChunk);
        const part_u32x4 *src = reinterpret_cast<const part_u32x4 *>(sb);
        for (uint32_t j = tid; j * 4 < total; j += T) nt2_st<4>(dst + j, src[j]);
        // (the next chunk rewrites spp / sob / c2 only after the barriers
        // that every reader of this chunk's values has passed)
        if (!SKE_SEG_D_PIPE && qn < nq) {
            nx = desc(qn);
            tload(nx, true);
        }
        q = qn;
        cur = nx;
    }
}

// D of the arena form: one block per chunk of the sub-batch (grid-stride, in
// bucket order), its slot fixed or from ctab, its records read whole (16-B loads), then
// the same window sort and outputs as k_seg_d (o2 / r2 row q = the bucket's
// first chunk + chunk, so E is unchanged).  It clears the chunk's ctab entry
// for the next sub-batch.
template <uint32_t T> struct SegDA {
    static constexpr uint32_t R = kSegChunk / T;        // records per thread
    static constexpr uint32_t BPC = T == 1024 ? 2 : 3;  // blocks per CU (80 VGPRs; LDS ~39 KiB each)
    static constexpr uint32_t WPE = BPC * (T / 64) / 4;
};
template <uint32_t T>
__global__ void __launch_bounds__(T, SegDA<T>::WPE) k_seg_da(const SegArgs S) {
    constexpr uint32_t R = SegDA<T>::R;
    static_assert(R % 4 == 0 && kSegMaxWpb <= T && kSegMaxB1 <= T, "D geometry");
    __shared__ uint32_t tot[kSegMaxB1], cbl[kSegMaxB1 + 1];
    __shared__ uint32_t c2[kSegMaxWpb + 1];
    __shared__ __attribute__((aligned(16))) uint32_t sb[kSegChunk];
    __shared__ uint32_t ws[T / 64];
    const uint32_t tid = threadIdx.x, wpb = 1u << S.wlog;
    const uint32_t *fl = S.fill + seg_fill_at(S, 0);
    uint32_t t = 0;
    if (tid < S.nb1) {
        t = fl[tid * kSegFillStride];
        tot[tid] = t;
    }
    uint32_t nq;
    const uint32_t cbase = seg_scan(tid < S.nb1 ? (t + kSegChunk - 1) / kSegChunk : 0u, ws, nq);
    if (tid < S.nb1) {
        cbl[tid] = cbase;
        if (blockIdx.x == 0) S.cb[size_t(S.s) * (S.nb1 + 1) + tid] = cbase;
    }
    if (tid == 0 && blockIdx.x == 0) S.cb[size_t(S.s) * (S.nb1 + 1) + S.nb1] = nq;
    lds_barrier();
    uint32_t *r2 = S.r2 + size_t(S.s) * S.maxch * kSegChunk;
    uint32_t *o2 = S.o2 + size_t(S.s) * S.maxch * (wpb + 1);
    // chunk q of the sub-batch (bucket order, dealt round robin): bucket h,
    // its chunk c, in a fixed slot or (c >= kstat) the counted one ctab names
    const uint32_t nstat = S.nb1 * S.kstat, nslot = nstat + fl[S.nb1 * kSegFillStride];
    const __amdgpu_buffer_rsrc_t rr1 = part_rsrc(S.r1, nslot * kSegChunk * 4);
    for (uint32_t q = blockIdx.x; q < nq; q += gridDim.x) {
        const uint32_t h = __builtin_amdgcn_readfirstlane(seg_last_le(cbl, S.nb1, q));  // (empty buckets share
        const uint32_t c = q - cbl[h];                                                   // the next one's base)
        uint32_t p = h * S.kstat + c;
        if (c >= S.kstat) {
            p = nstat + __builtin_amdgcn_readfirstlane(S.ctab[size_t(h) * S.kmaxc + c]) - 1;
            lds_barrier();  // every lane has read the entry
            if (tid == 0) S.ctab[size_t(h) * S.kmaxc + c] = 0;
        }
        const uint32_t w0 = c * kSegChunk, th = tot[h];
        const uint32_t n = th - w0 < kSegChunk ? th - w0 : kSegChunk;
        uint32_t rec[R];
#pragma unroll
        for (uint32_t k = 0; k < R / 4; k++) {
            const uint32_t x = (k * T + tid) * 4;  // the piece's first record in the chunk
            const part_u32x4 v = __builtin_bit_cast(
                part_u32x4, __builtin_amdgcn_raw_buffer_load_b128(rr1, x < n ? (p * kSegChunk + x) * 4 : kOOR, 0,
                                                                  nt2_aux<2>()));
            rec[4 * k] = v.x;
            rec[4 * k + 1] = v.y;
            rec[4 * k + 2] = v.z;
            rec[4 * k + 3] = v.w;
        }
        for (uint32_t j = tid; j <= wpb; j += T) c2[j] = 0;
        lds_barrier();
        uint32_t pos[R];
#pragma unroll
        for (uint32_t j = 0; j < R; j++) {
            pos[j] = 0xffffffffu;
            if ((j / 4 * T + tid) * 4 + j % 4 < n && (rec[j] & 63u) != 0) {  // (rank 0: a C1 pad)
                const uint32_t w2 = (rec[j] >> (kSegRecShift + S.klog)) & (wpb - 1);
                pos[j] = (w2 << 16) | atomicAdd(&c2[w2], 1u);
            }
        }
        lds_barrier();
        uint32_t total;
        const uint32_t ex = seg_scan(tid < wpb ? c2[tid] : 0u, ws, total);
        if (tid < wpb) {
            c2[tid] = ex;
            o2[size_t(q) * (wpb + 1) + tid] = ex;
        }
        if (tid == 0) o2[size_t(q) * (wpb + 1) + wpb] = total;
        lds_barrier();
#pragma unroll
        for (uint32_t j = 0; j < R; j++)
            if (pos[j] != 0xffffffffu) sb[c2[pos[j] >> 16] + (pos[j] & 0xffffu)] = rec[j];
        lds_barrier();
        part_u32x4 *dst = reinterpret_cast<part_u32x4 *>(r2 + size_t(q) * kSegChunk);
        const part_u32x4 *src = reinterpret_cast<const part_u32x4 *>(sb);
        for (uint32_t j = tid; j * 4 < total; j += T) nt2_st<4>(dst + j, src[j]);
        // (the next chunk rewrites c2 before its first barrier: the readers
        // of this chunk's c2 passed the barrier before the copy-out; sb is
        // rewritten only after two more barriers)
    }
}

// byte max of an LDS register (the window's copy); true if it rose
__device__ __forceinline__ bool seg_lds_max(uint32_t *w, uint32_t sh, uint32_t rank) {
    uint32_t old = *w;
    while (((old >> sh) & 0xffu) < rank) {
        const uint32_t prev = atomicCAS(w, old, (old & ~(0xffu << sh)) | (rank << sh));
        if (prev == old) return true;
        old = prev;
    }
    return false;
}

// The window pass.  A window whose records exceed its slice (a hot key's:
// at the 8-way shard the hottest lecture's day keys take ~1.8 M records of
// one window per step) is cut into slices so that no block reads more than
// slice of records (seg_slice): pass E1 (QUEUE = false) takes every window's first
// slice and queues the others; E2 (QUEUE = true) takes the queued slices;
// each slice of a cut window raises its own LDS copy of the window, stored
// whole to a copy buffer, and M (k_seg_m) stores the byte max of the copies.
// An uncut window's risen lines go straight back to the slab.
//
// Per window the block (1) issues the window's register loads (whole lines,
// 8 x 16 B per thread, kept in registers) and, at the same time, (2) reads
// the window's run table -- o2[chunk][window] of every chunk of its bucket
// in every sub-batch, the chunk bases from an LDS copy of cb -- then (3)
// reads the records 16 consecutive ones per thread (one search of the run
// prefix per thread, all 16 loads in flight), raises them in LDS and (4)
// stores the risen lines.  A window with fewer than dense_min records is
// raised in place instead (its register loads are dropped).
// Diagnostic per-item stamps of the window pass (-DSKE_SEG_STAMPS builds only;
// tools/stamps/run_seg_stamps.py): thread 0 records s_memrealtime (100 MHz)
// at 5 points of every window / queued slice, its record and run counts and
// its block and XCD, into a side buffer no output depends on.
#ifdef SKE_SEG_STAMPS
__device__ unsigned long long *ske_seg_stamp_buf;
hipError_t set_seg_stamp_buffer(void *p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(ske_seg_stamp_buf), &p, sizeof(void *));
}
#define SEG_STAMP(slot, k, v)                                                                  \
    do {                                                                                       \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        unsigned long long t_;                                                                 \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");        \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        if (threadIdx.x == 0 && ske_seg_stamp_buf) {                                           \
            ske_seg_stamp_buf[size_t(slot) * 8 + (k)] = t_;                                    \
            if ((k) == 4) {                                                                    \
                ske_seg_stamp_buf[size_t(slot) * 8 + 5] = (v);                                 \
                ske_seg_stamp_buf[size_t(slot) * 8 + 6] =                                      \
                    blockIdx.x | (uint64_t(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15) << 32); \
            }                                                                                  \
        }                                                                                      \
    } while (0)
#else
hipError_t set_seg_stamp_buffer(void *) { return hipErrorNotSupported; }
#define SEG_STAMP(slot, k, v) \
    do {                      \
    } while (0)
#endif
// Block shape per window size: windows of 2^KLOG keys (16 KiB each) in
// blocks of T threads, BPC blocks resident per CU (LDS: the window + its
// staging), so that small windows keep more windows in flight per CU.
#ifndef SKE_SEG_RPT1
#define SKE_SEG_RPT1 4
#endif
#ifndef SKE_SEG_BPC1
#define SKE_SEG_BPC1 4  // blocks per CU at klog 1
#endif
#ifndef SKE_SEG_CLAIM
#define SKE_SEG_CLAIM 1  // the window pass claims items from a counter
#endif
template <int KLOG> struct SegE {
    static constexpr uint32_t T = KLOG >= 2 ? 1024 : (KLOG == 1 ? 512 : 256);
    static constexpr uint32_t BPC = KLOG >= 3 ? 1 : (KLOG == 2 ? 2 : (KLOG == 1 ? SKE_SEG_BPC1 : 8));
    static constexpr uint32_t WPS = T / 64 * BPC / 4;  // waves per SIMD (launch bounds)
    static constexpr uint32_t RPT = KLOG >= 3 ? 16 : (KLOG == 2 ? 8 : SKE_SEG_RPT1);  // records per thread per round
    static constexpr uint32_t EP = KLOG == 2 ? 512 : T;  // runs staged at once
};
// records per slice of a cut window: SKE_SEG_SLICE << min(klog, 2) (64 k at
// klog 1: the window pass 0.930 -> 0.891 ms at N = 1 and 0.477 -> 0.427 ms at
// the 8-way shard against 32 k; 16 k / 8 k / 128 k slower --
// profiles/r05_ab_seg_slice.txt)
#ifndef SKE_SEG_SLICE
#define SKE_SEG_SLICE 32768
#endif
__host__ __device__ constexpr uint32_t seg_slice(uint32_t klog) { return uint32_t(SKE_SEG_SLICE) << (klog < 2 ? klog : 2); }

template <int KLOG, bool QUEUE>
__global__ void __launch_bounds__(SegE<KLOG>::T, SegE<KLOG>::WPS) k_seg_e(const PartArgs A, const SegArgs S) {
    using E = SegE<KLOG>;
    constexpr uint32_t T = E::T;
    constexpr uint32_t KW = 1u << KLOG, WB = KW << kHllP, NPC = WB / 16 / T;  // 16-B pieces per thread
    constexpr uint32_t NL = KW * (kHllRegs / 128);                              // 128-B lines
    constexpr uint32_t RPT = E::RPT, EP = E::EP;
    constexpr uint32_t SLICE = seg_slice(KLOG);
    __shared__ __attribute__((aligned(16))) uint8_t win[WB];
    __shared__ uint8_t dirty[NL];
    __shared__ uint32_t rb[EP], rp[EP + 1];
    __shared__ uint32_t spre[2][65], cq0[2][64], ws[T / 64], hdr[2];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t nb1m = S.nb1 - 1;  // buckets: a power of two, window W in bucket W & nb1m
    const uint32_t nitems = QUEUE ? S.q[0] : S.nwin;
    const __amdgpu_buffer_rsrc_t rr2 = part_rsrc(S.r2, S.nsub * S.maxch * kSegChunk * 4);
    // Items (E1: windows, E2: queued slices) go round robin over the blocks.
    // Each item's layout -- its bucket's chunk counts per sub-batch (spre:
    // prefix, cq0: the first chunk; nsub <= 64), double-buffered by item
    // parity -- its first EP runs and its window's registers are fetched in
    // phases while the previous item's records are raised and its lines
    // stored:
    //   P1  the bucket's chunk columns (loads), while the records are raised;
    //   P2  the column prefix (scan), then the item's first EP runs (loads),
    //       while the lines are stored; then the window's registers by
    //       LDS-DMA into `win`;
    //   P3  the runs' prefix (scan) and record count, when the item starts.
    // (Buckets interleave windows, so a hot key's windows fall in different
    // buckets and every bucket has about the same chunks: a window's runs
    // rarely exceed EP; more are counted and staged in batches.)
    uint32_t cq = 0, cc = 0;                // P1: this thread's sub-batch column
    uint32_t pbase = 0, plen = 0, pnp = 0;  // P2: this thread's run, the item's runs
    auto item = [&](uint32_t it, uint32_t &wi, uint32_t &sl, uint32_t &copy) {
        wi = it;
        sl = 0;
        copy = 0xffffffffu;
        if (QUEUE) {
            const uint4 e = S.qitems[it];
            wi = e.x;
            sl = e.y;
            copy = e.z;
        }
    };
    auto p1 = [&](uint32_t wi) {
        const uint32_t h = wi & nb1m;
        if (tid < S.nsub) {
            cq = S.cb[size_t(tid) * (S.nb1 + 1) + h];
            cc = S.cb[size_t(tid) * (S.nb1 + 1) + h + 1];
        }
    };
    // the window's registers into `win` by LDS-DMA (1 KiB per wave
    // instruction, no VGPRs; bytes past the slab read as zero), waited for by
    // the __syncthreads() before the records are raised
    auto image = [&](uint32_t wi) {
        const uint32_t slot0 = wi << KLOG;
        const uint32_t nk = A.nslots - slot0 < KW ? A.nslots - slot0 : KW;
        const __amdgpu_buffer_rsrc_t r = part_rsrc(A.regs + (size_t(slot0) << kHllP), nk << kHllP);
#pragma unroll
        for (uint32_t i = 0; i < NPC; i++) {
            const uint32_t piece = i * (T / 64) + wave;  // 1 KiB pieces
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                r, (__attribute__((address_space(3))) void *)(win + piece * 1024), 16,
                int(piece * 1024 + lane * 16), 0, 0, nt2_aux<16>());
        }
    };
    // run x of window column w2 of the bucket staged in buffer pb
    const uint32_t orow = (1u << S.wlog) + 1;
    auto run_of = [&](uint32_t pb, uint32_t x, uint32_t w2, uint32_t &base) -> uint32_t {
        const uint32_t s = seg_last_le(spre[pb], S.nsub, x);
        const size_t row = size_t(s) * S.maxch + cq0[pb][s] + (x - spre[pb][s]);
        const uint32_t *o = S.o2 + row * orow + w2;
        const uint32_t b = o[0];
        base = uint32_t(row * kSegChunk + b);  // < 2^32: the host plan checks nsub * maxch * kSegChunk
        return o[1] - b;
    };
    auto p2 = [&](uint32_t pb, uint32_t wi) {  // block-uniform; buffer pb is free
        const uint32_t c = tid < S.nsub ? cc - cq : 0u;
        const uint32_t ex = seg_scan(c, ws, pnp);
        if (tid < S.nsub) {
            spre[pb][tid] = ex;
            cq0[pb][tid] = cq;
        }
        lds_barrier();
        plen = 0;
        if (tid < EP && tid < pnp) plen = run_of(pb, tid, wi >> S.b1, pbase);
    };
    uint32_t it = blockIdx.x, par = 0;
    uint32_t wi_n = 0, sl_n = 0, copy_n = 0;
    if (it < nitems) {
        item(it, wi_n, sl_n, copy_n);
        p1(wi_n);
        p2(0, wi_n);
        image(wi_n);
    }
    // items past the first gridDim.x are claimed one ahead from a counter
    // (SKE_SEG_CLAIM; else every gridDim.x-th), so a block that drew a hot
    // window's long first slice takes fewer of the rest
    uint32_t nit = 0;
    for (; it < nitems; it = nit, par ^= 1) {
        const uint32_t wi = wi_n, sl = sl_n;
        uint32_t copy = copy_n;
        const uint32_t np = pnp;
        const uint32_t stamp = QUEUE ? S.nwin + it : wi;
        (void)stamp;
        SEG_STAMP(stamp, 0, 0);
        const uint32_t w2 = wi >> S.b1;
        const uint32_t slot0 = wi << KLOG;
        const uint32_t nk = A.nslots - slot0 < KW ? A.nslots - slot0 : KW;
        uint8_t *g = A.regs + (size_t(slot0) << kHllP);
        const uint32_t npc = nk << (kHllP - 4);  // the window's 16-B pieces in the slab
        // P3: the record count (the first batch of runs stays staged)
        uint32_t nrec, nrec0;
        {
            const uint32_t ex = seg_scan(plen, ws, nrec0);
            if (tid < EP) {
                rb[tid] = pbase;
                rp[tid] = ex;
            }
            if (tid == 0) rp[np < EP ? np : EP] = nrec0;
            nrec = nrec0;
            for (uint32_t x0 = EP; x0 < np; x0 += EP) {  // (more than EP runs: count the rest)
                uint32_t base = 0, len = 0, t;
                if (tid < EP && x0 + tid < np) len = run_of(par, x0 + tid, w2, base);
                (void)seg_scan(len, ws, t);
                nrec += t;
            }
        }
        SEG_STAMP(stamp, 1, 0);
        if (!QUEUE && nrec > SLICE) {
            // a hot window: cut into slices, the others queued for E2
            const uint32_t nsl = (nrec + SLICE - 1) / SLICE;
            if (tid == 0) {
                uint32_t base = atomicAdd(&S.q[1], nsl);
                if (base + nsl > S.ccap) {
                    base = 0xffffffffu;  // out of copies (cannot happen: see seg_scratch): one slice
                } else {
                    const uint32_t qp = atomicAdd(&S.q[0], nsl - 1);
                    for (uint32_t k = 1; k < nsl; k++) S.qitems[qp + k - 1] = make_uint4(wi, k, base + k, 0);
                    S.mlist[atomicAdd(&S.q[2], 1u)] = make_uint4(wi, base, nsl, 0);
                }
                hdr[0] = base;
            }
            lds_barrier();
            copy = hdr[0];
        }
        const bool cut = copy != 0xffffffffu;
        const uint32_t lo = cut ? sl * SLICE : 0;
        const uint32_t hi = cut ? (nrec - lo < SLICE ? nrec : lo + SLICE) : nrec;
        const bool dense = nrec > 0 && (cut || nrec >= S.dense_min);
        if (dense)
            for (uint32_t j = tid; j < NL; j += T) dirty[j] = 0;
        // (E1: per XCD -- block b takes items i = b mod 8 from counter b mod 8,
        // so the windows of a bucket (W mod nb1) stay on one XCD, whose L2
        // then serves the chunk lines two neighbouring windows' runs share)
        // (every residue mod 8 needs a block: a grid under 8 takes one counter)
        if (SKE_SEG_CLAIM && tid == 0)
            hdr[1] = QUEUE || gridDim.x < kPGroups
                         ? gridDim.x + atomicAdd(&S.q[QUEUE ? 5 : 4], 1u)
                         : gridDim.x + kPGroups * atomicAdd(&S.q[8 + blockIdx.x % kPGroups], 1u) +
                               blockIdx.x % kPGroups;
        __syncthreads();  // the window's registers landed in LDS (vmcnt), its first runs staged
        // P1 of the next item: its loads fly while this item's records are raised
        nit = SKE_SEG_CLAIM ? hdr[1] : it + gridDim.x;
        if (nit < nitems) {
            item(nit, wi_n, sl_n, copy_n);
            p1(wi_n);
        }
        SEG_STAMP(stamp, 2, 0);
        // records [lo, hi) of the concatenated runs, runs staged EP at a time
        for (uint32_t x0 = 0, p0 = 0; x0 < np && p0 < hi; x0 += EP) {
            const uint32_t nx = np - x0 < EP ? np - x0 : EP;
            uint32_t btot = nrec0;
            if (x0 > 0) {  // (a window with more than EP runs: restage)
                lds_barrier();
                uint32_t base = 0, len = 0;
                if (tid < nx) len = run_of(par, x0 + tid, w2, base);
                const uint32_t ex = seg_scan(len, ws, btot);
                if (tid < nx) {
                    rb[tid] = base;
                    rp[tid] = ex;
                }
                if (tid == 0) rp[nx] = btot;
                lds_barrier();
            }
            // this batch's records [p0, p0 + btot) of the window; ours: [lo, hi).
            // A wave takes 64 * RPT consecutive records per round, lane l the
            // ones at l + 64 c (coalesced loads); the run of the wave's first
            // record is searched once and every lane walks on from it.
            const uint32_t f_lo = lo > p0 ? lo - p0 : 0, f_hi = hi - p0 < btot ? hi - p0 : btot;
            // (dense: the window's registers in LDS; sparse: in place, in HBM)
            const __amdgpu_buffer_rsrc_t rgw = part_rsrc(g, npc * 16);
            auto round = [&](auto dense_c) {
                constexpr bool D = decltype(dense_c)::value;
                for (uint32_t r0 = f_lo + wave * 64 * RPT; r0 - wave * 64 * RPT < f_hi; r0 += T * RPT) {
                    uint32_t rec[RPT];
#pragma unroll
                    for (uint32_t c = 0; c < RPT; c++) rec[c] = 0;
                    if (r0 < f_hi) {  // wave-uniform
                        uint32_t j = seg_last_le(rp, nx, r0);
#pragma unroll
                        for (uint32_t c = 0; c < RPT; c++) {
                            const uint32_t f = r0 + c * 64 + lane;
                            if (f < f_hi) {
                                while (rp[j + 1] <= f) j++;
                                rec[c] = __builtin_amdgcn_raw_buffer_load_b32(rr2, (rb[j] + (f - rp[j])) * 4, 0, nt2_aux<8>());
                            }
                        }
                    }
                    // the registers' words, all read before any CAS (a raise
                    // is rare once the slab is warm)
                    uint32_t old[RPT];
#pragma unroll
                    for (uint32_t c = 0; c < RPT; c++) {
                        const uint32_t a = (((rec[c] >> kSegRecShift) & (KW - 1)) << kHllP) | ((rec[c] >> 6) & 0x3fffu);
                        old[c] = 0xffffffffu;
                        if (rec[c] & 63u)
                            old[c] = D ? reinterpret_cast<const uint32_t *>(win)[a >> 2]
                                       : __builtin_amdgcn_raw_buffer_load_b32(rgw, a & ~3u, 0, 0);
                    }
#pragma unroll
                    for (uint32_t c = 0; c < RPT; c++) {
                        const uint32_t a = (((rec[c] >> kSegRecShift) & (KW - 1)) << kHllP) | ((rec[c] >> 6) & 0x3fffu);
                        const uint32_t rank = rec[c] & 63u, sh = (a & 3u) * 8;
                        if (((old[c] >> sh) & 0xffu) >= rank) continue;
                        if constexpr (D) {
                            if (seg_lds_max(reinterpret_cast<uint32_t *>(win + (a & ~3u)), sh, rank)) dirty[a >> 7] = 1;
                        } else {
                            part_reg_max(reinterpret_cast<uint32_t *>(g + (a & ~3u)), sh, rank, old[c]);
                        }
                    }
                }
            };
            if (dense)
                round(std::true_type{});
            else
                round(std::false_type{});
            p0 += btot;
        }
        lds_barrier();  // every raise in LDS done; rb / rp free
        SEG_STAMP(stamp, 3, 0);
        // P2 of the next item (its layout into the other buffer), its runs'
        // loads flying while this item's lines are stored
        if (nit < nitems) p2(par ^ 1, wi_n);
        if (cut) {
            // a slice of a cut window: the whole LDS copy, merged by k_seg_m
            part_u32x4 *dst = reinterpret_cast<part_u32x4 *>(S.copies + size_t(copy) * WB);
#pragma unroll
            for (uint32_t i = 0; i < NPC; i++) dst[i * T + tid] = reinterpret_cast<const part_u32x4 *>(win)[i * T + tid];
        } else if (dense) {
            // the lines that rose, stored back whole
#pragma unroll
            for (uint32_t i = 0; i < NPC; i++) {
                const uint32_t j = i * T + tid;
                if (j < npc && dirty[j >> 3])
                    nt2_st<32>(reinterpret_cast<part_u32x4 *>(g) + j, reinterpret_cast<const part_u32x4 *>(win)[j]);
            }
        }
        lds_barrier();  // win, dirty and hdr are rewritten by the next item
        if (nit < nitems) image(wi_n);
        SEG_STAMP(stamp, 4, uint64_t(nrec) | (uint64_t(np) << 32) | (uint64_t(dense) << 63));
    }
}

// bytewise max of two 16-byte pieces
__device__ __forceinline__ part_u32x4 seg_max16(part_u32x4 a, part_u32x4 b) {
    typedef unsigned char u8x16 __attribute__((ext_vector_type(16)));
    return __builtin_bit_cast(part_u32x4,
                              __builtin_elementwise_max(__builtin_bit_cast(u8x16, a), __builtin_bit_cast(u8x16, b)));
}

// M: every cut window = the byte max of its slices' copies (each started
// from the slab's registers, so the max holds every slice's raises)
template <int KLOG>
__global__ void __launch_bounds__(1024) k_seg_m(const PartArgs A, const SegArgs S) {
    constexpr uint32_t KW = 1u << KLOG, WB = KW << kHllP;
    const uint32_t nm = S.q[2];
    for (uint32_t m = blockIdx.x; m < nm; m += gridDim.x) {
        const uint4 e = S.mlist[m];
        const uint32_t slot0 = e.x << KLOG;
        const uint32_t nk = A.nslots - slot0 < KW ? A.nslots - slot0 : KW;
        part_u32x4 *g = reinterpret_cast<part_u32x4 *>(A.regs + (size_t(slot0) << kHllP));
        for (uint32_t j = threadIdx.x; j < (nk << (kHllP - 4)); j += 1024) {
            part_u32x4 v = reinterpret_cast<const part_u32x4 *>(S.copies + size_t(e.y) * WB)[j];
            for (uint32_t c = 1; c < e.z; c++)
                v = seg_max16(v, reinterpret_cast<const part_u32x4 *>(S.copies + size_t(e.y + c) * WB)[j]);
            g[j] = v;
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
static uint32_t part_stride(uint32_t ksum, uint32_t tile) { return ((ksum * tile) + 31) & ~31u; }

// the fail-list instantiation: one link of k = 11 (C3/C5's filter), slice
// pairs (the sink pair must fit k_part_a3<11, 2048>'s counters)
static bool part_flist(const PartArgs &A) { return A.nlinks == 1 && A.ksum == 11 && A.nslices <= 2046; }
// swipes per tile: kTileFl for the fail-list chains, 1024 for the others
static uint32_t part_tile(const PartArgs &A) { return part_flist(A) ? kTileFl : kPaBlock; }

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
    A->nunits = (slices + 1) / 2;
    A->stride = part_stride(ksum, part_tile(*A));
    return true;
}

bool part_supported(const ChainDev &ch) {
    PartArgs A{};
    return part_plan(ch, &A);
}

// The group layout's geometry (k_part_a3<11, 1024, true>): a (group of 8
// tiles, unit) region holds the unit's expected records of the group plus
// six standard deviations, the runs' padding and a line; the overflow rows
// after the regions take k_part_a3's padded LDS layout (stride 13 312).
// False when the layout does not apply or its offsets would pass 2^31 bytes.
// Only on request (rec_groups 1): at C3 it moves pass B 0.195 -> 0.183 ms
// and pass A 0.226 -> 0.388 ms per 16 M sub-batch -- a run's edge lines are
// written by two tiles, partial-line writes.
static bool part_glayout(PartArgs *A, const SegOpts &so, uint32_t ntiles_max) {
    A->gcap = A->govf = 0;
    if (so.rec_groups != 1 || !part_flist(*A) || A->nunits >= 512 || kTileFl != 1024) return false;
    const double d = double(A->link[0].d);
    const double share = std::min(d, double(2 * kPSliceBits)) / d;  // of the largest unit
    const double mu = 8.0 * 1024 * A->ksum * share;
    const uint64_t cap = (uint64_t(mu + 6 * std::sqrt(mu) + 8 * 3 + 32) + 31) & ~uint64_t(31);
    const uint64_t stride = ((1024u * 11 + 4 * (1024 / 2)) + 31) & ~31u;
    const uint64_t govf = uint64_t((ntiles_max + 7) / 8) * A->nunits * cap;
    if (cap >= 65536 || (govf + uint64_t(ntiles_max) * stride) * 4 >= (uint64_t(1) << 31)) return false;
    A->gcap = uint32_t(cap);
    A->govf = uint32_t(govf);
    A->stride = uint32_t(stride);
    return true;
}

// the scratch of a sub-batch of up to `sub` swipes (context scratch slots
// 28-31 and 44: probe records, run boundaries, fail bytes, HLL words, and the
// fail lists of one-link chains)
static hipError_t part_scratch(PartArgs *A, uint64_t n, uint32_t sub, const SegOpts &so, Scratch *scr) {
    const uint32_t m = n < sub ? uint32_t(n) : sub;
    const uint32_t tile = part_tile(*A);
    const uint32_t ntiles_max = (m + tile - 1) / tile;
    const uint32_t fstride = (m + 255) & ~255u;
    A->off_stride = (ntiles_max + 15) & ~15u;
    hipError_t e = hipSuccess;
    part_glayout(A, so, ntiles_max);
    A->rec = (uint32_t *)scratch_get(scr, 28, (size_t(A->govf) + size_t(ntiles_max) * A->stride) * 4, &e);
    if (e == hipSuccess) A->off = (uint32_t *)scratch_get(scr, 29, size_t(A->off_stride) * (A->nslices + 1) * 4, &e);
    // (fail bytes: the fail-list chains keep their overflow flags in the HLL words)
    A->fail = nullptr;
    if (e == hipSuccess && !part_flist(*A))
        A->fail = (uint8_t *)scratch_get(scr, 30, size_t(fstride) * A->nlinks, &e);
    if (e == hipSuccess) A->hllw = (uint32_t *)scratch_get(scr, 31, size_t(m) * 4, &e);
    A->fail_stride = fstride;
    A->fl_stride = A->off_stride;
    A->flist = nullptr;
    if (e == hipSuccess && A->nlinks == 1)
        A->flist = (uint16_t *)scratch_get(scr, 44, size_t(A->nunits) * A->fl_stride * kPbLanes * 2, &e);
    return e;
}

// swipes per sub-batch: the option (at most the largest, kPSub, whose probe
// records of one XCD tile group stay within a 2^31-byte buffer range --
// k_part_b's rsrc, relative to the group's first tile; SKE_PB_SPLIT 1: of
// all tiles -- 2^26 for every chain the plan takes), or kPSubDefault: 2^25
// measured as fast as 2^26 at C3 and faster than 2^24 (profiles/r05_ab_subbatch.txt)
constexpr uint32_t kPSubDefault = 1u << 25;
static uint32_t part_sub(uint32_t sub_opt, const PartArgs &A) {
    const uint64_t tiles = ((uint64_t(1) << 31) - 1) / (uint64_t(A.stride) * 4);
    const uint64_t span = SKE_PB_SPLIT == 1 ? tiles : (tiles - 8) * kPGroups;  // tiles a sub-batch may have
    const uint32_t tile = part_tile(A);
    const uint32_t cap = uint32_t(std::min<uint64_t>(kPSub / tile * tile, span / 8 * 8 * tile));
    uint32_t sub = sub_opt ? sub_opt : std::min(cap, kPSubDefault);
    sub = (sub + tile - 1) / tile * tile;
    return sub < tile ? tile : (sub > cap ? cap : sub);
}

// the scratch before the first launch (so a graph recorded later holds it)
// The segmented PFADD's geometry for a slab of nslots keys and a batch of n
// swipes in sub-batches of `sub`: windows of 2^klog keys (W = slot >> klog);
// 2^b1 level-1 buckets of 2^wlog windows each, window W in bucket W mod
// 2^b1 (buckets interleave windows, so the consecutive windows of a hot
// lecture's day keys fall in different buckets and every bucket carries
// about the same records), b1 + wlog = ceil(log2(windows)) split evenly so
// that both levels' runs stay long; false when the slab needs more than 2^9
// buckets of 2^9 windows.
struct SegPlan {
    uint32_t s1, b1, wlog, klog, nb1, nwin, maxch, nsub, dense_min;
};
static bool seg_plan(uint32_t nslots, uint64_t n, uint32_t sub, const SegOpts &so, SegPlan *P) {
    if (nslots == 0 || n == 0 || so.klog < 0 || so.klog > 3) return false;
    const uint32_t klog = uint32_t(so.klog);
    const uint32_t nwin = uint32_t((uint64_t(nslots) + (1u << klog) - 1) >> klog);
    uint32_t tb = 0;
    while ((uint64_t(1) << tb) < nwin) tb++;
    // windows per bucket 2^wlog: at least half the window bits, and at least
    // tb - 5 (2^25 sub-batches: level-2 sorts over more windows beat longer
    // level-1 segments up to 2^9; profiles/r05_ab_seg_b1.txt: b1 7 at C3's
    // 2^16 windows, 5 at the 8-way shard's 2^13)
    uint32_t wlog = std::max((tb + 1) / 2, tb > 5 ? tb - 5 : 0u), b1 = tb - wlog;
    if (wlog > 9) {
        wlog = 9;
        b1 = tb - 9;
    }
    if (so.b1 >= 0) {  // the option: level-1 buckets 2^b1 (windows per bucket 2^(tb - b1) <= 2^9)
        b1 = uint32_t(so.b1) < tb ? uint32_t(so.b1) : tb;
        wlog = tb - b1;
    }
    if (b1 > 9) {
        b1 = 9;
        wlog = tb - 9;
    }
    if (wlog > 9) return false;
    P->klog = klog;
    P->wlog = wlog;
    P->b1 = b1;
    P->s1 = klog + wlog;
    P->nwin = nwin;
    P->nb1 = 1u << b1;
    P->maxch = (sub + kSegChunk - 1) / kSegChunk + P->nb1;
    // sub-batches per window pass: at most 64, and their level-2 records
    // within a 2^31-byte buffer range (the window pass's record loads); a
    // batch of more runs a window pass after every nsub of them
    const uint64_t kmax = ((uint64_t(1) << 29) - 1) / (uint64_t(P->maxch) * kSegChunk);
    const uint64_t ns = (n + sub - 1) / sub;
    if (kmax == 0) return false;
    P->nsub = uint32_t(std::min<uint64_t>(std::min<uint64_t>(ns, kmax), 64));
    const uint64_t dm = uint64_t(so.dense_min_x100) * ((uint64_t(1) << klog) * (kHllRegs / 128)) / 100;
    P->dense_min = dm < 1 ? 1u : (dm > 0xffffffffu ? 0xffffffffu : uint32_t(dm));
    return true;
}

// segmented for this batch: the fail-list chain, the option, and (auto) at
// least density_x100 / 100 swipes per 128-B register line of the slab
static bool seg_use(const PartArgs &A, const SegOpts &so, uint32_t nslots, uint64_t n, uint32_t sub, SegPlan *P) {
    if (so.mode == 0 || !part_flist(A) || !seg_plan(nslots, n, sub, so, P)) return false;
    if (so.mode == 1) return true;
    // break-evens measured at C3: ~5 swipes per line over a
    // 1.6 GB slab, ~12 over the 8-way shard's 205 MB one, which the 256 MiB
    // Infinity Cache holds (pass C's random requests are served there): the
    // threshold doubles for a slab of at most 256 MiB, so the shard's 16 M
    // step (~11 per line) takes pass C and its 2^27 step (~92) this form
    const uint64_t thr = uint64_t(so.density_x100) * ((uint64_t(nslots) << kHllP) <= (256ull << 20) ? 2 : 1);
    return n * 100 >= thr * nslots * (kHllRegs / 128);
}

// the segmented PFADD's scratch (context slots 32-38)
static hipError_t seg_scratch(const SegPlan &P, uint32_t sub, uint64_t n, Scratch *scr, SegArgs *S) {
    const uint64_t m = n < sub ? n : sub;
    const uint64_t mg = std::min<uint64_t>(n, uint64_t(P.nsub) * sub);  // swipes of one window pass
    hipError_t e = hipSuccess;
    if (SKE_SEG_ARENA) {
        // chunk slots: about twice a bucket's mean fixed per bucket, and as
        // many counted ones as the sub-batch could ever need (every bucket's
        // last chunk may be partial); slot numbers < 2^14 (k_seg_c1's packing)
        const uint64_t ch = (m + kSegChunk - 1) / kSegChunk, dyn = ch + P.nb1;
        uint64_t kst = 2 * ((ch + P.nb1 - 1) / P.nb1) + 2;
        kst = std::min<uint64_t>(kst, ((1u << 14) - 1 - dyn) / P.nb1);
        S->kstat = uint32_t(kst);
        S->kmaxc = uint32_t(ch + 1);
        S->r1 = (uint32_t *)scratch_get(scr, 32, size_t(P.nb1 * kst + dyn) * kSegChunk * 4, &e);
        if (e == hipSuccess)
            S->fill = (uint32_t *)scratch_get(scr, 40, size_t(P.nsub) * (P.nb1 + 1) * kSegFillStride * 4, &e);
        if (e == hipSuccess) S->ctab = (uint32_t *)scratch_get(scr, 41, size_t(P.nb1) * S->kmaxc * 4, &e);
    } else {
        S->r1 = (uint32_t *)scratch_get(scr, 32, size_t((m + kSegRunSw - 1) / kSegRunSw) * kSegRunSw * 4, &e);
        if (e == hipSuccess) S->o1 = (uint32_t *)scratch_get(scr, 33, size_t(P.nb1 + 1) * kSegMaxRuns * 4, &e);
        if (e == hipSuccess) S->p1 = (uint32_t *)scratch_get(scr, 34, size_t(P.nb1) * (kSegMaxRuns + 1) * 4, &e);
        if (e == hipSuccess) S->cst = (uint32_t *)scratch_get(scr, 35, size_t(P.nb1) * (kSegMaxRuns + 1) * 4, &e);
    }
    if (e == hipSuccess)
        S->r2 = (uint32_t *)scratch_get(scr, 36, size_t(P.nsub) * P.maxch * kSegChunk * 4, &e);
    if (e == hipSuccess)
        S->o2 = (uint32_t *)scratch_get(scr, 37, size_t(P.nsub) * P.maxch * ((1u << P.wlog) + 1) * 4, &e);
    if (e == hipSuccess) S->cb = (uint32_t *)scratch_get(scr, 38, size_t(P.nsub) * (P.nb1 + 1) * 4, &e);
    // the window pass's cut windows: a cut window has > slice records and
    // ceil(records / slice) < 2 records / slice slices, so 2 n / slice
    // copies, queue entries and cut windows always suffice
    const uint32_t ccap = uint32_t(2 * ((mg + seg_slice(P.klog) - 1) / seg_slice(P.klog)) + 2);
    const size_t wb = size_t(1) << (P.klog + kHllP);
    if (e == hipSuccess) S->q = (uint32_t *)scratch_get(scr, 39, 64, &e);
    if (e == hipSuccess) S->qitems = (uint4 *)scratch_get(scr, 42, size_t(ccap) * 16, &e);
    if (e == hipSuccess) S->mlist = (uint4 *)scratch_get(scr, 43, size_t(ccap) * 16, &e);
    if (e == hipSuccess) S->copies = (uint8_t *)scratch_get(scr, 45, size_t(ccap) * wb, &e);
    S->ccap = ccap;
    S->nb1 = P.nb1;
    S->s1 = P.s1;
    S->b1 = P.b1;
    S->wlog = P.wlog;
    S->klog = P.klog;
    S->nsub = P.nsub;
    S->maxch = P.maxch;
    S->nwin = P.nwin;
    S->dense_min = P.dense_min;
    return e;
}

hipError_t part_reserve(const ChainDev &ch, uint64_t n, uint32_t sub_opt, uint32_t nslots, const SegOpts &so,
                        Scratch *scr) {
    PartArgs A{};
    if (!part_plan(ch, &A)) return hipErrorInvalidValue;
    const uint32_t sub = part_sub(sub_opt, A);
    hipError_t e = part_scratch(&A, n ? n : 1, sub, so, scr);
    SegPlan P;
    if (e == hipSuccess && seg_use(A, so, nslots, n ? n : 1, sub, &P)) {
        SegArgs S{};
        e = seg_scratch(P, sub, n, scr, &S);
        // scratch that cannot grow under a recorded graph: such a batch takes
        // pass C instead (launch_swipes_part decides the same way)
        if (e == hipErrorStreamCaptureUnsupported) e = hipSuccess;
    }
    return e;
}

// Units = (batch, sub-batch of at most `sub` swipes), in order, each as the
// three passes on `st`.  `hook` (pass timing) brackets every kernel.
hipError_t launch_swipes_part(const ChainDev &ch, const PartBatch *bt, uint32_t nb, uint8_t *regs,
                              uint32_t nslots, Scratch *scr, unsigned int *err, int cus, uint32_t sub_opt,
                              const SegOpts &so, hipStream_t st, PassHook hook, void *hook_user) {
    PartArgs A{};
    if (!part_plan(ch, &A)) return hipErrorInvalidValue;
    const uint32_t sub = part_sub(sub_opt, A);
    uint64_t nmax = 0;
    for (uint32_t j = 0; j < nb; j++) nmax = bt[j].n > nmax ? bt[j].n : nmax;
    if (nmax == 0) return hipSuccess;
    hipError_t e = part_scratch(&A, nmax, sub, so, scr);
    if (e != hipSuccess) return e;
    const uint32_t tile = part_tile(A);
    A.regs = regs;
    A.nslots = nslots;
    A.err = err;
    const uint32_t km = part_km(A.ksum);
    // one link of k = 11 (C3/C5): slice pairs and fail lists
    const bool flist = part_flist(A) && A.flist != nullptr;
    const bool pairs = A.nlinks == 1;  // a one-link chain is probed in slice pairs (128 KiB images)
    const unsigned ga = unsigned(cus) * (km <= 11 ? 2u : 1u) / kPGroups * kPGroups;  // blocks past a group's tiles exit
    const unsigned g2 = unsigned(cus) * 2 / kPGroups * kPGroups;  // k_part_a3: two blocks per CU
    const unsigned gb = unsigned(cus) * (pairs ? 1 : 2) / kPGroups * kPGroups;  // all resident
    for (uint32_t j = 0; j < nb; j++) {
        const PartBatch &B = bt[j];
        // fixed-width ids: a sub-batch's byte offsets (swipe * width) stay 32-bit
        uint32_t subj = sub;
        if (!B.offs && B.fixed_w) {
            const uint64_t cap = (0xffffff00ull / B.fixed_w) / tile * tile;
            subj = cap < sub ? uint32_t(cap < tile ? tile : cap) : sub;
        }
        // sub-batches of even size (a 17.6 M batch as 2 x 8.8 M, not 16 M +
        // 1.6 M: a small last sub-batch cannot fill the chip)
        if (B.n > subj) {
            const uint64_t ns = (B.n + subj - 1) / subj;
            subj = uint32_t(((B.n + ns - 1) / ns + tile - 1) / tile * tile);
        }
        // the segmented PFADD (k_seg_*) for this batch, or pass C per sub-batch
        SegPlan P;
        SegArgs S{};
        bool seg = flist && seg_use(A, so, nslots, B.n, subj, &P);
        if (seg) {
            e = seg_scratch(P, subj, B.n, scr, &S);
            // (recording a graph with scratch too small for this batch's
            // segmented PFADD: the batch takes pass C, same answers and registers)
            if (e == hipErrorStreamCaptureUnsupported) {
                seg = false;
                e = hipSuccess;
            }
            if (e != hipSuccess) return e;
        }
        // every window of the slab once after each group of P.nsub
        // sub-batches (the whole batch unless it is very large): E1 (first
        // slices), E2 (queued slices of cut windows), M (cut windows merged)
        auto window_pass = [&](uint32_t ns) -> hipError_t {
            S.nsub = ns;
            A.n = 0;
            if (hook) hook(hook_user, 4, 0, st);
            hipError_t we = hipMemsetAsync(S.q, 0, 64, st);
            if (we != hipSuccess) return we;
            switch (P.klog) {
#define SEG_E_LAUNCH(K)                                                                                  \
    case K:                                                                                              \
        hipLaunchKernelGGL((k_seg_e<K, false>), dim3(unsigned(cus) * SegE<K>::BPC), dim3(SegE<K>::T), 0, st, A, S); \
        hipLaunchKernelGGL((k_seg_e<K, true>), dim3(unsigned(cus) * SegE<K>::BPC), dim3(SegE<K>::T), 0, st, A, S);  \
        hipLaunchKernelGGL(k_seg_m<K>, dim3(unsigned(cus)), dim3(1024), 0, st, A, S);                    \
        break;
                SEG_E_LAUNCH(0)
                SEG_E_LAUNCH(1)
                SEG_E_LAUNCH(2)
                SEG_E_LAUNCH(3)
#undef SEG_E_LAUNCH
            }
            if (hook) hook(hook_user, 4, 1, st);
            return hipGetLastError();
        };
        uint32_t si = 0;
        for (uint64_t s0 = 0; s0 < B.n; s0 += subj, si++) {
            const uint32_t ms = B.n - s0 < subj ? uint32_t(B.n - s0) : subj;
            A.fixed_w = B.fixed_w;
            A.n = ms;
            A.ntiles = (ms + tile - 1) / tile;
            A.bytes = B.offs ? B.bytes : B.bytes + s0 * B.fixed_w;
            A.offs = B.offs ? B.offs + s0 : nullptr;
            A.slot = B.slot + s0;
            A.out = B.out ? B.out + s0 : nullptr;
            if (hook) hook(hook_user, 0, 0, st);
            if (A.gcap)  // the group layout (C3/C5 by default)
                hipLaunchKernelGGL((k_part_a3<11, 1024, true>), dim3(g2), dim3(512), 0, st, A);
            else if (flist && A.nunits < 512)  // C3/C5: 152 pairs, two counters per thread
                hipLaunchKernelGGL((k_part_a3<11, 1024, false, kTileFl>), dim3(g2), dim3(512), 0, st, A);
            else if (flist)
                hipLaunchKernelGGL((k_part_a3<11, 2048, false, kTileFl>), dim3(g2), dim3(512), 0, st, A);
            else if (km <= 11)
                hipLaunchKernelGGL(k_part_a<11>, dim3(ga), dim3(kPaBlock), 0, st, A);
            else
                hipLaunchKernelGGL(k_part_a<22>, dim3(ga), dim3(kPaBlock), 0, st, A);
            if (hook) hook(hook_user, 0, 1, st);
            if (hook) hook(hook_user, 1, 0, st);
            if (A.gcap)
                hipLaunchKernelGGL((k_part_b<2, 4, true, true>), dim3(gb), dim3(kPbBlock), 0, st, A);
            else if (flist)
                hipLaunchKernelGGL((k_part_b<2, kPbRFl, true, false, kTileFl>), dim3(gb), dim3(kPbBlock), 0, st, A);
            else if (pairs)
                hipLaunchKernelGGL(k_part_b<2>, dim3(gb), dim3(kPbBlock), 0, st, A);
            else
                hipLaunchKernelGGL(k_part_b<1>, dim3(gb), dim3(kPbBlock), 0, st, A);
            if (hook) hook(hook_user, 1, 1, st);
            if (hook) hook(hook_user, 2, 0, st);
            if (seg) {
                S.s = si % P.nsub;
                S.nruns = (A.ntiles + kSegRunTiles - 1) / kSegRunTiles;
                if (SKE_SEG_ARENA && S.s == 0) {
                    // the group's fill counts, and the chunk table (D clears
                    // what C1 published, so this only matters for a fresh
                    // buffer or a call that stopped between C1 and D)
                    e = hipMemsetAsync(S.fill, 0, size_t(P.nsub) * (P.nb1 + 1) * kSegFillStride * 4, st);
                    if (e == hipSuccess) e = hipMemsetAsync(S.ctab, 0, size_t(P.nb1) * S.kmaxc * 4, st);
                    if (e != hipSuccess) return e;
                }
                hipLaunchKernelGGL(k_seg_c1<SKE_SEG_C1T>, dim3(std::min(S.nruns, unsigned(cus) * SegC1<SKE_SEG_C1T>::BPC)),
                                   dim3(SKE_SEG_C1T), 0, st, A, S);
                if (hook) hook(hook_user, 2, 1, st);
                if (hook) hook(hook_user, 3, 0, st);
                if (SKE_SEG_ARENA) {
                    hipLaunchKernelGGL(k_seg_da<SKE_SEG_DT>, dim3(unsigned(cus) * SegDA<SKE_SEG_DT>::BPC),
                                       dim3(SKE_SEG_DT), 0, st, S);
                } else {
                    hipLaunchKernelGGL(k_seg_scan, dim3(S.nb1), dim3(1024), 0, st, S);
                    hipLaunchKernelGGL(k_seg_d<SKE_SEG_DT>, dim3(unsigned(cus) * SegD<SKE_SEG_DT>::BPC),
                                       dim3(SKE_SEG_DT), 0, st, S);
                }
                if (hook) hook(hook_user, 3, 1, st);
            } else if (flist) {
                const unsigned gc =
                    (part_grid(ms, kTileFl * kPbGroup, unsigned(cus) * SKE_PC_BLOCKS_PER_CU) + kPGroups - 1) /
                    kPGroups * kPGroups;
                hipLaunchKernelGGL((k_part_c_fl<kPcFlT, kTileFl / kPcFlT, kTileFl>), dim3(gc), dim3(kPcFlT), 0, st, A);
            } else {
                const unsigned gc = (part_grid(ms, kPcBlock * 2, unsigned(cus) * 8) + kPGroups - 1) / kPGroups * kPGroups;
                hipLaunchKernelGGL(k_part_c<2>, dim3(gc), dim3(kPcBlock), 0, st, A);
            }
            if (!seg && hook) hook(hook_user, 2, 1, st);
            e = hipGetLastError();
            if (e != hipSuccess) return e;
            if (seg && ((si + 1) % P.nsub == 0 || s0 + subj >= B.n)) {
                e = window_pass(si % P.nsub + 1);
                if (e != hipSuccess) return e;
            }
        }
    }
    return hipSuccess;
}

}  // namespace ske
