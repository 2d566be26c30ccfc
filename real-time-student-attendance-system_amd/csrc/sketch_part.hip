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
#include "sketch_common.h"
#include "sketch_internal.h"

namespace ske {

constexpr uint32_t kPaBlock = 1024;
constexpr uint32_t kPbBlock = 1024;
constexpr uint32_t kPcBlock = 256;
constexpr uint32_t kPSliceMask = kPSliceBits - 1;
constexpr uint32_t kPSliceBytes = kPSliceBits / 8;  // 64 KiB
constexpr uint32_t kPSub = 1u << 24;                // swipes per sub-batch (passes A-B-C)
constexpr uint32_t kPbGroup = 8;                    // tiles a pass-B wave has in flight

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
    PartLink link[kPMaxLinks];
};

__device__ __forceinline__ Divisor part_div(const PartLink &L) { return Divisor{L.d, L.m, L.t, L.sh, 0}; }

// ---------------------------------------------------------------------------
// pass A: hash, probe records, counting sort by slice
// ---------------------------------------------------------------------------
// One tile = 1024 swipes, one per thread.  KM: the most probes per swipe the
// instantiation holds (every link's k summed); records of a tile live in LDS
// (KM = 11: 44 KiB, two blocks per CU, so one block's hashing overlaps the
// other's sort and copy-out).
template <int KM>
__global__ void __launch_bounds__(kPaBlock, KM <= 11 ? 8 : 4) k_part_a(const PartArgs A) {
    __shared__ __attribute__((aligned(16))) uint32_t srec[kPaBlock * KM];
    __shared__ uint32_t scnt[kPMaxSlices + 1];  // slice histogram, then run starts
    __shared__ uint32_t swsum[kPaBlock / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t S = A.nslices;
    for (uint32_t g = tid; g <= kPMaxSlices; g += kPaBlock) scnt[g] = 0;
    __syncthreads();
    for (uint32_t t = blockIdx.x; t < A.ntiles; t += gridDim.x) {
        uint32_t rv[KM], rp[KM];
        {
            const uint32_t i = t * kPaBlock + tid;
            const bool act = i < A.n;
            const uint32_t ic = act ? i : A.n - 1;
            const uint32_t b = A.offs ? A.offs[ic] : ic * A.fixed_w;
            const uint32_t e = A.offs ? A.offs[ic + 1] : b + A.fixed_w;
            const Item it = load_item(A.bytes, b, e);
            const bool sh = it.len <= 8;
            const uint64_t ha = sh ? murmur_short(it.w0, it.len, kBloomSeed) : murmur_item(it, kBloomSeed);
            const uint64_t hb = sh ? murmur_short(it.w0, it.len, ha) : murmur_item(it, ha);
            const uint64_t hh = sh ? murmur_short(it.w0, it.len, kHllSeed) : murmur_item(it, kHllSeed);
            if (act) {
                uint32_t idx, rank;
                hll_patlen(hh, idx, rank);
                A.hllw[i] = idx | (rank << 16);
                for (uint32_t l = 0; l < A.nlinks; l++) A.fail[size_t(l) * A.fail_stride + i] = 0;
            }
            // every link's k probes in RedisBloom's order, newest link first
            // (the order is immaterial to the answer; records carry no link:
            // a slice belongs to one link)
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
                    rv[q] = (x & kPSliceMask) | (tid << kPSliceLog);
                    if (act) rp[q] = (g << 16) | atomicAdd(&scnt[g], 1u);
                    wk.step(A.link[l].d);
                    jl++;
                }
            }
        }
        __syncthreads();
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
        __syncthreads();
        const uint32_t total = scnt[S];
        uint4 *dst = reinterpret_cast<uint4 *>(A.rec + size_t(t) * A.stride);
        const uint4 *src = reinterpret_cast<const uint4 *>(srec);
        for (uint32_t j = tid; j * 4 < total; j += kPaBlock) dst[j] = src[j];
        for (uint32_t g = tid; g <= S; g += kPaBlock) scnt[g] = 0;  // for the next tile
        __syncthreads();  // srec / scnt are reused by the next tile
    }
}

// ---------------------------------------------------------------------------
// pass B: one LDS-resident slice per block, probe its runs
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kPbBlock, 8) k_part_b(const PartArgs A, uint32_t splits) {
    __shared__ __attribute__((aligned(16))) uint8_t img[kPSliceBytes];
    const uint32_t g = blockIdx.x / splits, q = blockIdx.x % splits;
    uint32_t l = 0;
    while (l + 1 < A.nlinks && g >= A.link[l + 1].slice0) l++;
    const PartLink &L = A.link[l];
    const uint32_t b0 = (g - L.slice0) * kPSliceBytes;
    const uint32_t nb = L.nbytes16 - b0 < kPSliceBytes ? L.nbytes16 - b0 : kPSliceBytes;
    for (uint32_t o = threadIdx.x * 16; o < nb; o += kPbBlock * 16)
        *reinterpret_cast<uint4 *>(img + o) = *reinterpret_cast<const uint4 *>(L.bf + b0 + o);
    __syncthreads();
    const uint32_t t0 = uint32_t(uint64_t(A.ntiles) * q / splits);
    const uint32_t t1 = uint32_t(uint64_t(A.ntiles) * (q + 1) / splits);
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr uint32_t kWaves = kPbBlock / 64;
    uint8_t *fail = A.fail + size_t(l) * A.fail_stride;
    const uint32_t *obeg = A.off + size_t(g) * A.off_stride;
    const uint32_t *oend = obeg + A.off_stride;
    // a wave takes kPbGroup consecutive tiles at a time (wave-uniform): their
    // run boundaries are two rows of the slice-major table, and two 64-record
    // rounds of every run are in flight together; longer runs finish in a
    // tail loop
    for (uint32_t tg = t0 + wave * kPbGroup; tg < t1; tg += kWaves * kPbGroup) {
        uint32_t beg[kPbGroup], end[kPbGroup], r[2][kPbGroup];
#pragma unroll
        for (uint32_t k = 0; k < kPbGroup; k++) {
            const bool in = tg + k < t1;
            beg[k] = in ? obeg[tg + k] : 0;
            end[k] = in ? oend[tg + k] : 0;
        }
#pragma unroll
        for (uint32_t c = 0; c < 2; c++)
#pragma unroll
            for (uint32_t k = 0; k < kPbGroup; k++) {
                const uint32_t i = beg[k] + c * 64 + lane;
                r[c][k] = i < end[k] ? __builtin_nontemporal_load(&A.rec[size_t(tg + k) * A.stride + i])
                                     : 0xffffffffu;
            }
#pragma unroll
        for (uint32_t c = 0; c < 2; c++)
#pragma unroll
            for (uint32_t k = 0; k < kPbGroup; k++) {
                const uint32_t rr = r[c][k];
                if (rr == 0xffffffffu) continue;
                const uint32_t o = rr & kPSliceMask;
                if (!((img[o >> 3] >> (o & 7)) & 1)) fail[(tg + k) * kPaBlock + (rr >> kPSliceLog)] = 1;
            }
        for (uint32_t k = 0; k < kPbGroup; k++) {
            for (uint32_t i = beg[k] + 128 + lane; i < end[k]; i += 64) {
                const uint32_t rr = A.rec[size_t(tg + k) * A.stride + i];
                const uint32_t o = rr & kPSliceMask;
                if (!((img[o >> 3] >> (o & 7)) & 1)) fail[(tg + k) * kPaBlock + (rr >> kPSliceLog)] = 1;
            }
        }
    }
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
    const uint64_t stride = uint64_t(gridDim.x) * T * U;
    for (uint64_t base = uint64_t(blockIdx.x) * T * U; base < A.n; base += stride) {
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
            if (i < A.n) {
                for (uint32_t l = 0; l < A.nlinks; l++) valid[u] |= A.fail[size_t(l) * A.fail_stride + i] == 0;
                if (valid[u]) {
                    const uint32_t s = A.slot[i];
                    if (s >= A.nslots) {
                        atomicOr(A.err, 1u);
                    } else {
                        const uint32_t hv = A.hllw[i];
                        const uint32_t ridx = hv & 0xffffu;
                        w[u] = reinterpret_cast<uint32_t *>(A.regs + (uint64_t(s) << kHllP) + (ridx & ~3u));
                        sh[u] = (ridx & 3) * 8;
                        rank[u] = hv >> 16;
                    }
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) cur[u] = w[u] ? *w[u] : 0xffffffffu;
#pragma unroll
        for (int u = 0; u < U; u++)
            if (w[u]) part_reg_max(w[u], sh[u], rank[u], cur[u]);
        if (A.out) {
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint64_t i = base + uint64_t(u) * T + tid;
                if (i < A.n) A.out[i] = valid[u];
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
    A->stride = (kPaBlock * ksum + 3) & ~3u;
    return true;
}

bool part_supported(const ChainDev &ch) {
    PartArgs A{};
    return part_plan(ch, &A);
}

// the scratch of a sub-batch of up to `sub` swipes (slots 28-31 of the context
// scratch: probe records, run boundaries, fail bytes, HLL words)
static hipError_t part_scratch(PartArgs *A, uint64_t n, uint32_t sub, Scratch *scr) {
    const uint32_t m = n < sub ? uint32_t(n) : sub;
    const uint32_t ntiles_max = (m + kPaBlock - 1) / kPaBlock;
    const uint32_t fstride = (m + 255) & ~255u;
    A->off_stride = (ntiles_max + 15) & ~15u;
    hipError_t e = hipSuccess;
    A->rec = (uint32_t *)scratch_get(scr, 28, size_t(ntiles_max) * A->stride * 4, &e);
    if (e == hipSuccess) A->off = (uint32_t *)scratch_get(scr, 29, size_t(A->off_stride) * (A->nslices + 1) * 4, &e);
    if (e == hipSuccess) A->fail = (uint8_t *)scratch_get(scr, 30, size_t(fstride) * A->nlinks, &e);
    if (e == hipSuccess) A->hllw = (uint32_t *)scratch_get(scr, 31, size_t(m) * 4, &e);
    A->fail_stride = fstride;
    return e;
}

static uint32_t part_sub(uint32_t sub_opt) {
    uint32_t sub = sub_opt ? sub_opt : kPSub;
    sub = (sub + kPaBlock - 1) / kPaBlock * kPaBlock;
    return sub < kPaBlock ? kPaBlock : (sub > kPSub ? kPSub : sub);
}

hipError_t part_reserve(const ChainDev &ch, uint64_t n, uint32_t sub_opt, Scratch *scr) {
    PartArgs A{};
    if (!part_plan(ch, &A)) return hipErrorInvalidValue;
    return part_scratch(&A, n ? n : 1, part_sub(sub_opt), scr);
}

hipError_t launch_swipes_part(const ChainDev &ch, const uint8_t *bytes, const uint32_t *offs,
                              uint32_t fixed_w, const uint32_t *slot, uint64_t n, uint8_t *regs,
                              uint32_t nslots, uint8_t *out, Scratch *scr, unsigned int *err, int cus,
                              uint32_t sub_opt, hipStream_t st) {
    if (n == 0) return hipSuccess;
    PartArgs A{};
    if (!part_plan(ch, &A)) return hipErrorInvalidValue;
    const uint32_t sub = part_sub(sub_opt);
    hipError_t e = part_scratch(&A, n, sub, scr);
    if (e != hipSuccess) return e;
    A.regs = regs;
    A.nslots = nslots;
    A.err = err;
    A.fixed_w = fixed_w;
    const uint32_t km = part_km(A.ksum);
    for (uint64_t s0 = 0; s0 < n; s0 += sub) {
        const uint32_t ms = n - s0 < sub ? uint32_t(n - s0) : sub;
        A.n = ms;
        A.ntiles = (ms + kPaBlock - 1) / kPaBlock;
        A.bytes = offs ? bytes : bytes + s0 * fixed_w;
        A.offs = offs ? offs + s0 : nullptr;
        A.slot = slot + s0;
        A.out = out ? out + s0 : nullptr;
        const unsigned per_cu = km <= 11 ? 2 : 1;
        const unsigned ga = A.ntiles < unsigned(cus) * per_cu ? A.ntiles : unsigned(cus) * per_cu;
        if (km <= 11)
            hipLaunchKernelGGL(k_part_a<11>, dim3(ga), dim3(kPaBlock), 0, st, A);
        else
            hipLaunchKernelGGL(k_part_a<22>, dim3(ga), dim3(kPaBlock), 0, st, A);
        // about three rounds of 2 blocks per CU, at least one block per slice
        uint32_t splits = (uint32_t(cus) * 6 + A.nslices - 1) / A.nslices;
        const uint32_t maxsplit = (A.ntiles + kPbGroup - 1) / kPbGroup;
        splits = splits < 1 ? 1 : (splits > maxsplit ? maxsplit : splits);
        hipLaunchKernelGGL(k_part_b, dim3(A.nslices * splits), dim3(kPbBlock), 0, st, A, splits);
        hipLaunchKernelGGL(k_part_c<2>, dim3(part_grid(ms, kPcBlock * 2, cus * 8)), dim3(kPcBlock), 0,
                           st, A);
    }
    return hipGetLastError();
}

}  // namespace ske
