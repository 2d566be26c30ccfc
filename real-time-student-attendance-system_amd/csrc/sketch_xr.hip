// sketch_xr.hip -- K1 for Bloom chains too large for LDS (C3/C5: 19.8 MB),
// XCD-partitioned.
//
// A random probe into a 19.8 MB bit array misses the 4 MiB per-XCD L2 ~80 % of
// the time and is served by the Infinity Cache (PMC: 64 B fetched per probe,
// L2 hit 18 %).  Here the bit space of every link is cut into kRegions = 8
// slices (~2.5 MB each); block b tests only the probes that fall in slice
// b % 8 of the swipes of chunk b / 8.  With the dispatcher dealing blocks
// round-robin over the 8 XCDs, every XCD then keeps one slice L2-resident
// (PMC: L2 hit 93 %).  Placement is a speed matter only: every (chunk, slice)
// pair is processed by exactly one block, whatever XCD it lands on.
//
//   k_xr_hash:   once per swipe: MurmurHash64A a, b and, per link, the
//                32-bit probe state {x0 = a mod d, bm = b mod d, wrap mask}
//                (bit i set when a + i*b wraps 2^64 at step i), plus the
//                HLL word (register index | rank << 16) -- 12 B per link + 4 B.
//   k_xr_region: per (chunk, slice): walk each link's k probes in 32-bit
//                arithmetic, test the ones inside the slice (early exit when
//                no lane of the wave is still undecided); failures become a
//                per-wave ballot mask fail[slice][link][wave] (one u64 store).
//   k_xr_finish: link l passes iff no slice failed it; valid = any link
//                passes; then register max (pre-check, CAS) and the answer.
// The answer is SBChain_Check's: a link says "present" iff all k bits are
// set, the chain iff any link does.
#include "sketch_common.h"
#include "sketch_internal.h"

namespace ske {

constexpr int kXrMaxLinks = 8;

__device__ __forceinline__ void xr_reg_max(uint8_t *reg, uint32_t rank) {
    const uint32_t bsel = uint32_t(reinterpret_cast<uintptr_t>(reg) & 3);
    uint32_t *w = reinterpret_cast<uint32_t *>(reg - bsel);
    const uint32_t sh = bsel * 8;
    uint32_t old = *w;
    while (((old >> sh) & 0xffu) < rank) {
        const uint32_t prev = atomicCAS(w, old, (old & ~(0xffu << sh)) | (rank << sh));
        if (prev == old) return;
        old = prev;
    }
}

struct XrState {
    uint32_t *x0, *bm, *wrap;  // [link][n]
    uint32_t *hll;             // [n]: register | rank << 16 (0 = no HLL work)
};

__global__ void __launch_bounds__(256)
    k_xr_hash(const ChainDev ch, const uint8_t *__restrict__ bytes,
              const uint32_t *__restrict__ offs, uint32_t fixed_w, uint64_t n, XrState st) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t b = fixed_w ? i * fixed_w : offs[i];
        const uint64_t e = fixed_w ? b + fixed_w : offs[i + 1];
        const Item it = load_item(bytes, b, e);
        const bool sh = it.len <= 8;
        const uint64_t ha = sh ? murmur_short(it.w0, it.len, kBloomSeed) : murmur_item(it, kBloomSeed);
        const uint64_t hb = sh ? murmur_short(it.w0, it.len, ha) : murmur_item(it, ha);
        const uint64_t hh = sh ? murmur_short(it.w0, it.len, kHllSeed) : murmur_item(it, kHllSeed);
        for (int l = 0; l < ch.nlinks; l++) {
            const LinkDev &L = ch.link[l];
            uint32_t wrap = 0;
            uint64_t v = ha;
            for (uint32_t j = 1; j < L.k; j++) {
                const uint64_t vn = v + hb;
                wrap |= uint32_t(vn < v) << j;
                v = vn;
            }
            st.x0[uint64_t(l) * n + i] = uint32_t(fastmod(ha, L.div));
            st.bm[uint64_t(l) * n + i] = uint32_t(fastmod(hb, L.div));
            st.wrap[uint64_t(l) * n + i] = wrap;
        }
        uint32_t idx, rank;
        hll_patlen(hh, idx, rank);
        st.hll[i] = idx | (rank << 16);
    }
}

template <int U>
__global__ void __launch_bounds__(256)
    k_xr_region(const ChainDev ch, uint64_t n, uint64_t chunk, XrState st,
                unsigned long long *__restrict__ fail) {
    const uint32_t T = blockDim.x, tid = threadIdx.x;
    const uint32_t region = blockIdx.x % kRegions;
    const uint64_t c0 = uint64_t(blockIdx.x / kRegions) * chunk;
    const uint64_t c1 = c0 + chunk < n ? c0 + chunk : n;
    const uint64_t nwaves = (n + 63) / 64;
    for (int l = ch.nlinks - 1; l >= 0; --l) {
        const LinkDev &L = ch.link[l];
        const uint32_t d = uint32_t(L.div.d), t = uint32_t(L.div.t);
        // slice of this block: [lo, lo + len) bits, 1024-bit (128 B) aligned
        const uint32_t slice = ((d + kRegions - 1) / kRegions + 1023) & ~1023u;
        const uint32_t lo = region * slice;
        const uint32_t len = lo >= d ? 0u : (d - lo < slice ? d - lo : slice);
        // bit array through a buffer descriptor: 32-bit byte offsets, range
        // checked by the hardware
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(L.bf), 0, int(d >> 3), 0x00020000);
        for (uint64_t base = c0; base < c1; base += uint64_t(T) * U) {
            uint32_t x[U], inc0[U], inc1[U], wrap[U];
            bool ok[U], act[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint64_t i = base + uint64_t(u) * T + tid;
                act[u] = i < c1;
                ok[u] = act[u];
                x[u] = act[u] ? st.x0[uint64_t(l) * n + i] : 0u;
                inc0[u] = act[u] ? st.bm[uint64_t(l) * n + i] : 0u;
                wrap[u] = act[u] ? st.wrap[uint64_t(l) * n + i] : 0u;
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                // the step that wraps a + i*b adds bm - (2^64 mod d) instead
                const uint32_t m = inc0[u] - t;
                inc1[u] = umin32(m, m + d);
            }
            for (uint32_t j = 0; j < L.k; j++) {
                uint32_t byte[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const bool mine = ok[u] && (x[u] - lo) < len;
                    byte[u] = mine ? uint32_t(__builtin_amdgcn_raw_buffer_load_b8(rsrc, x[u] >> 3, 0, 0))
                                   : 0xffu;
                }
                bool any = false;
#pragma unroll
                for (int u = 0; u < U; u++) {
                    ok[u] = ok[u] && ((byte[u] >> (x[u] & 7)) & 1);
                    any |= ok[u];
                    x[u] += ((wrap[u] >> (j + 1)) & 1) ? inc1[u] : inc0[u];
                    x[u] = umin32(x[u], x[u] - d);
                }
                if (!__any(any)) break;
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const unsigned long long m = __ballot(act[u] && !ok[u]);
                // only waves holding swipes of this chunk store (a wave past
                // c1 would overwrite the next chunk's mask of this slice)
                const uint64_t first = base + uint64_t(u) * T + (tid & ~63u);
                if ((tid & 63) == 0 && first < c1)
                    fail[(uint64_t(region) * ch.nlinks + l) * nwaves + first / 64] = m;
            }
        }
    }
}

// The slice pass with every probe of a tile in flight at once (k <= 16): the
// walk for all k steps is computed first and each in-slice probe issued as a
// buffer load, then the bits are tested.  No wave-level exit between steps: a
// member (90 % of the swipes) is alive in every slice through all k steps, so
// a per-step exit test only serialises k memory round trips (the loop above
// waits for every probe before taking the next step).
constexpr int kXrBatchK = 16;

// KB: probes issued per swipe (the smallest instantiated count >= every
// link's k; loads past k are issued out of range, and every lane of an issued
// load costs address-unit time whether it is in the slice or not)
template <int U, int KB>
__global__ void __launch_bounds__(256)
    k_xr_region_b(const ChainDev ch, uint64_t n, uint64_t chunk, XrState st,
                  unsigned long long *__restrict__ fail) {
    const uint32_t T = blockDim.x, tid = threadIdx.x;
    const uint32_t region = blockIdx.x % kRegions;
    const uint64_t c0 = uint64_t(blockIdx.x / kRegions) * chunk;
    const uint64_t c1 = c0 + chunk < n ? c0 + chunk : n;
    const uint64_t nwaves = (n + 63) / 64;
    for (int l = ch.nlinks - 1; l >= 0; --l) {
        const LinkDev &L = ch.link[l];
        const uint32_t d = uint32_t(L.div.d), t = uint32_t(L.div.t), k = L.k;
        const uint32_t slice = ((d + kRegions - 1) / kRegions + 1023) & ~1023u;
        const uint32_t lo = region * slice;
        const uint32_t len = lo >= d ? 0u : (d - lo < slice ? d - lo : slice);
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(L.bf), 0, int(d >> 3), 0x00020000);
        for (uint64_t base = c0; base < c1; base += uint64_t(T) * U) {
            uint32_t x[U], inc0[U], inc1[U], wrap[U], ok[U];
            bool act[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint64_t i = base + uint64_t(u) * T + tid;
                act[u] = i < c1;
                const uint64_t ic = act[u] ? i : c0;
                x[u] = st.x0[uint64_t(l) * n + ic];
                inc0[u] = st.bm[uint64_t(l) * n + ic];
                wrap[u] = st.wrap[uint64_t(l) * n + ic];
            }
            uint32_t byte[U][KB], pos[U][KB];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t m = inc0[u] - t;
                inc1[u] = umin32(m, m + d);
#pragma unroll
                for (int j = 0; j < KB; j++) {
                    // a probe outside the slice (or past k) reads out of range: 0,
                    // and is not tested below
                    const bool mine = uint32_t(j) < k && (x[u] - lo) < len;
                    pos[u][j] = x[u];
                    byte[u][j] = __builtin_amdgcn_raw_buffer_load_b8(
                        rsrc, mine ? (x[u] >> 3) : 0x80000000u, 0, 0);
                    x[u] += ((wrap[u] >> (j + 1)) & 1) ? inc1[u] : inc0[u];
                    x[u] = umin32(x[u], x[u] - d);
                }
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                ok[u] = act[u];
#pragma unroll
                for (int j = 0; j < KB; j++) {
                    const bool mine = uint32_t(j) < k && (pos[u][j] - lo) < len;
                    ok[u] &= mine ? __builtin_amdgcn_ubfe(byte[u][j], pos[u][j] & 7, 1) : 1u;
                }
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const unsigned long long m = __ballot(act[u] && !ok[u]);
                const uint64_t first = base + uint64_t(u) * T + (tid & ~63u);
                if ((tid & 63) == 0 && first < c1)
                    fail[(uint64_t(region) * ch.nlinks + l) * nwaves + first / 64] = m;
            }
        }
    }
}

template <int U>
__global__ void __launch_bounds__(256)
    k_xr_finish(const ChainDev ch, const uint32_t *__restrict__ slot, uint64_t n,
                const uint32_t *__restrict__ hllw, uint8_t *__restrict__ regs, uint32_t nslots,
                uint8_t *__restrict__ out, const unsigned long long *__restrict__ fail,
                unsigned int *__restrict__ err) {
    const uint64_t nwaves = (n + 63) / 64;
    const uint32_t T = blockDim.x, tid = threadIdx.x;
    const uint64_t stride = uint64_t(gridDim.x) * T * U;
    for (uint64_t base = uint64_t(blockIdx.x) * T * U; base < n; base += stride) {
        bool valid[U];
        uint8_t *reg[U];
        uint32_t rank[U], cur[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t i = base + uint64_t(u) * T + tid;
            valid[u] = false;
            reg[u] = nullptr;
            rank[u] = 0;
            if (i < n) {
                const uint64_t w = i / 64;
                const uint32_t lane = uint32_t(i & 63);
                for (int l = 0; l < ch.nlinks && !valid[u]; l++) {
                    unsigned long long f = 0;
#pragma unroll
                    for (int r = 0; r < kRegions; r++)
                        f |= fail[(uint64_t(r) * ch.nlinks + l) * nwaves + w];
                    valid[u] = !((f >> lane) & 1);
                }
                if (valid[u]) {
                    const uint32_t s = slot[i];
                    if (s >= nslots) {
                        atomicOr(err, 1u);
                    } else {
                        const uint32_t hv = hllw[i];
                        reg[u] = regs + size_t(s) * kHllRegs + (hv & 0xffff);
                        rank[u] = hv >> 16;
                    }
                }
            }
        }
        // the U register pre-checks in flight together
#pragma unroll
        for (int u = 0; u < U; u++) cur[u] = reg[u] ? *reg[u] : 0xffu;
#pragma unroll
        for (int u = 0; u < U; u++)
            if (cur[u] < rank[u]) xr_reg_max(reg[u], rank[u]);
        if (out) {
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint64_t i = base + uint64_t(u) * T + tid;
                if (i < n) out[i] = valid[u];
            }
        }
    }
}

static inline unsigned grid_for(uint64_t n, unsigned block, unsigned cap) {
    uint64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    return unsigned(g < cap ? g : cap);
}

bool xr_supported(const ChainDev &ch) {
    if (ch.nlinks < 1 || ch.nlinks > kXrMaxLinks) return false;
    for (int l = 0; l < ch.nlinks; l++)
        if (ch.link[l].div.d > (uint64_t(1) << 31) || ch.link[l].k > 31) return false;
    return true;
}

uint64_t xr_scratch_bytes(uint64_t n, int nlinks) {
    const uint64_t fail = uint64_t(kRegions) * nlinks * ((n + 63) / 64) * 8;
    return fail + (uint64_t(nlinks) * 3 + 1) * n * 4 + 256;
}

hipError_t launch_swipes_xr(const ChainDev &ch, const uint8_t *bytes, const uint32_t *offs,
                            uint32_t fixed_w, const uint32_t *slot, uint64_t n, uint8_t *regs,
                            uint32_t nslots, uint8_t *out, void *scratch, unsigned int *err,
                            int cus, int region_u, int finish_u, hipStream_t st) {
    if (n == 0) return hipSuccess;
    auto *fail = reinterpret_cast<unsigned long long *>(scratch);
    uint32_t *p = reinterpret_cast<uint32_t *>(fail + uint64_t(kRegions) * ch.nlinks * ((n + 63) / 64));
    XrState s;
    s.x0 = p;
    s.bm = p + uint64_t(ch.nlinks) * n;
    s.wrap = p + 2 * uint64_t(ch.nlinks) * n;
    s.hll = p + 3 * uint64_t(ch.nlinks) * n;
    hipLaunchKernelGGL(k_xr_hash, dim3(grid_for(n, 256, cus * 8)), dim3(256), 0, st, ch, bytes, offs,
                       fixed_w, n, s);
    const int ru = region_u < 0 ? -region_u : region_u;
    const int U = ru >= 8 ? 8 : (ru >= 4 ? 4 : (ru >= 2 ? 2 : 1));
    const uint64_t tile = 256 * uint64_t(U);
    uint64_t chunks = uint64_t(cus) * 8 / kRegions;  // 8 blocks per CU in total
    uint64_t chunk = (n + chunks - 1) / chunks;
    chunk = (chunk + tile - 1) / tile * tile;
    chunks = (n + chunk - 1) / chunk;
    const dim3 g(unsigned(chunks * kRegions));
    uint32_t kmax = 0;
    for (int l = 0; l < ch.nlinks; l++) kmax = ch.link[l].k > kmax ? ch.link[l].k : kmax;
    const bool batch = region_u > 0 && kmax <= uint32_t(kXrBatchK);  // < 0: the per-step loop
    if (batch) {
#define SKE_XR_B(KB)                                                                               \
    if (U >= 2) hipLaunchKernelGGL((k_xr_region_b<2, KB>), g, dim3(256), 0, st, ch, n, chunk, s, fail); \
    else hipLaunchKernelGGL((k_xr_region_b<1, KB>), g, dim3(256), 0, st, ch, n, chunk, s, fail);
        if (kmax <= 7) { SKE_XR_B(7) }
        else if (kmax <= 8) { SKE_XR_B(8) }
        else if (kmax <= 10) { SKE_XR_B(10) }
        else if (kmax <= 11) { SKE_XR_B(11) }
        else if (kmax <= 13) { SKE_XR_B(13) }
        else { SKE_XR_B(16) }
#undef SKE_XR_B
    } else if (U == 8) hipLaunchKernelGGL(k_xr_region<8>, g, dim3(256), 0, st, ch, n, chunk, s, fail);
    else if (U == 4) hipLaunchKernelGGL(k_xr_region<4>, g, dim3(256), 0, st, ch, n, chunk, s, fail);
    else if (U == 2) hipLaunchKernelGGL(k_xr_region<2>, g, dim3(256), 0, st, ch, n, chunk, s, fail);
    else hipLaunchKernelGGL(k_xr_region<1>, g, dim3(256), 0, st, ch, n, chunk, s, fail);
    if (finish_u >= 4)
        hipLaunchKernelGGL(k_xr_finish<4>, dim3(grid_for(n, 256 * 4, cus * 8)), dim3(256), 0, st, ch,
                           slot, n, s.hll, regs, nslots, out, fail, err);
    else
        hipLaunchKernelGGL(k_xr_finish<1>, dim3(grid_for(n, 256, cus * 8)), dim3(256), 0, st, ch,
                           slot, n, s.hll, regs, nslots, out, fail, err);
    return hipGetLastError();
}

}  // namespace ske
