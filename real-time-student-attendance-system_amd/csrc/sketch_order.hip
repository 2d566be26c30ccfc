// sketch_order.hip -- order-exact paths: replies that depend on item order.
//
// Final Bloom bits and HLL registers are order independent (OR / max), but
// Redis's per-item replies are not:
//   - PFADD replies 1 when an element raised a register *given every element
//     before it* (pfaddCommand; attendance_processor.py:129 issues one call
//     per event, a pipeline many);
//   - BF.ADD / BF.MADD reply 1 only when the item was absent from the chain as
//     left by every earlier add, and SBChain_Add grows the chain when the
//     current link is full (data_generator.py:57-63 preload).
// Both are rebuilt here from order-free primitives (radix sort + segmented
// scan for PFADD; "first setter" per bit + prefix count for BF.MADD).
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_scan_by_key.hpp>

#include "sketch_common.h"
#include "sketch_internal.h"

namespace ske {

struct Scratch {
    void *p[kScratchSlots] = {};
    size_t cap[kScratchSlots] = {};
    bool recording = false;              // a stream capture is recording
    bool pinned[kScratchSlots] = {};     // handed out while recording
};

void scratch_set_recording(Scratch *s, bool on) { s->recording = on; }
void scratch_unpin(Scratch *s) {
    for (int i = 0; i < kScratchSlots; i++) s->pinned[i] = false;
}

// A slot grows by hipFree + hipMalloc.  A slot handed out while a graph was
// being recorded is pinned until every graph is freed: its growth is refused
// with hipErrorStreamCaptureUnsupported (the allocation would be prohibited
// inside a capture, and the hipFree would release memory that recorded nodes
// still point to).
void *scratch_get(Scratch *s, int slot, size_t bytes, hipError_t *err) {
    if (bytes == 0) bytes = 16;
    if (s->recording) s->pinned[slot] = true;
    if (s->cap[slot] < bytes && s->pinned[slot]) {
        *err = hipErrorStreamCaptureUnsupported;
        return nullptr;
    }
    if (s->cap[slot] < bytes) {
        if (s->p[slot]) (void)hipFree(s->p[slot]);
        s->p[slot] = nullptr;
        s->cap[slot] = 0;
        size_t want = bytes + bytes / 4 + 256;
        hipError_t e = hipMalloc(&s->p[slot], want);
        if (e != hipSuccess) {
            *err = e;
            return nullptr;
        }
        s->cap[slot] = want;
    }
    return s->p[slot];
}

void scratch_free_all(Scratch *s) {
    for (int i = 0; i < kScratchSlots; i++)
        if (s->p[i]) (void)hipFree(s->p[i]);
}

Scratch *scratch_new() { return new Scratch(); }
void scratch_delete(Scratch *s) {
    scratch_free_all(s);
    delete s;
}

static inline unsigned grid_for(uint64_t n, unsigned block, unsigned cap) {
    uint64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    return unsigned(g < cap ? g : cap);
}

#define SKE_GRID_LOOP(i, n)                                                                       \
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < (n);                   \
         i += uint64_t(gridDim.x) * blockDim.x)

// ---------------------------------------------------------------------------
// PFADD with exact per-element replies
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
    k_hll_prep(const uint32_t *__restrict__ slot, const uint8_t *__restrict__ bytes,
               const uint32_t *__restrict__ offs, uint64_t n, uint32_t nslots,
               uint64_t *__restrict__ keys, uint32_t *__restrict__ vals,
               uint8_t *__restrict__ rank_out, unsigned int *__restrict__ err) {
    SKE_GRID_LOOP(i, n) {
        uint32_t s = slot[i];
        const Item it = load_item(bytes, offs[i], offs[i + 1]);
        uint32_t idx, rank;
        hll_patlen(murmur_item(it, kHllSeed), idx, rank);
        if (s >= nslots) {  // reported as SKE_ERANGE; rank 0 never changes a register
            atomicOr(err, 1u);
            s = 0;
            idx = 0;
            rank = 0;
        }
        keys[i] = (uint64_t(s) << kHllP) | idx;
        vals[i] = uint32_t(i);
        rank_out[i] = uint8_t(rank);
    }
}

__global__ void __launch_bounds__(256)
    k_gather_u8(const uint32_t *__restrict__ idx, const uint8_t *__restrict__ src, uint64_t n,
                uint8_t *__restrict__ dst) {
    SKE_GRID_LOOP(i, n) dst[i] = src[idx[i]];
}

// changed = rank > max(register before the batch, ranks of earlier elements of
// the same register); reads registers only (updates happen in k_hll_apply).
__global__ void __launch_bounds__(256)
    k_hll_changed(const uint64_t *__restrict__ keys_s, const uint32_t *__restrict__ vals_s,
                  const uint8_t *__restrict__ rank_s, const uint8_t *__restrict__ prefmax,
                  const uint8_t *__restrict__ regs, uint64_t n, uint8_t *__restrict__ changed) {
    SKE_GRID_LOOP(j, n) {
        const uint8_t init = regs[keys_s[j]];
        const uint8_t before = prefmax[j] > init ? prefmax[j] : init;
        changed[vals_s[j]] = rank_s[j] > before;
    }
}

__global__ void __launch_bounds__(256)
    k_hll_apply(const uint64_t *__restrict__ keys_s, const uint8_t *__restrict__ rank_s,
                uint64_t n, uint8_t *__restrict__ regs) {
    SKE_GRID_LOOP(j, n) {
        // only the segment's last element needs to write: it carries the max
        // of the segment in the inclusive sense once combined with prefmax,
        // but a CAS max per element is simpler and exact.
        const uint64_t k = keys_s[j];
        uint8_t *reg = regs + k;
        uintptr_t a = reinterpret_cast<uintptr_t>(reg);
        uint32_t *w = reinterpret_cast<uint32_t *>(a & ~uintptr_t(3));
        const uint32_t sh = uint32_t(a & 3) * 8, rank = rank_s[j];
        uint32_t old = *w;
        while (((old >> sh) & 0xffu) < rank) {
            const uint32_t prev = atomicCAS(w, old, (old & ~(0xffu << sh)) | (rank << sh));
            if (prev == old) break;
            old = prev;
        }
    }
}

struct MaxU8 {
    __device__ __host__ uint8_t operator()(const uint8_t &a, const uint8_t &b) const {
        return a > b ? a : b;
    }
};

hipError_t pfadd_exact(Scratch *s, const uint32_t *slot, const uint8_t *bytes,
                       const uint32_t *offs, uint64_t n, uint8_t *regs, uint32_t nslots,
                       uint8_t *changed_dev, unsigned int *err_dev, int cus, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipError_t e = hipSuccess;
    uint64_t *keys = (uint64_t *)scratch_get(s, 0, n * 8, &e);
    uint64_t *keys_s = (uint64_t *)scratch_get(s, 1, n * 8, &e);
    uint32_t *vals = (uint32_t *)scratch_get(s, 2, n * 4, &e);
    uint32_t *vals_s = (uint32_t *)scratch_get(s, 3, n * 4, &e);
    uint8_t *rank = (uint8_t *)scratch_get(s, 4, n, &e);
    uint8_t *rank_s = (uint8_t *)scratch_get(s, 5, n, &e);
    uint8_t *pref = (uint8_t *)scratch_get(s, 6, n, &e);
    if (e != hipSuccess) return e;
    const unsigned grid = grid_for(n, 256, cus * 16);
    hipLaunchKernelGGL(k_hll_prep, dim3(grid), dim3(256), 0, st, slot, bytes, offs, n, nslots,
                       keys, vals, rank, err_dev);
    unsigned end_bit = kHllP;
    while (end_bit < 64 && (uint64_t(nslots) << kHllP) > (uint64_t(1) << end_bit)) end_bit++;
    size_t tb = 0;
    e = rocprim::radix_sort_pairs(nullptr, tb, keys, keys_s, vals, vals_s, n, 0u, end_bit, st);
    if (e != hipSuccess) return e;
    void *tmp = scratch_get(s, 7, tb, &e);
    if (e != hipSuccess) return e;
    e = rocprim::radix_sort_pairs(tmp, tb, keys, keys_s, vals, vals_s, n, 0u, end_bit, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_gather_u8, dim3(grid), dim3(256), 0, st, vals_s, rank, n, rank_s);
    size_t tb2 = 0;
    e = rocprim::exclusive_scan_by_key(nullptr, tb2, keys_s, rank_s, pref, uint8_t(0), size_t(n),
                                       MaxU8(), rocprim::equal_to<uint64_t>(), st);
    if (e != hipSuccess) return e;
    tmp = scratch_get(s, 8, tb2, &e);
    if (e != hipSuccess) return e;
    e = rocprim::exclusive_scan_by_key(tmp, tb2, keys_s, rank_s, pref, uint8_t(0), size_t(n),
                                       MaxU8(), rocprim::equal_to<uint64_t>(), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_hll_changed, dim3(grid), dim3(256), 0, st, keys_s, vals_s, rank_s, pref,
                       regs, n, changed_dev);
    hipLaunchKernelGGL(k_hll_apply, dim3(grid), dim3(256), 0, st, keys_s, rank_s, n, regs);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// BF.MADD building blocks
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
    k_bf_hash(const uint8_t *__restrict__ bytes, const uint32_t *__restrict__ offs, uint64_t n,
              uint64_t *__restrict__ ha, uint64_t *__restrict__ hb) {
    SKE_GRID_LOOP(i, n) {
        const Item it = load_item(bytes, offs[i], offs[i + 1]);
        const uint64_t a = murmur_item(it, kBloomSeed);
        ha[i] = a;
        hb[i] = murmur_item(it, a);
    }
}

__device__ __forceinline__ bool link_has(const LinkDev &L, uint64_t a, uint64_t b) {
    ProbeCursor c;
    c.init(a, b, L.div);
    for (uint32_t j = 0; j < L.k; j++) {
        const uint64_t x = c.x;
        if (!((L.bf[x >> 3] >> (x & 7)) & 1)) return false;
        c.step(L.div);
    }
    return true;
}

__global__ void __launch_bounds__(256)
    k_bf_settle_present(const ChainDev ch, uint64_t n, const uint64_t *__restrict__ ha,
                        const uint64_t *__restrict__ hb, uint8_t *__restrict__ state,
                        int8_t *__restrict__ res) {
    SKE_GRID_LOOP(i, n) {
        if (state[i]) continue;
        for (int l = ch.nlinks - 1; l >= 0; --l) {
            if (link_has(ch.link[l], ha[i], hb[i])) {
                state[i] = 1;
                res[i] = 0;
                break;
            }
        }
    }
}

// first[x] = min index of the candidates probing an initially-unset bit x
__global__ void __launch_bounds__(256)
    k_bf_first_setter(const LinkDev L, uint64_t n, const uint64_t *__restrict__ ha,
                      const uint64_t *__restrict__ hb, const uint8_t *__restrict__ state,
                      uint32_t *__restrict__ first) {
    SKE_GRID_LOOP(i, n) {
        if (state[i]) continue;
        ProbeCursor c;
        c.init(ha[i], hb[i], L.div);
        for (uint32_t j = 0; j < L.k; j++) {
            const uint64_t x = c.x;
            if (!((L.bf[x >> 3] >> (x & 7)) & 1)) atomicMin(&first[x], uint32_t(i));
            c.step(L.div);
        }
    }
}

// candidate i is absent from the link as left by the candidates before it iff
// one of its initially-unset bits has no earlier setter (first[x] == i).
__global__ void __launch_bounds__(256)
    k_bf_absent(const LinkDev L, uint64_t n, const uint64_t *__restrict__ ha,
                const uint64_t *__restrict__ hb, const uint8_t *__restrict__ state,
                const uint32_t *__restrict__ first, uint32_t *__restrict__ absent) {
    SKE_GRID_LOOP(i, n) {
        uint32_t ab = 0;
        if (!state[i]) {
            ProbeCursor c;
            c.init(ha[i], hb[i], L.div);
            for (uint32_t j = 0; j < L.k; j++) {
                const uint64_t x = c.x;
                if (!((L.bf[x >> 3] >> (x & 7)) & 1) && first[x] >= uint32_t(i)) {
                    ab = 1;
                    break;
                }
                c.step(L.div);
            }
        }
        absent[i] = ab;
    }
}

// resolve candidates that come before the (cap+1)-th absent one: the number
// of absent candidates strictly before i is pos[i] - absent[i].
__global__ void __launch_bounds__(256)
    k_bf_resolve(const LinkDev L, uint64_t n, const uint64_t *__restrict__ ha,
                 const uint64_t *__restrict__ hb, uint8_t *__restrict__ state,
                 const uint32_t *__restrict__ absent, const uint32_t *__restrict__ pos,
                 uint32_t cap, int8_t *__restrict__ res, uint8_t *__restrict__ bf) {
    SKE_GRID_LOOP(i, n) {
        if (state[i]) continue;
        if (pos[i] - absent[i] >= cap) continue;
        state[i] = 1;
        res[i] = absent[i] ? 1 : 0;
        if (absent[i]) {
            ProbeCursor c;
            c.init(ha[i], hb[i], L.div);
            for (uint32_t j = 0; j < L.k; j++) {
                const uint64_t x = c.x;
                atomicOr(reinterpret_cast<unsigned int *>(bf + ((x >> 3) & ~uint64_t(3))),
                         1u << (x & 31));
                c.step(L.div);
            }
        }
    }
}

__global__ void __launch_bounds__(256)
    k_bf_fill_rest(uint64_t n, uint8_t *__restrict__ state, int8_t *__restrict__ res, int8_t code) {
    SKE_GRID_LOOP(i, n) {
        if (!state[i]) {
            state[i] = 1;
            res[i] = code;
        }
    }
}

__global__ void __launch_bounds__(256)
    k_bf_count_cands(uint64_t n, const uint8_t *__restrict__ state,
                     unsigned long long *__restrict__ counter) {
    unsigned long long c = 0;
    SKE_GRID_LOOP(i, n) c += state[i] == 0;
    if (c) atomicAdd(counter, c);
}

hipError_t launch_bf_count_cands(uint64_t n, const uint8_t *state, unsigned long long *counter,
                                 int cus, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_bf_count_cands, dim3(grid_for(n, 256, cus * 4)), dim3(256), 0, st, n,
                       state, counter);
    return hipGetLastError();
}

hipError_t launch_bf_hash(const uint8_t *bytes, const uint32_t *offs, uint64_t n, uint64_t *ha,
                          uint64_t *hb, int cus, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_bf_hash, dim3(grid_for(n, 256, cus * 16)), dim3(256), 0, st, bytes, offs,
                       n, ha, hb);
    return hipGetLastError();
}
hipError_t launch_bf_settle_present(const ChainDev &ch, uint64_t n, const uint64_t *ha,
                                    const uint64_t *hb, uint8_t *state, int8_t *res, int cus,
                                    hipStream_t st) {
    if (!n || ch.nlinks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_bf_settle_present, dim3(grid_for(n, 256, cus * 16)), dim3(256), 0, st, ch,
                       n, ha, hb, state, res);
    return hipGetLastError();
}
hipError_t launch_bf_first_setter(const LinkDev &L, uint64_t n, const uint64_t *ha,
                                  const uint64_t *hb, const uint8_t *state, uint32_t *first,
                                  int cus, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_bf_first_setter, dim3(grid_for(n, 256, cus * 16)), dim3(256), 0, st, L, n,
                       ha, hb, state, first);
    return hipGetLastError();
}
hipError_t launch_bf_absent(const LinkDev &L, uint64_t n, const uint64_t *ha, const uint64_t *hb,
                            const uint8_t *state, const uint32_t *first, uint32_t *absent,
                            int cus, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_bf_absent, dim3(grid_for(n, 256, cus * 16)), dim3(256), 0, st, L, n, ha,
                       hb, state, first, absent);
    return hipGetLastError();
}
hipError_t scan_inclusive_u32(Scratch *s, const uint32_t *in, uint32_t *out, uint64_t n,
                              hipStream_t st) {
    if (!n) return hipSuccess;
    size_t tb = 0;
    hipError_t e = rocprim::inclusive_scan(nullptr, tb, in, out, size_t(n), rocprim::plus<uint32_t>(), st);
    if (e != hipSuccess) return e;
    void *tmp = scratch_get(s, 9, tb, &e);
    if (e != hipSuccess) return e;
    return rocprim::inclusive_scan(tmp, tb, in, out, size_t(n), rocprim::plus<uint32_t>(), st);
}
hipError_t launch_bf_resolve(const LinkDev &L, uint64_t n, const uint64_t *ha, const uint64_t *hb,
                             uint8_t *state, const uint32_t *absent, const uint32_t *pos,
                             uint32_t cap, int8_t *res, uint8_t *bf_mut, int cus,
                             hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_bf_resolve, dim3(grid_for(n, 256, cus * 16)), dim3(256), 0, st, L, n, ha,
                       hb, state, absent, pos, cap, res, bf_mut);
    return hipGetLastError();
}
hipError_t launch_bf_fill_rest(uint64_t n, uint8_t *state, int8_t *res, int8_t code, int cus,
                               hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_bf_fill_rest, dim3(grid_for(n, 256, cus * 16)), dim3(256), 0, st, n, state,
                       res, code);
    return hipGetLastError();
}

}  // namespace ske
