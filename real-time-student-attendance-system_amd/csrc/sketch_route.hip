// sketch_route.hip -- routing of unpartitioned swipes to their key owners
// ("if input is not pre-partitioned, use one alltoallv per
// batch"), the device half of distributed.SwipeExchange.
//
// Global key g (an index into the job's key universe) is owned by rank
// key_owner[g] as its local slot key_local[g] -- distributed.KeyMap's table,
// owner = MurmurHash64A(key name, 0) mod world, shared with ingest routing and
// the cross-shard queries; an index past the table goes to rank 0 with slot
// kNoSlot (K1 answers it and reports the slot).  A batch of fixed-width ids
// and global key indices is counting-sorted by owner into send
// buffers laid out owner by owner (the alltoallv input), remembering every
// swipe's position; after K1 on the owners and the reverse alltoallv, the
// answers are gathered back into input order through those positions.
//
//   k_route_count   per block of kRtTile swipes: owner histogram -> hist[o][b]
//   k_route_scan    exclusive scan over (owner, block), owner major -> base[o][b]
//                   (and the per-owner totals)
//   k_route_scatter per block: the same swipes, a rank within (owner, block)
//                   from one LDS atomic per (wave, owner), position =
//                   base[o][b] + rank; ids and local slots scattered there,
//                   pos[i] recorded
//   k_route_return  out[i] = answers[pos[i]]
//
// The capacity form (no host synchronisation) takes one packed route word per
// key, owner << 26 | local slot: k_route_count_cap gathers it once per swipe
// and parks it in pos[i], k_route_scatter_cap streams it back (no gather).
//
// The order inside an (owner, block) segment is whatever the LDS atomics
// give -- immaterial: every swipe keeps its position, and the registers are
// a max.  Streams of bytes: per swipe the id, the slot, the scattered id and
// slot, the position (2w + 12 B), and 1 + 4 + 1 B to return; the capacity
// form's count adds one gather from the route table (the L2's random rate:
// 60 us of its 0.17 ms per 16M swipes at N = 1) and writes the word, its
// scatter reads it back.
#include "sketch_common.h"
#include "sketch_internal.h"

namespace ske {

constexpr uint32_t kRtBlock = 256;
constexpr uint32_t kRtItems = 16;
constexpr uint32_t kRtTile = kRtBlock * kRtItems;  // swipes per block
constexpr uint32_t kRtMaxWorld = 64;

constexpr uint32_t kNoSlot = 0xffffffffu;

struct RouteArgs {
    const uint8_t *ids;    // n x width
    const uint32_t *slot;  // global key indices
    const uint32_t *kown;  // [nkeys] owner rank of each global key
    const uint32_t *kloc;  // [nkeys] local slot of each global key on its owner
    const uint32_t *kroute;  // [nkeys] owner << 26 | local slot (the capacity form), ~0: no owner
    uint8_t *sids;         // n x width, owner major
    uint32_t *sslot;       // local slots, owner major
    uint32_t *pos;         // input swipe -> position in the send buffers
    uint32_t *hist;        // [world][nblocks] counts, then bases
    uint32_t *tot;         // [world] swipes per owner
    uint64_t n;
    uint32_t width, world, nblocks, nkeys;
};

// (a table entry naming no rank of this world is treated as a missing key:
// rank 0, kNoSlot -- never an LDS index past the histogram)
__device__ __forceinline__ bool route_known(const RouteArgs &R, uint32_t g) {
    return g < R.nkeys && R.kown[g] < R.world;
}
__device__ __forceinline__ uint32_t route_owner(const RouteArgs &R, uint32_t g) {
    return route_known(R, g) ? R.kown[g] : 0u;
}

// Ranks within a wave by owner: one LDS atomic per distinct owner of the
// wave's active lanes (a lane-per-atomic form serialises all 64 lanes on one
// counter when one owner takes most swipes -- every swipe at world 1: 230 us
// per 16M-swipe batch for the scatter).  Returns this lane's slot from c[o].
__device__ __forceinline__ uint32_t route_wave_rank(uint32_t o, bool act, uint32_t *c) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t below = (uint64_t(1) << lane) - 1;
    uint64_t rem = __ballot(act);
    uint32_t r = 0;
    while (rem) {  // wave-uniform: one round per distinct owner
        const uint32_t leader = uint32_t(__builtin_ctzll(rem));
        const uint32_t ol = __builtin_amdgcn_readlane(o, leader);
        const bool mine = act && o == ol;
        const uint64_t m = __ballot(mine);
        uint32_t b = 0;
        if (lane == leader) b = atomicAdd(&c[ol], uint32_t(__popcll(m)));
        b = __builtin_amdgcn_readlane(b, leader);
        if (mine) r = b + uint32_t(__popcll(m & below));
        rem &= ~m;
    }
    return r;
}

// the owner (or kRtMaxWorld: a key past the table or naming no rank) and
// local slot of global key g
__device__ __forceinline__ uint32_t route_own_raw(const RouteArgs &R, uint32_t g) {
    return g < R.nkeys ? R.kown[g] : kRtMaxWorld;
}

// Items in batches of kRtBatch per thread: every global load of a batch is
// issued before the first wave rank, so a thread's loads are in flight
// together instead of one dependent chain (slot -> owner -> rank) per item.
constexpr uint32_t kRtBatch = 8;

__global__ void __launch_bounds__(kRtBlock) k_route_count(const RouteArgs R) {
    __shared__ uint32_t c[kRtMaxWorld];
    const uint32_t tid = threadIdx.x;
    if (tid < R.world) c[tid] = 0;
    __syncthreads();
    const uint64_t b0 = uint64_t(blockIdx.x) * kRtTile;
    for (uint32_t j0 = 0; j0 < kRtItems; j0 += kRtBatch) {
        uint32_t g[kRtBatch], o[kRtBatch];
#pragma unroll
        for (uint32_t b = 0; b < kRtBatch; b++) {
            const uint64_t i = b0 + (j0 + b) * kRtBlock + tid;
            g[b] = i < R.n ? R.slot[i] : 0xffffffffu;
        }
#pragma unroll
        for (uint32_t b = 0; b < kRtBatch; b++) o[b] = route_own_raw(R, g[b]);
#pragma unroll
        for (uint32_t b = 0; b < kRtBatch; b++) {
            const bool act = b0 + (j0 + b) * kRtBlock + tid < R.n;
            route_wave_rank(o[b] < R.world ? o[b] : 0u, act, c);
        }
    }
    __syncthreads();
    if (tid < R.world) R.hist[size_t(tid) * R.nblocks + blockIdx.x] = c[tid];
}

// one block: exclusive scan of hist (owner major), totals per owner
__global__ void __launch_bounds__(1024) k_route_scan(const RouteArgs R) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t total = uint64_t(R.world) * R.nblocks;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (uint64_t c0 = 0; c0 < total; c0 += 1024) {
        const uint64_t i = c0 + tid;
        const uint32_t v = i < total ? R.hist[i] : 0;
        uint32_t incl = v;
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        uint32_t pre = carry;
        for (uint32_t w = 0; w < wave; w++) pre += wsum[w];
        if (i < total) R.hist[i] = pre + incl - v;
        __syncthreads();
        if (tid == 1023) carry = pre + incl;
        __syncthreads();
    }
    // per-owner totals: the base of the next owner minus this one's
    if (tid < R.world) {
        const uint32_t b = R.hist[size_t(tid) * R.nblocks];
        const uint32_t e = tid + 1 < R.world ? R.hist[size_t(tid + 1) * R.nblocks] : uint32_t(R.n);
        R.tot[tid] = e - b;
    }
}

__global__ void __launch_bounds__(kRtBlock) k_route_scatter(const RouteArgs R) {
    __shared__ uint32_t c[kRtMaxWorld], base[kRtMaxWorld];
    const uint32_t tid = threadIdx.x;
    if (tid < R.world) {
        c[tid] = 0;
        base[tid] = R.hist[size_t(tid) * R.nblocks + blockIdx.x];
    }
    __syncthreads();
    const uint64_t b0 = uint64_t(blockIdx.x) * kRtTile;
#pragma unroll 4
    for (uint32_t j = 0; j < kRtItems; j++) {
        const uint64_t i = b0 + j * kRtBlock + tid;
        const bool act = i < R.n;
        const uint32_t g = act ? R.slot[i] : 0u;
        const uint32_t o = act ? route_owner(R, g) : 0u;
        const uint32_t p = base[o] + route_wave_rank(o, act, c);
        if (!act) continue;
        R.pos[i] = p;
        R.sslot[p] = route_known(R, g) ? R.kloc[g] : kNoSlot;
        const uint8_t *src = R.ids + i * R.width;
        uint8_t *dst = R.sids + uint64_t(p) * R.width;
        if (R.width == 8) {
            *reinterpret_cast<uint64_t *>(dst) = *reinterpret_cast<const uint64_t *>(src);
        } else {
            for (uint32_t k = 0; k < R.width; k++) dst[k] = src[k];
        }
    }
}

// Capacity-padded layout (the host-free exchange): owner o's swipes go to
// rows [o * cap, o * cap + tot[o]) of the send buffers, so every rank sends
// and receives exactly `cap` rows per peer (an all_to_all of equal splits,
// whose sizes the host knows without reading the device).  A swipe ranked
// past cap in its owner is not sent (pos = its row modulo cap: a row of the
// same owner, answered for another swipe) -- tot[o] > cap tells the host,
// which then re-runs the batch with exact splits (PFADD is idempotent and
// the answers are rewritten).
// The capacity form's count: one gather per swipe of its key's packed route
// word, kept in pos[i] for the scatter (which then gathers nothing: every
// access of k_route_scatter_cap is a coalesced stream).
// ~0 is "no owner" at every world size (at world 64 its owner field would
// read 63): such keys go to rank 0 with kNoSlot, as the torch path's
// owner_local; KeyMap.route_words keeps local slots below 2^26 - 1, so no
// real key packs to ~0
__device__ __forceinline__ bool route_word_owned(const RouteArgs &R, uint32_t kr) {
    return kr != 0xffffffffu && (kr >> 26) < R.world;
}
__device__ __forceinline__ uint32_t route_word_owner(const RouteArgs &R, uint32_t kr) {
    return route_word_owned(R, kr) ? kr >> 26 : 0u;
}
__device__ __forceinline__ uint32_t route_word_slot(const RouteArgs &R, uint32_t kr) {
    return route_word_owned(R, kr) ? kr & 0x3ffffffu : kNoSlot;
}

__global__ void __launch_bounds__(kRtBlock) k_route_count_cap(const RouteArgs R) {
    __shared__ uint32_t c[kRtMaxWorld];
    const uint32_t tid = threadIdx.x;
    if (tid < R.world) c[tid] = 0;
    __syncthreads();
    const uint64_t b0 = uint64_t(blockIdx.x) * kRtTile;
    for (uint32_t j0 = 0; j0 < kRtItems; j0 += kRtBatch) {
        uint32_t g[kRtBatch], kr[kRtBatch];
#pragma unroll
        for (uint32_t b = 0; b < kRtBatch; b++) {
            const uint64_t i = b0 + (j0 + b) * kRtBlock + tid;
            g[b] = i < R.n ? R.slot[i] : 0xffffffffu;
        }
#pragma unroll
        for (uint32_t b = 0; b < kRtBatch; b++) kr[b] = g[b] < R.nkeys ? R.kroute[g[b]] : 0xffffffffu;
#pragma unroll
        for (uint32_t b = 0; b < kRtBatch; b++) {
            const uint64_t i = b0 + (j0 + b) * kRtBlock + tid;
            const bool act = i < R.n;
            if (act) R.pos[i] = kr[b];
            route_wave_rank(route_word_owner(R, kr[b]), act, c);
        }
    }
    __syncthreads();
    if (tid < R.world) R.hist[size_t(tid) * R.nblocks + blockIdx.x] = c[tid];
}

__global__ void __launch_bounds__(kRtBlock) k_route_scatter_cap(const RouteArgs R, uint32_t cap) {
    __shared__ uint32_t c[kRtMaxWorld], base[kRtMaxWorld];
    const uint32_t tid = threadIdx.x;
    if (tid < R.world) {
        c[tid] = 0;
        // this block's first rank within its owner (the scan is owner major)
        base[tid] = R.hist[size_t(tid) * R.nblocks + blockIdx.x] - R.hist[size_t(tid) * R.nblocks];
    }
    __syncthreads();
    const uint64_t b0 = uint64_t(blockIdx.x) * kRtTile;
    const bool w8 = R.width == 8;
    for (uint32_t j0 = 0; j0 < kRtItems; j0 += kRtBatch) {
        uint32_t kr[kRtBatch];
        uint64_t id[kRtBatch];
#pragma unroll
        for (uint32_t b = 0; b < kRtBatch; b++) {
            const uint64_t i = b0 + (j0 + b) * kRtBlock + tid;
            const bool act = i < R.n;
            kr[b] = act ? R.pos[i] : 0xffffffffu;  // the count's route word
            id[b] = act && w8 ? *reinterpret_cast<const uint64_t *>(R.ids + i * 8) : 0;
        }
#pragma unroll
        for (uint32_t b = 0; b < kRtBatch; b++) {
            const uint64_t i = b0 + (j0 + b) * kRtBlock + tid;
            const bool act = i < R.n;
            const uint32_t ow = route_word_owner(R, kr[b]);
            const uint32_t r = base[ow] + route_wave_rank(ow, act, c);
            if (!act) continue;
            const uint32_t p = ow * cap + (r < cap ? r : r % cap);
            R.pos[i] = p;
            if (r >= cap) continue;  // overflow: tot[o] > cap reports it
            R.sslot[p] = route_word_slot(R, kr[b]);
            if (w8) {
                *reinterpret_cast<uint64_t *>(R.sids + uint64_t(p) * 8) = id[b];
            } else {
                const uint8_t *src = R.ids + i * R.width;
                uint8_t *dst = R.sids + uint64_t(p) * R.width;
                for (uint32_t k = 0; k < R.width; k++) dst[k] = src[k];
            }
        }
    }
}

// rows [tot[o], cap) of owner o (blockIdx.y): id bytes zero, slot sink[o]
// (a slot the owner keeps for nothing else, so the padding's PFADDs change no
// key); only the padding rows are visited
__global__ void __launch_bounds__(256) k_route_pad(const RouteArgs R, uint32_t cap, const uint32_t *sink) {
    const uint32_t o = blockIdx.y, t = R.tot[o], s = sink[o];
    for (uint32_t r = t + blockIdx.x * 256 + threadIdx.x; r < cap; r += gridDim.x * 256) {
        const uint64_t j = uint64_t(o) * cap + r;
        R.sslot[j] = s;
        uint8_t *dst = R.sids + j * R.width;
        if (R.width == 8)
            *reinterpret_cast<uint64_t *>(dst) = 0;
        else
            for (uint32_t k = 0; k < R.width; k++) dst[k] = 0;
    }
}

hipError_t launch_route_cap(const uint8_t *ids, uint32_t width, const uint32_t *slot, uint64_t n, uint32_t world,
                            const uint32_t *kroute, uint32_t nkeys, uint32_t cap, const uint32_t *sink, uint8_t *sids,
                            uint32_t *sslot, uint32_t *pos, uint32_t *hist, uint32_t *tot, int cus, hipStream_t st) {
    if (world == 0 || world > kRtMaxWorld || width == 0 || n >= (uint64_t(1) << 32) || cap == 0 ||
        uint64_t(cap) * world >= (uint64_t(1) << 32))
        return hipErrorInvalidValue;
    RouteArgs R{ids, slot, nullptr, nullptr, kroute, sids, sslot, pos, hist, tot, n, width, world,
                uint32_t((n + kRtTile - 1) / kRtTile), nkeys};
    if (n == 0) {
        hipError_t e = hipMemsetAsync(tot, 0, size_t(world) * 4, st);
        if (e != hipSuccess) return e;
    } else {
        hipLaunchKernelGGL(k_route_count_cap, dim3(R.nblocks), dim3(kRtBlock), 0, st, R);
        hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(1024), 0, st, R);
        hipLaunchKernelGGL(k_route_scatter_cap, dim3(R.nblocks), dim3(kRtBlock), 0, st, R, cap);
    }
    const uint64_t g = (uint64_t(cap) + 255) / 256;
    const unsigned gx = unsigned(g < uint64_t(cus) * 4 / world + 1 ? g : uint64_t(cus) * 4 / world + 1);
    hipLaunchKernelGGL(k_route_pad, dim3(gx, world), dim3(256), 0, st, R, cap, sink);
    return hipGetLastError();
}

// The exchange at world 1 is the identity: K1 reads the batch in place and
// answers in input order, so only the keys are mapped -- out[i] = the local
// slot of gkey[i] (route word & 2^26 - 1), or kNoSlot for a key past the
// table or owned by no rank of this world (K1 then reports it as SKE_ERANGE,
// as the routed forms do).  8 B per swipe + the table gather (a random L2
// read per swipe: 0.52 ms per 2^27 swipes); kroute == nullptr is the
// identity table of a one-rank key map (KeyMap: local slot = the key's index
// in the universe), no gather: 8 B per swipe, streamed.
__device__ __forceinline__ uint32_t route_slot1(uint32_t g, const uint32_t *kroute, uint32_t nkeys, uint32_t world) {
    if (!kroute) return g < nkeys ? g : kNoSlot;
    const uint32_t kr = g < nkeys ? kroute[g] : 0xffffffffu;
    return kr != 0xffffffffu && (kr >> 26) < world ? kr & 0x3ffffffu : kNoSlot;
}
__global__ void __launch_bounds__(256) k_route_slots1(const uint32_t *gkey, uint64_t n, const uint32_t *kroute,
                                                      uint32_t nkeys, uint32_t world, uint32_t *out) {
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256)
        out[i] = route_slot1(gkey[i], kroute, nkeys, world);
}
__global__ void __launch_bounds__(256) k_route_slots(const uint32_t *gkey, uint64_t n, const uint32_t *kroute,
                                                     uint32_t nkeys, uint32_t world, uint32_t *out) {
    const uint64_t n4 = n / 4;
    for (uint64_t q = uint64_t(blockIdx.x) * 256 + threadIdx.x; q < n4; q += uint64_t(gridDim.x) * 256) {
        const uint4 g = reinterpret_cast<const uint4 *>(gkey)[q];
        reinterpret_cast<uint4 *>(out)[q] =
            make_uint4(route_slot1(g.x, kroute, nkeys, world), route_slot1(g.y, kroute, nkeys, world),
                       route_slot1(g.z, kroute, nkeys, world), route_slot1(g.w, kroute, nkeys, world));
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        const uint64_t i = n4 * 4 + threadIdx.x;
        out[i] = route_slot1(gkey[i], kroute, nkeys, world);
    }
}

hipError_t launch_route_slots(const uint32_t *gkey, uint64_t n, const uint32_t *kroute, uint32_t nkeys,
                              uint32_t world, uint32_t *out, int cus, hipStream_t st) {
    if (n == 0) return hipSuccess;
    // four keys per thread when both arrays are 16-B aligned, else one
    const bool v4 = !(reinterpret_cast<uintptr_t>(gkey) & 15) && !(reinterpret_cast<uintptr_t>(out) & 15);
    const uint64_t g = ((v4 ? n / 4 : n) + 255) / 256;
    const unsigned grid = unsigned(g < 1 ? 1 : g < uint64_t(cus) * 8 ? g : uint64_t(cus) * 8);
    if (v4)
        hipLaunchKernelGGL(k_route_slots, dim3(grid), dim3(256), 0, st, gkey, n, kroute, nkeys, world, out);
    else
        hipLaunchKernelGGL(k_route_slots1, dim3(grid), dim3(256), 0, st, gkey, n, kroute, nkeys, world, out);
    return hipGetLastError();
}

// four answers per thread: one 16-B load of positions, one 4-B store (pos
// and out 16-B / 4-B aligned, checked by the host; else one per thread)
__global__ void __launch_bounds__(256) k_route_return(const uint8_t *ans, const uint32_t *pos, uint64_t n,
                                                      uint8_t *out) {
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256)
        out[i] = ans[pos[i]];
}
__global__ void __launch_bounds__(256) k_route_return4(const uint8_t *ans, const uint32_t *pos, uint64_t n,
                                                       uint8_t *out) {
    const uint64_t n4 = n / 4;
    for (uint64_t q = uint64_t(blockIdx.x) * 256 + threadIdx.x; q < n4; q += uint64_t(gridDim.x) * 256) {
        const uint4 p = reinterpret_cast<const uint4 *>(pos)[q];
        const uint32_t v = uint32_t(ans[p.x]) | uint32_t(ans[p.y]) << 8 | uint32_t(ans[p.z]) << 16 |
                           uint32_t(ans[p.w]) << 24;
        reinterpret_cast<uint32_t *>(out)[q] = v;
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) out[n4 * 4 + threadIdx.x] = ans[pos[n4 * 4 + threadIdx.x]];
}

hipError_t launch_route(const uint8_t *ids, uint32_t width, const uint32_t *slot, uint64_t n, uint32_t world,
                        const uint32_t *kown, const uint32_t *kloc, uint32_t nkeys, uint8_t *sids,
                        uint32_t *sslot, uint32_t *pos, uint32_t *hist, uint32_t *tot, hipStream_t st) {
    if (world == 0 || world > kRtMaxWorld || width == 0 || n >= (uint64_t(1) << 32)) return hipErrorInvalidValue;
    RouteArgs R{ids, slot, kown, kloc, nullptr, sids, sslot, pos, hist, tot, n, width, world,
                uint32_t((n + kRtTile - 1) / kRtTile), nkeys};
    if (n == 0) return hipMemsetAsync(tot, 0, size_t(world) * 4, st);
    hipLaunchKernelGGL(k_route_count, dim3(R.nblocks), dim3(kRtBlock), 0, st, R);
    hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(1024), 0, st, R);
    hipLaunchKernelGGL(k_route_scatter, dim3(R.nblocks), dim3(kRtBlock), 0, st, R);
    return hipGetLastError();
}

// out[j] bit b = (in[8j + b] != 0): answers packed LSB first (numpy's
// packbits(bitorder="little")), 1 bit per swipe on the device-to-host leg
__global__ void __launch_bounds__(256) k_pack_bits(const uint8_t *in, uint64_t n, uint8_t *out) {
    const uint64_t nb = (n + 7) / 8;
    for (uint64_t j = uint64_t(blockIdx.x) * 256 + threadIdx.x; j < nb; j += uint64_t(gridDim.x) * 256) {
        uint32_t v = 0;
        if (8 * j + 8 <= n) {
            const uint2 w = *reinterpret_cast<const uint2 *>(in + 8 * j);
#pragma unroll
            for (int b = 0; b < 4; b++) v |= uint32_t(((w.x >> (8 * b)) & 0xffu) != 0) << b;
#pragma unroll
            for (int b = 0; b < 4; b++) v |= uint32_t(((w.y >> (8 * b)) & 0xffu) != 0) << (4 + b);
        } else {
            for (uint64_t b = 0; 8 * j + b < n; b++) v |= uint32_t(in[8 * j + b] != 0) << b;
        }
        out[j] = uint8_t(v);
    }
}

hipError_t launch_pack_bits(const uint8_t *in, uint64_t n, uint8_t *out, int cus, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint64_t g = ((n + 7) / 8 + 255) / 256;
    const unsigned grid = unsigned(g < uint64_t(cus) * 8 ? g : uint64_t(cus) * 8);
    hipLaunchKernelGGL(k_pack_bits, dim3(grid), dim3(256), 0, st, in, n, out);
    return hipGetLastError();
}

uint64_t route_hist_words(uint64_t n, uint32_t world) { return uint64_t(world) * ((n + kRtTile - 1) / kRtTile); }

hipError_t launch_route_return(const uint8_t *ans, const uint32_t *pos, uint64_t n, uint8_t *out, int cus,
                               hipStream_t st) {
    if (n == 0) return hipSuccess;
    const bool v4 = (reinterpret_cast<uintptr_t>(pos) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 3) == 0;
    const uint64_t g = ((v4 ? n / 4 : n) + 255) / 256;
    const unsigned grid = unsigned(g < 1 ? 1 : g < uint64_t(cus) * 8 ? g : uint64_t(cus) * 8);
    if (v4)
        hipLaunchKernelGGL(k_route_return4, dim3(grid), dim3(256), 0, st, ans, pos, n, out);
    else
        hipLaunchKernelGGL(k_route_return, dim3(grid), dim3(256), 0, st, ans, pos, n, out);
    return hipGetLastError();
}

}  // namespace ske
