// sketch_common.h -- shared host/device arithmetic for libsketch (gfx950).
//
// Everything here is the bit-exact arithmetic of the upstream routines the
// reference reaches through redis-py (attendance_processor.py:109-113 BF.EXISTS,
// :127-129 PFADD; data_generator.py:57-63 BF.ADD), re-expressed for 64-wide
// wavefronts: items are loaded as aligned little-endian 64-bit words, the
// Bloom probe sequence (a + i*b) mod 2^64 mod bits is stepped incrementally
// with an exact carry correction instead of k 64-bit divisions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SKE_HD __host__ __device__ __forceinline__

namespace ske {

constexpr uint64_t kMurmurM = 0xc6a4a7935bd1e995ULL;
constexpr uint64_t kBloomSeed = 0xc6a4a7935bd1e995ULL;  // bloom_calc_hash64() first seed
constexpr uint64_t kHllSeed = 0xadc83b19ULL;            // hllPatLen() seed
constexpr int kHllP = 14;
constexpr int kHllQ = 64 - kHllP;
constexpr uint32_t kHllRegs = 1u << kHllP;
constexpr int kMaxLinks = 48;

// ---------------------------------------------------------------------------
// MurmurHash64A (Redis src/hyperloglog.c MurmurHash64A, RedisBloom
// deps/murmur2/MurmurHash2.c MurmurHash64A_Bloom -- identical arithmetic).
// ---------------------------------------------------------------------------
SKE_HD uint64_t mm_block(uint64_t h, uint64_t k) {
    k *= kMurmurM;
    k ^= k >> 47;
    k *= kMurmurM;
    h ^= k;
    h *= kMurmurM;
    return h;
}
SKE_HD uint64_t mm_final(uint64_t h) {
    h ^= h >> 47;
    h *= kMurmurM;
    h ^= h >> 47;
    return h;
}

// Little-endian value of nb (1..8) bytes at p, zero padded, from aligned
// 64-bit words only (never touches a word that holds no byte of the item).
// (pointer arithmetic on p itself, never an integer round trip, so the load
// stays a global_load and does not become a flat_load.)
__device__ __forceinline__ uint64_t load_le(const uint8_t *p, uint32_t nb) {
    const uint32_t off = uint32_t(reinterpret_cast<uintptr_t>(p) & 7);
    const uint64_t *w = reinterpret_cast<const uint64_t *>(p - off);
    uint64_t v = w[0] >> (off * 8);
    if (off + nb > 8) v |= w[1] << (64 - off * 8);
    if (nb < 8) v &= (uint64_t(1) << (nb * 8)) - 1;
    return v;
}

// An item held as its first two 8-byte blocks (enough for every student id
// of the configs: 5..8 decimal digits); longer items re-read blocks 2.. .
struct Item {
    const uint8_t *p;
    uint32_t len;
    uint64_t w0, w1;
};

__device__ __forceinline__ Item load_item(const uint8_t *bytes, uint32_t b, uint32_t e) {
    Item it;
    it.p = bytes + b;
    it.len = e - b;
    it.w0 = it.len ? load_le(it.p, it.len < 8 ? it.len : 8) : 0;
    it.w1 = it.len > 8 ? load_le(it.p + 8, it.len < 16 ? it.len - 8 : 8) : 0;
    return it;
}

__device__ __forceinline__ uint64_t murmur_item(const Item &it, uint64_t seed) {
    uint64_t h = seed ^ (uint64_t(it.len) * kMurmurM);
    const uint32_t nblk = it.len >> 3, rem = it.len & 7;
    if (nblk >= 1) h = mm_block(h, it.w0);
    if (nblk >= 2) h = mm_block(h, it.w1);
    for (uint32_t j = 2; j < nblk; j++) h = mm_block(h, load_le(it.p + 8 * j, 8));
    if (rem) {
        uint64_t t = nblk == 0 ? it.w0 : (nblk == 1 ? it.w1 : load_le(it.p + 8 * nblk, rem));
        h ^= t;
        h *= kMurmurM;
    }
    return mm_final(h);
}

// MurmurHash64A of an item of at most 8 bytes held in w (zero padded).
SKE_HD uint64_t murmur_short(uint64_t w, uint32_t len, uint64_t seed) {
    uint64_t h = seed ^ (uint64_t(len) * kMurmurM);
    if (len == 8) {
        h = mm_block(h, w);
    } else if (len) {
        h ^= w;
        h *= kMurmurM;
    }
    return mm_final(h);
}

// hllPatLen(): index = low 14 bits, count = 1 + trailing zeros of
// (hash >> 14) | 1<<50, in [1, 51].
SKE_HD void hll_patlen(uint64_t hash, uint32_t &idx, uint32_t &rank) {
    idx = uint32_t(hash & (kHllRegs - 1));
    uint64_t w = (hash >> kHllP) | (uint64_t(1) << kHllQ);
#ifdef __HIP_DEVICE_COMPILE__
    rank = uint32_t(__builtin_ctzll(w)) + 1;
#else
    rank = uint32_t(__builtin_ctzll(w)) + 1;
#endif
}

// ---------------------------------------------------------------------------
// Exact n mod d for a runtime divisor (Granlund-Montgomery, "Division by
// invariant integers using multiplication", fig. 4.1): l = ceil(log2 d),
// m = floor(2^64 (2^l - d) / d) + 1, q = (t + ((n - t) >> 1)) >> (l - 1),
// t = mulhi(m, n).  Valid for every 64-bit n and 2 <= d < 2^63.
// ---------------------------------------------------------------------------
struct Divisor {
    uint64_t d;    // bloom->bits
    uint64_t m;    // magic
    uint64_t t;    // 2^64 mod d (carry correction of the probe stepping)
    uint32_t sh;   // l - 1
    uint32_t pad_;
};

SKE_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#ifdef __HIP_DEVICE_COMPILE__
    return __umul64hi(a, b);
#else
    return uint64_t((unsigned __int128)a * b >> 64);
#endif
}

SKE_HD uint64_t fastmod(uint64_t n, const Divisor &D) {
    uint64_t t1 = mulhi64(D.m, n);
    uint64_t q = (t1 + ((n - t1) >> 1)) >> D.sh;
    return n - q * D.d;
}

inline Divisor make_divisor(uint64_t d) {
    Divisor D{};
    D.d = d;
    uint32_t l = 0;
    while (l < 64 && (uint64_t(1) << l) < d) l++;
    unsigned __int128 num = ((unsigned __int128)1 << 64) * ((uint64_t(1) << l) - d);
    D.m = uint64_t(num / d) + 1;
    D.sh = l - 1;
    D.t = uint64_t((((unsigned __int128)1) << 64) % d);
    return D;
}

// Probe cursor over x_i = (a + i*b) mod 2^64 mod d  (CHECK_ADD_FUNC with
// bloom_check_add_compat's modulus bloom->bits).  step() keeps v_i = a+i*b
// (mod 2^64) and x_i; when v wraps, x drops by 2^64 mod d.
struct ProbeCursor {
    uint64_t v, b, x, bm;
    SKE_HD void init(uint64_t a, uint64_t b_, const Divisor &D) {
        v = a;
        b = b_;
        x = fastmod(a, D);
        bm = fastmod(b_, D);
    }
    SKE_HD void step(const Divisor &D) {
        uint64_t vn = v + b;
        bool carry = vn < v;
        v = vn;
        x += bm;
        if (x >= D.d) x -= D.d;
        if (carry) x = (x >= D.t) ? x - D.t : x + D.d - D.t;
    }
};

SKE_HD uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }  // v_min_u32

// The same cursor with x kept in 32 bits, valid when d <= 2^31 (every Bloom
// link up to ~2^31 bits: all configs; x + bm < 2^32 cannot overflow).  v, the
// 64-bit running sum a + i*b, is still tracked for its carry.
struct ProbeCursor32 {
    uint64_t v, b;
    uint32_t x, bm;
    SKE_HD void init(uint64_t a, uint64_t b_, const Divisor &D) {
        v = a;
        b = b_;
        x = uint32_t(fastmod(a, D));
        bm = uint32_t(fastmod(b_, D));
    }
    SKE_HD void step(const Divisor &D) { step(uint32_t(D.d), uint32_t(D.t)); }
    // x, bm < d <= 2^31: "x = min(x, x - d)" is the conditional subtract (a
    // wrapped x - d is the larger one); the wrap of v subtracts t = 2^64 mod d,
    // and "min(x, x + d)" undoes an underflow the same way.
    SKE_HD void step(uint32_t d, uint32_t t) {
        const uint64_t vn = v + b;
        const uint32_t tsel = vn < v ? t : 0u;
        v = vn;
        x += bm;
        x = umin32(x, x - d);
        x -= tsel;
        x = umin32(x, x + d);
    }
};

// The same walk with both increments precomputed: the step whose a + i*b
// wraps 2^64 adds inc1 = (bm - 2^64 mod d) mod d, every other step inc0 = bm,
// so a step is the 64-bit add (its carry selects the increment), one 32-bit
// add and one conditional subtract.  d <= 2^31.
struct ProbeWalk32 {
    uint64_t v, b;
    uint32_t x, inc0, inc1;
    SKE_HD void init(uint64_t a, uint64_t b_, const Divisor &D) {
        v = a;
        b = b_;
        x = uint32_t(fastmod(a, D));
        inc0 = uint32_t(fastmod(b_, D));
        const uint32_t m = inc0 - uint32_t(D.t);
        inc1 = umin32(m, m + uint32_t(D.d));
    }
    SKE_HD void step(uint32_t d) {
        const uint64_t vn = v + b;
        x += vn < v ? inc1 : inc0;
        v = vn;
        x = umin32(x, x - d);
    }
};

// One link of a RedisBloom scalable chain (SBLink.inner), device view.
struct LinkDev {
    const uint8_t *bf;  // bit array (bytes multiple of 8; LSB-first bits)
    Divisor div;
    uint32_t k;          // bloom->hashes
    uint32_t lds_off;    // byte offset of this link inside the LDS image
    uint32_t rmul;       // XCD-region split: region(x) = umulhi(x, rmul) in [0, 8)
    uint32_t pad_;
};

constexpr int kRegions = 8;  // one slice of every link per XCD

struct ChainDev {
    int32_t nlinks;
    uint32_t lds_bytes;  // sum of link bytes, 16-B aligned per link
    uint32_t pad_[2];
    LinkDev link[kMaxLinks];
};

// ---------------------------------------------------------------------------
// Synthetic stream (counter based).  mix(seed, i, j) = SplitMix64 finaliser
// of seed + golden * (i*256 + j + 1).  Restated in tests/golden/gen_ref.py.
// ---------------------------------------------------------------------------
SKE_HD uint64_t splitmix_fin(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
SKE_HD uint64_t mix(uint64_t seed, uint64_t i, uint32_t j) {
    return splitmix_fin(seed + 0x9e3779b97f4a7c15ULL * (i * 256 + j + 1));
}

struct GenDev {
    uint64_t seed, lo, R, N, mul, add, inv;
    uint32_t inv_thr, near_thr, n_keys, slot_base, width;
    const uint32_t *key_cdf;
    uint64_t pow10[20];
};

SKE_HD uint64_t gen_member(const GenDev &g, uint64_t i) { return g.lo + (g.mul * i + g.add) % g.R; }
SKE_HD bool gen_is_member(const GenDev &g, uint64_t x) {
    if (x < g.lo || x >= g.lo + g.R) return false;
    uint64_t r = (x - g.lo + g.R - g.add % g.R) % g.R;
    return (r * g.inv) % g.R < g.N;
}

}  // namespace ske
