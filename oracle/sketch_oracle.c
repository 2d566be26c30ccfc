/*
 * sketch_oracle.c -- CPU ORACLE (test infrastructure only; see header).
 *
 * Scalar C restatement of the Redis / RedisBloom routines behind the
 * reference's BF.EXISTS / BF.ADD / BF.RESERVE / PFADD / PFCOUNT / PFMERGE
 * calls.  Each function names the upstream routine it follows and the
 * reference call site that reaches it.  Compiled with -ffp-contract=off so
 * that the PFCOUNT estimator performs exactly the IEEE double operations of
 * Redis's hllCount().
 */
#define _POSIX_C_SOURCE 200809L /* pthread_barrier_t under -std=c11 */
#include "sketch_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================
 * MurmurHash64A
 *   Redis src/hyperloglog.c MurmurHash64A (seed 0xadc83b19 for HLL)
 *   RedisBloom deps/murmur2/MurmurHash2.c MurmurHash64A_Bloom
 *     (seed 0xc6a4a7935bd1e995, then the first hash as the second seed)
 * Both are Austin Appleby's MurmurHash64A: 8-byte little-endian blocks,
 * tail bytes folded in LSB-first, final avalanche.  Pinned by the SMHasher
 * verification value 0x1F0D3804 (tests/test_oracle_kat.py).
 * ==================================================================== */
uint64_t orc_murmur64a(const void *key, int len, uint64_t seed) {
    const uint64_t m = 0xc6a4a7935bd1e995ULL;
    const int r = 47;
    uint64_t h = seed ^ ((uint64_t)len * m);
    const uint8_t *data = (const uint8_t *)key;
    const uint8_t *end = data + (len - (len & 7));
    while (data != end) {
        uint64_t k;
        memcpy(&k, data, 8); /* little-endian host */
        k *= m;
        k ^= k >> r;
        k *= m;
        h ^= k;
        h *= m;
        data += 8;
    }
    switch (len & 7) {
    case 7: h ^= (uint64_t)data[6] << 48; /* fall through */
    case 6: h ^= (uint64_t)data[5] << 40; /* fall through */
    case 5: h ^= (uint64_t)data[4] << 32; /* fall through */
    case 4: h ^= (uint64_t)data[3] << 24; /* fall through */
    case 3: h ^= (uint64_t)data[2] << 16; /* fall through */
    case 2: h ^= (uint64_t)data[1] << 8;  /* fall through */
    case 1:
        h ^= (uint64_t)data[0];
        h *= m;
    }
    h ^= h >> r;
    h *= m;
    h ^= h >> r;
    return h;
}

/* SMHasher VerificationTest(): keys {0..i-1} hashed with seed 256-i, the
 * 256 little-endian 8-byte hashes hashed again with seed 0. */
uint32_t orc_smhasher_verification(void) {
    uint8_t key[256];
    uint8_t hashes[8 * 256];
    for (int i = 0; i < 256; i++) {
        key[i] = (uint8_t)i;
        uint64_t h = orc_murmur64a(key, i, (uint64_t)(256 - i));
        memcpy(&hashes[i * 8], &h, 8);
    }
    uint64_t f = orc_murmur64a(hashes, 8 * 256, 0);
    return (uint32_t)(f & 0xffffffffu);
}

/* ======================================================================
 * HyperLogLog -- Redis src/hyperloglog.c, P = 14, Q = 50
 * ==================================================================== */
#define HLL_SEED 0xadc83b19ULL

/* hllPatLen(): register index = low 14 bits of the hash; count = length of
 * the "000..1" run in the remaining 50 bits (bit 50 forced to 1) + 1. */
int orc_hll_patlen(const uint8_t *ele, size_t len, long *regp) {
    uint64_t hash = orc_murmur64a(ele, (int)len, HLL_SEED);
    uint64_t index = hash & (ORC_HLL_REGISTERS - 1);
    hash >>= ORC_HLL_P;
    hash |= ((uint64_t)1 << ORC_HLL_Q);
    uint64_t bit = 1;
    int count = 1;
    while ((hash & bit) == 0) {
        count++;
        bit <<= 1;
    }
    *regp = (long)index;
    return count;
}

/* hllDenseAdd()/hllSparseAdd() collapse, on the raw register view, to
 * reg = max(reg, count); returns 1 when the register changed (the value
 * that makes PFADD reply 1, attendance_processor.py:129). */
int orc_hll_add(uint8_t *regs, const uint8_t *ele, size_t len) {
    long idx;
    int count = orc_hll_patlen(ele, len, &idx);
    if (count > regs[idx]) {
        regs[idx] = (uint8_t)count;
        return 1;
    }
    return 0;
}

/* hllRawRegHisto() */
void orc_hll_histo(const uint8_t *regs, int *histo64) {
    memset(histo64, 0, 64 * sizeof(int));
    for (int j = 0; j < ORC_HLL_REGISTERS; j++) histo64[regs[j] & 63]++;
}

/* hllSigma() -- Ertl, "New cardinality estimation algorithms for
 * HyperLogLog sketches", arXiv:1702.01284, as coded in Redis. */
double orc_hll_sigma(double x) {
    if (x == 1.) return INFINITY;
    double zPrime;
    double y = 1;
    double z = x;
    do {
        x *= x;
        zPrime = z;
        z += x * y;
        y += y;
    } while (zPrime != z);
    return z;
}

/* hllTau() */
double orc_hll_tau(double x) {
    if (x == 0. || x == 1.) return 0.;
    double zPrime;
    double y = 1.0;
    double z = 1 - x;
    do {
        x = sqrt(x);
        zPrime = z;
        y *= 0.5;
        z -= pow(1 - x, 2) * y;
    } while (zPrime != z);
    return z / 3;
}

/* hllCount() estimator part (after the register histogram). */
uint64_t orc_hll_estimate(const int *reghisto) {
    double m = ORC_HLL_REGISTERS;
    double z = m * orc_hll_tau((m - reghisto[ORC_HLL_Q + 1]) / (double)m);
    for (int j = ORC_HLL_Q; j >= 1; --j) {
        z += reghisto[j];
        z *= 0.5;
    }
    z += m * orc_hll_sigma(reghisto[0] / (double)m);
    double E = (double)llroundl(0.721347520444481703680 * m * m / z);
    return (uint64_t)E;
}

uint64_t orc_hll_count(const uint8_t *regs) {
    int h[64];
    orc_hll_histo(regs, h);
    return orc_hll_estimate(h);
}

/* hllMerge(): per-register max (PFMERGE and multi-key PFCOUNT). */
void orc_hll_merge(uint8_t *dst, const uint8_t *src) {
    for (int j = 0; j < ORC_HLL_REGISTERS; j++)
        if (src[j] > dst[j]) dst[j] = src[j];
}

/* HLL_DENSE_SET_REGISTER / HLL_DENSE_GET_REGISTER: 6-bit registers packed
 * LSB-first.  The dense buffer is ORC_HLL_DENSE_BYTES long; the macro's
 * byte+1 access past the last register lands on the sds terminator in Redis
 * and is skipped here. */
void orc_hll_dense_encode(const uint8_t *regs, uint8_t *p) {
    memset(p, 0, ORC_HLL_DENSE_BYTES);
    for (unsigned long regnum = 0; regnum < ORC_HLL_REGISTERS; regnum++) {
        unsigned long byte = regnum * ORC_HLL_BITS / 8;
        unsigned long fb = regnum * ORC_HLL_BITS & 7;
        unsigned long fb8 = 8 - fb;
        unsigned long v = regs[regnum];
        p[byte] &= (uint8_t)~(63UL << fb);
        p[byte] |= (uint8_t)(v << fb);
        if (byte + 1 < ORC_HLL_DENSE_BYTES) {
            p[byte + 1] &= (uint8_t)~(63UL >> fb8);
            p[byte + 1] |= (uint8_t)(v >> fb8);
        }
    }
}

void orc_hll_dense_decode(const uint8_t *p, uint8_t *regs) {
    for (unsigned long regnum = 0; regnum < ORC_HLL_REGISTERS; regnum++) {
        unsigned long byte = regnum * ORC_HLL_BITS / 8;
        unsigned long fb = regnum * ORC_HLL_BITS & 7;
        unsigned long fb8 = 8 - fb;
        unsigned long b0 = p[byte];
        unsigned long b1 = byte + 1 < ORC_HLL_DENSE_BYTES ? p[byte + 1] : 0;
        regs[regnum] = (uint8_t)(((b0 >> fb) | (b1 << fb8)) & 63);
    }
}

/* Sparse opcodes (hllSparseRegHisto / hllSparseToDense):
 *   ZERO  00xxxxxx           run of xxxxxx+1 zero registers
 *   XZERO 01xxxxxx yyyyyyyy  run of 14-bit len+1 zero registers
 *   VAL   1vvvvvxx           run of xx+1 registers of value vvvvv+1 */
int orc_hll_decode_string(const uint8_t *s, size_t len, uint8_t *regs) {
    if (len < ORC_HLL_HDR_SIZE || memcmp(s, "HYLL", 4) != 0) return -1;
    uint8_t enc = s[4];
    const uint8_t *p = s + ORC_HLL_HDR_SIZE;
    const uint8_t *end = s + len;
    if (enc == 0) { /* HLL_DENSE */
        if (len != ORC_HLL_HDR_SIZE + ORC_HLL_DENSE_BYTES) return -1;
        orc_hll_dense_decode(p, regs);
        return 0;
    }
    if (enc != 1) return -1;
    long idx = 0;
    while (p < end) {
        long runlen;
        int val = 0;
        if ((*p & 0xc0) == 0x00) {
            runlen = (*p & 0x3f) + 1;
            p++;
        } else if ((*p & 0xc0) == 0x40) {
            if (p + 1 >= end) return -1;
            runlen = (((long)(*p & 0x3f) << 8) | p[1]) + 1;
            p += 2;
        } else {
            val = ((*p >> 2) & 0x1f) + 1;
            runlen = (*p & 0x3) + 1;
            p++;
        }
        if (idx + runlen > ORC_HLL_REGISTERS) return -1;
        for (long j = 0; j < runlen; j++) regs[idx++] = (uint8_t)val;
    }
    return idx == ORC_HLL_REGISTERS ? 0 : -1;
}

/* ======================================================================
 * RedisBloom deps/bloom/bloom.c
 * ==================================================================== */
#define LN2 (0.693147180559945)

/* calc_bpe() */
static double calc_bpe(double error) {
    static const double denom = 0.480453013918201; /* ln(2)^2 */
    double num = log(error);
    double bpe = -(num / denom);
    if (bpe < 0) bpe = -bpe;
    return bpe;
}

/* bloom_init() */
int orc_bloom_init(orc_bloom *bloom, uint64_t entries, double error, unsigned options) {
    memset(bloom, 0, sizeof(*bloom));
    if (entries < 1 || error <= 0 || error >= 1.0) return 1;
    bloom->error = error;
    bloom->bits = 0;
    bloom->entries = entries;
    bloom->bpe = calc_bpe(error);
    uint64_t bits;
    if (options & ORC_BLOOM_OPT_ENTS_IS_BITS) {
        if (entries > 64) return 1;
        bloom->n2 = (uint8_t)entries;
        bits = 1ULL << bloom->n2;
        bloom->entries = (uint64_t)(bits / bloom->bpe);
    } else if (options & ORC_BLOOM_OPT_NOROUND) {
        bits = bloom->bits = (uint64_t)(entries * bloom->bpe);
        if (bits == 0) bits = bloom->bits = 1;
        bloom->n2 = 0;
    } else {
        double bn2 = logb(entries * bloom->bpe);
        if (bn2 > 63 || bn2 == INFINITY) return 1;
        bloom->n2 = (uint8_t)(bn2 + 1);
        bits = 1ULL << bloom->n2;
        size_t bitDiff = bits - (entries * bloom->bpe);
        size_t itemDiff = bitDiff / bloom->bpe;
        bloom->entries += itemDiff;
    }
    if (bits % 64) {
        bloom->bytes = ((bits / 64) + 1) * 8;
    } else {
        bloom->bytes = bits / 8;
    }
    bloom->bits = bloom->bytes * 8;
    bloom->force64 = (options & ORC_BLOOM_OPT_FORCE64) ? 1 : 0;
    bloom->hashes = (int)ceil(LN2 * bloom->bpe);
    bloom->bf = (uint8_t *)calloc(bloom->bytes ? bloom->bytes : 1, 1);
    return bloom->bf == NULL;
}

/* bloom_calc_hash64() */
void orc_bloom_hash64(const void *buf, int len, uint64_t *a, uint64_t *b) {
    *a = orc_murmur64a(buf, len, 0xc6a4a7935bd1e995ULL);
    *b = orc_murmur64a(buf, len, *a);
}

/* test_bit_set_bit(): byte x>>3, mask 1<<(x%8). */
static int test_bit_set_bit(uint8_t *buf, uint64_t x, int mode) {
    uint64_t byte = x >> 3;
    uint8_t mask = (uint8_t)(1 << (x % 8));
    uint8_t c = buf[byte];
    if (c & mask) return 1;
    if (mode == 1) buf[byte] = c | mask;
    return 0;
}

/* CHECK_ADD_FUNC(T, modExp) with the three instantiations
 * bloom_check_add32 (mod 1<<n2, uint32 arithmetic), bloom_check_add64
 * (mod 1<<n2, uint64) and bloom_check_add_compat (mod bits, uint64), chosen
 * as bloom_check_h()/bloom_add_h() choose them. */
int orc_bloom_check_add(orc_bloom *bloom, uint64_t ha, uint64_t hb, int mode, uint64_t *probes) {
    int found_unset = 0;
    if (bloom->n2 > 0 && !(bloom->force64 || bloom->n2 > 31)) {
        const uint32_t mod = (uint32_t)(1u << bloom->n2);
        for (uint32_t i = 0; i < (uint32_t)bloom->hashes; i++) {
            uint32_t x = (uint32_t)((ha + i * hb) % mod);
            if (probes) (*probes)++;
            if (!test_bit_set_bit(bloom->bf, x, mode)) {
                if (mode == 0) return 0;
                found_unset = 1;
            }
        }
    } else {
        const uint64_t mod = bloom->n2 > 0 ? (1ULL << bloom->n2) : bloom->bits;
        for (uint64_t i = 0; i < (uint64_t)bloom->hashes; i++) {
            uint64_t x = (ha + i * hb) % mod;
            if (probes) (*probes)++;
            if (!test_bit_set_bit(bloom->bf, x, mode)) {
                if (mode == 0) return 0;
                found_unset = 1;
            }
        }
    }
    if (mode == 0) return 1;
    return found_unset;
}

/* ======================================================================
 * RedisBloom src/sb.c -- scalable chain
 * ==================================================================== */
#define ERROR_TIGHTENING_RATIO 0.5

/* SBChain_AddLink() */
static int chain_add_link(orc_chain *c, uint64_t size, double error) {
    orc_bloom *nl = (orc_bloom *)realloc(c->links, sizeof(orc_bloom) * (size_t)(c->nlinks + 1));
    if (!nl) return -1;
    c->links = nl;
    orc_bloom *link = &c->links[c->nlinks];
    c->nlinks++;
    int rc = orc_bloom_init(link, size, error, c->options);
    link->size = 0;
    return rc;
}

/* SB_NewChain(): the first link gets error * 0.5 unless NO_SCALING.
 * rebloom.c bfCreateChain() passes FORCE64 | NOROUND (| NO_SCALING). */
orc_chain *orc_chain_new(uint64_t capacity, double error, unsigned options, unsigned growth) {
    if (capacity == 0 || error == 0 || error >= 1) return NULL;
    orc_chain *c = (orc_chain *)calloc(1, sizeof(orc_chain));
    if (!c) return NULL;
    c->growth = growth;
    c->options = options;
    double tightening = (options & ORC_BLOOM_OPT_NO_SCALING) ? 1 : ERROR_TIGHTENING_RATIO;
    if (chain_add_link(c, capacity, error * tightening) != 0) {
        orc_chain_free(c);
        return NULL;
    }
    return c;
}

void orc_chain_free(orc_chain *c) {
    if (!c) return;
    for (int i = 0; i < c->nlinks; i++) free(c->links[i].bf);
    free(c->links);
    free(c);
}

/* SBChain_Check(): newest link first. */
int orc_chain_check(const orc_chain *c, const void *data, size_t len, uint64_t *probes) {
    uint64_t a, b;
    orc_bloom_hash64(data, (int)len, &a, &b);
    for (int ii = c->nlinks - 1; ii >= 0; --ii)
        if (orc_bloom_check_add(&c->links[ii], a, b, 0, probes)) return 1;
    return 0;
}

/* SBChain_Add(): skip if any link has it; grow when the current link's size
 * reached its entries (next link: entries*growth, error*0.5); set bits. */
int orc_chain_add(orc_chain *c, const void *data, size_t len) {
    uint64_t a, b;
    orc_bloom_hash64(data, (int)len, &a, &b);
    for (int ii = c->nlinks - 1; ii >= 0; --ii)
        if (orc_bloom_check_add(&c->links[ii], a, b, 0, NULL)) return 0;
    orc_bloom *cur = &c->links[c->nlinks - 1];
    if (cur->size >= cur->entries) {
        if (c->options & ORC_BLOOM_OPT_NO_SCALING) return -2;
        double error = cur->error * ERROR_TIGHTENING_RATIO;
        if (chain_add_link(c, cur->entries * (uint64_t)c->growth, error) != 0) return -1;
        cur = &c->links[c->nlinks - 1];
    }
    int rv = orc_bloom_check_add(cur, a, b, 1, NULL);
    if (rv) {
        cur->size++;
        c->size++;
    }
    return rv;
}

int orc_chain_nlinks(const orc_chain *c) { return c->nlinks; }
uint64_t orc_chain_size(const orc_chain *c) { return c->size; }

int orc_chain_link_info(const orc_chain *c, int i, uint64_t *entries, uint64_t *bytes,
                        uint64_t *bits, int *hashes, uint64_t *size, double *error) {
    if (i < 0 || i >= c->nlinks) return -1;
    const orc_bloom *l = &c->links[i];
    *entries = l->entries;
    *bytes = l->bytes;
    *bits = l->bits;
    *hashes = l->hashes;
    *size = l->size;
    *error = l->error;
    return 0;
}

const uint8_t *orc_chain_link_bits(const orc_chain *c, int i) {
    if (i < 0 || i >= c->nlinks) return NULL;
    return c->links[i].bf;
}

/* ======================================================================
 * BF.SCANDUMP / BF.LOADCHUNK -- RedisBloom src/sb.c [recall]:
 *   dumpedChainHeader (packed, little-endian on x86):
 *     u64 size; u32 nfilters; u32 options; u32 growth;  dumpedChainLink[nfilters]
 *   dumpedChainLink (packed), X_ENCODED_LINK's fields in declaration order:
 *     u64 bytes; u64 bits; u64 size; double error; double bpe; u32 hashes;
 *     u64 entries; u8 n2
 *   SBChain_GetEncodedHeader -> reply (SB_CHUNKITER_INIT = 1, header);
 *   SBChain_GetEncodedChunk: iter - 1 is a byte offset into the links' bit
 *   arrays laid end to end (getLinkPos); a chunk never crosses a link and is
 *   at most MAX_SCANDUMP_SIZE bytes; the next iterator is iter + len; past
 *   the end: iterator 0, no data.  SB_NewChainFromHeader: the chain of the
 *   header's links with zeroed bit arrays (force64 from the options);
 *   SBChain_LoadEncodedChunk: the chunk goes to offset (iter - len) - 1.
 * Written field by field here (no packed struct), as an encoder independent
 * of the product's formats.bf_dump_header.
 * ==================================================================== */
static void put_le(uint8_t **p, uint64_t v, int n) {
    for (int i = 0; i < n; i++) (*p)[i] = (uint8_t)(v >> (8 * i));
    *p += n;
}
static uint64_t get_le(const uint8_t **p, int n) {
    uint64_t v = 0;
    for (int i = 0; i < n; i++) v |= (uint64_t)(*p)[i] << (8 * i);
    *p += n;
    return v;
}
static uint64_t dbl_bits(double d) {
    uint64_t v;
    memcpy(&v, &d, 8);
    return v;
}
static double bits_dbl(uint64_t v) {
    double d;
    memcpy(&d, &v, 8);
    return d;
}

size_t orc_chain_dump_header(const orc_chain *c, uint8_t *out, size_t cap) {
    const size_t len = ORC_SB_HEADER_BYTES + (size_t)c->nlinks * ORC_SB_LINK_BYTES;
    if (!out || cap < len) return len;
    uint8_t *p = out;
    put_le(&p, c->size, 8);
    put_le(&p, (uint64_t)c->nlinks, 4);
    put_le(&p, c->options, 4);
    put_le(&p, c->growth, 4);
    for (int i = 0; i < c->nlinks; i++) {
        const orc_bloom *l = &c->links[i];
        put_le(&p, l->bytes, 8);
        put_le(&p, l->bits, 8);
        put_le(&p, l->size, 8);
        put_le(&p, dbl_bits(l->error), 8);
        put_le(&p, dbl_bits(l->bpe), 8);
        put_le(&p, (uint64_t)(uint32_t)l->hashes, 4);
        put_le(&p, l->entries, 8);
        put_le(&p, l->n2, 1);
    }
    return len;
}

/* getLinkPos(): the link holding byte iter - 1 of the concatenated arrays */
static int link_pos(const orc_chain *c, long long iter, uint64_t *offset) {
    if (iter < 1) return -1;
    uint64_t cur = (uint64_t)(iter - 1), seek = 0;
    for (int i = 0; i < c->nlinks; i++) {
        if (seek + c->links[i].bytes > cur) {
            *offset = cur - seek;
            return i;
        }
        seek += c->links[i].bytes;
    }
    return -1;
}

size_t orc_chain_dump_chunk(const orc_chain *c, long long *iter, size_t max_chunk, const uint8_t **data) {
    uint64_t off = 0;
    const int i = link_pos(c, *iter, &off);
    if (i < 0) {
        *iter = 0;
        *data = NULL;
        return 0;
    }
    size_t len = max_chunk;
    const uint64_t remaining = c->links[i].bytes - off;
    if (remaining < len) len = (size_t)remaining;
    *iter += (long long)len;
    *data = c->links[i].bf + off;
    return len;
}

orc_chain *orc_chain_from_header(const uint8_t *buf, size_t len) {
    if (!buf || len < ORC_SB_HEADER_BYTES) return NULL;
    const uint8_t *p = buf;
    const uint64_t size = get_le(&p, 8);
    const uint32_t nf = (uint32_t)get_le(&p, 4);
    const uint32_t options = (uint32_t)get_le(&p, 4);
    const uint32_t growth = (uint32_t)get_le(&p, 4);
    if (nf == 0 || len < ORC_SB_HEADER_BYTES + (size_t)nf * ORC_SB_LINK_BYTES) return NULL;
    orc_chain *c = (orc_chain *)calloc(1, sizeof(orc_chain));
    if (!c) return NULL;
    c->links = (orc_bloom *)calloc(nf, sizeof(orc_bloom));
    if (!c->links) {
        free(c);
        return NULL;
    }
    c->nlinks = (int)nf;
    c->size = size;
    c->options = options;
    c->growth = growth;
    for (uint32_t i = 0; i < nf; i++) {
        orc_bloom *l = &c->links[i];
        l->bytes = get_le(&p, 8);
        l->bits = get_le(&p, 8);
        l->size = get_le(&p, 8);
        l->error = bits_dbl(get_le(&p, 8));
        l->bpe = bits_dbl(get_le(&p, 8));
        l->hashes = (int)(uint32_t)get_le(&p, 4);
        l->entries = get_le(&p, 8);
        l->n2 = (uint8_t)get_le(&p, 1);
        l->force64 = (options & ORC_BLOOM_OPT_FORCE64) ? 1 : 0;
        l->bf = (uint8_t *)calloc(1, l->bytes ? l->bytes : 1);
        if (!l->bf) {
            orc_chain_free(c);
            return NULL;
        }
    }
    return c;
}

int orc_chain_load_chunk(orc_chain *c, long long iter, const uint8_t *buf, size_t len) {
    if (!buf || iter <= 0 || iter < (long long)len) return -1; /* "ERR received bad data" */
    uint64_t off = 0;
    const int i = link_pos(c, iter - (long long)len, &off);
    if (i < 0) return -2;                                      /* "ERR invalid offset - no link found" */
    if (len > c->links[i].bytes - off) return -3;              /* "ERR invalid chunk - Too big ..." */
    memcpy(c->links[i].bf + off, buf, len);
    return 0;
}

/* ======================================================================
 * Batched helpers
 * ==================================================================== */
void orc_chain_madd(orc_chain *c, const uint8_t *bytes, const uint32_t *offs, uint64_t n,
                    int8_t *out) {
    for (uint64_t i = 0; i < n; i++) {
        int rv = orc_chain_add(c, bytes + offs[i], offs[i + 1] - offs[i]);
        if (out) out[i] = (int8_t)rv;
    }
}

uint64_t orc_chain_mexists(const orc_chain *c, const uint8_t *bytes, const uint32_t *offs,
                           uint64_t n, uint8_t *out) {
    uint64_t probes = 0;
    for (uint64_t i = 0; i < n; i++)
        out[i] = (uint8_t)orc_chain_check(c, bytes + offs[i], offs[i + 1] - offs[i], &probes);
    return probes;
}

/* attendance_processor.py:100-137, transport removed: for each event,
 * BF.EXISTS (:109-113) then PFADD when valid (:127-129). */
uint64_t orc_process_swipes(const orc_chain *c, uint8_t *regs, const uint32_t *slot,
                            const uint8_t *bytes, const uint32_t *offs, uint64_t n,
                            uint8_t *out_valid, uint64_t *probes) {
    uint64_t nvalid = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t *id = bytes + offs[i];
        size_t len = offs[i + 1] - offs[i];
        int valid = c ? orc_chain_check(c, id, len, probes) : 0;
        if (out_valid) out_valid[i] = (uint8_t)valid;
        if (valid) {
            orc_hll_add(regs + (size_t)slot[i] * ORC_HLL_REGISTERS, id, len);
            nvalid++;
        }
    }
    return nvalid;
}

/* The same loop on T host threads (SURVEY.md §8d "all host cores"): the
 * BF.EXISTS answers of a contiguous share of the swipes per thread, then the
 * valid-gated PFADDs with each key owned by one thread (slot % T), so the
 * register writes never race and the result is the sequential one (register
 * max commutes).  Timing counterpart only; the checker is orc_process_swipes. */
typedef struct {
    const orc_chain *c;
    uint8_t *regs;
    const uint32_t *slot;
    const uint8_t *bytes;
    const uint32_t *offs;
    uint8_t *valid;
    uint64_t n, nvalid, probes;
    pthread_barrier_t *bar;
    int t, nt;
} orc_mt_arg;

static void *orc_mt_worker(void *p) {
    orc_mt_arg *a = (orc_mt_arg *)p;
    uint64_t lo = a->n * (uint64_t)a->t / (uint64_t)a->nt;
    uint64_t hi = a->n * (uint64_t)(a->t + 1) / (uint64_t)a->nt;
    uint64_t probes = 0, nvalid = 0;
    for (uint64_t i = lo; i < hi; i++) {
        const uint8_t *id = a->bytes + a->offs[i];
        a->valid[i] = a->c ? (uint8_t)orc_chain_check(a->c, id, a->offs[i + 1] - a->offs[i], &probes) : 0;
    }
    pthread_barrier_wait(a->bar);
    for (uint64_t i = 0; i < a->n; i++) {
        if (!a->valid[i] || a->slot[i] % (uint32_t)a->nt != (uint32_t)a->t) continue;
        orc_hll_add(a->regs + (size_t)a->slot[i] * ORC_HLL_REGISTERS, a->bytes + a->offs[i],
                    a->offs[i + 1] - a->offs[i]);
        nvalid++;
    }
    a->probes = probes;
    a->nvalid = nvalid;
    return NULL;
}

uint64_t orc_process_swipes_mt(const orc_chain *c, uint8_t *regs, const uint32_t *slot,
                               const uint8_t *bytes, const uint32_t *offs, uint64_t n,
                               uint8_t *out_valid, uint64_t *probes, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    orc_mt_arg args[256];
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
    uint8_t *valid = out_valid ? out_valid : (uint8_t *)malloc(n ? n : 1);
    for (int t = 0; t < nthreads; t++) {
        args[t] = (orc_mt_arg){c, regs, slot, bytes, offs, valid, n, 0, 0, &bar, t, nthreads};
        if (t) pthread_create(&th[t], NULL, orc_mt_worker, &args[t]);
    }
    orc_mt_worker(&args[0]);
    uint64_t nvalid = args[0].nvalid;
    if (probes) *probes += args[0].probes;
    for (int t = 1; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        nvalid += args[t].nvalid;
        if (probes) *probes += args[t].probes;
    }
    pthread_barrier_destroy(&bar);
    if (!out_valid) free(valid);
    return nvalid;
}

void orc_hll_madd(uint8_t *regs, const uint32_t *slot, const uint8_t *bytes,
                  const uint32_t *offs, uint64_t n, uint8_t *changed) {
    for (uint64_t i = 0; i < n; i++) {
        int ch = orc_hll_add(regs + (size_t)slot[i] * ORC_HLL_REGISTERS, bytes + offs[i],
                             offs[i + 1] - offs[i]);
        if (changed) changed[i] = (uint8_t)ch;
    }
}
