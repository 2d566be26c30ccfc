/*
 * sketch_oracle.h -- CPU ORACLE (test infrastructure only).
 *
 * This is a plain-C restatement of the arithmetic that the reference
 * (devarshpatel1506/Real-Time-Student-Attendance-System) reaches through
 * redis-py on its validate-and-count hot path.  None of that arithmetic is in
 * the reference's own Python; it lives in two third-party servers that the
 * reference talks to over TCP and that are NOT present in this container:
 *
 *   - Redis  src/hyperloglog.c  (MurmurHash64A, hllPatLen, dense registers,
 *     hllCount / hllTau / hllSigma, hllMerge, sparse opcodes)
 *     -- docker image `redis/redis-stack-server:latest` (README.md:218),
 *        version unpinned; restated as of Redis >= 5.0 (Ertl estimator).
 *   - RedisBloom  deps/murmur2/MurmurHash2.c (MurmurHash64A_Bloom),
 *     deps/bloom/bloom.c (bloom_init, calc_bpe, bloom_calc_hash64,
 *     CHECK_ADD_FUNC / bloom_check_add_compat, test_bit_set_bit),
 *     src/sb.c (SB_NewChain, SBChain_AddLink, SBChain_Add, SBChain_Check),
 *     src/rebloom.c (BF.* defaults: error 0.01, capacity 100, expansion 2)
 *     -- same docker image, version unpinned (RedisBloom >= 2.x).
 *
 * Reference call sites this oracle must reproduce (file:line in
 * /root/reference):
 *   attendance_processor.py:109-113  BF.EXISTS bf <student_id>
 *   attendance_processor.py:127-129  PFADD <prefix><lecture_id> <student_id>
 *   attendance_processor.py:74-92    BF.RESERVE (creation semantics)
 *   data_generator.py:57-63          BF.ADD per valid id (preload)
 *   attendance_processor.py:152      PFCOUNT
 *   attendance_analysis.py:87-97     lecture ranking (PFCOUNT variant)
 *
 * Pinning: MurmurHash64A is pinned by the SMHasher verification value
 * 0x1F0D3804; HLL by the Redis command-docs examples (PFCOUNT 7 / 3 / 6).
 * The RedisBloom geometry and SBChain growth rules are restated from the
 * published upstream source and are NOT pinned by any fixture the reference
 * holds (the reference has no tests): "Bloom parity unpinned vs Redis".
 *
 * ONLY tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  The product (libsketch) never links or calls it.
 */
#ifndef SKETCH_ORACLE_H
#define SKETCH_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- MurmurHash64A ---------------- */
uint64_t orc_murmur64a(const void *key, int len, uint64_t seed);
uint32_t orc_smhasher_verification(void);

/* ---------------- HyperLogLog (p = 14) ---------------- */
#define ORC_HLL_P 14
#define ORC_HLL_Q (64 - ORC_HLL_P)
#define ORC_HLL_REGISTERS (1 << ORC_HLL_P)
#define ORC_HLL_BITS 6
#define ORC_HLL_DENSE_BYTES ((ORC_HLL_REGISTERS * ORC_HLL_BITS + 7) / 8)
#define ORC_HLL_HDR_SIZE 16

int orc_hll_patlen(const uint8_t *ele, size_t len, long *regp);
/* raw registers: one byte per register (Redis HLL_RAW layout) */
int orc_hll_add(uint8_t *regs, const uint8_t *ele, size_t len);
void orc_hll_histo(const uint8_t *regs, int *histo64);
double orc_hll_tau(double x);
double orc_hll_sigma(double x);
uint64_t orc_hll_estimate(const int *histo64);
uint64_t orc_hll_count(const uint8_t *regs);
void orc_hll_merge(uint8_t *dst, const uint8_t *src);
void orc_hll_dense_encode(const uint8_t *regs, uint8_t *dense /* ORC_HLL_DENSE_BYTES */);
void orc_hll_dense_decode(const uint8_t *dense, uint8_t *regs);
/* Decode a full Redis HLL string ("HYLL" header + dense or sparse payload).
 * Returns 0 on success, -1 on a malformed string. */
int orc_hll_decode_string(const uint8_t *s, size_t len, uint8_t *regs);

/* ---------------- RedisBloom ---------------- */
#define ORC_BLOOM_OPT_NOROUND 1
#define ORC_BLOOM_OPT_ENTS_IS_BITS 2
#define ORC_BLOOM_OPT_FORCE64 4
#define ORC_BLOOM_OPT_NO_SCALING 8

typedef struct {
    uint64_t entries;
    uint64_t bits;
    uint64_t bytes;
    double error;
    double bpe;
    int hashes;
    uint8_t n2;
    uint8_t force64;
    uint8_t *bf;
    uint64_t size; /* SBLink.size */
} orc_bloom;

typedef struct {
    orc_bloom *links;
    int nlinks;
    uint64_t size;
    unsigned growth;
    unsigned options;
} orc_chain;

int orc_bloom_init(orc_bloom *b, uint64_t entries, double error, unsigned options);
void orc_bloom_hash64(const void *buf, int len, uint64_t *a, uint64_t *b);
/* mode 0 = read, 1 = write; returns Redis semantics; *probes += tests done */
int orc_bloom_check_add(orc_bloom *b, uint64_t ha, uint64_t hb, int mode, uint64_t *probes);

orc_chain *orc_chain_new(uint64_t capacity, double error, unsigned options, unsigned growth);
void orc_chain_free(orc_chain *c);
/* returns 1 added, 0 existed, -2 non-scaling full, -1 alloc failure */
int orc_chain_add(orc_chain *c, const void *data, size_t len);
int orc_chain_check(const orc_chain *c, const void *data, size_t len, uint64_t *probes);
/* convenience accessors for ctypes */
int orc_chain_nlinks(const orc_chain *c);
uint64_t orc_chain_size(const orc_chain *c);
int orc_chain_link_info(const orc_chain *c, int i, uint64_t *entries, uint64_t *bytes,
                        uint64_t *bits, int *hashes, uint64_t *size, double *error);
const uint8_t *orc_chain_link_bits(const orc_chain *c, int i);

/* ---------------- BF.SCANDUMP / BF.LOADCHUNK (RedisBloom src/sb.c) ---------------- */
#define ORC_SB_CHUNKITER_INIT 1
#define ORC_SB_HEADER_BYTES 20 /* dumpedChainHeader: u64 size, u32 nfilters, u32 options, u32 growth */
#define ORC_SB_LINK_BYTES 53   /* dumpedChainLink: u64 bytes, bits, size; f64 error, bpe; u32 hashes;
                                  u64 entries; u8 n2 */
/* SBChain_GetEncodedHeader: writes the header if cap allows; returns its length */
size_t orc_chain_dump_header(const orc_chain *c, uint8_t *out, size_t cap);
/* SBChain_GetEncodedChunk: *iter in/out (past the end: 0 and no data) */
size_t orc_chain_dump_chunk(const orc_chain *c, long long *iter, size_t max_chunk, const uint8_t **data);
/* SB_NewChainFromHeader (NULL on bad data) / SBChain_LoadEncodedChunk (0 ok,
 * -1 bad data, -2 no link at that offset, -3 chunk too big for its link) */
orc_chain *orc_chain_from_header(const uint8_t *buf, size_t len);
int orc_chain_load_chunk(orc_chain *c, long long iter, const uint8_t *buf, size_t len);

/* ---------------- batched helpers (ctypes-friendly) ---------------- */
/* packed ids: bytes + offs[n+1] */
void orc_chain_madd(orc_chain *c, const uint8_t *bytes, const uint32_t *offs, uint64_t n,
                    int8_t *out);
uint64_t orc_chain_mexists(const orc_chain *c, const uint8_t *bytes, const uint32_t *offs,
                           uint64_t n, uint8_t *out);
/* Per-event processor loop (attendance_processor.py:100-137 without the
 * transport): BF.EXISTS, then PFADD into regs[slot[i]] when valid.
 * regs = nkeys * 16384 raw registers.  Returns the number of valid events;
 * *probes (optional) accumulates Bloom bit tests. */
uint64_t orc_process_swipes(const orc_chain *c, uint8_t *regs, const uint32_t *slot,
                            const uint8_t *bytes, const uint32_t *offs, uint64_t n,
                            uint8_t *out_valid, uint64_t *probes);
/* The same on nthreads host threads (BF.EXISTS by swipe share, PFADD by key
 * owner); identical results.  CPU-baseline timing only. */
uint64_t orc_process_swipes_mt(const orc_chain *c, uint8_t *regs, const uint32_t *slot,
                               const uint8_t *bytes, const uint32_t *offs, uint64_t n,
                               uint8_t *out_valid, uint64_t *probes, int nthreads);
/* PFADD of many elements with per-element "this element changed a register"
 * flags (sequential Redis order). */
void orc_hll_madd(uint8_t *regs, const uint32_t *slot, const uint8_t *bytes,
                  const uint32_t *offs, uint64_t n, uint8_t *changed);

#ifdef __cplusplus
}
#endif
#endif
