/*
 * sketch.h -- C-ABI of libsketch, the MI355X (gfx950) sketch engine for the
 * attendance validate-and-count hot path.
 *
 * The reference (devarshpatel1506/Real-Time-Student-Attendance-System) reaches
 * this path through a redis-py client object (attendance_processor.py:37-41,
 * data_generator.py:45-49).  Each entry point below replaces one family of the
 * RESP round trips that client makes; the Python facade
 * (real-time-student-attendance-system_amd/client.py) keeps the redis-py call
 * surface and binds these symbols through ctypes (INTEGRATION.md shows the
 * binding).
 *
 * Conventions
 *   - return 0 (SKE_OK) or a negative SKE_E* code; no exception crosses the ABI;
 *     ske_strerror() maps a code to the Redis / RedisBloom error text.
 *   - the caller owns every input / output buffer.  `mem` says where the
 *     buffers live: SKE_MEM_HOST (host memory, staged through the context's
 *     device buffers; pageable inputs above 8 MB go through two pinned 32 MB
 *     buffers filled by up to 8 host threads the context starts on first use)
 *     or SKE_MEM_DEVICE (HIP device pointers, e.g. torch-ROCm data_ptr(), used
 *     in place on the context stream).  SKE_MEM_HOST inputs must not be
 *     modified until the call returns (pinned ones are read by the DMA engine
 *     directly; the offsets are checked on the copy that is moved).
 *   - packed items: `bytes` + `offs[n+1]` (u32 byte offsets, offs[0] may be
 *     non-zero).  Device byte buffers must stay readable up to the next 8-byte
 *     boundary after bytes+offs[n] (any hipMalloc / torch allocation is).
 *   - a context is single-threaded and stream-ordered; every call returns
 *     after its work on the context stream completed, except ske_swipes_async.
 *   - filters are addressed by a caller-chosen id `fid` < SKE_MAX_FILTERS, HLL
 *     keys by a caller-chosen register-slab slot.  The facade maps Redis key
 *     names to fids / slots.
 */
#ifndef SKETCH_H
#define SKETCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SKE_OK 0
#define SKE_EINVAL -1        /* bad argument */
#define SKE_ENOMEM -2        /* device or host allocation failed */
#define SKE_EHIP -3          /* HIP runtime error (see ske_last_hip_error) */
#define SKE_ENOFILTER -4     /* fid not reserved */
#define SKE_EEXISTS -5       /* BF.RESERVE on an existing key: "ERR item exists" */
#define SKE_EFULL -6         /* non-scaling filter full */
#define SKE_ERANGE -7        /* HLL slot outside the reserved slab */
#define SKE_EBADRATE -8      /* "ERR (0 < error rate range < 1)" */
#define SKE_EBADCAP -9       /* "ERR (capacity should be larger than 0)" */
#define SKE_EBADEXP -10      /* "ERR expansion should be greater or equal to 1" */
#define SKE_EBADHLL -11      /* corrupted HLL string on import */
#define SKE_ETOOLONG -12     /* item longer than the supported maximum */
#define SKE_EBUSY -13        /* device buffers (scratch, HLL slab) pinned by a recorded graph */

#define SKE_MEM_HOST 0
#define SKE_MEM_DEVICE 1

#define SKE_MAX_FILTERS 4096
#define SKE_MAX_LINKS 48
#define SKE_HLL_REGISTERS 16384
#define SKE_HLL_DENSE_BYTES 12288

typedef struct ske_ctx ske_ctx;

typedef struct {
    uint64_t capacity;      /* sum of link entries   (BF.INFO Capacity) */
    uint64_t size_bytes;    /* bytes of all bit arrays + headers (BF.INFO Size) */
    uint32_t nfilters;      /* links in the chain    (BF.INFO Number of filters) */
    uint32_t expansion;     /* growth factor         (BF.INFO Expansion rate) */
    uint64_t inserted;      /* items added           (BF.INFO Number of items inserted) */
    int32_t nonscaling;
    int32_t pad_;
} ske_bf_info_t;

typedef struct {
    uint64_t entries;  /* bloom->entries */
    uint64_t bytes;    /* bloom->bytes */
    uint64_t bits;     /* bloom->bits (modulus of the probe sequence) */
    uint64_t size;     /* SBLink.size (items added to this link) */
    double error;      /* bloom->error */
    double bpe;        /* bloom->bpe */
    int32_t hashes;    /* bloom->hashes (k) */
    int32_t pad_;
} ske_bf_link_t;

/* Synthetic swipe stream (counter-based, device-side).  See DESIGN.md
 * "Synthetic workload" for the exact definition; tests restate it in numpy. */
typedef struct {
    uint64_t seed;
    uint64_t id_lo, id_hi;        /* IDs in [id_lo, id_hi), all with the same digit count */
    uint64_t n_members;           /* valid population: first n_members of the permutation */
    uint64_t perm_mul, perm_add;  /* member(i) = id_lo + (perm_mul*i + perm_add) mod R */
    uint64_t perm_mul_inv;        /* perm_mul^-1 mod R (R = id_hi - id_lo < 2^32) */
    uint32_t invalid_thresh;      /* P(invalid) * 2^32 */
    uint32_t near_thresh;         /* P(near-collision | invalid) * 2^32 */
    uint32_t n_keys;              /* HLL keys of this stream: slot_base + [0, n_keys) */
    uint32_t slot_base;
    const uint32_t *key_cdf;      /* optional device table (n_keys u32 CDF * 2^32); NULL = uniform */
} ske_gen_params_t;

/* ---- context ---- */
int ske_open(int device, ske_ctx **out);
int ske_close(ske_ctx *ctx);
const char *ske_strerror(int code);
const char *ske_last_hip_error(ske_ctx *ctx);
int ske_set_stream(ske_ctx *ctx, void *hip_stream); /* NULL = the context's own stream */
int ske_get_stream(ske_ctx *ctx, void **hip_stream); /* the stream calls enqueue on now */
/* Wait for the context stream.  Also reports (and clears) the sticky device
 * error word that enqueue-only calls leave set: SKE_ERANGE when a valid swipe
 * named an HLL slot outside the slab since the last check.  The word is read
 * and cleared by device-side atomic exchanges (no flag set concurrently on
 * another stream is lost).  A synchronous K1 / PFADD / ingest call reports
 * the out-of-range slots flagged while it ran: its own, and those of any work
 * that was running at the same time on other streams (enqueue-only calls
 * still in flight may be attributed to it -- the flag is one device word);
 * what finished before it began is kept for the next ske_sync /
 * ske_check_errors. */
int ske_sync(ske_ctx *ctx);
int ske_check_errors(ske_ctx *ctx);  /* the same check: sync + report + clear */
int ske_device_alloc(ske_ctx *ctx, uint64_t bytes, void **out); /* device scratch for callers */
int ske_device_free(ske_ctx *ctx, void *p);
int ske_memcpy(ske_ctx *ctx, void *dst, const void *src, uint64_t bytes, int kind); /* 0 H2D 1 D2H 2 D2D */

/* ---- Bloom (RedisBloom SBChain) ----
 * BF.RESERVE key error_rate capacity [EXPANSION e] [NONSCALING]
 *   replaces: execute_command('BF.RESERVE', ...) attendance_processor.py:83-88
 *   (also the implicit auto-create of BF.ADD: data_generator.py:59-63). */
int ske_bf_reserve(ske_ctx *ctx, uint32_t fid, double error_rate, uint64_t capacity,
                   uint32_t expansion, int nonscaling);
int ske_bf_exists_key(ske_ctx *ctx, uint32_t fid); /* 1 if reserved, 0 if not */
int ske_bf_free(ske_ctx *ctx, uint32_t fid);
/* BF.MADD key item...  (BF.ADD = n 1), sequential RedisBloom semantics:
 *   out[i] = 1 added, 0 already present, -2 non-scaling filter full.
 *   replaces: execute_command('BF.ADD', BLOOM_FILTER_KEY, id) data_generator.py:59-63 */
int ske_bf_madd(ske_ctx *ctx, uint32_t fid, const uint8_t *bytes, const uint32_t *offs,
                uint64_t n, int8_t *out_or_null, int mem);
/* BF.MEXISTS key item...  (BF.EXISTS = n 1); a missing key answers 0s.
 *   replaces: execute_command('BF.EXISTS', BLOOM_FILTER_KEY, student_id)
 *   attendance_processor.py:109-113 and the probe at :78 */
int ske_bf_mexists(ske_ctx *ctx, uint32_t fid, const uint8_t *bytes, const uint32_t *offs,
                   uint64_t n, uint8_t *out, int mem);
/* BF.INFO / BF.DEBUG and BF.SCANDUMP-style raw bit arrays */
int ske_bf_info(ske_ctx *ctx, uint32_t fid, ske_bf_info_t *out);
int ske_bf_link_info(ske_ctx *ctx, uint32_t fid, uint32_t link, ske_bf_link_t *out);
int ske_bf_export_link(ske_ctx *ctx, uint32_t fid, uint32_t link, uint8_t *out, uint64_t cap);
int ske_bf_import_link(ske_ctx *ctx, uint32_t fid, uint32_t link, const uint8_t *in,
                       uint64_t nbytes);
/* BF.LOADCHUNK key <iter> <data>: bytes [offset, offset + nbytes) of one link's
 * bit array (SBChain_LoadEncodedChunk); the range must lie inside the link. */
int ske_bf_link_write(ske_ctx *ctx, uint32_t fid, uint32_t link, uint64_t offset,
                      const uint8_t *in, uint64_t nbytes);
/* BF.LOADCHUNK key 1 <header>: a chain with exactly the given links (geometry
 * and sizes as dumped by BF.SCANDUMP's header chunk, zeroed bit arrays; the
 * data chunks then go in through ske_bf_import_link / the facade).  Each
 * link needs bits == bytes * 8, 1 <= hashes <= 64.  SKE_EEXISTS if fid exists.
 *   replaces: SB_NewChainFromHeader (RedisBloom src/sb.c) behind BF.LOADCHUNK */
int ske_bf_load_header(ske_ctx *ctx, uint32_t fid, const ske_bf_link_t *links, uint32_t nlinks,
                       uint64_t inserted, uint32_t expansion, int nonscaling);

/* ---- HyperLogLog register slab (Redis p=14, one byte per register) ---- */
int ske_hll_reserve(ske_ctx *ctx, uint32_t nslots);  /* grow the slab to >= nslots keys */
uint32_t ske_hll_capacity(ske_ctx *ctx);
int ske_hll_clear(ske_ctx *ctx, uint32_t slot);      /* new / deleted key: zero registers */
/* PFADD key element...  for many (key, element) pairs at once.
 *   changed_or_null: per-element "this element raised a register" in the
 *   given order (sequential Redis semantics); the facade folds it per call.
 *   replaces: redis_client.pfadd(hll_key, student_id) attendance_processor.py:127-129 */
int ske_hll_pfadd(ske_ctx *ctx, const uint32_t *slot, const uint8_t *bytes,
                  const uint32_t *offs, uint64_t n, uint8_t *changed_or_null, int mem);
/* PFCOUNT key [key ...] (union), one answer.  attendance_processor.py:152 */
int ske_hll_pfcount(ske_ctx *ctx, const uint32_t *slots, uint32_t nkeys, uint64_t *out);
/* PFCOUNT of each key separately (rankings, attendance_analysis.py:87-97 as
 * README.md:179 describes); slots == NULL: keys 0..nkeys-1 of the slab.
 * Group form: union over slots[goffs[g]..goffs[g+1]).  With SKE_MEM_DEVICE the
 * slot list of the each form is range-checked on the device (SKE_ERANGE). */
int ske_hll_pfcount_each(ske_ctx *ctx, const uint32_t *slots, uint32_t nkeys, uint64_t *out,
                         int mem);
int ske_hll_pfcount_groups(ske_ctx *ctx, const uint32_t *slots, const uint32_t *goffs,
                           uint32_t ngroups, uint64_t *out, int mem);
/* PFMERGE dst src...  (dst's own registers take part, as in Redis) */
int ske_hll_pfmerge(ske_ctx *ctx, uint32_t dst, const uint32_t *srcs, uint32_t n);
/* the same with a device-resident source list (a plan kept on the GPU, e.g.
 * the campus PFMERGE of C5's 1.8M day keys): its range is checked on the
 * device (SKE_ERANGE), nothing is staged from the host.
 *   replaces: PFMERGE (north star; attendance_analysis.py:87-97 as README.md:179) */
int ske_hll_pfmerge_dev(ske_ctx *ctx, uint32_t dst, const uint32_t *srcs_dev, uint32_t n);
int ske_hll_histogram(ske_ctx *ctx, uint32_t slot, uint32_t *out64);
int ske_hll_export_raw(ske_ctx *ctx, uint32_t slot, uint8_t *out16384);
int ske_hll_export_dense(ske_ctx *ctx, uint32_t slot, uint8_t *out12288);
int ske_hll_import_raw(ske_ctx *ctx, uint32_t slot, const uint8_t *regs16384);
/* raw device pointer of the slab (slot s at + s*16384), for RCCL max-reduce */
int ske_hll_slab(ske_ctx *ctx, void **dev_ptr, uint64_t *bytes);
/* dst_dev[g*16384 ..] = register max over slots[goffs[g]..goffs[g+1]) (K3 into an
 * external device buffer, e.g. a torch tensor that RCCL then max-reduces);
 * an empty group yields zeros.  slots / goffs are host arrays. */
int ske_hll_merge_groups_dev(ske_ctx *ctx, const uint32_t *slots, const uint32_t *goffs,
                             uint32_t ngroups, uint8_t *dst_dev);
/* estimator only: PFCOUNT of raw register arrays already on the device */
int ske_hll_count_raw_dev(ske_ctx *ctx, const uint8_t *regs_dev, uint32_t nkeys, uint64_t *out);

/* ---- the fused hot path (K1) ----
 * For every swipe i: v = BF.EXISTS fid id_i; if v: PFADD slot_i id_i.
 *   replaces the per-event pair attendance_processor.py:109-113 + :127-129.
 * out_valid (may be NULL) receives v per swipe. */
int ske_swipes(ske_ctx *ctx, uint32_t fid, const uint32_t *slot, const uint8_t *bytes,
               const uint32_t *offs, uint64_t n, uint8_t *out_valid, int mem);
/* device-pointer form that only enqueues (no sync); for the benchmark */
int ske_swipes_async(ske_ctx *ctx, uint32_t fid, const uint32_t *slot, const uint8_t *bytes,
                     const uint32_t *offs, uint64_t n, uint8_t *out_valid);
/* fixed-width form: id i is the `width` bytes at bytes + i*width (no offset
 * array -- e.g. fixed-digit student ids, which every config uses).  Same
 * semantics as ske_swipes; the id load needs no offset load first. */
int ske_swipes_fixed(ske_ctx *ctx, uint32_t fid, const uint32_t *slot, const uint8_t *bytes,
                     uint32_t width, uint64_t n, uint8_t *out_valid, int mem);
int ske_swipes_fixed_async(ske_ctx *ctx, uint32_t fid, const uint32_t *slot,
                           const uint8_t *bytes, uint32_t width, uint64_t n, uint8_t *out_valid);
/* Fixed-width swipes with the answers packed 1 bit per swipe (bit i & 7 of
 * out_bits[i >> 3], LSB first -- numpy packbits(bitorder="little")).  Same
 * BF.EXISTS / PFADD semantics as ske_swipes.  With host memory the batch is
 * pipelined in chunks: a chunk's ids and slots cross the host link while K1
 * runs on the previous one; the link carries width + 4 bytes per swipe in and
 * 1/8 byte out (the offsets-and-bytes form: width + 9).  Synchronous; reports
 * the out-of-range slots flagged while it ran (SKE_ERANGE; see ske_sync).
 *   replaces the per-event pair attendance_processor.py:109-113 + :127-129
 *   for a batch of fixed-digit student ids (every config's ids) */
int ske_swipes_fixed_bits(ske_ctx *ctx, uint32_t fid, const uint32_t *slot, const uint8_t *bytes,
                          uint32_t width, uint64_t n, uint8_t *out_bits, int mem);
/* Swipes that arrive NOT partitioned by key owner (one
 * alltoallv per batch; distributed.SwipeExchange; no reference counterpart --
 * the reference's Shared subscription hands any event to any consumer,
 * attendance_processor.py:30-34).  Device pointers.  Swipe i (fixed-width id,
 * GLOBAL key index g into the job's key universe) goes to rank key_owner[g]
 * as local slot key_local[g] -- the key map every multi-GPU path shares
 * (distributed.KeyMap: owner = MurmurHash64A(key name, 0) mod world).  An
 * index g >= nkeys goes to rank 0 with local slot 0xffffffff (K1 answers it
 * and reports SKE_ERANGE for its PFADD).  send_ids / send_slots are filled
 * owner by owner (the alltoallv input), pos[i] = the swipe's position there,
 * counts[o] (host) = swipes for owner o (the split sizes; the call
 * synchronizes the context stream for them).  world <= 64, n < 2^32. */
int ske_route_swipes(ske_ctx *ctx, const uint8_t *ids, uint32_t width, const uint32_t *gkey, uint64_t n,
                     uint32_t world, const uint32_t *key_owner, const uint32_t *key_local, uint32_t nkeys,
                     uint8_t *send_ids, uint32_t *send_slots, uint32_t *pos, uint64_t *counts);
/* The same routing with no host synchronisation (enqueue only), through one
 * packed route word per key: key_route[g] = owner << 26 | local slot (local
 * slot < 2^26), or 0xffffffff for a key no rank owns (rank 0, slot
 * 0xffffffff, as above) -- one gather per swipe instead of two.  Owner o's
 * swipes fill rows [o*cap, o*cap + counts[o]) of send_ids / send_slots (device,
 * world*cap rows), so every peer pair exchanges exactly `cap` rows (an
 * all_to_all of equal splits the host sizes without reading the device).
 * Rows [counts[o], cap) get zero id bytes and slot sink_slots[o] (device,
 * [world]: a slot owner o keeps for no key, so padding changes no key's
 * registers).  counts (device, [world]) = swipes per owner; counts[o] > cap
 * means the swipes ranked past cap were NOT sent (their answers are another
 * row's): the caller re-runs the batch with ske_route_swipes, which is safe
 * (PFADD is idempotent, answers are rewritten).  world*cap < 2^32.
 * Replaces the per-event consumer loop's hand-off, attendance_processor.py:30-34. */
int ske_route_swipes_cap_async(ske_ctx *ctx, const uint8_t *ids, uint32_t width, const uint32_t *gkey, uint64_t n,
                               uint32_t world, const uint32_t *key_route, uint32_t nkeys, uint32_t cap,
                               const uint32_t *sink_slots, uint8_t *send_ids, uint32_t *send_slots, uint32_t *pos,
                               uint32_t *counts);
/* The routing of a one-rank world, where the exchange is the identity (K1
 * reads the batch in place, answers come in input order): out_slots[i] = the
 * local slot of global key gkey[i] from key_route (as above), or 0xffffffff
 * for a key past the table or owned by no rank < world (K1 reports it as
 * SKE_ERANGE).  key_route NULL (world 1 only): the identity table of a
 * one-rank key map, slot = gkey for gkey < nkeys (< 2^26).  Device arrays,
 * enqueue only. */
int ske_route_slots_async(ske_ctx *ctx, const uint32_t *gkey, uint64_t n, const uint32_t *key_route, uint32_t nkeys,
                          uint32_t world, uint32_t *out_slots);
/* out[i] = answers[pos[i]]: the owners' BF.EXISTS answers, received back in
 * send order, into input order (enqueue only). */
int ske_route_return_async(ske_ctx *ctx, const uint8_t *answers, const uint32_t *pos, uint64_t n,
                           uint8_t *out);
/* Several device-resident batches in one call (enqueue only, graph-capturable):
 * batch j runs on branch j mod `branches` (0: SKE_MANY_DEFAULT_BRANCHES), each
 * branch a side stream forked from and joined back into the context stream.
 * With more than one branch the short-id K1 runs on one block per two CUs
 * (unless the "k1_grid" option is set), so two batches share the chip.  A
 * batch with width > 0 is fixed-width (offs unused), else bytes + offsets.
 * Same answers and registers as calling ske_swipes_async per batch in order
 * (the register update is a commutative max).  nbatch == 0 only creates the
 * branches' side streams (do that once before recording the call into a
 * graph).  No reference counterpart: the
 * reference's processor handles one Pulsar message per loop iteration
 * (attendance_processor.py:100-137); this is its batched-throughput form. */
#define SKE_MANY_MAX_BRANCHES 32
#define SKE_MANY_DEFAULT_BRANCHES 16
typedef struct ske_swipe_batch {
    const uint32_t *slot;
    const uint8_t *bytes;
    const uint32_t *offs;
    uint32_t width;
    uint64_t n;
    uint8_t *out_valid;
} ske_swipe_batch;
int ske_swipes_many_async(ske_ctx *ctx, uint32_t fid, const ske_swipe_batch *batches,
                          uint32_t nbatch, uint32_t branches);
/* probe statistics of the same swipes (untimed): Bloom bit tests performed
 * and valid count, to price the algorithmic bytes of the roofline. */
int ske_swipes_stats(ske_ctx *ctx, uint32_t fid, const uint8_t *bytes, const uint32_t *offs,
                     uint64_t n, uint64_t *probes, uint64_t *nvalid);
/* which K1 variant the current chain and options select:
 *   0 = generic LDS / global-memory K1 (sketch_kernels.hip),
 *   1 = short-id LDS K1, the chain staged in LDS (sketch_k1.hip; C1/C2/C4),
 *   2 = XCD-partitioned K1 (sketch_xr.hip),
 *   3 = partitioned K1, passes A/B/C over LDS slices (sketch_part.hip; C3/C5) */
int ske_swipes_variant(ske_ctx *ctx, uint32_t fid);
/* Tuning options (no reference counterpart): "variant" (-1 auto, 0..3 as
 * above), "tile" (LDS K1 swipes per thread: 1, 2, 4, 8), "k1_grid" (LDS K1
 * blocks, 0 = one per CU), "k1_persistent" (0/1), "part_sub" (partitioned K1
 * swipes per sub-batch, at most 2^26; 0 = 2^25), "pass_timing" (0/1); the
 * partitioned K1's
 * segmented PFADD: "hll_seg" (-1 auto, 0 never, 1 whenever the
 * chain and slab allow), "seg_density" (auto: swipes per 128-B slab line at
 * which a batch is segmented, x100, default 600, doubled for a slab of at
 * most 192 MB), "seg_dense_min" (records per window line at which a window
 * is staged in LDS, x100), "seg_klog" (0..3: keys per window 1, 2, 4, 8;
 * default 1), "seg_b1" (-1 auto, 0..9: 2^b1 level-1 buckets); "rec_groups"
 * (1: pass A writes a slice unit's probe
 * records of 8 consecutive tiles adjacently, for one-link k = 11 chains;
 * -1 auto and 0: per-tile runs, the faster form).  Any other name or an out-of-range value: SKE_EINVAL.  None
 * changes an answer or a register. */
int ske_set_option(ske_ctx *ctx, const char *name, int64_t value);
/* Kernel timing for the benchmark's roofline: with option "pass_timing" = 1
 * every K1 kernel launched outside a capture is bracketed by a HIP event pair
 * recorded on the stream it runs on.  ske_pass_times waits for them and
 * returns, per pass kind, the summed milliseconds and the kernel count:
 * [0] single-kernel K1 (LDS / global / XCD-partitioned variants), [1] [2] [3]
 * the partitioned K1's passes A (hash + probe records), B (slice probes),
 * C (answers + register max, or the segmented PFADD's answers + level-1
 * records), [4] the segmented PFADD's level-2 sort, [5] its window apply;
 * and the stages of a host-fed call (ske_swipes / ske_swipes_fixed_bits with
 * SKE_MEM_HOST): [6] its host -> device copies (per chunk, on the copy
 * stream), [7] its device -> host copies of the answers, [8] the whole call
 * (from its first enqueued operation to the end of its last).
 * reset != 0 zeroes the sums after reading. */
#define SKE_PASS_KINDS 9
int ske_pass_times(ske_ctx *ctx, double *ms_out, uint64_t *count_out, int reset);

/* ---- ingest: JSON event decode + key-slot resolution ----
 * The reference decodes each Pulsar payload on the CPU (attendance_processor.py
 * :103-106) and builds the HLL key from lecture_id (:128; README.md:105-106
 * adds the UTC day).  ske_ingest_parse decodes a batch of messages on the
 * device: for each message, status 0 = decoded (the fast JSON / ISO-8601 path,
 * see sketch_ingest.hip), 1 = left for the host (Python semantics), and for a
 * decoded one the spans of student_id / lecture_id / timestamp inside msgs,
 * the UTC day number and a 128-bit key hash.  The context's key table maps
 * key hashes to HLL slots; the host inserts a key the first time it misses.
 * All column pointers are device pointers owned by the caller (n entries,
 * kh 2n); msgs must stay readable to the next 8-byte boundary. */
typedef struct {
    uint8_t *status;
    uint32_t *id_start, *id_len, *lec_start, *lec_len, *ts_start, *ts_len;
    int32_t *day;
    uint64_t *kh;
} ske_ingest_cols_t;
int ske_ingest_parse(ske_ctx *ctx, const uint8_t *msgs, const uint32_t *moffs, uint64_t n,
                     int day_form, const ske_ingest_cols_t *cols);
/* slot_dev[i] = the slot of message i's key, 0xffffffff when not in the table
 * (or not decoded); *nmiss = decoded messages whose key missed */
int ske_keytab_lookup(ske_ctx *ctx, const ske_ingest_cols_t *cols, uint64_t n, uint32_t *slot_dev,
                      uint64_t *nmiss);
int ske_keytab_insert(ske_ctx *ctx, const uint64_t *kh_host, const uint32_t *slots_host, uint64_t n);
int ske_keytab_clear(ske_ctx *ctx);
/* the fused path (K1) over the decoded messages whose key is in the table:
 * valid_dev[i] = BF.EXISTS of message i's id (0 for the others); PFADD of the
 * valid ones.  *ntaken = messages that went through K1. */
int ske_ingest_swipes(ske_ctx *ctx, uint32_t fid, const uint8_t *msgs,
                      const ske_ingest_cols_t *cols, uint64_t n, uint8_t *valid_dev,
                      uint64_t *ntaken);

/* ---- stream capture (HIP graphs) ----
 * Record the device work of the calls made between begin and end on the
 * context stream (only enqueue-only calls: ske_swipes_async,
 * ske_swipes_fixed_async) into an executable graph, uploaded to the device;
 * each ske_graph_launch replays it on the context stream.  A consumer that
 * processes a ring of fixed device batch slots replays one graph per turn of
 * the ring instead of one launch per batch (SURVEY.md §8a-1's processor loop at
 * batch granularity).  The graph keeps the pointers it was recorded with. */
int ske_capture_begin(ske_ctx *ctx);
int ske_capture_end(ske_ctx *ctx, void **graph_out);
int ske_graph_launch(ske_ctx *ctx, void *graph);
int ske_graph_free(ske_ctx *ctx, void *graph);

/* ---- synthetic stream (device buffers) ---- */
int ske_gen_members(ske_ctx *ctx, const ske_gen_params_t *p, uint64_t start, uint64_t n,
                    uint8_t *bytes_dev, uint32_t *offs_dev);
int ske_gen_swipes(ske_ctx *ctx, const ske_gen_params_t *p, uint64_t start, uint64_t n,
                   uint8_t *bytes_dev, uint32_t *offs_dev, uint32_t *slot_dev);
int ske_gen_id_width(const ske_gen_params_t *p); /* digits per ID */

#ifdef __cplusplus
}
#endif
#endif
