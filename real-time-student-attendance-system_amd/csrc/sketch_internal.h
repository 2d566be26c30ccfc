// sketch_internal.h -- launcher declarations shared by the libsketch TUs.
#pragma once
#include "sketch_common.h"

namespace ske {

// sketch_kernels.hip
hipError_t launch_swipes(int mode, const ChainDev &ch, bool lds, int tile, const uint8_t *bytes,
                         const uint32_t *offs, uint32_t fixed_w, const uint32_t *slot, uint64_t n,
                         uint8_t *regs,
                         uint32_t nslots, uint8_t *out, unsigned long long *stats, int cus,
                         hipStream_t st);
hipError_t lds_bloom_setup();
hipError_t set_stamp_buffer(void *p);  // -DSKE_STAMPS diagnostic build only
uint32_t lds_bloom_max();
hipError_t launch_pfadd(const uint32_t *slot, const uint8_t *bytes, const uint32_t *offs,
                        uint64_t n, uint8_t *regs, uint32_t nslots, unsigned int *err, int cus,
                        hipStream_t st);
hipError_t launch_pfcount(const uint8_t *regs, const uint32_t *slots, const uint32_t *goffs,
                          uint32_t ngroups, const double *tau, const double *sig, uint64_t *out,
                          int cus, hipStream_t st);
hipError_t launch_histogram(const uint8_t *regs, uint32_t *out64, hipStream_t st);
hipError_t launch_pfmerge(uint8_t *regs, uint32_t dst, const uint32_t *srcs, uint32_t n,
                          hipStream_t st);
uint32_t pfmerge_partitions(uint32_t n, int cus, uint32_t *per);
hipError_t launch_pfmerge_wide(uint8_t *regs, uint32_t dst, const uint32_t *srcs, uint32_t n,
                               uint8_t *partial, uint32_t per, uint32_t P, hipStream_t st);
hipError_t launch_slots_max(const uint32_t *slots, uint64_t n, unsigned int *out, int cus, hipStream_t st);
hipError_t launch_merge_groups(const uint8_t *regs, const uint32_t *slots, const uint32_t *goffs,
                               uint32_t ngroups, uint8_t *dst, int cus, hipStream_t st);
hipError_t launch_dense(const uint8_t *regs, uint8_t *dense, hipStream_t st);
hipError_t launch_gen_swipes(const GenDev &g, uint64_t start, uint64_t n, uint8_t *bytes,
                             uint32_t *offs, uint32_t *slot, int cus, hipStream_t st);
hipError_t launch_gen_members(const GenDev &g, uint64_t start, uint64_t n, uint8_t *bytes,
                              uint32_t *offs, int cus, hipStream_t st);

// sketch_k1.hip -- K1 for chains that fit the LDS image, short-id fast path
constexpr int kK1MaxLinks = 8;
constexpr int kLdsBloomMaxBytes = 152 * 1024;  // LDS image budget (160 KiB per CU)

struct K1Link {
    const uint8_t *bf;   // device bit array (readable to nbytes16)
    uint64_t m;          // Granlund-Montgomery magic of d
    uint32_t d;          // bloom->bits (<= 2^31)
    uint32_t t;          // 2^64 mod d
    uint32_t sh;         // l - 1 of the magic
    uint32_t k;          // bloom->hashes
    uint32_t nbytes16;   // bloom->bytes rounded up to 16
    uint32_t piece0;     // first 1 KiB LDS piece of the link (LDS offset piece0 * 1024)
};

struct K1Args {
    const uint8_t *bytes;
    const uint32_t *offs;   // nullptr: fixed-width ids (fixed_w bytes each)
    const uint32_t *slot;
    uint8_t *regs;
    uint8_t *out;           // may be nullptr
    unsigned int *err;      // set when a valid swipe names a slot >= nslots
    const uint8_t *zero16;  // 16 readable zero bytes (load address of empty ids)
    uint32_t n, nslots, fixed_w, nlinks, npieces;
    K1Link link[kK1MaxLinks];
};

// ske_swipes_many_async through the short-id LDS K1: one persistent launch over
// up to kK1ManyMax batches (passed by value: the kernel arguments are captured
// with a graph), tpre[j] = tiles of the batches before j
constexpr uint32_t kK1ManyMax = 48;
struct K1Batch {
    const uint8_t *bytes;
    const uint32_t *offs;  // nullptr: fixed-width ids
    const uint32_t *slot;
    uint8_t *out;          // may be nullptr
    uint32_t n, fixed_w;
};
struct K1Many {
    K1Batch b[kK1ManyMax];
    uint32_t tpre[kK1ManyMax + 1];
    uint32_t nb;
};
uint32_t k1_many_tile(int tile);  // swipes per tile of the many kernel
hipError_t launch_swipes_lds_many(const K1Args &A, const K1Many &M, int tile, int cus, hipStream_t st);

// sketch_route.hip -- unpartitioned swipes to their key owners (alltoallv halves)
hipError_t launch_route(const uint8_t *ids, uint32_t width, const uint32_t *slot, uint64_t n, uint32_t world,
                        const uint32_t *kown, const uint32_t *kloc, uint32_t nkeys, uint8_t *sids,
                        uint32_t *sslot, uint32_t *pos, uint32_t *hist, uint32_t *tot, hipStream_t st);
uint64_t route_hist_words(uint64_t n, uint32_t world);
// out (device) = answers in[0..n) packed 1 bit per swipe, LSB first; in must be 8-B aligned
hipError_t launch_pack_bits(const uint8_t *in, uint64_t n, uint8_t *out, int cus, hipStream_t st);
hipError_t launch_route_cap(const uint8_t *ids, uint32_t width, const uint32_t *slot, uint64_t n, uint32_t world,
                            const uint32_t *kroute, uint32_t nkeys, uint32_t cap, const uint32_t *sink, uint8_t *sids,
                            uint32_t *sslot, uint32_t *pos, uint32_t *hist, uint32_t *tot, int cus, hipStream_t st);
hipError_t launch_route_return(const uint8_t *ans, const uint32_t *pos, uint64_t n, uint8_t *out, int cus,
                               hipStream_t st);
hipError_t launch_route_slots(const uint32_t *gkey, uint64_t n, const uint32_t *kroute, uint32_t nkeys,
                              uint32_t world, uint32_t *out, int cus, hipStream_t st);

// fills A's chain fields; false when the chain does not fit this variant
bool k1_lds_plan(const ChainDev &ch, K1Args *A);
hipError_t launch_swipes_lds(const K1Args &A, bool hll, int tile, int cus, hipStream_t st);
hipError_t k1_lds_setup();
hipError_t set_k1_stamp_buffer(void *p);  // -DSKE_STAMPS diagnostic build only
hipError_t set_pb_stamp_buffer(void *p);  // -DSKE_STAMPS diagnostic build only
hipError_t set_seg_stamp_buffer(void *p);  // -DSKE_SEG_STAMPS diagnostic build only

// sketch_ingest.hip -- JSON event decode and key-slot resolution (device columns)
struct IngestCols {
    uint8_t *status;  // 0 decoded on the device, 1 for the host
    uint32_t *id_start, *id_len, *lec_start, *lec_len, *ts_start, *ts_len;
    int32_t *day;     // UTC day number (README key form)
    uint64_t *kh;     // 2 per message: key hash
};
hipError_t launch_ingest_parse(const uint8_t *msgs, const uint32_t *moffs, uint64_t n, int day_form,
                               const IngestCols &out, int cus, hipStream_t st);
hipError_t launch_keytab_insert(uint64_t *tk, uint32_t *tslot, uint64_t mask, const uint64_t *kh,
                                const uint32_t *slots, uint64_t n, int cus, hipStream_t st);
hipError_t launch_keytab_lookup(const uint64_t *tk, const uint32_t *tslot, uint64_t mask,
                                const uint64_t *kh, const uint8_t *status, const uint32_t *id_len,
                                uint64_t n, uint32_t *slot, uint32_t *flag, uint32_t *mlen, int cus,
                                hipStream_t st);
hipError_t launch_ingest_pack(const uint8_t *msgs, const IngestCols &c, const uint32_t *slot,
                              const uint32_t *flag_incl, const uint32_t *len_incl, uint64_t n,
                              uint8_t *ids, uint32_t *ids_offs, uint32_t *kslot, int cus,
                              hipStream_t st);
hipError_t launch_ingest_unpack(const IngestCols &c, const uint32_t *slot, const uint32_t *flag_incl,
                                const uint8_t *kvalid, uint64_t n, uint8_t *valid, int cus,
                                hipStream_t st);

// sketch_xr.hip -- XCD-partitioned K1 for chains larger than the LDS image
bool xr_supported(const ChainDev &ch);
uint64_t xr_scratch_bytes(uint64_t n, int nlinks);
hipError_t launch_swipes_xr(const ChainDev &ch, const uint8_t *bytes, const uint32_t *offs,
                            uint32_t fixed_w, const uint32_t *slot, uint64_t n, uint8_t *regs,
                            uint32_t nslots, uint8_t *out, void *scratch, unsigned int *err,
                            int cus, int region_u, int finish_u, hipStream_t st);

// sketch_part.hip -- partitioned K1 (probe records routed to LDS-resident
// 64 KiB slices of each link) for chains larger than the LDS image
constexpr int kPSliceLog = 19;
constexpr uint32_t kPSliceBits = 1u << kPSliceLog;
constexpr uint32_t kPMaxSlices = 2047;
constexpr int kPMaxLinks = 8;
struct Scratch;
bool part_supported(const ChainDev &ch);
// The segmented PFADD (k_seg_*, the pass C of one-link chains when a batch's
// register updates are dense in the slab) -- options "hll_seg" (mode),
// "seg_density" and "seg_dense_min" (x100), "seg_klog".
struct SegOpts {
    int mode = -1;                  // -1 auto, 0 never (pass C), 1 whenever the chain and slab allow
    uint32_t density_x100 = 600;    // auto: a batch's swipes per 128-B line of the slab, x100 (x2 when the
                                    // slab fits the Infinity Cache, where pass C's random requests are cheaper)
    uint32_t dense_min_x100 = 100;  // a window is staged in LDS from this many records per line, x100
    int klog = 1;                   // keys per window: 2^klog (16 KiB each; 0..3)
    // option "rec_groups": pass A's probe records in the group layout (a
    // unit's runs of 8 tiles adjacent; one-link k = 11 chains under 1024
    // slices): 1 whenever the chain allows; -1 auto and 0: per-tile runs
    // (the group layout costs pass A more than it saves pass B)
    int rec_groups = -1;
    int b1 = -1;  // option "seg_b1": 2^b1 level-1 buckets (-1: auto, seg_plan)
};
// sizes the context scratch for batches of up to n swipes (no launch)
// sub: swipes per sub-batch of the three passes (0: the default, 2^25 = kPSubDefault)
hipError_t part_reserve(const ChainDev &ch, uint64_t n, uint32_t sub, uint32_t nslots, const SegOpts &so,
                        Scratch *scr);
// hook (may be null): called as hook(user, pass, 0) right before and
// hook(user, pass, 1) right after each pass's launch (pass 0..4 = A, B, C or
// the segmented C1, the segmented level-2 sort, the segmented window apply)
typedef void (*PassHook)(void *user, int pass, int end, hipStream_t st);
struct PartBatch {
    const uint8_t *bytes;
    const uint32_t *offs;  // nullptr: fixed-width ids
    uint32_t fixed_w;
    const uint32_t *slot;
    uint64_t n;
    uint8_t *out;          // may be nullptr
};
// every pass of every (batch, sub-batch) unit on st, in order
hipError_t launch_swipes_part(const ChainDev &ch, const PartBatch *bt, uint32_t nb, uint8_t *regs,
                              uint32_t nslots, Scratch *scr, unsigned int *err, int cus, uint32_t sub,
                              const SegOpts &so, hipStream_t st, PassHook hook = nullptr,
                              void *hook_user = nullptr);


// sketch_order.hip -- order-exact paths (replies that depend on item order)
struct Scratch;  // growable device scratch, owned by the context
constexpr int kScratchSlots = 48;
void *scratch_get(Scratch *s, int slot, size_t bytes, hipError_t *err);
void scratch_set_recording(Scratch *s, bool on);  // slots handed out now get pinned
void scratch_unpin(Scratch *s);                    // every graph freed: slots may grow

// PFADD with per-element "changed" flags in sequential order.
hipError_t pfadd_exact(Scratch *s, const uint32_t *slot, const uint8_t *bytes,
                       const uint32_t *offs, uint64_t n, uint8_t *regs, uint32_t nslots,
                       uint8_t *changed_dev, unsigned int *err_dev, int cus, hipStream_t st);

// BF.MADD helpers (the epoch driver lives in the API TU, which owns links)
hipError_t launch_bf_hash(const uint8_t *bytes, const uint32_t *offs, uint64_t n, uint64_t *ha,
                          uint64_t *hb, int cus, hipStream_t st);
// items with state==0 that are present in any of ch's links: state=1, res=0
hipError_t launch_bf_settle_present(const ChainDev &ch, uint64_t n, const uint64_t *ha,
                                    const uint64_t *hb, uint8_t *state, int8_t *res, int cus,
                                    hipStream_t st);
hipError_t launch_bf_first_setter(const LinkDev &L, uint64_t n, const uint64_t *ha,
                                  const uint64_t *hb, const uint8_t *state, uint32_t *first,
                                  int cus, hipStream_t st);
hipError_t launch_bf_absent(const LinkDev &L, uint64_t n, const uint64_t *ha, const uint64_t *hb,
                            const uint8_t *state, const uint32_t *first, uint32_t *absent,
                            int cus, hipStream_t st);
hipError_t scan_inclusive_u32(Scratch *s, const uint32_t *in, uint32_t *out, uint64_t n,
                              hipStream_t st);
// resolve candidates with index <= cutoff; absent ones are added (bits set)
hipError_t launch_bf_resolve(const LinkDev &L, uint64_t n, const uint64_t *ha, const uint64_t *hb,
                             uint8_t *state, const uint32_t *absent, const uint32_t *pos,
                             uint32_t cap, int8_t *res, uint8_t *bf_mut, int cus,
                             hipStream_t st);
// mark every remaining candidate with a result code (non-scaling full)
hipError_t launch_bf_fill_rest(uint64_t n, uint8_t *state, int8_t *res, int8_t code, int cus,
                               hipStream_t st);

// host -> device staging of pageable caller buffers (sketch_host.cpp)
struct HostStager;
HostStager *stager_new();
void stager_delete(HostStager *s);
hipError_t stage_h2d(HostStager *s, void *dst, const void *src, size_t bytes, hipStream_t st, bool mono,
                     bool *ok);

}  // namespace ske
