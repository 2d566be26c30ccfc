// sketch_ingest.hip -- the ingest step before the hot path:
// batched JSON event decode and (lecture_id, day) -> HLL key-slot resolution
// on the device.
//
// The reference decodes one Pulsar payload at a time on the CPU
// (attendance_processor.py:103-106: json.loads, data['student_id'],
// data['lecture_id'], datetime.fromisoformat(data['timestamp'])) and builds
// the HLL key from the lecture id (:128; README.md:105-106 adds the day).
// Here one thread parses one message:
//   - a flat JSON object of ASCII bytes whose keys and string values carry no
//     escapes, values strings / numbers / true / false / null;
//   - student_id an integer literal (its redis-py encoding str(int) is the
//     literal itself; "-0" excluded) or a string;
//   - lecture_id a string or an integer literal;
//   - timestamp "YYYY-MM-DD", optionally followed by one separator character
//     and "HH:MM:SS" with an optional ".fff" / ".ffffff" and an optional
//     "+HH:MM" / "-HH:MM" offset (the forms Python 3.10's fromisoformat reads
//     that this fast path accepts; values range-checked).
// A message outside that fast path is marked for the host, which applies
// Python's own json / datetime semantics to it -- answers are identical
// either way.  For a fast message the kernel emits the id span, the lecture
// span, the UTC day (README key form) and a 128-bit key hash; a device
// open-addressing table maps key hashes to HLL slots (the host inserts keys
// the first time it sees them).
#include "sketch_common.h"
#include "sketch_internal.h"

namespace ske {

namespace {

constexpr uint32_t kMiss = 0xffffffffu;

// byte p of the message (p < end), through a one-word cache
struct Reader {
    const uint8_t *base;
    uint32_t end;
    uint32_t wpos;  // word-aligned position of `word`
    uint64_t word;
    __device__ __forceinline__ uint32_t at(uint32_t p) {
        const uint32_t a = p & ~7u;
        if (a != wpos) {
            // aligned 8-byte loads of the message buffer; the caller's buffer is
            // readable to the next 8-byte boundary past its last message
            word = *reinterpret_cast<const uint64_t *>(base + a);
            wpos = a;
        }
        return uint32_t(word >> ((p & 7) * 8)) & 0xffu;
    }
};

__device__ __forceinline__ bool is_ws(uint32_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
__device__ __forceinline__ bool is_digit(uint32_t c) { return c - '0' < 10u; }

// days since 1970-01-01 of a proleptic Gregorian date (H. Hinnant's days_from_civil)
__device__ __forceinline__ int32_t days_from_civil(int32_t y, uint32_t m, uint32_t d) {
    y -= m <= 2;
    const int32_t era = (y >= 0 ? y : y - 399) / 400;
    const uint32_t yoe = uint32_t(y - era * 400);
    const uint32_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const uint32_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + int32_t(doe) - 719468;
}

__device__ __forceinline__ bool leap(int32_t y) { return (y % 4 == 0 && y % 100 != 0) || y % 400 == 0; }

__device__ __forceinline__ uint32_t num2(Reader &r, uint32_t p, bool &ok) {
    const uint32_t a = r.at(p), b = r.at(p + 1);
    ok = ok && is_digit(a) && is_digit(b);
    return (a - '0') * 10 + (b - '0');
}

// the fast-path ISO timestamp at [s, e) -> UTC day number; false: host
__device__ bool parse_iso(Reader &r, uint32_t s, uint32_t e, int32_t &day) {
    const uint32_t len = e - s;
    bool ok = true;
    if (len < 10) return false;
    const uint32_t y = num2(r, s, ok) * 100 + num2(r, s + 2, ok);
    ok = ok && r.at(s + 4) == '-' && r.at(s + 7) == '-';
    const uint32_t mo = num2(r, s + 5, ok), d = num2(r, s + 8, ok);
    if (!ok || y < 1 || mo < 1 || mo > 12 || d < 1) return false;
    const uint32_t mdays = mo == 2 ? (leap(int32_t(y)) ? 29u : 28u)
                                   : ((mo == 4 || mo == 6 || mo == 9 || mo == 11) ? 30u : 31u);
    if (d > mdays) return false;
    int32_t dd = days_from_civil(int32_t(y), mo, d);
    if (len == 10) {
        day = dd;
        return true;
    }
    // separator (any character), HH:MM:SS
    if (len < 19) return false;
    const uint32_t hh = num2(r, s + 11, ok), mi = num2(r, s + 14, ok), ss = num2(r, s + 17, ok);
    ok = ok && r.at(s + 13) == ':' && r.at(s + 16) == ':';
    if (!ok || hh > 23 || mi > 59 || ss > 59) return false;
    uint32_t p = s + 19;
    if (p < e && r.at(p) == '.') {  // exactly 3 or 6 fraction digits
        uint32_t nd = 0;
        while (p + 1 + nd < e && is_digit(r.at(p + 1 + nd))) nd++;
        if (nd != 3 && nd != 6) return false;
        p += 1 + nd;
    }
    if (p == e) {  // naive: the date as written
        day = dd;
        return true;
    }
    // +HH:MM / -HH:MM: the UTC date of the instant
    if (e - p != 6) return false;
    const uint32_t sg = r.at(p);
    if (sg != '+' && sg != '-') return false;
    const uint32_t oh = num2(r, p + 1, ok), om = num2(r, p + 4, ok);
    ok = ok && r.at(p + 3) == ':';
    if (!ok || oh > 23 || om > 59) return false;
    if (y == 1 || y == 9999) return false;  // a UTC shift may leave the date range: host
    const int64_t local = int64_t(dd) * 86400 + hh * 3600 + mi * 60 + ss;
    const int64_t off = int64_t(oh * 3600 + om * 60) * (sg == '+' ? 1 : -1);
    const int64_t utc = local - off;
    day = int32_t(utc >= 0 ? utc / 86400 : -((-utc + 86399) / 86400));
    return true;
}

// value kinds
enum : uint32_t { kVNone = 0, kVString = 1, kVInt = 2, kVOther = 3 };

}  // namespace

__global__ void __launch_bounds__(256)
    k_ingest_parse(const uint8_t *__restrict__ msgs, const uint32_t *__restrict__ moffs, uint64_t n,
                   int day_form, IngestCols out) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t m = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; m < n; m += stride) {
        const uint32_t s0 = moffs[m], e0 = moffs[m + 1];
        Reader r{msgs, e0, 0xffffffffu, 0};
        bool ok = true;
        // spans of the three fields (last occurrence wins, as in json.loads)
        uint32_t id_s = 0, id_e = 0, id_k = kVNone;
        uint32_t lec_s = 0, lec_e = 0, lec_k = kVNone;
        uint32_t ts_s = 0, ts_e = 0, ts_k = kVNone;
        uint32_t p = s0;
        while (p < e0 && is_ws(r.at(p))) p++;
        ok = p < e0 && r.at(p) == '{';
        p++;
        bool first = true, closed = false;
        while (ok && p < e0) {
            while (p < e0 && is_ws(r.at(p))) p++;
            if (p >= e0) { ok = false; break; }
            uint32_t c = r.at(p);
            if (c == '}' && first) { closed = true; p++; break; }
            if (c != '"') { ok = false; break; }
            // key
            const uint32_t ks = ++p;
            while (p < e0 && (c = r.at(p)) != '"') {
                if (c == '\\' || c < 0x20 || c >= 0x80) ok = false;
                p++;
            }
            if (!ok || p >= e0) { ok = false; break; }
            const uint32_t ke = p++;
            while (p < e0 && is_ws(r.at(p))) p++;
            if (p >= e0 || r.at(p) != ':') { ok = false; break; }
            p++;
            while (p < e0 && is_ws(r.at(p))) p++;
            if (p >= e0) { ok = false; break; }
            // value
            c = r.at(p);
            uint32_t vs = p, ve, kind;
            if (c == '"') {
                vs = ++p;
                while (p < e0 && (c = r.at(p)) != '"') {
                    if (c == '\\' || c < 0x20 || c >= 0x80) ok = false;
                    p++;
                }
                if (!ok || p >= e0) { ok = false; break; }
                ve = p++;
                kind = kVString;
            } else if (c == '-' || is_digit(c)) {
                // -?(0|[1-9][0-9]*) with no fraction / exponent; anything else: host
                uint32_t q = p + (c == '-');
                if (q >= e0 || !is_digit(r.at(q))) { ok = false; break; }
                const bool zero = r.at(q) == '0';
                uint32_t nd = 0;
                while (q < e0 && is_digit(r.at(q))) { q++; nd++; }
                if (zero && nd > 1) { ok = false; break; }
                if (q < e0 && (r.at(q) == '.' || r.at(q) == 'e' || r.at(q) == 'E')) { ok = false; break; }
                if (c == '-' && zero) { ok = false; break; }  // "-0": str(int) is "0"
                ve = p = q;
                kind = kVInt;
            } else if (c == 't' || c == 'f' || c == 'n') {
                const uint32_t L = c == 'f' ? 5 : 4;
                if (p + L > e0) { ok = false; break; }
                const char *lit = c == 't' ? "true" : (c == 'f' ? "false" : "null");
                for (uint32_t i = 0; i < L; i++) ok = ok && r.at(p + i) == uint32_t(lit[i]);
                p += L;
                ve = p;
                kind = kVOther;
            } else {
                ok = false;  // nested object / array, NaN, Infinity, ...: host
                break;
            }
            if (!ok) break;
            // which field
            const uint32_t kl = ke - ks;
            auto key_is = [&](const char *name, uint32_t L) {
                if (kl != L) return false;
                bool eq = true;
                for (uint32_t i = 0; i < L; i++) eq = eq && r.at(ks + i) == uint32_t(name[i]);
                return eq;
            };
            if (key_is("student_id", 10)) { id_s = vs; id_e = ve; id_k = kind; }
            else if (key_is("lecture_id", 10)) { lec_s = vs; lec_e = ve; lec_k = kind; }
            else if (key_is("timestamp", 9)) { ts_s = vs; ts_e = ve; ts_k = kind; }
            first = false;
            while (p < e0 && is_ws(r.at(p))) p++;
            if (p >= e0) { ok = false; break; }
            c = r.at(p++);
            if (c == '}') { closed = true; break; }
            if (c != ',') { ok = false; break; }
        }
        ok = ok && closed;
        while (ok && p < e0) ok = is_ws(r.at(p++));
        // the three fields, fast-path kinds only
        ok = ok && (id_k == kVInt || id_k == kVString) && (lec_k == kVString || lec_k == kVInt) &&
             ts_k == kVString;
        int32_t day = 0;
        if (ok && day_form) ok = parse_iso(r, ts_s, ts_e, day);
        else if (ok) {
            int32_t dummy;
            ok = parse_iso(r, ts_s, ts_e, dummy);  // fromisoformat must still accept it
        }
        out.status[m] = ok ? 0 : 1;
        out.id_start[m] = id_s;
        out.id_len[m] = ok ? id_e - id_s : 0;
        out.lec_start[m] = lec_s;
        out.lec_len[m] = lec_e - lec_s;
        out.ts_start[m] = ts_s;
        out.ts_len[m] = ts_e - ts_s;
        out.day[m] = day;
        // key hash: MurmurHash64A of the lecture bytes under two seeds, each
        // mixed with the day (the key string is prefix + lecture [+ ':' + day],
        // an injective function of (lecture bytes, day))
        uint64_t h0 = 0, h1 = 0;
        if (ok) {
            const Item it = load_item(msgs, lec_s, lec_e);
            const uint64_t dz = uint64_t(uint32_t(day_form ? day : 0));
            h0 = murmur_item(it, 0x9e3779b97f4a7c15ULL) ^ splitmix_fin(dz + 0x632be59bd9b4e019ULL);
            h1 = murmur_item(it, 0xc2b2ae3d27d4eb4fULL) ^ splitmix_fin(dz ^ 0x85ebca6b27d4eb2fULL);
            h0 |= 1;  // 0 marks an empty table entry
        }
        out.kh[2 * m] = h0;
        out.kh[2 * m + 1] = h1;
    }
}

// key table: open addressing on kh0, linear probing; capacity a power of two
__global__ void __launch_bounds__(256)
    k_keytab_insert(uint64_t *__restrict__ tk, uint32_t *__restrict__ tslot, uint64_t mask,
                    const uint64_t *__restrict__ kh, const uint32_t *__restrict__ slots, uint64_t n) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t k0 = kh[2 * i], k1 = kh[2 * i + 1];
        if (k0 == 0) continue;  // an empty entry of a table being rehashed
        for (uint64_t h = k0 & mask;; h = (h + 1) & mask) {
            const unsigned long long prev = atomicCAS(reinterpret_cast<unsigned long long *>(tk + 2 * h),
                                                      0ull, (unsigned long long)k0);
            if (prev == 0) {
                tk[2 * h + 1] = k1;
                tslot[h] = slots[i];
                break;
            }
        }
    }
}

// slot of every decoded message's key (kMiss: not in the table) and, for the
// dense K1 batch, its take flag and id length
__global__ void __launch_bounds__(256)
    k_keytab_lookup(const uint64_t *__restrict__ tk, const uint32_t *__restrict__ tslot,
                    uint64_t mask, const uint64_t *__restrict__ kh,
                    const uint8_t *__restrict__ status, const uint32_t *__restrict__ id_len,
                    uint64_t n, uint32_t *__restrict__ slot, uint32_t *__restrict__ flag,
                    uint32_t *__restrict__ mlen) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint32_t s = kMiss;
        if (status[i] == 0 && tk) {
            const uint64_t k0 = kh[2 * i], k1 = kh[2 * i + 1];
            for (uint64_t h = k0 & mask;; h = (h + 1) & mask) {
                const uint64_t t0 = tk[2 * h];
                if (t0 == 0) break;
                if (t0 == k0 && tk[2 * h + 1] == k1) {
                    s = tslot[h];
                    break;
                }
            }
        }
        slot[i] = s;
        flag[i] = s != kMiss;
        mlen[i] = s != kMiss ? id_len[i] : 0;
    }
}

// fast messages with a slot -> dense K1 batch: ids packed at pos[m] (exclusive
// scan of their lengths), slots at rank[m] (exclusive scan of the flags)
__global__ void __launch_bounds__(256)
    k_ingest_pack(const uint8_t *__restrict__ msgs, const IngestCols c, const uint32_t *__restrict__ slot,
                  const uint32_t *__restrict__ flag_incl, const uint32_t *__restrict__ len_incl,
                  uint64_t n, uint8_t *__restrict__ ids, uint32_t *__restrict__ ids_offs,
                  uint32_t *__restrict__ kslot) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t m = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; m < n; m += stride) {
        const uint32_t take = c.status[m] == 0 && slot[m] != kMiss;
        const uint32_t len = take ? c.id_len[m] : 0;
        const uint32_t r = flag_incl[m] - take, pos = len_incl[m] - len;
        if (take) {
            for (uint32_t j = 0; j < len; j++) ids[pos + j] = msgs[c.id_start[m] + j];
            ids_offs[r] = pos;
            kslot[r] = slot[m];
        }
        if (m == n - 1) ids_offs[flag_incl[m]] = len_incl[m];
    }
}

// K1 answers of the dense batch back to message order
__global__ void __launch_bounds__(256)
    k_ingest_unpack(const IngestCols c, const uint32_t *__restrict__ slot,
                    const uint32_t *__restrict__ flag_incl, const uint8_t *__restrict__ kvalid,
                    uint64_t n, uint8_t *__restrict__ valid) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t m = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; m < n; m += stride) {
        const bool take = c.status[m] == 0 && slot[m] != kMiss;
        valid[m] = take ? kvalid[flag_incl[m] - 1] : 0;
    }
}

static inline unsigned grid_for(uint64_t n, unsigned block, unsigned cap) {
    uint64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    return unsigned(g < cap ? g : cap);
}

hipError_t launch_ingest_parse(const uint8_t *msgs, const uint32_t *moffs, uint64_t n, int day_form,
                               const IngestCols &out, int cus, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_ingest_parse, dim3(grid_for(n, 256, cus * 16)), dim3(256), 0, st, msgs, moffs,
                       n, day_form, out);
    return hipGetLastError();
}

hipError_t launch_keytab_insert(uint64_t *tk, uint32_t *tslot, uint64_t mask, const uint64_t *kh,
                                const uint32_t *slots, uint64_t n, int cus, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_keytab_insert, dim3(grid_for(n, 256, cus * 16)), dim3(256), 0, st, tk, tslot,
                       mask, kh, slots, n);
    return hipGetLastError();
}

hipError_t launch_keytab_lookup(const uint64_t *tk, const uint32_t *tslot, uint64_t mask,
                                const uint64_t *kh, const uint8_t *status, const uint32_t *id_len,
                                uint64_t n, uint32_t *slot, uint32_t *flag, uint32_t *mlen, int cus,
                                hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_keytab_lookup, dim3(grid_for(n, 256, cus * 16)), dim3(256), 0, st, tk, tslot,
                       mask, kh, status, id_len, n, slot, flag, mlen);
    return hipGetLastError();
}

hipError_t launch_ingest_pack(const uint8_t *msgs, const IngestCols &c, const uint32_t *slot,
                              const uint32_t *flag_incl, const uint32_t *len_incl, uint64_t n,
                              uint8_t *ids, uint32_t *ids_offs, uint32_t *kslot, int cus,
                              hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_ingest_pack, dim3(grid_for(n, 256, cus * 16)), dim3(256), 0, st, msgs, c, slot,
                       flag_incl, len_incl, n, ids, ids_offs, kslot);
    return hipGetLastError();
}

hipError_t launch_ingest_unpack(const IngestCols &c, const uint32_t *slot, const uint32_t *flag_incl,
                                const uint8_t *kvalid, uint64_t n, uint8_t *valid, int cus,
                                hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_ingest_unpack, dim3(grid_for(n, 256, cus * 16)), dim3(256), 0, st, c, slot,
                       flag_incl, kvalid, n, valid);
    return hipGetLastError();
}

}  // namespace ske
