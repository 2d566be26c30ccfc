// Host-side check of the exact probe arithmetic in sketch_common.h:
// fastmod (Granlund-Montgomery) vs %, and ProbeCursor stepping vs the
// direct RedisBloom formula (a + i*b) mod 2^64 mod bits.  Built by
// tests/test_native_host.py with hipcc (host code only, no GPU needed).
#include <cstdio>
#include <cstdint>
#include <vector>
#include "../../real-time-student-attendance-system_amd/csrc/sketch_common.h"

static uint64_t s = 0x12345678abcdefULL;
static uint64_t rnd() { s = ske::splitmix_fin(s + 0x9e3779b97f4a7c15ULL); return s; }

int main() {
    std::vector<uint64_t> divs = {64, 128, 1152, 2496, 5568, 12288, 1102784, 158202880,
                                  (1ULL << 31), (1ULL << 31) - 64, 3019840,
                                  (1ULL << 32), (1ULL << 32) + 64, 3ULL << 40, (1ULL << 62) + 64};
    for (int i = 0; i < 200; i++) divs.push_back(64 * (1 + rnd() % (1ULL << 30)));
    for (int i = 0; i < 50; i++) divs.push_back(2 + rnd() % (1ULL << 61));
    long bad = 0, checks = 0;
    for (uint64_t d : divs) {
        ske::Divisor D = ske::make_divisor(d);
        std::vector<uint64_t> ns = {0, 1, d - 1, d, d + 1, 2 * d - 1, ~0ULL, ~0ULL - 1, 1ULL << 63,
                                    (1ULL << 63) - 1, ~0ULL - (~0ULL % d), ~0ULL - (~0ULL % d) - 1};
        for (int i = 0; i < 2000; i++) ns.push_back(rnd());
        for (uint64_t n : ns) {
            checks++;
            if (ske::fastmod(n, D) != n % d) {
                if (bad++ < 5) printf("fastmod mismatch d=%llu n=%llu\n", (unsigned long long)d, (unsigned long long)n);
            }
        }
        if (D.t != (uint64_t)((((unsigned __int128)1) << 64) % d)) bad++;
        for (int t = 0; t < 200; t++) {
            uint64_t a = rnd(), b = rnd();
            if (t == 0) { a = ~0ULL; b = ~0ULL; }
            if (t == 1) { a = 0; b = 0; }
            ske::ProbeCursor c;
            c.init(a, b, D);
            for (uint64_t i = 0; i < 40; i++) {
                checks++;
                uint64_t want = (a + i * b) % d;
                if (c.x != want) {
                    if (bad++ < 5) printf("cursor mismatch d=%llu i=%llu\n", (unsigned long long)d, (unsigned long long)i);
                    break;
                }
                c.step(D);
            }
            if (d <= (1ULL << 31)) {  // the 32-bit cursor of the LDS / small-filter path
                ske::ProbeCursor32 c32;
                c32.init(a, b, D);
                for (uint64_t i = 0; i < 40; i++) {
                    checks++;
                    if (c32.x != (a + i * b) % d) {
                        if (bad++ < 5) printf("cursor32 mismatch d=%llu i=%llu\n", (unsigned long long)d, (unsigned long long)i);
                        break;
                    }
                    c32.step(D);
                }
                ske::ProbeWalk32 w32;  // precomputed-increment walk (LDS K1)
                w32.init(a, b, D);
                for (uint64_t i = 0; i < 40; i++) {
                    checks++;
                    if (w32.x != (a + i * b) % d) {
                        if (bad++ < 5) printf("walk32 mismatch d=%llu i=%llu\n", (unsigned long long)d, (unsigned long long)i);
                        break;
                    }
                    w32.step(uint32_t(D.d));
                }
            }
        }
    }
    // hll_patlen vs its definition
    for (int i = 0; i < 100000; i++) {
        uint64_t h = rnd();
        if (i == 0) h = 0;
        uint32_t idx, rank;
        ske::hll_patlen(h, idx, rank);
        uint64_t w = h >> 14; int cnt = 1; uint64_t bit = 1;
        w |= 1ULL << 50;
        while ((w & bit) == 0) { cnt++; bit <<= 1; }
        checks++;
        if (idx != (h & 16383) || (int)rank != cnt) bad++;
    }
    printf("checks=%ld bad=%ld\n", checks, bad);
    return bad ? 1 : 0;
}
