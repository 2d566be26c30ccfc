/* Self-test driver for the oracle under ASan + UBSan (tests/test_oracle_sanitize.py).
 * Exercises every routine with ragged inputs; exits non-zero on a KAT miss. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "sketch_oracle.h"

int main(void) {
    int bad = 0;
    if (orc_smhasher_verification() != 0x1F0D3804u) bad++;
    uint8_t *regs = calloc(ORC_HLL_REGISTERS, 1), *r2 = calloc(ORC_HLL_REGISTERS, 1);
    const char *e[] = {"a", "b", "c", "d", "e", "f", "g"};
    for (int i = 0; i < 7; i++) orc_hll_add(regs, (const uint8_t *)e[i], 1);
    if (orc_hll_count(regs) != 7) bad++;
    uint8_t buf[300];
    for (int i = 0; i < 300; i++) buf[i] = (uint8_t)(i * 37 + 11);
    for (int len = 0; len < 300; len++) orc_hll_add(r2, buf, (size_t)len);
    orc_hll_merge(regs, r2);
    uint8_t dense[ORC_HLL_DENSE_BYTES], back[ORC_HLL_REGISTERS];
    orc_hll_dense_encode(regs, dense);
    orc_hll_dense_decode(dense, back);
    if (memcmp(back, regs, ORC_HLL_REGISTERS)) bad++;
    orc_chain *c = orc_chain_new(100, 0.01, ORC_BLOOM_OPT_FORCE64 | ORC_BLOOM_OPT_NOROUND, 2);
    char id[32];
    for (int i = 0; i < 3000; i++) {
        int n = snprintf(id, sizeof id, "%d", 10000 + i);
        orc_chain_add(c, id, (size_t)n);
    }
    if (orc_chain_nlinks(c) < 5) bad++;
    for (int i = 0; i < 3000; i++) {
        int n = snprintf(id, sizeof id, "%d", 10000 + i);
        if (!orc_chain_check(c, id, (size_t)n, NULL)) bad++;
    }
    orc_chain_free(c);
    free(regs);
    free(r2);
    printf("selftest bad=%d\n", bad);
    return bad != 0;
}
