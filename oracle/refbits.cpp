// ORACLE — test infrastructure only. Prints what the reference's own BitManipulateMacros.h (compiled
// in place from /root/reference/src/commons by the Makefile's `ref` target, no copy, no stand-ins)
// extracts: GET_3_BITS of every 9-bit value (the codon field getHammingDistanceSum / getHammings
// read, KmerMatcher.h:348-416) and the 2-bit field macros, as JSON for tests/golden/make_ref_tables.py.
#include <cstdio>

#include "BitManipulateMacros.h"

int main() {
    printf("{\"get3\": [");
    for (unsigned x = 0; x < 512; x++) printf("%s%u", x ? "," : "", (unsigned)GET_3_BITS(x));
    printf("], \"get2\": [");
    for (unsigned x = 0; x < 16; x++) printf("%s%d", x ? "," : "", (int)GET_2_BITS(x));
    printf("], \"get15\": [%u, %u], \"is_last\": [%u, %u]}\n", (unsigned)GET_15_BITS(0xFFFFu), (unsigned)GET_15_BITS(0x1234u),
           (unsigned)IS_LAST_15_BITS(0x8001u), (unsigned)IS_LAST_15_BITS(0x7FFFu));
    return 0;
}
