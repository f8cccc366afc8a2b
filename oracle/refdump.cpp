// ORACLE — test infrastructure only. Dumps the reference's own GeneticCode tables (compiled in
// place from /root/reference/src/commons/GeneticCode.h by the Makefile's `ref` target) as JSON so
// that tests/golden/genetic_code.json pins the oracle's restated tables (oracle/orc_core.h).
#include <cstdio>
#include <string>
#include <vector>

#include "GeneticCode.h"

int main() {
    GeneticCode gc(false);
    const int codes[5] = {0, 1, 2, 3, 7};
    printf("{\n  \"nuc2aa\": [");
    bool first = true;
    for (int a : codes) for (int b : codes) for (int c : codes) {
        printf("%s[%d,%d,%d,%d]", first ? "" : ",", a, b, c, gc.nuc2aa[a][b][c]);
        first = false;
    }
    printf("],\n  \"nuc2num\": [");
    first = true;
    for (int a : codes) for (int b : codes) for (int c : codes) {
        printf("%s[%d,%d,%d,%d]", first ? "" : ",", a, b, c, gc.nuc2num[a][b][c]);
        first = false;
    }
    printf("],\n  \"atcg\": [");
    for (int i = 0; i < 256; i++) printf("%s%d", i ? "," : "", (int)(unsigned char)gc.atcg[i]);
    printf("],\n  \"iRCT\": [");
    for (int i = 0; i < 256; i++) printf("%s%d", i ? "," : "", (int)(unsigned char)gc.iRCT[i]);
    printf("]\n}\n");
    return 0;
}
