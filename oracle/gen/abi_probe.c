/* Prints the byte layout of the boundary types as JSON.
 * Built twice by oracle/gen/make_abi_layout.sh: once against the reference
 * headers (-DREF, /root/reference/SRC) to produce tests/golden/abi_layout.json,
 * and by tests/test_abi.py against include/slu_abi.h.  Test infrastructure. */
#include <stdio.h>
#include <stddef.h>
#ifdef REF
#include "superlu_ddefs.h"
#include "superlu_sdefs.h"
#include "superlu_zdefs.h"
#else
#include "slu_abi.h"
#endif
#include "abi_fields.h"
int main(void) {
    int first = 1;
    printf("{");
#define T(t) printf("%s\"sizeof(%s)\": %zu", first ? "" : ", ", #t, sizeof(t)); first = 0;
    ABI_TYPES(T)
#define F(t, f) printf(", \"%s.%s\": %zu", #t, #f, offsetof(t, f));
    ABI_FIELDS(F)
    printf("}\n");
    return 0;
}
