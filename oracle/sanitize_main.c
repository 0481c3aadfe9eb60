/* sanitize_main.c -- TEST INFRASTRUCTURE: the CPU restatement (mas_oracle.c)
 * under AddressSanitizer + UndefinedBehaviorSanitizer (make -C oracle
 * sanitize; tests/test_oracle_sanitize.py).  Reads one case written by the
 * test (little-endian):
 *   int32 nV, nE, nF, nnz, maxLevels, nEF, nEE, nVF, threads
 *   float pos4[nV*4]; int32 starts[nV+1], idx[nnz], edges4[nE*4], faces4[nF*4]
 *   float diag9[nV*9], off9[nnz*9]; bytes ef[nEF*48], ee[nEE*48], vf[nVF*48]
 *   float r4[nV*4]
 * runs Allocate -> Prepare -> Preconditioning and writes z4 to the output
 * file.  Any sanitizer report aborts with a nonzero status. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mas_oracle.h"

static void* rd(FILE* f, size_t bytes) {
    void* p = malloc(bytes ? bytes : 1);
    if (!p || (bytes && fread(p, 1, bytes, f) != bytes)) {
        fprintf(stderr, "short read (%zu bytes)\n", bytes);
        exit(2);
    }
    return p;
}

int main(int argc, char** argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: %s case.bin z.bin\n", argv[0]);
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    int hd[9];
    if (fread(hd, 4, 9, f) != 9) return 2;
    const int nV = hd[0], nE = hd[1], nF = hd[2], nnz = hd[3], L = hd[4], nEF = hd[5], nEE = hd[6], nVF = hd[7];
    float* pos = rd(f, (size_t)nV * 16);
    int* starts = rd(f, (size_t)(nV + 1) * 4);
    int* idx = rd(f, (size_t)nnz * 4);
    int* edges = rd(f, (size_t)nE * 16);
    int* faces = rd(f, (size_t)nF * 16);
    float* diag = rd(f, (size_t)nV * 36);
    float* off = rd(f, (size_t)nnz * 36);
    void* ef = rd(f, (size_t)nEF * 48);
    void* ee = rd(f, (size_t)nEE * 48);
    void* vf = rd(f, (size_t)nVF * 48);
    float* r = rd(f, (size_t)nV * 16);
    fclose(f);
    unsigned* efC = calloc((size_t)nE + 1, 4);
    unsigned* eeC = calloc((size_t)nE + 1, 4);
    unsigned* vfC = calloc((size_t)nV + 1, 4);
    efC[nE] = (unsigned)nEF;
    eeC[nE] = (unsigned)nEE;
    vfC[nV] = (unsigned)nVF;
    orc_state* s = orc_create(nV, nE, nF, L, hd[8]);
    if (!s) return 3;
    int rc = orc_allocate(s, pos, starts, idx, nE ? edges : NULL, nF ? faces : NULL);
    if (!rc) rc = orc_prepare(s, diag, off, starts, nEF ? ef : NULL, nEE ? ee : NULL, nVF ? vf : NULL, efC, eeC, vfC, 0);
    float* z = calloc((size_t)nV * 4, 4);
    if (!rc) rc = orc_apply(s, z, r);
    if (rc) {
        fprintf(stderr, "oracle rc %d\n", rc);
        return 4;
    }
    FILE* o = fopen(argv[2], "wb");
    if (!o || fwrite(z, 16, (size_t)nV, o) != (size_t)nV) return 5;
    fclose(o);
    orc_destroy(s);
    free(pos); free(starts); free(idx); free(edges); free(faces); free(diag); free(off);
    free(ef); free(ee); free(vf); free(r); free(efC); free(eeC); free(vfC); free(z);
    return 0;
}
