// Diagnostic probe: lane/K layout of v_mfma_i32_32x32x32_i8 on gfx950,
// checked with exact integer data (hypothesis: lane l holds A[l&31][16*(l>>5)+j],
// B[16*(l>>5)+j][l&31], j = byte index 0..15 of its 4 VGPRs; C as the f32 forms).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k(const int *a, const int *b, int *c) {
    int l = threadIdx.x;
    v4i av, bv;
    for (int i = 0; i < 4; ++i) { av[i] = a[l * 4 + i]; bv[i] = b[l * 4 + i]; }
    v16i acc = {0};
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, acc, 0, 0, 0);
    for (int r = 0; r < 16; ++r) c[l * 16 + r] = acc[r];
}

int main() {
    static int8_t A[32][32], B[32][32];
    srand(3);
    for (int m = 0; m < 32; ++m) for (int kk = 0; kk < 32; ++kk) A[m][kk] = (int8_t)(rand() & 255);
    for (int kk = 0; kk < 32; ++kk) for (int n = 0; n < 32; ++n) B[kk][n] = (int8_t)(rand() & 255);
    long C[32][32];
    for (int m = 0; m < 32; ++m) for (int n = 0; n < 32; ++n) { long s = 0; for (int kk = 0; kk < 32; ++kk) s += (long)A[m][kk] * B[kk][n]; C[m][n] = s; }
    int ha[64 * 4] = {0}, hb[64 * 4] = {0};
    for (int l = 0; l < 64; ++l) for (int j = 0; j < 16; ++j) {
        int kk = 16 * (l >> 5) + j;
        ((uint8_t *)ha)[l * 16 + j] = (uint8_t)A[l & 31][kk];
        ((uint8_t *)hb)[l * 16 + j] = (uint8_t)B[kk][l & 31];
    }
    int *da, *db, *dc;
    (void)hipMalloc(&da, sizeof(ha)); (void)hipMalloc(&db, sizeof(hb)); (void)hipMalloc(&dc, 64 * 16 * 4);
    (void)hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice);
    (void)hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
    k<<<1, 64>>>(da, db, dc);
    int out[64 * 16];
    (void)hipMemcpy(out, dc, sizeof(out), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) for (int r = 0; r < 16; ++r) {
        int n = l & 31, m = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
        if (out[l * 16 + r] != C[m][n]) { if (bad < 5) printf("mismatch lane %d reg %d: got %d want %ld\n", l, r, out[l*16+r], C[m][n]); ++bad; }
    }
    printf("i8 32x32x32 layout hypothesis (A[l&31][16*(l>>5)+j]): %s (%d mismatches)\n", bad ? "FAIL" : "PASS", bad);
    return bad ? 1 : 0;
}
