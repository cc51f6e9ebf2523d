// Diagnostic probe: lane/K layout of v_mfma_scale_f32_32x32x64_f8f6f4 with
// fp4 (e2m1) operands on gfx950, checked with exact small-integer data.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <math.h>
#include <stdlib.h>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void k(const uint32_t *a, const uint32_t *b, float *c) {
    int l = threadIdx.x;
    v8i av = {0}, bv = {0};
    for (int i = 0; i < 4; ++i) { av[i] = a[l * 4 + i]; bv[i] = b[l * 4 + i]; }
    v16f acc = {0};
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc, 4, 4, 0, 127, 0, 127);
    for (int r = 0; r < 16; ++r) c[l * 16 + r] = acc[r];
}

static const float E2M1[16] = {0, 0.5f, 1, 1.5f, 2, 3, 4, 6, -0.f, -0.5f, -1, -1.5f, -2, -3, -4, -6};

int main() {
    // A[m][k], B[k][n] as fp4 codes
    static uint8_t A[32][64], B[64][32];
    srand(1);
    for (int m = 0; m < 32; ++m) for (int kk = 0; kk < 64; ++kk) A[m][kk] = rand() & 15;
    for (int kk = 0; kk < 64; ++kk) for (int n = 0; n < 32; ++n) B[kk][n] = rand() & 15;
    double C[32][32];
    for (int m = 0; m < 32; ++m) for (int n = 0; n < 32; ++n) {
        double s = 0; for (int kk = 0; kk < 64; ++kk) s += (double)E2M1[A[m][kk]] * E2M1[B[kk][n]]; C[m][n] = s; }
    // hypothesis: lane l holds A[l&31][32*(l>>5)+j] and B[32*(l>>5)+j][l&31], j = nibble index (dword j/8, bits 4*(j%8))
    uint32_t ha[64 * 4] = {0}, hb[64 * 4] = {0};
    for (int l = 0; l < 64; ++l) for (int j = 0; j < 32; ++j) {
        int kk = 32 * (l >> 5) + j;
        ha[l * 4 + j / 8] |= (uint32_t)A[l & 31][kk] << (4 * (j % 8));
        hb[l * 4 + j / 8] |= (uint32_t)B[kk][l & 31] << (4 * (j % 8));
    }
    uint32_t *da, *db; float *dc;
    hipMalloc(&da, sizeof(ha)); hipMalloc(&db, sizeof(hb)); hipMalloc(&dc, 64 * 16 * 4);
    hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
    k<<<1, 64>>>(da, db, dc);
    float out[64 * 16];
    hipMemcpy(out, dc, sizeof(out), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) for (int r = 0; r < 16; ++r) {
        int n = l & 31, m = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
        if ((double)out[l * 16 + r] != C[m][n]) { if (bad < 5) printf("mismatch lane %d reg %d: got %g want %g\n", l, r, out[l*16+r], C[m][n]); ++bad; }
    }
    printf("fp4 32x32x64 layout hypothesis (A[l&31][32*(l>>5)+j], C row=(r&3)+8*(r>>2)+4*(l>>5), col=l&31): %s (%d mismatches)\n", bad ? "FAIL" : "PASS", bad);
    return bad ? 1 : 0;
}
