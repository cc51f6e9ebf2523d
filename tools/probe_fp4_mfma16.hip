// Diagnostic probe: lane/K layout of v_mfma_scale_f32_16x16x128_f8f6f4 with
// fp4 (e2m1) operands on gfx950, checked with exact small-integer data, and the
// v_permlane16_swap row exchange used to regroup 32-record tiles into 16-record
// column blocks.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void k(const uint32_t *a, const uint32_t *b, float *c) {
    int l = threadIdx.x;
    v8i av = {0}, bv = {0};
    for (int i = 0; i < 4; ++i) {
        av[i] = a[l * 4 + i];
        bv[i] = b[l * 4 + i];
    }
    v4f acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, 4, 4, 0, 127, 0, 127);
    for (int r = 0; r < 4; ++r) c[l * 4 + r] = acc[r];
}

__global__ void swapk(const uint32_t *x, const uint32_t *y, uint32_t *ox, uint32_t *oy) {
    int l = threadIdx.x;
    auto r = __builtin_amdgcn_permlane16_swap(x[l], y[l], false, false);
    ox[l] = r[0];
    oy[l] = r[1];
}

static const float E2M1[16] = {0, 0.5f, 1, 1.5f, 2, 3, 4, 6, -0.f, -0.5f, -1, -1.5f, -2, -3, -4, -6};

int main() {
    static uint8_t A[16][128], B[128][16];
    srand(1);
    for (int m = 0; m < 16; ++m)
        for (int kk = 0; kk < 128; ++kk) A[m][kk] = rand() & 15;
    for (int kk = 0; kk < 128; ++kk)
        for (int n = 0; n < 16; ++n) B[kk][n] = rand() & 15;
    double C[16][16];
    for (int m = 0; m < 16; ++m)
        for (int n = 0; n < 16; ++n) {
            double s = 0;
            for (int kk = 0; kk < 128; ++kk) s += (double)E2M1[A[m][kk]] * E2M1[B[kk][n]];
            C[m][n] = s;
        }
    // hypothesis: lane l holds A[l&15][32*(l>>4)+j] and B[32*(l>>4)+j][l&15], j = nibble index
    uint32_t ha[64 * 4] = {0}, hb[64 * 4] = {0};
    for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 32; ++j) {
            int kk = 32 * (l >> 4) + j;
            ha[l * 4 + j / 8] |= (uint32_t)A[l & 15][kk] << (4 * (j % 8));
            hb[l * 4 + j / 8] |= (uint32_t)B[kk][l & 15] << (4 * (j % 8));
        }
    uint32_t *da, *db;
    float *dc;
    (void)hipMalloc(&da, sizeof(ha));
    (void)hipMalloc(&db, sizeof(hb));
    (void)hipMalloc(&dc, 64 * 4 * 4);
    (void)hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice);
    (void)hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
    k<<<1, 64>>>(da, db, dc);
    float out[64 * 4];
    (void)hipMemcpy(out, dc, sizeof(out), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r) {
            int n = l & 15, m = r + 4 * (l >> 4);
            if ((double)out[l * 4 + r] != C[m][n]) {
                if (bad < 5) printf("mismatch lane %d reg %d: got %g want %g\n", l, r, out[l * 4 + r], C[m][n]);
                ++bad;
            }
        }
    printf("fp4 16x16x128 layout hypothesis (A[l&15][32*(l>>4)+j], C row=r+4*(l>>4), col=l&15): %s (%d mismatches)\n",
           bad ? "FAIL" : "PASS", bad);

    // permlane16_swap: expected ox = x with odd rows replaced by y's even rows, oy = y's even rows replaced
    uint32_t hx[64], hy[64], rx[64], ry[64];
    for (int l = 0; l < 64; ++l) {
        hx[l] = 1000 + l;
        hy[l] = 2000 + l;
    }
    uint32_t *dx, *dy, *dox, *doy;
    (void)hipMalloc(&dx, 256);
    (void)hipMalloc(&dy, 256);
    (void)hipMalloc(&dox, 256);
    (void)hipMalloc(&doy, 256);
    (void)hipMemcpy(dx, hx, 256, hipMemcpyHostToDevice);
    (void)hipMemcpy(dy, hy, 256, hipMemcpyHostToDevice);
    swapk<<<1, 64>>>(dx, dy, dox, doy);
    (void)hipMemcpy(rx, dox, 256, hipMemcpyDeviceToHost);
    (void)hipMemcpy(ry, doy, 256, hipMemcpyDeviceToHost);
    int sbad = 0;
    for (int l = 0; l < 64; ++l) {
        const int row = l >> 4, j = l & 15;
        const uint32_t ex = (row & 1) ? hy[(row - 1) * 16 + j] : hx[l];
        const uint32_t ey = (row & 1) ? hy[l] : hx[(row + 1) * 16 + j];
        if (rx[l] != ex || ry[l] != ey) {
            if (sbad < 5) printf("swap lane %d: got (%u,%u) want (%u,%u)\n", l, rx[l], ry[l], ex, ey);
            ++sbad;
        }
    }
    printf("permlane16_swap hypothesis (x odd rows <-> y even rows): %s (%d mismatches)\n", sbad ? "FAIL" : "PASS",
           sbad);
    return bad || sbad ? 1 : 0;
}
