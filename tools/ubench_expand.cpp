// Host expansion of packed MasksEngine rows (csrc/iris_host.cpp expand_avx512): plain 64-B
// stores vs 32-record blocks staged in L1 and written with non-temporal stores, one thread,
// 5000-record calls (a quarter of a 20k chunk: the copy-out's share per thread) into a 186-MB
// array (3M records of [u16; 31]).  g++ -O3 -o tools/ubench_expand tools/ubench_expand.cpp
#include <immintrin.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include <chrono>
#include <vector>
constexpr int kRot=31;
__attribute__((target("avx512bw,avx512vl"))) void expand_plain(uint16_t *out, const uint8_t *pk, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        const uint8_t *p = pk + 32 * i; uint32_t b = p[31];
        const __m512i w = _mm512_add_epi16(_mm512_cvtepu8_epi16(_mm256_loadu_si256((const __m256i *)p)), _mm512_set1_epi16((short)(b << 6)));
        if (i + 1 < n) _mm512_storeu_si512((void *)(out + kRot * i), w); else _mm512_mask_storeu_epi16(out + kRot * i, 0x7FFFFFFFu, w);
    }
}
// NT: head records plain until the record start is 64B-aligned, then 32-record blocks via L1 staging + stream stores
__attribute__((target("avx512bw,avx512vl"))) void expand_nt(uint16_t *out, const uint8_t *pk, size_t n) {
    size_t i = 0;
    while (i < n && ((uintptr_t)(out + kRot * i) & 63)) ++i;
    if (i >= n) { expand_plain(out, pk, n); return; }
    expand_plain(out, pk, i);
    alignas(64) uint16_t st[32 * kRot + 32];
    for (; i + 32 <= n; i += 32) {
        for (int r = 0; r < 32; ++r) {
            const uint8_t *p = pk + 32 * (i + r); uint32_t b = p[31];
            const __m512i w = _mm512_add_epi16(_mm512_cvtepu8_epi16(_mm256_loadu_si256((const __m256i *)p)), _mm512_set1_epi16((short)(b << 6)));
            _mm512_storeu_si512((void *)(st + kRot * r), w);
        }
        __m512i *d = (__m512i *)(out + kRot * i);
        for (int l = 0; l < 31; ++l) _mm512_stream_si512(d + l, _mm512_load_si512((const __m512i *)st + l));
    }
    expand_plain(out + kRot * i, pk + 32 * i, n - i);
}
int main() {
    size_t N = 3000000; size_t call = 5000;
    std::vector<uint8_t> pk(N*32); for (size_t i=0;i<pk.size();++i) pk[i]=(uint8_t)(i*7); for(size_t i=0;i<N;++i) pk[32*i+31]=50;
    uint16_t *out = (uint16_t*)aligned_alloc(64, N*62+128); out += 8; // misalign like numpy
    memset(out, 0, N*62);
    for (int v=0; v<2; ++v) for (int rep=0; rep<3; ++rep) {
        auto t=std::chrono::steady_clock::now();
        for (size_t a=0;a<N;a+=call) (v? expand_nt: expand_plain)(out+31*a, pk.data()+32*a, std::min(call, N-a));
        _mm_sfence();
        double s=std::chrono::duration<double>(std::chrono::steady_clock::now()-t).count();
        printf("%s %.2f ns/rec %.1f GB/s out\n", v?"nt":"plain", s/N*1e9, N*62/s/1e9);
    }
}
