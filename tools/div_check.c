// Exhaustive check of he_math.h div_byf (f32 Markstein division by a constant) against
// IEEE a / b over all 2^32 numerators, per divisor given on the command line.
//   gcc -O2 -mfma -fopenmp -ffp-contract=off -o /tmp/div_check tools/div_check.c -lm
//   /tmp/div_check 25 496.480011 200 252
// Result (this container, r01): 0 mismatches for 25, 496.480011, 200, 252, 7, 3, 0.3, 1.99999988,
// 0.001, 300000 (the dividend guard matters for tiny divisors: r ~ ulp(a) must stay normal).
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static inline float div_byf(float a, float b, float y) {
    float q = a * y;
    float aq = fabsf(q), aa = fabsf(a);
    if (!(aq > 0x1p-100f && aq < 0x1p+100f && aa > 0x1p-100f)) return a / b;
    float r = fmaf(-q, b, a);
    return fmaf(r, y, q);
}
int main(int argc, char** argv) {
    for (int k = 1; k < argc; ++k) {
        float b = strtof(argv[k], NULL);
        volatile float one = 1.0f;
        float y = one / b;
        uint64_t bad = 0;
        #pragma omp parallel for reduction(+:bad) schedule(static)
        for (int64_t u = 0; u < (1ll << 32); ++u) {
            uint32_t bits = (uint32_t)u; float a; memcpy(&a, &bits, 4);
            volatile float ref = a / b;
            float got = div_byf(a, b, y);
            uint32_t rb, gb; float rr = ref; memcpy(&rb, &rr, 4); memcpy(&gb, &got, 4);
            if (rb != gb && !(rr != rr && got != got)) bad++;
        }
        printf("b=%.9g y=%.9g mismatches=%llu\n", b, y, (unsigned long long)bad);
    }
    return 0;
}
