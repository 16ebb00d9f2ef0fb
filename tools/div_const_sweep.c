/* Sweep of fvp_device.h div_const over integer divisors: for every
 * odd b in [lo, hi] and every one of the 2^23 mantissas of a in [1, 2),
 *   q = RN(a * RN(1/b)),  q' = RN(q + RN(a - q*b) * RN(1/b))   (two fmas)
 * must equal the correctly rounded a / b.  The three operations and a / b
 * scale exactly by powers of two in a and in b while every value stays
 * normal, and are odd in a, so this covers every integer divisor in [1, hi]
 * and every a with a normal quotient (the subnormal / -0 cases are absorbed
 * by pixel_to_sample's `* 2 - 1`).  Test tooling (tests/test_div_const.py runs
 * a part of it; the whole range 3..65535 was run once:
 * profiles/round4/div_const_sweep_65535.txt).
 *   gcc -O2 -fopenmp -ffp-contract=off -mfma tools/div_const_sweep.c -lm && ./a.out 3 65535 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline float bits_f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t f_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(int argc, char **argv) {
    const int lo = argc > 1 ? atoi(argv[1]) : 3, hi = argc > 2 ? atoi(argv[2]) : 4095;
    long long checked = 0;
    int failing = 0;
#pragma omp parallel for schedule(dynamic) reduction(+ : checked, failing)
    for (int n = lo | 1; n <= hi; n += 2) {
        const float b = (float)n, rb = 1.0f / b;
        long long bad = 0;
        for (uint32_t m = 0; m < (1u << 23); ++m) {
            const float a = bits_f(0x3f800000u | m);
            const float q = a * rb;
            const float got = fmaf(fmaf(-q, b, a), rb, q);
            bad += f_bits(got) != f_bits(a / b);
        }
        checked += 1LL << 23;
        if (bad) {
#pragma omp critical
            printf("b=%d: %lld mantissas differ\n", n, bad);
            ++failing;
        }
    }
    printf("odd divisors %d..%d: %lld quotients checked, %d divisors with a difference\n", lo | 1, hi, checked, failing);
    return failing != 0;
}
