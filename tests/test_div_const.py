"""Host check of fvp_device.h's div_const (the division by a launch-constant
divisor inside pixel_to_sample): q = a*rb, q' = fma(fma(-q, b, a), rb, q)
with rb = RN(1/b) equals the correctly rounded a / b, except where the
quotient is subnormal or a = -0 (the cases pixel_to_sample absorbs in
`* 2 - 1`, see its comment).  Every mantissa and both signs of a at the
exponents where the result can leave the normal range (subnormal a, the
smallest normal exponents, the largest ones) and at a spread of exponents
between -- all three operations scale exactly by powers of two while the
values stay normal, so these cover every a whose quotient is normal.  (The
full 2^32 sweep, run once for these divisors and 199, 151, 7 and 3, found
the same: no mismatch outside the subnormal / -0 set.)  Divisors: the
image and heatmap constants of the BASELINE configs (960 x 512 and 800 x 608
images; 239 and 127 = heatmap size - 1).  The host program reproduces the
device arithmetic (IEEE fp32 mul / fma / div, no contraction).  CPU only (gcc
+ OpenMP)."""
import os
import shutil
import subprocess
import tempfile

import pytest

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static float div_const(float a, float b, float rb) {  /* fvp_device.h div_const */
    const float q = a * rb;
    return fmaf(fmaf(-q, b, a), rb, q);
}
int main(int argc, char **argv) {
    int fail = 0;
    for (int k = 1; k < argc; ++k) {
        const float b = strtof(argv[k], 0), rb = 1.0f / b;
        long long bad = 0, allowed = 0;
        static const int ex[] = {0, 1, 2, 3, 4, 5, 20, 60, 100, 126, 127, 128, 150, 200, 250, 251, 252, 253, 254};
        const int nex = (int)(sizeof ex / sizeof ex[0]);
        #pragma omp parallel for reduction(+:bad, allowed) schedule(static)
        for (long long i = 0; i < (long long)nex << 24; ++i) {
            const uint32_t u = ((uint32_t)(i & 1) << 31) | ((uint32_t)ex[i >> 24] << 23) |
                               (uint32_t)((i >> 1) & 0x7fffff);  /* sign, exponent, mantissa */
            float a;
            memcpy(&a, &u, 4);
            if (!isfinite(a)) continue;
            const float ref = a / b, got = div_const(a, b, rb);
            if (memcmp(&ref, &got, 4) == 0) continue;
            if (fabsf(ref) < 1.17549435e-38f) ++allowed;  /* subnormal quotient or a = -0 */
            else ++bad;
        }
        printf("b=%g bad=%lld subnormal_or_signed_zero=%lld\n", b, bad, allowed);
        fail |= bad != 0;
    }
    return fail;
}
"""

DIVISORS = ["960", "512", "800", "608", "239", "127"]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_div_const_matches_ieee_division():
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "divc.c"), os.path.join(d, "divc")
        with open(c, "w") as f:
            f.write(SRC)
        subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-fno-fast-math", "-msse2", "-mfpmath=sse",
                        "-mfma", c, "-o", exe, "-lm"], check=True)
        env = dict(os.environ, OMP_NUM_THREADS=str(min(8, os.cpu_count() or 1)))
        r = subprocess.run([exe] + DIVISORS, capture_output=True, text=True, timeout=600, env=env)
        print(r.stdout)
        assert r.returncode == 0, r.stdout
        assert r.stdout.count("bad=0 ") == len(DIVISORS)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_div_const_integer_divisor_sweep():
    """tools/div_const_sweep.c over the odd divisors 3..4095 (every mantissa of
    a in [1, 2); with the power-of-two scaling this covers every integer
    divisor up to 4095 -- every image / heatmap size of the reference's
    configs) -- exactly the range ImageConsts::exact admits (div_const_covered);
    any other divisor takes the IEEE division on the device."""
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "sweep")
        subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-fno-fast-math", "-mfma",
                        os.path.join(repo, "tools", "div_const_sweep.c"), "-o", exe, "-lm"], check=True)
        env = dict(os.environ, OMP_NUM_THREADS=str(min(8, os.cpu_count() or 1)))
        r = subprocess.run([exe, "3", "4095"], capture_output=True, text=True, timeout=600, env=env)
        print(r.stdout)
        assert r.returncode == 0 and "0 divisors with a difference" in r.stdout, r.stdout


DIV_PAIR_SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static inline float bits_f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t f_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
/* fvp_device.h div_pair, one numerator, from a reciprocal seed r0 (v_rcp_f32 is
   within 1 ulp of 1/b; its exact value is the hardware's, so every seed in
   {RN(1/b) - 1 ulp, RN(1/b), RN(1/b) + 1 ulp} is tried) */
static inline float div_pair1(float a, float b, float r0) {
    const float r = fmaf(fmaf(-b, r0, 1.0f), r0, r0);
    float q = a * r;
    q = fmaf(fmaf(-b, q, a), r, q);
    return fmaf(fmaf(-b, q, a), r, q);
}
static inline uint64_t mix(uint64_t x) { x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; return x ^ (x >> 33); }
int main(int argc, char **argv) {
    const int per_b = argc > 1 ? atoi(argv[1]) : 8;
    const uint32_t bstep = argc > 2 ? (uint32_t)atoi(argv[2]) : 1;
    long long checked = 0, bad = 0;
    /* every (bstep-th) mantissa of b in [1, 2): the quotient, the reciprocal and the
       remainders scale exactly by powers of two in a and b while everything stays
       normal (|a|, |b| in [2^-40, 2^40] on the device), so mantissas decide */
#pragma omp parallel for schedule(static) reduction(+ : checked, bad)
    for (uint32_t mb = 0; mb < (1u << 23); mb += bstep) {
        const float b = bits_f(0x3f800000u | mb);
        const float rn = 1.0f / b;
        const float seeds[3] = {bits_f(f_bits(rn) - 1), rn, bits_f(f_bits(rn) + 1)};
        for (int k = 0; k < per_b; ++k) {
            const uint64_t h = mix(((uint64_t)mb << 20) ^ (uint64_t)k);
            float as[6];
            /* a random numerator in [1, 2) and [2, 4), and the numerators whose
               quotient lies next to a rounding midpoint (the hard cases):
               a = RN(b * (q + ulp(q)/2)) and its neighbours */
            as[0] = bits_f(0x3f800000u | (uint32_t)(h & 0x7fffff));
            as[1] = bits_f(0x40000000u | (uint32_t)((h >> 23) & 0x7fffff));
            const float q = bits_f(0x3f000000u | (uint32_t)((h >> 40) & 0x7fffff));  /* [0.5, 1) */
            const double mid = (double)q + ldexp(1.0, -25);
            const float a0 = (float)(mid * (double)b);
            as[2] = a0; as[3] = bits_f(f_bits(a0) + 1); as[4] = bits_f(f_bits(a0) - 1);
            as[5] = -as[0];
            for (int i = 0; i < 6; ++i) {
                const float ref = as[i] / b;
                for (int s = 0; s < 3; ++s) {
                    ++checked;
                    bad += f_bits(div_pair1(as[i], b, seeds[s])) != f_bits(ref);
                }
            }
        }
    }
    printf("div_pair: %lld quotients checked, %lld differ\n", checked, bad);
    return bad != 0;
}
"""


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_div_pair_matches_ieee_division():
    """fvp_device.h div_pair (project_point's two quotients by one divisor): the
    unscaled core of the IEEE division sequence, from reciprocal seeds 1 ulp
    either side of RN(1/b), against a / b -- every mantissa of b in [1, 2) with
    random numerators in two binades and the numerators whose quotients sit next
    to rounding midpoints."""
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "divp.c"), os.path.join(d, "divp")
        with open(c, "w") as f:
            f.write(DIV_PAIR_SRC)
        subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-fno-fast-math", "-mfma", c, "-o", exe,
                        "-lm"], check=True)
        env = dict(os.environ, OMP_NUM_THREADS=str(min(8, os.cpu_count() or 1)))
        r = subprocess.run([exe, "4", "1"], capture_output=True, text=True, timeout=600, env=env)
        print(r.stdout)
        assert r.returncode == 0 and " 0 differ" in r.stdout, r.stdout
