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
    configs).  The whole range 3..65535 that ImageConsts::exact admits was run
    once (profiles/round4/div_const_sweep_65535.txt, 2.7e11 quotients, no
    difference); any other divisor takes the IEEE division on the device."""
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "sweep")
        subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-fno-fast-math", "-mfma",
                        os.path.join(repo, "tools", "div_const_sweep.c"), "-o", exe, "-lm"], check=True)
        env = dict(os.environ, OMP_NUM_THREADS=str(min(8, os.cpu_count() or 1)))
        r = subprocess.run([exe, "3", "4095"], capture_output=True, text=True, timeout=600, env=env)
        print(r.stdout)
        assert r.returncode == 0 and "0 divisors with a difference" in r.stdout, r.stdout
    with open(os.path.join(repo, "profiles", "round4", "div_const_sweep_65535.txt")) as f:
        assert "odd divisors 3..65535:" in f.read()
