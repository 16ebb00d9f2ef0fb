"""Exhaustive host check of fvp_proposal.hip's div_small (the NMS index decode
without an integer division): for every 0 <= e < 2^16 and 1 <= Y < 2^16,
q = (int)((float)e * (1.0f / Y)) corrected once by the remainder's sign equals
e / Y.  The fp32 ops are IEEE-exact on both sides (the kernel is built with
-ffp-contract=off and correctly rounded division), so the host program
reproduces the device arithmetic.  CPU only (gcc), ~2^32 cases in seconds."""
import os
import shutil
import subprocess
import tempfile

import pytest

SRC = r"""
#include <stdio.h>
static int div_small(int e, int Y, float rY) {  /* fvp_proposal.hip div_small */
    int q = (int)((float)e * rY);
    const int r = e - q * Y;
    q += (r >= Y) - (r < 0);
    return q;
}
int main(void) {
    long long bad = 0;
    for (int Y = 1; Y < 65536; ++Y) {
        const float rY = 1.0f / (float)Y;
        for (int e = 0; e < 65536; ++e)
            if (div_small(e, Y, rY) != e / Y) { if (bad < 5) printf("e=%d Y=%d\n", e, Y); ++bad; }
    }
    printf("bad %lld\n", bad);
    return bad != 0;
}
"""


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_div_small_exhaustive():
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "div.c"), os.path.join(d, "div")
        with open(c, "w") as f:
            f.write(SRC)
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-msse2", "-mfpmath=sse", c, "-o", exe],
                       check=True)
        r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout
        assert r.stdout.strip().endswith("bad 0")
