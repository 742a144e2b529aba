"""The rescale division of the single-matrix kernels (csrc/pcx_matrix.hip div_rn): (r - lo) /
range as q0 = d y, r = fma(-q0, b, d), q = fma(r, y, q0) with y = RN(1 / b), falling back to the
division where an intermediate leaves the normal range.  The reference divides
(pyconsensus/__init__.py:266-269, numpy's IEEE division), so the sequence with its guard must
equal d / b bit for bit for every input; this test restates it in C (the same operations in the
same order; fma and the magnitude tests are exact on both the host and gfx950) and compares it with
the division over realistic, near-tie, extreme-exponent and special inputs.
"""
import subprocess
import textwrap

import pytest

SRC = textwrap.dedent(r"""
    #include <math.h>
    #include <stdint.h>
    #include <stdio.h>
    #include <stdlib.h>
    #include <string.h>
    static uint64_t s = 88172645463325252ull;
    static uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
    static double bits(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
    static uint64_t ubits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
    static double range_rcp(double b) {
        double a = fabs(b);
        return (a >= 0x1p-100 && a <= 0x1p100) ? 1.0 / b : NAN;
    }
    static double div_rn(double d, double b, double y) {  /* pcx_matrix.hip div_rn */
        volatile double q0 = d * y;
        volatile double r = fma(-q0, b, d);
        double q = fma(r, y, q0);
        if (isnan(y) || fabs(q0) < 0x1p-860 || fabs(q0) > 0x1p1000) q = d / b;
        return q;
    }
    static double any_double(void) {  /* every exponent, including subnormals, inf and NaN */
        return bits(xr());
    }
    int main(int argc, char** argv) {
        long n = atol(argv[1]), bad = 0, fast = 0;
        s ^= (uint64_t)atol(argv[2]);
        for (long k = 0; k < n; k++) {
            double b, d;
            switch (k % 6) {
            case 0:  /* the synthetic recipe: lo ~ U(-100, 0), range ~ U(1, 200) */
                b = 1.0 + (xr() >> 11) * 0x1p-53 * 199.0;
                d = (xr() >> 11) * 0x1p-53 * 300.0 - 100.0;
                break;
            case 1:  /* full mantissas, moderate exponents */
                b = bits((0x3ffull << 52) | (xr() >> 12));
                d = bits(((0x3ffull + (xr() % 40) - 20) << 52) | (xr() >> 12));
                break;
            case 2:  /* divisors just below a power of two */
                b = bits((0x3ffull << 52) | ((1ull << 52) - 1 - (xr() % 4096)));
                d = bits(((0x3ffull + (xr() % 8) - 4) << 52) | (xr() >> 12));
                break;
            case 3: {  /* near-exact quotients: the rounding ties' neighbourhood */
                b = bits((0x3ffull << 52) | (xr() >> 12));
                double q = bits((0x3ffull << 52) | (xr() >> 12));
                d = bits(ubits(q * b) + (int)(xr() % 5) - 2);
                break;
            }
            case 4:  /* extreme exponents either side (and the range limits of y) */
                b = bits(((uint64_t)(1023 + (int)(xr() % 202) - 101) << 52) | (xr() >> 12));
                d = any_double();
                break;
            default:  /* anything */
                b = any_double();
                d = any_double();
                if (xr() % 8 == 0) d = (xr() & 1) ? 0.0 : -0.0;
                if (xr() % 8 == 0) d = (xr() & 1) ? INFINITY : -INFINITY;
            }
            if (b == 0 || isnan(b)) continue;  /* a scaled column's range is finite and non-zero */
            double y = range_rcp(b);
            double e = d / b, f = div_rn(d, b, y);
            if (!isnan(y) && !(fabs(d * y) < 0x1p-860 || fabs(d * y) > 0x1p1000)) fast++;
            if (isnan(e) ? !isnan(f) : ubits(e) != ubits(f)) {
                if (bad < 5) printf("b=%a d=%a expect=%a got=%a\n", b, d, e, f);
                bad++;
            }
        }
        printf("n=%ld fast=%ld bad=%ld\n", n, fast, bad);
        return bad != 0;
    }
""")


@pytest.fixture(scope="module")
def fastdiv_bin(tmp_path_factory):
    d = tmp_path_factory.mktemp("fastdiv")
    src, exe = d / "fastdiv.c", d / "fastdiv"
    src.write_text(SRC)
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", str(src), "-o", str(exe), "-lm"],
                   check=True)
    return exe


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_div_rn_equals_division(fastdiv_bin, seed):
    r = subprocess.run([str(fastdiv_bin), "6000000", str(seed)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bad=0" in r.stdout
    fast = int(r.stdout.split("fast=")[1].split()[0])
    assert fast > 4_000_000  # (most cases exercise the fast path, not the fallback)
