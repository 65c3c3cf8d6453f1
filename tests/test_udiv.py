"""The one-pass step's division by a wave-uniform row metric (sw_kernels.hip udiv: Markstein's
q = RN(x r), t = RN(q d - x) (fma), RN(q - t r) (fma) with r = RN(1/d) from the row table) against
IEEE division, bit for bit (signed zeros included), over the domain the kernel uses it on: d a
real(4) metric promoted to real(8) with d in [2^-60, 2^60] (launch_prepare flags other divisors and the step then
does not run), x = 0 or 2^-900 <= |x| < 2^900 (the kernel re-runs a row with IEEE divisions
when a dividend is outside).  fma and IEEE division are correctly rounded on the host as on the
GPU (v_fma_f64), so the host check pins the arithmetic; the GPU tests pin the kernel."""
import subprocess

HARNESS = r"""
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
static uint64_t s = 0x1234567890abcdefull;
static inline uint64_t rnd() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static inline double asd(uint64_t u) { double x; std::memcpy(&x, &u, 8); return x; }
// (volatile: keeps g++ from folding -fma(q, d, -x) into fma(-q, d, x), which loses the sign of
// a zero residual; the device compiler keeps IEEE signed zeros without fast-math flags)
static double udiv(double x, double d, double r) { double q = x * r; volatile double t = std::fma(q, d, -x); double mt = -t; return std::fma(mt, r, q); }
int main(int argc, char **argv) {
    const long n = std::atol(argv[1]);
    long bad = 0;
    for (long i = 0; i < n; ++i) {
        uint32_t fb = (uint32_t)(rnd() & 0x7fffff) | ((uint32_t)(127 - 60 + rnd() % 121) << 23);   // 2^-60 .. 2^60
        if ((i & 15) == 0) fb |= 0x7fffff;          // all-ones significands
        if ((i & 31) == 1) fb &= ~0x7fffffu;        // powers of two
        float f; std::memcpy(&f, &fb, 4);
        double d = (double)f;
        uint64_t xb = (rnd() & 0x000fffffffffffffull) | ((uint64_t)(1023 - 900 + rnd() % 1800) << 52);
        if ((i & 7) == 0) xb &= ~0x000ffffffffff000ull;
        if ((i & 7) == 1) xb |= 0x000fffffffffff00ull;
        double x = asd(xb);
        if (rnd() & 1) x = -x;
        if ((i & 63) == 7) x = 0.0;
        if ((i & 63) == 8) x = -0.0;
        const double r = 1.0 / d, a = x / d, b = udiv(x, d, r);
        if (std::memcmp(&a, &b, 8)) { if (bad < 5) std::printf("x=%a d=%a ieee=%a udiv=%a\n", x, d, a, b); ++bad; }
    }
    std::printf("%ld of %ld differ\n", bad, n);
    return bad != 0;
}
"""


def test_udiv_matches_ieee_division(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text(HARNESS)
    exe = tmp_path / "t"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", str(src), "-o", str(exe)])
    r = subprocess.run([str(exe), "20000000"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.startswith("0 of"), r.stdout + r.stderr
