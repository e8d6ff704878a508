/* The fast float floor division by the tick of hftlob.hip (tick_ffloordiv) against the oracle's
 * jnp.floor_divide restatement (_float_divmod + round), bit for bit, with the hardware reciprocal
 * modelled as 1/y perturbed by up to +-4 ulp (v_rcp_f32 is within 1 ulp): every float x in
 * [-2^22, 2^22) on a 1/4 grid near multiples of the tick, every 1021st float bit pattern of both
 * signs, and the edge values (+-0, +-2^24, NaN, inf).  gcc -O2 -ffp-contract=off ffloordiv_check.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static float ref(float x, float y) {
    float mod = fmodf(x, y);
    float div = (x - mod) / y;
    int ind = (mod != 0.0f) && ((y > 0) - (y < 0)) != ((mod > 0) - (mod < 0));
    if (ind) div = div - 1.0f;
    return roundf(div);
}
static float fast(float x, int tick, float rcp) {
    const float y = (float)tick, a = fabsf(x);
    const float q = a * rcp;
    if (!((a < 16777216.0f) & (q < 524288.0f) & (tick < (1 << 24)))) return ref(x, y);
    float k = floorf(q), r = fmaf(-k, y, a);
    if (r < 0.0f) { k -= 1.0f; r += y; }
    else if (r >= y) { k += 1.0f; r -= y; }
    return (x < 0.0f ? -(k + (r != 0.0f ? 1.0f : 0.0f)) : k) + 0.0f;
}
static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static long long bad, n;
static void check(float x, int tick) {
    const float y = (float)tick, r0 = 1.0f / y;
    for (int p = -4; p <= 4; p += 2) {
        float rcp = r0;
        for (int k = 0; k < (p < 0 ? -p : p); ++k) rcp = nextafterf(rcp, p < 0 ? 0.0f : 2.0f);
        const float a = fast(x, tick, rcp), b = ref(x, y);
        ++n;
        if (bits(a) != bits(b) && !(a != a && b != b)) {
            if (bad < 8) printf("bad tick=%d x=%.9g (0x%08x) rcp%+d: fast %.9g ref %.9g\n", tick, x, bits(x), p, a, b);
            ++bad;
        }
    }
}
int main(int argc, char** argv) {
    /* argv[1] == "quick" (tests/test_tick_division.py): the grid at +-4000 multiples and every
     * 65521st bit pattern */
    const int quick = argc > 1 && argv[1][0] == 'q';
    const long long mmax = quick ? 4000 : 40000;
    const uint64_t bstep = quick ? 65521 : 1021;
    const int ticks[] = {1, 2, 3, 7, 10, 25, 100, 128, 1000, 12345, 65537, 1 << 20, (1 << 24) - 1, 1 << 24};
    for (unsigned t = 0; t < sizeof ticks / sizeof ticks[0]; ++t) {
        const int tick = ticks[t];
        for (long long m = -mmax; m <= mmax; ++m)  /* around multiples of the tick */
            for (int d = -8; d <= 8; ++d) {
                const double xv = (double)m * tick + d * 0.25;
                if (fabs(xv) < 16777216.0) check((float)xv, tick);
            }
        for (uint64_t u = 0; u < 0x80000000ull; u += bstep) {  /* float bit patterns, both signs */
            uint32_t v = (uint32_t)u;
            float x;
            memcpy(&x, &v, 4);
            check(x, tick);
            check(-x, tick);
        }
        const float edge[] = {0.0f, -0.0f, 16777216.0f, -16777216.0f, 16777215.0f, -16777215.0f, INFINITY, -INFINITY, NAN,
                              0.5f, -0.5f, 1e-30f, -1e-30f};
        for (unsigned i = 0; i < sizeof edge / sizeof edge[0]; ++i) check(edge[i], tick);
    }
    printf("checked %lld, mismatches: %lld\n", n, bad);
    return bad != 0;
}
