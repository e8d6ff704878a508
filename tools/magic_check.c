/* The exact floor division by the tick of hftlob.hip (tick_floordiv): every int32 numerator for
 * d = 1, 3, 100, every 97th for other divisors, against C floor division ("quick": a sample, see
 * main).  gcc -O2 magic_check.c */
#include <stdio.h>
#include <stdint.h>
static uint32_t magic(int32_t d, int* sh) {
    int l = d > 1 ? 32 - __builtin_clz((uint32_t)(d - 1)) : 0;
    *sh = 31 + l;
    unsigned __int128 num = ((unsigned __int128)1) << (31 + l);
    unsigned long long m = (unsigned long long)((num + (unsigned)d - 1) / (unsigned)d);
    if (m >> 32) { printf("magic overflow d=%d\n", d); }
    return (uint32_t)m;
}
static int32_t fd_ref(int32_t a, int32_t b) { int32_t q = a / b; if ((a % b != 0) && ((a < 0) != (b < 0))) q -= 1; return q; }
static int32_t fd_mag(int32_t a, uint32_t m, int sh) {
    uint32_t n = a < 0 ? ~(uint32_t)a : (uint32_t)a;
    uint32_t q = (uint32_t)(((unsigned long long)n * m) >> sh);
    return a < 0 ? (int32_t)~q : (int32_t)q;
}
int main(int argc, char** argv) {
    /* argv[1] == "quick" (tests/test_tick_division.py): every 65537th numerator plus the 2^20
     * numerators at each end of the range and around 0, for every divisor */
    const int quick = argc > 1 && argv[1][0] == 'q';
    int32_t ds[] = {1, 2, 3, 5, 7, 10, 25, 50, 100, 128, 1000, 12345, 65537, 1 << 20, (1 << 20) + 1, 1 << 30, 2147483647, 99, 101, 1024, 3000};
    long long bad = 0;
    for (unsigned i = 0; i < sizeof ds / sizeof ds[0]; ++i) {
        int sh; uint32_t m = magic(ds[i], &sh);
        const long long stride = quick ? 65537 : ((ds[i] == 100 || ds[i] == 1 || ds[i] == 3) ? 1 : 97);
        for (long long a = -2147483648LL; a <= 2147483647LL; a += stride) {
            if (fd_mag((int32_t)a, m, sh) != fd_ref((int32_t)a, ds[i])) { if (bad < 5) printf("bad d=%d a=%lld\n", ds[i], a); ++bad; }
        }
        if (quick) {
            const long long lo[3] = {-2147483648LL, -(1LL << 19), 2147483647LL - (1LL << 20) + 1};
            for (int k = 0; k < 3; ++k)
                for (long long a = lo[k]; a < lo[k] + (1LL << 20); ++a)
                    if (fd_mag((int32_t)a, m, sh) != fd_ref((int32_t)a, ds[i])) { if (bad < 5) printf("bad d=%d a=%lld\n", ds[i], a); ++bad; }
        }
    }
    printf("mismatches: %lld\n", bad);
    return 0;
}
