/* The exact floor division by the tick of hftlob.hip (tick_floordiv): every int32 numerator for
 * d = 1, 3, 100, every 97th for other divisors, against C floor division.  gcc -O2 magic_check.c */
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
int main() {
    int32_t ds[] = {1, 2, 3, 5, 7, 10, 25, 50, 100, 128, 1000, 12345, 65537, 1 << 20, (1 << 20) + 1, 1 << 30, 2147483647, 99, 101, 1024, 3000};
    long long bad = 0;
    for (unsigned i = 0; i < sizeof ds / sizeof ds[0]; ++i) {
        int sh; uint32_t m = magic(ds[i], &sh);
        for (long long a = -2147483648LL; a <= 2147483647LL; a += (ds[i] == 100 || ds[i] == 1 || ds[i] == 3) ? 1 : 97) {
            if (fd_mag((int32_t)a, m, sh) != fd_ref((int32_t)a, ds[i])) { if (bad < 5) printf("bad d=%d a=%lld\n", ds[i], a); ++bad; }
        }
    }
    printf("mismatches: %lld\n", bad);
    return 0;
}
