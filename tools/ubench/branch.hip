// Micro-benchmark: cost of a taken wave-uniform branch vs a select on gfx950
// (guides the message-dispatch design of k_env_step).  Usage: ./branch
#include <hip/hip_runtime.h>
#include <cstdio>

#define B1(L) "s_cmp_eq_u32 %1, 0\n s_cbranch_scc1 " #L "f\n s_add_u32 %0, %0, 1\n" #L ":\n"
#define S1 "s_cmp_eq_u32 %1, 0\n s_cselect_b32 s0, 1, 2\n s_add_u32 %0, %0, s0\n"

template <int MODE>
__global__ __launch_bounds__(64) void k(int x, int iters, unsigned long long* out, int* sink) {
    unsigned acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) {
            asm volatile(B1(1) B1(2) B1(3) B1(4) B1(5) B1(6) B1(7) B1(8) : "+s"(acc) : "s"(x) : "scc");
        } else {
            asm volatile(S1 S1 S1 S1 S1 S1 S1 S1 : "+s"(acc) : "s"(x) : "scc", "s0");
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[blockIdx.x] = t1 - t0;
        sink[blockIdx.x] = acc;
    }
}

template <int MODE> double run(int x, int blocks, int iters, unsigned long long* d, int* s) {
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, x, iters, d, s);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, x, iters, d, s);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1e6 / iters / 8;  // ns per branch (or select) per wave-iteration
}

int main() {
    unsigned long long* d;
    int* s;
    hipMalloc(&d, 65536 * 8);
    hipMalloc(&s, 65536 * 4);
    const int iters = 20000;
    for (int blocks : {1, 256, 1024, 4096}) {
        printf("blocks %5d: taken branch %.2f ns, not-taken %.2f ns, select %.2f ns (per op, per wave)\n", blocks,
               run<0>(0, blocks, iters, d, s), run<0>(1, blocks, iters, d, s), run<1>(0, blocks, iters, d, s));
    }
    return 0;
}
