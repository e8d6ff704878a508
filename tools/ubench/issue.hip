// Micro-benchmark of the instruction costs that bound k_env_step on gfx950 at the
// metric's occupancy (4096 one-wave workgroups = 16 waves per CU), per op per wave:
// scalar ALU (independent / dependent), uniform branches (taken / not taken), the
// select that replaces a branch, VALU, v_readlane -> SALU, a DPP step, an LDS round
// trip, and SALU/VALU interleaved.  Usage: ./issue  (hipcc -O3 --offload-arch=gfx950)
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(x) x x x x x x x x
// independent SALU: 4 accumulators
#define SIND "s_add_u32 %0, %0, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %2, %2, 1\n s_add_u32 %3, %3, 1\n"
// dependent SALU chain
#define SDEP "s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n"
#define BR(L, c) "s_cmp_eq_u32 %4, " #c "\n s_cbranch_scc1 " #L "f\n s_add_u32 %0, %0, 1\n" #L ":\n"
#define SEL "s_cmp_eq_u32 %4, 0\n s_cselect_b32 %1, 1, 2\n s_add_u32 %0, %0, %1\n"
#define VIND "v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1\n"
#define RDL "v_readlane_b32 %1, %4, 3\n s_add_u32 %0, %0, %1\n"
#define DPP "v_min_i32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 1\n"
#define LDS "ds_read_b32 %0, %4\n s_waitcnt lgkmcnt(0)\n v_add_u32 %4, %0, %4\n"
#define MIX "s_add_u32 %0, %0, 1\n v_add_u32 %4, %4, 1\n s_add_u32 %1, %1, 1\n v_add_u32 %5, %5, 1\n"

template <int MODE>
__global__ __launch_bounds__(64) void k(int x, int iters, int* sink) {
    __shared__ int lds[64];
    lds[threadIdx.x] = 0;
    __syncthreads();
    unsigned a = 0, b = 0, c = 0, d = 0;
    int va = threadIdx.x, vb = 0, vc = 0, vd = 0;
    int vaddr = 0;
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) asm volatile(R8(SIND) : "+s"(a), "+s"(b), "+s"(c), "+s"(d) : "s"(x) : "scc");
        if (MODE == 1) asm volatile(R8(SDEP) : "+s"(a), "+s"(b), "+s"(c), "+s"(d) : "s"(x) : "scc");
        if (MODE == 2)
            asm volatile(BR(1, 0) BR(2, 0) BR(3, 0) BR(4, 0) BR(5, 0) BR(6, 0) BR(7, 0) BR(8, 0)
                         : "+s"(a), "+s"(b), "+s"(c), "+s"(d) : "s"(x) : "scc");
        if (MODE == 3)
            asm volatile(BR(1, 1) BR(2, 1) BR(3, 1) BR(4, 1) BR(5, 1) BR(6, 1) BR(7, 1) BR(8, 1)
                         : "+s"(a), "+s"(b), "+s"(c), "+s"(d) : "s"(x) : "scc");
        if (MODE == 4) asm volatile(R8(SEL) : "+s"(a), "+s"(b), "+s"(c), "+s"(d) : "s"(x) : "scc");
        if (MODE == 5) asm volatile(R8(VIND) : "+v"(va), "+v"(vb), "+v"(vc), "+v"(vd));
        if (MODE == 6) asm volatile(R8(RDL) : "+s"(a), "+s"(b), "+s"(c), "+s"(d) : "v"(va) : "scc");
        if (MODE == 7) asm volatile(R8(DPP) : "+v"(va));
        if (MODE == 8) asm volatile(R8(LDS) : "+v"(va), "+v"(vb), "+v"(vc), "+v"(vd), "+v"(vaddr));
        if (MODE == 9) asm volatile(R8(MIX) : "+s"(a), "+s"(b), "+s"(c), "+s"(d), "+v"(va), "+v"(vb) : : "scc");
    }
    if (threadIdx.x == 0) sink[blockIdx.x] = a + b + c + d + va + vb + vc + vd + lds[0];
}

static const char* NAMES[] = {"SALU indep x4 (per instr)", "SALU dependent (per instr)", "branch taken (cmp+br)",
                              "branch not taken (cmp+br+add)", "select (cmp+cselect+add)", "VALU indep x4 (per instr)",
                              "v_readlane + s_add (pair)", "DPP step + s_nop 1 (pair)", "LDS read round trip",
                              "SALU/VALU alternating (per instr)"};
static const int OPS[] = {32, 32, 8, 8, 8, 32, 8, 8, 8, 32};

template <int MODE> double run(int blocks, int iters, int* s) {
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, 0, iters, s);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, 0, iters, s);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1e6 / iters / OPS[MODE];  // ns per op per wave
}

template <int MODE> void row(int* s) {
    const int iters = 20000;
    printf("%-36s", NAMES[MODE]);
    for (int blocks : {1, 256, 1024, 4096}) printf(" %8.2f", run<MODE>(blocks, iters, s));
    printf("\n");
}

int main() {
    int* s;
    hipMalloc(&s, 65536 * 4);
    printf("ns per op per wave; waves per CU: %36s\n", "1/256      1      4     16");
    row<0>(s); row<1>(s); row<2>(s); row<3>(s); row<4>(s); row<5>(s); row<6>(s); row<7>(s); row<8>(s); row<9>(s);
    return 0;
}
