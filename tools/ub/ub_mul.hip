// Microbenchmark: issue rate of v_mul_lo_u32 against full-rate VALU ops on gfx950
// (independent chains per lane, every CU busy). Prints ns per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t iters) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const uint32_t c = 0xcc9e2d51u + blockIdx.x;
    for (uint32_t i = 0; i < iters; i++) {
#define STEP(x)                                                                    \
    if (OP == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "s"(c));      \
    else if (OP == 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "s"(c));   \
    else if (OP == 2) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "s"(c)); \
    else asm volatile("v_alignbit_b32 %0, %0, %0, 19" : "+v"(x));
        STEP(a0) STEP(a1) STEP(a2) STEP(a3) STEP(a4) STEP(a5) STEP(a6) STEP(a7)
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;  // 8 waves... 32 waves per CU
    uint32_t* out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    const uint32_t iters = 20000;
    const char* names[] = {"v_mul_lo_u32", "v_add_u32", "v_mul_u32_u24", "v_alignbit_b32"};
    for (int op = 0; op < 4; op++) {
        for (int rep = 0; rep < 2; rep++) {
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0);
            if (op == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters);
            if (op == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters);
            if (op == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters);
            if (op == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            // wave-instructions per SIMD: blocks*4 waves / (cus*4 SIMDs) * iters * 8
            const double per_simd = (double)blocks * 4 / (cus * 4.0) * iters * 8;
            if (rep) printf("%-16s %.3f ms  %.3f ns per wave-instr per SIMD (%.2f cycles at 2.4 GHz)\n", names[op], ms,
                            ms * 1e6 / per_simd, ms * 1e6 / per_simd * 2.4);
        }
    }
    return 0;
}
