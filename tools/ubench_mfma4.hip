// tools/ubench_mfma4.hip -- v_mfma_f64_4x4x4_4b_f64 on gfx950: throughput
// against v_mfma_f64_16x16x4_f64, and the operand layout seen with A = ones
// (a column-sum building block: D[b][i][j] = sum_k B[b][k][j]).
//
// hipcc --offload-arch=gfx950 -O3 tools/ubench_mfma4.hip -o /tmp/ubench_mfma4 && /tmp/ubench_mfma4
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef double d4v __attribute__((ext_vector_type(4)));

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            printf("%s failed: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

__global__ __launch_bounds__(256) void k16(int iters, double *out) {
    const int lane = threadIdx.x & 63;
    d4v acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = d4v{0, 0, 0, 0};
    double a = 1.0 + lane * 1e-3, b = 0.5 - lane * 1e-4;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0;
    for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k4(int iters, double *out) {
    const int lane = threadIdx.x & 63;
    double acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = 0;
    double a = 1.0 + lane * 1e-3, b = 0.5 - lane * 1e-4;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0;
    for (int i = 0; i < 16; ++i) s += acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// one dependent chain (latency)
__global__ __launch_bounds__(64) void k4chain(int iters, double *out) {
    const int lane = threadIdx.x & 63;
    double acc = 0, a = 1.0, b = 1e-9 * lane;
    for (int it = 0; it < iters; ++it) acc = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc, 0, 0, 0);
    out[threadIdx.x] = acc;
}

__global__ void klayout(double *out) {
    const int lane = threadIdx.x;
    const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, (double)(1 << (lane & 15)) + 65536.0 * (lane >> 4), 0.0, 0, 0, 0);
    out[lane] = d;
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cu = prop.multiProcessorCount;
    double *out;
    CK(hipMalloc(&out, (size_t)cu * 8 * 256 * sizeof(double)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 20000;
    for (int rep = 0; rep < 2; ++rep) {
        float ms;
        hipLaunchKernelGGL(k16, dim3(cu * 2), dim3(256), 0, 0, iters, out);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k16, dim3(cu * 2), dim3(256), 0, 0, iters, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double n16 = (double)cu * 2 * 4 * iters * 16;  // wave-level instructions
        printf("16x16x4 f64: %.3f ms, %.2f TF/s, %.1f ns per instr per SIMD\n", ms,
               n16 * 2048.0 / ms / 1e9, ms * 1e6 / (n16 / (cu * 4)));
        hipLaunchKernelGGL(k4, dim3(cu * 2), dim3(256), 0, 0, iters, out);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k4, dim3(cu * 2), dim3(256), 0, 0, iters, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("4x4x4_4b f64: %.3f ms, %.2f TF/s (512 flop/instr), %.1f ns per instr per SIMD\n", ms,
               n16 * 512.0 / ms / 1e9, ms * 1e6 / (n16 / (cu * 4)));
        hipLaunchKernelGGL(k4chain, dim3(1), dim3(64), 0, 0, iters, out);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k4chain, dim3(1), dim3(64), 0, 0, iters, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("4x4x4_4b f64 dependent chain: %.1f ns per instr\n", ms * 1e6 / iters);
    }
    hipLaunchKernelGGL(klayout, dim3(1), dim3(64), 0, 0, out);
    double h[64];
    CK(hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost));
    printf("layout (A = 1, B[l] = 2^(l&15) + 65536 (l>>4)): D[l] = sum of B over the lanes in l's k-group\n");
    for (int l = 0; l < 64; ++l) {
        const unsigned long long v = (unsigned long long)h[l];
        printf("lane %2d: blockpart %llu lanes-mask 0x%04llx\n", l, v >> 16, v & 0xFFFF);
    }
    return 0;
}
