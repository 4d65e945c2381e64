// tools/ubench_i8.hip -- the int8 matrix ceiling, for the fp64-emulation
// (Ozaki-scheme) estimate in DESIGN.md §10: K1 priced as s(s+1)/2 exact int8
// slice products instead of one fp64 product.
//
//   i8_16 : v_mfma_i32_16x16x64_i8 back-to-back, 8 independent accumulators
//   i8_32 : v_mfma_i32_32x32x32_i8 back-to-back, 4 independent accumulators
//   f64   : v_mfma_f64_16x16x4_f64 back-to-back, 16 accumulators (same box, same run)
//
// Two waves per SIMD (512 threads, 2 workgroups per CU over 256 CUs).
// hipcc --offload-arch=gfx950 -O3 tools/ubench_i8.hip -o ubench_i8 && ./ubench_i8
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef double d4v __attribute__((ext_vector_type(4)));

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            printf("%s failed: %s\n", #x, hipGetErrorString(e));                     \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ __launch_bounds__(512) void k_i8_16(int iters, int *out) {
    const int lane = threadIdx.x & 63;
    v4i a = {lane * 0x01010101, 0x02020202, -0x01010101, lane};
    v4i b = {0x7f7f7f7f, lane, 0x01020304, -lane};
    v4i acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = v4i{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[i], 0, 0, 0);
    }
    int s = 0;
    for (int i = 0; i < 8; ++i) s += acc[i][0] ^ acc[i][1] ^ acc[i][2] ^ acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(512) void k_i8_32(int iters, int *out) {
    const int lane = threadIdx.x & 63;
    v4i a = {lane * 0x01010101, 0x02020202, -0x01010101, lane};
    v4i b = {0x7f7f7f7f, lane, 0x01020304, -lane};
    v16i acc[4];
    for (int i = 0; i < 4; ++i) acc[i] = v16i{};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
    }
    int s = 0;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 16; ++j) s ^= acc[i][j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(512) void k_f64(int iters, int *out) {
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
    out[blockIdx.x * blockDim.x + threadIdx.x] = (int)s;
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cu = p.multiProcessorCount, grid = cu * 2, block = 512;
    int *out;
    CK(hipMalloc(&out, (size_t)grid * block * sizeof(int)));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int waves = grid * block / 64;
    struct {
        const char *name;
        void (*k)(int, int *);
        int per_iter;       // MFMAs per iteration per wave
        double ops_per_mfma;
        int iters;
    } runs[] = {
        {"i8 16x16x64", k_i8_16, 8, 2.0 * 16 * 16 * 64, 20000},
        {"i8 32x32x32", k_i8_32, 4, 2.0 * 32 * 32 * 32, 20000},
        {"f64 16x16x4", k_f64, 16, 2.0 * 16 * 16 * 4, 4000},
    };
    for (auto &r : runs) {
        hipLaunchKernelGGL(r.k, dim3(grid), dim3(block), 0, 0, 100, out);  // warm
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(r.k, dim3(grid), dim3(block), 0, 0, r.iters, out);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
        }
        const double ops = (double)waves * r.iters * r.per_iter * r.ops_per_mfma;
        printf("%-12s %8.3f ms  %8.1f TOPS\n", r.name, best, ops / (best * 1e-3) / 1e12);
    }
    CK(hipFree(out));
    return 0;
}
