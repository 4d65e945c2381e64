// tools/ubench_fp64.hip -- measure the fp64 ceilings K1 is priced against.
//
//   mfma   : v_mfma_f64_16x16x4_f64 back-to-back, 16 independent accumulators
//   valu   : v_fma_f64 chains, 16 independent per lane
//   mixed  : half the waves of each workgroup on MFMA, half on VALU FMA
//   stream : K1's global-load pattern alone (register ring, no MFMA)
//
// hipcc --offload-arch=gfx950 -O3 tools/ubench_fp64.hip -o ubench && ./ubench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef double d4v __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            printf("%s failed: %s\n", #x, hipGetErrorString(e));                     \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__device__ __forceinline__ void mfma_loop(int iters, double *out) {
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

__device__ __forceinline__ void valu_loop(int iters, double *out) {
    const int lane = threadIdx.x & 63;
    double x[16];
    for (int i = 0; i < 16; ++i) x[i] = i * 1e-3 + lane;
    const double a = 0.999999, b = 1e-7;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = __builtin_fma(x[i], a, b);
    }
    double s = 0;
    for (int i = 0; i < 16; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_mfma(int iters, double *out) { mfma_loop(iters, out); }
__global__ __launch_bounds__(256) void k_valu(int iters, double *out) { valu_loop(iters, out); }
__global__ __launch_bounds__(512) void k_mixed(int mi, int vi, double *out) {
    if ((threadIdx.x >> 6) < 4)
        mfma_loop(mi, out);
    else
        valu_loop(vi, out);
}
__global__ __launch_bounds__(512) void k_mfma8(int iters, double *out) { mfma_loop(iters, out); }

// K1's load pattern: 8 row-groups x 16 B per lane per 8-column block, ring of P=4
__global__ __launch_bounds__(256, 1) void k_stream(const double *X, long ld, int n, long d, int S,
                                                   long kc, double *out) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, rr = lane & 15, g = lane >> 4;
    const int task = blockIdx.x * 4 + wave;
    const int u = task % 36, s = task / 36;
    if (s >= S) return;
    int bi = 0, off = 0;
    while (u >= off + (8 - bi)) { off += 8 - bi; ++bi; }
    const int bj = bi + (u - off);
    const long k0 = (long)s * kc, k1 = min(d, k0 + kc);
    const double *p[8];
    for (int i = 0; i < 4; ++i) {
        p[i] = X + (long)(bi * 64 + i * 16 + rr) * ld + k0 + 2 * g;
        p[4 + i] = X + (long)(bj * 64 + i * 16 + rr) * ld + k0 + 2 * g;
    }
    const long nb = (k1 - k0) >> 3;
    d2v acc = {0, 0};
    for (long kb = 0; kb < nb; ++kb) {
        d2v v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = *(const d2v *)(p[i] + kb * 8);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc += v[i];
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y;
}

int main() {
    int cu = 0;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    cu = prop.multiProcessorCount;
    printf("device %s, %d CUs, clock %d kHz\n", prop.name, cu, prop.clockRate);
    double *out;
    CK(hipMalloc(&out, (size_t)cu * 8 * 512 * sizeof(double)));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float ms;
    const int iters = 20000;
    for (int wpc = 1; wpc <= 2; ++wpc) {
        // MFMA: 16 MFMA x 2048 flop per wave-iteration
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(k_mfma, dim3(cu * wpc), dim3(256), 0, 0, iters, out);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
        }
        CK(hipEventElapsedTime(&ms, a, b));
        double fl = (double)cu * wpc * 4 * iters * 16 * 2048.0;
        printf("mfma f64 16x16x4, %d wave/SIMD: %.3f ms  %.2f TF/s\n", wpc, ms, fl / ms / 1e9);
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(k_valu, dim3(cu * wpc), dim3(256), 0, 0, iters / 4, out);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
        }
        CK(hipEventElapsedTime(&ms, a, b));
        fl = (double)cu * wpc * 256 * (iters / 4) * 8 * 16 * 2.0;
        printf("valu fma f64,   %d wave/SIMD: %.3f ms  %.2f TF/s\n", wpc, ms, fl / ms / 1e9);
    }
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_mixed, dim3(cu), dim3(512), 0, 0, iters, iters / 4, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
    }
    CK(hipEventElapsedTime(&ms, a, b));
    double flm = (double)cu * 4 * iters * 16 * 2048.0;
    double flv = (double)cu * 256 * (iters / 4) * 8 * 16 * 2.0;
    printf("mixed (4 mfma waves + 4 valu waves per CU): %.3f ms  %.2f TF/s (mfma part alone %.2f)\n",
           ms, (flm + flv) / ms / 1e9, flm / ms / 1e9);
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_mfma8, dim3(cu), dim3(512), 0, 0, iters, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
    }
    CK(hipEventElapsedTime(&ms, a, b));
    printf("mfma 8 waves/CU: %.2f TF/s\n", (double)cu * 8 * iters * 16 * 2048.0 / ms / 1e9);

    // stream: K1's loads for the 512 x 1M batch, 28 pieces
    const int n = 512;
    const long d = 1 << 20;
    double *X;
    CK(hipMalloc(&X, (size_t)n * d * sizeof(double)));
    CK(hipMemset(X, 0, (size_t)n * d * sizeof(double)));
    const int S = 28;
    const long kc = ((d + S - 1) / S + 7) / 8 * 8;
    const int nwg = (36 * S + 3) / 4;
    double *o2;
    CK(hipMalloc(&o2, (size_t)nwg * 256 * sizeof(double)));
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_stream, dim3(nwg), dim3(256), 0, 0, X, d, n, d, S, kc, o2);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
    }
    CK(hipEventElapsedTime(&ms, a, b));
    // requested bytes: 36 tasks per piece x 128 rows x d x 8 B
    double req = 36.0 * 128 * d * 8;
    printf("K1 load pattern alone: %.3f ms, requested %.1f GB -> %.2f TB/s to the CUs, unique %.2f GB -> %.2f TB/s\n",
           ms, req / 1e9, req / ms / 1e9, (double)n * d * 8 / 1e9, (double)n * d * 8 / ms / 1e9);
    return 0;
}
