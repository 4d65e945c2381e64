// Probe: how fast can a kernel read PINNED HOST memory over PCIe (zero-copy),
// against the copy engine's H2D of the same bytes?  The question behind it:
// could the host small path (bk_multikrum at config B, 100 x 7850 fp64 =
// 6.28 MB) let k_small's G items read the caller's pinned batch directly, so
// the Gram overlaps the transfer, instead of an H2D copy followed by the kernel?
//
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_zc.hip -o tools/ubench_zc
//   ./tools/ubench_zc            (prints one line per case)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

// every workgroup reads a contiguous slice, all of its 16-B loads in flight
// (U per thread per round), and writes one partial sum (so nothing is elided)
template <int U>
__global__ __launch_bounds__(512) void k_read(const d2 *src, size_t n16, double *out) {
    const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const size_t b0 = per * blockIdx.x, b1 = b0 + per < n16 ? b0 + per : n16;
    double acc = 0.0;
    for (size_t i = b0 + threadIdx.x; i < b1; i += 512 * U) {
        d2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t j = i + 512 * (size_t)u;
            v[u] = j < b1 ? src[j] : d2{0.0, 0.0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y;
    }
    if (acc == 12345.678) out[blockIdx.x] = acc;  // practically never: keeps the loads
}

static float time_kernel(const d2 *src, size_t n16, double *out, int grid, int reps, hipStream_t st) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_read<8>), dim3(grid), dim3(512), 0, st, src, n16, out);
    CK(hipEventRecord(a, st));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_read<8>), dim3(grid), dim3(512), 0, st, src, n16, out);
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    double *out;
    CK(hipMalloc(&out, 4096 * sizeof(double)));
    const size_t sizes[] = {(size_t)100 * 7850 * 8, (size_t)64 << 20};
    const unsigned flags[] = {hipHostMallocNonCoherent, hipHostMallocCoherent};
    const char *fname[] = {"noncoherent", "coherent"};
    for (size_t bytes : sizes) {
        const size_t n16 = bytes / 16;
        void *dev;
        CK(hipMalloc(&dev, bytes));
        for (int fi = 0; fi < 2; ++fi) {
            void *h;
            CK(hipHostMalloc(&h, bytes, hipHostMallocMapped | flags[fi]));
            for (size_t i = 0; i < bytes / 8; ++i) ((double *)h)[i] = (double)(i % 1000);
            void *hd;
            CK(hipHostGetDevicePointer(&hd, h, 0));
            // copy engine H2D of the same bytes
            hipEvent_t a, b;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&b));
            for (int w = 0; w < 3; ++w) CK(hipMemcpyAsync(dev, h, bytes, hipMemcpyHostToDevice, st));
            const int reps = bytes < (8u << 20) ? 50 : 10;
            CK(hipEventRecord(a, st));
            for (int r = 0; r < reps; ++r) CK(hipMemcpyAsync(dev, h, bytes, hipMemcpyHostToDevice, st));
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float cms;
            CK(hipEventElapsedTime(&cms, a, b));
            cms /= reps;
            printf("%-11s %9zu B  H2D copy %8.1f us %6.1f GB/s |", fname[fi], bytes, cms * 1e3,
                   bytes / (cms * 1e-3) / 1e9);
            for (int grid : {64, 128, 256, 1024}) {
                const float ms = time_kernel((const d2 *)hd, n16, out, grid, reps, st);
                printf("  zc grid %4d %8.1f us %6.1f GB/s", grid, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
            }
            // the same kernel on device memory, for scale
            const float dms = time_kernel((const d2 *)dev, n16, out, 256, reps, st);
            printf("  | device %6.1f us\n", dms * 1e3);
            CK(hipHostFree(h));
        }
        CK(hipFree(dev));
    }
    return 0;
}
