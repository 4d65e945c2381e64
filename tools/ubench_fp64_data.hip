// tools/ubench_fp64_data.hip -- the fp64 MFMA ceiling on the DATA K1 sees.
//
// MI355X_MICROARCH.md 'DVFS give-back': the chip holds its clock down under
// MFMA load, by how much depends on the energy per MFMA, and that depends on
// the operands' bits (zero-filled bf16 operands ran +19 %).  K1 multiplies
// random full-mantissa fp64 values; tools/ubench_fp64.hip's 77.9 TF/s used one
// constant operand per lane (no toggling).  Here every variant runs the same
// instruction stream -- v_mfma_f64_16x16x4_f64 back-to-back, 16 independent
// accumulators, one wave per SIMD, every CU -- for >= 2 s of back-to-back
// launches, and reports TF/s and the in-kernel clock (s_memtime over
// s_memrealtime x 100 MHz, median over workgroups), differing only in the
// operand bits:
//   const   : one constant per lane (the old ubench)
//   rand64  : random fp64 (full 52-bit mantissas), a new pair every MFMA
//   rand32w : random fp32 values widened to fp64 (29 low mantissa bits zero:
//             config E's exact path)
//   lds64   : rand64 operands re-read from LDS by ds_read_b128 at K1's rate
//             (one 16-B granule per 4 MFMAs per operand side)
//   rand64_2w, lds64_2w : the same with two waves per SIMD (512 threads, K1's
//             occupancy)
//
// hipcc --offload-arch=gfx950 -O3 tools/ubench_fp64_data.hip -o tools/ubench_fp64_data
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef double d4v __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            printf("%s failed: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

constexpr int NOP = 16;  // operand values cycled per lane (registers)

// MODE 0: operands from registers (cycled), 1: re-read from LDS each k-step
template <int MODE, int NT>
__global__ __launch_bounds__(NT, 1) void k_mfma(const double *__restrict__ src, int iters,
                                                double *__restrict__ out,
                                                long long *__restrict__ clk) {
    __shared__ __attribute__((aligned(16))) double lds[NT / 64][2][64 * 8];  // per wave: A, B
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const double *s = src + ((size_t)blockIdx.x * NT + threadIdx.x) * 2 * NOP;
    double a[NOP], b[NOP];
#pragma unroll
    for (int i = 0; i < NOP; ++i) {
        a[i] = s[2 * i];
        b[i] = s[2 * i + 1];
    }
    if (MODE == 1) {
        for (int i = 0; i < 8; ++i) {
            lds[wave][0][i * 64 + lane] = a[i];
            lds[wave][1][i * 64 + lane] = b[i];
        }
        __syncthreads();
    }
    d4v acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = d4v{0, 0, 0, 0};
    const long long m0 = (long long)__builtin_amdgcn_s_memtime();
    const long long r0 = (long long)__builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        if constexpr (MODE == 0) {
            // 16 x 16 MFMAs per trip, every pair of operands different from
            // the last (compile-time register indices)
#pragma unroll
            for (int r = 0; r < NOP; ++r)
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[(i + r) & (NOP - 1)],
                                                                  acc[i], 0, 0, 0);
        } else {
            // K1's ratio: one 16-B granule (ds_read_b128) per 4 MFMAs,
            // alternating the A and B sides; 16 x 16 MFMAs per trip
            d2v ga = {a[0], a[1]}, gb = {b[0], b[1]};
#pragma unroll
            for (int q = 0; q < 64; ++q) {
                const int o = ((it + q) & 3) * 128 + 2 * lane;
                if (q & 1)
                    gb = *reinterpret_cast<const d2v *>(&lds[wave][1][o]);
                else
                    ga = *reinterpret_cast<const d2v *>(&lds[wave][0][o]);
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    acc[(4 * q + i) & 15] = __builtin_amdgcn_mfma_f64_16x16x4f64(
                        i & 1 ? ga.y : ga.x, i & 2 ? gb.y : gb.x, acc[(4 * q + i) & 15], 0, 0, 0);
            }
        }
    }
    const long long m1 = (long long)__builtin_amdgcn_s_memtime();
    const long long r1 = (long long)__builtin_amdgcn_s_memrealtime();
    double t = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[(size_t)blockIdx.x * NT + threadIdx.x] = t;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = m1 - m0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

static uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

int main(int argc, char **argv) {
    const double seconds = argc > 1 ? atof(argv[1]) : 2.5;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount, grid = ncu;  // one 4-wave workgroup per CU
    const size_t nop = (size_t)grid * 512 * 2 * NOP;
    std::vector<double> h(nop);
    double *dsrc, *dout;
    long long *dclk;
    CK(hipMalloc(&dsrc, nop * sizeof(double)));
    CK(hipMalloc(&dout, (size_t)grid * 512 * sizeof(double)));
    CK(hipMalloc(&dclk, (size_t)grid * 2 * sizeof(long long)));
    std::vector<long long> hc((size_t)grid * 2);
    const int iters = 250;  // 250 x 256 = 64,000 MFMAs per wave per launch
    const char *names[] = {"const", "rand64", "rand32w", "lds64", "rand64_2w", "lds64_2w"};
    printf("{\"cus\": %d, \"results\": [", ncu);
    for (int v = 0; v < 6; ++v) {
        const int nt = v >= 4 ? 512 : 256;  // waves per CU: 4 (one per SIMD) or 8
        for (size_t i = 0; i < nop; ++i) {
            const uint64_t r = sm64(i * 7919 + 12345);
            const double u = (double)(r >> 11) * 0x1p-53;  // [0, 1): full mantissa
            double x = 0.5 + u;                              // [0.5, 1.5)
            if (v == 0) x = 1.0 + (double)((i >> 5) & 63) * 1e-3;  // one constant per lane
            if (v == 2) x = (double)(float)x;                       // fp32 widened
            h[i] = x;
        }
        CK(hipMemcpy(dsrc, h.data(), nop * sizeof(double), hipMemcpyHostToDevice));
        auto launch = [&] {
            if (v == 3)
                hipLaunchKernelGGL((k_mfma<1, 256>), dim3(grid), dim3(256), 0, 0, dsrc, iters, dout, dclk);
            else if (v == 4)
                hipLaunchKernelGGL((k_mfma<0, 512>), dim3(grid), dim3(512), 0, 0, dsrc, iters, dout, dclk);
            else if (v == 5)
                hipLaunchKernelGGL((k_mfma<1, 512>), dim3(grid), dim3(512), 0, 0, dsrc, iters, dout, dclk);
            else
                hipLaunchKernelGGL((k_mfma<0, 256>), dim3(grid), dim3(256), 0, 0, dsrc, iters, dout, dclk);
        };
        launch();
        CK(hipDeviceSynchronize());
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        // back-to-back launches for `seconds` (warm: the clock settles), then
        // a timed window of 50 launches
        const double flop_per_launch = (double)grid * (nt / 64) * iters * 256 * 2048.0;
        float ms = 0;
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        const int warm = std::max(1, (int)(seconds * 1e3 / std::max(ms, 0.01f)));
        for (int i = 0; i < warm; ++i) launch();
        CK(hipEventRecord(e0));
        for (int i = 0; i < 50; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpy(hc.data(), dclk, hc.size() * sizeof(long long), hipMemcpyDeviceToHost));
        std::vector<double> ghz;
        for (int b = 0; b < grid; ++b)
            if (hc[2 * b + 1] > 0) ghz.push_back((double)hc[2 * b] / (double)hc[2 * b + 1] * 0.1);
        std::sort(ghz.begin(), ghz.end());
        const double tf = flop_per_launch * 50 / (ms * 1e-3) / 1e12;
        printf("%s{\"operands\": \"%s\", \"tflops\": %.2f, \"frac_of_78.6\": %.4f, "
               "\"clock_ghz_median\": %.3f, \"clock_ghz_min\": %.3f, \"clock_ghz_max\": %.3f, "
               "\"warm_launches\": %d}",
               v ? ", " : "", names[v], tf, tf / 78.6, ghz[ghz.size() / 2], ghz.front(), ghz.back(),
               warm);
        fflush(stdout);
    }
    printf("]}\n");
    return 0;
}
