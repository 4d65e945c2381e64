// tools/probe_mfma_order.hip -- how v_mfma_f64_16x16x4_f64 rounds on gfx950:
// is a chain of MFMAs over k ascending the same, bit for bit, as a chain of
// fp64 FMAs over k ascending (acc = fma(a_k, b_k, acc), k = 0, 1, ...)?  If it
// is, the RONI kernels (K7, K8: sequential-FMA logits, restated by the oracle)
// can run on the matrix pipe and keep their bit-exact parity.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/probe_mfma_order.hip -o /tmp/pmo && /tmp/pmo
// Layout (fp64 16x16x4): A lane l = (row l & 15, k l >> 4); B lane l = (k l >> 4,
// col l & 15); D reg r of lane l = (row (l >> 4) + 4 r, col l & 15).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef double d4 __attribute__((ext_vector_type(4)));

// A: 16 x K row-major, B: K x 16 row-major, C0: 16 x 16 initial; out 16 x 16
__global__ void k_mfma(const double *A, const double *B, const double *C0, int K, double *out) {
    const int l = threadIdx.x;
    d4 acc;
    for (int r = 0; r < 4; ++r) acc[r] = C0[((l >> 4) + 4 * r) * 16 + (l & 15)];
    for (int k0 = 0; k0 < K; k0 += 4) {
        const double a = A[(l & 15) * K + k0 + (l >> 4)];
        const double b = B[(k0 + (l >> 4)) * 16 + (l & 15)];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
    for (int r = 0; r < 4; ++r) out[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

// the sequential FMA chain on the VALU, k ascending
__global__ void k_fma(const double *A, const double *B, const double *C0, int K, double *out) {
    const int t = threadIdx.x;  // 256 threads, one element each
    const int i = t >> 4, j = t & 15;
    double acc = C0[t];
    for (int k = 0; k < K; ++k) acc = __builtin_fma(A[i * K + k], B[k * 16 + j], acc);
    out[t] = acc;
}

static uint64_t s_state = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() {
    uint64_t z = (s_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double unif() { return (double)(rnd() >> 11) * 0x1.0p-53 * 2.0 - 1.0; }

// host references: sequential fma (k ascending), and "4 products summed exactly
// (long double is not enough in general; we use the sequential chain's ulp
// distance as the diagnostic)"
static void host_seq(const double *A, const double *B, const double *C0, int K, double *o) {
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            double acc = C0[i * 16 + j];
            for (int k = 0; k < K; ++k) acc = fma(A[i * K + k], B[k * 16 + j], acc);
            o[i * 16 + j] = acc;
        }
}

static int64_t ulpd(double a, double b) {
    int64_t x, y;
    memcpy(&x, &a, 8);
    memcpy(&y, &b, 8);
    if (x < 0) x = INT64_MIN - x;
    if (y < 0) y = INT64_MIN - y;
    return x > y ? x - y : y - x;
}

#define CK(x)                                                         \
    do {                                                              \
        if ((x) != hipSuccess) {                                      \
            fprintf(stderr, "HIP error %s at %d\n", #x, __LINE__);    \
            return 1;                                                 \
        }                                                             \
    } while (0)

static int run(const char *name, const double *A, const double *B, const double *C0, int K) {
    double *dA, *dB, *dC, *dO1, *dO2;
    CK(hipMalloc(&dA, 16 * K * 8));
    CK(hipMalloc(&dB, 16 * K * 8));
    CK(hipMalloc(&dC, 256 * 8));
    CK(hipMalloc(&dO1, 256 * 8));
    CK(hipMalloc(&dO2, 256 * 8));
    CK(hipMemcpy(dA, A, 16 * K * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B, 16 * K * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dC, C0, 256 * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, dA, dB, dC, K, dO1);
    hipLaunchKernelGGL(k_fma, dim3(1), dim3(256), 0, 0, dA, dB, dC, K, dO2);
    CK(hipDeviceSynchronize());
    double m[256], f[256], h[256];
    CK(hipMemcpy(m, dO1, sizeof(m), hipMemcpyDeviceToHost));
    CK(hipMemcpy(f, dO2, sizeof(f), hipMemcpyDeviceToHost));
    host_seq(A, B, C0, K, h);
    int eq_mf = 0, eq_fh = 0;
    int64_t maxu = 0;
    for (int t = 0; t < 256; ++t) {
        eq_mf += memcmp(&m[t], &f[t], 8) == 0;
        eq_fh += memcmp(&f[t], &h[t], 8) == 0;
        int64_t u = ulpd(m[t], f[t]);
        if (u > maxu) maxu = u;
    }
    printf("%-34s K=%4d  mfma==valu_fma %3d/256  valu==host %3d/256  max ulp(mfma,fma) %lld  [0]=%a vs %a\n",
           name, K, eq_mf, eq_fh, (long long)maxu, m[0], f[0]);
    hipFree(dA);
    hipFree(dB);
    hipFree(dC);
    hipFree(dO1);
    hipFree(dO2);
    return 0;
}

int main() {
    const int Ks[] = {4, 28, 784, 8192};
    for (int v = 0; v < 3; ++v)
        for (int ki = 0; ki < 4; ++ki) {
            const int K = Ks[ki];
            double *A = (double *)malloc(16 * K * 8), *B = (double *)malloc(16 * K * 8), C0[256];
            for (int e = 0; e < 16 * K; ++e) {
                double a = unif(), b = unif();
                if (v == 0) {  // fp32 values: exact products (the RONI case)
                    a = (double)(float)a;
                    b = (double)(float)(b * 0.01);
                } else if (v == 2) {  // wide exponent range
                    a = ldexp(a, (int)(rnd() % 40) - 20);
                    b = ldexp(b, (int)(rnd() % 40) - 20);
                }
                A[e] = a;
                B[e] = b;
            }
            for (int t = 0; t < 256; ++t) C0[t] = v == 1 ? unif() : 0.0;
            const char *nm = v == 0 ? "fp32-valued operands, C0 = 0" : v == 1 ? "full fp64, random C0" : "wide exponents, C0 = 0";
            if (run(nm, A, B, C0, K)) return 1;
            free(A);
            free(B);
        }
    // designed case: c = 1, four products of 2^-53 each.  Sequential rounding
    // (ties to even) keeps 1 every step; one rounding of the exact sum gives 1 + 2^-51.
    {
        const int K = 4;
        double A[64], B[64], C0[256];
        for (int e = 0; e < 64; ++e) A[e] = 0x1.0p-27;
        for (int e = 0; e < 64; ++e) B[e] = 0x1.0p-26;
        for (int t = 0; t < 256; ++t) C0[t] = 1.0;
        if (run("designed: 1 + 4 x 2^-53", A, B, C0, K)) return 1;
        // order probe: products +big, -big, small, small with c = 0 in k order,
        // and the same in reverse k order
        for (int e = 0; e < 64; ++e) B[e] = 1.0;
        for (int i = 0; i < 16; ++i) {
            A[i * 4 + 0] = 0x1.0p60;
            A[i * 4 + 1] = 1.0;
            A[i * 4 + 2] = -0x1.0p60;
            A[i * 4 + 3] = 1.0;
        }
        for (int t = 0; t < 256; ++t) C0[t] = 0.0;
        if (run("order: 2^60, 1, -2^60, 1", A, B, C0, K)) return 1;
    }
    return 0;
}
