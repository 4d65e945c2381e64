// bk_synth.h -- synthetic update batches (spec: DESIGN.md "Synthetic inputs").
//
// Counter-based: element (original row r, column c) depends only on
// (seed, r, c, d_total), so any column shard of the batch can be generated on
// the GPU that owns it.  SplitMix64 hashing + Irwin-Hall(4) standardised
// normals; IEEE add/mul only (the library is built with -ffp-contract=off), so
// the device output is bit-identical to oracle/krum_oracle.c and the numpy spec
// in tests/golden/synth_np.py.
//
// Shape of the batch: honest rows mu + sigma*z, Byzantine
// rows (original index >= n - nbyz, cf. the POISONING index rule at
// DistSys/main.go:839-843) mu + byz_scale*z1 + sigma*z, then rows shuffled by a
// seeded Fisher-Yates permutation.  BK_SYNTH_FP32ROUND mimics mnist deltas that
// are fp32 gradients widened to fp64 (ML/Pytorch/client.py:61-64) plus fp64
// noise (DistSys/main.go:1530-1537).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define BK_HD __host__ __device__ __forceinline__
#else
#define BK_HD static inline
#endif

namespace bk {

BK_HD uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

BK_HD uint64_t stream_base(uint64_t seed, uint64_t stream) {
    return sm64(sm64(seed) ^ (stream * 0xD1B54A32D192ED03ULL));
}

BK_HD double u01(uint64_t h) { return (double)(h >> 11) * 0x1.0p-53; }

BK_HD double gauss(uint64_t base, uint64_t idx) {
    const uint64_t c = base + 4ULL * idx;
    const double u0 = u01(sm64(c)), u1 = u01(sm64(c + 1));
    const double u2 = u01(sm64(c + 2)), u3 = u01(sm64(c + 3));
    const double s01 = u0 + u1;
    const double s23 = u2 + u3;
    const double s = s01 + s23;
    const double t = s - 2.0;
    return t * 1.7320508075688772;
}

struct SynthParams {
    uint64_t b0, b1, b2, b4;   // stream bases: mu, byzantine shift, row noise, fp32-round noise
    int64_t n, nbyz, d_total;
    double mu_scale, byz_scale, sigma;
    int flags;
};

BK_HD double synth_elem(const SynthParams &P, int64_t r, int64_t c) {
    const double mu = P.mu_scale * gauss(P.b0, (uint64_t)c);
    double base = mu;
    if (r >= P.n - P.nbyz) {
        const double sh = P.byz_scale * gauss(P.b1, (uint64_t)c);
        base = mu + sh;
    }
    const uint64_t e = (uint64_t)r * (uint64_t)P.d_total + (uint64_t)c;
    const double nz = P.sigma * gauss(P.b2, e);
    double x = base + nz;
    if (P.flags & 1) {
        const double w = (double)(float)x;
        const double nz2 = 1e-6 * gauss(P.b4, e);
        x = w + nz2;
    }
    return x;
}

}  // namespace bk
