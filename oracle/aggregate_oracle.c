/*
 * oracle/aggregate_oracle.c -- CPU restatement of the steps either side of
 * Biscotti's Krum verifier.
 *
 * TEST INFRASTRUCTURE ONLY (see krum_oracle.c's header): tests/ use it as the
 * checker; nothing in biscotti_amd/ links, loads or calls it.
 *
 * Restated from the Go reference (@ /root/reference, DistributedML/Biscotti):
 *   oracle_aggregate   Honest.createBlock update loop, DistSys/honest.go:360-375:
 *                      pulledGradientM.Add(pulledGradientM, deltaM) for every
 *                      accepted update in blockUpdates order -- one IEEE fp64
 *                      add per element per update, left to right.
 *   oracle_qsum        updateFloatToInt, DistSys/kyber.go:698-710:
 *                      int64(update[i] * math.Pow(10, precision)); the miners
 *                      sum the shares of the accepted updates (honest.go:401-409,
 *                      442-502); updateIntToFloat, kyber.go:745-757:
 *                      float64(v) / math.Pow(10, precision).  Go's int64(float64)
 *                      on amd64 is CVTTSD2SQ: truncation toward zero, NaN and
 *                      out-of-range -> 0x8000000000000000.  int64 sums wrap.
 *   oracle_noise       requestNoiseFromNoisers, DistSys/main.go:1606-1653
 *                      (noiseVec starts at 0, += each received vector in
 *                      order, then /= noisesReceived as float64), and
 *                      NoisedDelta = Delta + noise, main.go:1524-1537.
 *
 * PARITY PINNING: the Go reference cannot be built here (no Go toolchain,
 * go-python unvendored) and the reference holds no tests or
 * fixtures for these functions, so this restatement is "parity unpinned" by
 * the reference itself.  It is pinned by the Go language's IEEE-754 semantics
 * (no FMA contraction in these loops, sequential order as written) and by
 * hand-checked known answers in tests/test_aggregate_oracle.py.
 *
 * Compiled with -ffp-contract=off (oracle/Makefile).
 */
#include <math.h>
#include <stdint.h>

int64_t oracle_go_f64_to_i64(double y)
{
    if (y >= -9223372036854775808.0 && y < 9223372036854775808.0) return (int64_t)y;
    return INT64_MIN;
}

double oracle_pow10(int p)
{
    /* Go's math.Pow(10, p) for 0 <= p <= 22: exact (every partial product is an
     * integer below 2^53, or 10^p itself is exactly representable) */
    double s = 1.0;
    for (int i = 0; i < p; ++i) s *= 10.0;
    return s;
}

void oracle_aggregate(const double *X, int64_t d, int64_t ld, const int64_t *idx, int64_t m,
                      double *global)
{
    for (int64_t r = 0; r < m; ++r) {
        const double *row = X + idx[r] * ld;
        for (int64_t c = 0; c < d; ++c) global[c] = global[c] + row[c];
    }
}

void oracle_qsum(const double *X, int64_t d, int64_t ld, const int64_t *idx, int64_t m,
                 int precision, int64_t *sum, double *sumf)
{
    const double scale = oracle_pow10(precision);
    for (int64_t c = 0; c < d; ++c) {
        uint64_t acc = 0;
        for (int64_t r = 0; r < m; ++r)
            acc += (uint64_t)oracle_go_f64_to_i64(X[idx[r] * ld + c] * scale);
        sum[c] = (int64_t)acc;
        if (sumf) sumf[c] = (double)(int64_t)acc / scale;
    }
}

void oracle_noise(const double *delta, int64_t n, int64_t d, int64_t ld, const double *noise,
                  int64_t k, int64_t nld, double *out, int64_t old)
{
    const double dk = (double)k;
    for (int64_t i = 0; i < n; ++i)
        for (int64_t c = 0; c < d; ++c) {
            double s = 0.0;
            for (int64_t j = 0; j < k; ++j) s += noise[(i * k + j) * nld + c];
            s /= dk;
            out[i * old + c] = delta[i * ld + c] + s;
        }
}
