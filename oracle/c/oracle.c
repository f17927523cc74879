/*
 * CPU oracle, C part — TEST INFRASTRUCTURE (see oracle/__init__.py).
 *
 * Scalar C restatements of the reference's fp32 arithmetic, compiled with
 * -ffp-contract=off so that every a*b and a+b rounds once and every fused
 * multiply-add is an explicit fmaf().  Used by tests/ and bench.py's
 * cpu_baseline only.  Built by oracle/Makefile (gcc) into oracle/_build/.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

/* FedServer.get_subset_model, servers/fed_server.py:44-66:
 *   tmp = p * n_i / N ; first client assigns, later ones accumulate (:62-65). */
void orc_fedavg_ref(const float *U, int64_t ldu, const int32_t *order, const int64_t *n,
                    int32_t K, int64_t P, float *out) {
    int64_t total = 0;
    for (int32_t j = 0; j < K; ++j) total += n[order[j]];
    const float N = (float)total;
    for (int32_t j = 0; j < K; ++j) {
        const float *row = U + (int64_t)order[j] * ldu;
        const float w = (float)n[order[j]];
        if (j == 0) {
            for (int64_t e = 0; e < P; ++e) out[e] = (row[e] * w) / N;
        } else {
            for (int64_t e = 0; e < P; ++e) out[e] = out[e] + (row[e] * w) / N;
        }
    }
}

/* FedQuantServer._process_client_parameter, servers/fed_quant_server.py:25-33:
 *   weight = weight.float(); weight[c] = (weight[c] - zp[c]) * scale[c]
 * torch casts the 0-dim float64 scale / int64 zero point to fp32 first. */
void orc_dequant_rows(const int32_t *q, int64_t C, int64_t row_len, const double *scale,
                      const int64_t *zp, float *out) {
    for (int64_t c = 0; c < C; ++c) {
        const float s = (float)scale[c];
        const float z = (float)zp[c];
        for (int64_t e = 0; e < row_len; ++e) {
            const float v = (float)q[c * row_len + e];
            out[c * row_len + e] = (v - z) * s;
        }
    }
}

/* workers/sign_sgd_worker.py:32-42 (momentum / dampening / nesterov).
 * buf.mul_(m).add_(g, alpha=1-d) == fma(g, fl32(1-d), fl32(buf*m));
 * g.add(buf, alpha=m) == fma(buf, fl32(m), g). */
void orc_sign_direction(const float *g, float *buf, float *d, int64_t P, double momentum,
                        double dampening, int32_t nesterov, int32_t first) {
    const float m = (float)momentum, a = (float)(1.0 - dampening);
    for (int64_t e = 0; e < P; ++e) {
        if (momentum == 0.0) {
            d[e] = g[e];
            continue;
        }
        float b = first ? g[e] : fmaf(g[e], a, buf[e] * m);
        buf[e] = b;
        d[e] = nesterov ? fmaf(b, m, g[e]) : b;
    }
}

/* workers/sign_sgd_worker.py:48-57: d = vote (+ wd*p) ; p += -lr * d. */
void orc_sign_apply(float *p, const float *vote, int64_t P, double lr, double wd) {
    const float nlr = (float)(-lr), w = (float)wd;
    for (int64_t e = 0; e < P; ++e) {
        float d = vote[e];
        if (wd != 0.0) d = fmaf(p[e], w, d);
        p[e] = fmaf(d, nlr, p[e]);
    }
}

/* Exhaustive check of the kernels' division a/b -> q0=a*y; r=fma(-q0,b,a);
 * q=fma(r,y,q0) with y=RN(1/b), over every fp32 mantissa of a in [1,2).
 * FP ops are scale-invariant away from under/overflow, so a zero return
 * proves the kernel's guarded fast path for this b. Returns mismatches. */
int64_t orc_fastdiv_check(float b) {
    const float y = (float)(1.0 / (double)b);
    int64_t bad = 0;
    for (uint32_t m = 0; m < (1u << 23); ++m) {
        uint32_t u = 0x3f800000u | m;
        float a;
        memcpy(&a, &u, 4);
        const float q0 = a * y;
        const float r = fmaf(-q0, b, a);
        const float q = fmaf(r, y, q0);
        if (q != a / b) ++bad;
    }
    return bad;
}
