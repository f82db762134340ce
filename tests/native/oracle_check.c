/* oracle_check.c -- runs the C restatement of the oracle (oracle/fa2_oracle.c) under
 * AddressSanitizer (make -C oracle asan; tests/test_asan_cpu.py).  Test
 * infrastructure only.
 *
 * Ragged shapes with more threads than heads and heads than threads, forward and
 * backward, every output checked by properties the math guarantees (O inside the
 * hull of V's rows, LSE >= the row's max score, sum_k dV = sum_q dO,
 * sum_k dK = 0), plus a direct double-precision recomputation of one head's
 * forward.  Exit status 0 = every check held; ASan aborts on a memory error. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

int oracle_fa2_forward(const float *q, const float *k, const float *v, float *o, float *lse, int B, int H, int S,
                       int D, int nthreads);
int oracle_fa2_backward(const float *q, const float *k, const float *v, const float *o, const float *dout,
                        const float *lse, float *dq, float *dk, float *dv, int B, int H, int S, int D, int nthreads);
void oracle_fa2_delta(const float *dout, const float *o, float *dvec, int B, int H, int S, int D);

static int failed = 0;
#define CHECK(c)                                                               \
    do {                                                                       \
        if (!(c)) {                                                            \
            fprintf(stderr, "check failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++failed;                                                          \
        }                                                                      \
    } while (0)

static float urand(unsigned *s) {
    *s = *s * 1664525u + 1013904223u;
    return (float)((*s >> 8) & 0xffffff) / 16777216.0f;
}

static void one_case(int B, int H, int S, int D, int nthreads) {
    const long n = (long)B * H * S * D, nl = (long)B * H * S;
    float *q = malloc(n * 4), *k = malloc(n * 4), *v = malloc(n * 4), *o = malloc(n * 4), *dout = malloc(n * 4);
    float *dq = malloc(n * 4), *dk = malloc(n * 4), *dv = malloc(n * 4), *lse = malloc(nl * 4), *dl = malloc(nl * 4);
    unsigned s = 42u + (unsigned)(S * 131 + D);
    for (long i = 0; i < n; ++i) {
        q[i] = urand(&s);
        k[i] = urand(&s);
        v[i] = urand(&s);
        dout[i] = urand(&s) - 0.5f;
    }
    CHECK(oracle_fa2_forward(q, k, v, o, lse, B, H, S, D, nthreads) == 0);
    CHECK(oracle_fa2_backward(q, k, v, o, dout, lse, dq, dk, dv, B, H, S, D, nthreads) == 0);
    oracle_fa2_delta(dout, o, dl, B, H, S, D);
    const double scale = 1.0 / sqrt((double)D);
    for (long h = 0; h < (long)B * H; ++h) {
        const long base = h * S * D;
        for (int d = 0; d < D; ++d) {
            double vmin = 1e30, vmax = -1e30, sdv = 0, sdo = 0, sdk = 0;
            for (int j = 0; j < S; ++j) {
                const double x = v[base + (long)j * D + d];
                vmin = x < vmin ? x : vmin;
                vmax = x > vmax ? x : vmax;
                sdv += dv[base + (long)j * D + d];
                sdo += dout[base + (long)j * D + d];
                sdk += dk[base + (long)j * D + d];
            }
            for (int i = 0; i < S; ++i) {
                const float x = o[base + (long)i * D + d];
                CHECK(x >= vmin - 1e-5 && x <= vmax + 1e-5);
            }
            CHECK(fabs(sdv - sdo) <= 1e-3 * (1 + fabs(sdo)));
            CHECK(fabs(sdk) <= 1e-3);
        }
        for (int i = 0; i < S; ++i) {
            double mx = -1e30;
            for (int j = 0; j < S; ++j) {
                double dot = 0;
                for (int d = 0; d < D; ++d) dot += (double)q[base + (long)i * D + d] * k[base + (long)j * D + d];
                mx = dot * scale > mx ? dot * scale : mx;
            }
            CHECK(lse[h * S + i] >= mx - 1e-4);
            CHECK(isfinite(dl[h * S + i]));
        }
    }
    /* direct recomputation of the last head's forward in double */
    {
        const long h = (long)B * H - 1, base = h * S * D;
        double *p = malloc(sizeof(double) * S);
        for (int i = 0; i < S; ++i) {
            double mx = -1e300, l = 0;
            for (int j = 0; j < S; ++j) {
                double dot = 0;
                for (int d = 0; d < D; ++d) dot += (double)q[base + (long)i * D + d] * k[base + (long)j * D + d];
                p[j] = dot * scale;
                mx = p[j] > mx ? p[j] : mx;
            }
            for (int j = 0; j < S; ++j) l += (p[j] = exp(p[j] - mx));
            CHECK(fabs(lse[h * S + i] - (mx + log(l))) <= 1e-5);
            for (int d = 0; d < D; ++d) {
                double acc = 0;
                for (int j = 0; j < S; ++j) acc += p[j] * v[base + (long)j * D + d];
                CHECK(fabs(o[base + (long)i * D + d] - acc / l) <= 1e-5);
            }
        }
        free(p);
    }
    free(q); free(k); free(v); free(o); free(dout); free(dq); free(dk); free(dv); free(lse); free(dl);
}

int main(void) {
    one_case(1, 1, 1, 32, 1);
    one_case(1, 2, 33, 32, 4);
    one_case(2, 3, 100, 64, 3);
    one_case(1, 1, 77, 128, 8);
    one_case(1, 5, 65, 64, 2);
    CHECK(oracle_fa2_forward(NULL, NULL, NULL, NULL, NULL, 0, 1, 1, 64, 1) == -1);
    printf("oracle_check: %s (%d failed)\n", failed ? "FAIL" : "ok", failed);
    return failed ? 1 : 0;
}
