/*
 * fa2_oracle.c -- plain-C CPU restatement of the FA2 forward+backward.
 *
 * TEST INFRASTRUCTURE ONLY (checker + the "port" CPU baseline of bench.py).
 * Nothing under cuda-flash-attention_amd/ links or calls this file.
 *
 * Restates the reference's algorithm (detker/CUDA-Flash-Attention):
 *   forward  : O = softmax(Q K^T / sqrt(D)) V, LSE = ln(sum exp) + max
 *              test_flash_attention2.py:197-208 (math), :917-921 (LSE);
 *              kernel_fa2_optimized.cu:336-343 (what the kernel writes).
 *   delta    : D_i = sum_d dO_id * O_id        f-attn2-backward.cu:341-380
 *   backward : P = exp(S/sqrt(D) - LSE)         f-attn2-backward.cu:151-184
 *              dV += P^T dO                     f-attn2-backward.cu:218-240
 *              dS = P * (dO V^T - D_i)/sqrt(D)  f-attn2-backward.cu:242-267
 *              dQ += dS K                       f-attn2-backward.cu:269-301
 *              dK += dS^T Q                     f-attn2-backward.cu:303-323
 * Layout: fp32 [B,H,S,D] row-major; LSE and D are [B,H,S].
 * Dot products accumulate in double; one worker thread per (b,h) head.
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    const float *q, *k, *v, *o, *dout, *lse;
    float *out, *lse_out, *dq, *dk, *dv;
    int S, D, backward;
    int next_head, n_heads;
    pthread_mutex_t mu;
} job_t;

static double dotf(const float *a, const float *b, int n) {
    double acc = 0.0;
    for (int i = 0; i < n; ++i) acc += (double)a[i] * (double)b[i];
    return acc;
}

static void fwd_head(const job_t *j, long base, double *s, double *acc) {
    const int S = j->S, D = j->D;
    const double inv = 1.0 / sqrt((double)D);
    for (int i = 0; i < S; ++i) {
        const float *qi = j->q + base + (long)i * D;
        double m = -INFINITY;
        for (int c = 0; c < S; ++c) {
            s[c] = dotf(qi, j->k + base + (long)c * D, D) * inv;
            if (s[c] > m) m = s[c];
        }
        double l = 0.0;
        for (int d = 0; d < D; ++d) acc[d] = 0.0;
        for (int c = 0; c < S; ++c) {
            const double p = exp(s[c] - m);
            const float *vc = j->v + base + (long)c * D;
            l += p;
            for (int d = 0; d < D; ++d) acc[d] += p * (double)vc[d];
        }
        float *oi = j->out + base + (long)i * D;
        for (int d = 0; d < D; ++d) oi[d] = (float)(acc[d] / l);
        j->lse_out[base / D + i] = (float)(m + log(l));
    }
}

static void bwd_head(const job_t *j, long base, double *s, double *acc) {
    const int S = j->S, D = j->D;
    const double inv = 1.0 / sqrt((double)D);
    double *dk = acc + D;             /* [S][D] */
    double *dv = dk + (long)S * D;    /* [S][D] */
    memset(dk, 0, sizeof(double) * 2 * (size_t)S * D);
    for (int i = 0; i < S; ++i) {
        const float *qi = j->q + base + (long)i * D;
        const float *doi = j->dout + base + (long)i * D;
        const double lse_i = j->lse[base / D + i];
        const double di = dotf(doi, j->o + base + (long)i * D, D);
        for (int d = 0; d < D; ++d) acc[d] = 0.0;
        for (int c = 0; c < S; ++c) {
            const float *kc = j->k + base + (long)c * D;
            const float *vc = j->v + base + (long)c * D;
            const double p = exp(dotf(qi, kc, D) * inv - lse_i);
            const double ds = p * (dotf(doi, vc, D) - di) * inv;
            double *dkc = dk + (long)c * D, *dvc = dv + (long)c * D;
            for (int d = 0; d < D; ++d) {
                acc[d] += ds * (double)kc[d];
                dkc[d] += ds * (double)qi[d];
                dvc[d] += p * (double)doi[d];
            }
        }
        float *dqi = j->dq + base + (long)i * D;
        for (int d = 0; d < D; ++d) dqi[d] = (float)acc[d];
    }
    for (long x = 0; x < (long)S * D; ++x) {
        j->dk[base + x] = (float)dk[x];
        j->dv[base + x] = (float)dv[x];
    }
    (void)s;
}

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    const int S = j->S, D = j->D;
    double *s = (double *)malloc(sizeof(double) * (size_t)S);
    double *acc = (double *)malloc(sizeof(double) * ((size_t)D + 2 * (size_t)S * D));
    for (;;) {
        pthread_mutex_lock(&j->mu);
        const int h = j->next_head++;
        pthread_mutex_unlock(&j->mu);
        if (h >= j->n_heads) break;
        const long base = (long)h * S * D;
        if (j->backward) bwd_head(j, base, s, acc);
        else fwd_head(j, base, s, acc);
    }
    free(s);
    free(acc);
    return NULL;
}

static int run(job_t *j, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > j->n_heads) nthreads = j->n_heads;
    pthread_t tid[256];
    if (nthreads > 256) nthreads = 256;
    pthread_mutex_init(&j->mu, NULL);
    for (int t = 0; t < nthreads; ++t) pthread_create(&tid[t], NULL, worker, j);
    for (int t = 0; t < nthreads; ++t) pthread_join(tid[t], NULL);
    pthread_mutex_destroy(&j->mu);
    return 0;
}

int oracle_fa2_forward(const float *q, const float *k, const float *v, float *o, float *lse,
                       int B, int H, int S, int D, int nthreads) {
    if (B <= 0 || H <= 0 || S <= 0 || D <= 0) return -1;
    job_t j;
    memset(&j, 0, sizeof j);
    j.q = q; j.k = k; j.v = v; j.out = o; j.lse_out = lse;
    j.S = S; j.D = D; j.n_heads = B * H;
    return run(&j, nthreads);
}

int oracle_fa2_backward(const float *q, const float *k, const float *v, const float *o,
                        const float *dout, const float *lse, float *dq, float *dk, float *dv,
                        int B, int H, int S, int D, int nthreads) {
    if (B <= 0 || H <= 0 || S <= 0 || D <= 0) return -1;
    job_t j;
    memset(&j, 0, sizeof j);
    j.q = q; j.k = k; j.v = v; j.o = o; j.dout = dout; j.lse = lse;
    j.dq = dq; j.dk = dk; j.dv = dv;
    j.S = S; j.D = D; j.n_heads = B * H; j.backward = 1;
    return run(&j, nthreads);
}

void oracle_fa2_delta(const float *dout, const float *o, float *dvec, int B, int H, int S, int D) {
    const long rows = (long)B * H * S;
    for (long r = 0; r < rows; ++r) dvec[r] = (float)dotf(dout + r * D, o + r * D, D);
}
