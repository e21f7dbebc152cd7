/*
 * fa_cpu.c — CPU restatement ("port") of the reference's threaded blockwise
 * forward dense_fa!(O, l, m, Q, K, V), src/dense.jl:21-102.
 *
 * TEST INFRASTRUCTURE ONLY: used by tests/ as a second oracle and by
 * bench.py's cpu_baseline leg as the reference-CPU-path stand-in (the Julia
 * reference cannot run here or on the GPU box: no Julia; and the reference's
 * own C++ src_cpp/FlashAttention.cpp needs Eigen3, which the image lacks, so
 * it is unbuildable — DESIGN.md).  Never linked into the product library.
 *
 * Faithful to the reference algorithm:
 *   - tile policy Bc = clamp(cld(M, d), 1, N), Br = clamp(min(d, cld(M, d)), 1, N),
 *     M = 32000 (src/dense.jl:28-36): d = 64 -> Br = 64, Bc = 500;
 *   - parallel over (batch x row-block) tasks (src/dense.jl:45), OpenMP here
 *     instead of Julia tasks;
 *   - per tile: S = tau Qi Kj^T (:77), rowmax (:78), P = exp(S - mij) (:79),
 *     rowsum (:80), running-stat update (:82-85), Oi = (li ei Oi + eij Pij Vj)
 *     / li_new with O kept normalised every step (:88-89);
 *   - tau = 1/sqrt(d) in the element type (:43); l, m in the element type.
 * Layout: Julia column-major (N, d, B): X[n + N*k + N*d*b].
 * The two GEMMs are plain loops over row-major gathered tiles (the reference
 * calls BLAS through NNlib.batched_mul!, :77/:88); arithmetic order differs
 * from BLAS only in summation order.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#define CACHE_M 32000

static int64_t cld64(int64_t a, int64_t b) { return (a + b - 1) / b; }
static int64_t clamp64(int64_t x, int64_t lo, int64_t hi) { return x < lo ? lo : (x > hi ? hi : x); }

#define DEFINE_FA_CPU(REAL, SUFFIX, EXP)                                                         \
int fa_cpu_dense_fwd_##SUFFIX(const REAL* Q, const REAL* K, const REAL* V, REAL* O, REAL* l,       \
                              REAL* m, int64_t N, int64_t Nk, int64_t d, int64_t dv, int64_t B,    \
                              int nthreads) {                                                     \
    if (N < 1 || Nk < 1 || d < 1 || dv < 1 || B < 1) return 1;                                    \
    const int64_t Bc = clamp64(cld64(CACHE_M, d), 1, Nk);                                        \
    const int64_t Br = clamp64(cld64(CACHE_M, d) < d ? cld64(CACHE_M, d) : d, 1, N);             \
    const int64_t Tr = cld64(N, Br), Tc = cld64(Nk, Bc);                                          \
    const REAL tau = (REAL)1 / (REAL)sqrt((double)d);                                             \
    if (nthreads > 0) omp_set_num_threads(nthreads);                                              \
    int err = 0;                                                                                  \
    _Pragma("omp parallel")                                                                       \
    {                                                                                             \
        REAL* Qt = (REAL*)malloc(sizeof(REAL) * Br * d);                                           \
        REAL* Kt = (REAL*)malloc(sizeof(REAL) * Bc * d);                                           \
        REAL* Vt = (REAL*)malloc(sizeof(REAL) * Bc * dv);                                          \
        REAL* P = (REAL*)malloc(sizeof(REAL) * Br * Bc);                                           \
        REAL* Oi = (REAL*)malloc(sizeof(REAL) * Br * dv);                                          \
        REAL* On = (REAL*)malloc(sizeof(REAL) * Br * dv);                                          \
        REAL* li = (REAL*)malloc(sizeof(REAL) * Br);                                               \
        REAL* mi = (REAL*)malloc(sizeof(REAL) * Br);                                               \
        if (!Qt || !Kt || !Vt || !P || !Oi || !On || !li || !mi) {                                 \
            _Pragma("omp atomic write") err = 2;                                                   \
        } else {                                                                                  \
            _Pragma("omp for collapse(2) schedule(dynamic, 1)")                                    \
            for (int64_t b = 0; b < B; ++b)                                                       \
                for (int64_t i = 0; i < Tr; ++i) {                                                \
                    const REAL* Qb = Q + N * d * b;                                                \
                    const REAL* Kb = K + Nk * d * b;                                               \
                    const REAL* Vb = V + Nk * dv * b;                                              \
                    const int64_t r0 = i * Br, nr = (r0 + Br <= N ? Br : N - r0);                  \
                    for (int64_t r = 0; r < nr; ++r)                                               \
                        for (int64_t k = 0; k < d; ++k) Qt[r * d + k] = Qb[k * N + r0 + r];        \
                    for (int64_t r = 0; r < nr; ++r) { li[r] = 0; mi[r] = -INFINITY; }             \
                    memset(Oi, 0, sizeof(REAL) * nr * dv);                                         \
                    for (int64_t j = 0; j < Tc; ++j) {                                            \
                        const int64_t c0 = j * Bc, nc = (c0 + Bc <= Nk ? Bc : Nk - c0);            \
                        for (int64_t c = 0; c < nc; ++c) {                                         \
                            for (int64_t k = 0; k < d; ++k) Kt[c * d + k] = Kb[k * Nk + c0 + c];   \
                            for (int64_t x = 0; x < dv; ++x) Vt[c * dv + x] = Vb[x * Nk + c0 + c]; \
                        }                                                                         \
                        for (int64_t r = 0; r < nr; ++r) {                                         \
                            const REAL* qr = Qt + r * d;                                           \
                            REAL* pr = P + r * Bc;                                                 \
                            REAL mij = -INFINITY;                                                  \
                            for (int64_t c = 0; c < nc; ++c) {                                     \
                                const REAL* kc = Kt + c * d;                                       \
                                REAL acc = 0;                                                      \
                                _Pragma("omp simd reduction(+:acc)")                               \
                                for (int64_t k = 0; k < d; ++k) acc += qr[k] * kc[k];              \
                                pr[c] = tau * acc;                                                 \
                                mij = pr[c] > mij ? pr[c] : mij;                                   \
                            }                                                                     \
                            REAL lij = 0;                                                          \
                            for (int64_t c = 0; c < nc; ++c) { pr[c] = EXP(pr[c] - mij); lij += pr[c]; } \
                            const REAL mnew = mi[r] > mij ? mi[r] : mij;                           \
                            const REAL ei = EXP(mi[r] - mnew), eij = EXP(mij - mnew);              \
                            const REAL lnew = ei * li[r] + eij * lij;                              \
                            REAL* on = On + r * dv;                                                \
                            for (int64_t x = 0; x < dv; ++x) on[x] = 0;                            \
                            for (int64_t c = 0; c < nc; ++c) {                                     \
                                const REAL pc = pr[c];                                             \
                                const REAL* vc = Vt + c * dv;                                      \
                                _Pragma("omp simd")                                                \
                                for (int64_t x = 0; x < dv; ++x) on[x] += pc * vc[x];              \
                            }                                                                     \
                            REAL* oi = Oi + r * dv;                                                \
                            const REAL a = li[r] * ei, bb = eij;                                   \
                            for (int64_t x = 0; x < dv; ++x) oi[x] = (a * oi[x] + bb * on[x]) / lnew; \
                            li[r] = lnew; mi[r] = mnew;                                            \
                        }                                                                         \
                    }                                                                             \
                    REAL* Ob = O + N * dv * b;                                                     \
                    for (int64_t r = 0; r < nr; ++r) {                                             \
                        for (int64_t x = 0; x < dv; ++x) Ob[x * N + r0 + r] = Oi[r * dv + x];     \
                        l[N * b + r0 + r] = li[r];                                                 \
                        m[N * b + r0 + r] = mi[r];                                                 \
                    }                                                                             \
                }                                                                                 \
        }                                                                                         \
        free(Qt); free(Kt); free(Vt); free(P); free(Oi); free(On); free(li); free(mi);             \
    }                                                                                             \
    return err;                                                                                   \
}

DEFINE_FA_CPU(float, f32, expf)
DEFINE_FA_CPU(double, f64, exp)


/*
 * BLAS-backed port — the reference's arithmetic structure exactly: per task
 * (slab b, row block i) and key tile j, Pij = tau * Qi * Kj^T is ONE gemm on
 * the strided views (batched_mul!, src/dense.jl:77), then the row max / exp /
 * row sum / stat update broadcasts (:78-86), Oi_new = Pij * Vj one gemm (:88)
 * and the renormalised blend (:89).  The reference's BLAS is whatever Julia
 * links (OpenBLAS by default); here the CBLAS entry points are passed in at
 * run time (fa_cpu_set_blas) — numpy's bundled OpenBLAS, resolved by
 * oracle/cpu_port.py — so nothing is linked at build time.  BLAS runs
 * single-threaded inside each OpenMP task (the tasks are the parallelism, as
 * the reference's @threads loop, :45).
 */
typedef void (*gemm32_fn)(int, int, int, int64_t, int64_t, int64_t, float, const float*, int64_t,
                          const float*, int64_t, float, float*, int64_t);
typedef void (*gemm64_fn)(int, int, int, int64_t, int64_t, int64_t, double, const double*, int64_t,
                          const double*, int64_t, double, double*, int64_t);
typedef void (*set_threads_fn)(int);
static gemm32_fn g_sgemm = 0;
static gemm64_fn g_dgemm = 0;
static set_threads_fn g_blas_threads = 0;

int fa_cpu_set_blas(void* sgemm, void* dgemm, void* set_threads) {
    g_sgemm = (gemm32_fn)sgemm;
    g_dgemm = (gemm64_fn)dgemm;
    g_blas_threads = (set_threads_fn)set_threads;
    return (g_sgemm && g_dgemm) ? 0 : 1;
}

enum { CB_COL = 102, CB_N = 111, CB_T = 112 };

#define DEFINE_FA_CPU_BLAS(REAL, SUFFIX, EXP, GEMM)                                               \
int fa_cpu_dense_fwd_blas_##SUFFIX(const REAL* Q, const REAL* K, const REAL* V, REAL* O, REAL* l,  \
                                   REAL* m, int64_t N, int64_t Nk, int64_t d, int64_t dv,         \
                                   int64_t B, int nthreads) {                                     \
    if (!GEMM) return 3;                                                                          \
    if (N < 1 || Nk < 1 || d < 1 || dv < 1 || B < 1) return 1;                                    \
    const int64_t Bc = clamp64(cld64(CACHE_M, d), 1, Nk);                                        \
    const int64_t Br = clamp64(cld64(CACHE_M, d) < d ? cld64(CACHE_M, d) : d, 1, N);             \
    const int64_t Tr = cld64(N, Br), Tc = cld64(Nk, Bc);                                          \
    const REAL tau = (REAL)1 / (REAL)sqrt((double)d);                                             \
    if (g_blas_threads) g_blas_threads(1);                                                        \
    if (nthreads > 0) omp_set_num_threads(nthreads);                                              \
    int err = 0;                                                                                  \
    _Pragma("omp parallel")                                                                       \
    {                                                                                             \
        REAL* P = (REAL*)malloc(sizeof(REAL) * Br * Bc);                                           \
        REAL* On = (REAL*)malloc(sizeof(REAL) * Br * dv);                                          \
        REAL* mij = (REAL*)malloc(sizeof(REAL) * Br);                                              \
        REAL* lij = (REAL*)malloc(sizeof(REAL) * Br);                                              \
        if (!P || !On || !mij || !lij) {                                                          \
            _Pragma("omp atomic write") err = 2;                                                   \
        } else {                                                                                  \
            _Pragma("omp for collapse(2) schedule(dynamic, 1)")                                    \
            for (int64_t b = 0; b < B; ++b)                                                       \
                for (int64_t i = 0; i < Tr; ++i) {                                                \
                    const int64_t r0 = i * Br, nr = (r0 + Br <= N ? Br : N - r0);                  \
                    const REAL* Qi = Q + N * d * b + r0;                                           \
                    REAL* Oi = O + N * dv * b + r0;                                                \
                    REAL* li = l + N * b + r0;                                                     \
                    REAL* mi = m + N * b + r0;                                                     \
                    for (int64_t x = 0; x < dv; ++x)                                               \
                        for (int64_t r = 0; r < nr; ++r) Oi[x * N + r] = 0;                        \
                    for (int64_t r = 0; r < nr; ++r) { li[r] = 0; mi[r] = -INFINITY; }             \
                    for (int64_t j = 0; j < Tc; ++j) {                                            \
                        const int64_t c0 = j * Bc, nc = (c0 + Bc <= Nk ? Bc : Nk - c0);            \
                        const REAL* Kj = K + Nk * d * b + c0;                                      \
                        const REAL* Vj = V + Nk * dv * b + c0;                                     \
                        /* Pij (nr x nc, col-major) = tau Qi Kj^T   (:77) */                       \
                        GEMM(CB_COL, CB_N, CB_T, nr, nc, d, tau, Qi, N, Kj, Nk, (REAL)0, P, nr);   \
                        for (int64_t r = 0; r < nr; ++r) { mij[r] = -INFINITY; lij[r] = 0; }       \
                        for (int64_t c = 0; c < nc; ++c)               /* maximum! (:78) */        \
                            for (int64_t r = 0; r < nr; ++r)                                       \
                                mij[r] = P[c * nr + r] > mij[r] ? P[c * nr + r] : mij[r];          \
                        for (int64_t c = 0; c < nc; ++c)               /* exp, sum! (:79-80) */    \
                            for (int64_t r = 0; r < nr; ++r) {                                     \
                                const REAL e = EXP(P[c * nr + r] - mij[r]);                        \
                                P[c * nr + r] = e;                                                 \
                                lij[r] += e;                                                       \
                            }                                                                     \
                        /* Oi_new (nr x dv) = Pij Vj   (:88) */                                    \
                        GEMM(CB_COL, CB_N, CB_N, nr, dv, nc, (REAL)1, P, nr, Vj, Nk, (REAL)0, On, nr); \
                        for (int64_t r = 0; r < nr; ++r) {             /* (:82-86, :89-91) */      \
                            const REAL mnew = mi[r] > mij[r] ? mi[r] : mij[r];                     \
                            const REAL ei = EXP(mi[r] - mnew), eij = EXP(mij[r] - mnew);           \
                            const REAL lnew = ei * li[r] + eij * lij[r];                           \
                            const REAL a = li[r] * ei;                                             \
                            for (int64_t x = 0; x < dv; ++x)                                       \
                                Oi[x * N + r] = (a * Oi[x * N + r] + eij * On[x * nr + r]) / lnew; \
                            li[r] = lnew; mi[r] = mnew;                                            \
                        }                                                                         \
                    }                                                                             \
                }                                                                                 \
        }                                                                                         \
        free(P); free(On); free(mij); free(lij);                                                   \
    }                                                                                             \
    return err;                                                                                   \
}

DEFINE_FA_CPU_BLAS(float, f32, expf, g_sgemm)
DEFINE_FA_CPU_BLAS(double, f64, exp, g_dgemm)

int fa_cpu_max_threads(void) { return omp_get_max_threads(); }
