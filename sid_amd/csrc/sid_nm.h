// sid_nm.h — Nelder-Mead vertex arithmetic for the Lynch estimate, shared by
// the host driver (lynch_host.cpp) and the device-resident estimate
// (lynch.hip sid_nm_kernel), so both follow one restatement of GSL 2.7.1
// multimin/nmsimplex2.c for 2 parameters (optimization.hpp:35-89 calls it
// through gsl_multimin_fminimizer_nmsimplex2), with the gslcblas kernels it
// uses (dnrm2 with scale/ssq, daxpy).  Built with -ffp-contract=off on both
// sides, so host and device produce the same doubles for the same inputs.
//
// The vertex arithmetic depends only on the sequence of comparisons between
// objective values, so agreeing comparisons give bit-identical (pi, eps).
#pragma once

#include <hip/hip_runtime.h>

#define SID_NM_N 2
#define SID_NM_P 3

// the dist-only constants of sid_lynch_eval (sid_math.h), computed once per
// estimate on the host
struct sid_nm_dist {
    double ld[4];
    double ldd[6];
    double lnorm;
};

// what the device-resident estimate (lynch.hip sid_nm_kernel) reports
struct sid_nm_result {
    double x[2];
    double fval;
    double size;
    int iterations;
    int converged;
    int status;   // 0 ok, 1 non-finite objective (EBADFUNC), 2 deadline/abort, 3 round cap, 4 internal
    int rounds;
    unsigned long long evals;    // objective calls of the algorithm (cached or not)
    unsigned long long points;   // objective points evaluated on the device
    long long ticks[4];          // block 0 wall clock: evaluate, barrier wait, fold, advance (measurement)
};

struct sid_nm_simplex {
    double x1[SID_NM_P][SID_NM_N];
    double y1[SID_NM_P];
    double center[SID_NM_N];
    double S2;
};

// gslcblas dnrm2 (scaled sum of squares)
__host__ __device__ inline double sid_nm_nrm2(const double* x)
{
    double scale = 0.0, ssq = 1.0;
    for (int i = 0; i < SID_NM_N; ++i) {
        if (x[i] != 0.0) {
            double ax = fabs(x[i]);
            if (scale < ax) {
                ssq = 1.0 + ssq * (scale / ax) * (scale / ax);
                scale = ax;
            } else {
                ssq += (ax / scale) * (ax / scale);
            }
        }
    }
    return scale * sqrt(ssq);
}

// gslcblas daxpy (a == 0 returns early, as gsl_blas_daxpy does)
__host__ __device__ inline void sid_nm_axpy(double a, const double* x, double* y)
{
    if (a == 0.0) return;
    for (int i = 0; i < SID_NM_N; ++i) y[i] += a * x[i];
}

// nmsimplex2.c compute_center
__host__ __device__ inline void sid_nm_compute_center(sid_nm_simplex& s)
{
    for (int j = 0; j < SID_NM_N; ++j) s.center[j] = 0.0;
    for (int i = 0; i < SID_NM_P; ++i) sid_nm_axpy(1.0, s.x1[i], s.center);
    for (int j = 0; j < SID_NM_N; ++j) s.center[j] *= 1.0 / SID_NM_P;
}

// nmsimplex2.c compute_size (also resets the running S2)
__host__ __device__ inline double sid_nm_compute_size(sid_nm_simplex& s)
{
    double ss = 0.0;
    for (int i = 0; i < SID_NM_P; ++i) {
        double v[SID_NM_N];
        for (int j = 0; j < SID_NM_N; ++j) v[j] = s.x1[i][j];
        sid_nm_axpy(-1.0, s.center, v);
        double t = sid_nm_nrm2(v);
        ss += t * t;
    }
    s.S2 = ss / SID_NM_P;
    return sqrt(ss / SID_NM_P);
}

// nmsimplex2.c try_corner_move: the point, not its value
__host__ __device__ inline void sid_nm_corner_point(const sid_nm_simplex& s, double coeff, int corner, double* xc)
{
    const size_t p = SID_NM_P;
    double alpha = (1 - coeff) * p / (p - 1.0);
    double beta = (p * coeff - 1.0) / (p - 1.0);
    for (int j = 0; j < SID_NM_N; ++j) xc[j] = s.center[j] * alpha;
    sid_nm_axpy(beta, s.x1[corner], xc);
}

// nmsimplex2.c update_point
__host__ __device__ inline void sid_nm_update_point(sid_nm_simplex& s, int i, const double* x, double val)
{
    const size_t p = SID_NM_P;
    double delta[SID_NM_N], xmc[SID_NM_N];
    for (int j = 0; j < SID_NM_N; ++j) delta[j] = x[j];
    sid_nm_axpy(-1.0, s.x1[i], delta);
    for (int j = 0; j < SID_NM_N; ++j) xmc[j] = s.x1[i][j];
    sid_nm_axpy(-1.0, s.center, xmc);
    double d = sid_nm_nrm2(delta);
    double xmcd = 0.0;
    for (int j = 0; j < SID_NM_N; ++j) xmcd += xmc[j] * delta[j];
    s.S2 += (2.0 / p) * xmcd + ((p - 1.0) / p) * (d * d / p);
    sid_nm_axpy(-1.0 / p, s.x1[i], s.center);
    sid_nm_axpy(1.0 / p, x, s.center);
    for (int j = 0; j < SID_NM_N; ++j) s.x1[i][j] = x[j];
    s.y1[i] = val;
}

// nmsimplex2_iterate: indices of the highest, second highest and lowest vertex
__host__ __device__ inline void sid_nm_order(const sid_nm_simplex& s, int& hi, int& s_hi, int& lo)
{
    hi = 0;
    lo = 0;
    s_hi = 1;
    double dhi = s.y1[0], dlo = s.y1[0], ds_hi = s.y1[1];
    for (int i = 1; i < SID_NM_P; ++i) {
        double v = s.y1[i];
        if (v < dlo) {
            dlo = v;
            lo = i;
        } else if (v > dhi) {
            ds_hi = dhi;
            s_hi = hi;
            dhi = v;
            hi = i;
        } else if (v > ds_hi) {
            ds_hi = v;
            s_hi = i;
        }
    }
}

// the candidate points of an iteration whose worst vertex is h: reflection,
// expansion, inside contraction, and the contraction after the reflected
// point is accepted
__host__ __device__ inline void sid_nm_candidates(const sid_nm_simplex& s, int h, double (*pts)[SID_NM_N])
{
    sid_nm_corner_point(s, -1.0, h, pts[0]);
    sid_nm_corner_point(s, -2.0, h, pts[1]);
    sid_nm_corner_point(s, 0.5, h, pts[2]);
    sid_nm_simplex t = s;
    sid_nm_update_point(t, h, pts[0], 0.0);
    sid_nm_corner_point(t, 0.5, h, pts[3]);
}

// gsl_vector_min_index over y1 (a NaN wins)
__host__ __device__ inline int sid_nm_min_index(const sid_nm_simplex& s)
{
    int imin = 0;
    double mn = s.y1[0];
    for (int i = 0; i < SID_NM_P; ++i) {
        if (s.y1[i] < mn) {
            mn = s.y1[i];
            imin = i;
        }
        if (__builtin_isnan(s.y1[i])) {
            imin = i;
            break;
        }
    }
    return imin;
}

// appends x to pts[0..k) unless present (capacity cap)
__host__ __device__ inline void sid_nm_add_point(double (*pts)[SID_NM_N], int& k, int cap, const double* x)
{
    for (int i = 0; i < k; ++i)
        if (pts[i][0] == x[0] && pts[i][1] == x[1]) return;
    if (k < cap) {
        pts[k][0] = x[0];
        pts[k][1] = x[1];
        ++k;
    }
}

// The points to evaluate before an iteration whose worst vertex is hi: its
// four candidates and, with lookahead, the next iteration's candidates after
// each outcome of this one (only the worst vertex moves, so the new worst is
// the old second worst, or the moved vertex after a contraction).  The
// trajectory does not depend on what is evaluated ahead.
__host__ __device__ inline int sid_nm_request(const sid_nm_simplex& s, bool lookahead, double (*pts)[SID_NM_N],
                                              int cap)
{
    int hi, s_hi, lo;
    sid_nm_order(s, hi, s_hi, lo);
    double c1[4][SID_NM_N];
    sid_nm_candidates(s, hi, c1);
    int k = 0;
    for (int i = 0; i < 4; ++i) sid_nm_add_point(pts, k, cap, c1[i]);
    if (!lookahead) return k;
    for (int o = 0; o < 4; ++o) {
        sid_nm_simplex t = s;
        if (o == 0) sid_nm_update_point(t, hi, c1[0], 0.0);   // reflection accepted
        if (o == 1) sid_nm_update_point(t, hi, c1[1], 0.0);   // expansion accepted
        if (o == 2) {                                         // outside contraction
            sid_nm_update_point(t, hi, c1[0], 0.0);
            sid_nm_update_point(t, hi, c1[3], 0.0);
        }
        if (o == 3) sid_nm_update_point(t, hi, c1[2], 0.0);   // inside contraction
        const int h2s[2] = {s_hi, hi};
        for (int q = 0; q < 2; ++q) {
            const int h2 = h2s[q];
            if (h2 == hi && o < 2) continue;
            double c2[4][SID_NM_N];
            sid_nm_candidates(t, h2, c2);
            for (int i = 0; i < 4; ++i) sid_nm_add_point(pts, k, cap, c2[i]);
        }
    }
    return k;
}
