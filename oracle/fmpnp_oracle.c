/*
 * fmpnp_oracle.c -- CPU restatement of the reference feature-metric PnP
 * Levenberg-Marquardt loop.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity oracle for the HIP product path.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker / the timed CPU baseline -- never as a fallback for the
 * product library (featuremetric-pnp_amd/), which fails loudly without its
 * HIP kernels.
 *
 * It is a deliberately *faithful* restatement of the reference
 * (aunagar/FeatureMetric-PnP, featurePnP/model.py + helpers/utils.py):
 *   - layout as the reference holds it: fp64 [C][Hf][Wf] maps, fp64 [N][C]
 *     reference descriptors;
 *   - two evaluations per iteration exactly as model.py:300-486 does them
 *     (linearise at (R,t), then evaluate the trial (R',t')), including the
 *     identical re-linearisation after a rejected step;
 *   - projection P = R X + t, p = round_half_even(K P / P_z) - 1 as the
 *     reference's torch.mm (sequential, no FMA) computes it.
 * Summation orders over points/channels are plain index order; they differ
 * from torch's in the last bits only.  Parity is pinned by the golden vectors
 * in tests/golden/ produced by running the reference itself
 * (tests/golden/gen_golden.py).
 *
 * Build: oracle/Makefile  (gcc -O2 -fopenmp -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "fmpnp_oracle.h"

/* torch.finfo(torch.float).eps as the reference uses it (utils.py:25,58) */
static const double EPS_F32 = 1.1920928955078125e-07;

/* ------------------------------------------------------------------------ */
/* robust losses: featurePnP/helpers/utils.py:15-78                          */
/* ------------------------------------------------------------------------ */
static void loss_eval(int loss, double alpha, double x, double *rho, double *d1)
{
    switch (loss) {
    case ORC_SQUARED: /* utils.py:16-17 */
        *rho = x;
        *d1 = 1.0;
        return;
    case ORC_HUBER: { /* utils.py:20-29 (rho = 1) */
        double sx = sqrt(x);
        double inv = 1.0 / sx;
        double isx = (inv > EPS_F32 || isnan(inv)) ? inv : EPS_F32; /* torch.max propagates NaN */
        if (x <= 1.0) { *rho = x; *d1 = 1.0; }
        else { *rho = 2.0 * sx - 1.0; *d1 = isx; }
        return;
    }
    case ORC_CAUCHY: /* utils.py:32-34 -> barron alpha = 0 */
        alpha = 0.0;
        break;
    case ORC_GEMAN_MCCLURE: /* utils.py:37-38 -> barron alpha = -2 */
        alpha = -2.0;
        break;
    default: /* ORC_BARRON */
        break;
    }
    /* utils.py:40-78 */
    if (alpha == 0.0) {
        double h = 0.5 * x;
        if (!(h <= 33e37)) h = isnan(h) ? h : 33e37;
        *rho = 2.0 * log1p(h);
        *d1 = 2.0 / (x + 2.0);
    } else if (alpha == 2.0) {
        *rho = x;
        *d1 = 1.0;
    } else {
        double beta_safe = fabs(alpha - 2.0);
        if (beta_safe < EPS_F32) beta_safe = EPS_F32;
        double aa = fabs(alpha);
        if (aa < EPS_F32) aa = EPS_F32;
        double alpha_safe = (alpha >= 0.0 ? 1.0 : -1.0) * aa;
        double b = x / beta_safe + 1.0;
        *rho = 2.0 * (beta_safe / alpha_safe) * (pow(b, 0.5 * alpha) - 1.0);
        *d1 = pow(b, 0.5 * alpha - 1.0);
    }
}

/* ------------------------------------------------------------------------ */
/* geometry                                                                  */
/* ------------------------------------------------------------------------ */
/* P = R X + t  (model.py:303, torch.mm then + t: sequential, no FMA) */
static void transform(const double R[9], const double t[3], const double X[3], double P[3])
{
    for (int i = 0; i < 3; ++i) {
        double s = R[3 * i + 0] * X[0];
        s = s + R[3 * i + 1] * X[1];
        s = s + R[3 * i + 2] * X[2];
        P[i] = s + t[i];
    }
}

/* p = round(K P / P_z) - 1 as int, then the mask (model.py:306-311,99-117).
 * Returns 1 if supported; *x,*y are the image pixel indices, *qx,*qy the
 * unrounded K P / P_z (used by the bilinear extension). */
static int project(const double K[9], const double P[3], int W, int H, long *x, long *y, double *qx, double *qy)
{
    double u[3];
    for (int i = 0; i < 3; ++i) {
        double s = K[3 * i + 0] * P[0];
        s = s + K[3 * i + 1] * P[1];
        s = s + K[3 * i + 2] * P[2];
        u[i] = s;
    }
    *qx = u[0] / u[2];
    *qy = u[1] / u[2];
    double px = rint(*qx) - 1.0; /* torch.round: half to even */
    double py = rint(*qy) - 1.0;
    /* int32 cast of a non-finite / out-of-range value lands outside [0,W) in
     * the reference (INT_MIN - 1 wraps); here the test on the double is
     * equivalent for every value that can be inside the image. */
    if (!(px >= 0.0 && px < (double)W && py >= 0.0 && py < (double)H)) return 0;
    *x = (long)px;
    *y = (long)py;
    return 1;
}

/* ------------------------------------------------------------------------ */
/* Bilinear sampling (EXTENSION, not in the reference: its indexing_ is      */
/* nearest-texel).  Definition shared bit-for-bit with the HIP kernel        */
/* (fmpnp_device.h bilinear_taps):                                           */
/*   sx = ((qx - 0.5) * Wf) / W - 0.5,  sy = ((qy - 0.5) * Hf) / H - 0.5     */
/* (qx, qy = K P / P_z unrounded; the centre of image pixel index i, which   */
/* the reference writes as round(q) - 1, is q = i + 1, and texel c's centre  */
/* is sx = c), x0 = floor(sx), ax = sx - x0, taps at columns x0, x0 + 1 and  */
/* rows y0, y0 + 1 clamped to the map, weights                               */
/*   w00 = (1-ax)(1-ay), w01 = ax(1-ay), w10 = (1-ax)ay, w11 = ax ay,        */
/* and every sampled value (f, gx, gy per channel) is                        */
/*   fma(w11, v11, fma(w10, v10, fma(w01, v01, w00 * v00))).                 */
/* The support set is the reference's (the rounded pixel inside the image).  */
/* ------------------------------------------------------------------------ */
typedef struct { long off[4]; double w[4]; } taps4;

static void bilinear_taps(double qx, double qy, int Hf, int Wf, int im_w, int im_h, taps4 *tp)
{
    double sx = ((qx - 0.5) * (double)Wf) / (double)im_w - 0.5;
    double sy = ((qy - 0.5) * (double)Hf) / (double)im_h - 0.5;
    double fx0 = floor(sx), fy0 = floor(sy);
    double ax = sx - fx0, ay = sy - fy0;
    long x0 = (long)fx0, y0 = (long)fy0, x1 = x0 + 1, y1 = y0 + 1;
    x0 = x0 < 0 ? 0 : (x0 > Wf - 1 ? Wf - 1 : x0);
    x1 = x1 < 0 ? 0 : (x1 > Wf - 1 ? Wf - 1 : x1);
    y0 = y0 < 0 ? 0 : (y0 > Hf - 1 ? Hf - 1 : y0);
    y1 = y1 < 0 ? 0 : (y1 > Hf - 1 ? Hf - 1 : y1);
    tp->off[0] = y0 * Wf + x0;
    tp->off[1] = y0 * Wf + x1;
    tp->off[2] = y1 * Wf + x0;
    tp->off[3] = y1 * Wf + x1;
    tp->w[0] = (1.0 - ax) * (1.0 - ay);
    tp->w[1] = ax * (1.0 - ay);
    tp->w[2] = (1.0 - ax) * ay;
    tp->w[3] = ax * ay;
}

static double sample4(const double *plane_c, const taps4 *tp)
{
    return fma(tp->w[3], plane_c[tp->off[3]],
               fma(tp->w[2], plane_c[tp->off[2]], fma(tp->w[1], plane_c[tp->off[1]], tp->w[0] * plane_c[tp->off[0]])));
}

/* ------------------------------------------------------------------------ */
/* one evaluation at a pose: model.py:303-339 (+ Jacobians :364-405)          */
/* ------------------------------------------------------------------------ */
typedef struct {
    int n_supported;   /* points inside the image (model.py:311-316) */
    int n_kept;        /* after the optional ratio test (model.py:324-336) */
    double cost_mean;  /* mean rho over kept points (NaN if none kept) */
    double g[6];       /* sum rho' J^T e  (model.py:397-399) */
    double H[36];      /* sum rho' J^T J  (model.py:403-405) */
} eval_out;

static void evaluate(const orc_problem *pb, const orc_options *op, const double R[9], const double t[3],
                     int want_normal, eval_out *eo, double *rho_buf, unsigned char *sup_buf,
                     double *err_buf, long *pix_buf, taps4 *tap_buf)
{
    const int N = pb->N, C = pb->C;
    const long plane = (long)pb->Hf * pb->Wf;
    eo->n_supported = 0;
    /* pass 1: projection, gather, residual, rho */
    double rho_max = 0.0;
    int first = 1;
    const int bil = op->sampling == ORC_BILINEAR;
    for (int n = 0; n < N; ++n) {
        double P[3], qx, qy;
        long x, y;
        transform(R, t, pb->pts + 3 * n, P);
        sup_buf[n] = (unsigned char)project(pb->K, P, pb->im_w, pb->im_h, &x, &y, &qx, &qy);
        if (!sup_buf[n]) continue;
        eo->n_supported++;
        double s = 0.0;
        const double *fr = pb->fref + (long)n * pb->ld_ref;
        if (bil) {
            bilinear_taps(qx, qy, pb->Hf, pb->Wf, pb->im_w, pb->im_h, &tap_buf[n]);
            for (int c = 0; c < C; ++c) {
                double e = sample4(pb->fmap + c * plane, &tap_buf[n]) - fr[c];
                err_buf[(long)n * C + c] = e;
                s += e * e;
            }
        } else {
            /* indexing_ (model.py:88-89): row = floor(y*Hf/H), col = floor(x*Wf/W) */
            long row = (y * (long)pb->Hf) / pb->im_h;
            long col = (x * (long)pb->Wf) / pb->im_w;
            long off = row * pb->Wf + col;
            pix_buf[n] = off;
            for (int c = 0; c < C; ++c) {
                double e = pb->fmap[c * plane + off] - fr[c];
                err_buf[(long)n * C + c] = e;
                s += e * e;
            }
        }
        double xcost = 0.5 * s, rho, d1;
        loss_eval(op->loss, op->barron_alpha, xcost, &rho, &d1);
        rho_buf[2 * n] = rho;
        rho_buf[2 * n + 1] = d1;
        double a = fabs(rho);
        if (first || a > rho_max || isnan(a)) { rho_max = (isnan(rho_max) ? rho_max : a); first = 0; }
    }
    /* ratio test (model.py:120-129): keep |rho| < max|rho| * thr */
    double limit = rho_max * op->ratio_threshold;
    int use_ratio = op->use_ratio;
    double csum = 0.0;
    int kept = 0;
    memset(eo->g, 0, sizeof(eo->g));
    memset(eo->H, 0, sizeof(eo->H));
    for (int n = 0; n < N; ++n) {
        if (!sup_buf[n]) continue;
        double rho = rho_buf[2 * n], w = rho_buf[2 * n + 1];
        if (use_ratio && !(fabs(rho) < limit)) continue;
        kept++;
        csum += rho;
        if (!want_normal) continue;
        double P[3];
        transform(R, t, pb->pts + 3 * n, P);
        /* J_px_p (model.py:377-382): rows [fx/z, 0, (-fx X / z)/z], [0, fy/z, (-fy Y / z)/z] */
        double fx = pb->K[0], fy = pb->K[4], z = P[2];
        double Jpx[2][3] = {{fx / z, 0.0 / z, ((-fx) * P[0] / z) / z},
                            {0.0 / z, fy / z, ((-fy) * P[1] / z) / z}};
        /* J_p_T = [I | -[P]x] (model.py:369-370) */
        double Jp[3][6] = {{1, 0, 0, 0, P[2], -P[1]}, {0, 1, 0, -P[2], 0, P[0]}, {0, 0, 1, P[1], -P[0], 0}};
        /* J = (J_f_px @ J_px_p) @ J_p_T per channel (model.py:386-394, left to right);
         * per point J^T e and J^T J summed over channels (einsum :397,403), then
         * scaled by rho' and summed over points (:398-399, :404-405). */
        const double *err = err_buf + (long)n * C;
        long off = bil ? 0 : pix_buf[n];
        double gp[6] = {0, 0, 0, 0, 0, 0}, Hp[36];
        memset(Hp, 0, sizeof(Hp));
        for (int c = 0; c < C; ++c) {
            double gxv, gyv;
            if (bil) {
                gxv = sample4(pb->gx + c * plane, &tap_buf[n]);
                gyv = sample4(pb->gy + c * plane, &tap_buf[n]);
            } else {
                gxv = pb->gx[c * plane + off];
                gyv = pb->gy[c * plane + off];
            }
            double B[3], Jc[6];
            for (int m = 0; m < 3; ++m) B[m] = gxv * Jpx[0][m] + gyv * Jpx[1][m];
            for (int k = 0; k < 6; ++k) {
                double s = B[0] * Jp[0][k];
                s = s + B[1] * Jp[1][k];
                s = s + B[2] * Jp[2][k];
                Jc[k] = s;
            }
            double e = err[c];
            for (int k = 0; k < 6; ++k) {
                gp[k] += Jc[k] * e;
                for (int l = 0; l < 6; ++l) Hp[6 * k + l] += Jc[k] * Jc[l];
            }
        }
        for (int k = 0; k < 6; ++k) {
            eo->g[k] += w * gp[k];
            for (int l = 0; l < 6; ++l) eo->H[6 * k + l] += w * Hp[6 * k + l];
        }
    }
    eo->n_kept = kept;
    eo->cost_mean = csum / (double)kept; /* torch mean of an empty tensor is NaN */
}

/* ------------------------------------------------------------------------ */
/* optimizer_step (model.py:37-72): damped LU solve, delta = -lr x           */
/* ------------------------------------------------------------------------ */
static void optimizer_step(const double g[6], const double Hin[36], double lambda, double lr, double delta[6])
{
    double A[36];
    memcpy(A, Hin, sizeof(A));
    if (lambda != 0.0) /* `if lambda_:` */
        for (int i = 0; i < 6; ++i) A[7 * i] = A[7 * i] + (A[7 * i] + 1e-9) * lambda;
    /* LU with partial pivoting (getrf), then getrs */
    int piv[6];
    for (int j = 0; j < 6; ++j) {
        int p = j;
        double best = fabs(A[6 * j + j]);
        for (int i = j + 1; i < 6; ++i)
            if (fabs(A[6 * i + j]) > best) { best = fabs(A[6 * i + j]); p = i; }
        piv[j] = p;
        if (p != j)
            for (int k = 0; k < 6; ++k) { double tmp = A[6 * j + k]; A[6 * j + k] = A[6 * p + k]; A[6 * p + k] = tmp; }
        double inv = 1.0 / A[6 * j + j];
        for (int i = j + 1; i < 6; ++i) {
            A[6 * i + j] *= inv;
            for (int k = j + 1; k < 6; ++k) A[6 * i + k] -= A[6 * i + j] * A[6 * j + k];
        }
    }
    double b[6];
    memcpy(b, g, sizeof(b));
    for (int j = 0; j < 6; ++j)
        if (piv[j] != j) { double tmp = b[j]; b[j] = b[piv[j]]; b[piv[j]] = tmp; }
    for (int i = 0; i < 6; ++i)
        for (int k = 0; k < i; ++k) b[i] -= A[6 * i + k] * b[k];
    for (int i = 5; i >= 0; --i) {
        for (int k = i + 1; k < 6; ++k) b[i] -= A[6 * i + k] * b[k];
        b[i] /= A[6 * i + i];
    }
    for (int i = 0; i < 6; ++i) delta[i] = -lr * b[i];
}

/* so3exp_map (utils.py:209-221) */
static void so3exp(const double w[3], double R[9])
{
    double theta = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
    if (theta < 1e-12 || isnan(theta)) {
        if (isnan(theta))
            for (int i = 0; i < 9; ++i) R[i] = NAN;
        return;
    }
    double k[3] = {w[0] / theta, w[1] / theta, w[2] / theta};
    double W[9] = {0, -k[2], k[1], k[2], 0, -k[0], -k[1], k[0], 0};
    double s = sin(theta), c1 = 1.0 - cos(theta);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double ww = W[3 * i + 0] * W[0 + j] + W[3 * i + 1] * W[3 + j] + W[3 * i + 2] * W[6 + j];
            R[3 * i + j] += W[3 * i + j] * s + ww * c1;
        }
}

static void matmul3(const double A[9], const double B[9], double C[9])
{
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            C[3 * i + j] = A[3 * i + 0] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

/* ------------------------------------------------------------------------ */
/* sparseFeaturePnP.forward (model.py:245-494)                               */
/* ------------------------------------------------------------------------ */
int orc_forward(const orc_problem *pb, const orc_options *op, orc_result *res, orc_trace *tr)
{
    const int N = pb->N, C = pb->C;
    double *rho_buf = (double *)malloc(sizeof(double) * 2 * (N > 0 ? N : 1));
    unsigned char *sup = (unsigned char *)malloc(N > 0 ? N : 1);
    double *err = (double *)malloc(sizeof(double) * (size_t)(N > 0 ? N : 1) * (C > 0 ? C : 1));
    long *pix = (long *)malloc(sizeof(long) * (N > 0 ? N : 1));
    taps4 *taps = (taps4 *)malloc(sizeof(taps4) * (N > 0 ? N : 1));
    if (!rho_buf || !sup || !err || !pix || !taps) {
        free(rho_buf); free(sup); free(err); free(pix); free(taps);
        return -1;
    }

    double R[9], t[3], Rb[9], tb[3];
    memcpy(R, pb->R0, sizeof(R));
    memcpy(t, pb->t0, sizeof(t));
    memcpy(Rb, R, sizeof(R));
    memcpy(tb, t, sizeof(t));
    double lambda = op->lambda0, lr = 1.0, prev = NAN;
    res->status = ORC_OK;
    res->has_best = 0;
    res->best_cost = NAN;
    res->initial_cost = NAN;
    res->best_num_inliers = -1;
    res->n_evals = 0;
    res->n_steps = 0;
    res->n_accepted = 0;
    int returned_current = 0;

    for (int i = 0; i < op->n_iters; ++i) {
        eval_out lin;
        evaluate(pb, op, R, t, 1, &lin, rho_buf, sup, err, pix, taps);
        if (lin.n_supported == 0) { /* model.py:316-320: return the CURRENT pose */
            res->status = ORC_NO_SUPPORT;
            returned_current = 1;
            break;
        }
        if (i == 0) { /* model.py:347-359 */
            prev = lin.cost_mean;
            res->best_cost = prev;
            res->has_best = 1;
            res->best_num_inliers = lin.n_kept;
            memcpy(Rb, R, sizeof(R));
            memcpy(tb, t, sizeof(t));
            res->initial_cost = prev;
            if (tr && tr->cap > res->n_evals) {
                int k = res->n_evals;
                memcpy(tr->R + 9 * k, R, sizeof(R));
                memcpy(tr->t + 3 * k, t, sizeof(t));
                tr->cost[k] = lin.cost_mean;
                tr->n_supported[k] = lin.n_supported;
                tr->n_kept[k] = lin.n_kept;
            }
            res->n_evals++;
        }
        double delta[6];
        optimizer_step(lin.g, lin.H, lambda, lr, delta);
        if (tr && tr->cap > res->n_steps) {
            int k = res->n_steps;
            memcpy(tr->g + 6 * k, lin.g, sizeof(lin.g));
            memcpy(tr->H + 36 * k, lin.H, sizeof(lin.H));
            tr->lam[k] = lambda;
            tr->lr[k] = lr;
            memcpy(tr->delta + 6 * k, delta, sizeof(delta));
        }
        res->n_steps++;
        int bad = 0;
        for (int k = 0; k < 6; ++k) bad |= isnan(delta[k]);
        if (bad) { /* model.py:411-413 (the reference then dies on an unimported `logging`) */
            res->status = ORC_NAN;
            break;
        }
        double dR[9], Rn[9], tn[3];
        so3exp(delta + 3, dR);
        matmul3(dR, R, Rn); /* model.py:425-426 */
        for (int r = 0; r < 3; ++r) tn[r] = (dR[3 * r] * t[0] + dR[3 * r + 1] * t[1] + dR[3 * r + 2] * t[2]) + delta[r];
        eval_out tri;
        evaluate(pb, op, Rn, tn, 0, &tri, rho_buf, sup, err, pix, taps);
        if (tri.n_supported == 0) { /* model.py:441-445: return the CURRENT pose */
            res->status = ORC_NO_SUPPORT_TRIAL;
            returned_current = 1;
            break;
        }
        double nc = tri.cost_mean;
        if (tr && tr->cap > res->n_evals) {
            int k = res->n_evals;
            memcpy(tr->R + 9 * k, Rn, sizeof(Rn));
            memcpy(tr->t + 3 * k, tn, sizeof(tn));
            tr->cost[k] = nc;
            tr->n_supported[k] = tri.n_supported;
            tr->n_kept[k] = tri.n_kept;
        }
        res->n_evals++;
        /* model.py:469-486 */
        lambda = lambda * (nc > prev ? 10.0 : 0.1);
        lambda = lambda < 1e-6 ? 1e-6 : (lambda > 1e4 ? 1e4 : lambda);
        if (nc > prev) {
            lr = 0.1 * lr;
            lr = lr < 1e-3 ? 1e-3 : (lr > 1.0 ? 1.0 : lr);
            continue;
        }
        lr = 1.0;
        res->n_accepted++;
        if (nc < res->best_cost) {
            memcpy(Rb, Rn, sizeof(Rn));
            memcpy(tb, tn, sizeof(tn));
            res->best_num_inliers = tri.n_kept;
            res->best_cost = nc;
        }
        prev = nc;
        memcpy(R, Rn, sizeof(R));
        memcpy(t, tn, sizeof(t));
    }
    if (returned_current) {
        memcpy(res->R, R, sizeof(R));
        memcpy(res->t, t, sizeof(t));
    } else {
        memcpy(res->R, Rb, sizeof(Rb));
        memcpy(res->t, tb, sizeof(tb));
    }
    res->final_lambda = lambda;
    res->final_lr = lr;
    free(rho_buf);
    free(sup);
    free(err);
    free(pix);
    free(taps);
    return 0;
}

/* compute_cost (model.py:216-243): mean 0.5||e||^2 over supported points, the
 * optional ratio test on that raw cost (ratio_threshold NaN = off); returns NaN
 * when nothing is supported (the reference returns None). */
double orc_compute_cost(const orc_problem *pb, double ratio_threshold, const double R[9], const double t[3])
{
    orc_options op;
    memset(&op, 0, sizeof(op));
    op.loss = ORC_SQUARED;
    op.ratio_threshold = ratio_threshold;
    op.use_ratio = !isnan(ratio_threshold);
    const int N = pb->N, C = pb->C;
    double *rho_buf = (double *)malloc(sizeof(double) * 2 * (N > 0 ? N : 1));
    unsigned char *sup = (unsigned char *)malloc(N > 0 ? N : 1);
    double *err = (double *)malloc(sizeof(double) * (size_t)(N > 0 ? N : 1) * (C > 0 ? C : 1));
    long *pix = (long *)malloc(sizeof(long) * (N > 0 ? N : 1));
    eval_out eo;
    evaluate(pb, &op, R, t, 0, &eo, rho_buf, sup, err, pix, NULL);
    free(rho_buf);
    free(sup);
    free(err);
    free(pix);
    return eo.n_supported == 0 ? NAN : eo.cost_mean;
}

/* find_inliers (model.py:132-152, mode "ratio_max"): project at (R, t), support mask
 * (points_within_image), NN gather (indexing_), cost = 0.5 ||e||^2, (rho, .) = loss(cost),
 * then ratio_threshold_feature_errors (model.py:120-129) over the supported points:
 * mask[n] = supported and |rho_n| < max |rho| * threshold.  cost_out[n] = 0.5 ||e||^2
 * (0 if unsupported).  Returns the number of supported points (0: the reference's
 * torch.max of an empty tensor raises). */
int orc_find_inliers(const orc_problem *pb, const double R[9], const double t[3], int loss, double alpha,
                     double threshold, unsigned char *mask, double *cost_out)
{
    const int N = pb->N, C = pb->C;
    const long plane = (long)pb->Hf * pb->Wf;
    double *rho = (double *)malloc(sizeof(double) * (N > 0 ? N : 1));
    int nsup = 0;
    double rmax = 0.0;
    for (int n = 0; n < N; ++n) {
        double P[3], qx, qy, d1;
        long x, y;
        transform(R, t, pb->pts + 3 * n, P);
        mask[n] = (unsigned char)project(pb->K, P, pb->im_w, pb->im_h, &x, &y, &qx, &qy);
        cost_out[n] = 0.0;
        if (!mask[n]) continue;
        const long off = ((y * (long)pb->Hf) / pb->im_h) * pb->Wf + (x * (long)pb->Wf) / pb->im_w;
        const double *fr = pb->fref + (long)n * pb->ld_ref;
        double s = 0.0;
        for (int c = 0; c < C; ++c) {
            const double e = pb->fmap[c * plane + off] - fr[c];
            s += e * e;
        }
        cost_out[n] = 0.5 * s;
        loss_eval(loss, alpha, cost_out[n], &rho[n], &d1);
        const double a = fabs(rho[n]);
        if (nsup == 0 || a > rmax || isnan(a)) rmax = isnan(rmax) ? rmax : a;
        nsup++;
    }
    const double limit = rmax * threshold;
    for (int n = 0; n < N; ++n)
        if (mask[n]) mask[n] = (unsigned char)(fabs(rho[n]) < limit);
    free(rho);
    return nsup;
}

/* Sobel (helpers/sobel_pytorch.py:9-59 via utils.py:81-104): cross-correlation
 * with kx = [[-1,0,1],[-2,0,2],[-1,0,1]], ky = kx^T, zero padding, unnormalised. */
void orc_sobel(const double *x, int C, int H, int W, double *gx, double *gy)
{
    for (int c = 0; c < C; ++c) {
        const double *p = x + (long)c * H * W;
#define PX(yy, xx) (((yy) < 0 || (yy) >= H || (xx) < 0 || (xx) >= W) ? 0.0 : p[(long)(yy) * W + (xx)])
        for (int y = 0; y < H; ++y)
            for (int xx = 0; xx < W; ++xx) {
                double a = PX(y - 1, xx - 1), b = PX(y - 1, xx), cc = PX(y - 1, xx + 1);
                double d = PX(y, xx - 1), f = PX(y, xx + 1);
                double g = PX(y + 1, xx - 1), h = PX(y + 1, xx), k = PX(y + 1, xx + 1);
                gx[(long)c * H * W + (long)y * W + xx] = ((-a + cc) + (-2.0 * d + 2.0 * f)) + (-g + k);
                gy[(long)c * H * W + (long)y * W + xx] = ((-a - 2.0 * b) - cc) + ((g + 2.0 * h) + k);
            }
#undef PX
    }
}

/* Batch of independent forwards, OpenMP over problems (the CPU baseline). */
int orc_forward_batch(const orc_problem *pbs, int n, const orc_options *op, orc_result *res, int nthreads)
{
    int err = 0;
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err) num_threads(nthreads)
    for (int i = 0; i < n; ++i) err |= orc_forward(pbs + i, op, res + i, NULL) != 0;
    return err ? -1 : 0;
}
