// fmpnp_cpu.cpp -- fmpnp_refine_batch_cpu: the CPU twin of fmpnp_refine_batch.
//
// Same problem descriptors, options and result / trace structs as the HIP entry point, with HOST
// pointers: the packed channels-last maps of fmpnp_pack_features ([Hf][Wf][3][cstride], or the
// f-only [Hf][Wf][cstride] of FMPNP_LAYOUT_F), fref [N][ld_ref], pts3d [N][3].  It is an explicit
// CPU entry point -- the timed CPU baseline beside the GPU and a parity bridge for callers without
// a GPU -- and never a fallback: fmpnp_refine_batch does not call it, and the Python façade reaches
// it only through fmpnp.cpu.
//
// The algorithm is sparseFeaturePnP.forward (featurePnP/model.py:245-494) in the form the LM kernel
// runs it (fmpnp_lm_impl.h), restated for a CPU core:
//   * one evaluation per iteration: the trial evaluation at (R', t') also yields that pose's normal
//     equations; on acceptance they are the next linearisation, on rejection the cached ones are
//     reused -- identical to the reference's re-linearisation at the unchanged pose (model.py:472-476);
//   * the per-point C x 6 Jacobian (model.py:369-394) is never formed: each point keeps the six
//     channel sums  sum e^2, sum gx e, sum gy e, sum gx^2, sum gx gy, sum gy^2  of its texel, and
//     J^T e = A^T (G^T e), J^T J = A^T (G^T G) A with the point's 2 x 6 chain A;
//   * the sums depend only on the texel and the point's fixed descriptor, so a point re-reads its
//     texel only when its pixel changes texel (memoisation; texel_gathers counts the reads);
//   * the projection is the reference's: P = R X + t and K P sequentially without FMA, the pixel
//     round_half_even(K P / P_z) - 1 with IEEE divisions, indexing_'s floor rescale as an integer
//     division (model.py:74-117, 303-311); z < 0 is not masked;
//   * the damped solve is LU with partial pivoting of H + lambda diag(diag(H) + 1e-9)
//     (optimizer_step, model.py:37-72); so3exp_map (helpers/utils.py:209-221) in its normalised form.
// Losses (helpers/utils.py:15-78) and the ratio test (model.py:120-129) as the reference.  Problems
// run in parallel over host threads (queries are independent: SURVEY.md 8e).
// Nearest sampling only (the reference's); FMPNP_BILINEAR returns FMPNP_EINVAL.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "fmpnp.h"

namespace {

constexpr double kEpsF32 = 1.1920928955078125e-07;  // torch.finfo(torch.float).eps (utils.py:25,58)

// rho and rho' of helpers/utils.py:15-78 (the second derivative the reference returns is zero and unused)
void loss_cpu(int loss, double alpha, double x, double &rho, double &d1) {
    switch (loss) {
    case FMPNP_SQUARED:
        rho = x;
        d1 = 1.0;
        return;
    case FMPNP_HUBER: {
        const double sx = sqrt(x), inv = 1.0 / sx;
        const double isx = (inv > kEpsF32 || isnan(inv)) ? inv : kEpsF32;
        if (x <= 1.0) {
            rho = x;
            d1 = 1.0;
        } else {
            rho = 2.0 * sx - 1.0;
            d1 = isx;
        }
        return;
    }
    case FMPNP_CAUCHY: alpha = 0.0; break;
    case FMPNP_GEMAN_MCCLURE: alpha = -2.0; break;
    default: break;
    }
    if (alpha == 0.0) {
        double h = 0.5 * x;
        if (!(h <= 33e37)) h = isnan(h) ? h : 33e37;
        rho = 2.0 * log1p(h);
        d1 = 2.0 / (x + 2.0);
    } else if (alpha == 2.0) {
        rho = x;
        d1 = 1.0;
    } else {
        double bs = fabs(alpha - 2.0);
        bs = bs < kEpsF32 ? kEpsF32 : bs;
        double aa = fabs(alpha);
        aa = aa < kEpsF32 ? kEpsF32 : aa;
        const double as = (alpha >= 0.0 ? 1.0 : -1.0) * aa;
        const double b = x / bs + 1.0;
        rho = 2.0 * (bs / as) * (pow(b, 0.5 * alpha) - 1.0);
        d1 = pow(b, 0.5 * alpha - 1.0);
    }
}

// The reference's projection and indexing_ (see the file comment).  Returns the texel offset or -1.
long texel_of(const fmpnp_problem &p, const double R[9], const double t[3], const double X[3], double P[3]) {
    for (int i = 0; i < 3; ++i) {
        double s = R[3 * i] * X[0];
        s = s + R[3 * i + 1] * X[1];
        s = s + R[3 * i + 2] * X[2];
        P[i] = s + t[i];
    }
    double u[3];
    for (int i = 0; i < 3; ++i) {
        double s = p.K[3 * i] * P[0];
        s = s + p.K[3 * i + 1] * P[1];
        s = s + p.K[3 * i + 2] * P[2];
        u[i] = s;
    }
    const double px = rint(u[0] / u[2]) - 1.0, py = rint(u[1] / u[2]) - 1.0;
    if (!(px >= 0.0 && px < (double)p.im_width && py >= 0.0 && py < (double)p.im_height)) return -1;
    const long x = (long)px, y = (long)py;
    const long row = (y * (long)p.Hf) / p.im_height, col = (x * (long)p.Wf) / p.im_width;
    return row * p.Wf + col;
}

// Six channel sums of one texel against one descriptor, fp64, four interleaved partial sums per
// quantity (a fixed order: vectorisable without reassociation).
template <typename T>
void sums_fgrad(const T *tx, const T *fr, int cs, int cb, int ce, double out[6]) {
    double a[6][4] = {};
    int c = cb;
    for (; c + 4 <= ce; c += 4)
        for (int k = 0; k < 4; ++k) {
            const double f = (double)tx[c + k], g = (double)tx[cs + c + k], h = (double)tx[2 * cs + c + k];
            const double e = f - (double)fr[c + k];
            a[0][k] += e * e;
            a[1][k] += g * e;
            a[2][k] += h * e;
            a[3][k] += g * g;
            a[4][k] += g * h;
            a[5][k] += h * h;
        }
    for (int k = 0; c < ce; ++c, ++k) {
        const double f = (double)tx[c], g = (double)tx[cs + c], h = (double)tx[2 * cs + c];
        const double e = f - (double)fr[c];
        a[0][k] += e * e;
        a[1][k] += g * e;
        a[2][k] += h * e;
        a[3][k] += g * g;
        a[4][k] += g * h;
        a[5][k] += h * h;
    }
    for (int q = 0; q < 6; ++q) out[q] = (a[q][0] + a[q][1]) + (a[q][2] + a[q][3]);
}

// FMPNP_LAYOUT_F: the Sobel gradients of the texel's 3x3 neighbourhood (helpers/sobel_pytorch.py:
// cross-correlation with [[-1,0,1],[-2,0,2],[-1,0,1]] and its transpose; zero or replicate padding,
// /8 when normalised), formed in fp64 per channel.
void sums_f(const float *feat, const float *fr, const fmpnp_problem &p, long off, int flags, double out[6]) {
    const int r0 = (int)(off / p.Wf), c0 = (int)(off % p.Wf);
    const bool norm = flags & 1, rep = (flags >> 1) & 1;
    const float *tap[3][3];
    bool ok[3][3];
    for (int dy = 0; dy < 3; ++dy)
        for (int dx = 0; dx < 3; ++dx) {
            int r = r0 + dy - 1, c = c0 + dx - 1;
            ok[dy][dx] = r >= 0 && r < p.Hf && c >= 0 && c < p.Wf;
            if (rep) {
                r = std::min(std::max(r, 0), p.Hf - 1);
                c = std::min(std::max(c, 0), p.Wf - 1);
                ok[dy][dx] = true;
            }
            tap[dy][dx] = ok[dy][dx] ? feat + ((long)r * p.Wf + c) * p.cstride : nullptr;
        }
    double a[6] = {0, 0, 0, 0, 0, 0};
    for (int ch = p.c_begin; ch < p.c_end; ++ch) {
        double v[3][3];
        for (int dy = 0; dy < 3; ++dy)
            for (int dx = 0; dx < 3; ++dx) v[dy][dx] = ok[dy][dx] ? (double)tap[dy][dx][ch] : 0.0;
        double g = (v[0][2] + 2.0 * v[1][2] + v[2][2]) - (v[0][0] + 2.0 * v[1][0] + v[2][0]);
        double h = (v[2][0] + 2.0 * v[2][1] + v[2][2]) - (v[0][0] + 2.0 * v[0][1] + v[0][2]);
        if (norm) {
            g *= 0.125;
            h *= 0.125;
        }
        const double e = v[1][1] - (double)fr[ch];
        a[0] += e * e;
        a[1] += g * e;
        a[2] += h * e;
        a[3] += g * g;
        a[4] += g * h;
        a[5] += h * h;
    }
    memcpy(out, a, sizeof(a));
}

struct Eval {
    double cost;      // mean rho over the kept points (NaN when none)
    int nsup, kept;
    double H[21], g[6];  // upper triangle of H row by row, then g
};

// so3exp_map (helpers/utils.py:209-221) and the update R' = dR R, t' = dR t + dt (model.py:416-426)
void step_pose(const double R[9], const double t[3], const double d[6], double Rn[9], double tn[3]) {
    const double w[3] = {d[3], d[4], d[5]};
    const double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    double dR[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (isnan(th)) {
        for (double &x : dR) x = NAN;
    } else if (th >= 1e-12) {
        const double k0 = w[0] / th, k1 = w[1] / th, k2 = w[2] / th;
        const double W[9] = {0, -k2, k1, k2, 0, -k0, -k1, k0, 0};
        const double sn = sin(th), c1 = 1.0 - cos(th);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                const double ww = W[3 * i] * W[j] + W[3 * i + 1] * W[3 + j] + W[3 * i + 2] * W[6 + j];
                dR[3 * i + j] += W[3 * i + j] * sn + ww * c1;
            }
    }
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) Rn[3 * i + j] = dR[3 * i] * R[j] + dR[3 * i + 1] * R[3 + j] + dR[3 * i + 2] * R[6 + j];
        tn[i] = (dR[3 * i] * t[0] + dR[3 * i + 1] * t[1] + dR[3 * i + 2] * t[2]) + d[i];
    }
}

// optimizer_step (model.py:37-72): delta = -lr * (H + lambda diag(diag(H) + 1e-9))^-1 g, LU with
// partial pivoting (getrf's pivot choice: the first largest |a|)
void damped_step(const double Hu[21], const double g[6], double lambda, double lr, double delta[6]) {
    double A[6][6], b[6];
    for (int i = 0, k = 0; i < 6; ++i)
        for (int j = i; j < 6; ++j, ++k) A[i][j] = A[j][i] = Hu[k];
    if (lambda != 0.0)
        for (int i = 0; i < 6; ++i) A[i][i] = A[i][i] + (A[i][i] + 1e-9) * lambda;
    memcpy(b, g, sizeof(b));
    for (int j = 0; j < 6; ++j) {
        int piv = j;
        for (int i = j + 1; i < 6; ++i)
            if (fabs(A[i][j]) > fabs(A[piv][j])) piv = i;
        if (piv != j) {
            std::swap(A[piv], A[j]);
            std::swap(b[piv], b[j]);
        }
        const double inv = 1.0 / A[j][j];
        for (int i = j + 1; i < 6; ++i) {
            const double m = A[i][j] * inv;
            for (int k = j + 1; k < 6; ++k) A[i][k] -= m * A[j][k];
            b[i] -= m * b[j];
        }
    }
    for (int i = 5; i >= 0; --i) {
        double v = b[i];
        for (int k = i + 1; k < 6; ++k) v -= A[i][k] * delta[k];
        delta[i] = v / A[i][i];
    }
    for (int i = 0; i < 6; ++i) delta[i] = -lr * delta[i];
}

// One problem, whole LM loop.  rec: per point {six sums, texel}, reused across evaluations.
class Problem {
  public:
    Problem(const fmpnp_problem &p, const fmpnp_options &o) : p_(p), o_(o), sums_(6 * (size_t)p.N), tex_(p.N, -2),
                                                              rho_(p.N), d1_(p.N), off_(p.N), P_(3 * (size_t)p.N) {}

    void run(fmpnp_result &r, fmpnp_trace_entry *tr, int trace_stride) {
        memset(&r, 0, sizeof(r));
        double R[9], t[3], Rb[9], tb[3];
        memcpy(R, p_.R0, sizeof(R));
        memcpy(t, p_.t0, sizeof(t));
        memcpy(Rb, R, sizeof(R));
        memcpy(tb, t, sizeof(t));
        double lambda = o_.lambda0, lr = 1.0, prev = NAN, best = NAN;
        r.initial_cost = NAN;
        r.best_cost = NAN;
        r.best_num_inliers = -1;
        Eval cur{}, ev{};
        bool ret_current = false;
        auto track = [&](const double *Re, const double *te, const Eval &e, bool acc) {
            if (!tr || r.n_evals >= trace_stride) return;
            fmpnp_trace_entry &x = tr[r.n_evals];
            memcpy(x.R, Re, sizeof(x.R));
            memcpy(x.t, te, sizeof(x.t));
            x.cost = e.cost;
            x.lambda_after = lambda;
            x.lr_after = lr;
            x.n_supported = e.nsup;
            x.n_kept = e.kept;
            x.accepted = acc ? 1 : 0;
        };
        if (o_.mode == FMPNP_MODE_COMPUTE_COST) {  // compute_cost (model.py:216-243) at (R0, t0)
            evaluate(R, t, false, ev);
            r.initial_cost = ev.nsup == 0 ? NAN : ev.cost;
            if (ev.nsup == 0) r.status |= FMPNP_STATUS_NO_SUPPORT;
            r.n_evals = 1;  // (no trace entry: the LM kernel's books are the same)
            ret_current = true;
        } else if (o_.n_iters > 0) {
            evaluate(R, t, true, cur);  // model.py:300-359
            if (cur.nsup == 0) {        // model.py:316-320: the current pose, nothing set (no evaluation booked)
                r.status |= FMPNP_STATUS_NO_SUPPORT;
                ret_current = true;
            } else {
                prev = best = r.initial_cost = cur.cost;
                r.best_num_inliers = cur.kept;
                r.has_best = 1;
                track(R, t, cur, true);
                r.n_evals = 1;
                for (int it = 0; it < o_.n_iters; ++it) {
                    double d[6], Rn[9], tn[3];
                    damped_step(cur.H, cur.g, lambda, lr, d);
                    r.n_steps++;  // (a NaN step counts, model.py:411-413)
                    bool bad = false;
                    for (double x : d) bad |= isnan(x);
                    if (bad) {
                        r.status |= FMPNP_STATUS_NAN;
                        break;
                    }
                    step_pose(R, t, d, Rn, tn);
                    evaluate(Rn, tn, true, ev);  // the trial (model.py:428-445) and its normal equations
                    if (ev.nsup == 0) {          // model.py:441-445: the current pose (the trial is not booked)
                        r.status |= FMPNP_STATUS_NO_SUPPORT_TRIAL;
                        ret_current = true;
                        break;
                    }
                    const bool accept = !(ev.cost > prev);  // model.py:469-486
                    lambda = std::min(std::max(lambda * (accept ? 0.1 : 10.0), 1e-6), 1e4);
                    lr = accept ? 1.0 : std::min(std::max(0.1 * lr, 1e-3), 1.0);
                    track(Rn, tn, ev, accept);
                    r.n_evals++;
                    if (!accept) continue;  // the cached linearisation at (R, t) stays
                    r.n_accepted++;
                    if (ev.cost < best) {
                        best = ev.cost;
                        r.best_num_inliers = ev.kept;
                        memcpy(Rb, Rn, sizeof(Rb));
                        memcpy(tb, tn, sizeof(tb));
                    }
                    prev = ev.cost;
                    memcpy(R, Rn, sizeof(R));
                    memcpy(t, tn, sizeof(t));
                    cur = ev;
                }
            }
        }
        memcpy(r.R, ret_current ? R : Rb, sizeof(r.R));
        memcpy(r.t, ret_current ? t : tb, sizeof(r.t));
        r.best_cost = r.has_best ? best : NAN;
        r.final_lambda = lambda;
        r.final_lr = lr;
        r.texel_gathers = gathers_;
    }

  private:
    void evaluate(const double R[9], const double t[3], bool normal, Eval &ev) {
        const int N = p_.N;
        const bool fp64 = o_.dtype == FMPNP_F64;
        const int loss = o_.mode == FMPNP_MODE_COMPUTE_COST ? (int)FMPNP_SQUARED : o_.loss;
        ev.nsup = 0;
        double rmax = -1.0;  // NaN-propagating max |rho| over the supported points (the ratio test)
        for (int i = 0; i < N; ++i) {
            off_[i] = texel_of(p_, R, t, p_.pts3d + 3 * (size_t)i, &P_[3 * (size_t)i]);
            if (off_[i] < 0) continue;
            ++ev.nsup;
            double *s = &sums_[6 * (size_t)i];
            if (off_[i] != tex_[i]) {  // the texel changed: read it (otherwise its sums are reused)
                if (o_.layout == FMPNP_LAYOUT_F)
                    sums_f((const float *)p_.feat, (const float *)p_.fref + (size_t)i * p_.ld_ref, p_, off_[i],
                           o_.sobel_flags, s);
                else if (fp64)
                    sums_fgrad((const double *)p_.feat + off_[i] * 3 * p_.cstride,
                               (const double *)p_.fref + (size_t)i * p_.ld_ref, p_.cstride, p_.c_begin, p_.c_end, s);
                else
                    sums_fgrad((const float *)p_.feat + off_[i] * 3 * p_.cstride,
                               (const float *)p_.fref + (size_t)i * p_.ld_ref, p_.cstride, p_.c_begin, p_.c_end, s);
                tex_[i] = off_[i];
                ++gathers_;
            }
            loss_cpu(loss, o_.barron_alpha, 0.5 * s[0], rho_[i], d1_[i]);
            const double a = fabs(rho_[i]);
            if (isnan(a) || a > rmax) rmax = isnan(rmax) ? rmax : a;
        }
        const bool ratio = o_.use_ratio != 0;
        const double limit = rmax * o_.ratio_threshold;  // model.py:120-129
        double csum = 0.0;
        ev.kept = 0;
        memset(ev.H, 0, sizeof(ev.H));
        memset(ev.g, 0, sizeof(ev.g));
        const double fx = p_.K[0], fy = p_.K[4];
        for (int i = 0; i < N; ++i) {
            if (off_[i] < 0) continue;
            if (ratio && !(fabs(rho_[i]) < limit)) continue;
            ++ev.kept;
            csum += rho_[i];
            if (!normal) continue;
            // A = J_px_p (model.py:377-382) J_p_T (model.py:369-370), 2 x 6; w folded into the 2 x 2 moments
            const double *P = &P_[3 * (size_t)i], *s = &sums_[6 * (size_t)i];
            const double z = P[2], iz = 1.0 / z;
            const double j00 = fx * iz, j02 = ((-fx) * P[0] * iz) * iz, j11 = fy * iz, j12 = ((-fy) * P[1] * iz) * iz;
            const double A0[6] = {j00, 0.0, j02, j02 * P[1], j00 * z - j02 * P[0], -j00 * P[1]};
            const double A1[6] = {0.0, j11, j12, -j11 * z + j12 * P[1], -j12 * P[0], j11 * P[0]};
            const double w = d1_[i];
            const double wxx = w * s[3], wxy = w * s[4], wyy = w * s[5], wex = w * s[1], wey = w * s[2];
            double M0[6], M1[6];
            for (int l = 0; l < 6; ++l) {
                M0[l] = wxx * A0[l] + wxy * A1[l];
                M1[l] = wxy * A0[l] + wyy * A1[l];
            }
            for (int a = 0, k = 0; a < 6; ++a) {
                for (int b = a; b < 6; ++b, ++k) ev.H[k] += A0[a] * M0[b] + A1[a] * M1[b];
                ev.g[a] += A0[a] * wex + A1[a] * wey;
            }
        }
        ev.cost = csum / (double)ev.kept;  // torch mean of an empty tensor: NaN
    }

    const fmpnp_problem &p_;
    const fmpnp_options &o_;
    std::vector<double> sums_;
    std::vector<long> tex_;
    std::vector<double> rho_, d1_;
    std::vector<long> off_;
    std::vector<double> P_;
    long long gathers_ = 0;
};

int validate(const fmpnp_problem &p, const fmpnp_options &o) {
    if (p.N < 0 || p.Hf <= 0 || p.Wf <= 0 || p.im_width <= 0 || p.im_height <= 0) return FMPNP_EINVAL;
    if (p.c_begin < 0 || p.c_end <= p.c_begin || p.c_end > p.cstride || p.ld_ref < p.c_end) return FMPNP_EINVAL;
    if (p.N > 0 && (!p.feat || !p.fref || !p.pts3d)) return FMPNP_EINVAL;
    if (p.window) return FMPNP_EINVAL;  // (windowed packs are a device-side economy)
    if (o.layout == FMPNP_LAYOUT_F && o.dtype != FMPNP_F32) return FMPNP_EINVAL;
    return 0;
}

}  // namespace

extern "C" int fmpnp_refine_batch_cpu(const fmpnp_problem *probs, int n, const fmpnp_options *opt,
                                      fmpnp_result *results, fmpnp_trace_entry *trace, int trace_stride,
                                      int n_threads) {
    if (n == 0) return 0;
    if (n < 0 || !probs || !opt || !results || (trace && trace_stride < 1)) return FMPNP_EINVAL;
    const fmpnp_options o = *opt;
    if (o.mode != FMPNP_MODE_FORWARD && o.mode != FMPNP_MODE_COMPUTE_COST) return FMPNP_EINVAL;
    if (o.sampling != FMPNP_NEAREST || (o.dtype != FMPNP_F32 && o.dtype != FMPNP_F64)) return FMPNP_EINVAL;
    if (o.layout != FMPNP_LAYOUT_FGRAD && o.layout != FMPNP_LAYOUT_F) return FMPNP_EINVAL;
    if (o.loss < FMPNP_SQUARED || o.loss > FMPNP_BARRON) return FMPNP_EINVAL;
    for (int i = 0; i < n; ++i) {
        const int rc = validate(probs[i], o);
        if (rc) return rc;
    }
    if (trace) memset(trace, 0, sizeof(fmpnp_trace_entry) * (size_t)n * trace_stride);
    int nt = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
    nt = std::min(nt, n);
    std::atomic<int> next{0};
    auto work = [&]() {
        for (int i; (i = next.fetch_add(1)) < n;) {
            Problem pr(probs[i], o);
            pr.run(results[i], trace ? trace + (size_t)i * trace_stride : nullptr, trace_stride);
        }
    };
    if (nt == 1) {
        work();
        return 0;
    }
    std::vector<std::thread> pool;
    for (int k = 0; k < nt; ++k) pool.emplace_back(work);
    for (auto &th : pool) th.join();
    return 0;
}
