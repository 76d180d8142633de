// fmpnp_points.hip -- per-point residual costs at one pose (fmpnp_point_costs): the
// projection, points_within_image and indexing_ of find_inliers (featurePnP/model.py:132-146),
// on a packed map of either layout.  The LM kernel never needs per-point output; this is
// the building block of the façade's find_inliers / feature_pnp_multi
// (s2dhm/pose_prediction/optimize_feature_pnp.py:20-47).
//
// One wave per point (4 per 256-thread workgroup): the lanes read the point's texel row of the
// f plane (channels-last: one coalesced run of c_end - c_begin values) and its descriptor, and
// a butterfly reduction sums the squared differences in fp64.  Pixels use the LM kernel's
// transform_pt / project_px, so the support set is the reference's bit for bit.
#include "fmpnp_device.h"
#include "fmpnp_internal.h"

namespace fmpnp {

struct PointCostArgs {
    double K[9], R[9], t[3];
    int N, Hf, Wf, cstride, c_begin, c_end, ld_ref, im_w, im_h, planes;
};

template <typename T>
__global__ __launch_bounds__(256) void point_cost_kernel(const T *__restrict__ feat, const T *__restrict__ fref,
                                                         const double *__restrict__ pts, PointCostArgs a,
                                                         double *__restrict__ cost, int *__restrict__ supported) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.N) return;  // wave-uniform
    double P[3];
    transform_pt(a.R, a.t, pts[3 * i], pts[3 * i + 1], pts[3 * i + 2], P);
    int x = 0, y = 0;
    double qx, qy;
    const bool in = project_px(a.K, P, a.im_w, a.im_h, x, y, qx, qy);  // model.py:134-138
    double s = 0.0;
    if (in) {
        // indexing_ (model.py:88-89): floor(y Hf / H), floor(x Wf / W) of exact integer products
        const int row = (int)(((unsigned)y * (unsigned)a.Hf) / (unsigned)a.im_h);
        const int col = (int)(((unsigned)x * (unsigned)a.Wf) / (unsigned)a.im_w);
        const T *f = feat + ((size_t)row * a.Wf + col) * (size_t)a.planes * a.cstride;  // plane 0 = f
        const T *r = fref + (size_t)i * a.ld_ref;
        for (int c = a.c_begin + lane; c < a.c_end; c += 64) {
            const double e = (double)f[c] - (double)r[c];  // model.py:144
            s += e * e;
        }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
    if (lane == 0) {
        cost[i] = in ? 0.5 * s : 0.0;  // model.py:146
        supported[i] = in ? 1 : 0;
    }
}

hipError_t launch_point_costs(const fmpnp_problem &p, int layout, int dtype, double *cost, int *supported,
                              hipStream_t stream) {
    PointCostArgs a;
    for (int k = 0; k < 9; ++k) {
        a.K[k] = p.K[k];
        a.R[k] = p.R0[k];
    }
    for (int k = 0; k < 3; ++k) a.t[k] = p.t0[k];
    a.N = p.N;
    a.Hf = p.Hf;
    a.Wf = p.Wf;
    a.cstride = p.cstride;
    a.c_begin = p.c_begin;
    a.c_end = p.c_end;
    a.ld_ref = p.ld_ref;
    a.im_w = p.im_width;
    a.im_h = p.im_height;
    a.planes = layout == FMPNP_LAYOUT_F ? 1 : 3;
    const unsigned grid = (unsigned)((p.N + 3) / 4);
    if (dtype == FMPNP_F32)
        hipLaunchKernelGGL(point_cost_kernel<float>, dim3(grid), dim3(256), 0, stream, (const float *)p.feat,
                           (const float *)p.fref, p.pts3d, a, cost, supported);
    else
        hipLaunchKernelGGL(point_cost_kernel<double>, dim3(grid), dim3(256), 0, stream, (const double *)p.feat,
                           (const double *)p.fref, p.pts3d, a, cost, supported);
    return hipGetLastError();
}

// compute_cost (featurePnP/model.py:216-243) from the per-point costs: ONE workgroup, a fixed
// summation order (thread t sums points t, t + 256, ... in order, then a fixed tree), so the value
// depends only on the costs.  With the ratio test the points with |cost| >= max|cost| * thr over the
// supported ones are dropped (ratio_threshold_feature_errors, model.py:120-129: a NaN maximum keeps
// none); the mean over none is NaN (torch's mean of an empty tensor).  No supported point: status
// NO_SUPPORT (the reference returns None, model.py:226-227).
struct CostMeanArgs {
    double R[9], t[3];
    int N, use_ratio;
    double thr;
};
__global__ __launch_bounds__(256) void cost_mean_kernel(const double *__restrict__ cost, const int *__restrict__ sup,
                                                        CostMeanArgs a, fmpnp_result *__restrict__ out) {
    __shared__ double sh[256];
    __shared__ int shn[256];
    const int t = threadIdx.x;
    double mx = -1.0;  // (costs are >= 0 or NaN)
    int ns = 0;
    for (int i = t; i < a.N; i += 256)
        if (sup[i]) {
            ++ns;
            const double c = fabs(cost[i]);
            mx = (isnan(c) || isnan(mx)) ? NAN : fmax(mx, c);
        }
    sh[t] = mx;
    shn[t] = ns;
    __syncthreads();
    for (int w = 128; w >= 1; w >>= 1) {
        if (t < w) {
            const double o = sh[t + w];
            sh[t] = (isnan(o) || isnan(sh[t])) ? NAN : fmax(sh[t], o);
            shn[t] += shn[t + w];
        }
        __syncthreads();
    }
    const double limit = sh[0] * a.thr;
    const int n_sup = shn[0];
    __syncthreads();
    double s = 0.0;
    int nk = 0;
    for (int i = t; i < a.N; i += 256)
        if (sup[i] && (!a.use_ratio || fabs(cost[i]) < limit)) {
            s += cost[i];
            ++nk;
        }
    sh[t] = s;
    shn[t] = nk;
    __syncthreads();
    for (int w = 128; w >= 1; w >>= 1) {
        if (t < w) {
            sh[t] += sh[t + w];
            shn[t] += shn[t + w];
        }
        __syncthreads();
    }
    if (t == 0) {
        fmpnp_result r;
        for (int k = 0; k < 9; ++k) r.R[k] = a.R[k];
        for (int k = 0; k < 3; ++k) r.t[k] = a.t[k];
        r.initial_cost = n_sup ? (shn[0] ? sh[0] / (double)shn[0] : NAN) : NAN;
        r.best_cost = NAN;
        r.final_lambda = r.final_lr = NAN;
        r.best_num_inliers = -1;
        r.n_evals = 1;
        r.n_steps = r.n_accepted = 0;
        r.status = n_sup ? 0 : FMPNP_STATUS_NO_SUPPORT;
        r.has_best = 0;
        r.texel_gathers = n_sup;
        *out = r;
    }
}

hipError_t launch_compute_cost(const fmpnp_problem &p, int layout, int dtype, int use_ratio, double thr,
                               double *cost, int *supported, fmpnp_result *out, hipStream_t stream) {
    if (p.N > 0) {
        const hipError_t e = launch_point_costs(p, layout, dtype, cost, supported, stream);
        if (e != hipSuccess) return e;
    }
    return launch_cost_mean(p, use_ratio, thr, cost, supported, out, stream);
}

hipError_t launch_cost_mean(const fmpnp_problem &p, int use_ratio, double thr, const double *cost,
                            const int *supported, fmpnp_result *out, hipStream_t stream) {
    CostMeanArgs a;
    for (int k = 0; k < 9; ++k) a.R[k] = p.R0[k];
    for (int k = 0; k < 3; ++k) a.t[k] = p.t0[k];
    a.N = p.N;
    a.use_ratio = use_ratio;
    a.thr = thr;
    hipLaunchKernelGGL(cost_mean_kernel, dim3(1), dim3(256), 0, stream, cost, supported, a, out);
    return hipGetLastError();
}

}  // namespace fmpnp
