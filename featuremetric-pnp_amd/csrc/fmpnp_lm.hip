// fmpnp_lm.hip -- the feature-metric LM refiner on gfx950 (MI355X).
//
// One launch runs the WHOLE Levenberg-Marquardt loop of every problem of a batch
// (sparseFeaturePnP.forward, featurePnP/model.py:245-494) on the device.
//
// Work decomposition
//   * A "team" of G workgroups (256 threads each) owns one problem at a time;
//     teams walk the batch persistently (problem = team, team + T, ...).
//   * Points are cut into chunks of CH = 16.  Workgroup s of a team owns a
//     contiguous range of chunks.  Per evaluation it
//       A0  projects its points (thread per point, fp64, exact pixel rounding),
//       A   gathers f / gx / gy / fref at the nearest texel with one 16-lane group
//           per point -- 16-byte loads of the channels-last [H][W][3][C] texel, so a
//           point's channels are one contiguous coalesced read -- and reduces the six
//           channel sums  sum e^2, sum gx e, sum gy e, sum gx^2, sum gx gy, sum gy^2
//           in fp64 (the C x 6 Jacobian is never materialised: J = G A with the 2x6
//           pose chain A, so J^T e = A^T (G^T e), J^T J = A^T (G^T G) A),
//       B   turns each point's record into its 21 + 6 normal-equation entries, its
//           rho and counters (thread per point) and reduces every chunk with a
//           fixed transposed shuffle tree to one 32-double partial.
//   * The chunk partials are summed in CHUNK ORDER.  Results are therefore
//     deterministic and independent of G: the LM accept test `new > prev`
//     (model.py:469-472) compares costs that tie exactly whenever the pixel sets
//     are equal, and a scheduling-dependent sum would break those ties.
//   * G > 1: chunk partials go to a per-team slot with write-through (sc1) stores,
//     every storing wave drains, one lane bumps the team's arrival counter, one
//     lane polls it (bounded spin), one agent-scope acquire, then every
//     workgroup re-reads all partials and runs the identical 6x6 solve + LM
//     update redundantly (no second exchange).
//   * One evaluation per iteration: the trial evaluation at (R', t') also
//     produces that pose's normal equations.  On acceptance they are the next
//     linearisation; on rejection the cached ones are reused -- bit-identical to
//     the reference's recomputation at the unchanged pose (model.py:472-476).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "fmpnp.h"
#include "fmpnp_device.h"
#include "fmpnp_internal.h"

namespace fmpnp {

struct LMState {
    double R[9], t[3];      // current (last accepted) pose
    double Re[9], te[3];    // pose evaluated next
    double Rb[9], tb[3];    // best pose
    double Hc[21], gc[6];   // cached linearisation at (R, t)
    double tot[NV];         // reduced totals of the last evaluation
    double lambda, lr, prev, best, initial, rho_max;
    int best_inl, n_evals, n_steps, n_accepted, status, done, has_best, ret_current;
    int abort_flag, pad_;
};
static_assert(sizeof(LMState) + 16 + 8 * (NT / 64) <= lds_fixed_bytes(), "LDS head too small");

// ---------------------------------------------------------------------------
// 6x6 damped solve (optimizer_step, model.py:37-72): LU with partial pivoting.
// ---------------------------------------------------------------------------
__device__ static void lm_step(const double *Hu, const double *g, double lambda, double lr, double delta[6]) {
    double A[36];
    int k = 0;
    for (int i = 0; i < 6; ++i)
        for (int j = i; j < 6; ++j, ++k) { A[6 * i + j] = Hu[k]; A[6 * j + i] = Hu[k]; }
    if (lambda != 0.0)
        for (int i = 0; i < 6; ++i) A[7 * i] = A[7 * i] + (A[7 * i] + 1e-9) * lambda;
    int piv[6];
    for (int j = 0; j < 6; ++j) {
        int p = j;
        double best = fabs(A[6 * j + j]);
        for (int i = j + 1; i < 6; ++i)
            if (fabs(A[6 * i + j]) > best) { best = fabs(A[6 * i + j]); p = i; }
        piv[j] = p;
        if (p != j)
            for (int c = 0; c < 6; ++c) { double tmp = A[6 * j + c]; A[6 * j + c] = A[6 * p + c]; A[6 * p + c] = tmp; }
        double inv = 1.0 / A[6 * j + j];
        for (int i = j + 1; i < 6; ++i) {
            A[6 * i + j] *= inv;
            for (int c = j + 1; c < 6; ++c) A[6 * i + c] -= A[6 * i + j] * A[6 * j + c];
        }
    }
    double b[6];
    for (int i = 0; i < 6; ++i) b[i] = g[i];
    for (int j = 0; j < 6; ++j)
        if (piv[j] != j) { double tmp = b[j]; b[j] = b[piv[j]]; b[piv[j]] = tmp; }
    for (int i = 0; i < 6; ++i)
        for (int c = 0; c < i; ++c) b[i] -= A[6 * i + c] * b[c];
    for (int i = 5; i >= 0; --i) {
        for (int c = i + 1; c < 6; ++c) b[i] -= A[6 * i + c] * b[c];
        b[i] /= A[6 * i + i];
    }
    for (int i = 0; i < 6; ++i) delta[i] = -lr * b[i];
}

// so3exp_map (helpers/utils.py:209-221) and the update R' = dR R, t' = dR t + dt
// (model.py:416-426).
__device__ static void pose_update(const double *R, const double *t, const double delta[6], double *Rn, double *tn) {
    const double *w = delta + 3;
    double theta = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    double dR[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (isnan(theta)) {
        for (int i = 0; i < 9; ++i) dR[i] = NAN;
    } else if (!(theta < 1e-12)) {
        double k0 = w[0] / theta, k1 = w[1] / theta, k2 = w[2] / theta;
        double W[9] = {0, -k2, k1, k2, 0, -k0, -k1, k0, 0};
        double s = sin(theta), c1 = 1.0 - cos(theta);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                double ww = W[3 * i + 0] * W[0 + j] + W[3 * i + 1] * W[3 + j] + W[3 * i + 2] * W[6 + j];
                dR[3 * i + j] += W[3 * i + j] * s + ww * c1;
            }
    }
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j)
            Rn[3 * i + j] = dR[3 * i + 0] * R[j] + dR[3 * i + 1] * R[3 + j] + dR[3 * i + 2] * R[6 + j];
        tn[i] = (dR[3 * i + 0] * t[0] + dR[3 * i + 1] * t[1] + dR[3 * i + 2] * t[2]) + delta[i];
    }
}

// ---------------------------------------------------------------------------
// Cross-workgroup exchange inside a team (G > 1).  Payload is stored write-through
// (sc1, agent-scope relaxed atomic stores); the arrival counter is monotonic within
// a launch and zeroed by the launcher (hipMemsetAsync) before every launch.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void st_sc1(double *p, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), __double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double *p) {
    return __longlong_as_double(__hip_atomic_load(reinterpret_cast<const unsigned long long *>(p), __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT));
}

// Every thread calls this after its sc1 stores.  Returns false on timeout.
__device__ static bool team_arrive_wait(unsigned *counter, unsigned target, int *lds_flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int ok = 1;
        // bounded spin: give up after ~2 s of wall time (s_memrealtime ticks at 100 MHz)
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) { ok = 0; break; }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        *lds_flag = ok;
    }
    __syncthreads();
    return *lds_flag != 0;
}

// ---------------------------------------------------------------------------
// phase A: one point's channel sums by a 16-lane group (l16 = lane in group).
// Lane l16 owns channels cb + l16*V + r*16*V + k (k < V, V = 16 B / sizeof(T)) and
// accumulates them in that order in BOTH forms, so the vector form (one 16-byte load
// per plane per round) and the scalar form (unaligned / ragged channel ranges) give
// bit-identical sums: a problem's result never depends on which form ran.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void acc6(double a[6], double f, double r, double gx, double gy) {
    double e = f - r;
    a[0] = fma(e, e, a[0]);
    a[1] = fma(gx, e, a[1]);
    a[2] = fma(gy, e, a[2]);
    a[3] = fma(gx, gx, a[3]);
    a[4] = fma(gx, gy, a[4]);
    a[5] = fma(gy, gy, a[5]);
}

template <typename T, bool VEC>
__device__ __forceinline__ void gather_sums(const T *__restrict__ tex, const T *__restrict__ fr, int cs, int cb,
                                            int ce, int l16, double a[6]) {
    using VT = typename V16<T>::type;
    constexpr int V = V16<T>::n;
    if constexpr (VEC) {
#pragma unroll 2
        for (int c = cb + l16 * V; c < ce; c += 16 * V) {
            VT fv = *reinterpret_cast<const VT *>(tex + c);
            VT xv = *reinterpret_cast<const VT *>(tex + cs + c);
            VT yv = *reinterpret_cast<const VT *>(tex + 2 * cs + c);
            VT rv = *reinterpret_cast<const VT *>(fr + c);
            const T *pf = reinterpret_cast<const T *>(&fv);
            const T *px = reinterpret_cast<const T *>(&xv);
            const T *py = reinterpret_cast<const T *>(&yv);
            const T *pr = reinterpret_cast<const T *>(&rv);
#pragma unroll
            for (int k = 0; k < V; ++k) acc6(a, (double)pf[k], (double)pr[k], (double)px[k], (double)py[k]);
        }
    } else {
        for (int c = cb + l16 * V; c < ce; c += 16 * V) {
#pragma unroll
            for (int k = 0; k < V; ++k)
                if (c + k < ce)
                    acc6(a, (double)tex[c + k], (double)fr[c + k], (double)tex[cs + c + k], (double)tex[2 * cs + c + k]);
        }
    }
}

// Transposed reduction of 8 values over the 16 lanes of a group: 7 shuffles instead
// of 8 x 4.  Returns the group total of value index (4*b3 + 2*b2 + b1) of l16.
__device__ __forceinline__ double reduce8_in16(double v[8], int l16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        bool hi = l16 & 8;
        double send = hi ? v[i] : v[i + 4];
        double keep = hi ? v[i + 4] : v[i];
        v[i] = keep + __shfl_xor(send, 8);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        bool hi = l16 & 4;
        double send = hi ? v[i] : v[i + 2];
        double keep = hi ? v[i + 2] : v[i];
        v[i] = keep + __shfl_xor(send, 4);
    }
    {
        bool hi = l16 & 2;
        double send = hi ? v[0] : v[1];
        double keep = hi ? v[1] : v[0];
        v[0] = keep + __shfl_xor(send, 2);
    }
    return v[0] + __shfl_xor(v[0], 1);
}

// Transposed reduction of NV = 32 values over 16 lanes: after it, lane l16 holds the
// group totals of indices start, start + 1 with start = 16 b3 + 8 b2 + 4 b1 + 2 b0.
__device__ __forceinline__ int reduce32_in16(double v[NV], int l16) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        bool hi = l16 & 8;
        double send = hi ? v[i] : v[i + 16];
        double keep = hi ? v[i + 16] : v[i];
        v[i] = keep + __shfl_xor(send, 8);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        bool hi = l16 & 4;
        double send = hi ? v[i] : v[i + 8];
        double keep = hi ? v[i + 8] : v[i];
        v[i] = keep + __shfl_xor(send, 4);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        bool hi = l16 & 2;
        double send = hi ? v[i] : v[i + 4];
        double keep = hi ? v[i + 4] : v[i];
        v[i] = keep + __shfl_xor(send, 2);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        bool hi = l16 & 1;
        double send = hi ? v[i] : v[i + 2];
        double keep = hi ? v[i + 2] : v[i];
        v[i] = keep + __shfl_xor(send, 1);
    }
    return 16 * ((l16 >> 3) & 1) + 8 * ((l16 >> 2) & 1) + 4 * ((l16 >> 1) & 1) + 2 * (l16 & 1);
}

// ---------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(NT) void lm_kernel(LaunchArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    LMState &st = *reinterpret_cast<LMState *>(smem);
    int *sync_flag = reinterpret_cast<int *>(smem + sizeof(LMState));
    double *wg_max = reinterpret_cast<double *>(smem + sizeof(LMState) + 16);  // [NT/64]
    unsigned char *dyn = smem + lds_fixed_bytes();
    const int G = a.G;
    // XCD-aware team placement: members of one team share blockIdx % 8 (same XCD under
    // the observed round-robin dispatch; speed only, never correctness).
    const int b = blockIdx.x, gw = a.gw;
    const int grp = b / (gw * G), rem = b % (gw * G);
    const int s = rem / gw;
    const int team = grp * gw + rem % gw;
    if (team >= a.teams) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = tid & 15, g16 = tid >> 4;
    unsigned epoch = 0;
    unsigned *counter = a.counters + team * 16;
    const fmpnp_options &op = a.opt;
    const bool cost_only = op.mode == FMPNP_MODE_COMPUTE_COST;
    const int loss = cost_only ? (int)FMPNP_SQUARED : op.loss;
    bool team_dead = false;

    for (int p = team; p < a.n; p += a.teams) {
        const fmpnp_problem &pb = a.probs[p];
        const int N = pb.N;
        const int NC = (N + CH - 1) / CH;
        const int c0 = (int)(((long)NC * s) / G), c1 = (int)(((long)NC * (s + 1)) / G);
        const int p0 = c0 * CH, p1 = min(c1 * CH, N), M = max(p1 - p0, 0);
        const int LC = c1 - c0;
        int *tex = reinterpret_cast<int *>(dyn);                                   // [Mmax]
        double *rec = reinterpret_cast<double *>(dyn + a.tex_bytes);             // [Mmax][RECW]
        double *part_lds = reinterpret_cast<double *>(dyn + a.tex_bytes + a.rec_bytes);  // [NC][NV] (G == 1)
        double *part_g = a.partials + (size_t)team * 2 * a.nc_max * NV;         // [2][NCmax][NV] (G > 1)
        double *max_g = a.maxslots + (size_t)team * 2 * a.G;                     // [2][G]
        const T *feat = reinterpret_cast<const T *>(pb.feat);
        const T *fref = reinterpret_cast<const T *>(pb.fref);
        const int cs = pb.cstride, cb = pb.c_begin, ce = pb.c_end;
        constexpr int V = V16<T>::n;
        const bool vec = ((((uintptr_t)pb.feat) | ((uintptr_t)pb.fref)) & 15) == 0 && cs % V == 0 &&
                         pb.ld_ref % V == 0 && cb % V == 0 && (ce - cb) % V == 0;

        if (tid == 0) {
            for (int i = 0; i < 9; ++i) { st.R[i] = st.Re[i] = st.Rb[i] = pb.R0[i]; }
            for (int i = 0; i < 3; ++i) { st.t[i] = st.te[i] = st.tb[i] = pb.t0[i]; }
            st.lambda = op.lambda0;
            st.lr = 1.0;
            st.prev = st.best = st.initial = NAN;
            st.best_inl = -1;
            st.n_evals = st.n_steps = st.n_accepted = 0;
            st.status = team_dead ? FMPNP_STATUS_SYNC_TIMEOUT : 0;
            st.has_best = 0;
            st.ret_current = 0;
            st.done = team_dead || (!cost_only && op.n_iters <= 0);
            st.abort_flag = 0;
        }
        __syncthreads();

        while (!st.done) {
            // ---- A0: projection (thread per local point) ---------------------
            for (int i = tid; i < M; i += NT) {
                const double *X = pb.pts3d + 3 * (size_t)(p0 + i);
                double P[3];
                transform_pt(st.Re, st.te, X[0], X[1], X[2], P);
                int x, y;
                int off = -1;
                if (project_px(pb.K, P, pb.im_width, pb.im_height, x, y)) {
                    // indexing_ (model.py:88-89): floor(y*Hf/H), floor(x*Wf/W), exact in integers
                    int row = (int)(((long)y * pb.Hf) / pb.im_height);
                    int col = (int)(((long)x * pb.Wf) / pb.im_width);
                    off = row * pb.Wf + col;
                }
                tex[i] = off;
            }
            __syncthreads();
            // ---- A: channel sums per point (16-lane group per point) ----------
            for (int i = g16; i < M; i += NGRP) {
                const int off = tex[i];
                double v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                if (off >= 0) {
                    const T *texp = feat + (size_t)off * 3 * cs;
                    const T *frp = fref + (size_t)(p0 + i) * pb.ld_ref;
                    if (vec) gather_sums<T, true>(texp, frp, cs, cb, ce, l16, v);
                    else gather_sums<T, false>(texp, frp, cs, cb, ce, l16, v);
                }
                double r = reduce8_in16(v, l16);
                int idx = 4 * ((l16 >> 3) & 1) + 2 * ((l16 >> 2) & 1) + ((l16 >> 1) & 1);
                if ((l16 & 1) == 0 && idx < 6) rec[(size_t)i * RECW + idx] = r;
            }
            __syncthreads();
            // ---- B1: rho per point; team max |rho| for the ratio test ---------
            const bool ratio = op.use_ratio != 0;
            {
                double lmax = -1.0;  // -1: nothing supported seen yet
                for (int i = tid; i < M; i += NT) {
                    double rho = 0.0, d1 = 0.0;
                    if (tex[i] >= 0) {
                        loss_eval(loss, op.barron_alpha, 0.5 * rec[(size_t)i * RECW + 0], rho, d1);
                        double am = fabs(rho);
                        if (isnan(am) || am > lmax) lmax = isnan(lmax) ? lmax : am;
                    }
                    rec[(size_t)i * RECW + 6] = rho;
                    rec[(size_t)i * RECW + 7] = d1;
                }
                if (ratio) {
                    // wave max then workgroup max (max is order-independent: exact)
                    for (int o = 32; o > 0; o >>= 1) {
                        double other = __shfl_xor(lmax, o);
                        if (isnan(other) || other > lmax) lmax = isnan(lmax) ? lmax : other;
                    }
                    if (lane == 0) wg_max[wave] = lmax;
                    __syncthreads();
                    if (tid == 0) {
                        double m = wg_max[0];
                        for (int w = 1; w < NT / 64; ++w)
                            if (isnan(wg_max[w]) || wg_max[w] > m) m = isnan(m) ? m : wg_max[w];
                        st.rho_max = m;
                    }
                    __syncthreads();
                    if (G > 1) {
                        ++epoch;
                        if (tid == 0) st_sc1(max_g + (epoch & 1) * G + s, st.rho_max);
                        if (!team_arrive_wait(counter, epoch * (unsigned)G, sync_flag)) {
                            if (tid == 0) st.abort_flag = 1;
                        } else if (tid == 0) {
                            double m = -1.0;
                            for (int w = 0; w < G; ++w) {
                                double o = ld_sc1(max_g + (epoch & 1) * G + w);
                                if (isnan(o) || o > m) m = isnan(m) ? m : o;
                            }
                            st.rho_max = m;
                        }
                        __syncthreads();
                        if (st.abort_flag) break;
                    }
                }
            }
            // ---- B2: normal-equation contributions, chunk partials ------------
            {
                const double limit = st.rho_max * op.ratio_threshold;
                const double fx = pb.K[0], fy = pb.K[4];
                for (int base = wave * 4; base < LC; base += 4 * (NT / 64)) {
                    const int lc = base + (lane >> 4);
                    const int i = lc * CH + l16;  // local point index
                    double v[NV];
#pragma unroll
                    for (int k = 0; k < NV; ++k) v[k] = 0.0;
                    if (lc < LC && i < M && tex[i] >= 0) {
                        const double *r = rec + (size_t)i * RECW;
                        const double rho = r[6], w = r[7];
                        v[29] = 1.0;  // supported
                        if (!ratio || fabs(rho) < limit) {
                            v[27] = rho;
                            v[28] = 1.0;  // kept
                            const double *X = pb.pts3d + 3 * (size_t)(p0 + i);
                            double P[3];
                            transform_pt(st.Re, st.te, X[0], X[1], X[2], P);
                            const double z = P[2];
                            // J_px_p (model.py:377-382) times J_p_T (model.py:369-370): A (2x6)
                            const double j00 = fx / z, j02 = ((-fx) * P[0] / z) / z;
                            const double j11 = fy / z, j12 = ((-fy) * P[1] / z) / z;
                            double A0[6] = {j00, 0.0, j02, j02 * P[1], j00 * P[2] - j02 * P[0], -j00 * P[1]};
                            double A1[6] = {0.0, j11, j12, -j11 * P[2] + j12 * P[1], -j12 * P[0], j11 * P[0]};
                            const double sex = r[1], sey = r[2], sxx = r[3], sxy = r[4], syy = r[5];
                            double M0[6], M1[6];
#pragma unroll
                            for (int l = 0; l < 6; ++l) {
                                M0[l] = sxx * A0[l] + sxy * A1[l];
                                M1[l] = sxy * A0[l] + syy * A1[l];
                            }
                            int kk = 0;
#pragma unroll
                            for (int k = 0; k < 6; ++k)
#pragma unroll
                                for (int l = k; l < 6; ++l, ++kk) v[kk] = w * (A0[k] * M0[l] + A1[k] * M1[l]);
#pragma unroll
                            for (int k = 0; k < 6; ++k) v[21 + k] = w * (A0[k] * sex + A1[k] * sey);
                        }
                    }
                    const int start = reduce32_in16(v, l16);
                    if (lc < LC) {
                        const int chunk = c0 + lc;
                        if (G == 1) {
                            part_lds[chunk * NV + start] = v[0];
                            part_lds[chunk * NV + start + 1] = v[1];
                        } else {
                            double *dst = part_g + ((size_t)((epoch + 1) & 1) * a.nc_max + chunk) * NV;
                            st_sc1(dst + start, v[0]);
                            st_sc1(dst + start + 1, v[1]);
                        }
                    }
                }
            }
            if (G == 1) {
                __syncthreads();
                if (tid < NV) {
                    double acc = 0.0;
                    for (int c = 0; c < NC; ++c) acc += part_lds[c * NV + tid];
                    st.tot[tid] = acc;
                }
            } else {
                ++epoch;
                if (!team_arrive_wait(counter, epoch * (unsigned)G, sync_flag)) {
                    if (tid == 0) st.abort_flag = 1;
                } else if (tid < NV) {
                    const double *src = part_g + (size_t)(epoch & 1) * a.nc_max * NV;
                    double acc = 0.0;
                    for (int c = 0; c < NC; ++c) acc += ld_sc1(src + c * NV + tid);
                    st.tot[tid] = acc;
                }
            }
            __syncthreads();
            if (st.abort_flag) break;

            // ---- LM state machine (one lane; every team member computes it identically)
            if (tid == 0) {
                const int nsup = (int)st.tot[29];
                const int kept = (int)st.tot[28];
                const double cost = st.tot[27] / st.tot[28];  // torch mean of empty = NaN
                if (cost_only) {
                    st.initial = nsup == 0 ? NAN : cost;
                    if (nsup == 0) st.status |= FMPNP_STATUS_NO_SUPPORT;
                    st.n_evals = 1;
                    st.done = 1;
                } else {
                    fmpnp_trace_entry *tr = a.trace ? a.trace + (size_t)p * a.trace_stride : nullptr;
                    const bool first = st.n_evals == 0;
                    bool accepted = true;
                    if (nsup == 0) {  // model.py:316-320 / :441-445: return the current pose
                        st.status |= first ? FMPNP_STATUS_NO_SUPPORT : FMPNP_STATUS_NO_SUPPORT_TRIAL;
                        st.ret_current = 1;
                        st.done = 1;
                    } else if (first) {  // model.py:347-359
                        st.prev = st.best = st.initial = cost;
                        st.best_inl = kept;
                        st.has_best = 1;
                        for (int k = 0; k < 21; ++k) st.Hc[k] = st.tot[k];
                        for (int k = 0; k < 6; ++k) st.gc[k] = st.tot[21 + k];
                    } else {  // model.py:469-486
                        accepted = !(cost > st.prev);
                        double lam = st.lambda * (cost > st.prev ? 10.0 : 0.1);
                        st.lambda = lam < 1e-6 ? 1e-6 : (lam > 1e4 ? 1e4 : lam);
                        if (!accepted) {
                            double lr = 0.1 * st.lr;
                            st.lr = lr < 1e-3 ? 1e-3 : (lr > 1.0 ? 1.0 : lr);
                        } else {
                            st.lr = 1.0;
                            st.n_accepted++;
                            if (cost < st.best) {
                                for (int k = 0; k < 9; ++k) st.Rb[k] = st.Re[k];
                                for (int k = 0; k < 3; ++k) st.tb[k] = st.te[k];
                                st.best_inl = kept;
                                st.best = cost;
                            }
                            st.prev = cost;
                            for (int k = 0; k < 9; ++k) st.R[k] = st.Re[k];
                            for (int k = 0; k < 3; ++k) st.t[k] = st.te[k];
                            for (int k = 0; k < 21; ++k) st.Hc[k] = st.tot[k];
                            for (int k = 0; k < 6; ++k) st.gc[k] = st.tot[21 + k];
                        }
                    }
                    if (nsup != 0) {
                        if (tr && s == 0 && st.n_evals < a.trace_stride) {
                            fmpnp_trace_entry &e = tr[st.n_evals];
                            for (int k = 0; k < 9; ++k) e.R[k] = st.Re[k];
                            for (int k = 0; k < 3; ++k) e.t[k] = st.te[k];
                            e.cost = cost;
                            e.lambda_after = st.lambda;
                            e.lr_after = st.lr;
                            e.n_supported = nsup;
                            e.n_kept = kept;
                            e.accepted = accepted ? 1 : 0;
                        }
                        st.n_evals++;
                        if (st.n_steps >= op.n_iters) st.done = 1;
                    }
                    if (!st.done) {  // next step from the cached linearisation
                        double delta[6];
                        lm_step(st.Hc, st.gc, st.lambda, st.lr, delta);
                        st.n_steps++;
                        bool bad = false;
                        for (int k = 0; k < 6; ++k) bad |= isnan(delta[k]);
                        if (bad) {  // model.py:411-413
                            st.status |= FMPNP_STATUS_NAN;
                            st.done = 1;
                        } else {
                            pose_update(st.R, st.t, delta, st.Re, st.te);
                        }
                    }
                }
            }
            __syncthreads();
        }
        if (st.abort_flag) {
            team_dead = true;  // a member vanished: finish every remaining problem as failed
            if (tid == 0) st.status |= FMPNP_STATUS_SYNC_TIMEOUT;
        }
        // ---- result ---------------------------------------------------------
        if (s == 0 && tid == 0) {
            fmpnp_result &r = a.results[p];
            const bool cur = st.ret_current || cost_only;
            for (int k = 0; k < 9; ++k) r.R[k] = cur ? st.R[k] : st.Rb[k];
            for (int k = 0; k < 3; ++k) r.t[k] = cur ? st.t[k] : st.tb[k];
            r.initial_cost = st.initial;
            r.best_cost = st.has_best ? st.best : NAN;
            r.final_lambda = st.lambda;
            r.final_lr = st.lr;
            r.best_num_inliers = st.has_best ? st.best_inl : -1;
            r.n_evals = st.n_evals;
            r.n_steps = st.n_steps;
            r.n_accepted = st.n_accepted;
            r.status = st.status;
            r.has_best = st.has_best;
        }
        __syncthreads();
    }
}

// explicit instantiations + a dispatch table for the launcher
template __global__ void lm_kernel<float>(LaunchArgs);
template __global__ void lm_kernel<double>(LaunchArgs);

hipError_t launch_lm(const LaunchArgs &a, int dtype, int grid, size_t lds, hipStream_t stream) {
    if (dtype == FMPNP_F32) hipLaunchKernelGGL((lm_kernel<float>), dim3(grid), dim3(NT), lds, stream, a);
    else hipLaunchKernelGGL((lm_kernel<double>), dim3(grid), dim3(NT), lds, stream, a);
    return hipGetLastError();
}

const void *lm_kernel_ptr(int dtype) {
    return dtype == FMPNP_F32 ? (const void *)lm_kernel<float> : (const void *)lm_kernel<double>;
}

}  // namespace fmpnp
