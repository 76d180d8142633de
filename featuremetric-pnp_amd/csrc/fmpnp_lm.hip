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
//           point's channels are contiguous coalesced reads -- and reduces the six
//           channel sums  sum e^2, sum gx e, sum gy e, sum gx^2, sum gx gy, sum gy^2
//           in fp64 (the C x 6 Jacobian is never materialised: J = G A with the 2x6
//           pose chain A, so J^T e = A^T (G^T e), J^T J = A^T (G^T G) A),
//       B   turns each point's record into its 21 + 6 normal-equation entries, its
//           rho and counters (thread per point) and reduces every chunk with a
//           fixed transposed shuffle tree to one 32-double partial.
//   * The chunk partials are summed by a fixed tree over CHUNK INDICES.  Results are
//     therefore deterministic and independent of G: the LM accept test `new > prev`
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
//
// Code shape: every phase reads what it needs from LDS (the per-problem context `Ctx`
// and the LM state) after a barrier, so no value stays live in registers from one
// phase to the next; the 6x6 solve runs row-parallel on wave 0.  That keeps the
// 1024-thread workgroup within 128 VGPRs.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "fmpnp.h"
#include "fmpnp_device.h"
#include "fmpnp_internal.h"

namespace fmpnp {

// dynamic LDS of the LM kernel (the only kernel in this file that uses LDS)
extern __shared__ __attribute__((aligned(16))) unsigned char lm_lds[];

struct Ctx {
    // launch constants
    fmpnp_result *results;
    fmpnp_trace_entry *trace;
    unsigned *counter;
    double *part_g;       // [2][nc_max][NV] of this team
    double *max_g;        // [2][G] of this team
    double lambda0, ratio_thr, alpha;
    int mode, n_iters, use_ratio, loss, G, s, trace_stride, nc_max, no_memo;
    unsigned epoch;       // exchanges done by this team in this launch
    int dead;             // a team exchange timed out: finish remaining problems as failed
    int stamps_on;        // debug phase stamps enabled
    // problem constants
    const void *feat;
    const void *fref;
    const double *pts;
    double K[9];
    int p, N, Hf, Wf, cs, cb, ce, ld_ref, im_w, im_h, vec;
    int p0, M, c0, LC, NC;
};

struct LMState {
    double R[9], t[3];      // current (last accepted) pose
    double Re[9], te[3];    // pose evaluated next
    double Rb[9], tb[3];    // best pose
    double Hc[21], gc[6];   // cached linearisation at (R, t)
    double tot[NV];         // reduced totals of the last evaluation
    double lambda, lr, prev, best, initial, rho_max;
    int best_inl, n_evals, n_steps, n_accepted, status, done, has_best, ret_current;
    int abort_flag, sync_ok;
    int ndirty;             // points whose texel changed this evaluation (gather list length)
    long long gathers;      // texel gathers done for the current problem
    double wg_max[NT / 64];
    double tree[NT / NV][NV];  // ordered-sum tree level
    unsigned long long stamp_t, stamp_ph[NSTAMP];  // debug phase stamps (lane 0)
    Ctx c;
};
static_assert(sizeof(LMState) <= lds_fixed_bytes(), "LDS head too small");

__device__ __forceinline__ LMState &S() { return *reinterpret_cast<LMState *>(lm_lds); }
// debug: add the cycles since the previous stamp to phase k (lane 0 of the workgroup only)
__device__ __forceinline__ void dbg_stamp(int k) {
    LMState &st = *reinterpret_cast<LMState *>(lm_lds);
    if (st.c.stamps_on && threadIdx.x == 0) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        st.stamp_ph[k] += now - st.stamp_t;
        st.stamp_t = now;
    }
}
__device__ __forceinline__ unsigned char *dyn() { return lm_lds + lds_fixed_bytes(); }
// dynamic carve (mmax = max local points, a multiple of CH):
//   X[mmax][3], P[mmax][3], rec[mmax][RECW] doubles, tex[mmax] + list[mmax] ints, part[nc_max][NV] doubles
__device__ __forceinline__ double *lds_X(int mmax) { return reinterpret_cast<double *>(dyn()); }
__device__ __forceinline__ double *lds_P(int mmax) { return reinterpret_cast<double *>(dyn()) + 3 * mmax; }
__device__ __forceinline__ double *lds_rec(int mmax) { return reinterpret_cast<double *>(dyn()) + 6 * mmax; }
__device__ __forceinline__ int *lds_tex(int mmax) {
    return reinterpret_cast<int *>(reinterpret_cast<double *>(dyn()) + (6 + RECW) * mmax);
}
__device__ __forceinline__ int *lds_list(int mmax) { return lds_tex(mmax) + mmax; }
__device__ __forceinline__ double *lds_part(int mmax) {
    return reinterpret_cast<double *>(dyn()) + (6 + RECW) * mmax + mmax + 2;
}

// so3exp_map (helpers/utils.py:209-221) and the update R' = dR R, t' = dR t + dt
// (model.py:416-426).
__device__ __forceinline__ void pose_update(const double *R, const double *t, const double delta[6], double *Rn,
                                            double *tn) {
    const double w0 = delta[3], w1 = delta[4], w2 = delta[5];
    const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
    double dR[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (isnan(theta)) {
#pragma unroll
        for (int i = 0; i < 9; ++i) dR[i] = NAN;
    } else if (!(theta < 1e-12)) {
        const double k0 = w0 / theta, k1 = w1 / theta, k2 = w2 / theta;
        const double W[9] = {0, -k2, k1, k2, 0, -k0, -k1, k0, 0};
        double s, c;
        sincos(theta, &s, &c);
        const double c1 = 1.0 - c;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                double ww = W[3 * i + 0] * W[0 + j] + W[3 * i + 1] * W[3 + j] + W[3 * i + 2] * W[6 + j];
                dR[3 * i + j] += W[3 * i + j] * s + ww * c1;
            }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
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

// Every thread calls this after its sc1 stores; on return S().c.epoch is the epoch
// just completed.  Returns false on timeout.
__device__ __forceinline__ bool team_sync() {
    LMState &st = S();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned ep = ++st.c.epoch;
        const unsigned target = ep * (unsigned)st.c.G;
        unsigned *counter = st.c.counter;
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
        st.sync_ok = ok;
        if (!ok) st.abort_flag = 1;
    }
    __syncthreads();
    return st.sync_ok != 0;
}

// ---------------------------------------------------------------------------
// problem begin / end
// ---------------------------------------------------------------------------
__device__ __forceinline__ void problem_begin(const fmpnp_problem *pb, int p, int mmax) {
    LMState &st = S();
    const int tid = threadIdx.x;
    if (tid == 0) {
        Ctx &c = st.c;
        c.p = p;
        c.feat = pb->feat;
        c.fref = pb->fref;
        c.pts = pb->pts3d;
        c.N = pb->N;
        c.Hf = pb->Hf;
        c.Wf = pb->Wf;
        c.cs = pb->cstride;
        c.cb = pb->c_begin;
        c.ce = pb->c_end;
        c.ld_ref = pb->ld_ref;
        c.im_w = pb->im_width;
        c.im_h = pb->im_height;
        for (int k = 0; k < 9; ++k) c.K[k] = pb->K[k];
        c.NC = (c.N + CH - 1) / CH;
        c.c0 = (int)(((long)c.NC * c.s) / c.G);
        const int c1 = (int)(((long)c.NC * (c.s + 1)) / c.G);
        c.LC = c1 - c.c0;
        c.p0 = c.c0 * CH;
        c.M = max(min(c1 * CH, c.N) - c.p0, 0);
        c.vec = 0;
        for (int k = 0; k < 9; ++k) { st.R[k] = st.Re[k] = st.Rb[k] = pb->R0[k]; }
        for (int k = 0; k < 3; ++k) { st.t[k] = st.te[k] = st.tb[k] = pb->t0[k]; }
        st.lambda = c.lambda0;
        st.lr = 1.0;
        st.prev = st.best = st.initial = NAN;
        st.best_inl = -1;
        st.n_evals = st.n_steps = st.n_accepted = 0;
        st.status = c.dead ? FMPNP_STATUS_SYNC_TIMEOUT : 0;
        st.has_best = 0;
        st.ret_current = 0;
        st.done = c.dead || (c.mode != FMPNP_MODE_COMPUTE_COST && c.n_iters <= 0);
        st.abort_flag = 0;
        st.ndirty = 0;
        st.gathers = 0;
    }
    __syncthreads();
    // this workgroup's points -> LDS once per problem
    const Ctx &c = st.c;
    double *X = lds_X(mmax);
    const double *src = c.pts + 3 * (size_t)c.p0;
    for (int e = tid; e < 3 * c.M; e += NT) X[e] = src[e];
    int *tex = lds_tex(mmax);
    for (int i = tid; i < mmax; i += NT) tex[i] = -2;  // no texel cached yet
    __syncthreads();
}

__device__ __forceinline__ void problem_end() {
    LMState &st = S();
    if (threadIdx.x == 0) {
        if (st.abort_flag) {
            st.c.dead = 1;
            st.status |= FMPNP_STATUS_SYNC_TIMEOUT;
        }
        if (st.c.s == 0) {
            fmpnp_result &r = st.c.results[st.c.p];
            const bool cur = st.ret_current || st.c.mode == FMPNP_MODE_COMPUTE_COST;
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
        // every team member adds its share (results are zeroed by the launcher)
        atomicAdd(reinterpret_cast<unsigned long long *>(&st.c.results[st.c.p].texel_gathers),
                  (unsigned long long)st.gathers);
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// A0: projection (thread per local point) -> texel offset + camera-frame point
// ---------------------------------------------------------------------------
__device__ __forceinline__ void phase_project(int mmax) {
    LMState &st = S();
    const Ctx &c = st.c;
    const double *X = lds_X(mmax);
    double *P = lds_P(mmax);
    int *tex = lds_tex(mmax);
    for (int i = threadIdx.x; i < c.M; i += NT) {
        double Pc[3];
        transform_pt(st.Re, st.te, X[3 * i], X[3 * i + 1], X[3 * i + 2], Pc);
        int x, y;
        int off = -1;
        if (project_px(c.K, Pc, c.im_w, c.im_h, x, y)) {
            // indexing_ (model.py:88-89): floor(y*Hf/H), floor(x*Wf/W), exact in integers
            // y*Hf and x*Wf are exact in fp64, and a correctly rounded quotient of two
            // integers floors to the integer quotient: exact, without a software int division
            const int row = (int)floor(((double)y * (double)c.Hf) / (double)c.im_h);
            const int col = (int)floor(((double)x * (double)c.Wf) / (double)c.im_w);
            off = row * c.Wf + col;
        }
        // memoised gather: a point whose texel did not change keeps its record (the six
        // channel sums depend only on the texel and the point's fixed descriptor)
        if (off >= 0 && (off != tex[i] || c.no_memo)) lds_list(mmax)[atomicAdd(&st.ndirty, 1)] = i;
        tex[i] = off;
        P[3 * i] = Pc[0];
        P[3 * i + 1] = Pc[1];
        P[3 * i + 2] = Pc[2];
    }
}

// ---------------------------------------------------------------------------
// A: channel sums, one half-wave (32 lanes) per point, two points per wave.  Lane l of
// a half owns channels cb + l*V + r*32*V + k (k < V, V = 16 B / sizeof(T)) and
// accumulates them in (r, k) order in BOTH forms, so the vector form (16-byte loads)
// and the scalar form (unaligned / ragged channel ranges) give bit-identical sums.  At
// C = 256 fp32 a point is two rounds whose 8 loads per lane are all issued before the
// first use: f, gx, gy and fref of a point arrive in ONE memory round trip.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void acc6(double a[8], double f, double r, double gx, double gy) {
    double e = f - r;
    a[0] = fma(e, e, a[0]);
    a[1] = fma(gx, e, a[1]);
    a[2] = fma(gy, e, a[2]);
    a[3] = fma(gx, gx, a[3]);
    a[4] = fma(gx, gy, a[4]);
    a[5] = fma(gy, gy, a[5]);
}

template <typename VT>
__device__ __forceinline__ VT gload(const void *p) {  // global (not flat) 16-byte load
#if defined(__HIP_DEVICE_COMPILE__)
    return *reinterpret_cast<const __attribute__((address_space(1))) VT *>(reinterpret_cast<uintptr_t>(p));
#else
    return *reinterpret_cast<const VT *>(p);  // host pass: never executed
#endif
}

template <typename T, bool VEC>
__device__ __forceinline__ void gather_half(const T *__restrict__ t, const T *__restrict__ rf, int cs, int cb,
                                            int ce, int l32, double a[8]) {
    using VT = typename V16<T>::type;
    constexpr int V = V16<T>::n;
    if constexpr (VEC) {
        // two rounds per trip, all eight loads issued before the first use (one round trip
        // for C <= 64 V); a missing second round reads round one again and adds exact zeros
        for (int c = cb + l32 * V; c < ce; c += 64 * V) {
            const bool has2 = c + 32 * V < ce;
            const int c2 = has2 ? c + 32 * V : c;
            const VT f0 = gload<VT>(t + c), x0 = gload<VT>(t + cs + c), y0 = gload<VT>(t + 2 * cs + c);
            const VT q0 = gload<VT>(rf + c);
            const VT f1 = gload<VT>(t + c2), x1 = gload<VT>(t + cs + c2), y1 = gload<VT>(t + 2 * cs + c2);
            const VT q1 = gload<VT>(rf + c2);
            const T *pf = reinterpret_cast<const T *>(&f0), *px = reinterpret_cast<const T *>(&x0);
            const T *py = reinterpret_cast<const T *>(&y0), *pr = reinterpret_cast<const T *>(&q0);
#pragma unroll
            for (int k = 0; k < V; ++k) acc6(a, (double)pf[k], (double)pr[k], (double)px[k], (double)py[k]);
            const T *sf = reinterpret_cast<const T *>(&f1), *sx = reinterpret_cast<const T *>(&x1);
            const T *sy = reinterpret_cast<const T *>(&y1), *sr = reinterpret_cast<const T *>(&q1);
#pragma unroll
            for (int k = 0; k < V; ++k) {
                const double z = 0.0;
                acc6(a, has2 ? (double)sf[k] : z, has2 ? (double)sr[k] : z, has2 ? (double)sx[k] : z,
                     has2 ? (double)sy[k] : z);
            }
        }
    } else {
        for (int c = cb + l32 * V; c < ce; c += 32 * V) {
#pragma unroll
            for (int k = 0; k < V; ++k)
                if (c + k < ce)
                    acc6(a, (double)t[c + k], (double)rf[c + k], (double)t[cs + c + k], (double)t[2 * cs + c + k]);
        }
    }
}

// Transposed reduction of 8 values over the 32 lanes of a half-wave: halving exchanges
// at bit 4 (permlane16 swap), bit 3 (row mirror), bit 2 (half-row mirror), then
// butterflies at bits 1, 0 -- no LDS traffic.  Returns the half's total of value index
// 4*b4 + 2*b3 + b2 of the lane; only equal indices are ever added.
__device__ __forceinline__ double reduce8_in32(double v[8], int lane) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double a = v[i], b = v[i + 4];
        swap16(a, b);  // even rows keep index i, odd rows i + 4
        v[i] = a + b;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) v[i] = tstep<DPP_MIRROR16>(v[i], v[i + 2], lane & 8);
    v[0] = tstep<DPP_MIRROR8>(v[0], v[1], lane & 4);
    v[0] = v[0] + dpp64<DPP_XOR2>(v[0]);
    return v[0] + dpp64<DPP_XOR1>(v[0]);
}

template <typename T>
__device__ __forceinline__ void phase_gather(int mmax) {
    LMState &st = S();
    const Ctx &c = st.c;
    const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, half = tid >> 5;
    constexpr int NH = NT / 32;
    const int *tex = lds_tex(mmax);
    double *rec = lds_rec(mmax);
    const T *feat = reinterpret_cast<const T *>(c.feat);
    const T *fref = reinterpret_cast<const T *>(c.fref);
    const int cs = c.cs, cb = c.cb, ce = c.ce, p0 = c.p0, ld = c.ld_ref;
    constexpr int V = V16<T>::n;
    const bool vec = ((((uintptr_t)feat) | ((uintptr_t)fref)) & 15) == 0 && cs % V == 0 && ld % V == 0 &&
                     cb % V == 0 && (ce - cb) % V == 0;
    const int *list = lds_list(mmax);
    const int nd = st.ndirty;
    // every lane of a wave runs the same trip count (the shuffles need the whole wave)
    for (int k0 = (tid >> 6) * 2; k0 < nd; k0 += NH) {
        const int k = k0 + (half & 1);
        const bool live = k < nd;
        const int i = live ? list[k] : list[k0];
        const T *t = feat + (size_t)tex[i] * 3 * cs;
        const T *rf = fref + (size_t)(p0 + i) * ld;
        double v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = 0.0;
        if (vec) gather_half<T, true>(t, rf, cs, cb, ce, l32, v);
        else gather_half<T, false>(t, rf, cs, cb, ce, l32, v);
        const double r = reduce8_in32(v, lane);
        const int e = 4 * ((lane >> 4) & 1) + 2 * ((lane >> 3) & 1) + ((lane >> 2) & 1);
        if (live && (lane & 3) == 0 && e < 6) rec[(size_t)i * RECW + e] = r;
    }
}

// Transposed reduction of 8 values over the 16 lanes of a row (DPP only): halving at
// bits 3, 2, 1 then a butterfly at bit 0.  Returns the row total of value index
// 4*b3 + 2*b2 + b1 of l16.
__device__ __forceinline__ double reduce8_in16(double v[8], int l16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = tstep<DPP_MIRROR16>(v[i], v[i + 4], l16 & 8);
#pragma unroll
    for (int i = 0; i < 2; ++i) v[i] = tstep<DPP_MIRROR8>(v[i], v[i + 2], l16 & 4);
    v[0] = tstep<DPP_XOR2>(v[0], v[1], l16 & 2);
    return v[0] + dpp64<DPP_XOR1>(v[0]);
}

// ---------------------------------------------------------------------------
// B1: rho, rho' per point; team max |rho| for the ratio test.  Returns false on abort.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool phase_loss(int mmax) {
    LMState &st = S();
    const Ctx &c = st.c;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int *tex = lds_tex(mmax);
    double *rec = lds_rec(mmax);
    const int loss = c.mode == FMPNP_MODE_COMPUTE_COST ? (int)FMPNP_SQUARED : c.loss;
    double lmax = -1.0;  // -1: nothing supported seen yet
    if (tid == 0) {
        st.gathers += st.ndirty;
        st.ndirty = 0;  // next write: the next projection, several barriers later
    }
    for (int i = tid; i < c.M; i += NT) {
        double rho = 0.0, d1 = 0.0;
        if (tex[i] >= 0) {
            loss_eval(loss, c.alpha, 0.5 * rec[(size_t)i * RECW + 0], rho, d1);
            const double am = fabs(rho);
            if (isnan(am) || am > lmax) lmax = isnan(lmax) ? lmax : am;
        }
        rec[(size_t)i * RECW + 6] = rho;
        rec[(size_t)i * RECW + 7] = d1;
    }
    if (!c.use_ratio) return true;
    // wave max then workgroup max (max is order-independent: exact)
    lmax = wave_nanmax(lmax);
    if (lane == 0) st.wg_max[wave] = lmax;
    __syncthreads();
    if (tid == 0) {
        double m = st.wg_max[0];
        for (int w = 1; w < NT / 64; ++w)
            if (isnan(st.wg_max[w]) || st.wg_max[w] > m) m = isnan(m) ? m : st.wg_max[w];
        st.rho_max = m;
        if (c.G > 1) st_sc1(c.max_g + ((c.epoch + 1) & 1) * c.G + c.s, m);
    }
    __syncthreads();
    if (c.G > 1) {
        if (!team_sync()) return false;
        if (tid == 0) {
            double m = -1.0;
            for (int w = 0; w < c.G; ++w) {
                const double o = ld_sc1(c.max_g + (c.epoch & 1) * c.G + w);
                if (isnan(o) || o > m) m = isnan(m) ? m : o;
            }
            st.rho_max = m;
        }
        __syncthreads();
    }
    return true;
}

// ---------------------------------------------------------------------------
// B2: per-point normal-equation contributions -> one 32-double partial per chunk
// (LDS when G == 1, the team's global slot with sc1 stores when G > 1).
// ---------------------------------------------------------------------------
// value index -> (row, col) of the upper triangle of H (0..20), then g (21..26)
__device__ __forceinline__ constexpr int h_row(int k) {
    return k < 6 ? 0 : k < 11 ? 1 : k < 15 ? 2 : k < 18 ? 3 : k < 20 ? 4 : 5;
}
__device__ __forceinline__ constexpr int h_col(int k) {
    return k < 6 ? k : k < 11 ? k - 5 : k < 15 ? k - 9 : k < 18 ? k - 12 : k < 20 ? k - 14 : 5;
}

__device__ __forceinline__ void phase_contrib(int mmax) {
    LMState &st = S();
    const Ctx &c = st.c;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l16 = tid & 15;
    const int *tex = lds_tex(mmax);
    const double *rec = lds_rec(mmax);
    const double *Pl = lds_P(mmax);
    double *part_lds = lds_part(mmax);
    const double limit = st.rho_max * c.ratio_thr;
    const bool ratio = c.use_ratio != 0;
    const double fx = c.K[0], fy = c.K[4];
    const int LC = c.LC, M = c.M;
    double *part_g = c.part_g + (size_t)((c.epoch + 1) & 1) * c.nc_max * NV;
    for (int base = wave * 4; base < LC; base += 4 * (NT / 64)) {
        const int lc = base + (lane >> 4);
        const int i = lc * CH + l16;  // local point index
        const bool sup = lc < LC && i < M && tex[i] >= 0;
        const double *r = rec + (size_t)(sup ? i : 0) * RECW;
        const bool kept = sup && (!ratio || fabs(r[6]) < limit);
        // points that do not contribute get w = 0 and a harmless geometry (z = 1)
        const double w = kept ? r[7] : 0.0, rho = kept ? r[6] : 0.0;
        const double P0 = kept ? Pl[3 * i] : 0.0, P1 = kept ? Pl[3 * i + 1] : 0.0, z = kept ? Pl[3 * i + 2] : 1.0;
        const double sex = kept ? r[1] : 0.0, sey = kept ? r[2] : 0.0;
        const double sxx = kept ? r[3] : 0.0, sxy = kept ? r[4] : 0.0, syy = kept ? r[5] : 0.0;
        // J_px_p (model.py:377-382) times J_p_T (model.py:369-370): A (2x6), A0[1] = A1[0] = 0
        // one reciprocal instead of six divisions (Jacobian entries only: last-bit level)
        const double iz = 1.0 / z;
        const double j00 = fx * iz, j02 = ((-fx) * P0 * iz) * iz;
        const double j11 = fy * iz, j12 = ((-fy) * P1 * iz) * iz;
        const double A0[6] = {j00, 0.0, j02, j02 * P1, j00 * z - j02 * P0, -j00 * P1};
        const double A1[6] = {0.0, j11, j12, -j11 * z + j12 * P1, -j12 * P0, j11 * P0};
        double M0[6], M1[6];
#pragma unroll
        for (int l = 0; l < 6; ++l) {
            M0[l] = sxx * A0[l] + sxy * A1[l];
            M1[l] = sxy * A0[l] + syy * A1[l];
        }
        const int chunk = c.c0 + lc;
        double *dst = c.G == 1 ? part_lds + (size_t)chunk * NV : part_g + (size_t)chunk * NV;
        // the 32-value vector in four quarters of 8: only 8 doubles live per reduction
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            double v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int k = 8 * q + e;
                if (k < 21) {
                    const int a = h_row(k), b = h_col(k);
                    v[e] = w * (A0[a] * M0[b] + A1[a] * M1[b]);
                } else if (k < 27) {
                    v[e] = w * (A0[k - 21] * sex + A1[k - 21] * sey);
                } else if (k == 27) {
                    v[e] = rho;
                } else if (k == 28) {
                    v[e] = kept ? 1.0 : 0.0;
                } else if (k == 29) {
                    v[e] = sup ? 1.0 : 0.0;
                } else {
                    v[e] = 0.0;
                }
            }
            const double tot = reduce8_in16(v, l16);
            const int idx = 8 * q + 4 * ((l16 >> 3) & 1) + 2 * ((l16 >> 2) & 1) + ((l16 >> 1) & 1);
            if (lc < LC && (l16 & 1) == 0) {
                if (c.G == 1) dst[idx] = tot;
                else st_sc1(dst + idx, tot);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// ---------------------------------------------------------------------------
// Combine: (G > 1: exchange + stage every chunk partial in LDS), then the ordered sum
// over chunk indices: tree[q][j] = sum_{c = q, q+NQ, ...} part[c][j] in c order
// (NQ = NT/32 = 32 rows), then a fixed pairwise tree over the NQ rows.  Depends only on
// the chunk partials and NC -- not on G, placement or timing.
// ---------------------------------------------------------------------------
constexpr int NQ = NT / NV;

__device__ __forceinline__ bool phase_combine(int mmax) {
    LMState &st = S();
    const Ctx &c = st.c;
    const int tid = threadIdx.x;
    double *part_lds = lds_part(mmax);
    const int NC = c.NC;
    if (c.G > 1) {
        if (!team_sync()) return false;
        const double *src = c.part_g + (size_t)(c.epoch & 1) * c.nc_max * NV;
        for (int e = tid; e < NC * NV; e += NT) part_lds[e] = ld_sc1(src + e);
    }
    __syncthreads();
    {
        const int j = tid & (NV - 1), q = tid / NV;
        double acc = 0.0;
        for (int ch = q; ch < NC; ch += NQ) acc += part_lds[ch * NV + j];
        st.tree[q][j] = acc;
    }
    __syncthreads();
    return true;
}

// Final level of the ordered sum on wave 0 (no barrier: the LM update that reads the
// totals runs on the same wave): lane l sums rows 16*(l>>5) .. +15 of value l&31 with a
// fixed pairwise tree, the two halves are added across the wave -- the same tree as a
// single pairwise tree over the NQ = 32 rows.
static_assert(NQ == 32, "final tree assumes 32 rows");
__device__ __forceinline__ void combine_final_wave() {
    LMState &st = S();
    const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
    double t[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) t[q] = st.tree[16 * h + q][j];
#pragma unroll
    for (int w = 1; w < 16; w *= 2)
#pragma unroll
        for (int q = 0; q < 16; q += 2 * w) t[q] = t[q] + t[q + w];
    double a = t[0], b = t[0];
    swap32(a, b);  // low half: (own, partner); high half: (partner, own)
    const double tot = a + b;  // rows 0..15 + rows 16..31 in both halves
    if (lane < NV) st.tot[lane] = tot;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// ---------------------------------------------------------------------------
// 6x6 damped solve on one wave: lanes 0..5 own the rows of H + lambda diag(diag(H)+1e-9)
// (model.py:46-48) and run LU with partial pivoting (model.py:51,61) row-parallel.
// Pivot choice = the serial scan's (first position with the largest |A[.][j]|), the
// elimination and the forward substitution are the serial arithmetic; the back
// substitution runs column-wise with the pivots' reciprocals.  Uniform values move
// between lanes with v_readlane only.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double rlane(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__host__ __device__ constexpr int tri6(int i, int j) { return i * 6 - (i * (i - 1)) / 2 + (j - i); }

__device__ __forceinline__ void lm_step_rows(const double *Hu, const double *g, double lambda, double lr,
                                             double delta[6]) {
    const int lane = threadIdx.x & 63;
    const int r = lane < 6 ? lane : 5;
    double A[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) A[c] = Hu[r <= c ? tri6(r, c) : tri6(c, r)];
    double b = g[r];
    if (lambda != 0.0) {
#pragma unroll
        for (int c = 0; c < 6; ++c)
            if (c == r) A[c] = A[c] + (A[c] + 1e-9) * lambda;
    }
    int pos = lane < 6 ? lane : 64;  // current position of this lane's row (64: no row)
    int lane_at[6] = {0, 1, 2, 3, 4, 5};
    double inv[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const double rj = 1.0 / A[j];  // every row's candidate pivot reciprocal, off the critical path
        int p = j;
        double best = fabs(rlane(A[j], lane_at[j]));
#pragma unroll
        for (int i = j + 1; i < 6; ++i) {
            const double v = fabs(rlane(A[j], lane_at[i]));
            if (v > best) { best = v; p = i; }
        }
        const int lj = lane_at[j];
        int lp = lj;
#pragma unroll
        for (int k = j + 1; k < 6; ++k) lp = (p == k) ? lane_at[k] : lp;
#pragma unroll
        for (int k = j + 1; k < 6; ++k) lane_at[k] = (p == k) ? lj : lane_at[k];
        lane_at[j] = lp;
        if (lane == lp) pos = j;
        else if (lane == lj) pos = p;
        double prow[6];
#pragma unroll
        for (int c = j + 1; c < 6; ++c) prow[c] = rlane(A[c], lp);
        const double pb = rlane(b, lp);
        const double iv = rlane(rj, lp);  // = 1 / A[p][j], computed before the pivot was known
        inv[j] = iv;
        if (pos > j && pos < 6) {
            const double m = A[j] * iv;
            A[j] = m;
#pragma unroll
            for (int c = j + 1; c < 6; ++c) A[c] -= m * prow[c];
            b -= m * pb;
        }
    }
    double x[6];
#pragma unroll
    for (int i = 5; i >= 0; --i) {
        const double xi = rlane(b, lane_at[i]) * inv[i];
        x[i] = xi;
        if (pos < i) b -= A[i] * xi;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) delta[i] = -lr * x[i];
}

// ---------------------------------------------------------------------------
// Fast path of the damped solve: H + lambda diag(diag(H) + 1e-9) is symmetric positive
// definite whenever lambda > 0 (H = sum rho' J^T J with rho' > 0 for every loss), so an
// LDL^T factorisation needs no pivoting and no cross-lane traffic: every lane of wave 0
// runs the same ~160 register-resident fp64 instructions.  The reference's LU solve
// (model.py:51,61) and this one agree to rounding (cond(H) * eps, far inside the pose
// tolerance; tests/test_gpu_parity.py).  Returns false -- and the caller falls back to
// the pivoted LU -- when a pivot is not positive (lambda = 0 on a singular H, NaN).
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool ldlt_step(const double *Hu, const double *g, double lambda, double lr,
                                          double delta[6]) {
    double a[6][6];  // lower triangle used: a[i][j], i >= j
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) a[i][j] = Hu[tri6(j, i)];
    if (lambda != 0.0) {
#pragma unroll
        for (int j = 0; j < 6; ++j) a[j][j] = a[j][j] + (a[j][j] + 1e-9) * lambda;
    }
    double b[6], inv[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) b[i] = g[i];
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        ok &= a[j][j] > 0.0;  // false for NaN
        inv[j] = 1.0 / a[j][j];
        double u[6];
#pragma unroll
        for (int i = j + 1; i < 6; ++i) u[i] = a[i][j];
#pragma unroll
        for (int i = j + 1; i < 6; ++i) {
            const double l = u[i] * inv[j];
#pragma unroll
            for (int c = j + 1; c <= i; ++c) a[i][c] = fma(-l, u[c], a[i][c]);
            b[i] = fma(-l, b[j], b[i]);  // forward substitution L y = g, folded in
            a[i][j] = l;
        }
    }
    double x[6];
#pragma unroll
    for (int j = 5; j >= 0; --j) {
        double v = b[j] * inv[j];
#pragma unroll
        for (int i = j + 1; i < 6; ++i) v = fma(-a[i][j], x[i], v);
        x[j] = v;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) delta[i] = -lr * x[i];
    return ok;
}

// ---------------------------------------------------------------------------
// LM state machine (model.py:300-486) on wave 0: every lane computes the same uniform
// state (lane 0 alone writes it back) and the wave solves the 6x6 system together.
// Every team member computes the same from identical totals.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void lm_update_wave() {
    LMState &st = S();
    const Ctx &c = st.c;
    const int lane = threadIdx.x & 63;
    const bool w0 = lane == 0;
    const int nsup = (int)st.tot[29];
    const int kept = (int)st.tot[28];
    const double cost = st.tot[27] / st.tot[28];  // torch mean of an empty tensor = NaN
    if (c.mode == FMPNP_MODE_COMPUTE_COST) {
        if (w0) {
            st.initial = nsup == 0 ? NAN : cost;
            if (nsup == 0) st.status |= FMPNP_STATUS_NO_SUPPORT;
            st.n_evals = 1;
            st.done = 1;
        }
        return;
    }
    const int n_evals = st.n_evals, n_steps = st.n_steps;
    const bool first = n_evals == 0;
    if (nsup == 0) {  // model.py:316-320 / :441-445: return the current pose
        if (w0) {
            st.status |= first ? FMPNP_STATUS_NO_SUPPORT : FMPNP_STATUS_NO_SUPPORT_TRIAL;
            st.ret_current = 1;
            st.done = 1;
        }
        return;
    }
    double lambda = st.lambda, lr = st.lr;
    bool accepted = true;
    if (!first) {  // model.py:469-478
        const double prev = st.prev;
        accepted = !(cost > prev);
        const double lam = lambda * (cost > prev ? 10.0 : 0.1);
        lambda = lam < 1e-6 ? 1e-6 : (lam > 1e4 ? 1e4 : lam);
        if (!accepted) {
            const double l2 = 0.1 * lr;
            lr = l2 < 1e-3 ? 1e-3 : (l2 > 1.0 ? 1.0 : l2);
        } else {
            lr = 1.0;
        }
    }
    // the evaluated pose becomes current and its normal equations the linearisation
    const bool take = first || accepted;
    const bool new_best = !first && accepted && cost < st.best;
    // pose / linearisation copies: one element per lane
    if (new_best && lane < 12) {
        if (lane < 9) st.Rb[lane] = st.Re[lane];
        else st.tb[lane - 9] = st.te[lane - 9];
    }
    if (take && lane < 12) {
        if (lane < 9) st.R[lane] = st.Re[lane];
        else st.t[lane - 9] = st.te[lane - 9];
    }
    if (take && lane < 27) {
        if (lane < 21) st.Hc[lane] = st.tot[lane];
        else st.gc[lane - 21] = st.tot[lane];
    }
    if (w0) {
        if (first) {  // model.py:347-359
            st.prev = st.best = st.initial = cost;
            st.best_inl = kept;
            st.has_best = 1;
        } else if (accepted) {  // model.py:477-486
            st.n_accepted++;
            if (new_best) {
                st.best_inl = kept;
                st.best = cost;
            }
            st.prev = cost;
        }
        st.lambda = lambda;
        st.lr = lr;
        if (c.trace && c.s == 0 && n_evals < c.trace_stride) {
            fmpnp_trace_entry &e = c.trace[(size_t)c.p * c.trace_stride + n_evals];
            for (int k = 0; k < 9; ++k) e.R[k] = st.Re[k];
            for (int k = 0; k < 3; ++k) e.t[k] = st.te[k];
            e.cost = cost;
            e.lambda_after = lambda;
            e.lr_after = lr;
            e.n_supported = nsup;
            e.n_kept = kept;
            e.accepted = accepted ? 1 : 0;
        }
        st.n_evals = n_evals + 1;
    }
    if (n_steps >= c.n_iters) {
        if (w0) st.done = 1;
        return;
    }
    // next step from the linearisation at the current pose (model.py:408-426)
    double delta[6];
    dbg_stamp(5);  // LM bookkeeping
    {
        const double *Hu = take ? st.tot : st.Hc, *gv = take ? st.tot + 21 : st.gc;
        if (!ldlt_step(Hu, gv, lambda, lr, delta)) lm_step_rows(Hu, gv, lambda, lr, delta);
    }
    dbg_stamp(6);  // 6x6 solve
    bool bad = false;
#pragma unroll
    for (int k = 0; k < 6; ++k) bad |= isnan(delta[k]);
    if (bad) {  // model.py:411-413
        if (w0) {
            st.n_steps = n_steps + 1;
            st.status |= FMPNP_STATUS_NAN;
            st.done = 1;
        }
        return;
    }
    const double *R = take ? st.Re : st.R;
    const double *t = take ? st.te : st.t;
    double Rc[9], tc[3], Rn[9], tn[3];
#pragma unroll
    for (int k = 0; k < 9; ++k) Rc[k] = R[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) tc[k] = t[k];
    pose_update(Rc, tc, delta, Rn, tn);
    if (w0) {
        st.n_steps = n_steps + 1;
        for (int k = 0; k < 9; ++k) st.Re[k] = Rn[k];
        for (int k = 0; k < 3; ++k) st.te[k] = tn[k];
    }
}

// ---------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(NT, FMPNP_LM_WAVES_PER_SIMD) void lm_kernel(LaunchArgs a) {
    LMState &st = S();
    const int G = a.G;
    // XCD-aware team placement: members of one team share blockIdx % gw (the same XCD
    // under the observed round-robin dispatch; speed only, never correctness).
    const int b = blockIdx.x, gw = a.gw;
    const int grp = b / (gw * G), rem = b % (gw * G);
    const int s = rem / gw;
    const int team = grp * gw + rem % gw;
    if (team >= a.teams) return;
    const int tid = threadIdx.x;
    const int mmax = a.mmax;
    if (tid == 0) {
        Ctx &c = st.c;
        c.results = a.results;
        c.trace = a.trace;
        c.trace_stride = a.trace_stride;
        c.counter = a.counters + team * 16;
        c.part_g = a.partials + (size_t)team * 2 * a.nc_max * NV;
        c.max_g = a.maxslots + (size_t)team * 2 * G;
        c.nc_max = a.nc_max;
        c.lambda0 = a.opt.lambda0;
        c.ratio_thr = a.opt.ratio_threshold;
        c.alpha = a.opt.barron_alpha;
        c.mode = a.opt.mode;
        c.n_iters = a.opt.n_iters;
        c.use_ratio = a.opt.use_ratio;
        c.loss = a.opt.loss;
        c.no_memo = a.opt.no_memo;
        c.stamps_on = a.stamps != nullptr;
        c.G = G;
        c.s = s;
        c.epoch = 0;
        c.dead = 0;
    }
    __syncthreads();
    // optional phase stamps (debug: a.stamps != null): s_memtime deltas on lane 0 after barriers
    const bool stamps_on = a.stamps != nullptr;
    if (stamps_on && tid == 0) {
        for (int k = 0; k < NSTAMP; ++k) st.stamp_ph[k] = 0;
        st.stamp_t = __builtin_amdgcn_s_memtime();
    }
#define STAMP(k)                                                \
    if (stamps_on && tid == 0) {                                \
        unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
        st.stamp_ph[(k) < 4 && st.n_evals == 0 ? 8 + (k) : (k)] += now_ - st.stamp_t; \
        st.stamp_t = now_;                                      \
    }

    for (int p = team; p < a.n; p += a.teams) {
        problem_begin(a.probs + p, p, mmax);
        while (!st.done) {
            phase_project(mmax);
            __syncthreads();
            STAMP(0);
            phase_gather<T>(mmax);
            __syncthreads();
            STAMP(1);
            if (!phase_loss(mmax)) break;
            STAMP(2);
            phase_contrib(mmax);
            STAMP(3);
            if (!phase_combine(mmax)) break;
            if (tid < 64) {
                combine_final_wave();
                STAMP(4);
                lm_update_wave();
            }
            __syncthreads();
            STAMP(7);  // pose update + barrier
        }
        problem_end();
    }
    if (stamps_on && tid == 0)
        for (int k = 0; k < NSTAMP; ++k) a.stamps[(size_t)blockIdx.x * NSTAMP + k] = st.stamp_ph[k];
#undef STAMP
}

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

size_t lm_dyn_lds_bytes(int mmax, int nc_max) {
    // X[3M] + P[3M] + rec[RECW M] doubles, tex[M] + list[M] ints (+16 B pad), part[nc_max][NV] doubles
    return (size_t)(6 + RECW) * mmax * 8 + ((size_t)mmax + 2) * 8 + (size_t)nc_max * NV * 8;
}

}  // namespace fmpnp
