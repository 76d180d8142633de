// fmpnp_lm_impl.h -- the LM kernel template (included by the per-storage-type
// instantiation units fmpnp_lm_f32.hip / fmpnp_lm_f64.hip).
#pragma once
// The feature-metric LM refiner on gfx950 (MI355X): one launch runs the WHOLE
// Levenberg-Marquardt loop of every problem of a batch (sparseFeaturePnP.forward,
// featurePnP/model.py:245-494) on the device.
//
// Work decomposition
//   * A "team" of G workgroups (512 threads = 8 waves each) owns one problem at a time;
//     teams walk the batch persistently (problem = team, team + T, ...).
//   * Points are cut into chunks of CH = 64, one wave block each; workgroup s of a team owns a
//     contiguous range of chunks, and wave w of the workgroup owns the blocks w, w+8, ... of that
//     range.  Per evaluation a wave carries each of its blocks from projection to its chunk
//     partial with NO workgroup barrier:
//       project  (lane per point, fp64, exact pixel rounding) -> texel offset, P;
//       gather   the points whose texel changed (ballot), two per wave: each half-wave
//                issues 16-byte loads of the channels-last [H][W][3][C] texel and fref
//                and reduces the six channel sums  sum e^2, sum gx e, sum gy e, sum gx^2,
//                sum gx gy, sum gy^2  in fp64 (the C x 6 Jacobian is never materialised:
//                J = G A with the 2x6 pose chain A, so J^T e = A^T (G^T e),
//                J^T J = A^T (G^T G) A); unchanged texels keep their sums (memoisation);
//       loss + normal equations (lane per point) -> 21 + 6 entries, rho and counters,
//                reduced per 64-point chunk by a fixed transposed permlane/DPP tree.
//   * The chunk partials are summed by wave 0 with a fixed tree over CHUNK INDICES.  Results
//     are therefore deterministic and independent of G: the LM accept test `new > prev`
//     (model.py:469-472) compares costs that tie exactly whenever the pixel sets are
//     equal, and a scheduling-dependent sum would break those ties.
//   * G > 1: chunk partials go to a per-team slot with write-through (sc1) stores,
//     every storing wave drains, one lane bumps the team's arrival counter, one lane
//     polls it (bounded spin), one agent-scope acquire; then wave 0 of every member
//     reads all partials and runs the identical 6x6 solve + LM update (no second exchange).
//   * One evaluation per iteration: the trial evaluation at (R', t') also produces that
//     pose's normal equations.  On acceptance they are the next linearisation; on
//     rejection the cached ones are reused -- bit-identical to the reference's
//     recomputation at the unchanged pose (model.py:472-476).
//   * The ratio test (model.py:324-336) needs max|rho| over the problem before any point's
//     weight is known.  One workgroup per problem of at most 8 blocks: the partials are formed
//     with the previous evaluation's limit and a block whose kept set the true limit changes is
//     re-formed (ratio_guess_check); otherwise loss values are parked in LDS, the maximum is
//     exchanged, and a second pass over the blocks forms the normal equations (contrib_pass).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#include "fmpnp.h"
#include "fmpnp_device.h"
#include "fmpnp_internal.h"

namespace fmpnp {

constexpr bool kSpecBuild = FMPNP_SPEC != 0;
// Debug instrumentation (fmpnp_debug_stamps: phase totals, per-evaluation stamps, the evaluation
// timeline) is compiled in only with -DFMPNP_STAMPS=1 (a diagnostics build, tools/build_ab.sh):
// its flags and pointers would otherwise hold scalar registers across the evaluation loop.
// (FMPNP_STAMPS itself is defined in fmpnp_internal.h: it also sizes the LDS head)
constexpr bool kStamps = FMPNP_STAMPS != 0;
#ifndef FMPNP_VCONST
#define FMPNP_VCONST 1
#endif
#ifndef FMPNP_LANE_NOW
#define FMPNP_LANE_NOW 1
#endif
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
    int mode, n_iters, use_ratio, loss, G, s, trace_stride, nc_max, no_memo, sampling, sobel_flags;
    int spec;             // speculative gathers of the predicted next texels (memoised nearest modes)
    int spec_cap;         // ... at most this many per wave per evaluation
    int spec_w0;          // ... by the waves >= spec_w0
    int dbg;
    unsigned epoch;       // exchanges done by this team in this launch
    int dead;             // a team exchange timed out: finish remaining problems as failed
    int stamps_on;        // debug phase stamps enabled
    // problem constants
    const void *feat;
    const void *fref;
    const double *pts;
    const unsigned char *win_ok;  // packed window: texels whose 3x3 neighbourhood is packed (NULL: all)
    double K[9];
    int p, N, Hf, Wf, cs, cb, ce, ld_ref, im_w, im_h, vec;
    float txpx, typx, pxtx, pypx;  // texels per image pixel, image pixels per texel (x, y)
    UDiv div_h, div_w;    // exact floor division by im_h, im_w (indexing_)
    int p0, M, c0, LC, NC;
};

// Per-problem constants of the point phases, held in registers (every value wave-uniform:
// the compiler keeps them in SGPRs) instead of being re-read from the LDS Ctx at every use
// -- each LDS read is a ~100-cycle round trip on the evaluation's critical path.
struct PC {
    const void *feat, *fref;
    // K: a pinhole matrix [[fx, 0, cx], [0, fy, cy], [0, 0, 1]] (kstd; the reference's intrinsics)
    // keeps only its four parameters in scalar registers; any other K is read from the LDS Ctx
    double fx, cx, fy, cy;
    int kstd;
    int Hf, Wf, cs, cb, ce, ld, im_w, im_h, p0, M, c0, LC, G;
    UDiv dh, dw;
    int loss, no_memo, use_ratio, bilinear;
    int spec;               // speculative next-texel gathers on (runtime: launch option)
    int spec_cap;           // speculative gathers per wave per evaluation
    int spec_w0;            // the first wave that speculates
    int helpers;            // first-evaluation helper workgroups per problem (0: none)
    int hfirst;             // this is the problem's first evaluation
    int prob;               // the problem's index (helpers' record slots)
    const double *hrec;     // the helpers' records [n][nc_max * CH][HREC]
    const unsigned long long *hflag;
    unsigned long long htag;
    int dbg;
    int sob_norm, sob_rep;  // FMPNP_LAYOUT_F: the in-gather Sobel's flags
    double alpha;
    double *part_g;       // this team's partial slots [2][nc_max][NV] (G > 1)
    int nc_max;
    bool stamps;          // debug phase stamps on
    // debug timeline (FMPNP_DBG bit 4, evaluation FMPNP_DBG >> 8): absolute s_memtime of each
    // wave at the tl_stamp sites of one evaluation of the team's first problem, [8][16] per WG
    unsigned long long *tl;
    int tl_eval, cur_eval;
    int cur_ev;             // the evaluation being run (its pose is Ret[cur_ev & 1], its state sc[cur_ev & 1])
};

// The lane index, recomputed where it is used (v_mbcnt inside volatile asm: neither hoisted out of the
// evaluation loop nor merged with another copy).  Lane masks formed from threadIdx.x (lane < 12, lane < NV,
// ...) are loop invariants the compiler hoists into SGPR pairs, which the kernel's scalar pressure then
// spills to VGPR lanes: two v_readlane reloads and a wait state per use on the LM tail, against one
// v_cmp on a fresh lane index.
__device__ __forceinline__ int lane_now() {
#if defined(__HIP_DEVICE_COMPILE__) && FMPNP_LANE_NOW
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
#else
    return (int)(threadIdx.x & 63);
#endif
}
__device__ __forceinline__ int ufirst(int v) { return __builtin_amdgcn_readfirstlane(v); }
// waves of this workgroup: 8 (NT threads, the latency build) or 4 (the throughput build's
// 256-thread workgroups, two per CU)
__device__ __forceinline__ int nwaves() { return (int)(blockDim.x >> 6); }
__device__ __forceinline__ unsigned ufirst(unsigned v) { return (unsigned)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ double ufirst(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)b), hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ unsigned long long ufirst(unsigned long long v) {
    const unsigned lo = ufirst((unsigned)v), hi = ufirst((unsigned)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
}
template <typename P>
__device__ __forceinline__ P *ufirst(P *p) {
    const uintptr_t b = (uintptr_t)p;
    const unsigned lo = ufirst((unsigned)b), hi = ufirst((unsigned)(b >> 32));
    return (P *)(((uintptr_t)hi << 32) | lo);
}

// The LM schedule's scalar state (model.py:281-283,347-359,469-486).  Two copies: evaluation k
// reads sc[k & 1] and its tail writes sc[(k + 1) & 1], so the tail's waves (lm_tail_split) read
// the state before the evaluation while one of them writes the next.
struct LMScal {
    double lambda, lr, prev, best, initial;
    int done;
    int nan;                // a step came out NaN (model.py:411-413): written by the stepping wave only
    int best_inl, n_evals, n_steps, n_accepted, status, has_best, ret_current;
};
static_assert(offsetof(LMScal, nan) == offsetof(LMScal, done) + 4 && offsetof(LMScal, done) % 8 == 0,
              "done / nan: one 8-byte read at the top of every evaluation");
constexpr int TAIL_ROLES = 3;  // tail waves of the split tail: accept stepper, reject stepper, bookkeeper
struct LMState {
    double tot[TAIL_ROLES][NV];  // each tail wave's combined totals of the evaluation (broadcast operands)
    double hc[NV];          // cached linearisation at (R, t): H upper triangle, then g
    double Rt[12];          // current (last accepted) pose [R | t]
    double Ret[2][12];      // pose [R | t] evaluated by evaluation k: Ret[k & 1]
    double Rbt[12];         // best pose
    LMScal sc[2];
    double rho_max;
    int abort_flag, sync_ok;
    int win_miss;           // a gather left the packed window (with abort_flag: FMPNP_STATUS_WINDOW)
    int helper_absent;      // a first-evaluation helper never published: the other blocks skip the wait
    // the ratio test with a guessed limit (at most 8 blocks): evaluation k's guess is rguess[k & 1];
    // rstat[b] = max|rho| of block b's supported points (NaN-propagating)
    double rguess[2];
    double rstat[8];
#if FMPNP_STAMPS
    unsigned long long tlb[NT / 64][16];  // debug timeline (FMPNP_DBG bit 4), flushed at problem end
#endif
    double wg_max[NT / 64];
    unsigned long long bil_dirty[BIL_MAX_M / 64];  // bilinear memo: each block's points whose cell changed
    long long wg_gath[NT / 64];                     // per-wave texel gathers of the problem (G = 1)
#if FMPNP_STAMPS
    unsigned long long stamp_t[NT / 64], stamp_ph[NT / 64][NSTAMP];  // debug phase stamps (lane 0 per wave)
#endif
    Ctx c;
};
static_assert(sizeof(LMState) <= lds_fixed_bytes(), "LDS head too small");
static_assert(offsetof(LMState, Ret) % 16 == 0, "Ret: 16-byte LDS writes of the next pose");

__device__ __forceinline__ LMState &S() { return *reinterpret_cast<LMState *>(lm_lds); }

// Registers <- the LDS Ctx, once per problem (after problem_begin's barrier).
__device__ __forceinline__ PC load_pc() {
    const Ctx &c = S().c;
    PC q;
    q.feat = ufirst(c.feat);
    q.fref = ufirst(c.fref);
    q.fx = ufirst(c.K[0]);
    q.cx = ufirst(c.K[2]);
    q.fy = ufirst(c.K[4]);
    q.cy = ufirst(c.K[5]);
    q.kstd = ufirst((c.K[1] == 0.0 && c.K[3] == 0.0 && c.K[6] == 0.0 && c.K[7] == 0.0 && c.K[8] == 1.0) ? 1 : 0);
    q.Hf = ufirst(c.Hf); q.Wf = ufirst(c.Wf); q.cs = ufirst(c.cs); q.cb = ufirst(c.cb); q.ce = ufirst(c.ce);
    q.ld = ufirst(c.ld_ref); q.im_w = ufirst(c.im_w); q.im_h = ufirst(c.im_h); q.p0 = ufirst(c.p0);
    q.M = ufirst(c.M); q.c0 = ufirst(c.c0); q.LC = ufirst(c.LC); q.G = ufirst(c.G);
    q.dh = UDiv{ufirst(c.div_h.m), ufirst(c.div_h.s1), ufirst(c.div_h.s2)};
    q.dw = UDiv{ufirst(c.div_w.m), ufirst(c.div_w.s1), ufirst(c.div_w.s2)};
#if FMPNP_VCONST
    // the projection's constants in VGPRs (wave-uniform values, but the kernel's scalar registers are
    // spilled to VGPR lanes: each SGPR operand of the projection was a v_readlane reload + s_nop)
    asm volatile("" : "+v"(q.cx), "+v"(q.cy));
    asm volatile("" : "+v"(q.dh.m), "+v"(q.dh.s1), "+v"(q.dh.s2), "+v"(q.dw.m), "+v"(q.dw.s1), "+v"(q.dw.s2));
#endif
    q.loss = ufirst(c.mode == FMPNP_MODE_COMPUTE_COST ? (int)FMPNP_SQUARED : c.loss);
    q.no_memo = ufirst(c.no_memo);
    q.spec = ufirst(c.spec);
    q.spec_cap = ufirst(c.spec_cap);
    q.spec_w0 = ufirst(c.spec_w0);
    q.dbg = ufirst(c.dbg);
    q.bilinear = ufirst(c.sampling == FMPNP_BILINEAR ? 1 : 0);
    q.use_ratio = ufirst(c.use_ratio);
    q.alpha = ufirst(c.alpha);
    q.sob_norm = ufirst(c.sobel_flags & 1);
    q.sob_rep = ufirst((c.sobel_flags >> 1) & 1);
    q.part_g = ufirst(c.part_g);
    q.nc_max = ufirst(c.nc_max);
    q.stamps = kStamps && ufirst(c.stamps_on) != 0;
    q.tl = nullptr;
    q.tl_eval = q.cur_eval = -1;
    q.cur_ev = 0;
    return q;
}
// debug: add the cycles since the wave's previous stamp to its phase k (lane 0 of each
// wave); phases 0..3 of the first evaluation go to slots 8..11
__device__ __forceinline__ void dbg_stamp(bool on, int k) {
#if FMPNP_STAMPS
    LMState &st = *reinterpret_cast<LMState *>(lm_lds);
    if (on && (threadIdx.x & 63) == 0) {
        const int w = threadIdx.x >> 6;
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        st.stamp_ph[w][k < 4 && st.sc[1].n_evals == 0 ? 8 + k : k] += now - st.stamp_t[w];
        st.stamp_t[w] = now;
    }
#endif
}
__device__ __forceinline__ void tl_stamp(const PC &q, int k) {
#if FMPNP_ISA_MARKS  // (ISA census build, tools/isa_census.py: a comment in the assembly at every stamp site)
    asm volatile(";@@TL %0" ::"i"(k));
#endif
#if FMPNP_STAMPS
    if (q.tl && q.cur_eval == q.tl_eval && (threadIdx.x & 63) == 0)
        reinterpret_cast<LMState *>(lm_lds)->tlb[threadIdx.x >> 6][k] = __builtin_amdgcn_s_memtime();
#endif
}
// project_px (fmpnp_device.h) for the problem's K.  With a pinhole K the products of its zero
// entries are dropped: (fx P0 + 0 P1) + cx P2 equals fx P0 + cx P2 and (0 P0 + 0 P1) + 1 P2
// equals P2 except in the sign of a zero or for a non-finite coordinate, and each of those makes
// the quotient non-finite or rounds the pixel to -1 either way -- the point is unsupported in
// both forms, so the support set and every pixel are the reference's.
// rz: recip(P[2]) (the Jacobian chain's 1/z, geo_of_iz: formed once per point and evaluation)
__device__ __forceinline__ bool project_pc(const PC &q, const double P[3], int &x, int &y, double &qx, double &qy,
                                           double &rz) {
    if (q.kstd) {
#pragma clang fp contract(off)
        const double u0 = q.fx * P[0] + q.cx * P[2];
        const double u1 = q.fy * P[1] + q.cy * P[2];
        if (q.bilinear) {  // the taps use the unrounded quotients: the reference's exact division
            qx = u0 / P[2];
            qy = u1 / P[2];
            rz = recip(P[2]);
        } else {
            // Only the rounded pixel matters here: the quotients by one refined reciprocal (within
            // ~3 ulp of the correctly rounded u / z) round to the same integers as the IEEE
            // quotients unless one lies within 8 ulp of a half-integer (rint's boundary, ties to
            // even) -- those lanes, and any z outside [2^-1000, 2^1000] or a non-finite quotient,
            // take the exact divisions.  So px, py and the support test are the reference's; qx, qy
            // only feed the speculation's next-texel prediction.
            const double z = P[2], r = recip(z);
            rz = r;
            double ax = u0 * r, ay = u1 * r;
            const double ex = fabs(fabs(ax - rint(ax)) - 0.5), ey = fabs(fabs(ay - rint(ay)) - 0.5);
            const bool fast = fabs(z) > 0x1p-1000 && fabs(z) < 0x1p+1000 && ex > fabs(ax) * 0x1p-49 &&
                              ey > fabs(ay) * 0x1p-49;  // (false for NaN / infinite quotients)
            if (!fast) {
                ax = u0 / z;
                ay = u1 / z;
            }
            qx = ax;
            qy = ay;
        }
        const double px = rint(qx) - 1.0, py = rint(qy) - 1.0;
        if (!(px >= 0.0 && px < (double)q.im_w && py >= 0.0 && py < (double)q.im_h)) return false;
        x = (int)px;
        y = (int)py;
        return true;
    }
    const double *Kl = reinterpret_cast<const LMState *>(lm_lds)->c.K;  // broadcast reads (rare: non-pinhole K)
    double K[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) K[k] = Kl[k];
    rz = recip(P[2]);
    return project_px(K, P, q.im_w, q.im_h, x, y, qx, qy);
}
__device__ __forceinline__ unsigned char *dyn() { return lm_lds + lds_fixed_bytes(); }
// dynamic carve (mmax = max local points, a multiple of CH), structure of arrays with the
// odd row stride rs = lds_rs(mmax) doubles:
//   X[3][rs], rec[RECW][rs] doubles, tex[mmax] ints (16-B padded), part[nc_max][NV] doubles
// A lane-per-point read of coordinate / record field k (X[k][i], rec[k][i]) is 64 consecutive
// doubles: conflict-free.  A gather's six writers (field e6 of one point j) hit banks
// 2 (e6 rs + j) mod 64, distinct because rs is odd.
//   speculation (lds_spec_doubles / lds_words: only tex when it is off): a second record slot
//   rec2[6][rs] doubles, then after tex: tex2[mmax] (the texel of the slot not in use),
//   spec[mmax] (this evaluation's prediction), slot[mmax] (the slot in use: 0 rec, 1 rec2),
//   qp[2][mmax] floats (the last projected pixel position)
__device__ __forceinline__ double *lds_X(int mmax) { return reinterpret_cast<double *>(dyn()); }
__device__ __forceinline__ double *lds_rec(int mmax) { return reinterpret_cast<double *>(dyn()) + 3 * lds_rs(mmax); }
__device__ __forceinline__ double *lds_rec2(int mmax) {
    return reinterpret_cast<double *>(dyn()) + (3 + RECW) * lds_rs(mmax);
}
__device__ __forceinline__ int *lds_tex(int mmax, bool spec) {
    return reinterpret_cast<int *>(reinterpret_cast<double *>(dyn()) + (3 + RECW) * lds_rs(mmax) +
                                   lds_spec_doubles(mmax, spec));
}
__device__ __forceinline__ int *lds_tex2(int mmax, bool spec) { return lds_tex(mmax, spec) + mmax; }
__device__ __forceinline__ int *lds_spec(int mmax, bool spec) { return lds_tex(mmax, spec) + 2 * mmax; }
__device__ __forceinline__ int *lds_slot(int mmax, bool spec) { return lds_tex(mmax, spec) + 3 * mmax; }
__device__ __forceinline__ float *lds_qp(int mmax, bool spec) {
    return reinterpret_cast<float *>(lds_tex(mmax, spec) + 4 * mmax);
}
__device__ __forceinline__ double *lds_part(int mmax, bool spec) {
    return reinterpret_cast<double *>(lds_tex(mmax, spec) + lds_words(mmax, spec));
}
// the bilinear cell memo memo[BIL_NB][rs] (after part[nc_max][NV]; never with speculation)
__device__ __forceinline__ double *lds_memo(int mmax, int nc_max) { return lds_part(mmax, false) + (size_t)nc_max * NV; }

// so3exp_map (helpers/utils.py:209-221) and the update R' = dR R, t' = dR t + dt
// (model.py:416-426).  Steps up to 45 degrees (every LM step in practice) take the sqrt- and
// division-free form dR = cos(theta) I + (sin(theta)/theta) W + ((1 - cos theta)/theta^2) w w^T
// (so3_coeffs_small: three independent polynomials in z = |w|^2, a short dependency chain on the
// LM tail); larger steps the reference's normalised form.
__device__ __forceinline__ void pose_update(const double *R, const double *t, const double delta[6], double *Rn,
                                            double *tn) {
    const double w0 = delta[3], w1 = delta[4], w2 = delta[5];
    const double z = fma(w2, w2, fma(w1, w1, w0 * w0));
    double dR[9];
    // (the common case first and alone: no identity / NaN matrix materialised on its path)
    if (z >= 1e-24 && z <= 0.61685027506808487) {  // 1e-12 <= theta <= pi/4 (false for NaN)
        double cz, az, bz;
        so3_coeffs_small(z, cz, az, bz);
        const double bw0 = bz * w0, bw1 = bz * w1, bw2 = bz * w2;
        const double aw0 = az * w0, aw1 = az * w1, aw2 = az * w2;
        dR[0] = fma(bw0, w0, cz);
        dR[1] = fma(bw0, w1, -aw2);
        dR[2] = fma(bw0, w2, aw1);
        dR[3] = fma(bw1, w0, aw2);
        dR[4] = fma(bw1, w1, cz);
        dR[5] = fma(bw1, w2, -aw0);
        dR[6] = fma(bw2, w0, -aw1);
        dR[7] = fma(bw2, w1, aw0);
        dR[8] = fma(bw2, w2, cz);
    } else if (isnan(z)) {
#pragma unroll
        for (int i = 0; i < 9; ++i) dR[i] = NAN;
    } else {
#pragma unroll
        for (int i = 0; i < 9; ++i) dR[i] = (i % 4 == 0) ? 1.0 : 0.0;
        if (!(z < 1e-24)) {  // theta > pi/4 (below 1e-12: the identity, as the reference)
            const double theta = sqrt(z);
            const double it = 1.0 / theta;
            const double k0 = w0 * it, k1 = w1 * it, k2 = w2 * it;
            const double W[9] = {0, -k2, k1, k2, 0, -k0, -k1, k0, 0};
            double sn, cs;
            sincos_rr(theta, sn, cs);
            const double c1 = 1.0 - cs;
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    double ww = W[3 * i + 0] * W[0 + j] + W[3 * i + 1] * W[3 + j] + W[3 * i + 2] * W[6 + j];
                    dR[3 * i + j] += W[3 * i + j] * sn + ww * c1;
                }
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
// Cross-workgroup exchange inside a team (G > 1), MI355X_MICROARCH.md "sc1 loads in place
// of the acquire", first row: every byte handed off is stored write-through (sc1) and
// read back with global sc1 loads; every storing wave drains (vmcnt(0)) before a workgroup
// barrier, behind which ONE lane per workgroup adds to the team's arrival counter (agent
// scope); the consumer is the polling wave itself (wave 0), which loads only after its
// poll has matched -- no L1 invalidate, no second barrier.  The counter is monotonic
// within a launch and zeroed by the launcher (hipMemsetAsync) before every launch.
// One workgroup per CU (the planner's launch bounds), memory from hipMalloc.
// ---------------------------------------------------------------------------
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(1))) unsigned long long g_u64;
typedef __attribute__((address_space(1))) unsigned g_u32;
#else
typedef unsigned long long g_u64;  // host pass: never executed
typedef unsigned g_u32;
#endif
__device__ __forceinline__ void st_sc1(double *p, double v) {
    __hip_atomic_store(reinterpret_cast<g_u64 *>(reinterpret_cast<uintptr_t>(p)), (unsigned long long)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double *p) {
    return __longlong_as_double((long long)__hip_atomic_load(
        reinterpret_cast<g_u64 *>(reinterpret_cast<uintptr_t>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Every thread calls this after its sc1 stores: this workgroup's arrival for the next epoch.
__device__ __forceinline__ void team_arrive() {
    LMState &st = S();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x == 0) {
        ++st.c.epoch;
        __hip_atomic_fetch_add(reinterpret_cast<g_u32 *>(reinterpret_cast<uintptr_t>(st.c.counter)), 1u,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Wave 0 (all its lanes) after team_arrive: thread 0 polls until every member has arrived
// for the current epoch (bounded: ~2 s of wall time, s_memrealtime ticks at 100 MHz).
// Returns false -- and raises the workgroup's abort flag -- on timeout.
__device__ __forceinline__ bool team_wait() {
    LMState &st = S();
    int ok = 1;
    if (threadIdx.x == 0) {
        const unsigned target = st.c.epoch * (unsigned)st.c.G;
        g_u32 *counter = reinterpret_cast<g_u32 *>(reinterpret_cast<uintptr_t>(st.c.counter));
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) { ok = 0; break; }
        }
        if (!ok) st.abort_flag = 1;
    }
    return __builtin_amdgcn_readfirstlane(ok) != 0;
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
        c.win_ok = pb->window ? pb->window + (size_t)pb->Hf * pb->Wf : nullptr;
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
        c.div_h = udiv_make((unsigned)c.im_h);
        c.div_w = udiv_make((unsigned)c.im_w);
        c.txpx = (float)c.Wf / (float)c.im_w;
        c.typx = (float)c.Hf / (float)c.im_h;
        c.pxtx = (float)c.im_w / (float)c.Wf;
        c.pypx = (float)c.im_h / (float)c.Hf;
        c.NC = (c.N + CH - 1) / CH;
        c.c0 = (int)(((long)c.NC * c.s) / c.G);
        const int c1 = (int)(((long)c.NC * (c.s + 1)) / c.G);
        c.LC = c1 - c.c0;
        c.p0 = c.c0 * CH;
        c.M = max(min(c1 * CH, c.N) - c.p0, 0);
        c.vec = 0;
        for (int k = 0; k < 12; ++k) st.Rt[k] = st.Ret[0][k] = st.Rbt[k] = k < 9 ? pb->R0[k] : pb->t0[k - 9];
        for (int par = 0; par < 2; ++par) {
            LMScal &sc = st.sc[par];
            sc.lambda = c.lambda0;
            sc.lr = 1.0;
            sc.prev = sc.best = sc.initial = NAN;
            sc.best_inl = -1;
            sc.n_evals = sc.n_steps = sc.n_accepted = 0;
            sc.status = c.dead ? FMPNP_STATUS_SYNC_TIMEOUT : 0;
            sc.has_best = 0;
            sc.ret_current = 0;
            sc.done = c.dead || (c.mode != FMPNP_MODE_COMPUTE_COST && c.n_iters <= 0);
            sc.nan = 0;
        }
        st.abort_flag = 0;
        st.win_miss = 0;
        st.rguess[0] = st.rguess[1] = INFINITY;  // (evaluation 0: no guess -- every supported point kept)
        st.helper_absent = 0;
    }
    __syncthreads();
    // this workgroup's points -> LDS once per problem
    const Ctx &c = st.c;
    double *X = lds_X(mmax);
    const double *src = c.pts + 3 * (size_t)c.p0;
    const int rs = lds_rs(mmax);
    const int nt = (int)blockDim.x;
    for (int e = tid; e < 3 * c.M; e += nt) X[(e % 3) * rs + e / 3] = src[e];
    int *tex = lds_tex(mmax, c.spec);
    for (int i = tid; i < mmax; i += nt) tex[i] = -2;  // no texel cached yet
#if FMPNP_STAMPS
    for (int i = tid; i < (NT / 64) * 16; i += nt) st.tlb[i >> 4][i & 15] = 0;  // debug timeline
#endif
    if (c.spec) {
        int *tex2 = lds_tex2(mmax, true), *slot = lds_slot(mmax, true), *spec = lds_spec(mmax, true);
        float *qp = lds_qp(mmax, true);
        for (int i = tid; i < mmax; i += nt) {
            tex2[i] = -2;
            slot[i] = 0;
            spec[i] = -1;
            qp[i] = qp[mmax + i] = __builtin_nanf("");  // no motion known: no prediction at evaluation 0
        }
    }
    __syncthreads();
}

// k: the evaluations completed (the state is sc[k & 1])
// miss_aborts: the f-only layout, where a window miss itself raises abort_flag (one workgroup per
// problem); elsewhere abort_flag means a timed-out team exchange, whatever else happened
__device__ __forceinline__ void problem_end(bool own_gathers, int k, unsigned long long *tl, bool miss_aborts) {
    LMState &st = S();
#if FMPNP_STAMPS
    if (tl && (threadIdx.x & 63) == 0)  // debug timeline: this wave's stamps
        for (int j = 0; j < 16; ++j) tl[(threadIdx.x >> 6) * 16 + j] = st.tlb[threadIdx.x >> 6][j];
#endif
    if (threadIdx.x == 0) {
        LMScal &sc = st.sc[k & 1];
        if (st.win_miss) sc.status |= FMPNP_STATUS_WINDOW;
        if (st.abort_flag && !(st.win_miss && miss_aborts)) {
            st.c.dead = 1;
            sc.status |= FMPNP_STATUS_SYNC_TIMEOUT;
        }
        if (sc.nan) sc.status |= FMPNP_STATUS_NAN;
        if (st.c.s == 0) {
            fmpnp_result &r = st.c.results[st.c.p];
            const bool cur = sc.ret_current || st.c.mode == FMPNP_MODE_COMPUTE_COST;
            for (int j = 0; j < 9; ++j) r.R[j] = cur ? st.Rt[j] : st.Rbt[j];
            for (int j = 0; j < 3; ++j) r.t[j] = cur ? st.Rt[9 + j] : st.Rbt[9 + j];
            r.initial_cost = sc.initial;
            r.best_cost = sc.has_best ? sc.best : NAN;
            r.final_lambda = sc.lambda;
            r.final_lr = sc.lr;
            r.best_num_inliers = sc.has_best ? sc.best_inl : -1;
            r.n_evals = sc.n_evals;
            r.n_steps = sc.n_steps;
            r.n_accepted = sc.n_accepted;
            // (a team's results were zeroed: every member ORs in its window misses, below)
            if (!own_gathers) atomicOr(&r.status, sc.status);
            else r.status = sc.status;
            r.has_best = sc.has_best;
            if (own_gathers) {
                long long g = 0;
                for (int w = 0; w < nwaves(); ++w) g += st.wg_gath[w];
                r.texel_gathers = g;
            }
        } else if (!own_gathers && st.win_miss) {
            atomicOr(&st.c.results[st.c.p].status, FMPNP_STATUS_WINDOW);  // (another team member's miss)
        }
    }
    __syncthreads();
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
        if (ce - cb > 64 * V) {
            // C > 64 V (C = 512 fp32, the pyramid's coarse level and cfg5; C = 1024 of the RobotCar
            // hypercolumn's [640:1664] slice): chunks of four rounds whose sixteen loads are all
            // issued before the first use -- one memory round trip per 128 V channels instead of
            // one per 64 V.  Rounds are consumed in the loop's (r, k) order, so the sums are the
            // loop's bit for bit; missing rounds read round one again and add exact zeros (a sum
            // of fma(0, 0, s) steps from +0 is never -0: the zeros change no bit).
            for (int c = cb + l32 * V; c < ce; c += 128 * V) {
                VT f[4], x[4], y[4], q[4];
                bool has[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    has[r] = c + r * 32 * V < ce;
                    const int cr = has[r] ? c + r * 32 * V : c;
                    f[r] = gload<VT>(t + cr);
                    x[r] = gload<VT>(t + cs + cr);
                    y[r] = gload<VT>(t + 2 * cs + cr);
                    q[r] = gload<VT>(rf + cr);
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const T *pf = reinterpret_cast<const T *>(&f[r]), *px = reinterpret_cast<const T *>(&x[r]);
                    const T *py = reinterpret_cast<const T *>(&y[r]), *pr = reinterpret_cast<const T *>(&q[r]);
#pragma unroll
                    for (int k = 0; k < V; ++k) {
                        const double z = 0.0;
                        acc6(a, has[r] ? (double)pf[k] : z, has[r] ? (double)pr[k] : z, has[r] ? (double)px[k] : z,
                             has[r] ? (double)py[k] : z);
                    }
                }
            }
            return;
        }
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

// Transposed reduction of the 32-value vector over all 64 lanes of a wave.  `val(k)`
// yields value k of the lane; values are produced in pairs (i, i+16) and folded at once by
// the permlane32 swap (bit 5), so at most 16 doubles are live; then bit 4 (permlane16 swap)
// and the in-row DPP steps.  Lane l returns the wave total of value index
// 16*b5 + 8*b4 + 4*b3 + 2*b2 + b1 (b0 duplicates).  Only equal indices are ever added.
template <typename F>
__device__ __forceinline__ double reduce32_in64(F &&val, int lane) {
    double v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        double a = val(i), b = val(i + 16);
        swap32(a, b);  // low half keeps index i, high half i + 16
        v[i] = a + b;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        double a = v[i], b = v[i + 8];
        swap16(a, b);  // even rows keep index i, odd rows i + 8
        v[i] = a + b;
    }
    return reduce8_in16(v, lane & 15);
}
__device__ __forceinline__ int reduce32_index(int lane) {
    return 16 * ((lane >> 5) & 1) + 8 * ((lane >> 4) & 1) + 4 * ((lane >> 3) & 1) + 2 * ((lane >> 2) & 1) +
           ((lane >> 1) & 1);
}

// ---------------------------------------------------------------------------
// Ratio test (model.py:120-129): the team's max |rho| (order-free: exact) from every
// wave's maximum.  Returns false on abort.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool ratio_exchange(double lmax) {
    LMState &st = S();
    const Ctx &c = st.c;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    lmax = wave_nanmax(lmax);
    if (lane == 0) st.wg_max[wave] = lmax;
    __syncthreads();
    if (tid == 0) {
        double m = st.wg_max[0];
        for (int w = 1; w < nwaves(); ++w) m = nanmax(m, st.wg_max[w]);
        st.rho_max = m;
        if (c.G > 1) st_sc1(c.max_g + ((c.epoch + 1) & 1) * c.G + c.s, m);
    }
    if (c.G > 1) {
        team_arrive();
        if (tid < 64 && team_wait() && tid == 0) {
            double m = -1.0;
            for (int w = 0; w < c.G; ++w) m = nanmax(m, ld_sc1(c.max_g + (c.epoch & 1) * c.G + w));
            st.rho_max = m;
        }
    }
    __syncthreads();
    return !st.abort_flag;
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

// One 64-point block of a wave: lane = point.  Points that do not contribute get w = 0
// and a harmless geometry (z = 1).  Writes the block's partial (one chunk: LDS when
// G == 1, the team's global slot `dst_g` with sc1 stores when G > 1).
// J_px_p (model.py:377-382) times J_p_T (model.py:369-370) of a point: A (2x6), A0[1] = A1[0] = 0
// (a point that does not contribute gets the harmless geometry P = (0, 0, 1))
struct Geo {
    double A0[6], A1[6];
};
// izk: recip(Pc[2]) (from project_pc); a point that does not contribute takes z = 1, 1 / z = 1
__device__ __forceinline__ Geo geo_of_iz(const PC &q, bool kept, const double Pc[3], double izk) {
    const double fx = q.fx, fy = q.fy;
    const double P0 = kept ? Pc[0] : 0.0, P1 = kept ? Pc[1] : 0.0, z = kept ? Pc[2] : 1.0;
    // one reciprocal instead of six divisions (Jacobian entries only: last-bit level)
    const double iz = kept ? izk : 1.0;
    const double j00 = fx * iz, j02 = ((-fx) * P0 * iz) * iz;
    const double j11 = fy * iz, j12 = ((-fy) * P1 * iz) * iz;
    return Geo{{j00, 0.0, j02, j02 * P1, j00 * z - j02 * P0, -j00 * P1},
               {0.0, j11, j12, -j11 * z + j12 * P1, -j12 * P0, j11 * P0}};
}
__device__ __forceinline__ void contrib_geo(const PC &q, int mmax, int blk, bool sup, bool kept, double rho,
                                            double d1, const double *r, int rs, const Geo &G, double *dst_g);
__device__ __forceinline__ void contrib_block(const PC &q, int mmax, int blk, bool sup, bool kept, double rho,
                                              double d1, const double *r, int rs, const double Pc[3],
                                              double *dst_g) {
    contrib_geo(q, mmax, blk, sup, kept, rho, d1, r, rs, geo_of_iz(q, kept, Pc, recip(Pc[2])), dst_g);
}
// ... with the point's recip(Pc[2]) already formed by project_pc
__device__ __forceinline__ void contrib_block_iz(const PC &q, int mmax, int blk, bool sup, bool kept, double rho,
                                                 double d1, const double *r, int rs, const double Pc[3], double izk,
                                                 double *dst_g) {
    contrib_geo(q, mmax, blk, sup, kept, rho, d1, r, rs, geo_of_iz(q, kept, Pc, izk), dst_g);
}
__device__ __forceinline__ void contrib_geo(const PC &q, int mmax, int blk, bool sup, bool kept, double rho,
                                            double d1, const double *r, int rs, const Geo &G, double *dst_g) {
    const int lane = threadIdx.x & 63;
    const int lc = blk;  // one chunk per 64-point block
    const double w = kept ? d1 : 0.0, rh = kept ? rho : 0.0;
    // the point's record fields (SoA, stride rs): sum gx e, sum gy e, sum gx^2, sum gx gy, sum gy^2
    const double sex = kept ? r[rs] : 0.0, sey = kept ? r[2 * rs] : 0.0;
    const double sxx = kept ? r[3 * rs] : 0.0, sxy = kept ? r[4 * rs] : 0.0, syy = kept ? r[5 * rs] : 0.0;
    const double *A0 = G.A0, *A1 = G.A1;
    // w folded into the 2x2 channel moments; the structural zeros A0[1] = A1[0] = 0 are
    // skipped explicitly (IEEE arithmetic cannot drop 0 * x by itself)
    const double wxx = w * sxx, wxy = w * sxy, wyy = w * syy, wex = w * sex, wey = w * sey;
    double M0[6], M1[6];  // (w S) A: M0 = row x, M1 = row y
    M0[0] = wxx * A0[0];
    M1[0] = wxy * A0[0];
    M0[1] = wxy * A1[1];
    M1[1] = wyy * A1[1];
#pragma unroll
    for (int l = 2; l < 6; ++l) {
        M0[l] = wxx * A0[l] + wxy * A1[l];
        M1[l] = wxy * A0[l] + wyy * A1[l];
    }
    auto val = [&](int k) -> double {
        if (k < 21) {  // H[a][b] = A_a^T (w S) A_b
            const int a = h_row(k), b = h_col(k);
            return a == 0 ? A0[0] * M0[b] : a == 1 ? A1[1] * M1[b] : A0[a] * M0[b] + A1[a] * M1[b];
        } else if (k < 27) {  // g = A^T (w G^T e)
            const int l = k - 21;
            return l == 0 ? A0[0] * wex : l == 1 ? A1[1] * wey : A0[l] * wex + A1[l] * wey;
        } else if (k == 27) {
            return rh;
        } else if (k == 28) {
            return kept ? 1.0 : 0.0;
        } else if (k == 29) {
            return sup ? 1.0 : 0.0;
        }
        return 0.0;
    };
    const double tot = reduce32_in64(val, lane);
    if (lc < q.LC && (lane & 1) == 0) {
        const int idx = reduce32_index(lane);
        if (q.G == 1) lds_part(mmax, q.spec)[(size_t)(q.c0 + lc) * NV + idx] = tot;  // G == 1 (LDS)
        else st_sc1(dst_g + (size_t)(q.c0 + lc) * NV + idx, tot);
    }
}

// The eight 16-byte loads of one point's texel for one half-wave lane (C <= 64 V channels:
// a point is one memory round trip), issued ahead of their use so that the next pair's
// loads are in flight while the current pair is reduced.
template <typename T>
struct GLoad {
    typename V16<T>::type f0, x0, y0, q0, f1, x1, y1, q1;
};
template <typename T>
__device__ __forceinline__ void g_issue(GLoad<T> &g, const T *t, const T *rf, int cs, int c, int c2) {
    using VT = typename V16<T>::type;
    g.f0 = gload<VT>(t + c);
    g.x0 = gload<VT>(t + cs + c);
    g.y0 = gload<VT>(t + 2 * cs + c);
    g.q0 = gload<VT>(rf + c);
    g.f1 = gload<VT>(t + c2);
    g.x1 = gload<VT>(t + cs + c2);
    g.y1 = gload<VT>(t + 2 * cs + c2);
    g.q1 = gload<VT>(rf + c2);
}
// Same accumulation order as gather_half<T, true> (round one, then round two or exact
// zeros), so both paths give bit-identical sums; has1 = false lanes add nothing.
// FULL: every lane has both rounds (C == 64 V, e.g. C = 256 fp32): no per-lane selects.
template <typename T, bool FULL>
__device__ __forceinline__ void g_consume(const GLoad<T> &g, bool has1, bool has2, double a[8]) {
    constexpr int V = V16<T>::n;
    if (FULL) has1 = has2 = true;
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = 0.0;
    if (!has1) return;
    const T *pf = reinterpret_cast<const T *>(&g.f0), *px = reinterpret_cast<const T *>(&g.x0);
    const T *py = reinterpret_cast<const T *>(&g.y0), *pr = reinterpret_cast<const T *>(&g.q0);
#pragma unroll
    for (int k = 0; k < V; ++k) acc6(a, (double)pf[k], (double)pr[k], (double)px[k], (double)py[k]);
    const T *sf = reinterpret_cast<const T *>(&g.f1), *sx = reinterpret_cast<const T *>(&g.x1);
    const T *sy = reinterpret_cast<const T *>(&g.y1), *sr = reinterpret_cast<const T *>(&g.q1);
#pragma unroll
    for (int k = 0; k < V; ++k) {
        const double z = 0.0;
        acc6(a, has2 ? (double)sf[k] : z, has2 ? (double)sr[k] : z, has2 ? (double)sx[k] : z,
             has2 ? (double)sy[k] : z);
    }
}

// Where a gathered point's record fields go: this lane's field column (e6) at the block start
// in the two record slots.  A gather always fills the slot a point is NOT currently using
// (its current slot keeps serving until the evaluation switches over): point j is written
// into slot a when bit j of `sel` is set (its current slot is b), else into b.  a == b: one
// slot (no speculation).
struct RecDst {
    double *a, *b;
    unsigned long long sel;
    __device__ __forceinline__ double *col(int j) const { return ((sel >> j) & 1ull) ? a : b; }
};

// Pair selection from a dirty mask: the half-waves take the two lowest set lanes.
struct GPair {
    int j;      // this half-wave's point (lane index in the block)
    int to;     // its texel offset
    bool two;   // a second point exists (the high half's point is real)
};
__device__ __forceinline__ GPair pick_pair(unsigned long long &m, int off, bool hi) {
    const int a = __builtin_ctzll(m);
    m &= m - 1;
    const bool two = m != 0;
    const int b = two ? __builtin_ctzll(m) : a;
    if (two) m &= m - 1;
    const int oa = __builtin_amdgcn_readlane(off, a), ob = __builtin_amdgcn_readlane(off, b);
    return GPair{hi ? b : a, hi ? ob : oa, two};
}

// Bilinear channel sums of one point for one half-wave lane (FMPNP_BILINEAR): the four
// taps' f, gx, gy and fref of the lane's channels per round (13 loads of 16 B at fp32),
// sampled with the point's weights (sample4) and accumulated like the nearest gather.
template <typename T, bool VEC>
__device__ __forceinline__ void gather_bil_half(const T *__restrict__ feat, const int o[4], const double w[4],
                                                const T *__restrict__ rf, int cs, int cb, int ce, int l32,
                                                double a[8]) {
    using VT = typename V16<T>::type;
    constexpr int V = V16<T>::n;
    const T *t0 = feat + (size_t)o[0] * 3 * cs, *t1 = feat + (size_t)o[1] * 3 * cs;
    const T *t2 = feat + (size_t)o[2] * 3 * cs, *t3 = feat + (size_t)o[3] * 3 * cs;
    if constexpr (VEC) {
        for (int c = cb + l32 * V; c < ce; c += 32 * V) {
            VT f[4], x[4], y[4];
            const T *tp[4] = {t0, t1, t2, t3};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                f[k] = gload<VT>(tp[k] + c);
                x[k] = gload<VT>(tp[k] + cs + c);
                y[k] = gload<VT>(tp[k] + 2 * cs + c);
            }
            const VT q = gload<VT>(rf + c);
            const T *pq = reinterpret_cast<const T *>(&q);
            const T *pf[4], *px[4], *py[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                pf[k] = reinterpret_cast<const T *>(&f[k]);
                px[k] = reinterpret_cast<const T *>(&x[k]);
                py[k] = reinterpret_cast<const T *>(&y[k]);
            }
#pragma unroll
            for (int e = 0; e < V; ++e)
                acc6(a, sample4(w, pf[0][e], pf[1][e], pf[2][e], pf[3][e]), (double)pq[e],
                     sample4(w, px[0][e], px[1][e], px[2][e], px[3][e]),
                     sample4(w, py[0][e], py[1][e], py[2][e], py[3][e]));
        }
    } else {
        for (int c = cb + l32 * V; c < ce; c += 32 * V) {
#pragma unroll
            for (int e = 0; e < V; ++e)
                if (c + e < ce) {
                    const int ch = c + e;
                    acc6(a, sample4(w, t0[ch], t1[ch], t2[ch], t3[ch]), (double)rf[ch],
                         sample4(w, t0[cs + ch], t1[cs + ch], t2[cs + ch], t3[cs + ch]),
                         sample4(w, t0[2 * cs + ch], t1[2 * cs + ch], t2[2 * cs + ch], t3[2 * cs + ch]));
                }
        }
    }
}

// Every supported point of a block, two per trip (one per half-wave); each half-wave takes
// its point's taps from the point's lane.
template <typename T>
__device__ __forceinline__ void gather_bil_block(unsigned long long m, const Taps &tp, bool hi, int lane,
                                                 const T *feat, const T *fref0, int cs, int cb, int ce, int ld,
                                                 bool vec, const RecDst &rd, bool wlane) {
    const int l32 = lane & 31;
    while (m) {
        const int pa = __builtin_ctzll(m);
        m &= m - 1;
        const bool two = m != 0;
        const int pb = two ? __builtin_ctzll(m) : pa;
        if (two) m &= m - 1;
        const int src = hi ? pb : pa;
        int o[4];
        double w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int oa = __builtin_amdgcn_readlane(tp.off[k], pa), ob = __builtin_amdgcn_readlane(tp.off[k], pb);
            const double wa = rlane64(tp.w[k], pa), wb = rlane64(tp.w[k], pb);
            o[k] = hi ? ob : oa;
            w[k] = hi ? wb : wa;
        }
        double v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = 0.0;
        const T *rf = fref0 + (size_t)src * ld;
        if (vec) gather_bil_half<T, true>(feat, o, w, rf, cs, cb, ce, l32, v);
        else gather_bil_half<T, false>(feat, o, w, rf, cs, cb, ce, l32, v);
        const double r = reduce8_in32(v, lane);
        if (wlane && (!hi || two)) rd.col(src)[src] = r;
    }
}

// ---------------------------------------------------------------------------
// Bilinear cell memo (FMPNP_BILINEAR, memoised).  Inside one 2x2 cell a point's sampled
// vectors are s(ax, ay) = sum_ij u_i(ay) v_j(ax) T_ij with u = (1 - ay, ay), v = (1 - ax, ax),
// so every channel sum of two sampled vectors is a tensor-product quadratic in (ay, ax):
//   sum_c A_s B_s = sum_pq b_pq By_p Bx_q,  By = ((1-ay)^2, ay (1-ay), ay^2), Bx likewise,
// b_00 = <A00,B00>, b_01 = <A00,B01> + <A01,B00>, b_02 = <A01,B01>, b_10 = <A00,B10> + <A10,B00>,
// b_11 = <A00,B11> + <A01,B10> + <A10,B01> + <A11,B00>, b_12 = <A01,B11> + <A11,B01>,
// b_20 = <A10,B10>, b_21 = <A10,B11> + <A11,B10>, b_22 = <A11,B11>  (A_ij: row i, column j).
// The six sums need the pairs (D,D), (X,D), (Y,D), (X,X), (X,Y), (Y,Y) with D_ij = F_ij - fref
// (e = f_s - fref = sum w D because the weights sum to one): 54 coefficients per point, which
// depend only on the cell and the point's descriptor.  They are formed once when the point
// enters a cell (the 2x2 x 3 x C neighbourhood and fref read once, reduced across C in fp64)
// and kept in LDS; every evaluation inside the cell costs 54 LDS reads and 72 FMAs instead of
// 52C bytes of taps.  Same sums as sampling first (gather_bil_half) up to fp64 rounding.
// ---------------------------------------------------------------------------
// one channel's contributions, symmetric pair (A = B: cross coefficients halved here, doubled
// after the reduction, exactly)
__device__ __forceinline__ void bern_sym(double *acc, double a0, double a1, double a2, double a3) {
    acc[0] = fma(a0, a0, acc[0]);
    acc[1] = fma(a0, a1, acc[1]);
    acc[2] = fma(a1, a1, acc[2]);
    acc[3] = fma(a0, a2, acc[3]);
    acc[4] = fma(a1, a2, fma(a0, a3, acc[4]));
    acc[5] = fma(a1, a3, acc[5]);
    acc[6] = fma(a2, a2, acc[6]);
    acc[7] = fma(a2, a3, acc[7]);
    acc[8] = fma(a3, a3, acc[8]);
}
__device__ __forceinline__ void bern_asym(double *acc, const double a[4], const double b[4]) {
    acc[0] = fma(a[0], b[0], acc[0]);
    acc[1] = fma(a[1], b[0], fma(a[0], b[1], acc[1]));
    acc[2] = fma(a[1], b[1], acc[2]);
    acc[3] = fma(a[2], b[0], fma(a[0], b[2], acc[3]));
    acc[4] = fma(a[3], b[0], fma(a[2], b[1], fma(a[1], b[2], fma(a[0], b[3], acc[4]))));
    acc[5] = fma(a[3], b[1], fma(a[1], b[3], acc[5]));
    acc[6] = fma(a[2], b[2], acc[6]);
    acc[7] = fma(a[3], b[2], fma(a[2], b[3], acc[7]));
    acc[8] = fma(a[3], b[3], acc[8]);
}
// pass 0: (D,D), (X,D), (Y,D); pass 1: (X,X), (X,Y), (Y,Y) -- 27 accumulators each
constexpr int BIL_PASSES = 2, BIL_PW = 27;
__device__ __forceinline__ void bern_ch(double acc[BIL_PW], int pass, const double f[4], double r, const double x[4],
                                        const double y[4]) {
    if (pass == 0) {
        const double d[4] = {f[0] - r, f[1] - r, f[2] - r, f[3] - r};  // exact for fp32 texels
        bern_sym(acc, d[0], d[1], d[2], d[3]);
        bern_asym(acc + 9, x, d);
        bern_asym(acc + 18, y, d);
    } else {
        bern_sym(acc, x[0], x[1], x[2], x[3]);
        bern_asym(acc + 9, x, y);
        bern_sym(acc + 18, y[0], y[1], y[2], y[3]);
    }
}
// Wave-reduce a pass's accumulators and store them into the point's memo column (groups
// 3 pass .. 3 pass + 2 of the order DD, XD, YD, XX, XY, YY; symmetric: DD, XX, YY).
__device__ __forceinline__ void bern_store(double acc[BIL_PW], int pass, double *mcol, int rs, int lane) {
    auto val = [&](int k) -> double { return k < BIL_PW ? acc[k] : 0.0; };
    const double tot = reduce32_in64(val, lane);
    const int idx = reduce32_index(lane);
    if ((lane & 1) == 0 && idx < BIL_PW) {
        const int g = 3 * pass + idx / 9, c = idx % 9;
        const bool sym = g == 0 || g == 3 || g == 5;
        const bool cross = c == 1 || c == 3 || c == 4 || c == 5 || c == 7;
        mcol[(size_t)(9 * g + c) * rs] = (sym && cross) ? 2.0 * tot : tot;
    }
}

// One point's 13 16-byte loads of a lane's channel round (four taps x f, gx, gy, and fref).
template <typename T>
struct BilLoad {
    typename V16<T>::type f[4], x[4], y[4], q;
};
template <typename T>
__device__ __forceinline__ void bil_issue(BilLoad<T> &g, const T *feat, const int o[4], const T *rf, int cs, int c) {
    using VT = typename V16<T>::type;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const T *t = feat + (size_t)o[k] * 3 * cs + c;
        g.f[k] = gload<VT>(t);
        g.x[k] = gload<VT>(t + cs);
        g.y[k] = gload<VT>(t + 2 * cs);
    }
    g.q = gload<VT>(rf + c);
}
template <typename T>
__device__ __forceinline__ void bil_acc(double acc[BIL_PW], int pass, const BilLoad<T> &g) {
    constexpr int V = V16<T>::n;
    const T *pq = reinterpret_cast<const T *>(&g.q);
#pragma unroll
    for (int e = 0; e < V; ++e) {
        double f[4], x[4], y[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            f[k] = (double)reinterpret_cast<const T *>(&g.f[k])[e];
            x[k] = (double)reinterpret_cast<const T *>(&g.x[k])[e];
            y[k] = (double)reinterpret_cast<const T *>(&g.y[k])[e];
        }
        bern_ch(acc, pass, f, (double)pq[e], x, y);
    }
}

// Both passes of one point from one loaded round (C <= 64 V: every lane's channels in one
// 16-byte round; lanes past the slice read the first vector and contribute zeros).
template <typename T>
__device__ __forceinline__ void bil_consume1(const BilLoad<T> &g, bool has, double *mcol, int rs, int lane) {
#pragma unroll
    for (int pass = 0; pass < BIL_PASSES; ++pass) {
        double acc[BIL_PW];
#pragma unroll
        for (int k = 0; k < BIL_PW; ++k) acc[k] = 0.0;
        bil_acc<T>(acc, pass, g);
        if (!has) {
#pragma unroll
            for (int k = 0; k < BIL_PW; ++k) acc[k] = 0.0;
        }
        bern_store(acc, pass, mcol, rs, lane);
    }
}

// This wave's share of the workgroup's changed cells: the points of bil_dirty[0..nb) in block
// and lane order, every nw-th one starting at rank w (balanced across the waves whatever the
// blocks' counts).  Scalar state only.
struct BilCursor {
    const unsigned long long *dirty;
    unsigned long long m;
    int b, nb, r, w, nwm;  // nwm = nwaves - 1 (a power of two minus one)
    __device__ __forceinline__ bool next(int &pb, int &pj) {
        while (true) {
            while (!m) {
                if (++b >= nb) return false;
                m = ufirst(dirty[b]);
            }
            const int j = __builtin_ctzll(m);
            m &= m - 1;
            if (((r++) & nwm) == w) {
                pb = b;
                pj = j;
                return true;
            }
        }
    }
};

// The memo columns of this wave's share of the changed cells: one point per trip, the whole
// wave on its channels; one-round slices keep the next point's loads in flight while the
// current one is reduced.
template <typename T>
__device__ __forceinline__ void bil_memo_build(BilCursor cur, const T *feat, const int *tex, const T *fref0,
                                               double *memo, int rs, bool vec, int cs, int cb, int ce, int ld, int Hf,
                                               int Wf) {
    constexpr int V = V16<T>::n;
    const int lane = threadIdx.x & 63;
    int pb, pj;
    if (vec && ce - cb <= 64 * V) {
        const int c0 = cb + lane * V;
        const bool has = c0 < ce;
        const int c = has ? c0 : cb;
        BilLoad<T> A, B;
        int ia = 0, ib = 0;
        auto issue = [&](BilLoad<T> &g, int &pi) {
            pi = pb * 64 + pj;
            int o[4];
            bil_cell_taps(ufirst(tex[pi]), Hf, Wf, o);
            bil_issue<T>(g, feat, o, fref0 + (size_t)pi * ld, cs, c);
        };
        if (!cur.next(pb, pj)) return;
        issue(A, ia);
        while (true) {
            const bool moreB = cur.next(pb, pj);
            if (moreB) issue(B, ib);
            bil_consume1<T>(A, has, memo + ia, rs, lane);
            if (!moreB) break;
            const bool moreA = cur.next(pb, pj);
            if (moreA) issue(A, ia);
            bil_consume1<T>(B, has, memo + ib, rs, lane);
            if (!moreA) break;
        }
        return;
    }
    while (cur.next(pb, pj)) {  // several rounds per lane, or unaligned slices: per pass, rounds in order
        const int pi = pb * 64 + pj;
        int o[4];
        bil_cell_taps(ufirst(tex[pi]), Hf, Wf, o);
        const T *rf = fref0 + (size_t)pi * ld;
        const T *t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) t[k] = feat + (size_t)o[k] * 3 * cs;
        for (int pass = 0; pass < BIL_PASSES; ++pass) {
            double acc[BIL_PW];
#pragma unroll
            for (int k = 0; k < BIL_PW; ++k) acc[k] = 0.0;
            if (vec) {
                for (int c = cb + lane * V; c < ce; c += 64 * V) {
                    BilLoad<T> g;
                    bil_issue<T>(g, feat, o, rf, cs, c);
                    bil_acc<T>(acc, pass, g);
                }
            } else {
                for (int c = cb + lane * V; c < ce; c += 64 * V) {
#pragma unroll 1
                    for (int e = 0; e < V; ++e) {
                        const int ch = c + e;
                        if (ch < ce) {
                            double f[4], x[4], y[4];
#pragma unroll
                            for (int k = 0; k < 4; ++k) {
                                f[k] = (double)t[k][ch];
                                x[k] = (double)t[k][cs + ch];
                                y[k] = (double)t[k][2 * cs + ch];
                            }
                            bern_ch(acc, pass, f, (double)rf[ch], x, y);
                        }
                    }
                }
            }
            bern_store(acc, pass, memo + pi, rs, lane);
        }
    }
}

// The six channel sums of a point at (ax, ay) from its memo column (lane per point).
__device__ __forceinline__ void bil_memo_sums(const double *mcol, int rs, double ax, double ay, double s[6]) {
    const double ux = 1.0 - ax, uy = 1.0 - ay;
    const double bx0 = ux * ux, bx1 = ax * ux, bx2 = ax * ax;
    const double by0 = uy * uy, by1 = ay * uy, by2 = ay * ay;
#pragma unroll
    for (int g = 0; g < 6; ++g) {
        const double *b = mcol + (size_t)9 * g * rs;
        const double t0 = fma(b[2 * rs], bx2, fma(b[rs], bx1, b[0] * bx0));
        const double t1 = fma(b[5 * rs], bx2, fma(b[4 * rs], bx1, b[3 * rs] * bx0));
        const double t2 = fma(b[8 * rs], bx2, fma(b[7 * rs], bx1, b[6 * rs] * bx0));
        s[g] = fma(t2, by2, fma(t1, by1, t0 * by0));
        __builtin_amdgcn_sched_barrier(0);  // nine LDS reads in flight at a time, not 54
    }
}

// Double-buffered pair gathers of one block: the next pair's loads are issued before this
// pair's channel sums are reduced (one exposed round trip per block, not one per pair).
// fref0: the block's first descriptor row; rd: where the records go.
template <typename T, bool FULL>
__device__ __forceinline__ void gather_pipe(unsigned long long m, int off, bool hi, int lane, const T *feat,
                                            const T *fref0, int cs, int ld, int gc1, int gc2, bool has1, bool has2,
                                            const RecDst &rd, bool wlane) {
    if (!m) return;
    GLoad<T> A, B;
    GPair pa = pick_pair(m, off, hi), pb;
    g_issue<T>(A, feat + (size_t)pa.to * 3 * cs, fref0 + (size_t)pa.j * ld, cs, gc1, gc2);
    while (true) {
        const bool moreB = m != 0;
        if (moreB) {
            pb = pick_pair(m, off, hi);
            g_issue<T>(B, feat + (size_t)pb.to * 3 * cs, fref0 + (size_t)pb.j * ld, cs, gc1, gc2);
        }
        {
            double v[8];
            g_consume<T, FULL>(A, has1, has2, v);
            const double r = reduce8_in32(v, lane);
            if (wlane && (!hi || pa.two)) rd.col(pa.j)[pa.j] = r;
        }
        if (!moreB) break;
        const bool moreA = m != 0;
        if (moreA) {
            pa = pick_pair(m, off, hi);
            g_issue<T>(A, feat + (size_t)pa.to * 3 * cs, fref0 + (size_t)pa.j * ld, cs, gc1, gc2);
        }
        {
            double v[8];
            g_consume<T, FULL>(B, has1, has2, v);
            const double r = reduce8_in32(v, lane);
            if (wlane && (!hi || pb.two)) rd.col(pb.j)[pb.j] = r;
        }
        if (!moreA) break;
    }
}

// ---------------------------------------------------------------------------
// FMPNP_LAYOUT_F: a dirty point's channel sums from the f plane alone.  The half-wave's
// point reads its texel's 3x3 neighbourhood (zero outside the map, or clamped with
// replicate padding) and forms gx, gy per channel in fp64 with the pack kernel's separable
// expression (sx_j = (a_j + 2 d_j) + g_j, sy_j = g_j - a_j; gx = sx_+ - sx_-,
// gy = (sy_- + 2 sy_0) + sy_+; a, d, g = rows above, at, below): exact for fp32 maps, i.e.
// the reference's fp64 Sobel of the hypercolumn (helpers/utils.py:81-104) without the fp32
// rounding the packed gradients carry.  Channel order and zero-filled second rounds as in
// gather_half, so the sums do not depend on where the point sits.
// ---------------------------------------------------------------------------
// One channel: the 3x3 values v (rows above / at / below x columns left / at / right),
// gradients by the separable form, then the six sums.
__device__ __forceinline__ void sobel_acc_v(double a[8], const double v[9], double r, bool norm) {
    const double sxm = (v[0] + 2.0 * v[3]) + v[6], sym = v[6] - v[0];
    const double sy0 = v[7] - v[1];
    const double sxp = (v[2] + 2.0 * v[5]) + v[8], syp = v[8] - v[2];
    double gx = sxp - sxm, gy = (sym + 2.0 * sy0) + syp;
    if (norm) {
        gx *= 0.125;
        gy *= 0.125;
    }
    acc6(a, v[4], r, gx, gy);
}

// Element e of the nine tap vectors (and of fref): zero = the lane's channel lies past the
// slice, mask = the point's neighbourhood is cut by the map edge (ok[k] false: a zero tap).
template <typename T>
__device__ __forceinline__ void sobel_acc(double a[8], const T *tap[9], int e, const T *pr, bool mask,
                                          const bool ok[9], bool norm, bool zero) {
    double v[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) v[k] = (zero || (mask && !ok[k])) ? 0.0 : (double)tap[k][e];
    sobel_acc_v(a, v, zero ? 0.0 : (double)pr[e], norm);
}
// One point per trip, the whole wave on its channels (lane l: channels cb + l V + r 64 V):
// the nine tap addresses and border masks are wave-uniform (scalar registers), ten 16-byte
// loads per lane per round.
template <typename T, bool MASK>
__device__ __forceinline__ void gather_f_point(const T *__restrict__ feat, const int o[9], const bool ok[9],
                                               const T *__restrict__ rf, int cs, int cb, int ce, int lane, bool vec,
                                               bool norm, double a[8]) {
    using VT = typename V16<T>::type;
    constexpr int V = V16<T>::n;
    if (vec) {
        for (int c = cb + lane * V; c < ce; c += 64 * V) {
            VT x[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) x[k] = gload<VT>(feat + (size_t)o[k] * cs + c);
            const VT qv = gload<VT>(rf + c);
            const T *t[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) t[k] = reinterpret_cast<const T *>(&x[k]);
#pragma unroll
            for (int e = 0; e < V; ++e) sobel_acc<T>(a, t, e, reinterpret_cast<const T *>(&qv), MASK, ok, norm, false);
        }
    } else {
        for (int c = cb + lane * V; c < ce; c += 64 * V) {
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const int ch = c + e;
                const bool in = ch < ce;
                const int chs = in ? ch : cb;
                const T *tap[9];
#pragma unroll
                for (int k = 0; k < 9; ++k) tap[k] = feat + (size_t)o[k] * cs + chs;
                sobel_acc<T>(a, tap, 0, rf + chs, MASK, ok, norm, !in);
            }
        }
    }
}

// One trip's state for the double-buffered form (one channel round, 16-byte loads): the
// point, its nine tap loads, fref, and its (wave-uniform) border masks.
template <typename T>
struct FTrip {
    typename V16<T>::type x[9], q;
    int p;
    bool ok[9], interior;
};

__device__ __forceinline__ void f_taps(int prc, int Hf, int Wf, bool rep, int o[9], bool ok[9], bool &interior) {
    const int row = prc >> 16, col = prc & 0xffff;
#pragma unroll
    for (int dr = 0; dr < 3; ++dr)
#pragma unroll
        for (int dc = 0; dc < 3; ++dc) {
            const int r = row + dr - 1, c = col + dc - 1;
            const int rr = min(max(r, 0), Hf - 1), cc = min(max(c, 0), Wf - 1);
            o[3 * dr + dc] = rr * Wf + cc;
            ok[3 * dr + dc] = rep || (r == rr && c == cc);
        }
    interior = rep || (row > 0 && row < Hf - 1 && col > 0 && col < Wf - 1);
}

template <typename T>
__device__ __forceinline__ void f_issue(FTrip<T> &tr, unsigned long long &m, int rc, const T *feat, const T *fref0,
                                        int cs, int ld, int c, int Hf, int Wf, bool rep) {
    using VT = typename V16<T>::type;
    tr.p = __builtin_ctzll(m);
    m &= m - 1;
    int o[9];
    f_taps(__builtin_amdgcn_readlane(rc, tr.p), Hf, Wf, rep, o, tr.ok, tr.interior);
#pragma unroll
    for (int k = 0; k < 9; ++k) tr.x[k] = gload<VT>(feat + (size_t)o[k] * cs + c);
    tr.q = gload<VT>(fref0 + (size_t)tr.p * ld + c);
}

template <typename T, bool FULL>
__device__ __forceinline__ void f_consume(const FTrip<T> &tr, bool has, bool norm, int lane, const RecDst &rd,
                                          bool wlane) {
    constexpr int V = V16<T>::n;
    double a[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = 0.0;
    const T *t[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) t[k] = reinterpret_cast<const T *>(&tr.x[k]);
    const T *pq = reinterpret_cast<const T *>(&tr.q);
    if (tr.interior) {
#pragma unroll
        for (int e = 0; e < V; ++e) sobel_acc<T>(a, t, e, pq, false, tr.ok, norm, !has);
    } else {
#pragma unroll
        for (int e = 0; e < V; ++e) sobel_acc<T>(a, t, e, pq, true, tr.ok, norm, !has);
    }
    double r = reduce8_in32(a, lane), r2 = r;
    swap32(r, r2);
    r = r + r2;
    if (wlane && lane < 32) rd.col(tr.p)[tr.p] = r;
}

// Double-buffered form for C <= 64 V with 16-byte loads (one channel round per lane): the
// next point's ten loads are in flight while this point's sums are formed and reduced.
// Same per-lane arithmetic as gather_f_point, so the records are identical.
template <typename T, bool FULL>
__device__ __forceinline__ void gather_f_pipe(unsigned long long m, int rc, int lane, const T *feat, const T *fref0,
                                              int cs, int cb, int ce, int ld, int Hf, int Wf, bool norm, bool rep,
                                              const RecDst &rd, bool wlane) {
    constexpr int V = V16<T>::n;
    if (!m) return;
    const int c0 = cb + lane * V;
    const bool has = c0 < ce;
    const int c = has ? c0 : cb;  // lanes past the slice read (and zero) the first vector
    FTrip<T> A, B;
    f_issue<T>(A, m, rc, feat, fref0, cs, ld, c, Hf, Wf, rep);
    while (true) {
        const bool moreB = m != 0;
        if (moreB) f_issue<T>(B, m, rc, feat, fref0, cs, ld, c, Hf, Wf, rep);
        f_consume<T, FULL>(A, has, norm, lane, rd, wlane);
        if (!moreB) break;
        const bool moreA = m != 0;
        if (moreA) f_issue<T>(A, m, rc, feat, fref0, cs, ld, c, Hf, Wf, rep);
        f_consume<T, FULL>(B, has, norm, lane, rd, wlane);
        if (!moreA) break;
    }
}

// Every dirty point of a block, one per trip; rc = (row << 16) | col of each lane's point.
template <typename T>
__device__ __forceinline__ void gather_f_block(unsigned long long m, int rc, bool hi, int lane, const T *feat,
                                               const T *fref0, int cs, int cb, int ce, int ld, int Hf, int Wf,
                                               bool vec, bool norm, bool rep, const RecDst &rd, bool wlane) {
    while (m) {
        const int p = __builtin_ctzll(m);
        m &= m - 1;
        const int prc = __builtin_amdgcn_readlane(rc, p);
        const int row = prc >> 16, col = prc & 0xffff;
        int o[9];
        bool ok[9];
#pragma unroll
        for (int dr = 0; dr < 3; ++dr)
#pragma unroll
            for (int dc = 0; dc < 3; ++dc) {
                const int r = row + dr - 1, c = col + dc - 1;
                const int rr = min(max(r, 0), Hf - 1), cc = min(max(c, 0), Wf - 1);
                o[3 * dr + dc] = rr * Wf + cc;
                ok[3 * dr + dc] = rep || (r == rr && c == cc);
            }
        const bool interior = rep || (row > 0 && row < Hf - 1 && col > 0 && col < Wf - 1);
        double v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = 0.0;
        const T *rf = fref0 + (size_t)p * ld;
        if (interior) gather_f_point<T, false>(feat, o, ok, rf, cs, cb, ce, lane, vec, norm, v);
        else gather_f_point<T, true>(feat, o, ok, rf, cs, cb, ce, lane, vec, norm, v);
        double r = reduce8_in32(v, lane), r2 = r;
        swap32(r, r2);  // the two halves hold the point's even / odd channel groups
        r = r + r2;
        if (wlane && !hi) rd.col(p)[p] = r;
    }
}

// ---------------------------------------------------------------------------
// The channel sums of the points of block `blk` set in the wave mask m, from the texels
// `off` (lane-wise; FL: rc = (row << 16) | col), into the record columns recb (this lane's
// field e6 at the block start: rec for the evaluation, rec2 for speculation).  Nearest
// sampling: packed f/gx/gy or, FL, the f-only layout with the in-gather Sobel.
// ---------------------------------------------------------------------------
template <typename T, bool PIPE, bool FL>
__device__ __forceinline__ void gather_records(const PC &q, unsigned long long m, int off, int rc, int blk,
                                               const RecDst &rd, bool wlane) {
    const int lane = threadIdx.x & 63, l32 = lane & 31;
    const bool hi = lane >= 32;
    const T *feat = reinterpret_cast<const T *>(q.feat);
    const T *fref = reinterpret_cast<const T *>(q.fref);
    const int cs = q.cs, cb = q.cb, ce = q.ce, p0 = q.p0, ld = q.ld;
    constexpr int V = V16<T>::n;
    const bool vec = ((((uintptr_t)feat) | ((uintptr_t)fref)) & 15) == 0 && cs % V == 0 && ld % V == 0 &&
                     cb % V == 0 && (ce - cb) % V == 0;
    const T *fref0 = fref + (size_t)(p0 + blk * 64) * ld;
    if constexpr (FL) {
        if (PIPE && vec && ce - cb <= 64 * V)  // one channel round per lane
            gather_f_pipe<T, true>(m, rc, lane, feat, fref0, cs, cb, ce, ld, q.Hf, q.Wf, q.sob_norm != 0,
                                   q.sob_rep != 0, rd, wlane);
        else
            gather_f_block<T>(m, rc, hi, lane, feat, fref0, cs, cb, ce, ld, q.Hf, q.Wf, vec, q.sob_norm != 0,
                              q.sob_rep != 0, rd, wlane);
    } else if (PIPE && vec && ce - cb <= 64 * V) {
        // one round trip per point (every channel within the lane's two rounds), double-buffered
        // pairs: the next pair's loads are issued before this pair's channel sums are reduced
        // (one exposed round trip per block, not one per pair)
        const int gc = cb + l32 * V;
        const bool has1 = gc < ce, has2 = gc + 32 * V < ce;
        const int gc1 = has1 ? gc : cb, gc2 = has2 ? gc + 32 * V : gc1;
        if (ce - cb == 64 * V)
            gather_pipe<T, true>(m, off, hi, lane, feat, fref0, cs, ld, gc1, gc2, has1, has2, rd, wlane);
        else
            gather_pipe<T, false>(m, off, hi, lane, feat, fref0, cs, ld, gc1, gc2, has1, has2, rd, wlane);
    } else {
        while (m) {  // wave-uniform: two dirty points per trip, one per half-wave
            const GPair pp = pick_pair(m, off, hi);
            const T *t = feat + (size_t)pp.to * 3 * cs;
            const T *rf = fref0 + (size_t)pp.j * ld;
            double v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = 0.0;
            if (vec) gather_half<T, true>(t, rf, cs, cb, ce, l32, v);
            else gather_half<T, false>(t, rf, cs, cb, ce, l32, v);
            const double r = reduce8_in32(v, lane);
            if (wlane && (!hi || pp.two)) rd.col(pp.j)[pp.j] = r;
        }
    }
}

// ---------------------------------------------------------------------------
// Speculative next-texel gathers.  A point changes texel (and needs a gather) only when its
// pixel crosses a texel edge, and -- measured over the reference's own LM trajectories at
// the BASELINE shapes (tools/sim_spec.py) -- a point that crosses in the next evaluation
// almost always lies closer to that edge, along each axis, than it moved in this one: the
// predicted texel is the neighbour across the near edge of every such axis (97 % of the
// next evaluation's dirty points, about two predictions per dirty point).  Waves 1..7 gather
// the predicted texels' sums into rec2 while wave 0 runs the LM tail (the gathers leave the
// evaluation's critical path); a dirty point whose new texel is rec2's takes its sums from
// there -- the same gather code, so bit-identical records -- and only the mispredicted ones
// are gathered in the evaluation itself.  Results do not depend on the predictions.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int spec_target(const PC &q, double qx, double qy, int row, int col, float *qpx,
                                           float *qpy) {
    const float fx = (float)qx, fy = (float)qy;
    const float mx = fabsf(fx - *qpx), my = fabsf(fy - *qpy);  // NaN before the first motion: none
    *qpx = fx;
    *qpy = fy;
    const Ctx &c = reinterpret_cast<const LMState *>(lm_lds)->c;  // (broadcast reads: not held in registers)
    const float sx = (fx - 0.5f) * c.txpx, sy = (fy - 0.5f) * c.typx;  // continuous texel coordinates
    const float ax = sx - floorf(sx), ay = sy - floorf(sy);
    const bool cx = fminf(ax, 1.0f - ax) * c.pxtx < mx, cy = fminf(ay, 1.0f - ay) * c.pypx < my;
    const int c2 = col + (cx ? (ax < 0.5f ? -1 : 1) : 0), r2 = row + (cy ? (ay < 0.5f ? -1 : 1) : 0);
    return ((cx || cy) && c2 >= 0 && c2 < q.Wf && r2 >= 0 && r2 < q.Hf) ? r2 * q.Wf + c2 : -1;
}

// The same prediction with its urgency: the smaller of (distance to the crossed edge) / motion over
// the predicted axes (< 1; smaller = the crossing is more likely), +inf without a prediction.
__device__ __forceinline__ int spec_target_u(const PC &q, double qx, double qy, int row, int col, float *qpx,
                                             float *qpy, float &urg) {
    const float fx = (float)qx, fy = (float)qy;
    const float mx = fabsf(fx - *qpx), my = fabsf(fy - *qpy);
    *qpx = fx;
    *qpy = fy;
    const Ctx &c = reinterpret_cast<const LMState *>(lm_lds)->c;
    const float sx = (fx - 0.5f) * c.txpx, sy = (fy - 0.5f) * c.typx;
    const float ax = sx - floorf(sx), ay = sy - floorf(sy);
    const float dx = fminf(ax, 1.0f - ax) * c.pxtx, dy = fminf(ay, 1.0f - ay) * c.pypx;
    const bool cx = dx < mx, cy = dy < my;
    const int c2 = col + (cx ? (ax < 0.5f ? -1 : 1) : 0), r2 = row + (cy ? (ay < 0.5f ? -1 : 1) : 0);
    const bool ok = (cx || cy) && c2 >= 0 && c2 < q.Wf && r2 >= 0 && r2 < q.Hf;
    urg = ok ? fminf(cx ? dx / mx : INFINITY, cy ? dy / my : INFINITY) : INFINITY;
    return ok ? r2 * q.Wf + c2 : -1;
}

// Every wave for its own blocks (wave 0 before the evaluation's barrier, in the slack it has
// while the later waves of its SIMDs finish; waves 1..7 after it, beside wave 0's LM tail):
// gather the predicted texels into each point's idle slot, which then holds tex2.
// At most `budget` gathers per call (q.spec_cap; 0 for wave 0's further blocks): a prediction
// left out is withdrawn (spec = -1), so the next evaluation gathers that point on demand if
// it does move there.
template <typename T, bool PIPE, bool FL>
__device__ __forceinline__ void spec_pass(const PC &q, int mmax, long long &ngath, int first_blk = -1,
                                          int budget = 1 << 30) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int *spec_w = lds_spec(mmax, true);
    const int *tex = lds_tex(mmax, true), *spec = spec_w, *slot = lds_slot(mmax, true);
    const int *tex2 = lds_tex2(mmax, true);
    double *rec = lds_rec(mmax), *rec2 = lds_rec2(mmax);
    const int rs = lds_rs(mmax);
    const int e6 = 4 * ((lane >> 4) & 1) + 2 * ((lane >> 3) & 1) + ((lane >> 2) & 1);
    const bool wlane = (lane & 3) == 0 && e6 < 6;
    const size_t fo = (size_t)(wlane ? e6 : 0) * rs;
    for (int blk = first_blk >= 0 ? first_blk : wave; blk * 64 < q.M; blk += nwaves()) {
        const int i = blk * 64 + lane;
        const bool valid = i < q.M;
        const int ii = valid ? i : 0;
        const int sp = valid ? spec[ii] : -1, cur = tex[ii], t2 = tex2[ii], sl = slot[ii];
        const bool want = sp >= 0 && sp != cur && sp != t2;
        unsigned long long m = __ballot(want);
        if (!m) continue;
        {
            unsigned long long kept = 0, mm = m;
            for (int k = 0; k < budget && mm; ++k) {
                kept |= mm & (~mm + 1);
                mm &= mm - 1;
            }
            budget -= __popcll(kept);
            if (valid && ((m & ~kept) >> lane) & 1ull) spec_w[i] = -1;  // not gathered: withdrawn
            m = kept;
            if (!m) continue;
        }
        ngath += __popcll(m);
        int rc = 0;
        if (FL && want) rc = ((sp / q.Wf) << 16) | (sp % q.Wf);
        const RecDst rd{rec + fo + blk * 64, rec2 + fo + blk * 64, __ballot(valid && sl != 0)};
        gather_records<T, PIPE, FL>(q, m, sp, rc, blk, rd, wlane);
        // (the idle slot's texel tag becomes spec at the next evaluation: see eval_pass)
    }
}

// ---------------------------------------------------------------------------
// One evaluation at (Re, te) over the wave's blocks (no workgroup barrier inside).
// Without the ratio test each block goes straight on to its chunk partials; with it the
// loss values are parked in the records and the wave's max |rho| is returned.
// PIPE: double-buffered gathers (latency variant: the VGPRs for two pairs in flight).
// SP: the variant can speculate (nearest sampling; bilinear never memoises).
// ---------------------------------------------------------------------------
// R1: the ratio test with a guessed limit (ratio_guess_check): the block partials are formed in
// this pass with the previous evaluation's limit, and each block's |rho| statistics are parked.
// WN: the packed-window check (the _W variants: a window on the packed f, gx, gy planes).
template <typename T, bool PIPE, bool FL, bool SP, bool HELP, bool R1 = false, bool WN = false>
__device__ __forceinline__ double eval_pass(const PC &q, int mmax, long long &ngath, const double pose[12]) {
    LMState &st = S();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool hi = lane >= 32;
    const double *X = lds_X(mmax);
    double *rec = lds_rec(mmax);
    int *tex = lds_tex(mmax, q.spec);
    const int rs = lds_rs(mmax);
    const T *feat = reinterpret_cast<const T *>(q.feat);
    const T *fref = reinterpret_cast<const T *>(q.fref);
    const int cs = q.cs, cb = q.cb, ce = q.ce, p0 = q.p0, ld = q.ld, M = q.M;
    constexpr int V = V16<T>::n;
    const bool vec = ((((uintptr_t)feat) | ((uintptr_t)fref)) & 15) == 0 && cs % V == 0 && ld % V == 0 &&
                     cb % V == 0 && (ce - cb) % V == 0;
    const bool defer = q.use_ratio != 0;
    // (the guessed-limit ratio test: one workgroup per problem of at most 8 blocks)
    const bool r1 = R1 && defer && q.M <= 8 * 64;
    const double rguess = r1 ? ufirst(st.rguess[q.cur_ev & 1]) : 0.0;
    // (a wave below spec_w0 keeps slot 0 and no predictions: the memoised path)
    const bool spec_on = SP && q.spec != 0 && wave >= q.spec_w0;
    int *tex2 = lds_tex2(mmax, true), *spec = lds_spec(mmax, true), *slot = lds_slot(mmax, true);
    float *qp = lds_qp(mmax, true);
    double *rec2 = lds_rec2(mmax);
    double *dst_g = q.part_g;
    if (q.G > 1) dst_g += (size_t)((ufirst((int)st.c.epoch) + 1) & 1) * q.nc_max * NV;
    // the pose evaluated (read by the caller with the loop's state, one LDS burst; kept in VGPRs:
    // moving it to SGPRs costs 24 v_readfirstlane and SGPR spills)
    double Re[9], te[3];
#pragma unroll
    for (int k = 0; k < 9; ++k) Re[k] = pose[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) te[k] = pose[9 + k];
    double lmax = -1.0;  // -1: nothing supported seen yet
    for (int blk = wave; blk * 64 < M; blk += nwaves()) {
        const int i = blk * 64 + lane;
        const bool valid = i < M;
        // projection (model.py:303-311) and indexing_ (model.py:88-89): floor(y*Hf/H),
        // floor(x*Wf/W) of the reference's fp64 expression equal the integer quotients
        // (exact products, a correctly rounded quotient of integers floors to the integer
        // quotient), computed here with invariant-multiplier division
        double Pc[3] = {0.0, 0.0, 1.0};
        int off = -1, rc = 0, pred = -1;
        Taps tp;
        // the point's coordinates and memo state in one burst of LDS reads (clamped index, no
        // per-lane branch: a single round trip before the projection; none depends on the pose)
        const int ii = valid ? i : 0;
        const double X0 = X[ii], X1 = X[rs + ii], X2 = X[2 * rs + ii];
        const int old_r = tex[ii];
        int t2 = -1, sl = 0, sp = -1;
        float qpx = 0.0f, qpy = 0.0f;
        if (SP) {  // (the speculating variants' arrays; unused below spec_w0)
            t2 = tex2[ii];
            sl = slot[ii];
            qpx = qp[ii];
            qpy = qp[mmax + ii];
            sp = spec[ii];
        }
        const int old = valid ? old_r : -1;
        if (spec_on) {
            // the last spec pass filled the idle slot with the predicted texel when it was
            // neither slot's (spec_pass / spec_pooled apply this same test)
            if (sp >= 0 && sp != old && sp != t2) t2 = sp;
        } else {
            t2 = -1;
            sl = 0;
        }
        double rzp = 1.0;  // recip(Pc[2]) of the point (the Jacobian chain's 1 / z)
        if (valid) {
            transform_pt(Re, te, X0, X1, X2, Pc);
            int x, y;
            double qx, qy;
            if (project_pc(q, Pc, x, y, qx, qy, rzp)) {
                const int row = (int)udiv((unsigned)y * (unsigned)q.Hf, q.dh);
                const int col = (int)udiv((unsigned)x * (unsigned)q.Wf, q.dw);
                off = row * q.Wf + col;
                if (FL) rc = (row << 16) | col;
                if (q.bilinear) bilinear_taps(qx, qy, q.Hf, q.Wf, q.im_w, q.im_h, tp);
                if (spec_on) {
                    pred = spec_target(q, qx, qy, row, col, &qpx, &qpy);
                    qp[i] = qpx;
                    qp[mmax + i] = qpy;
                }
            }
        }
        // memoised gather: a point whose texel did not change keeps its record (the six
        // channel sums depend only on the texel and the point's fixed descriptor)
        // (bilinear: the taps' weights move with the pose, every supported point is sampled)
        bool dirty = off >= 0 && (off != old || q.no_memo || q.bilinear);
        // with speculation a point has two record slots: a new texel that the idle slot holds
        // (predicted and gathered by spec_pass, or the texel the point just left) is a switch,
        // any other new texel is gathered into the idle slot and switched to
        const unsigned long long slot_b = __ballot(sl != 0);
        const bool moved = spec_on && dirty;
        if (moved) dirty = off != t2;
        if (spec_on) sl ^= moved ? 1 : 0;
        if (valid) {
            tex[i] = off;
            if (spec_on) {
                tex2[i] = moved ? old : t2;
                if (moved) slot[i] = sl;
                spec[i] = pred;
            }
        }
        unsigned long long m = __ballot(dirty);
        // packed windows (fmpnp_pack_features_f_window_batch; fmpnp_feature_pnp's windowed packs): every
        // texel gathered must be packed.  A miss marks the problem's result invalid (FMPNP_STATUS_WINDOW:
        // the caller packs in full and refines again).
        if constexpr (FL) {
            // the f-only layout: the texel's whole 3x3 neighbourhood (plane 1, st.c.win_ok); a miss is
            // never read and stops the problem after this evaluation (abort_flag, read only after
            // barriers: one workgroup per problem)
            const unsigned char *wok = ufirst(st.c.win_ok);
            if (wok != nullptr && m) {
                const bool miss = ((m >> lane) & 1ull) && wok[off] == 0;
                const unsigned long long mm = __ballot(miss);
                if (mm) {
                    m &= ~mm;  // (never read an unpacked texel)
                    if (lane == 0) {
                        st.win_miss = 1;
                        st.abort_flag = 1;
                    }
                }
            }
        } else if constexpr (WN) {
            // the packed f, gx, gy planes: the texel itself (plane 0, Hf * Wf bytes before plane 1).  A
            // miss is only flagged: the texel is read as usual (inside the full-size map, its bytes
            // stale) and the problem finishes, so a team's members never wait on a stopped one.  Only the
            // _W variants carry the check: compiled into the plain non-speculating variants it cost them up
            // to 6 % with no window at all (profiles/r05_window_check_fgrad_ab.txt), and 1 % of the
            // headline in the speculating ones (profiles/r05_window_check_ab.txt)
            const unsigned char *wok = ufirst(st.c.win_ok);
            if (wok != nullptr && m) {
                const bool miss = ((m >> lane) & 1ull) && wok[off - q.Hf * q.Wf] == 0;
                if (__ballot(miss) && lane == 0) st.win_miss = 1;
            }
        }
#if FMPNP_STAMPS
        if ((q.dbg & 128) && q.cur_ev > 0) m = 0;  // (diagnostics build, FMPNP_DBG bit 7: no gathers after eval 0 -- WRONG results, timing floor only)
#endif
        ngath += __popcll(m);
        if (HELP && q.hfirst && m) {
            // first evaluation with helpers: the block's records at the initial pose come from a
            // helper workgroup (the same gather code at the same pose: identical sums); a point
            // whose texel the helper saw differently, or a helper that never publishes, is
            // gathered here as usual
            // Hand-off (MI355X_MICROARCH.md, Workgroup dispatch: producer release + flag, consumer
            // relaxed poll + ONE agent-scope acquire): the helper stored its records, drained,
            // released (buffer_wbl2) and then stored this launch's tag; lane 0 polls the tag, and
            // after the match the wave acquires before any lane reads a record, so no read can see
            // bytes older than the tag -- in particular not an earlier launch's records left in a
            // reused workspace (the tag is launch-unique, the texel offset is checked as well).
            const unsigned long long *flag = q.hflag + (size_t)q.prob * q.nc_max + blk;
            int ok = 1;
            if (lane == 0) {
                // one bounded wait per workgroup: once any block's helper has timed out, the other
                // blocks gather themselves at once (so the whole problem waits at most 0.2 s)
                if (*reinterpret_cast<volatile int *>(&st.helper_absent)) ok = 0;
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                while (ok && __hip_atomic_load(reinterpret_cast<const g_u64 *>(reinterpret_cast<uintptr_t>(flag)),
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != q.htag) {
                    __builtin_amdgcn_s_sleep(1);
                    if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {  // 0.2 s
                        ok = 0;
                        *reinterpret_cast<volatile int *>(&st.helper_absent) = 1;
                    }
                }
                // a helper that never published (kept from being resident by other kernels): the
                // block is gathered here as usual; reported, results unaffected
                if (!ok) atomicOr(&st.sc[0].status, FMPNP_STATUS_HELPER_WAIT);  // (the first evaluation's state)
            }
            if (__builtin_amdgcn_readfirstlane(ok)) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every lane: no record read above the poll
                const double *hr = q.hrec + ((size_t)q.prob * q.nc_max * CH + i) * HREC;
                double hv[HREC];
#pragma unroll
                for (int e = 0; e < HREC; ++e) hv[e] = valid ? ld_sc1(hr + e) : -1.0;
                const bool use = dirty && hv[6] == (double)off;
                if (use) {
                    double *dst = (sl ? rec2 : rec) + i;  // the slot the point uses from now on
#pragma unroll
                    for (int e = 0; e < 6; ++e) dst[(size_t)e * rs] = hv[e];
                }
                m &= ~__ballot(use);
            }
        }
        dbg_stamp(q.stamps, 0);
        tl_stamp(q, 1);
        const int e6 = 4 * ((lane >> 4) & 1) + 2 * ((lane >> 3) & 1) + ((lane >> 2) & 1);
        const bool wlane = (lane & 3) == 0 && e6 < 6;
        const size_t fo = (size_t)(wlane ? e6 : 0) * rs + blk * 64;  // this lane's field column
        const RecDst rd{rec + fo, spec_on ? rec2 + fo : rec + fo, slot_b};
        if (!FL && q.bilinear) {
            gather_bil_block<T>(m, tp, hi, lane, feat, fref + (size_t)(p0 + blk * 64) * ld, cs, cb, ce, ld, vec,
                                rd, wlane);
        } else if (m) {
            gather_records<T, PIPE, FL>(q, m, off, rc, blk, rd, wlane);
        }
        // the records just written are read by other lanes of this wave: LDS operations of
        // a wave complete in order; the clobber keeps the compiler from reordering them
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        dbg_stamp(q.stamps, 1);
        tl_stamp(q, 2);
        const bool sup = off >= 0;
        const double *r = (sl ? rec2 : rec) + ii;  // the record slot in use
        double rho = 0.0, d1 = 0.0;
        if (sup) loss_eval(q.loss, q.alpha, 0.5 * r[0], rho, d1);
        if (defer) {
            if (valid) {
                rec[6 * rs + i] = rho;
                rec[7 * rs + i] = d1;
            }
            if (R1 && r1) {
                // the partials with the guessed limit, and the statistics that tell whether the
                // true limit keeps the same points (ratio_guess_check)
                const double a = fabs(rho);
                contrib_block_iz(q, mmax, blk, sup, sup && a < rguess, rho, d1, r, rs, Pc, rzp, dst_g);
                const double bmax = wave_nanmax(sup ? a : -1.0);
                if (lane == 0) st.rstat[blk] = bmax;
            } else if (sup) {
                lmax = nanmax(lmax, fabs(rho));
            }
        } else {
            contrib_block_iz(q, mmax, blk, sup, sup, rho, d1, r, rs, Pc, rzp, dst_g);
        }
        dbg_stamp(q.stamps, 2);
        tl_stamp(q, 3);
    }
    return lmax;
}

// One evaluation with bilinear sampling and the cell memo.  The workgroup holds at most four
// 64-point blocks (the memo's LDS; planner), so wave w < nb owns block w:
//   A  project its block (lane per point): cell key, (ax, ay), support; ballot the points
//      whose cell changed into bil_dirty[w];                                    -- barrier
//   B  every wave builds memo columns: waves w, w + nb, ... share block w mod nb's changed
//      points (interleaved lanes), one point per trip across the channels;      -- barrier
//   C  the owner evaluates its points' six sums from the memo, then loss and partials exactly
//      as eval_pass (rec fields 0..5 hold the sums).
// The memo columns and the reduction order depend only on the point, so results do not
// depend on G or on which wave builds a column.
template <typename T>
__device__ __forceinline__ double eval_pass_bil(const PC &q, int mmax, long long &ngath) {
    LMState &st = S();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const double *X = lds_X(mmax);
    double *rec = lds_rec(mmax);
    int *tex = lds_tex(mmax, false);
    double *memo = lds_memo(mmax, q.nc_max);
    const int rs = lds_rs(mmax);
    const T *feat = reinterpret_cast<const T *>(q.feat);
    const T *fref = reinterpret_cast<const T *>(q.fref);
    constexpr int V = V16<T>::n;
    const bool vec = ((((uintptr_t)feat) | ((uintptr_t)fref)) & 15) == 0 && q.cs % V == 0 && q.ld % V == 0 &&
                     q.cb % V == 0 && (q.ce - q.cb) % V == 0;
    double *dst_g = q.part_g;
    if (q.G > 1) dst_g += (size_t)((ufirst((int)st.c.epoch) + 1) & 1) * q.nc_max * NV;
    const int nb = (q.M + 63) >> 6;  // <= BIL_MAX_M / 64 <= nwaves()
    const bool own = wave < nb;
    const int i = wave * 64 + lane;
    const bool valid = own && i < q.M;
    double Pc[3] = {0.0, 0.0, 1.0};
    double ax = 0.0, ay = 0.0;
    int key = -1;
    if (own) {
        double Re[9], te[3];
        const double *pev = st.Ret[q.cur_ev & 1];
#pragma unroll
        for (int k = 0; k < 9; ++k) Re[k] = pev[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) te[k] = pev[9 + k];
        const int old = valid ? tex[i] : -1;
        if (valid) {
            transform_pt(Re, te, X[i], X[rs + i], X[2 * rs + i], Pc);
            int x, y;
            double qx, qy, rz_unused;
            if (project_pc(q, Pc, x, y, qx, qy, rz_unused)) {
                Taps tp;
                bilinear_taps(qx, qy, q.Hf, q.Wf, q.im_w, q.im_h, tp);
                key = tp.key;
                ax = tp.ax;
                ay = tp.ay;
            }
            tex[i] = key;
        }
        const unsigned long long m = __ballot(key >= 0 && key != old);
        ngath += __popcll(m);
        if (lane == 0) st.bil_dirty[wave] = m;
    }
    dbg_stamp(q.stamps, 0);
    __syncthreads();
    {
        // every wave takes every nwaves()-th changed cell of the workgroup (ranks in block order);
        // wave 0, which runs the LM tail after the barrier, takes the last residue
        const int nwm = nwaves() - 1;
        const BilCursor cur{st.bil_dirty, nb > 0 ? ufirst(st.bil_dirty[0]) : 0ull, 0, nb, 0, (wave + nwm) & nwm, nwm};
        bil_memo_build<T>(cur, feat, tex, fref + (size_t)q.p0 * q.ld, memo, rs, vec, q.cs, q.cb, q.ce, q.ld, q.Hf,
                          q.Wf);
    }
    dbg_stamp(q.stamps, 1);
    __syncthreads();
    double lmax = -1.0;
    if (own) {
        const bool sup = key >= 0;
        const int ii = valid ? i : 0;
        if (sup) {
            double s6[6];
            bil_memo_sums(memo + ii, rs, ax, ay, s6);
#pragma unroll
            for (int k = 0; k < 6; ++k) rec[k * rs + ii] = s6[k];
        }
        const double *r = rec + ii;
        double rho = 0.0, d1 = 0.0;
        if (sup) loss_eval(q.loss, q.alpha, 0.5 * r[0], rho, d1);
        if (q.use_ratio) {
            if (valid) {
                rec[6 * rs + i] = rho;
                rec[7 * rs + i] = d1;
            }
            if (sup) lmax = nanmax(lmax, fabs(rho));
        } else {
            contrib_block(q, mmax, wave, sup, sup, rho, d1, r, rs, Pc, dst_g);
        }
    }
    dbg_stamp(q.stamps, 2);
    return lmax;
}

// Second pass of the ratio test: the weights of points with |rho| >= max|rho| * thr
// are zero (model.py:324-336); P is recomputed bit-identically from X.
__device__ __forceinline__ void contrib_block_at(const PC &q, int mmax, int blk, double limit, const double Re[9],
                                                 const double te[3], double *dst_g) {
    const int lane = threadIdx.x & 63;
    const double *X = lds_X(mmax);
    const double *rec = lds_rec(mmax);
    const int *tex = lds_tex(mmax, q.spec);
    const int rs = lds_rs(mmax);
    const int i = blk * 64 + lane;
    const bool valid = i < q.M;
    const bool sup = valid && tex[i] >= 0;
    double Pc[3] = {0.0, 0.0, 1.0};
    if (sup) transform_pt(Re, te, X[i], X[rs + i], X[2 * rs + i], Pc);
    const int ii = valid ? i : 0;
    const double *r = rec + ii;  // rho, rho' (fields 6, 7: slot 0 only)
    const double *rs6 = (q.spec && lds_slot(mmax, true)[ii]) ? lds_rec2(mmax) + ii : r;  // the sums' slot
    const bool kept = sup && fabs(r[6 * rs]) < limit;
    contrib_block(q, mmax, blk, sup, kept, r[6 * rs], r[7 * rs], rs6, rs, Pc, dst_g);
}
__device__ __forceinline__ void contrib_pass(const PC &q, int mmax, double limit) {
    LMState &st = S();
    const int wave = threadIdx.x >> 6;
    double *dst_g = q.part_g;
    if (q.G > 1) dst_g += (size_t)((ufirst((int)st.c.epoch) + 1) & 1) * q.nc_max * NV;
    double Re[9], te[3];
    const double *pev = st.Ret[q.cur_ev & 1];
#pragma unroll
    for (int k = 0; k < 9; ++k) Re[k] = ufirst(pev[k]);
#pragma unroll
    for (int k = 0; k < 3; ++k) te[k] = ufirst(pev[9 + k]);
    for (int blk = wave; blk * 64 < q.M; blk += nwaves()) contrib_block_at(q, mmax, blk, limit, Re, te, dst_g);
}
__device__ __forceinline__ void contrib_pass_block(const PC &q, int mmax, int blk, double limit) {
    LMState &st = S();
    double *dst_g = q.part_g;
    if (q.G > 1) dst_g += (size_t)((ufirst((int)st.c.epoch) + 1) & 1) * q.nc_max * NV;
    double Re[9], te[3];
    const double *pev = st.Ret[q.cur_ev & 1];
#pragma unroll
    for (int k = 0; k < 9; ++k) Re[k] = ufirst(pev[k]);
#pragma unroll
    for (int k = 0; k < 3; ++k) te[k] = ufirst(pev[9 + k]);
    contrib_block_at(q, mmax, blk, limit, Re, te, dst_g);
}

// The guessed-limit ratio test (every wave, after barrier 1; one workgroup per problem, at most 8
// blocks: one per wave in the latency build, two in the throughput build's four waves).  The reference keeps a supported point iff |rho| < max|rho| * thr over
// every supported point (model.py:120-129, 324-336): known only once every block's loss is.
// eval_pass<R1> formed each block partial at once with the previous evaluation's limit g and parked
// each block's max|rho|.  Here every wave takes the true limit L from those maxima and checks the
// blocks it owns (eval_pass's blk = wave, wave + nwaves(), ...): where no supported point lies
// between g and L, the guess kept exactly the points L keeps and the block partial is the one
// contrib_pass would form (same points, same code, same bits); otherwise (a NaN |rho|, the first
// evaluation, a limit that crossed a point) the wave re-forms that block with L.  The caller's barrier then publishes the re-formed partials.  Returns L.
__device__ __forceinline__ double ratio_guess_check(const PC &q, int mmax, double guess, bool force,
                                                    long long &nredo) {
    LMState &st = S();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, M = q.M, nb = (M + 63) >> 6;
    double b = lane < nb ? st.rstat[lane] : -1.0;
    // (nb <= 8: lanes 0..7 of one row -- three DPP steps)
    b = nanmax(b, dpp64<DPP_XOR1>(b));
    b = nanmax(b, dpp64<DPP_XOR2>(b));
    b = nanmax(b, dpp64<DPP_MIRROR8>(b));
    const double limit = ufirst(b) * st.c.ratio_thr;
    for (int blk = wave; blk < nb; blk += nwaves()) {
        const int i = blk * 64 + lane;
        const bool valid = i < M;
        const int ii = valid ? i : 0;
        const double a = fabs(lds_rec(mmax)[6 * lds_rs(mmax) + ii]);
        const bool sup = valid && lds_tex(mmax, q.spec)[ii] >= 0;
        const bool miss = sup && ((a < limit) != (a < guess));  // (a NaN limit keeps nothing)
        if (__ballot(miss) || force) {
            ++nredo;
            contrib_pass_block(q, mmax, blk, limit);
        }
    }
    return limit;
}

// ---------------------------------------------------------------------------
// Combine on wave 0 (after the barrier / team exchange): the ordered sum over chunk
// (= block) indices.  Lane (j, h) (value j = lane & 31, half h = lane >> 5) sums chunks
// h, h+2, h+4, ... in order; the halves are then added.  Depends only on the chunk
// partials and NC -- not on G, placement or timing.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double combine_final_wave(int mmax, bool team, bool spec) {
    LMState &st = S();
    const Ctx &c = st.c;
    const int lane = lane_now(), j = lane & 31, h = lane >> 5;
    const int NC = c.NC;
    double t = 0.0;
    if (!team) {
        const double *src = lds_part(mmax, spec);
        double v[4];
        for (int r0 = h; r0 < NC; r0 += 8) {  // four loads in flight, adds in chunk order
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = r0 + 2 * u < NC ? src[(r0 + 2 * u) * NV + j] : 0.0;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (r0 + 2 * u < NC) t += v[u];
        }
    } else {
        const double *src = c.part_g + (size_t)(c.epoch & 1) * c.nc_max * NV;
        double v[4];
        for (int r0 = h; r0 < NC; r0 += 8) {
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = r0 + 2 * u < NC ? ld_sc1(src + (r0 + 2 * u) * NV + j) : 0.0;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (r0 + 2 * u < NC) t += v[u];
        }
    }
    double a = t, b = t;
    swap32(a, b);  // low half: (own, partner); high half: (partner, own)
    const double tot = a + b;  // even chunks + odd chunks, in both halves
    if (lane < NV) st.tot[threadIdx.x >> 6][lane] = tot;  // this tail wave's copy, for its solve's broadcast reads
    return tot;
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
        // reciprocal by v_rcp_f64 + one Newton step (~1 ulp; the solve is not bit-pinned to
        // the reference's LU anyway) instead of a full IEEE division on the critical path
        const double r0 = __builtin_amdgcn_rcp(a[j][j]);
        inv[j] = fma(fma(-a[j][j], r0, 1.0), r0, r0);
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
        for (int i = 5; i > j; --i) v = fma(-a[i][j], x[i], v);  // x[j + 1], the newest, last: one fma per step
        x[j] = v;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) delta[i] = -lr * x[i];
    return ok;
}

// ---------------------------------------------------------------------------
// LM state machine (model.py:300-486): the tail of evaluation k.  The evaluation's totals arrive
// lane-distributed (lane j holds value j, from the combine, which also stored them to the wave's
// st.tot row); the three the schedule needs are taken by v_readlane.
//
// The tail is the serial part of every evaluation (combine -> damped 6x6 solve -> pose update
// -> next evaluation), and one wave issues it alone on its SIMD.  With one workgroup per problem
// it is therefore split over three waves on three SIMDs, each of which combines the partials
// itself (same fixed order: identical totals) and takes the accept / reject decision itself:
//   role ACC   (wave 0) solves the evaluation's own normal equations with the accept branch's
//              damping (model.py:469-478: lambda / 10 clipped, lr = 1; the first evaluation
//              keeps lambda0) before the decision is known, and if the evaluation is accepted
//              (or is the first) steps from the evaluated pose and stores the next pose;
//   role REJ   (wave 1) solves the cached linearisation with the reject branch's damping
//              (lambda * 10, lr / 10, clipped) and steps from the current pose if it is rejected;
//   role BOOK  (wave 2) keeps the books: the schedule's scalars, best pose, the linearisation
//              cache, the current pose, the trace.
// The state before the evaluation is sc[k & 1] / Ret[k & 1] and the tail writes sc[(k+1) & 1] /
// Ret[(k+1) & 1], so no tail wave reads what another one writes.  Same operands and code as a
// decide-first tail: bit-identical steps.  Teams (G > 1, one polling wave) run every role on
// wave 0 (ROLE_ALL) with the decision first.
// ---------------------------------------------------------------------------
constexpr int ROLE_ACC = 1, ROLE_REJ = 2, ROLE_BOOK = 4, ROLE_ALL = 7;

struct Decision {
    double cost, lambda, lr;
    int kept, nsup;
    bool first, accepted, take, new_best, stop;  // stop: no step follows (cost mode, no support, last)
};

__device__ __forceinline__ Decision lm_decide(double tot, const LMScal &s, int mode, int n_iters) {
    Decision d;
    const double kept_d = rlane(tot, 28);
    d.nsup = (int)rlane(tot, 29);
    d.kept = (int)kept_d;
    d.cost = rlane(tot, 27) / kept_d;  // torch mean of an empty tensor = NaN
    d.first = s.n_evals == 0;
    d.lambda = s.lambda;
    d.lr = s.lr;
    d.accepted = true;
    if (!d.first) {  // model.py:469-478
        d.accepted = !(d.cost > s.prev);
        const double lam = d.lambda * (d.cost > s.prev ? 10.0 : 0.1);
        d.lambda = lam < 1e-6 ? 1e-6 : (lam > 1e4 ? 1e4 : lam);
        if (!d.accepted) {
            const double l2 = 0.1 * d.lr;
            d.lr = l2 < 1e-3 ? 1e-3 : (l2 > 1.0 ? 1.0 : l2);
        } else {
            d.lr = 1.0;
        }
    }
    // the evaluated pose becomes current and its normal equations the linearisation
    d.take = d.first || d.accepted;
    d.new_best = !d.first && d.accepted && d.cost < s.best;
    d.stop = mode == FMPNP_MODE_COMPUTE_COST || d.nsup == 0 || s.n_steps >= n_iters;
    return d;
}

// The books of evaluation k: sc[nxt] from sc[cur] and the decision, the best / current pose, the
// linearisation cache, the trace.  pe: this lane's element of the evaluated pose (lane < 12).
__device__ __forceinline__ void lm_book(const Decision &d, double tot, double pe, int cur, int mode) {
    LMState &st = S();
    const Ctx &c = st.c;
    const int lane = lane_now();
    const LMScal &s = st.sc[cur];
    LMScal &o = st.sc[cur ^ 1];
    if (mode == FMPNP_MODE_COMPUTE_COST) {
        if (lane == 0) {
            o = s;
            o.nan = 0;
            o.initial = d.nsup == 0 ? NAN : d.cost;
            if (d.nsup == 0) o.status |= FMPNP_STATUS_NO_SUPPORT;
            o.n_evals = 1;
            o.done = 1;
        }
        return;
    }
    if (d.nsup == 0) {  // model.py:316-320 / :441-445: return the current pose
        if (lane == 0) {
            o = s;
            o.nan = 0;
            o.status |= d.first ? FMPNP_STATUS_NO_SUPPORT : FMPNP_STATUS_NO_SUPPORT_TRIAL;
            o.ret_current = 1;
            o.done = 1;
        }
        return;
    }
    if (lane < 12) {
        if (d.new_best) st.Rbt[lane] = pe;
        if (d.take) st.Rt[lane] = pe;
    }
    if (d.take && lane < NV) st.hc[lane] = tot;
    if (lane == 0) {
        LMScal n = s;
        if (d.first) {  // model.py:347-359
            n.prev = n.best = n.initial = d.cost;
            n.best_inl = d.kept;
            n.has_best = 1;
        } else if (d.accepted) {  // model.py:477-486
            n.n_accepted++;
            if (d.new_best) {
                n.best_inl = d.kept;
                n.best = d.cost;
            }
            n.prev = d.cost;
        }
        n.lambda = d.lambda;
        n.lr = d.lr;
        n.n_evals = s.n_evals + 1;
        if (d.stop) n.done = 1;
        else n.n_steps = s.n_steps + 1;  // the step is taken (a NaN step counts, model.py:411-413)
        // (nan is the stepping wave's: never written here)
        o.lambda = n.lambda;
        o.lr = n.lr;
        o.prev = n.prev;
        o.best = n.best;
        o.initial = n.initial;
        o.best_inl = n.best_inl;
        o.n_evals = n.n_evals;
        o.n_steps = n.n_steps;
        o.n_accepted = n.n_accepted;
        o.status = n.status;
        o.done = n.done;
        o.has_best = n.has_best;
        o.ret_current = n.ret_current;
    }
    if (c.trace && c.s == 0 && s.n_evals < c.trace_stride) {
        fmpnp_trace_entry &e = c.trace[(size_t)c.p * c.trace_stride + s.n_evals];
        if (lane < 9) e.R[lane] = pe;
        else if (lane < 12) e.t[lane - 9] = pe;
        if (lane == 0) {
            e.cost = d.cost;
            e.lambda_after = d.lambda;
            e.lr_after = d.lr;
            e.n_supported = d.nsup;
            e.n_kept = d.kept;
            e.accepted = d.accepted ? 1 : 0;
        }
    }
}

// One step: delta from the damped system hs (21 + 6 doubles in LDS, already in Hu / gv when
// `solved` tells whether the LDL^T fast path succeeded), pose update from base, next pose stored.
__device__ __forceinline__ void lm_step_store(const double *hs, double delta[6], bool solved, double lambda,
                                              double lr, const double *base, int nxt) {
    LMState &st = S();
    const int lane = lane_now();
    // (the pivoted-LU fallback indexes H by lane: it reads the LDS copy, not a private array)
    if (!solved) lm_step_rows(hs, hs + 21, lambda, lr, delta);
    bool bad = false;
#pragma unroll
    for (int k = 0; k < 6; ++k) bad |= isnan(delta[k]);
    if (bad) {  // model.py:411-413
        if (lane == 0) st.sc[nxt].nan = 1;
        return;
    }
    double Rc[9], tc[3], Rn[9], tn[3];
#pragma unroll
    for (int k = 0; k < 9; ++k) Rc[k] = base[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) tc[k] = base[9 + k];
    pose_update(Rc, tc, delta, Rn, tn);
    double *o = st.Ret[nxt];
    if (lane == 0) {
        for (int k = 0; k < 9; ++k) o[k] = Rn[k];
        for (int k = 0; k < 3; ++k) o[9 + k] = tn[k];
    }
}

__device__ __forceinline__ double clip_lam(double l) { return l < 1e-6 ? 1e-6 : (l > 1e4 ? 1e4 : l); }
__device__ __forceinline__ double clip_lr(double l) { return l < 1e-3 ? 1e-3 : (l > 1.0 ? 1.0 : l); }

// One role (or all, ROLE_ALL) of the tail of evaluation k.  tot: this wave's combined totals.
__device__ __forceinline__ void lm_tail(int role, double tot, const PC &q, int k) {
    LMState &st = S();
    const Ctx &c = st.c;
    const int lane = lane_now();
    const int cur = k & 1, nxt = cur ^ 1;
    const int kk = lane < 12 ? lane : 0;
    const LMScal &s = st.sc[cur];
    const int mode = c.mode, n_iters = c.n_iters;
    const double *row = st.tot[threadIdx.x >> 6];  // this wave's totals, as stored by its combine
    if (role == ROLE_ALL) {
        const Decision d = lm_decide(tot, s, mode, n_iters);
        const double pe = st.Ret[cur][kk];
        lm_book(d, tot, pe, cur, mode);
        dbg_stamp(q.stamps, 5);  // LM bookkeeping
        tl_stamp(q, 7);
        if (d.stop) return;
        const double *hs = d.take ? row : st.hc;
        double Hu[21], gv[6], delta[6];
#pragma unroll
        for (int j = 0; j < 21; ++j) Hu[j] = hs[j];
#pragma unroll
        for (int j = 0; j < 6; ++j) gv[j] = hs[21 + j];
        const bool solved = ldlt_step(Hu, gv, d.lambda, d.lr, delta);
        dbg_stamp(q.stamps, 6);  // 6x6 solve
        tl_stamp(q, 8);
        lm_step_store(hs, delta, solved, d.lambda, d.lr, d.take ? st.Ret[cur] : st.Rt, nxt);
        return;
    }
    if (role == ROLE_BOOK) {
        const Decision d = lm_decide(tot, s, mode, n_iters);
        lm_book(d, tot, st.Ret[cur][kk], cur, mode);
        return;
    }
    // a stepper: its branch's operands and damping are known before the decision.  Everything it
    // reads from LDS -- the state, the step's base pose, the operands -- is read up front, so the
    // chain after the combine is the solve and the pose update with no LDS round trip between.
    const bool acc = role == ROLE_ACC;
    const LMScal sv = s;
    const bool first = sv.n_evals == 0;
    if (!acc && first) return;  // the first evaluation is always taken
    const double *basep = acc ? st.Ret[cur] : st.Rt;
    double base[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) base[j] = basep[j];
    const double *hs = acc ? row : st.hc;
    const double lam = acc ? (first ? sv.lambda : clip_lam(sv.lambda * 0.1)) : clip_lam(sv.lambda * 10.0);
    const double lr = acc ? (first ? sv.lr : 1.0) : clip_lr(0.1 * sv.lr);
    double Hu[21], gv[6], delta[6];
#pragma unroll
    for (int j = 0; j < 21; ++j) Hu[j] = hs[j];
#pragma unroll
    for (int j = 0; j < 6; ++j) gv[j] = hs[21 + j];
    tl_stamp(q, 12);  // (stamps build: the operands have arrived)
    const bool solved = ldlt_step(Hu, gv, lam, lr, delta);
    // (the step is formed here, not sunk past the decision's branch: the decision's instructions
    // then fill the solve's dependency stalls instead of adding to them)
    asm volatile("" ::"v"(delta[0]), "v"(delta[1]), "v"(delta[2]), "v"(delta[3]), "v"(delta[4]), "v"(delta[5]));
    tl_stamp(q, 13);
    const Decision d = lm_decide(tot, sv, mode, n_iters);
    tl_stamp(q, 14);
    if (d.stop || d.take != acc) return;
    tl_stamp(q, 8);
    lm_step_store(hs, delta, solved, lam, lr, base, nxt);
}

// ---------------------------------------------------------------------------
// First-evaluation helper workgroup: for its problem's blocks hb, hb + H, ... every wave
// projects the block at the initial pose and gathers the records of its eighth of the block's
// supported points (gather_records: the main workgroup's own code, so the sums are the ones
// it would form), then stores them with the texel offsets (write-through, drained) and, after
// the workgroup's barrier, publishes each block with the launch's tag (MI355X_MICROARCH.md, sc1
// hand-off).  No helper waits on anything.
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void helper_run(const LaunchArgs &a, int mmax) {
    LMState &st = S();
    const int h = (int)blockIdx.x - a.grid_main, p = h / a.helpers, hb = h % a.helpers;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    problem_begin(a.probs + p, p, mmax);
    PC q = load_pc();
    q.G = 1;
    q.spec = 0;
    q.helpers = q.hfirst = 0;
    const double *X = lds_X(mmax);
    double *rec = lds_rec(mmax);
    const int rs = lds_rs(mmax);
    double Re[9], te[3];
#pragma unroll
    for (int k = 0; k < 9; ++k) Re[k] = st.Ret[0][k];
#pragma unroll
    for (int k = 0; k < 3; ++k) te[k] = st.Ret[0][9 + k];
    double *out = a.hrec + (size_t)p * a.nc_max * CH * HREC;
    const int nw = nwaves(), per = 64 / nw;
    for (int blk = hb; blk * 64 < q.M; blk += a.helpers) {
        const int i = blk * 64 + lane;
        const bool valid = i < q.M;
        int off = -1;
        if (valid) {
            double Pc[3];
            transform_pt(Re, te, X[i], X[rs + i], X[2 * rs + i], Pc);
            int x, y;
            double qx, qy, rz_unused;
            if (project_pc(q, Pc, x, y, qx, qy, rz_unused)) {
                const int row = (int)udiv((unsigned)y * (unsigned)q.Hf, q.dh);
                const int col = (int)udiv((unsigned)x * (unsigned)q.Wf, q.dw);
                off = row * q.Wf + col;
            }
        }
        const bool mine = lane >= per * wave && lane < per * (wave + 1);
        const unsigned long long m = __ballot(off >= 0 && mine);
        const int e6 = 4 * ((lane >> 4) & 1) + 2 * ((lane >> 3) & 1) + ((lane >> 2) & 1);
        const bool wlane = (lane & 3) == 0 && e6 < 6;
        const size_t fo = (size_t)(wlane ? e6 : 0) * rs + blk * 64;
        const RecDst rd{rec + fo, rec + fo, 0ull};
        if (m) gather_records<T, true, false>(q, m, off, 0, blk, rd, wlane);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (valid && mine) {
            double *o = out + (size_t)i * HREC;
            for (int e = 0; e < 6; ++e) st_sc1(o + e, off >= 0 ? rec[(size_t)e * rs + i] : 0.0);
            st_sc1(o + 6, (double)off);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if (tid == 0 && !(a.dbg & 8)) {  // (debug bit 3: never publish -- the mains' bounded wait)
        // release the records before the tags (the explicit wait: the compiler may drop the one
        // after buffer_wbl2, MI355X_MICROARCH.md "Compiler hazard")
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int nb = (q.M + 63) / 64;
        for (int blk = hb; blk < nb; blk += a.helpers)
            __hip_atomic_store(reinterpret_cast<g_u64 *>(reinterpret_cast<uintptr_t>(a.hflag + (size_t)p * a.nc_max + blk)),
                               a.htag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------
// Specialised per launch (the launcher picks the variant): TEAM = G > 1, RATIO = the ratio
// test is on, VAR = VAR_GM (Geman-McClure forward, nearest sampling: the common case),
// VAR_NEAREST (any loss / mode, nearest) or VAR_BILINEAR -- constant-folding the other
// paths out shortens the per-point code and frees registers.
template <typename T, int WPS, bool TEAM, bool RATIO, int VAR>
__global__ __launch_bounds__(WPS == WPS_LATENCY ? NT : NT_THROUGHPUT,
                             WPS == WPS_WIDE ? 1 : 2) void lm_kernel(LaunchArgs a) {
    LMState &st = S();
    const int G = a.G;
    // XCD-aware team placement: members of one team share blockIdx % gw (the same XCD
    // under the observed round-robin dispatch; speed only, never correctness).
    const int b = blockIdx.x, gw = a.gw;
    const int grp = b / (gw * G), rem = b % (gw * G);
    const int s = rem / gw;
    // first-evaluation helpers (helper_run) after the main grid
    const bool helper = a.helpers > 0 && b >= a.grid_main;
    const int team = helper ? 0 : grp * gw + rem % gw;
    if (team >= a.teams) return;
    const int tid = threadIdx.x;
    // the _512 variants: the planner runs them only with a.mmax == 512, and their LDS carve is a
    // compile-time constant (immediate ds offsets, fewer scalar registers)
    constexpr bool kM512 = VAR == VAR_GM_SPEC_512 || VAR == VAR_GM_SPEC_H_512;
    const int mmax = kM512 ? MMAX_512 : a.mmax;
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
        c.no_memo = a.opt.no_memo == 1;  // 2: memoised without speculation (a.spec = 0)
        c.spec = a.spec;
        c.spec_cap = a.spec_cap;
        c.spec_w0 = a.spec_w0;
        c.dbg = a.dbg;
        c.sampling = a.opt.sampling;
        c.sobel_flags = a.opt.sobel_flags;
        c.stamps_on = a.stamps != nullptr && !(a.dbg & 20);  // dbg bit 2 / 4: per-evaluation stamps / timeline instead
        c.G = G;
        c.s = s;
        c.epoch = 0;
        c.dead = 0;
    }
    __syncthreads();
    // optional phase stamps (debug: a.stamps != null): s_memtime deltas on thread 0
    [[maybe_unused]] const bool stamps_on = kStamps && a.stamps != nullptr && !(a.dbg & 20);
    // debug (FMPNP_DBG bit 2): s_memtime at the start of every evaluation of the team's first
    // problem and after its last, [grid][64] in the stamps buffer
    unsigned long long *ev_stamps =
        (kStamps && a.stamps != nullptr && (a.dbg & 4)) ? a.stamps + (size_t)blockIdx.x * 64 : nullptr;
#if FMPNP_STAMPS
    if (stamps_on && (tid & 63) == 0) {
        for (int k = 0; k < NSTAMP; ++k) st.stamp_ph[tid >> 6][k] = 0;
        st.stamp_t[tid >> 6] = __builtin_amdgcn_s_memtime();
    }
#endif
    constexpr bool kHelp = WPS == WPS_LATENCY && !TEAM && (VAR == VAR_GM_SPEC_H || VAR == VAR_NEAREST_SPEC_H ||
                                                           VAR == VAR_GM_SPEC_H_512 ||
                                                           VAR == VAR_GM_H || VAR == VAR_NEAREST_H ||
                                                           VAR == VAR_GM_H_W || VAR == VAR_NEAREST_H_W);
    // the packed-window check (fmpnp_problem.window on the f, gx, gy planes)
    constexpr bool kWin = VAR == VAR_GM_W || VAR == VAR_NEAREST_W || VAR == VAR_GM_H_W || VAR == VAR_NEAREST_H_W;
    if (helper) {
        if constexpr (kHelp) helper_run<T>(a, mmax);
        return;
    }
    for (int p = team; p < a.n; p += a.teams) {
        problem_begin(a.probs + p, p, mmax);
        // speculation: the nearest-sampling variants of the latency build.  The planner runs a
        // _SPEC variant exactly when it enables speculation (memoised), so the flag is a constant
        // the ratio test with a guessed limit (ratio_guess_check): one workgroup per problem, nearest
        constexpr bool kRatio1 = RATIO && !TEAM && VAR != VAR_BILINEAR;
        constexpr bool kSpec = kSpecBuild && WPS == WPS_LATENCY &&
                               (VAR == VAR_GM_SPEC || VAR == VAR_NEAREST_SPEC || VAR == VAR_GM_SPEC_H ||
                                VAR == VAR_GM_SPEC_512 || VAR == VAR_GM_SPEC_H_512 ||
                                VAR == VAR_NEAREST_SPEC_H);
        // the problem's constants in registers (from the LDS Ctx), with this variant's constants
        auto make_q = [&]() {
            PC r = load_pc();
            r.helpers = kHelp ? a.helpers : 0;
            r.prob = p;
            r.hrec = a.hrec;
            r.hflag = a.hflag;
            r.htag = a.htag;
            r.tl = (kStamps && a.stamps != nullptr && (a.dbg & 16) && p == team) ? a.stamps + (size_t)blockIdx.x * 8 * 16
                                                                                 : nullptr;
            r.tl_eval = a.dbg >> 8;
            r.cur_eval = -1;
            if constexpr (!TEAM) {  // one workgroup: it owns every chunk (compile-time constants)
                r.G = 1;
                r.c0 = 0;
                r.p0 = 0;
            }
            r.use_ratio = RATIO ? 1 : 0;
            r.spec = kSpec ? 1 : 0;
            if constexpr (kSpec) r.no_memo = 0;
            if constexpr (VAR == VAR_GM || VAR == VAR_F_GM || VAR == VAR_GM_SPEC || VAR == VAR_GM_SPEC_H ||
                          VAR == VAR_GM_SPEC_512 || VAR == VAR_GM_SPEC_H_512 ||
                          VAR == VAR_GM_H || VAR == VAR_GM_W || VAR == VAR_GM_H_W)
                r.loss = FMPNP_GEMAN_MCCLURE;
            r.bilinear = (VAR == VAR_BILINEAR || VAR == VAR_BIL_DIRECT) ? 1 : 0;
            return r;
        };
        PC q = make_q();
        bool first_eval = true;
        long long ngath = 0;  // texel gathers of this wave for this problem
        int k = 0;  // evaluations completed: the next one reads sc[k & 1] and Ret[k & 1]
        while (true) {
            // the loop's state and the pose to evaluate, read together (one LDS round trip)
            double pose[12];
            {
                const double *pev = st.Ret[k & 1];
#pragma unroll
                for (int j = 0; j < 12; ++j) pose[j] = pev[j];
                const int2 dn = *reinterpret_cast<const int2 *>(&st.sc[k & 1].done);
                if ((dn.x | dn.y) != 0) break;
            }
            if (ev_stamps && tid == 0 && p == team && k < 63) ev_stamps[k] = __builtin_amdgcn_s_memtime();
            q.cur_ev = q.cur_eval = k;
            tl_stamp(q, 0);
            q.hfirst = first_eval && q.helpers > 0 && p == team;  // helpers serve each team's first problem
            first_eval = false;
            // project, gather, loss (+ partials)
            // (double-buffered gathers in both builds; speculation in the latency build only)
            // (bilinear: the cell memo; VAR_BIL_DIRECT samples every point at every evaluation)
            double lmax;
            if constexpr (VAR == VAR_BILINEAR)
                lmax = eval_pass_bil<T>(q, mmax, ngath);
            else
                lmax = eval_pass<T, true, (VAR == VAR_F_GM || VAR == VAR_F_NEAREST), kSpec, kHelp, kRatio1, kWin>(
                    q, mmax, ngath, pose);
            // the ratio test: with one workgroup per problem of at most 8 blocks, the guessed limit
            // (ratio_guess_check, after barrier 1); otherwise the two passes (exchange, contrib_pass)
            const bool r1 = kRatio1 && q.use_ratio && q.M <= 8 * 64;
            if (q.use_ratio && !r1) {
                if (!ratio_exchange(lmax)) break;
                const double limit = ufirst(st.rho_max) * st.c.ratio_thr;
                contrib_pass(q, mmax, limit);
            }
            const int wave = tid >> 6;
            constexpr bool FLV = VAR == VAR_F_GM || VAR == VAR_F_NEAREST;
            tl_stamp(q, 4);
            if (TEAM) team_arrive();
            else __syncthreads();
            if (r1) {
                // (FMPNP_DBG bit 5: every block re-formed -- the two-pass partials, for A/B tests;
                // bit 6: the re-formed blocks counted in texel_gathers' high word)
                long long nredo = 0;
                const double limit = ratio_guess_check(q, mmax, ufirst(st.rguess[k & 1]), (q.dbg & 32) != 0, nredo);
                if ((q.dbg & 64) && (tid & 63) == 0) ngath += nredo << 32;
                tl_stamp(q, 15);  // (stamps build: the guess checked)
                __syncthreads();  // (the re-formed partials)
                if (tid == 0) st.rguess[(k + 1) & 1] = isnan(limit) ? INFINITY : limit;  // evaluation k + 1's guess
            }
            tl_stamp(q, 5);
            // the tail (lm_tail): one workgroup per problem -- three waves, one role each; a team --
            // wave 0 after the exchange, every role
            if (TEAM) {
                if (wave == 0 && team_wait()) {
                    dbg_stamp(q.stamps, 3);  // slowest wave + exchange
                    const double tot = combine_final_wave(mmax, true, kSpec);
                    dbg_stamp(q.stamps, 4);
                    tl_stamp(q, 6);
                    lm_tail(ROLE_ALL, tot, q, k);
                    tl_stamp(q, 9);
                }
            } else if (wave < TAIL_ROLES) {
                dbg_stamp(q.stamps, 3);
                const double tot = combine_final_wave(mmax, false, kSpec);
                dbg_stamp(q.stamps, 4);
                tl_stamp(q, 6);
                lm_tail(wave == 0 ? ROLE_ACC : wave == 1 ? ROLE_REJ : ROLE_BOOK, tot, q, k);
                tl_stamp(q, 9);
            }
            // speculative gathers of the predicted next texels (spec_pass), while wave 0 finishes the
            // tail: each wave >= max(1, spec_w0) for its own blocks (default spec_w0 = 3: wave 3, idle
            // in the tail, and waves 4-7; waves 1 and 2 after their tail roles when spec_w0 <= 2), and
            // with spec_w0 = 0 wave 3 for wave 0's blocks too.  Their channel sums then leave the next
            // evaluation's point phase, which issue-bounds the SIMDs.
            if (kSpec && q.spec) {
                if (wave >= 1 && wave >= q.spec_w0) {
                    spec_pass<T, WPS == WPS_LATENCY, FLV>(q, mmax, ngath, -1, q.spec_cap);
                    dbg_stamp(q.stamps, 4);  // the speculative gathers
                }
                if (wave == 3 && q.spec_w0 == 0) spec_pass<T, WPS == WPS_LATENCY, FLV>(q, mmax, ngath, 0, q.spec_cap);
                tl_stamp(q, 10);
            }
            __syncthreads();
            tl_stamp(q, 11);
            dbg_stamp(q.stamps, 7);  // pose update + barrier
            if (st.abort_flag) break;
            ++k;
        }
        if (ev_stamps && tid == 0 && p == team && k < 64) ev_stamps[k] = __builtin_amdgcn_s_memtime();
        // texel gathers of the problem: a team's members add their waves' counts to the zeroed
        // result (G > 1); one workgroup sums its waves' counts in LDS and stores the total with
        // the other result fields (G = 1: the launch needs no memset)
        if (TEAM) {
            if ((tid & 63) == 0 && ngath)
                atomicAdd(reinterpret_cast<unsigned long long *>(&a.results[p].texel_gathers),
                          (unsigned long long)ngath);
        } else {
            if ((tid & 63) == 0) st.wg_gath[tid >> 6] = ngath;
            __syncthreads();
        }
        problem_end(!TEAM, k, q.tl, VAR == VAR_F_GM || VAR == VAR_F_NEAREST);
    }
#if FMPNP_STAMPS
    if (stamps_on && (tid & 63) == 0)
        for (int k = 0; k < NSTAMP; ++k)
            a.stamps[((size_t)blockIdx.x * (NT / 64) + (tid >> 6)) * NSTAMP + k] = st.stamp_ph[tid >> 6][k];
#endif
}

}  // namespace fmpnp
