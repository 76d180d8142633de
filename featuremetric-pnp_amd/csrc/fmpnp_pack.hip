// fmpnp_pack.hip -- feature preparation kernels (gfx950).
//
// pack_kernel: fused 3x3 Sobel + channels-last packing.  The reference casts the
// query hypercolumn [C][H][W] to fp64 on the host and runs kornia's Sobel
// (optimize_feature_pnp.py:57,61 -> helpers/utils.py:81-104); the LM loop then
// gathers one texel across C channels per point with C strided reads per map
// (model.py:74-97).  Here the map is streamed once from HBM and written as
// [H][W][3][C] (f, gx, gy interleaved per texel), so the LM kernel's gather of a
// point is three contiguous C-long runs.
//
// Two kernels: sobel_pack_kernel (gradients computed here; the performance path, see its
// comment below) and pack_kernel<GIVEN=true> (gradients supplied by the caller, as
// forward() receives them -- parity runs only).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <stdlib.h>

#include "fmpnp.h"
#include "fmpnp_internal.h"

namespace fmpnp {

constexpr int PK_NT = 256;   // threads per workgroup of the pack kernels
constexpr int PK_CB = 64;    // channels per tile
constexpr int PK_XW = 64;    // columns per tile
constexpr int PK_RS = 8;     // rows per tile
constexpr int PK_LD = 67;    // LDS row stride (odd -> no bank conflicts on column reads)

template <typename Tin>
__device__ __forceinline__ double ldin(const Tin *p) { return (double)*p; }

// Load input row y (all tile channels, columns x0-1 .. x0+XW) of `src` into ring slot.
template <typename Tin>
__device__ __forceinline__ void load_row(const Tin *__restrict__ src, int C, int H, int W, int c0, int x0, int y,
                                         int replicate, Tin *slot) {
    const int ncol = PK_XW + 2;
    int yy = y;
    bool row_ok = (y >= 0 && y < H);
    if (!row_ok && replicate) { yy = y < 0 ? 0 : H - 1; row_ok = true; }
    for (int e = threadIdx.x; e < PK_CB * ncol; e += PK_NT) {
        int cc = e / ncol, xx = e - cc * ncol;
        int c = c0 + cc, x = x0 - 1 + xx;
        Tin v = 0;
        if (c < C && row_ok) {
            int xs = x;
            bool col_ok = (x >= 0 && x < W);
            if (!col_ok && replicate) { xs = x < 0 ? 0 : W - 1; col_ok = true; }
            if (col_ok) v = src[((size_t)c * H + yy) * W + xs];
        }
        slot[cc * PK_LD + xx] = v;
    }
}

template <typename Tin, typename Tout, bool GIVEN>
__global__ __launch_bounds__(PK_NT) void pack_kernel(const Tin *__restrict__ chw, const Tin *__restrict__ gxc,
                                                  const Tin *__restrict__ gyc, int C, int H, int W,
                                                  Tout *__restrict__ out, int cs, int normalized, int replicate) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Tin *ring = reinterpret_cast<Tin *>(smem);  // [3][PK_CB][PK_LD]
    const int slot_elems = PK_CB * PK_LD;
    const int c0 = blockIdx.x * PK_CB, x0 = blockIdx.y * PK_XW, y0 = blockIdx.z * PK_RS;
    const int y1 = min(y0 + PK_RS, H);
    const int cc = threadIdx.x & 63, xg = threadIdx.x >> 6;
    const int c = c0 + cc;
    const double scale = normalized ? 0.125 : 1.0;  // kornia normalized=True divides by 8

    if (!GIVEN) {
        load_row<Tin>(chw, C, H, W, c0, x0, y0 - 1, replicate, ring + ((y0 - 1 + 3) % 3) * slot_elems);
        load_row<Tin>(chw, C, H, W, c0, x0, y0, replicate, ring + (y0 % 3) * slot_elems);
    }
    for (int y = y0; y < y1; ++y) {
        if (!GIVEN) {
            load_row<Tin>(chw, C, H, W, c0, x0, y + 1, replicate, ring + ((y + 1) % 3) * slot_elems);
        } else {
            load_row<Tin>(chw, C, H, W, c0, x0, y, 0, ring + 0 * slot_elems);
            load_row<Tin>(gxc, C, H, W, c0, x0, y, 0, ring + 1 * slot_elems);
            load_row<Tin>(gyc, C, H, W, c0, x0, y, 0, ring + 2 * slot_elems);
        }
        __syncthreads();
        if (c < C) {
            for (int xi = xg; xi < PK_XW; xi += PK_NT / 64) {
                const int x = x0 + xi;
                if (x >= W) break;
                double f, gx, gy;
                if (!GIVEN) {
                    const Tin *rm = ring + ((y + 2) % 3) * slot_elems + cc * PK_LD + xi;  // row y-1
                    const Tin *r0 = ring + (y % 3) * slot_elems + cc * PK_LD + xi;
                    const Tin *rp = ring + ((y + 1) % 3) * slot_elems + cc * PK_LD + xi;
                    double a = rm[0], b = rm[1], c2 = rm[2];
                    double d = r0[0], m = r0[1], e = r0[2];
                    double g = rp[0], h = rp[1], k = rp[2];
                    f = m;
                    // cross-correlation with kx = [[-1,0,1],[-2,0,2],[-1,0,1]], ky = kx^T
                    // (helpers/sobel_pytorch.py:9-59), same association as the oracle
                    gx = ((-a + c2) + (-2.0 * d + 2.0 * e)) + (-g + k);
                    gy = ((-a - 2.0 * b) - c2) + ((g + 2.0 * h) + k);
                    gx *= scale;
                    gy *= scale;
                } else {
                    f = ring[0 * slot_elems + cc * PK_LD + xi + 1];
                    gx = ring[1 * slot_elems + cc * PK_LD + xi + 1];
                    gy = ring[2 * slot_elems + cc * PK_LD + xi + 1];
                }
                Tout *o = out + ((size_t)y * W + x) * 3 * cs + c;
                o[0] = (Tout)f;
                o[cs] = (Tout)gx;
                o[2 * cs] = (Tout)gy;
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------
// sobel_pack_kernel: the Sobel path (gradients computed here), tuned for the HBM roofline.
//
// Tile: SB_CB channels x SB_XW columns x `rs` rows (host-chosen so that the grid is about one
// resident wave of workgroups: 4 per CU).  Input rows stream through a 4-slot LDS ring
// [slot][SB_CB][SB_LD] (odd row stride: the channel-per-lane reads and the 4-column
// transposing writes are both bank-conflict free); row y+3's global loads (16-byte vectors
// along x, 8 lanes per 128-B channel row) are in flight while row y is computed, so one
// barrier per row and no exposed load latency.  Compute: lane = channel, wave = a run of 8
// columns, a 3x3 register window slides along x (3 LDS reads per output texel), and each
// plane store is 64 consecutive channels = 256 contiguous bytes per wave instruction.
// HBM traffic per texel: 4C * (rs+2)/rs read + 12C written.
constexpr int SB_NT = 256;
constexpr int SB_CB = 64;                 // channels per tile (one per lane)
constexpr int SB_XW = 32;                 // columns per tile (4 waves x 8-column runs)
constexpr int SB_RUN = SB_XW / (SB_NT / 64);
constexpr int SB_LD = SB_XW + 5;          // 37: odd, >= XW + 2 halo columns
constexpr int SB_SLOTS = 4;

template <typename Tin>
struct SbRow {
    static constexpr int VE = 16 / sizeof(Tin);                 // elements per 16-B vector
    static constexpr int QPC = SB_XW / VE;                      // vectors per channel row
    static constexpr int UNITS = SB_CB * QPC / SB_NT;           // vectors per thread
    Tin v[UNITS][VE];
    Tin halo;
    unsigned okm;     // FAST loads: bit i = unit i lies inside the map, bit 31 = the halo does
};

template <typename Tin, bool FAST>
__device__ __forceinline__ void sb_load(SbRow<Tin> &r, const Tin *__restrict__ src, int C, int H, int W, int c0,
                                        int x0, int y, int replicate) {
    using R = SbRow<Tin>;
    const int t = threadIdx.x;
    int yy = y;
    bool row_ok = (y >= 0 && y < H);
    if (!row_ok && replicate) { yy = y < 0 ? 0 : H - 1; row_ok = true; }
    if constexpr (FAST) {
        // straight-line: every lane issues its loads from a clamped (valid) address and
        // zeroes what lies outside the map, so the loads are a fixed count the compiler's
        // vmcnt bookkeeping can see across the row loop (stores of the current row need not
        // drain before the prefetched row is used)
        const int ys = min(max(yy, 0), H - 1);
        unsigned okm = 0;
#pragma unroll
        for (int i = 0; i < R::UNITS; ++i) {
            const int u = t + SB_NT * i, cc = u / R::QPC, q = u - cc * R::QPC;
            const int c = c0 + cc;
            okm |= (c < C && row_ok) ? (1u << i) : 0u;
            const Tin *p = src + ((size_t)min(c, C - 1) * H + ys) * W + x0 + q * R::VE;
            if constexpr (sizeof(Tin) == 4) {
                const float4 w = *reinterpret_cast<const float4 *>(p);
                r.v[i][0] = w.x; r.v[i][1] = w.y; r.v[i][2] = w.z; r.v[i][3] = w.w;
            } else {
                const double2 w = *reinterpret_cast<const double2 *>(p);
                r.v[i][0] = w.x; r.v[i][1] = w.y;
            }
        }
        const int th = t & (2 * SB_CB - 1);  // threads >= 128 repeat a load and drop it
        const int cc = th >> 1, c = c0 + cc;
        int x = (th & 1) ? x0 + SB_XW : x0 - 1;
        bool ok = (x >= 0 && x < W);
        if (!ok && replicate) { x = x < 0 ? 0 : W - 1; ok = true; }
        r.halo = src[((size_t)min(c, C - 1) * H + ys) * W + min(max(x, 0), W - 1)];
        okm |= (t < 2 * SB_CB && ok && c < C && row_ok) ? (1u << 31) : 0u;
        r.okm = okm;  // the zeroing waits for sb_store: no use of the loaded values here
        return;
    }
#pragma unroll
    for (int i = 0; i < R::UNITS; ++i) {
        const int u = t + SB_NT * i, cc = u / R::QPC, q = u - cc * R::QPC;
        const int c = c0 + cc, xb = x0 + q * R::VE;
        const Tin *p = src + ((size_t)c * H + yy) * W + xb;
#pragma unroll
        for (int k = 0; k < R::VE; ++k) {
            int x = xb + k;
            Tin val = 0;
            if (c < C && row_ok) {
                if (x < W) val = p[k];
                else if (replicate) val = src[((size_t)c * H + yy) * W + (W - 1)];
            }
            r.v[i][k] = val;
        }
    }
    r.halo = 0;
    if (t < 2 * SB_CB) {
        const int cc = t >> 1, c = c0 + cc;
        int x = (t & 1) ? x0 + SB_XW : x0 - 1;
        bool ok = (x >= 0 && x < W);
        if (!ok && replicate) { x = x < 0 ? 0 : W - 1; ok = true; }
        if (c < C && row_ok && ok) r.halo = src[((size_t)c * H + yy) * W + x];
    }
    r.okm = ~0u;
}

template <typename Tin>
__device__ __forceinline__ void sb_store(const SbRow<Tin> &r, Tin *slot) {
    using R = SbRow<Tin>;
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < R::UNITS; ++i) {
        const int u = t + SB_NT * i, cc = u / R::QPC, q = u - cc * R::QPC;
        const bool ok = (r.okm >> i) & 1u;
#pragma unroll
        for (int k = 0; k < R::VE; ++k) slot[cc * SB_LD + 1 + q * R::VE + k] = ok ? r.v[i][k] : (Tin)0;
    }
    if (t < 2 * SB_CB) slot[(t >> 1) * SB_LD + ((t & 1) ? SB_XW + 1 : 0)] = (r.okm >> 31) ? r.halo : (Tin)0;
}

// Store one output element through the row-tile buffer descriptor: voffset is the lane's
// channel offset (fixed per row), soffset the texel/plane offset (wave-uniform SGPR).
template <typename Tout, bool NTS>
__device__ __forceinline__ void sb_put(Tout v, __amdgpu_buffer_rsrc_t rsrc, int voff, int soff) {
    constexpr int aux = NTS ? 2 : 0;  // nt: streamed once, do not keep in L2
    if constexpr (sizeof(Tout) == 4)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rsrc, voff, soff, aux);
    else
        {
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rsrc, voff, soff, aux);
    }
}

// FULL: the tile's 32 columns are all inside the map (no per-column bound check).
// NORM: kornia normalized=True (x 1/8).  Arithmetic is fp64 (fp32 maps: exact), rounded once.
//   Tin = float : separable form, column sums then differences (6 fp64 ops per texel); exact
//                 in fp64 for fp32 inputs, so the rounded result is the oracle's.
//   Tin = double: the oracle's association (helpers/sobel_pytorch.py:9-59 order), bit-equal.
// WIN: wmask bit k = column k of the wave's run is marked in the packed window (the others are not
// written: the LM never reads them, fmpnp_feature_pnp's windowed pack)
template <typename Tin, typename Tout, bool FULL, bool NORM, bool NTS, bool GRAD, bool WIN = false>
__device__ __forceinline__ void sb_row(const Tin *rm, const Tin *r0, const Tin *rp, __amdgpu_buffer_rsrc_t rsrc,
                                       int voff, int soff0, int tstride, int pstride, int ncols, unsigned wmask = 0) {
    constexpr double sc = NORM ? 0.125 : 1.0;
    if constexpr (sizeof(Tin) == 4) {
        // column j: sx_j = a_j + 2 d_j + g_j (for gx), sy_j = g_j - a_j (for gy)
        double am = rm[0], dm = r0[0], gm = rp[0];
        double a1 = rm[1], d1 = r0[1], g1 = rp[1];
        double sxm = (am + 2.0 * dm) + gm, sym = gm - am;
        double sx0 = (a1 + 2.0 * d1) + g1, sy0 = g1 - a1;
        double f0 = d1;
#pragma unroll
        for (int k = 0; k < SB_RUN; ++k) {
            const double a2 = rm[k + 2], d2 = r0[k + 2], g2 = rp[k + 2];
            const double sxp = (a2 + 2.0 * d2) + g2, syp = g2 - a2;
            const double gx = sxp - sxm, gy = (sym + 2.0 * sy0) + syp;
            if ((FULL || k < ncols) && (!WIN || ((wmask >> k) & 1u))) {
                const int so = soff0 + k * tstride;
                sb_put<Tout, NTS>((Tout)f0, rsrc, voff, so);
                if constexpr (GRAD) {
                    sb_put<Tout, NTS>((Tout)(NORM ? gx * sc : gx), rsrc, voff, so + pstride);
                    sb_put<Tout, NTS>((Tout)(NORM ? gy * sc : gy), rsrc, voff, so + 2 * pstride);
                }
            }
            sxm = sx0; sym = sy0; sx0 = sxp; sy0 = syp; f0 = d2;
        }
    } else {
        double a0 = rm[0], a1 = rm[1], d0 = r0[0], d1 = r0[1], g0 = rp[0], g1 = rp[1];
#pragma unroll
        for (int k = 0; k < SB_RUN; ++k) {
            const double a2 = rm[k + 2], d2 = r0[k + 2], g2 = rp[k + 2];
            // cross-correlation with kx = [[-1,0,1],[-2,0,2],[-1,0,1]], ky = kx^T, oracle order
            const double gx = ((-a0 + a2) + (-2.0 * d0 + 2.0 * d2)) + (-g0 + g2);
            const double gy = ((-a0 - 2.0 * a1) - a2) + ((g0 + 2.0 * g1) + g2);
            if ((FULL || k < ncols) && (!WIN || ((wmask >> k) & 1u))) {
                const int so = soff0 + k * tstride;
                sb_put<Tout, NTS>((Tout)d1, rsrc, voff, so);
                if constexpr (GRAD) {
                    sb_put<Tout, NTS>((Tout)(NORM ? gx * sc : gx), rsrc, voff, so + pstride);
                    sb_put<Tout, NTS>((Tout)(NORM ? gy * sc : gy), rsrc, voff, so + 2 * pstride);
                }
            }
            a0 = a1; a1 = a2; d0 = d1; d1 = d2; g0 = g1; g1 = g2;
        }
    }
}

// FAST: 16-B vector loads (aligned rows) and all 32 tile columns inside the map.
template <typename Tin, typename Tout, bool NORM, bool NTS, bool FAST, bool GRAD, bool WIN = false>
__device__ __forceinline__ void sobel_pack_body(const Tin *__restrict__ chw, int C, int H, int W, int cs, int rs,
                                                int replicate, Tin *ring, __amdgpu_buffer_rsrc_t rsrc, int c0, int x0,
                                                int y0, int dir, const unsigned char *__restrict__ win = nullptr) {
    constexpr int SE = SB_CB * SB_LD;
    const int y1 = min(y0 + rs, H);
    const int cc = threadIdx.x & 63, run = threadIdx.x >> 6;
    const int c = c0 + cc;
    const int wrun = __builtin_amdgcn_readfirstlane(run);  // wave-uniform: store offsets stay in SGPRs
    const int voff = (c < C ? c : 0) * (int)sizeof(Tout);
    const int tstride = (GRAD ? 3 : 1) * cs * (int)sizeof(Tout), pstride = cs * (int)sizeof(Tout);
    const int ncols = W - (x0 + wrun * SB_RUN);

    SbRow<Tin> r;
    // Row order: dir = +1 walks y0 -> y1-1, dir = -1 walks y1-1 -> y0.  Tiles alternate
    // direction by row block, so the two tiles sharing a halo row reach it at about the same
    // time (both at their start or both at their end) and the second read hits the XCD's L2
    // instead of HBM (same-direction order re-reads every halo row from HBM: +20 % reads).
    const int n = y1 - y0, ys = dir > 0 ? y0 : y1 - 1;
    sb_load<Tin, FAST>(r, chw, C, H, W, c0, x0, ys - dir, replicate);
    sb_store<Tin>(r, ring + ((ys - dir) & 3) * SE);
    sb_load<Tin, FAST>(r, chw, C, H, W, c0, x0, ys, replicate);
    sb_store<Tin>(r, ring + (ys & 3) * SE);
    sb_load<Tin, FAST>(r, chw, C, H, W, c0, x0, ys + dir, replicate);
    sb_store<Tin>(r, ring + ((ys + dir) & 3) * SE);
    // Row loop.  The next row's loads are issued BEFORE this row's stores: vmcnt retires in
    // issue order, so waiting for the loads then leaves this row's stores in flight (issued
    // after them the loads would wait for every store).  Lanes past C store to an
    // out-of-range voffset, which the buffer range check drops (no divergent branch).
    const int voff_s = FAST ? (c < C ? voff : 0x40000000) : voff;
    for (int k = 0; k < n; ++k) {
        const int y = ys + k * dir;
        __syncthreads();  // rows y-1, y, y+1 in their slots; slot (y+2dir)&3 is free
        const bool more = k + 2 <= n;
        if (more) sb_load<Tin, FAST>(r, chw, C, H, W, c0, x0, y + 2 * dir, replicate);
        if (FAST || c < C) {
            const int lo = cc * SB_LD + run * SB_RUN;
            const Tin *rm = ring + ((y - 1) & 3) * SE + lo;
            const Tin *r0 = ring + (y & 3) * SE + lo;
            const Tin *rp = ring + ((y + 1) & 3) * SE + lo;
            const int soff0 = ((y - y0) * W + x0 + wrun * SB_RUN) * tstride;
            unsigned wm = 0;
            if constexpr (WIN) {  // the run's marks (wave-uniform bytes)
                const unsigned char *wr = win + (size_t)y * W + x0 + wrun * SB_RUN;
#pragma unroll
                for (int k = 0; k < SB_RUN; ++k) wm |= (k < ncols && wr[k]) ? (1u << k) : 0u;
            }
            if (!WIN || wm)
                sb_row<Tin, Tout, FAST, NORM, NTS, GRAD, WIN>(rm, r0, rp, rsrc, voff_s, soff0, tstride, pstride, ncols,
                                                              wm);
        }
        if (more) sb_store<Tin>(r, ring + ((y + 2 * dir) & 3) * SE);
    }
}

template <typename Tin, typename Tout, bool NORM, bool NTS, bool GRAD, bool WIN = false>
__global__ __launch_bounds__(SB_NT) void sobel_pack_kernel(const Tin *__restrict__ chw, int C, int H, int W,
                                                        Tout *__restrict__ out, int cs, int rs, int replicate,
                                                        int vec_ok, int ncb, int nxw, int ntiles, int xcd_map,
                                                        int alt_dir, const unsigned char *__restrict__ win = nullptr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Tin *ring = reinterpret_cast<Tin *>(smem);  // [SB_SLOTS][SB_CB][SB_LD]
    // Tile order: channel chunk fastest, then column block, then row block.  xcd_map: the
    // dispatcher deals consecutive workgroups round-robin over the 8 XCDs, so workgroup b
    // takes tile (b % 8) * (grid / 8) + b / 8 -- each XCD gets one contiguous run of tiles
    // (all channel chunks of a texel and the row/column neighbours that share halos go
    // through the same L2).  The grid is padded to a multiple of 8; surplus groups exit.
    const int b = blockIdx.x;
    int t;
    if (xcd_map == 2) {  // spatial tiles dealt round-robin over XCDs, all channel chunks of one together
        const int j = b >> 3, s = (j / ncb) * 8 + (b & 7);
        t = s * ncb + j % ncb;
        if (s * ncb >= ntiles) return;
    } else {
        t = xcd_map ? (b & 7) * (int)(gridDim.x >> 3) + (b >> 3) : b;
        if (t >= ntiles) return;
    }
    const int cb = t % ncb, xb = (t / ncb) % nxw, yb = t / (ncb * nxw);
    const int c0 = cb * SB_CB, x0 = xb * SB_XW, y0 = yb * rs;
    const int dir = (alt_dir && (yb & 1)) ? -1 : 1;
    const int y1 = min(y0 + rs, H);
    if constexpr (WIN) {  // a tile without a marked texel: nothing read, nothing written
        int any = 0;
        for (int e = threadIdx.x; e < (y1 - y0) * SB_XW; e += SB_NT) {
            const int yy = y0 + e / SB_XW, xx = x0 + e % SB_XW;
            any |= (xx < W && win[(size_t)yy * W + xx]) ? 1 : 0;
        }
        if (!__syncthreads_or(any)) return;
    }
    // descriptor over this tile's output rows [y0, y1) x all columns (byte offsets < 2^31)
    const size_t texel_elems = (size_t)(GRAD ? 3 : 1) * cs;
    Tout *tile_base = out + (size_t)y0 * W * texel_elems;
    const unsigned tile_bytes = (unsigned)((size_t)(y1 - y0) * W * texel_elems * sizeof(Tout));
    __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(tile_base, 0, tile_bytes, 0x00020000);
    if (vec_ok && x0 + SB_XW <= W)
        sobel_pack_body<Tin, Tout, NORM, NTS, true, GRAD, WIN>(chw, C, H, W, cs, rs, replicate, ring, rsrc, c0, x0, y0,
                                                               dir, win);
    else
        sobel_pack_body<Tin, Tout, NORM, NTS, false, GRAD, WIN>(chw, C, H, W, cs, rs, replicate, ring, rsrc, c0, x0, y0,
                                                                dir, win);
}

template <typename Tin, typename Tout>
static hipError_t pack_t(const void *chw, const void *gx, const void *gy, int C, int H, int W, void *out, int cs,
                         int normalized, int replicate, bool grad, hipStream_t stream,
                         const unsigned char *win = nullptr) {
    if (gx) {
        dim3 grid((C + PK_CB - 1) / PK_CB, (W + PK_XW - 1) / PK_XW, (H + PK_RS - 1) / PK_RS);
        size_t lds = 3 * PK_CB * PK_LD * sizeof(Tin);
        hipLaunchKernelGGL((pack_kernel<Tin, Tout, true>), grid, dim3(PK_NT), lds, stream, (const Tin *)chw,
                           (const Tin *)gx, (const Tin *)gy, C, H, W, (Tout *)out, cs, normalized, replicate);
        return hipGetLastError();
    }
    // rows per workgroup: about one resident wave of workgroups (4 per CU on 256 CUs), >= 4 rows
    const int ncb = (C + SB_CB - 1) / SB_CB, nxw = (W + SB_XW - 1) / SB_XW;
    int nyb = 1024 / (ncb * nxw);
    if (nyb < 1) nyb = 1;
    int rs = (H + nyb - 1) / nyb;
    if (rs < 4) rs = 4;
    nyb = (H + rs - 1) / rs;
    const int vec_ok = ((uintptr_t)chw % 16 == 0) && ((size_t)W * sizeof(Tin)) % 16 == 0;
    const int ntiles = ncb * nxw * nyb;
    static const int xcd_map = [] { const char *e = getenv("FMPNP_PACK_XCD"); return e ? atoi(e) : 1; }();
    static const int alt_dir = [] { const char *e = getenv("FMPNP_PACK_ALT"); return e ? atoi(e) : 1; }();
    const int nsp = nxw * nyb;
    dim3 grid(xcd_map == 2 ? (nsp + 7) / 8 * 8 * ncb : xcd_map ? (ntiles + 7) / 8 * 8 : ntiles);
    size_t lds = (size_t)SB_SLOTS * SB_CB * SB_LD * sizeof(Tin);
    // the output descriptor of a workgroup spans its rs rows: byte offsets must stay below 2^31
    if ((size_t)rs * W * (grad ? 3 : 1) * cs * sizeof(Tout) >= ((size_t)1 << 31)) return hipErrorInvalidValue;
    // nt stores by default (the packed map is streamed out once; measured 2-17 % faster than
    // plain stores over cfg2..cfg5 shapes); FMPNP_PACK_NT=0 selects plain stores
    static const int nts = [] { const char *e = getenv("FMPNP_PACK_NT"); return !(e && *e == '0'); }();
    if (win) {  // windowed (fmpnp_feature_pnp): the marked texels only, nt stores
        if (!grad) return hipErrorInvalidValue;
        if (normalized)
            hipLaunchKernelGGL((sobel_pack_kernel<Tin, Tout, true, true, true, true>), grid, dim3(SB_NT), lds, stream,
                               (const Tin *)chw, C, H, W, (Tout *)out, cs, rs, replicate, vec_ok, ncb, nxw, ntiles,
                               xcd_map, alt_dir, win);
        else
            hipLaunchKernelGGL((sobel_pack_kernel<Tin, Tout, false, true, true, true>), grid, dim3(SB_NT), lds, stream,
                               (const Tin *)chw, C, H, W, (Tout *)out, cs, rs, replicate, vec_ok, ncb, nxw, ntiles,
                               xcd_map, alt_dir, win);
        return hipGetLastError();
    }
#define SB_LAUNCH(NORM, NTS, GRAD)                                                                              \
    hipLaunchKernelGGL((sobel_pack_kernel<Tin, Tout, NORM, NTS, GRAD>), grid, dim3(SB_NT), lds, stream,        \
                       (const Tin *)chw, C, H, W, (Tout *)out, cs, rs, replicate, vec_ok, ncb, nxw, ntiles, xcd_map, alt_dir)
    if (!grad) {  // FMPNP_LAYOUT_F: the channels-last f plane only (the LM kernel forms the gradients)
        if (nts) SB_LAUNCH(false, true, false); else SB_LAUNCH(false, false, false);
    } else if (normalized) {
        if (nts) SB_LAUNCH(true, true, true); else SB_LAUNCH(true, false, true);
    } else {
        if (nts) SB_LAUNCH(false, true, true); else SB_LAUNCH(false, false, true);
    }
#undef SB_LAUNCH
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// hwc_kernel: the FMPNP_LAYOUT_F pack -- a channels-last copy [C][H][W] -> [H][W][cstride]
// fp32, padding channels zero-filled.  A workgroup moves one tile of HC_CT channels x HC_XT
// columns of one row through LDS: 128-byte row segments in (8 lanes x 16 B per channel
// row), 512-byte texel segments out (32 lanes x 16 B of consecutive channels per column,
// nt stores), i.e. 8C bytes per texel of HBM traffic and no gradient work.
constexpr int HC_NT = 256;
// the once-read CHW rows of the f-only packs: nontemporal loads (end to end with windowed packs
// 33.7-33.9 k vs 33.2-33.5 k queries/s, profiles/r04_window_tiles.txt); -DFMPNP_PACK_NT_LOAD=0 for A/B
#ifndef FMPNP_PACK_NT_LOAD
#define FMPNP_PACK_NT_LOAD 1
#endif
constexpr bool kNtLoad = FMPNP_PACK_NT_LOAD != 0;
typedef float nf4 __attribute__((ext_vector_type(4)));

template <typename Tin, int HC_CT, int HC_XT>
__device__ __forceinline__ void hwc_tile(const Tin *__restrict__ chw, int C, int H, int W, float *__restrict__ out,
                                         int cs, int nct, int nxt, int vec_ok, int b, float *tile) {
    constexpr int HC_LD = HC_XT + 1;  // odd row stride of the [channel][column] LDS tile
    const int ct = b % nct;
    b /= nct;
    const int xt = b % nxt, y = b / nxt;
    const int c0 = ct * HC_CT, x0 = xt * HC_XT;
    const bool full_x = x0 + HC_XT <= W;
    constexpr int QPR = HC_XT / 4;  // 16-byte (4-column) units per channel row
    for (int i = threadIdx.x; i < HC_CT * QPR; i += HC_NT) {
        const int cc = i / QPR, q = i - cc * QPR;
        const int c = c0 + cc, x = x0 + 4 * q;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if (c < C) {
            const Tin *src = chw + ((size_t)c * H + y) * W + x;
            if (vec_ok && full_x) {
                if constexpr (sizeof(Tin) == 4) {
                    const nf4 w = kNtLoad ? __builtin_nontemporal_load(reinterpret_cast<const nf4 *>(src))
                                          : *reinterpret_cast<const nf4 *>(src);
                    v[0] = w.x; v[1] = w.y; v[2] = w.z; v[3] = w.w;
                } else {
                    const double2 w0 = *reinterpret_cast<const double2 *>(src);
                    const double2 w1 = *reinterpret_cast<const double2 *>(src + 2);
                    v[0] = (float)w0.x; v[1] = (float)w0.y; v[2] = (float)w1.x; v[3] = (float)w1.y;
                }
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (x + k < W) v[k] = (float)src[k];
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) tile[cc * HC_LD + 4 * q + k] = v[k];
    }
    __syncthreads();
    constexpr int QPC = HC_CT / 4;  // 16-byte (4-channel) units per column
    typedef float f4 __attribute__((ext_vector_type(4)));
    for (int i = threadIdx.x; i < HC_XT * QPC; i += HC_NT) {
        const int xx = i / QPC, cq = i - xx * QPC;
        const int x = x0 + xx, c = c0 + 4 * cq;
        if (x < W && c < cs) {
            f4 o;
            o.x = tile[(4 * cq + 0) * HC_LD + xx];
            o.y = tile[(4 * cq + 1) * HC_LD + xx];
            o.z = tile[(4 * cq + 2) * HC_LD + xx];
            o.w = tile[(4 * cq + 3) * HC_LD + xx];
            __builtin_nontemporal_store(o, reinterpret_cast<f4 *>(out + ((size_t)y * W + x) * cs + c));
        }
    }
}

template <typename Tin, int HC_CT, int HC_XT>
__global__ __launch_bounds__(HC_NT) void hwc_kernel(const Tin *__restrict__ chw, int C, int H, int W,
                                                  float *__restrict__ out, int cs, int nct, int nxt, int vec_ok) {
    __shared__ float tile[HC_CT * (HC_XT + 1)];
    hwc_tile<Tin, HC_CT, HC_XT>(chw, C, H, W, out, cs, nct, nxt, vec_ok, blockIdx.x, tile);
}

// Many maps in one launch (fmpnp_pack_features_batch, FMPNP_LAYOUT_F): the item table in the
// kernel arguments, workgroup b takes tile b - start[i] of the item i whose range holds b --
// one grid for the batch instead of one ramp-up and tail per map.
constexpr int HB_MAX = 32;
struct HwcItems {
    const void *chw[HB_MAX];
    float *out[HB_MAX];
    int C[HB_MAX], H[HB_MAX], W[HB_MAX], cs[HB_MAX], nct[HB_MAX], nxt[HB_MAX], vec[HB_MAX];
    int start[HB_MAX + 1];
    int n;
};

template <typename Tin, int HC_CT, int HC_XT>
__global__ __launch_bounds__(HC_NT) void hwc_batch_kernel(HwcItems it) {
    __shared__ float tile[HC_CT * (HC_XT + 1)];
    const int b = blockIdx.x;
    int lo = 0, hi = it.n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (it.start[mid] <= b) lo = mid;
        else hi = mid - 1;
    }
    hwc_tile<Tin, HC_CT, HC_XT>(reinterpret_cast<const Tin *>(it.chw[lo]), it.C[lo], it.H[lo], it.W[lo], it.out[lo],
                                it.cs[lo], it.nct[lo], it.nxt[lo], it.vec[lo], b - it.start[lo], tile);
}

template <typename Tin, int CT, int XT>
static hipError_t hwc_ct(const void *chw, int C, int H, int W, void *out, int cs, hipStream_t stream) {
    const int nct = (cs + CT - 1) / CT, nxt = (W + XT - 1) / XT;
    const long grid = (long)nct * nxt * H;
    if (grid >= (1L << 31) || cs % 4 != 0 || ((uintptr_t)out % 16) != 0) return hipErrorInvalidValue;
    const int vec_ok = ((uintptr_t)chw % 16 == 0) && ((size_t)W * sizeof(Tin)) % 16 == 0;
    hipLaunchKernelGGL((hwc_kernel<Tin, CT, XT>), dim3((unsigned)grid), dim3(HC_NT), 0, stream, (const Tin *)chw, C, H,
                       W, (float *)out, cs, nct, nxt, vec_ok);
    return hipGetLastError();
}

template <typename Tin>
static hipError_t hwc_t(const void *chw, int C, int H, int W, void *out, int cs, hipStream_t stream) {
    static const int ct = [] { const char *e = getenv("FMPNP_PACK_F_CT"); return e ? atoi(e) : 64; }();
    static const int xt = [] { const char *e = getenv("FMPNP_PACK_F_XT"); return e ? atoi(e) : 32; }();
    if (xt == 64) return ct == 128 ? hwc_ct<Tin, 128, 64>(chw, C, H, W, out, cs, stream)
                                   : hwc_ct<Tin, 64, 64>(chw, C, H, W, out, cs, stream);
    if (ct == 128) return hwc_ct<Tin, 128, 32>(chw, C, H, W, out, cs, stream);
    return hwc_ct<Tin, 64, 32>(chw, C, H, W, out, cs, stream);
}

template <typename Tin, int CT, int XT>
static hipError_t hwc_batch_t(const HwcItems &it, int total, hipStream_t stream) {
    hipLaunchKernelGGL((hwc_batch_kernel<Tin, CT, XT>), dim3((unsigned)total), dim3(HC_NT), 0, stream, it);
    return hipGetLastError();
}

template <int CT, int XT>
static hipError_t pack_f_batch_tiles(int n, const void *const *chw, void *const *out, const int *shape,
                                     int dtype_in, hipStream_t stream) {
    for (int i0 = 0; i0 < n; i0 += HB_MAX) {
        HwcItems it{};
        const int m = n - i0 < HB_MAX ? n - i0 : HB_MAX;
        long total = 0;
        for (int j = 0; j < m; ++j) {
            const int *sh = shape + 4 * (i0 + j);
            const int C = sh[0], H = sh[1], W = sh[2], cs = sh[3];
            if (cs % 4 != 0 || ((uintptr_t)out[i0 + j] % 16) != 0) return hipErrorInvalidValue;
            it.chw[j] = chw[i0 + j];
            it.out[j] = reinterpret_cast<float *>(out[i0 + j]);
            it.C[j] = C; it.H[j] = H; it.W[j] = W; it.cs[j] = cs;
            it.nct[j] = (cs + CT - 1) / CT;
            it.nxt[j] = (W + XT - 1) / XT;
            const size_t es = dtype_in == FMPNP_F64 ? 8 : 4;
            it.vec[j] = ((uintptr_t)chw[i0 + j] % 16 == 0) && ((size_t)W * es) % 16 == 0;
            it.start[j] = (int)total;
            total += (long)it.nct[j] * it.nxt[j] * H;
            if (total >= (1L << 31)) return hipErrorInvalidValue;
        }
        it.start[m] = (int)total;
        it.n = m;
        const hipError_t e = dtype_in == FMPNP_F32 ? hwc_batch_t<float, CT, XT>(it, (int)total, stream)
                                                   : hwc_batch_t<double, CT, XT>(it, (int)total, stream);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_pack_f_batch(int n, const void *const *chw, void *const *out, const int *shape, int dtype_in,
                               hipStream_t stream) {
    // tile (channels x columns), FMPNP_PACK_F_BTILE: 1: 64 x 64 (default), 0: 64 x 32 (end to end with
    // the full pack: 25.2 k vs 24.2 k queries/s, profiles/r04_window_tiles.txt)
    static const int tile = [] { const char *e = getenv("FMPNP_PACK_F_BTILE"); return e ? atoi(e) : 1; }();
    return tile == 1 ? pack_f_batch_tiles<64, 64>(n, chw, out, shape, dtype_in, stream)
                     : pack_f_batch_tiles<64, 32>(n, chw, out, shape, dtype_in, stream);
}

// ---------------------------------------------------------------------------------------
// Windowed f-only pack (fmpnp_pack_features_f_window_batch).  The refinement reads only the
// 3x3 neighbourhoods of the texels its points visit, a few texels from where they start, so
// three kernels replace the full copy:
//   win_clear_kernel  zero both planes of every problem's window map ([2][Hf][Wf] bytes);
//   win_mark_kernel   one thread per point: its texel at (R0, t0) (the LM's projection and
//                     indexing_, fmpnp_lm_impl.h project_pc) -> plane 0 over the square of
//                     radius r, plane 1 over radius r - 1 (texels whose 3x3 neighbourhood is packed);
//   hwc_win_kernel    hwc_tile's 64-channel x 32-column tiles, skipping a tile whose 32 texels are
//                     all unmarked (its 128-byte channel rows are never read) and storing only
//                     the marked texels.
// A point whose projection differs in rounding from the LM's lands at most one texel off: the
// LM checks plane 1 itself at every gather, so a miss is caught there (FMPNP_STATUS_WINDOW).
__global__ __launch_bounds__(PK_NT) void win_clear_kernel(const fmpnp_problem *__restrict__ pd) {
    const fmpnp_problem &p = pd[blockIdx.y];
    const long nb = 2L * p.Hf * p.Wf;
    unsigned char *w = const_cast<unsigned char *>(p.window);
    const long n16 = ((uintptr_t)w % 16) == 0 ? nb / 16 : 0;  // 16-byte stores, then the tail bytes
    for (long e = (long)blockIdx.x * PK_NT + threadIdx.x; e < n16; e += (long)gridDim.x * PK_NT)
        reinterpret_cast<uint4 *>(w)[e] = make_uint4(0u, 0u, 0u, 0u);
    for (long e = 16 * n16 + (long)blockIdx.x * PK_NT + threadIdx.x; e < nb; e += (long)gridDim.x * PK_NT) w[e] = 0;
}

// one thread per (point, window row): 2r + 1 rows of the point's square (a thread per point with
// (2r + 1)^2 serial stores left most CUs idle: 67 us per 64-query batch)
__global__ __launch_bounds__(PK_NT) void win_mark_kernel(const fmpnp_problem *__restrict__ pd, int r) {
    const fmpnp_problem &p = pd[blockIdx.y];
    const int e = blockIdx.x * PK_NT + threadIdx.x, span = 2 * r + 1;
    const int i = e / span, dy = e - i * span - r;
    if (i >= p.N) return;
    const double *X = p.pts3d + 3 * (size_t)i;
    double P[3];
    for (int a = 0; a < 3; ++a) P[a] = p.R0[3 * a] * X[0] + p.R0[3 * a + 1] * X[1] + p.R0[3 * a + 2] * X[2] + p.t0[a];
    const double u0 = p.K[0] * P[0] + p.K[1] * P[1] + p.K[2] * P[2];
    const double u1 = p.K[3] * P[0] + p.K[4] * P[1] + p.K[5] * P[2];
    const double u2 = p.K[6] * P[0] + p.K[7] * P[1] + p.K[8] * P[2];
    const double px = rint(u0 / u2) - 1.0, py = rint(u1 / u2) - 1.0;
    if (!(px >= 0.0 && px < (double)p.im_width && py >= 0.0 && py < (double)p.im_height)) return;
    const int row = (int)(((unsigned long long)py * (unsigned)p.Hf) / (unsigned)p.im_height);
    const int col = (int)(((unsigned long long)px * (unsigned)p.Wf) / (unsigned)p.im_width);
    unsigned char *w0 = const_cast<unsigned char *>(p.window), *w1 = w0 + (size_t)p.Hf * p.Wf;
    const int y = row + dy;
    if (y < 0 || y >= p.Hf) return;
    for (int x = max(col - r, 0); x <= min(col + r, p.Wf - 1); ++x) {
        w0[(size_t)y * p.Wf + x] = 1;
        if (abs(dy) < r && abs(x - col) < r) w1[(size_t)y * p.Wf + x] = 1;
    }
}

constexpr int WB_MAX = 64;  // maps per windowed-pack launch (a pipeline batch of 64 queries in one grid)
struct WinItems {
    const void *chw[WB_MAX];
    int start[WB_MAX + 1];
    int nct[WB_MAX], nxt[WB_MAX], vec[WB_MAX];
    int n;
    const fmpnp_problem *pd;  // the items' device descriptors (feat, window, sizes)
};

template <typename Tin, int HC_CT, int HC_XT>
__global__ __launch_bounds__(HC_NT) void hwc_win_kernel(WinItems it) {
    constexpr int HC_LD = HC_XT + 1;
    __shared__ float tile[HC_CT * HC_LD];
    __shared__ int flag[HC_XT];
    int b = blockIdx.x;
    int lo = 0, hi = it.n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (it.start[mid] <= b) lo = mid;
        else hi = mid - 1;
    }
    const fmpnp_problem &p = it.pd[lo];
    const Tin *chw = reinterpret_cast<const Tin *>(it.chw[lo]);
    const int C = p.c_end, H = p.Hf, W = p.Wf, cs = p.cstride, nct = it.nct[lo], nxt = it.nxt[lo];
    float *out = reinterpret_cast<float *>(const_cast<void *>(p.feat));
    b -= it.start[lo];
    const int ct = b % nct;
    b /= nct;
    const int xt = b % nxt, y = b / nxt;
    const int c0 = ct * HC_CT, x0 = xt * HC_XT;
    (void)H;
    int mine = 0;
    if (threadIdx.x < HC_XT) {
        const int x = x0 + threadIdx.x;
        mine = x < W ? p.window[(size_t)y * W + x] : 0;
        flag[threadIdx.x] = mine;
    }
    if (!__syncthreads_or(mine)) return;  // no marked texel in the tile: nothing read, nothing written
    const bool full_x = x0 + HC_XT <= W;
    constexpr int QPR = HC_XT / 4;
    for (int i = threadIdx.x; i < HC_CT * QPR; i += HC_NT) {
        const int cc = i / QPR, q = i - cc * QPR;
        const int c = c0 + cc, x = x0 + 4 * q;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if (c < C && (flag[4 * q] | flag[4 * q + 1] | flag[4 * q + 2] | flag[4 * q + 3])) {
            const Tin *src = chw + ((size_t)c * p.Hf + y) * W + x;
            if (it.vec[lo] && full_x) {
                if constexpr (sizeof(Tin) == 4) {
                    const nf4 w = kNtLoad ? __builtin_nontemporal_load(reinterpret_cast<const nf4 *>(src))
                                          : *reinterpret_cast<const nf4 *>(src);
                    v[0] = w.x; v[1] = w.y; v[2] = w.z; v[3] = w.w;
                } else {
                    const double2 w0 = *reinterpret_cast<const double2 *>(src);
                    const double2 w1 = *reinterpret_cast<const double2 *>(src + 2);
                    v[0] = (float)w0.x; v[1] = (float)w0.y; v[2] = (float)w1.x; v[3] = (float)w1.y;
                }
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (x + k < W) v[k] = (float)src[k];
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) tile[cc * HC_LD + 4 * q + k] = v[k];
    }
    __syncthreads();
    constexpr int QPC = HC_CT / 4;
    typedef float f4 __attribute__((ext_vector_type(4)));
    for (int i = threadIdx.x; i < HC_XT * QPC; i += HC_NT) {
        const int xx = i / QPC, cq = i - xx * QPC;
        const int x = x0 + xx, c = c0 + 4 * cq;
        if (x < W && c < cs && flag[xx]) {
            f4 o;
            o.x = tile[(4 * cq + 0) * HC_LD + xx];
            o.y = tile[(4 * cq + 1) * HC_LD + xx];
            o.z = tile[(4 * cq + 2) * HC_LD + xx];
            o.w = tile[(4 * cq + 3) * HC_LD + xx];
            __builtin_nontemporal_store(o, reinterpret_cast<f4 *>(out + ((size_t)y * W + x) * cs + c));
        }
    }
}

template <int CT, int XT>
static hipError_t pack_f_window_tiles(const fmpnp_problem *probs_dev, const fmpnp_problem *probs_host, int n,
                                      const void *const *chw, int dtype_in, hipStream_t stream) {
    for (int i0 = 0; i0 < n; i0 += WB_MAX) {
        WinItems it{};
        const int m = std::min(n - i0, WB_MAX);
        long total = 0;
        for (int j = 0; j < m; ++j) {
            const fmpnp_problem &p = probs_host[i0 + j];
            it.chw[j] = chw[i0 + j];
            it.nct[j] = (p.cstride + CT - 1) / CT;
            it.nxt[j] = (p.Wf + XT - 1) / XT;
            const size_t es = dtype_in == FMPNP_F64 ? 8 : 4;
            it.vec[j] = ((uintptr_t)chw[i0 + j] % 16 == 0) && ((size_t)p.Wf * es) % 16 == 0;
            it.start[j] = (int)total;
            total += (long)it.nct[j] * it.nxt[j] * p.Hf;
            if (total >= (1L << 31)) return hipErrorInvalidValue;
        }
        it.start[m] = (int)total;
        it.n = m;
        it.pd = probs_dev + i0;
        if (dtype_in == FMPNP_F32)
            hipLaunchKernelGGL((hwc_win_kernel<float, CT, XT>), dim3((unsigned)total), dim3(HC_NT), 0, stream, it);
        else
            hipLaunchKernelGGL((hwc_win_kernel<double, CT, XT>), dim3((unsigned)total), dim3(HC_NT), 0, stream, it);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// ---------------------------------------------------------------------------------------
// Multi-row windowed f-only packs (round 5; FMPNP_PACK_F_ROWS=0 keeps the one-row hwc_win_kernel
// above for A/B).  A workgroup takes one 64-channel x 64-column tile over HR_R consecutive rows.  Per row: the
// channel rows (16 lanes x 16 B = one 256-byte run each) land in the LDS tile, and right after the
// barrier the NEXT row's loads are issued into the same registers, so they are in flight while
// the current row's texels (16 lanes x 16 B = 256 contiguous bytes of channels each) are stored;
// the grid has HR_R times fewer workgroups.  Plane 0 of the tile's rows is read once (wave r: row r);
// rows without a marked texel are skipped (the tile when none has one), only the 16-byte column quads
// holding a marked texel are loaded and only marked texels stored.  End to end at r = 5 (bench
// end_to_end, 2 x interleaved, profiles/r05_pack_rows_ab.txt): 34.5-35.1 k against 33.4 k queries/s,
// hard start 37.6-39.0 k against 35.5 k.  (The full pack keeps the one-row tiles: the same multi-row
// tiles cost the RobotCar leg's C = 1664 full packs 4-9 %.)
constexpr int HR_NT = 256, HR_CT = 64, HR_XT = 64, HR_R = HR_NT / HR_XT;  // 4 rows: wave r reads row r's flags
constexpr int HR_QPR = HR_XT / 4, HR_NL = HR_CT * HR_QPR / HR_NT;       // 16-B units per channel row; loads per lane

template <typename Tin>
__device__ __forceinline__ void hr_load(const Tin *__restrict__ chw, int C, int H, int W, int c0, int x0, int y,
                                        bool vec, const int *fl, float (&v)[HR_NL][4]) {
    const int q = threadIdx.x % HR_QPR, x = x0 + 4 * q;
    const bool quad = vec && x + 3 < W;
    const bool want = fl[4 * q] | fl[4 * q + 1] | fl[4 * q + 2] | fl[4 * q + 3];
#pragma unroll
    for (int l = 0; l < HR_NL; ++l) {
        const int c = c0 + (int)threadIdx.x / HR_QPR + l * (HR_NT / HR_QPR);
        v[l][0] = v[l][1] = v[l][2] = v[l][3] = 0.f;
        if (c < C && want) {
            const Tin *src = chw + ((size_t)c * H + y) * W + x;
            if (quad) {
                if constexpr (sizeof(Tin) == 4) {
                    const nf4 w = kNtLoad ? __builtin_nontemporal_load(reinterpret_cast<const nf4 *>(src))
                                          : *reinterpret_cast<const nf4 *>(src);
                    v[l][0] = w.x; v[l][1] = w.y; v[l][2] = w.z; v[l][3] = w.w;
                } else {
                    const double2 w0 = *reinterpret_cast<const double2 *>(src);
                    const double2 w1 = *reinterpret_cast<const double2 *>(src + 2);
                    v[l][0] = (float)w0.x; v[l][1] = (float)w0.y; v[l][2] = (float)w1.x; v[l][3] = (float)w1.y;
                }
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (x + k < W) v[l][k] = (float)src[k];
            }
        }
    }
}

template <typename Tin>
__device__ __forceinline__ void hr_tile(const Tin *__restrict__ chw, int C, int H, int W, float *__restrict__ out,
                                        int cs, const unsigned char *__restrict__ win, int nct, int nxt, int vec_ok,
                                        int b) {
    constexpr int LD = HR_XT + 1;
    __shared__ float tile[HR_CT * LD];
    __shared__ int flag[HR_R][HR_XT];
    __shared__ int rowany[HR_R];
    const int ct = b % nct;
    b /= nct;
    const int xt = b % nxt, y0 = (b / nxt) * HR_R;
    const int c0 = ct * HR_CT, x0 = xt * HR_XT;
    const int rows = min(HR_R, H - y0);
    const bool full_x = x0 + HR_XT <= W;
    {
        const int r = threadIdx.x / HR_XT, xx = threadIdx.x % HR_XT, x = x0 + xx;
        const int f = r < rows && x < W && win[(size_t)(y0 + r) * W + x];
        flag[r][xx] = f;
        const bool any = __any(f);  // (HR_XT == 64: wave r holds row r)
        if ((threadIdx.x & 63) == 0) rowany[r] = any;
    }
    __syncthreads();
    int r = 0;
    while (r < HR_R && !rowany[r]) ++r;
    if (r == HR_R) return;  // no marked texel in the tile: nothing read, nothing written
    float v[HR_NL][4];
    hr_load<Tin>(chw, C, H, W, c0, x0, y0 + r, vec_ok && full_x, flag[r], v);
    typedef float f4 __attribute__((ext_vector_type(4)));
    while (r < HR_R) {
#pragma unroll
        for (int l = 0; l < HR_NL; ++l) {
            const int cc = (int)threadIdx.x / HR_QPR + l * (HR_NT / HR_QPR), q = threadIdx.x % HR_QPR;
#pragma unroll
            for (int k = 0; k < 4; ++k) tile[cc * LD + 4 * q + k] = v[l][k];
        }
        __syncthreads();
        int nr = r + 1;
        while (nr < HR_R && !rowany[nr]) ++nr;
        if (nr < HR_R) hr_load<Tin>(chw, C, H, W, c0, x0, y0 + nr, vec_ok && full_x, flag[nr], v);
        constexpr int QPC = HR_CT / 4;
        const int y = y0 + r;
#pragma unroll
        for (int l = 0; l < HR_XT * QPC / HR_NT; ++l) {
            const int i = (int)threadIdx.x + l * HR_NT;
            const int xx = i / QPC, cq = i - xx * QPC;
            const int x = x0 + xx, c = c0 + 4 * cq;
            if (flag[r][xx] && c < cs) {  // (flag: x < W and marked)
                f4 o;
                o.x = tile[(4 * cq + 0) * LD + xx];
                o.y = tile[(4 * cq + 1) * LD + xx];
                o.z = tile[(4 * cq + 2) * LD + xx];
                o.w = tile[(4 * cq + 3) * LD + xx];
                __builtin_nontemporal_store(o, reinterpret_cast<f4 *>(out + ((size_t)y * W + x) * cs + c));
            }
        }
        __syncthreads();
        r = nr;
    }
}

template <typename Tin>
__global__ __launch_bounds__(HR_NT) void hwc_rows_win_kernel(WinItems it) {
    const int b = blockIdx.x;
    int lo = 0, hi = it.n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (it.start[mid] <= b) lo = mid;
        else hi = mid - 1;
    }
    const fmpnp_problem &p = it.pd[lo];
    hr_tile<Tin>(reinterpret_cast<const Tin *>(it.chw[lo]), p.c_end, p.Hf, p.Wf,
                       reinterpret_cast<float *>(const_cast<void *>(p.feat)), p.cstride, p.window, it.nct[lo],
                       it.nxt[lo], it.vec[lo], b - it.start[lo]);
}

static bool pack_f_rows() {
    static const bool on = [] { const char *e = getenv("FMPNP_PACK_F_ROWS"); return !e || *e != '0'; }();
    return on;
}

static hipError_t pack_f_window_rows(const fmpnp_problem *probs_dev, const fmpnp_problem *probs_host, int n,
                                    const void *const *chw, int dtype_in, hipStream_t stream) {
    const size_t es = dtype_in == FMPNP_F64 ? 8 : 4;
    for (int i0 = 0; i0 < n; i0 += WB_MAX) {
        WinItems it{};
        const int m = std::min(n - i0, WB_MAX);
        long total = 0;
        for (int j = 0; j < m; ++j) {
            const fmpnp_problem &p = probs_host[i0 + j];
            if (p.cstride % 4 != 0 || ((uintptr_t)p.feat % 16) != 0 || !p.window) return hipErrorInvalidValue;
            it.chw[j] = chw[i0 + j];
            it.nct[j] = (p.cstride + HR_CT - 1) / HR_CT;
            it.nxt[j] = (p.Wf + HR_XT - 1) / HR_XT;
            it.vec[j] = ((uintptr_t)chw[i0 + j] % 16 == 0) && ((size_t)p.Wf * es) % 16 == 0;
            it.start[j] = (int)total;
            total += (long)it.nct[j] * it.nxt[j] * ((p.Hf + HR_R - 1) / HR_R);
            if (total >= (1L << 31)) return hipErrorInvalidValue;
        }
        it.start[m] = (int)total;
        it.n = m;
        it.pd = probs_dev + i0;
        if (total == 0) continue;
        if (dtype_in == FMPNP_F32) hipLaunchKernelGGL(hwc_rows_win_kernel<float>, dim3((unsigned)total), dim3(HR_NT), 0, stream, it);
        else hipLaunchKernelGGL(hwc_rows_win_kernel<double>, dim3((unsigned)total), dim3(HR_NT), 0, stream, it);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_pack_f_window(const fmpnp_problem *probs_dev, const fmpnp_problem *probs_host, int n,
                                const void *const *chw, int dtype_in, int radius, int max_n, long max_hw,
                                hipStream_t stream) {
    const unsigned ny = (unsigned)n;
    const unsigned cb = (unsigned)std::min<long>((2 * max_hw + 16L * PK_NT - 1) / (16L * PK_NT), 1024);
    hipLaunchKernelGGL(win_clear_kernel, dim3(std::max(cb, 1u), ny), dim3(PK_NT), 0, stream, probs_dev);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (max_n > 0) {
        const long nt = (long)max_n * (2 * radius + 1);
        hipLaunchKernelGGL(win_mark_kernel, dim3((unsigned)((nt + PK_NT - 1) / PK_NT), ny), dim3(PK_NT), 0, stream,
                           probs_dev, radius);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    // tile (channels x columns), FMPNP_PACK_W_TILE: 1: 64 x 64 (default), 0: 64 x 32, 2: 128 x 32, 3: 32 x 64,
    // 4: 128 x 64, 5: 256 x 32, 6: 64 x 128.  End to end at radius 5 (tools/window_sweep.py, queries/s):
    // 64 x 64 33.1-33.2 k, 128 x 32 32.3-33.4 k, 64 x 32 30.7 k, 32 x 64 29.9 k, 256 x 32 26.5 k,
    // 128 x 64 25.5 k, 64 x 128 22.8 k (profiles/r04_window_tiles.txt)
    if (pack_f_rows()) return pack_f_window_rows(probs_dev, probs_host, n, chw, dtype_in, stream);
    static const int tile = [] { const char *e = getenv("FMPNP_PACK_W_TILE"); return e ? atoi(e) : 1; }();
    switch (tile) {
    case 1: return pack_f_window_tiles<64, 64>(probs_dev, probs_host, n, chw, dtype_in, stream);
    case 2: return pack_f_window_tiles<128, 32>(probs_dev, probs_host, n, chw, dtype_in, stream);
    case 3: return pack_f_window_tiles<32, 64>(probs_dev, probs_host, n, chw, dtype_in, stream);
    case 4: return pack_f_window_tiles<128, 64>(probs_dev, probs_host, n, chw, dtype_in, stream);
    case 5: return pack_f_window_tiles<256, 32>(probs_dev, probs_host, n, chw, dtype_in, stream);
    case 6: return pack_f_window_tiles<64, 128>(probs_dev, probs_host, n, chw, dtype_in, stream);
    default: return pack_f_window_tiles<64, 32>(probs_dev, probs_host, n, chw, dtype_in, stream);
    }
}

hipError_t launch_win_mark(const fmpnp_problem *probs_dev, int n, int radius, int max_n, long max_hw, hipStream_t stream) {
    const unsigned ny = (unsigned)n;
    const unsigned cb = (unsigned)std::min<long>((2 * max_hw + 16L * PK_NT - 1) / (16L * PK_NT), 1024);
    hipLaunchKernelGGL(win_clear_kernel, dim3(std::max(cb, 1u), ny), dim3(PK_NT), 0, stream, probs_dev);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || max_n <= 0) return e;
    const long nt = (long)max_n * (2 * radius + 1);
    hipLaunchKernelGGL(win_mark_kernel, dim3((unsigned)((nt + PK_NT - 1) / PK_NT), ny), dim3(PK_NT), 0, stream, probs_dev,
                       radius);
    return hipGetLastError();
}

hipError_t launch_pack_win(const void *chw, int dtype_in, int C, int H, int W, void *out, int dtype_out, int cs,
                           int normalized, int replicate, const unsigned char *win, hipStream_t stream) {
    if (!win) return hipErrorInvalidValue;
    if (dtype_in == FMPNP_F32 && dtype_out == FMPNP_F32)
        return pack_t<float, float>(chw, nullptr, nullptr, C, H, W, out, cs, normalized, replicate, true, stream, win);
    if (dtype_in == FMPNP_F32 && dtype_out == FMPNP_F64)
        return pack_t<float, double>(chw, nullptr, nullptr, C, H, W, out, cs, normalized, replicate, true, stream, win);
    if (dtype_in == FMPNP_F64 && dtype_out == FMPNP_F32)
        return pack_t<double, float>(chw, nullptr, nullptr, C, H, W, out, cs, normalized, replicate, true, stream, win);
    return pack_t<double, double>(chw, nullptr, nullptr, C, H, W, out, cs, normalized, replicate, true, stream, win);
}

hipError_t launch_pack(const void *chw, const void *gx, const void *gy, int dtype_in, int C, int H, int W, void *out,
                       int dtype_out, int cs, int normalized, int replicate, hipStream_t stream, int planes) {
    const bool grad = planes != 1;
    if (!grad && gx) return hipErrorInvalidValue;
    if (!grad) {  // FMPNP_LAYOUT_F: fp32 channels-last copy (FMPNP_PACK_F_SOBEL=1: the Sobel kernel's f-only mode)
        static const int via_sobel = [] { const char *e = getenv("FMPNP_PACK_F_SOBEL"); return e && *e == '1'; }();
        if (dtype_out != FMPNP_F32) return hipErrorInvalidValue;
        if (!via_sobel)
            return dtype_in == FMPNP_F32 ? hwc_t<float>(chw, C, H, W, out, cs, stream)
                                         : hwc_t<double>(chw, C, H, W, out, cs, stream);
    }
    if (dtype_in == FMPNP_F32 && dtype_out == FMPNP_F32)
        return pack_t<float, float>(chw, gx, gy, C, H, W, out, cs, normalized, replicate, grad, stream);
    if (dtype_in == FMPNP_F32 && dtype_out == FMPNP_F64)
        return pack_t<float, double>(chw, gx, gy, C, H, W, out, cs, normalized, replicate, grad, stream);
    if (dtype_in == FMPNP_F64 && dtype_out == FMPNP_F32)
        return pack_t<double, float>(chw, gx, gy, C, H, W, out, cs, normalized, replicate, grad, stream);
    return pack_t<double, double>(chw, gx, gy, C, H, W, out, cs, normalized, replicate, grad, stream);
}

// fref gather (optimize_feature_pnp.py:51-56): relative_shape = [H_ref/img0, W_ref/img1];
// ref2d = int(relative_shape * (x, y)) truncates toward zero, then flip -> (row, col) =
// (trunc(y * W_ref/img1), trunc(x * H_ref/img0)).  One thread per (point, channel).
template <typename Tin, typename Tout>
__global__ __launch_bounds__(PK_NT) void gather_ref_kernel(const Tin *__restrict__ ref, int C, int H, int W,
                                                        const double *__restrict__ inl, int N, int img0, int img1,
                                                        Tout *__restrict__ out, int ld, int *__restrict__ err) {
    const long total = (long)N * C;
    for (long e = blockIdx.x * (long)PK_NT + threadIdx.x; e < total; e += (long)gridDim.x * PK_NT) {
        const int n = (int)(e / C), c = (int)(e % C);
        const double rel0 = (double)H / (double)img0, rel1 = (double)W / (double)img1;
        const double x = inl[2 * n], y = inl[2 * n + 1];
        const double colf = rel0 * x, rowf = rel1 * y;
        // int32 cast of a double truncates toward zero (torch IntTensor conversion)
        int col = (int)colf, row = (int)rowf;
        // python indexing of the reference wraps negative indices (a 0-d int tensor index)
        if (row < 0 && row >= -H) row += H;
        if (col < 0 && col >= -W) col += W;
        if (row < 0 || row >= H || col < 0 || col >= W || !(colf == colf) || !(rowf == rowf)) {
            if (c == 0) atomicOr(err, 1);  // the reference raises IndexError here
            out[(size_t)n * ld + c] = (Tout)0;
            continue;
        }
        out[(size_t)n * ld + c] = (Tout)ref[((size_t)c * H + row) * W + col];
    }
}

template <typename Tin, typename Tout>
static hipError_t gather_t(const void *ref, int C, int H, int W, const double *inl, int N, int img0, int img1,
                           void *out, int ld, int *err, hipStream_t stream) {
    long total = (long)N * C;
    int grid = (int)((total + PK_NT - 1) / PK_NT);
    if (grid > 4096) grid = 4096;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((gather_ref_kernel<Tin, Tout>), dim3(grid), dim3(PK_NT), 0, stream, (const Tin *)ref, C, H, W, inl,
                       N, img0, img1, (Tout *)out, ld, err);
    return hipGetLastError();
}

// Many queries' gathers in one launch (fmpnp_gather_reference_batch): the item table rides
// in the kernel arguments, the grid strides over all items' (point, channel) elements --
// one query's grid (512 x 256 elements at cfg2) is too small to hide the scattered CHW
// reads' latency on its own.
constexpr int GB_MAX = 32;
struct GatherItems {
    const void *ref[GB_MAX];
    const double *inl[GB_MAX];
    void *out[GB_MAX];
    int C[GB_MAX], H[GB_MAX], W[GB_MAX], ld[GB_MAX];
    long start[GB_MAX + 1];  // element offsets: item i owns [start[i], start[i+1]) (empty items allowed)
    int n, img0, img1;
    int *err;                // [n] flags
};

template <typename Tin, typename Tout>
__global__ __launch_bounds__(PK_NT) void gather_ref_batch_kernel(GatherItems it) {
    const long total = it.start[it.n];
    for (long e = blockIdx.x * (long)PK_NT + threadIdx.x; e < total; e += (long)gridDim.x * PK_NT) {
        int lo = 0, hi = it.n - 1;  // the last item whose range starts at or before e
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (it.start[mid] <= e) lo = mid;
            else hi = mid - 1;
        }
        const int i = lo, C = it.C[i], H = it.H[i], W = it.W[i];
        const long k = e - it.start[i];
        const int n = (int)(k / C), c = (int)(k % C);
        const double rel0 = (double)H / (double)it.img0, rel1 = (double)W / (double)it.img1;
        const double *inl = it.inl[i];
        const double x = inl[2 * n], y = inl[2 * n + 1];
        const double colf = rel0 * x, rowf = rel1 * y;
        int col = (int)colf, row = (int)rowf;  // as gather_ref_kernel
        if (row < 0 && row >= -H) row += H;
        if (col < 0 && col >= -W) col += W;
        Tout *out = reinterpret_cast<Tout *>(it.out[i]) + (size_t)n * it.ld[i] + c;
        if (row < 0 || row >= H || col < 0 || col >= W || !(colf == colf) || !(rowf == rowf)) {
            if (c == 0) atomicOr(it.err + i, 1);
            *out = (Tout)0;
            continue;
        }
        *out = (Tout)reinterpret_cast<const Tin *>(it.ref[i])[((size_t)c * H + row) * W + col];
    }
}

template <typename Tin, typename Tout>
static hipError_t gather_batch_t(const GatherItems &it, hipStream_t stream) {
    const long total = it.start[it.n];
    long grid = (total + PK_NT - 1) / PK_NT;
    if (grid > 8192) grid = 8192;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((gather_ref_batch_kernel<Tin, Tout>), dim3((unsigned)grid), dim3(PK_NT), 0, stream, it);
    return hipGetLastError();
}

hipError_t launch_gather_ref_batch(int n, const void *const *ref, const int *ref_shape, const double *const *inl,
                                   const int *n_inl, int img0, int img1, void *const *out, const int *ld_out,
                                   int dtype_in, int dtype_out, int *err, hipStream_t stream) {
    for (int i0 = 0; i0 < n; i0 += GB_MAX) {
        GatherItems it{};
        const int m = n - i0 < GB_MAX ? n - i0 : GB_MAX;
        it.start[0] = 0;
        for (int j = 0; j < m; ++j) {
            const int i = i0 + j;
            it.ref[j] = ref[i];
            it.inl[j] = inl[i];
            it.out[j] = out[i];
            it.C[j] = ref_shape[3 * i];
            it.H[j] = ref_shape[3 * i + 1];
            it.W[j] = ref_shape[3 * i + 2];
            it.ld[j] = ld_out[i];
            it.start[j + 1] = it.start[j] + (long)n_inl[i] * it.C[j];
        }
        if (it.start[m] == 0) continue;
        it.n = m;
        it.img0 = img0;
        it.img1 = img1;
        it.err = err + i0;
        hipError_t e;
        if (dtype_in == FMPNP_F32 && dtype_out == FMPNP_F32) e = gather_batch_t<float, float>(it, stream);
        else if (dtype_in == FMPNP_F32 && dtype_out == FMPNP_F64) e = gather_batch_t<float, double>(it, stream);
        else if (dtype_in == FMPNP_F64 && dtype_out == FMPNP_F32) e = gather_batch_t<double, float>(it, stream);
        else e = gather_batch_t<double, double>(it, stream);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_gather_ref(const void *ref, int dtype_in, int C, int H, int W, const double *inl, int N, int img0,
                             int img1, void *out, int dtype_out, int ld_out, int *err, hipStream_t stream) {
    if (dtype_in == FMPNP_F32 && dtype_out == FMPNP_F32)
        return gather_t<float, float>(ref, C, H, W, inl, N, img0, img1, out, ld_out, err, stream);
    if (dtype_in == FMPNP_F32 && dtype_out == FMPNP_F64)
        return gather_t<float, double>(ref, C, H, W, inl, N, img0, img1, out, ld_out, err, stream);
    if (dtype_in == FMPNP_F64 && dtype_out == FMPNP_F32)
        return gather_t<double, float>(ref, C, H, W, inl, N, img0, img1, out, ld_out, err, stream);
    return gather_t<double, double>(ref, C, H, W, inl, N, img0, img1, out, ld_out, err, stream);
}

}  // namespace fmpnp
