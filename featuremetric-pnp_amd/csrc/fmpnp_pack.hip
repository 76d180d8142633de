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
// Tiling: a workgroup owns 64 channels x 64 columns x RS rows.  It keeps a ring
// of three input rows in LDS (row stride 67 elements: conflict-free column
// reads), loads row y+1 while computing row y, and writes the three output planes
// with lanes along channels (256-B coalesced stores).  Input is read (RS+2)/RS
// times, output written once: ~16.5 B of HBM traffic per fp32 element vs 16 ideal.
#include <hip/hip_runtime.h>
#include <stdint.h>

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

template <typename Tin, typename Tout>
static hipError_t pack_t(const void *chw, const void *gx, const void *gy, int C, int H, int W, void *out, int cs,
                         int normalized, int replicate, hipStream_t stream) {
    dim3 grid((C + PK_CB - 1) / PK_CB, (W + PK_XW - 1) / PK_XW, (H + PK_RS - 1) / PK_RS);
    size_t lds = 3 * PK_CB * PK_LD * sizeof(Tin);
    if (gx) {
        hipLaunchKernelGGL((pack_kernel<Tin, Tout, true>), grid, dim3(PK_NT), lds, stream, (const Tin *)chw,
                           (const Tin *)gx, (const Tin *)gy, C, H, W, (Tout *)out, cs, normalized, replicate);
    } else {
        hipLaunchKernelGGL((pack_kernel<Tin, Tout, false>), grid, dim3(PK_NT), lds, stream, (const Tin *)chw,
                           (const Tin *)nullptr, (const Tin *)nullptr, C, H, W, (Tout *)out, cs, normalized,
                           replicate);
    }
    return hipGetLastError();
}

hipError_t launch_pack(const void *chw, const void *gx, const void *gy, int dtype_in, int C, int H, int W, void *out,
                       int dtype_out, int cs, int normalized, int replicate, hipStream_t stream) {
    if (dtype_in == FMPNP_F32 && dtype_out == FMPNP_F32)
        return pack_t<float, float>(chw, gx, gy, C, H, W, out, cs, normalized, replicate, stream);
    if (dtype_in == FMPNP_F32 && dtype_out == FMPNP_F64)
        return pack_t<float, double>(chw, gx, gy, C, H, W, out, cs, normalized, replicate, stream);
    if (dtype_in == FMPNP_F64 && dtype_out == FMPNP_F32)
        return pack_t<double, float>(chw, gx, gy, C, H, W, out, cs, normalized, replicate, stream);
    return pack_t<double, double>(chw, gx, gy, C, H, W, out, cs, normalized, replicate, stream);
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
