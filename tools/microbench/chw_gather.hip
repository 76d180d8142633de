// Gathering a point's 3x3 x C neighbourhood straight from the CNN's CHW map versus from the
// channels-last [H][W][C] copy (FMPNP_LAYOUT_F).  One 512-thread workgroup per query (the LM
// kernel's shape at B = 128), each wave gathers its share of the query's point-neighbourhoods,
// lane l owns channels 4l..4l+3 (C = 256), two points in flight per wave.  Sizes the
// pack-free layout before it is built: if the CHW gathers of a refinement cost less than the
// pack they replace, the channels-last copy can go.
//
//   hipcc -O3 --offload-arch=gfx950 -o chw_gather chw_gather.hip && ./chw_gather
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int C = 256, H = 240, W = 320, NT = 512;

// CHW: per channel three row loads of 3 floats (12 B) at rows r-1..r+1, columns c-1..c+1
__device__ __forceinline__ double chw_point(const float *__restrict__ m, int r, int c, int lane) {
    float v[4][9];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float *p = m + ((size_t)(4 * lane + k) * H + (r - 1)) * W + (c - 1);
#pragma unroll
        for (int dr = 0; dr < 3; ++dr) {
#pragma unroll
            for (int dc = 0; dc < 3; ++dc) v[k][3 * dr + dc] = __builtin_nontemporal_load(p + dr * W + dc);
        }
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double gx = (double)v[k][2] - v[k][0] + 2.0 * ((double)v[k][5] - v[k][3]) + (double)v[k][8] - v[k][6];
        const double gy = (double)v[k][6] - v[k][0] + 2.0 * ((double)v[k][7] - v[k][1]) + (double)v[k][8] - v[k][2];
        s += gx * gx + gy * gy + (double)v[k][4];
    }
    return s;
}

// HWC: nine 16-byte texel loads (this lane's four channels of each neighbour)
__device__ __forceinline__ double hwc_point(const float *__restrict__ m, int r, int c, int lane) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    f4 v[9];
#pragma unroll
    for (int dr = 0; dr < 3; ++dr)
#pragma unroll
        for (int dc = 0; dc < 3; ++dc)
            v[3 * dr + dc] = __builtin_nontemporal_load(
                reinterpret_cast<const f4 *>(m + ((size_t)(r - 1 + dr) * W + (c - 1 + dc)) * C) + lane);
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double gx = (double)v[2][k] - v[0][k] + 2.0 * ((double)v[5][k] - v[3][k]) + (double)v[8][k] - v[6][k];
        const double gy = (double)v[6][k] - v[0][k] + 2.0 * ((double)v[7][k] - v[1][k]) + (double)v[8][k] - v[2][k];
        s += gx * gx + gy * gy + (double)v[4][k];
    }
    return s;
}

template <bool CHW>
__global__ __launch_bounds__(NT, 2) void gather(const float *maps, size_t map_elems, const int *pix, int npts,
                                                double *out) {
    const int q = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const float *m = maps + (size_t)q * map_elems;
    const int *pp = pix + (size_t)q * npts;
    double s = 0.0;
    for (int i = wave; i < npts; i += 2 * (NT / 64)) {
        const int a = pp[i], b = i + NT / 64 < npts ? pp[i + NT / 64] : a;
        const double x = CHW ? chw_point(m, a >> 16, a & 0xffff, lane) : hwc_point(m, a >> 16, a & 0xffff, lane);
        const double y = CHW ? chw_point(m, b >> 16, b & 0xffff, lane) : hwc_point(m, b >> 16, b & 0xffff, lane);
        s += x + y;
    }
    out[(size_t)q * NT + threadIdx.x] = s;
}

int main(int argc, char **argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 128;
    const int npts = argc > 2 ? atoi(argv[2]) : 1233;  // point-gathers per cfg2 refinement (bench.py layout_f)
    const size_t me = (size_t)C * H * W;
    float *maps;
    CK(hipMalloc(&maps, (size_t)B * me * 4));
    CK(hipMemset(maps, 0, (size_t)B * me * 4));
    std::vector<int> h((size_t)B * npts);
    srand(7);
    for (auto &v : h) {
        const int r = 1 + (int)(0.1 * H + (rand() % (int)(0.8 * H))) % (H - 2);
        const int c = 1 + (int)(0.1 * W + (rand() % (int)(0.8 * W))) % (W - 2);
        v = (r << 16) | c;
    }
    int *pix;
    double *out;
    CK(hipMalloc(&pix, h.size() * 4));
    CK(hipMemcpy(pix, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&out, (size_t)B * NT * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int layout = 0; layout < 2; ++layout) {
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0, 0));
            if (layout == 0) hipLaunchKernelGGL(gather<true>, B, NT, 0, 0, maps, me, pix, npts, out);
            else hipLaunchKernelGGL(gather<false>, B, NT, 0, 0, maps, me, pix, npts, out);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double g = (double)B * npts;
            printf("{\"layout\": \"%s\", \"B\": %d, \"gathers_per_query\": %d, \"rep\": %d, \"ms\": %.4f, "
                   "\"us_per_query\": %.3f, \"ns_per_gather_chipwide\": %.2f, \"useful_GB_per_s\": %.1f}\n",
                   layout == 0 ? "chw" : "hwc", B, npts, rep, ms, ms * 1e3 / B, ms * 1e6 / g,
                   g * 9.0 * C * 4 / (ms * 1e6));
        }
    }
    return 0;
}
