// VALU issue and dependent-latency costs on gfx950 (one CU, s_memtime per wave): what one wave
// alone and two waves per SIMD sustain for fp64 / fp32 FMAs, v_rcp_f64, v_readlane and an LDS
// broadcast read.  Sizes the LM kernel's single-wave tail (fmpnp_lm_impl.h lm_tail).
//   hipcc -O3 --offload-arch=gfx950 -o valu_issue valu_issue.hip && ./valu_issue
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int REP = 256;

template <int KIND>
__global__ void bench(double *out, unsigned long long *cyc, double seed) {
    __shared__ double lds[64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x < 64) lds[threadIdx.x] = seed + threadIdx.x;
    __syncthreads();
    double a0 = seed + lane, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
    float f0 = (float)a0, f1 = f0 + 1, f2 = f0 + 2, f3 = f0 + 3, f4 = f0 + 4, f5 = f0 + 5, f6 = f0 + 6, f7 = f0 + 7;
    const double m = 0.999999, c = 1e-9;
    int idx = lane & 7;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int r = 0; r < REP; ++r) {
        if constexpr (KIND == 0) {  // 8 independent fp64 FMA chains: throughput (8 instr per trip)
            a0 = fma(a0, m, c); a1 = fma(a1, m, c); a2 = fma(a2, m, c); a3 = fma(a3, m, c);
            a4 = fma(a4, m, c); a5 = fma(a5, m, c); a6 = fma(a6, m, c); a7 = fma(a7, m, c);
        } else if constexpr (KIND == 1) {  // one dependent fp64 chain (8 instr per trip)
#pragma unroll
            for (int k = 0; k < 8; ++k) a0 = fma(a0, m, c);
        } else if constexpr (KIND == 2) {  // 8 independent fp32 chains
            f0 = fmaf(f0, 0.999f, 1e-3f); f1 = fmaf(f1, 0.999f, 1e-3f); f2 = fmaf(f2, 0.999f, 1e-3f);
            f3 = fmaf(f3, 0.999f, 1e-3f); f4 = fmaf(f4, 0.999f, 1e-3f); f5 = fmaf(f5, 0.999f, 1e-3f);
            f6 = fmaf(f6, 0.999f, 1e-3f); f7 = fmaf(f7, 0.999f, 1e-3f);
        } else if constexpr (KIND == 3) {  // one dependent fp32 chain
#pragma unroll
            for (int k = 0; k < 8; ++k) f0 = fmaf(f0, 0.999f, 1e-3f);
        } else if constexpr (KIND == 4) {  // dependent rcp + Newton step (3 instr per link), 8 links
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const double r0 = __builtin_amdgcn_rcp(a0);
                a0 = fma(fma(-a0, r0, 1.0), r0, r0) + 1.0;
            }
        } else if constexpr (KIND == 5) {  // readlane of a double into SGPRs, then a dependent fp64 use (8 links)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const long long b = __double_as_longlong(a0);
                const int lo = __builtin_amdgcn_readlane((int)b, 5), hi = __builtin_amdgcn_readlane((int)(b >> 32), 5);
                const double s = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
                a0 = fma(s, m, c);
            }
        } else if constexpr (KIND == 6) {  // dependent LDS broadcast read (address from the data), 8 links
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const double v = lds[idx];
                idx = ((int)v) & 7;
                a0 += v;
            }
        } else if constexpr (KIND == 7) {  // 8 independent dpp64 moves + add (row_mirror)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const long long b = __double_as_longlong(a1);
                const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x140, 0xF, 0xF, false);
                const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x140, 0xF, 0xF, false);
                a0 += __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
            }
        }
        asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[w] = t1 - t0;
    out[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7 + idx;
}

template <int K>
void run(const char *name, int threads, double *out, unsigned long long *cyc) {
    unsigned long long h[16] = {0};
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(bench<K>, 1, threads, 0, 0, out, cyc, 1.5);
        hipDeviceSynchronize();
    }
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double mx = 0;
    for (int w = 0; w < threads / 64; ++w) mx = h[w] > mx ? h[w] : mx;
    printf("%-34s waves %2d: %6.2f cycles per instruction-slot (max over waves)\n", name, threads / 64,
           mx / (REP * 8.0));
}

int main() {
    double *out;
    unsigned long long *cyc;
    hipMalloc(&out, 1024 * sizeof(double));
    hipMalloc(&cyc, 16 * sizeof(unsigned long long));
    for (int t : {64, 256, 512}) {
        run<0>("fp64 fma, 8 independent", t, out, cyc);
        run<1>("fp64 fma, dependent", t, out, cyc);
        run<2>("fp32 fma, 8 independent", t, out, cyc);
        run<3>("fp32 fma, dependent", t, out, cyc);
        run<4>("rcp+newton link (per link)", t, out, cyc);
        run<5>("readlane x2 + fma link (per link)", t, out, cyc);
        run<6>("LDS broadcast read link", t, out, cyc);
        run<7>("dpp64 mov x2 + add (per step)", t, out, cyc);
    }
    return 0;
}
