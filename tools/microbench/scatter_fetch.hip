// Calibration of the memory-side read counters for SCATTERED 4-byte reads (the reference-descriptor
// gather's access: one fp32 per (point, channel) of a CHW map, H*W*4 bytes between channels).
// MI355X_MICROARCH.md calibrates FETCH_SIZE only for wide coalesced reads (FETCH_SIZE = RDREQ x 64 B =
// half the bytes); this program gives the counters a known count of isolated reads.
//   k_scatter<S>: thread i reads one float at byte offset i * S of a 4 GiB buffer (S >= 128: every read
//                 in its own 128-B line, no two reads of a wave in one line) -- n reads per launch;
//   k_pairs:      the same, two consecutive floats per 128-B line (8 B used per line).
// Each kernel runs on a fresh region (> the 256 MiB Infinity Cache apart), timed with events.
// usage: scatter_fetch [n_reads_millions]; profile with rocprofv3 --pmc FETCH_SIZE / TCC_EA0_RDREQ_sum ...
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

template <int S>
__global__ void k_scatter(const float *__restrict__ buf, size_t n, float *__restrict__ sink) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float v = buf[i * (S / 4)];
    if (v == 12345.0f) sink[0] = v;  // (never true: keeps the load)
}
__global__ void k_pairs(const float *__restrict__ buf, size_t n, float *__restrict__ sink) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float v = buf[(i >> 1) * 32 + (i & 1)];  // two floats per 128-B line
    if (v == 12345.0f) sink[0] = v;
}

int main(int argc, char **argv) {
    const size_t n = (size_t)((argc > 1 ? atof(argv[1]) : 4.0) * 1e6);
    const size_t bytes = (size_t)4 << 30;
    char *buf;
    float *sink;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, bytes);
    (void)hipDeviceSynchronize();
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    struct K { const char *name; int stride; };
    const K ks[] = {{"scatter128", 128}, {"scatter256", 256}, {"scatter1024", 1024}, {"pairs128", 128}};
    size_t off = 0;
    for (const K &k : ks) {
        const size_t span = (k.stride == 0 ? 128 : (size_t)k.stride) * n;
        if (off + span > bytes) off = 0;
        const float *p = (const float *)(buf + off);
        const unsigned grid = (unsigned)((n + 255) / 256);
        float ms = 0.f;
        for (int rep = 0; rep < 3; ++rep) {  // rep 0 warms the TLB; 1, 2 timed (the last one reported)
            (void)hipEventRecord(a);
            if (k.stride == 128 && k.name[0] == 's') hipLaunchKernelGGL(k_scatter<128>, dim3(grid), dim3(256), 0, 0, p, n, sink);
            else if (k.stride == 256) hipLaunchKernelGGL(k_scatter<256>, dim3(grid), dim3(256), 0, 0, p, n, sink);
            else if (k.stride == 1024) hipLaunchKernelGGL(k_scatter<1024>, dim3(grid), dim3(256), 0, 0, p, n, sink);
            else hipLaunchKernelGGL(k_pairs, dim3(grid), dim3(256), 0, 0, p, n, sink);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            (void)hipEventElapsedTime(&ms, a, b);
        }
        const double lines = k.name[0] == 'p' ? n / 2.0 : (double)n;
        printf("%-12s reads %zu lines %.0f  %.3f ms  %.1f G lines/s  (x128 B: %.2f TB/s, x64 B: %.2f TB/s)\n", k.name, n,
               lines, ms, lines / (ms * 1e-3) / 1e9, lines * 128 / (ms * 1e-3) / 1e12, lines * 64 / (ms * 1e-3) / 1e12);
        off += span + ((size_t)512 << 20);
    }
    return 0;
}
