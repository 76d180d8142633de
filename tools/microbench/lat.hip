// Dependent-load latency on MI355X for random 16-byte loads over a buffer of a given size
// (pointer chase, one wave, s_memtime).  Used to size the LM kernel's gather round trip.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>

__global__ void chase(const uint64_t *__restrict__ next, int steps, uint64_t start, unsigned long long *out) {
    uint64_t p = start;
    // warm nothing: every step is a dependent load
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < steps; ++i) {
        asm volatile("" : "+v"(p));  // keep the address in a VGPR: a vector (not scalar-cache) load
        p = next[p];
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = p; }
}

int main(int argc, char **argv) {
    const int steps = 2000;
    size_t sizes_mb[] = {2, 16, 128, 512, 4096, 32768};
    for (size_t mb : sizes_mb) {
        size_t bytes = mb << 20;
        size_t n = bytes / 8;
        uint64_t *d;
        if (hipMalloc(&d, bytes) != hipSuccess) { printf("alloc %zu MB failed\n", mb); continue; }
        // chain of `steps` random slots spaced >= 4 KB apart (each slot 8 B), rest untouched
        std::vector<uint64_t> idx(steps + 1);
        srand(1234);
        for (int i = 0; i <= steps; ++i) idx[i] = (((uint64_t)rand() << 31 | rand()) % (n / 512)) * 512;
        for (int i = 0; i < steps; ++i)
            hipMemcpy(d + idx[i], &idx[i + 1], 8, hipMemcpyHostToDevice);
        unsigned long long *o;
        hipMalloc(&o, 16);
        unsigned long long h[2];
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0, 0);
            hipLaunchKernelGGL(chase, 1, 64, 0, 0, d, steps, idx[0], o);
            hipEventRecord(e1, 0);
            hipMemcpy(h, o, 16, hipMemcpyDeviceToHost);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            printf("buffer %6zu MB  rep %d: %.0f memtime ticks per dependent load, %.1f ns per load (event), "
                   "tick rate %.2f GHz\n", mb, rep, (double)h[0] / steps, ms * 1e6 / steps, (double)h[0] / (ms * 1e6));
        }
        hipFree(o);
        hipFree(d);
    }
    return 0;
}
