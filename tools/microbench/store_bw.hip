// Store-bandwidth ceiling for the pack kernel's output pattern (MI355X).
//  k_dword : lane = channel, 4-B stores, 256 B per wave instruction (the pack kernel's pattern)
//  k_x4    : 16-B stores, 1 KB contiguous per wave instruction
//  k_copy  : read 1/3 of the bytes (16-B loads) and write them 3x (16-B stores): the pack's mix
// usage: store_bw [MB]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void k_dword(float *out, size_t n_texels, int cs) {
    // one workgroup of 256 threads = 4 waves; wave w writes texel (blk*4+w), lanes = 64 channels,
    // all cs/64 channel blocks and 3 planes
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (size_t tx = (size_t)blockIdx.x * 4 + w; tx < n_texels; tx += (size_t)gridDim.x * 4) {
        float *o = out + tx * 3 * cs;
        for (int p = 0; p < 3; ++p)
            for (int c = lane; c < cs; c += 64) __builtin_nontemporal_store((float)c, o + p * cs + c);
    }
}
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void k_x4(f4 *out, size_t n4) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        f4 v = {1.f, 2.f, 3.f, (float)i};
        __builtin_nontemporal_store(v, out + i);
    }
}
__global__ void k_copy(const f4 *in, f4 *out, size_t n4in) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4in; i += (size_t)gridDim.x * blockDim.x) {
        f4 v = in[i];
        __builtin_nontemporal_store(v, out + 3 * i);
        __builtin_nontemporal_store(v, out + 3 * i + 1);
        __builtin_nontemporal_store(v, out + 3 * i + 2);
    }
}

int main(int argc, char **argv) {
    const int cs = 256;
    const size_t texels = 240 * 320;
    const int NB = 4;  // rotate buffers: > Infinity Cache
    float *outs[NB], *ins[NB];
    const size_t out_bytes = texels * 3 * cs * 4, in_bytes = texels * cs * 4;
    for (int i = 0; i < NB; ++i) {
        hipMalloc(&outs[i], out_bytes);
        hipMalloc(&ins[i], in_bytes);
        hipMemset(ins[i], 0, in_bytes);
    }
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int reps = 32;
    for (int grid : {1024, 2048, 4096, 8192}) {
        float ms;
        for (int i = 0; i < NB; ++i) k_dword<<<grid, 256>>>(outs[i], texels, cs);
        hipEventRecord(a);
        for (int r = 0; r < reps; ++r) k_dword<<<grid, 256>>>(outs[r % NB], texels, cs);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        printf("dword  grid %5d: %.1f us  %.0f GB/s (writes)\n", grid, 1e3 * ms / reps, out_bytes / (ms / reps) / 1e6);
        hipEventRecord(a);
        for (int r = 0; r < reps; ++r) k_x4<<<grid, 256>>>((f4 *)outs[r % NB], out_bytes / 16);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        printf("x4     grid %5d: %.1f us  %.0f GB/s (writes)\n", grid, 1e3 * ms / reps, out_bytes / (ms / reps) / 1e6);
        hipEventRecord(a);
        for (int r = 0; r < reps; ++r) k_copy<<<grid, 256>>>((const f4 *)ins[r % NB], (f4 *)outs[r % NB], in_bytes / 16);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        printf("copy3x grid %5d: %.1f us  %.0f GB/s (read+write)\n", grid, 1e3 * ms / reps,
               (in_bytes + out_bytes) / (ms / reps) / 1e6);
    }
    return 0;
}
