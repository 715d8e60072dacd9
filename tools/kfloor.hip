// kfloor.hip -- what a dependent kernel costs before it does any work, by launch geometry: the
// floor under the short-prompt prefill kernels (k_quantize_q8_K_mmx, k_mmqd1). Back-to-back
// launches on one stream, HIP events around 400 of them (per-launch = the chain's step time).
//   hipcc --offload-arch=gfx950 -O3 tools/kfloor.hip -o tools/kfloor && tools/kfloor
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

// nothing but a store from one lane (keeps the kernel from being empty)
__global__ void k_empty(int * out) {
    extern __shared__ int lds[];
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
    (void) lds;
}

// one 16-byte load per lane from `src` (a fresh region each launch: cold HBM), one 4-byte store
__global__ void k_load1(const uint4 * __restrict__ src, int * out) {
    extern __shared__ int lds[];
    const uint4 v = src[(size_t) blockIdx.x * blockDim.x + threadIdx.x];
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345u) out[1] = 1;
    (void) lds;
}

// n dependent 16-byte loads per lane (pointer chase through the values: each waits for the last)
__global__ void k_chain(const uint4 * __restrict__ src, int * out, int n) {
    size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (int k = 0; k < n; k++) {
        const uint4 v = src[i];
        acc += v.x;
        i = (i + 4096 + (v.y & 1)) & ((1u << 24) - 1);
    }
    if (acc == 0x12345u) out[2] = 1;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    const size_t bytes = 1ull << 30;  // 1 GiB: rotated regions never sit in the 256 MB Infinity Cache
    uint4 * buf;
    int * out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMemset(buf, 0, bytes));
    CK(hipMalloc(&out, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 400;
    struct geo { int g, t; size_t lds; };
    const geo geos[] = {{256, 1024, 66 * 1024}, {256, 1024, 0}, {256, 256, 0}, {1024, 256, 0}, {2048, 512, 0}, {8, 64, 0}};
    for (const geo & G : geos) {
        const size_t per = (size_t) G.g * G.t;  // uint4 per launch
        const size_t regions = bytes / 16 / per;
        for (int kind = 0; kind < 2; kind++) {
            auto launch = [&](int r) {
                const uint4 * p = buf + (size_t) (r % regions) * per;
                if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(G.g), dim3(G.t), G.lds, s, out);
                else hipLaunchKernelGGL(k_load1, dim3(G.g), dim3(G.t), G.lds, s, p, out);
            };
            for (int r = 0; r < 20; r++) launch(r);
            CK(hipStreamSynchronize(s));
            CK(hipEventRecord(e0, s));
            for (int r = 0; r < reps; r++) launch(r);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("%-6s grid %5d x %4d, LDS %6zu: %6.2f us per launch\n", kind ? "load1" : "empty", G.g, G.t, G.lds, ms * 1e3 / reps);
        }
    }
    // dependent HBM round trips inside one kernel (latency under a chip-wide load)
    for (int n : {1, 4, 16}) {
        for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k_chain, dim3(256), dim3(256), 0, s, buf, out, n);
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < 100; r++) hipLaunchKernelGGL(k_chain, dim3(256), dim3(256), 0, s, buf, out, n);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("chain  %2d dependent loads, grid 256 x 256: %6.2f us per launch\n", n, ms * 1e3 / 100);
    }
    return 0;
}
