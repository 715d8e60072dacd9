// HBM streaming probe: back-to-back launches of a plain float4 read-reduce over 303 MB (one
// bench step's bytes), per-launch HIP-event durations, to see the chip's sustained-rate drift
// independently of the GEMV. Build: hipcc --offload-arch=gfx950 -O3 tools/stream_probe.hip -o tools/stream_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdint>
#include <cstdlib>

__global__ __launch_bounds__(256) void k_read(const float4 * __restrict__ x, size_t n4, float * out) {
    float s = 0.f;
    const size_t stride = (size_t) gridDim.x * blockDim.x;
    size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n4; i += 4 * stride) {
        const float4 a = x[i], b = x[i + stride], c = x[i + 2 * stride], d = x[i + 3 * stride];
        s += a.x + b.y + c.z + d.w;
    }
    for (; i < n4; i += stride) s += x[i].x;
    if (s == 12345.f) out[0] = s;
}

int main(int argc, char ** argv) {
    const size_t bytes = 303038464;
    const int iters = argc > 1 ? atoi(argv[1]) : 150;
    float4 * x; float * o;
    hipMalloc(&x, bytes); hipMalloc(&o, 4);
    {   // random bits (zero-filled data draws less power and runs faster)
        std::vector<uint32_t> h(bytes / 4);
        uint64_t st = 42;
        for (auto & v : h) { st = st * 6364136223846793005ull + 1442695040888963407ull; v = (uint32_t) (st >> 32); }
        hipMemcpy(x, h.data(), bytes, hipMemcpyHostToDevice);
    }
    std::vector<hipEvent_t> ev(iters + 1);
    for (auto & e : ev) hipEventCreate(&e);
    const int grid = 256 * 8;
    hipEventRecord(ev[0], 0);
    for (int i = 0; i < iters; i++) {
        hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, x, bytes / 16, o);
        hipEventRecord(ev[i + 1], 0);
    }
    hipDeviceSynchronize();
    float tot = 0;
    for (int i = 0; i < iters; i++) {
        float ms; hipEventElapsedTime(&ms, ev[i], ev[i + 1]);
        tot += ms;
        printf("%.1f%s", ms * 1e3, (i % 20 == 19) ? "\n" : " ");
    }
    printf("\nmean %.1f us  %.0f GB/s\n", tot / iters * 1e3, bytes / (tot / iters / 1e3) / 1e9);
    return 0;
}
