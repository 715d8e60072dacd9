// kernarg_probe.hip -- what a dependent kernel pays before its first useful load: a producer kernel
// writes a buffer, the probe kernel (launched behind it on the same stream) reads it. Stamps
// (s_memrealtime, 100 MHz) per workgroup: entry, the loaded value landed, exit; plus the
// producer's exit, so the boundary gap is visible too. Built twice by tools/kernarg_probe.sh:
// plain, and with the kernel arguments preloaded into SGPRs (-mllvm -amdgpu-kernarg-preload-count),
// which removes the scalar load of the argument block (an HBM round trip) from the critical path.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_produce(int * __restrict__ buf, int n, int v, uint64_t * __restrict__ st) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) buf[i] = v + i;
    __syncthreads();
    if (threadIdx.x == 0) st[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}

__global__ void k_probe(const int * __restrict__ src, int * __restrict__ out, uint64_t * __restrict__ st) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const int v = src[blockIdx.x * blockDim.x + threadIdx.x];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (v == 0x7fffffff) out[0] = v;
    if (threadIdx.x == 0) {
        st[3 * blockIdx.x] = t0;
        st[3 * blockIdx.x + 1] = t1;
        st[3 * blockIdx.x + 2] = __builtin_amdgcn_s_memrealtime();
    }
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    const int grid = 256, block = 256, n = grid * block;
    int *buf, *out;
    uint64_t *st_p, *st_q;
    CK(hipMalloc(&buf, n * 4));
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&st_p, grid * 8));
    CK(hipMalloc(&st_q, 3 * grid * 8));
    std::vector<uint64_t> hp(grid), hq(3 * grid);
    std::vector<double> first_load, gap, span;
    for (int rep = 0; rep < 50; rep++) {
        hipLaunchKernelGGL(k_produce, dim3(grid), dim3(block), 0, s, buf, n, rep, st_p);
        hipLaunchKernelGGL(k_probe, dim3(grid), dim3(block), 0, s, buf, out, st_q);
        CK(hipStreamSynchronize(s));
        if (rep < 10) continue;
        CK(hipMemcpy(hp.data(), st_p, grid * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hq.data(), st_q, 3 * grid * 8, hipMemcpyDeviceToHost));
        uint64_t pend = 0, qs = ~0ull, qe = 0;
        std::vector<double> fl;
        for (int b = 0; b < grid; b++) {
            pend = std::max(pend, hp[b]);
            qs = std::min(qs, hq[3 * b]);
            qe = std::max(qe, hq[3 * b + 2]);
            fl.push_back((hq[3 * b + 1] - hq[3 * b]) * 0.01);
        }
        std::sort(fl.begin(), fl.end());
        first_load.push_back(fl[grid / 2]);
        gap.push_back(((double) qs - (double) pend) * 0.01);
        span.push_back((qe - qs) * 0.01);
    }
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    printf("producer exit -> probe entry %.2f us; probe entry -> first load landed (median WG) %.2f us; probe span %.2f us\n",
           med(gap), med(first_load), med(span));
    return 0;
}
