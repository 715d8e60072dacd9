// launch_probe.hip -- per-kernel cost of a chain of dependent small kernels on one stream (the
// shape of a GPT-2 decode token: ~64 short kernels back to back), eager and hipGraph-replayed.
//   hipcc --offload-arch=gfx950 -O3 tools/launch_probe.hip -o tools/launch_probe && tools/launch_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

// y[i] = x[i] + 1 over n floats (the GPT-2 embedding add / a bias add)
__global__ void k_add1(const float * __restrict__ x, float * __restrict__ y, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = x[i] + 1.0f;
}

// a GEMV-shaped touch: every workgroup reads `bytes_per_wg` of w and writes one float
__global__ void k_touch(const uint4 * __restrict__ w, float * __restrict__ y, int u4_per_wg) {
    const uint4 * p = w + (size_t) blockIdx.x * u4_per_wg;
    uint32_t acc = 0;
    for (int i = threadIdx.x; i < u4_per_wg; i += blockDim.x) {
        const uint4 v = p[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) y[blockIdx.x] = 1.0f;  // keep the loads
    if (threadIdx.x == 0 && blockIdx.x == 0) y[gridDim.x] = (float) acc;
}

// the add with a large by-value argument block (as the backend's kernels take: tensor / epilogue
// descriptors), to see what the argument size costs per launch
struct big_args {
    const float * x;
    float * y;
    int n;
    char pad[240];
};
__global__ void k_add_big(big_args a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.n) a.y[i] = a.x[i] + 1.0f;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    float *a, *b;
    uint4 * w;
    const size_t wbytes = 256ull << 20;
    CK(hipMalloc(&a, 1 << 20));
    CK(hipMalloc(&b, 1 << 20));
    CK(hipMalloc(&w, wbytes));
    CK(hipMemset(w, 1, wbytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int chain = 64, reps = 50;

    auto run = [&](const char * name, auto launch_one) -> int {
        for (int r = 0; r < 3; r++) for (int k = 0; k < chain; k++) launch_one(k);
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < reps; r++) for (int k = 0; k < chain; k++) launch_one(k);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        // graph of one chain
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int k = 0; k < chain; k++) launch_one(k);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int r = 0; r < 3; r++) CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < reps; r++) CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float msg;
        CK(hipEventElapsedTime(&msg, e0, e1));
        printf("%-44s eager %6.2f us/kernel   graph %6.2f us/kernel\n", name, ms * 1e3 / (reps * chain), msg * 1e3 / (reps * chain));
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
        return 0;
    };
    if (run("add 768 floats, 1 WG x 256", [&](int k) { hipLaunchKernelGGL(k_add1, dim3(3), dim3(256), 0, s, (k & 1) ? b : a, (k & 1) ? a : b, 768); })) return 1;
    if (run("add 768 floats, 12 WG x 64", [&](int k) { hipLaunchKernelGGL(k_add1, dim3(12), dim3(64), 0, s, (k & 1) ? b : a, (k & 1) ? a : b, 768); })) return 1;
    if (run("add 768 floats, 1 WG x 512", [&](int k) { hipLaunchKernelGGL(k_add1, dim3(2), dim3(512), 0, s, (k & 1) ? b : a, (k & 1) ? a : b, 768); })) return 1;
    if (run("add 768 floats, 3 WG x 256, 256 B args", [&](int k) {
            big_args ba{(k & 1) ? b : a, (k & 1) ? a : b, 768, {}};
            hipLaunchKernelGGL(k_add_big, dim3(3), dim3(256), 0, s, ba); })) return 1;
    if (run("add 768 floats, 3 WG x 256, 256 B args, 16 KB LDS", [&](int k) {
            big_args ba{(k & 1) ? b : a, (k & 1) ? a : b, 768, {}};
            hipLaunchKernelGGL(k_add_big, dim3(3), dim3(256), 16384, s, ba); })) return 1;
    // GEMV-shaped: 192 / 576 / 768 one-wave workgroups each reading 6 KB / 1.5 KB (1.2-4.7 MB, distinct per kernel)
    for (int wgs : {192, 576, 768}) {
        for (int kb : {1536, 6144}) {
            const int u4 = kb / 16;
            char name[96];
            snprintf(name, sizeof name, "touch %d WG x 64, %d B each (%.1f MB)", wgs, kb, wgs * kb / 1e6);
            if (run(name, [&](int k) { hipLaunchKernelGGL(k_touch, dim3(wgs), dim3(64), 0, s, w + (size_t) (k % 40) * (wgs * u4), b, u4); })) return 1;
        }
    }
    return 0;
}
