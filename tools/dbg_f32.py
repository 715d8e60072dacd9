# debug: GPU f32 mul_mat vs reference CPU for small K, element-level
import sys, numpy as np
sys.path.insert(0, 'ggml-imax_amd')
from ggml_mi355x import ggml as G, synth
rt = G.runtime()
be = G.mi355x_backend(rt)
ref = G.Lib(['oracle/_ref/libggml_ref.so'], isolated=True)
cpu = ref.ggml_backend_cpu_init()
for K in (8, 13, 32, 37):
    N, B = 21, 3
    w = synth.uniform(11 + K, K * N); x = synth.uniform(12 + K, K * B)
    y = G.mul_mat_once(rt, be, 0, w.view(np.uint8), K, N, x, B).reshape(B, N)
    yr = G.mul_mat_once(ref, cpu, 0, w.view(np.uint8), K, N, x, B).reshape(B, N)
    d = np.argwhere(y != yr)
    print(K, "mismatch", len(d), d[:5].tolist(), [(float(y[i, j]), float(yr[i, j])) for i, j in d[:3]])
    wn = w.reshape(N, K); xn = x.reshape(B, K)
    print("   np.dot f64 of first mismatching:", [float(np.dot(wn[j].astype(np.float64), xn[i].astype(np.float64))) for i, j in d[:3]])
