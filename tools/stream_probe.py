"""HBM streaming probe: back-to-back launches of a pure read reduction (torch sum over a
303 MB buffer, the size of one bench step) to see how the sustained rate drifts over time,
independent of our kernels. Run under rocprofv3 --kernel-trace."""
import torch
n = 303038464 // 4
x = torch.ones(n, device="cuda", dtype=torch.float32)
out = torch.empty((), device="cuda")
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(150):
    torch.sum(x, dim=0, out=out)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 150
print(f"sum: {ms * 1e3:.1f} us/launch  {n * 4 / ms / 1e6:.0f} GB/s")
