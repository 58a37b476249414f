"""Write-bandwidth reference: torch fill_ of a 7.05 GB buffer (the dense CifHr map's size),
HIP events, best of 10 -- the practical ceiling for a pure streaming write on this GPU."""
import torch

n = 7_050_000_000
buf = torch.empty(n, dtype=torch.uint8, device='cuda')
for _ in range(3):
    buf.fill_(0)
torch.cuda.synchronize()
best = 1e9
for _ in range(10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    buf.fill_(0)
    e1.record()
    e1.synchronize()
    best = min(best, e0.elapsed_time(e1))
print('fill_ {:.3f} ms -> {:.0f} GB/s'.format(best, n / (best * 1e-3) / 1e9))
