import torch, sys
sys.path.insert(0, "sam2-video-training_amd")
from sam2_video.kernels import ops
n = 80_800_000
p, g, m, v = (torch.randn(n, device="cuda") for _ in range(4)); v.abs_()
sh = torch.empty(n, device="cuda", dtype=torch.bfloat16)
for _ in range(3): ops.adamw(p, g, m, v, None, 1e-3, 0.9, 0.999, 1e-8, 0.01, 5, shadow=sh)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20): ops.adamw(p, g, m, v, None, 1e-3, 0.9, 0.999, 1e-8, 0.01, 5, shadow=sh)
e.record(); torch.cuda.synchronize()
t = s.elapsed_time(e) / 20
print(f"adamw {n/1e6:.1f} M params: {t*1e3:.1f} us, {30*n/t/1e9:.2f} TB/s (30 B/param)")
