"""Score-net forward only (B views, 64x1024) -- a clean target for rocprofv3 PMC passes."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "simultaneous-diffusion-for-pointclouds_amd"))
import torch  # noqa: E402

from sdp.scorenet import ScoreNet  # noqa: E402

B = int(os.environ.get("B", "4"))
ITERS = int(os.environ.get("ITERS", "5"))
PREC = os.environ.get("PREC", "fp32x3")
net = ScoreNet(64, 1024, precision=PREC).load_synthetic()
x = torch.rand(B, 2, 64, 1024, device="cuda")
y = torch.full((B,), 100, dtype=torch.int64, device="cuda")
out = torch.empty_like(x)
net(x, y, out=out)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(ITERS):
    net(x, y, out=out)
torch.cuda.synchronize()
print(f"B={B} {PREC}: {(time.perf_counter() - t) / ITERS * 1e3:.2f} ms per forward")
