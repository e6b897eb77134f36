"""bf16 training gradients vs the float32 oracle: cosine per parameter (the quantity
tests/test_gpu_training.py::test_bf16_training_gradients_close gates at 0.99); prints the worst 5."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "simultaneous-diffusion-for-pointclouds_amd"), REPO, os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import golden_inputs as GI  # noqa: E402
from oracle import scorenet_ref as R  # noqa: E402
from sdp.weights import synthetic_state_dict  # noqa: E402
import test_gpu_training as T  # noqa: E402

P = R.to_torch_params(synthetic_state_dict(128))
r = GI.rng("dsm_gpu")
B, H, W = T.B, T.H, T.W
X = torch.from_numpy(r.random((B, 2, H, W)).astype(np.float32))
noise = torch.from_numpy(r.standard_normal((B, 2, H, W)).astype(np.float32))
mask = torch.from_numpy((r.random((B, 2, H, W)) > 0.3).astype(np.float32))
labels = torch.tensor([3, 200])
used = P["sigmas"][labels].view(B, 1, 1, 1)
noise = noise * used
loss, scores, grads = R.dsm_loss_and_grads(P, X + noise, noise, mask, labels)
case = dict(X=X + noise, noise=noise, mask=mask, labels=labels, used=used, loss=loss, scores=scores, grads=grads)
for prec in sys.argv[1:] or ["bf16"]:
    _, _, l, _, g = T._run(case, prec)
    cos = sorted((torch.nn.functional.cosine_similarity(g[k].flatten(), v.flatten(), dim=0).item(), k)
                 for k, v in grads.items())
    print(prec, f"loss {l:.6f} ref {loss.item():.6f}", " ".join(f"{k}={c:.4f}" for c, k in cos[:5]))
