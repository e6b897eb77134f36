"""A18: checkpoint load with the EMA shadow applied (runners/ncsn_runner_kitti_simultaneous.py:472-489,
models/ema.py:23-28).

The reference loads ``states[0]`` (keys ``module.``-prefixed by DataParallel) strictly, then
``EMAHelper.ema`` copies the shadow ``states[-1]`` (unprefixed keys, parameters only -- no
``sigmas`` buffer) over the parameters.  The checkpoint written here has a shadow that DIFFERS
from states[0], so a loader that ignored the shadow (or applied it partly) is caught: the
forward must match the oracle at the shadow weights (score-net tolerance 1e-4 of max) and must
NOT match it at states[0].
"""
import numpy as np
import pytest
import torch

from oracle import golden_inputs as GI

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
H, W = 64, 256


def _rel_err(out, ref):
    return max(np.abs(out[b] - ref[b]).max() / np.abs(ref[b]).max() for b in range(ref.shape[0]))


def test_checkpoint_forward_uses_the_ema_shadow(tmp_path):
    from oracle import scorenet_ref as R
    from sdp.scorenet import ScoreNet
    from sdp.weights import synthetic_state_dict
    sd = synthetic_state_dict(128)
    r = GI.rng("a18-shadow")
    # the shadow: every parameter moved by ~10 % of its own scale (sigmas is a buffer, not in it)
    shadow = {k: (v + 0.1 * np.abs(v).mean() * r.standard_normal(v.shape)).astype(np.float32)
              for k, v in sd.items() if k != "sigmas"}
    states = [{"module." + k: torch.from_numpy(v) for k, v in sd.items()},
              {"state": {}, "param_groups": [{"lr": 1e-4}]}, 3, 1000,
              {k: torch.from_numpy(v) for k, v in shadow.items()}]
    path = tmp_path / "checkpoint_1000.pth"
    torch.save(states, path)

    net = ScoreNet(H=H, W=W, precision="fp32x3").load_checkpoint(str(path))
    x = torch.from_numpy(GI.scorenet_input("a18", 2, H, W))
    y = torch.tensor([5, 200])
    out = net(x.to(DEV), y.to(DEV)).cpu().numpy()
    with torch.no_grad():
        want = R.scorenet_forward(R.to_torch_params({**sd, **shadow}), x, y).numpy()
        raw = R.scorenet_forward(R.to_torch_params(sd), x, y).numpy()
    err, err_raw = _rel_err(out, want), _rel_err(out, raw)
    print(f"vs shadow {err:.2e}, vs states[0] {err_raw:.2e}")
    assert err <= 1e-4
    assert err_raw > 1e-2              # the raw states[0] weights are NOT what runs
    # the sigma buffer comes from states[0] (the shadow holds no buffers)
    np.testing.assert_array_equal(net.sigmas.numpy(), sd["sigmas"])


def test_checkpoint_without_shadow_uses_states0(tmp_path):
    """A 4-element list (no EMA entry) loads states[0] as is (kitti:480-489 with ema off)."""
    from oracle import scorenet_ref as R
    from sdp.scorenet import ScoreNet
    from sdp.weights import synthetic_state_dict
    sd = synthetic_state_dict(128)
    torch.save([{"module." + k: torch.from_numpy(v) for k, v in sd.items()}, {}, 0, 0], tmp_path / "c.pth")
    net = ScoreNet(H=H, W=W, precision="fp32x3").load_checkpoint(str(tmp_path / "c.pth"))
    x = torch.from_numpy(GI.scorenet_input("a18b", 1, H, W))
    y = torch.tensor([17])
    out = net(x.to(DEV), y.to(DEV)).cpu().numpy()
    with torch.no_grad():
        want = R.scorenet_forward(R.to_torch_params(sd), x, y).numpy()
    assert _rel_err(out, want) <= 1e-4
