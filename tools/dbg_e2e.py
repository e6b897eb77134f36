import sys, os, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'simultaneous-diffusion-for-pointclouds_amd'); sys.path.insert(0, 'tests')
from oracle import golden_inputs as GI, scorenet_ref as R, sampling_ref as S
from sdp.sampling import anneal_Langevin_dynamics_inpainting_simultaneous_basic_kitti as samp
from sdp.scorenet import ScoreNet
from sdp.weights import get_sigmas_np, synthetic_state_dict
DEV='cuda:0'
f = np.load('tests/golden/kitti_e2e_b2_64x256.npz')
case = GI.merge_case("e2e", 2, 64, 256)
x0 = torch.from_numpy(GI.scorenet_input("e2e", 2, 64, 256)).to(DEV)
t = lambda a: torch.from_numpy(a).to(DEV)
P = R.to_torch_params(synthetic_state_dict(128))
def cpu_net(x, y):
    with torch.no_grad(): return R.scorenet_forward(P, x.cpu(), y.cpu())
gpu_net = ScoreNet(64, 256).load_synthetic()
def feed(tag):
    k=[0]
    def fn(shape):
        n = torch.from_numpy(GI.noise(tag, k[0], shape)); k[0]+=1; return n
    return fn
for name, net in (("cpu_net", cpu_net), ("gpu_net", gpu_net)):
    images, _, _ = samp(x0, t(case["ref"]), t(case["mask"]), t(case["sky"]), None, 2, 5, 10, net,
                        get_sigmas_np()[229:232], t(case["fromWorld"].reshape(2, 1, 4, 4)),
                        t(case["toWorld"].reshape(2, 1, 4, 4)), 2, n_steps_each=2, step_lr=6.2e-6,
                        existMask=t(case["exist"]), denoise=True, verbose=False, grad_ref=1,
                        correlation_coefficient=0.01, noise_fn=feed("e2e"))
    for i, (got, want) in enumerate(((images[0].numpy(), f["new"]), (images[-1].numpy(), f["final"]))):
        d = np.abs(got - want)
        print(name, i, 'maxdiff', d.max(), 'frac>1e-4', (d > 1e-4).mean(), 'per-chan', [float(d[:, c].max()) for c in range(2)])
        print('   got', got[0, 0, 10, :6], '\n   want', want[0, 0, 10, :6])
