"""sdp -- MI355X-native simultaneous-diffusion sampling hot path (score net, Langevin, merge).

Host mirror of the reference's sampling interface over the C ABI of libsdp.so
(include/sdp.h).  Heavy modules are imported lazily so that the CPU-only pieces
(weights, config) work without a GPU.
"""
from .weights import get_sigmas_np, param_spec, synthetic_state_dict  # noqa: F401

__all__ = ["ScoreNet", "Merger", "anneal_Langevin_dynamics_inpainting",
           "anneal_Langevin_dynamics_inpainting_simultaneous_basic_kitti",
           "anneal_Langevin_dynamics_inpainting_simultaneous_basic", "get_sigmas_np", "param_spec",
           "synthetic_state_dict"]


def __getattr__(name):
    if name == "ScoreNet":
        from .scorenet import ScoreNet
        return ScoreNet
    if name == "Merger":
        from .merge import Merger
        return Merger
    if name.startswith("anneal_"):
        from . import sampling
        return getattr(sampling, name)
    raise AttributeError(name)
