"""Point cloud -> range image on the GPU: the data front end of the KITTI-360 datasets
(SURVEY §8(f)-1).  ``point_cloud_to_range_image`` keeps the signature and return tuple of
LiDARGen/datasets/lidar_utils.py:54-347 (numpy in, numpy out, float64 images flipped in both
axes); the work runs in ``sdp_range_project`` (csrc/projection.hip).  ``project_device``
is the device-tensor form for callers that keep the scan in HBM.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


def project_device(points: torch.Tensor, origin, H: int = 64, W: int = 1024, with_intensity: bool = True):
    """points: cuda float64 [N, >=3 or >=4]; returns dict of cuda tensors (depth, intensity, obf, sky, index)."""
    if not points.is_cuda or points.dtype != torch.float64 or points.dim() != 2:
        raise ValueError("project_device expects a cuda float64 [N, C] tensor")
    points = points.contiguous()
    N, stride = points.shape
    dev = points.device
    depth = torch.empty(H, W, dtype=torch.float64, device=dev)
    inten = torch.empty(H, W, dtype=torch.float64, device=dev) if with_intensity else None
    obf = torch.empty(H, W, dtype=torch.uint8, device=dev)
    sky = torch.empty(H, W, dtype=torch.uint8, device=dev)
    index = torch.empty(H, W, dtype=torch.int64, device=dev)
    n = _lib.SZ()
    L = _lib.lib()
    _lib.check(L.sdp_range_project_workspace_size(H, W, _lib.C.byref(n)), "range_project_ws")
    ws = torch.empty(n.value, dtype=torch.uint8, device=dev)
    o = np.ascontiguousarray(np.asarray(origin, dtype=np.float64).reshape(3))
    _lib.check(L.sdp_range_project(points.data_ptr() if N else None, N, stride, 1 if with_intensity else 0,
                                   o.ctypes.data, H, W, depth.data_ptr(), _lib.ptr(inten), obf.data_ptr(),
                                   sky.data_ptr(), index.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream()),
               "range_project")
    return dict(depth=depth, intensity=inten, obf=obf, sky=sky, index=index)


def point_cloud_to_range_image(point_cloud, origin, return_remission=False, return_points=False,
                               provided_origin=False, rowMax=64, colMax=1024, saveNum=0, device="cuda"):
    """lidar_utils.py:54-347: returns (depth, intensity, obfuscationMask, saveNum, skyMask, indices)
    with return_remission, else (depth, obfuscationMask, saveNum, skyMask, indices)."""
    pc = torch.as_tensor(np.ascontiguousarray(np.asarray(point_cloud, dtype=np.float64)), device=device)
    r = project_device(pc, origin, rowMax, colMax, with_intensity=bool(return_remission))
    depth = r["depth"].cpu().numpy()
    obf = r["obf"].cpu().numpy().astype(bool)
    sky = r["sky"].cpu().numpy().astype(bool)
    index = r["index"].cpu().numpy().astype(np.float64)
    if return_remission:
        return depth, r["intensity"].cpu().numpy(), obf, saveNum, sky, index
    return depth, obf, saveNum, sky, index
