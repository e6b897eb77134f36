"""Records per merge tile (output view, big-grid row) and per-wave cell collisions for the bench geometry (32-view megabatch, 4 output views): the numbers behind the merge tile passes."""
import sys, numpy as np, torch
sys.path[:0] = ["/root/repo", "/root/repo/simultaneous-diffusion-for-pointclouds_amd"]
from oracle import sampling_ref as S
from sdp.synthetic import scene_views, exist_mask
H, W, n = 64, 1024, 32
sc = scene_views(n, H, W)
g = torch.Generator().manual_seed(1234)
x = torch.rand(n, 2, H, W, generator=g).numpy()
G = S.merge_geometry(H, W); smod = S.sigma_mod_of(0.5)
rd = S.real_distance(x[:, 0], smod).astype(np.float64)
caz, saz = np.cos(G["az"])[None, None, :], np.sin(G["az"])[None, None, :]
cel, sel = np.cos(G["el"])[None, :, None], np.sin(G["el"])[None, :, None]
P = np.stack([(rd*caz*cel).reshape(n,-1), (rd*saz*cel).reshape(n,-1), (rd*sel).reshape(n,-1), np.ones((n,H*W))],1)
Pw = np.einsum("bij,bjn->bin", sc["toWorld"], P)
ex = exist_mask(H, W)[:n].reshape(-1) if exist_mask(H, W).ndim == 3 else np.tile(exist_mask(H,W).reshape(-1), n)
thr = np.float64(S.min_depth_threshold(smod))
counts = []
for o in range(4):
    q = np.einsum("ij,vjn->vin", sc["fromWorld"][o], Pw)[:, :3].transpose(1,0,2).reshape(3,-1)
    row, col, d = S._bin(q, G)
    ell = np.log2(d+1)/6*np.float64(smod)
    valid = (col > -1) & (col < W) & (row > -1) & (row < G["big"]) & (ell > thr)
    c = np.bincount(row[valid].astype(int), minlength=G["big"])
    counts.append(c)
c = np.concatenate(counts)
print("total records", c.sum(), "pairs", 4*n*H*W, "tiles", c.size, "nonzero", (c>0).sum())
print("max", c.max(), "pcts", np.percentile(c, [50, 75, 90, 99]))
print(sorted(c)[-20:])
# conflicts inside 64-record groups of the biggest tile, records in source order
for o in range(1):
    q = np.einsum("ij,vjn->vin", sc["fromWorld"][o], Pw)[:, :3].transpose(1,0,2).reshape(3,-1)
    row, col, d = S._bin(q, G)
    ell = np.log2(d+1)/6*np.float64(smod)
    valid = (col > -1) & (col < W) & (row > -1) & (row < G["big"]) & (ell > thr)
    rows = row[valid].astype(int); cols = col[valid].astype(int)
    big = np.bincount(rows).argmax()
    cc = cols[rows == big]
    print("tile row", big, "records", cc.size, "distinct cols", np.unique(cc).size)
    n = cc.size // 64 * 64
    g = cc[:n].reshape(-1, 64)
    mult = np.array([np.bincount(x).max() for x in g])
    print("per-wave max multiplicity: mean", mult.mean(), "pcts", np.percentile(mult, [50, 90, 99]))
    hist = np.bincount(cc, minlength=W); print("top cells", np.sort(hist)[-5:], "median", np.median(hist))
