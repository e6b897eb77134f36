"""ORACLE (test infrastructure only) -- numpy restatement of the annealed-Langevin samplers
and the cross-view consistency merge.

Follows, with the reference's dtype semantics (float32 images, float64 projection):
  * Langevin update ...... LiDARGen/models/KITTISampling.py:133-156, models/__init__.py:1397-1416
  * kitti merge .......... LiDARGen/models/KITTISampling.py:160-490 (pose matrices)
  * AllForOne merge ...... LiDARGen/models/__init__.py:209-579 (origin offsets)
  * samplers ............. KITTISampling.py:6-513, models/__init__.py:112-602, :1385-1442

The reference sorts (argsort / 2 stable sorts / unique_consecutive) and sums duplicates
through sparse->dense; this restatement computes the same per-cell quantities with
scatter reductions (count, sum of log-depth, sum of intensity, nearest point).  Two
documented differences, both below the stated tolerances: duplicate sums are taken in
float64 (the reference sums intensities in float32 in depth order), and a tie between
equal nearest depths keeps the lowest source index (the reference's argsort is unstable,
so its choice is unspecified).  Pinned by tests/golden/merge_*.npz.
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32


# ----------------------------------------------------------------------------- geometry
def merge_geometry(H: int, W: int) -> dict:
    """Constants of KITTISampling.py:29-102 (identical in models/__init__.py:131-207)."""
    hA = math.radians(360) / W
    vA = math.radians(28) / H
    hMin = ((W * -180) // 360) * hA + hA / 2
    big = int((max(abs(-25), abs(3)) * 2) * H // 28)
    bigMin = (big // -2) * vA + vA / 2
    vMin = ((H * -25) // 28) * vA + vA / 2
    az = np.arange(W - 1, -1, -1) * hA + hMin
    el = np.arange(H - 1, -1, -1) * vA + vMin
    return dict(H=H, W=W, hA=hA, vA=vA, hMin=hMin, big=big, bigMin=bigMin, az=az, el=el)


def sigma_mod_of(sigma):
    """KITTISampling.py:124-126: sigmaMod = sigma if sigma > 1 else 1."""
    return F32(sigma) if sigma > 1 else F32(1.0)


def real_distance(x0: np.ndarray, smod) -> np.ndarray:
    """KITTISampling.py:164-166: (2^(|x|*6/smod) - 1) * (+1 | -1 for negative codes), float32."""
    v = (np.abs(x0) * F32(6)) / F32(smod)
    rd = np.exp2(v.astype(np.float64)).astype(F32) - F32(1)   # correctly rounded f32 2^v
    mod = np.where(x0 < 0, F32(-1), F32(1)).astype(F32)
    return (rd * mod).astype(F32)


def min_depth_threshold(smod) -> np.float32:
    """KITTISampling.py:272-274: log2(tensor(0.2)+1)/6*sigmaMod evaluated in float32."""
    l2 = F32(np.log2(np.float64(F32(F32(0.2) + F32(1)))))   # correctly rounded f32 log2
    return F32(F32(l2 / F32(6)) * F32(smod))


def _bin(q, g, raw=False):
    """Project relative points q [3,N] (float64) -> (row, col, logdepth-code before *smod); with
    raw=True also the unrounded bin coordinates (col, row) before rint."""
    xy = q[0] * q[0] + q[1] * q[1]
    d = np.sqrt(xy + q[2] * q[2])
    h = np.arctan2(q[1], q[0])
    e = np.arctan2(q[2], np.sqrt(xy))
    fc = (h - g["hMin"]) / g["hA"]
    fr = (e - g["bigMin"]) / g["vA"]
    col = np.rint(fc)
    row = np.rint(fr)
    col = (g["W"] - 1 - col)
    row = (g["big"] - 1 - row)
    if raw:
        return row, col, d, fc, fr
    return row, col, d


def _accumulate(row, col, ell, inten, valid, g):
    """Per-cell count / sum(l) / sum(I) / nearest point of one output view."""
    W, big = g["W"], g["big"]
    cells = big * W
    r = row[valid].astype(np.int64)
    c = col[valid].astype(np.int64)
    idx = r * W + c
    lv = ell[valid]
    iv = inten[valid].astype(np.float64)
    n = np.bincount(idx, minlength=cells)
    sl = np.bincount(idx, weights=lv, minlength=cells)
    si = np.bincount(idx, weights=iv, minlength=cells)
    # nearest point: smallest l, ties -> lowest source index
    order = np.lexsort((np.arange(idx.size), lv, idx))
    first = np.ones(order.size, bool)
    first[1:] = idx[order][1:] != idx[order][:-1]
    sel = order[first]
    lmin = np.zeros(cells)
    imin = np.zeros(cells, np.float32)
    lmin[idx[sel]] = lv[sel]
    imin[idx[sel]] = inten[valid][sel]
    return n, sl, si, lmin, imin


def _resolve(n, sl, si, lmin, imin, smod, allowance, controlled: bool):
    """KITTISampling.py:306-326 (controlled average) / models/__init__.py:441-481."""
    scaling = (n.astype(np.float32) + F32(1e-9)).astype(np.float32)
    A_code = sl / scaling.astype(np.float64)
    Ibar = (si / scaling.astype(np.float64)).astype(np.float32)
    if not controlled:
        return A_code, Ibar, n > 0
    A = np.power(2.0, np.abs(A_code) * 6 / np.float64(F32(smod))) - 1
    M = np.power(2.0, np.abs(lmin) * 6 / np.float64(F32(smod))) - 1
    cond = A > M + allowance
    I = np.where(cond, imin, Ibar).astype(np.float32)
    D = np.where(cond, M + allowance / 5, A)
    code = np.log2(D + 1) / 6 * np.float64(F32(smod))
    return code, I, n > 0


def _crop_flip(code, I, cm, isneg_o, g):
    """Crop rows big-H.. and use flip(roll(., W/2)) for negative pixels (KITTISampling.py:349-358)."""
    H, W, big = g["H"], g["W"], g["big"]
    code = code.reshape(big, W)
    I = I.reshape(big, W)
    cm = cm.reshape(big, W)
    top = slice(big - H, big)
    fcode = np.flip(np.roll(code, W // 2, axis=1), axis=0)[top]
    fI = np.flip(np.roll(I, W // 2, axis=1), axis=0)[top]
    fcm = np.flip(np.roll(cm, W // 2, axis=1), axis=0)[top]
    depth = np.where(isneg_o, -fcode, code[top])
    inten = np.where(isneg_o, fI, I[top])
    cmask = np.where(isneg_o, fcm, cm[top])
    return depth, inten, cmask


def _apply(x, new, maskimg, sky, refmask, too_high, cc):
    """KITTISampling.py:411-490: correction on unknown pixels, zeroed when tooHigh."""
    m = np.logical_and(maskimg[:, None], sky)  # [B,1,H,W]
    corr = -(m.astype(np.int32) * (1 - (refmask != 0)).astype(np.int32)).astype(np.float32) * (x - new)
    if too_high:
        corr = np.zeros_like(corr)
    return (x + F32(cc) * corr).astype(np.float32)



# ----------------------------------------------------------------------------- parity flags
# "exact mask and row/col bins; ties excluded".  A device merge computes the same
# float64 projection from the same float32 image, except that its float32 exp2 (the real distance,
# KITTISampling.py:164-166) may differ from the correctly rounded one by an ulp of 2^v and its float64
# atan2 by an ulp.  flag_cells marks every destination cell whose result such a perturbation can
# change: a point whose (row, col, validity) moves when its real distance moves by 2 ulp of (rd + 1)
# either way, or whose bin coordinate sits within 1e-9 of a rounding edge; a nearest-depth tie (the
# runner-up's code interval reaches the winner's); and a controlled-average branch
# (KITTISampling.py:306-326) that the code intervals can flip.  Everywhere else a device merge must
# agree exactly in its mask and within float rounding in its values (tests/test_gpu_parity.py).
RD_ULPS = 2.0


def _rd_perturbed(rd32):
    """(rd - delta, rd + delta) in float64, delta = RD_ULPS ulp of float32(rd + 1) (the exp2 result)."""
    rd = rd32.astype(np.float64)
    dl = RD_ULPS * np.spacing(np.abs(rd32).astype(F32) + F32(1)).astype(np.float64)
    mag = np.abs(rd)
    sgn = np.where(rd < 0, -1.0, 1.0)
    return sgn * np.maximum(mag - dl, 0.0), sgn * (mag + dl)


def _cells_of(row, col, valid, g):
    return (row[valid].astype(np.int64) * g["W"] + col[valid].astype(np.int64))


def flag_cells(proj, smod, allowance, controlled, thr, extra_valid, g):
    """Uncertain destination cells of one output view.  proj(k) -> (row, col, d, fc, fr) of every source
    point for the nominal (k = 0), lowered (1) and raised (2) real distances; extra_valid: the
    geometry-free validity (exist / sky).  Returns a bool [big * W] grid."""
    W, big = g["W"], g["big"]
    cells = big * W
    ev = []
    for k in range(3):
        row, col, d, fc, fr = proj(k)
        ell = np.log2(d + 1) / 6 * np.float64(smod)
        valid = (col > -1) & (col < W) & (row > -1) & (row < big) & extra_valid
        if thr is not None:
            valid &= ell > thr
        ev.append((row, col, ell, valid, fc, fr))
    (r0, c0, l0, v0, fc0, fr0), (r1, c1, l1, v1, _, _), (r2, c2, l2, v2, _, _) = ev
    edge = (np.abs(fc0 - np.floor(fc0) - 0.5) < 1e-9) | (np.abs(fr0 - np.floor(fr0) - 0.5) < 1e-9)
    moved = (v0 != v1) | (v0 != v2) | (v0 & ((r0 != r1) | (c0 != c1) | (r0 != r2) | (c0 != c2))) | edge
    flag = np.zeros(cells, bool)
    for row, col, _, valid, _, _ in ev:
        m = moved & valid
        flag[_cells_of(row, col, m, g)] = True
    # code intervals of the points that stay in their cell
    lo, hi = np.minimum(np.minimum(l0, l1), l2), np.maximum(np.maximum(l0, l1), l2)
    v = v0
    idx = _cells_of(r0, c0, v, g)
    lv, lov, hiv = l0[v], lo[v], hi[v]
    n = np.bincount(idx, minlength=cells)
    # nearest-depth ties: the runner-up (by nominal code) reaches the winner's interval
    order = np.lexsort((np.arange(idx.size), lv, idx))
    si = idx[order]
    first = np.ones(order.size, bool)
    first[1:] = si[1:] != si[:-1]
    second = np.zeros(order.size, bool)
    second[1:] = (~first[1:]) & first[:-1]
    win = order[np.flatnonzero(second) - 1]
    run = order[second]
    tie = lov[run] <= hiv[win]
    flag[idx[run][tie]] = True
    if controlled:
        scaling = (n.astype(np.float32) + F32(1e-9)).astype(np.float64)
        a_lo = np.bincount(idx, weights=lov, minlength=cells) / scaling
        a_hi = np.bincount(idx, weights=hiv, minlength=cells) / scaling
        m_lo = np.zeros(cells)
        m_hi = np.zeros(cells)
        wsel = order[first]
        m_lo[idx[wsel]] = lov[wsel]
        m_hi[idx[wsel]] = hiv[wsel]
        sm = np.float64(F32(smod))
        f = lambda c: np.power(2.0, np.abs(c) * 6 / sm) - 1
        c_hi = f(a_hi) > f(m_lo) + allowance      # the branch at its most likely...
        c_lo = f(a_lo) > f(m_hi) + allowance      # ...and least likely ends
        a0 = np.bincount(idx, weights=lv, minlength=cells) / scaling    # nominal (summation order aside)
        m0 = np.zeros(cells)
        m0[idx[wsel]] = lv[wsel]
        edge = np.abs(f(a0) - (f(m0) + allowance)) <= 1e-9 * (f(m0) + allowance)
        flag |= (n > 0) & ((c_hi != c_lo) | edge)
    return flag


def _flag_pixels(cellflag, isneg_o, g):
    """Output pixels that read a flagged cell (the crop / flip of _crop_flip)."""
    z = np.zeros(cellflag.shape, np.float32)
    _, _, fl = _crop_flip(z, z, cellflag, isneg_o, g)
    return fl


def kitti_merge(x, refmask, sky, exist, toWorld, fromWorld, aB, sigma, setting=5, allowance=10, cc=0.01,
                absmax=None, views=None, flags=False):
    """One consistency merge of the pose-matrix sampler (KITTISampling.py:160-490).

    x f32 [B,2,H,W] (after the Langevin update); returns (newImages f32, x corrected f32).
    absmax: max|x[:,0]| over every view of the step when x holds only some of them.
    views: compute only these output views (the others come back unmerged) -- large megabatches.
    flags: also return the bool [B,H,W] pixels whose result a float-rounding perturbation of the
    projection can change (flag_cells); the same pixels of the corrected x follow them.
    """
    B, _, H, W = x.shape
    g = merge_geometry(H, W)
    smod = sigma_mod_of(sigma)
    x0 = x[:, 0]
    isneg = x0 < 0
    m = F32(np.abs(x0).max()) if absmax is None else F32(absmax)
    too_high = bool(F32(m * F32(6)) / F32(smod) > 50)
    rd32 = real_distance(x0, smod)
    caz, saz = np.cos(g["az"])[None, None, :], np.sin(g["az"])[None, None, :]
    cel, sel = np.cos(g["el"])[None, :, None], np.sin(g["el"])[None, :, None]

    def world(rd):
        P = np.stack([(rd * caz * cel).reshape(B, -1), (rd * saz * cel).reshape(B, -1),
                      (rd * sel).reshape(B, -1), np.ones((B, H * W))], 1)
        return np.einsum("bij,bjn->bin", toWorld, P)
    Pws = [world(rd32.astype(np.float64))]
    if flags:
        Pws += [world(r) for r in _rd_perturbed(rd32)]
    thr = np.float64(min_depth_threshold(smod))
    ex = exist[:aB].reshape(-1)
    new = np.zeros_like(x)
    maskimg = np.zeros((B, H, W), bool)
    flagged = np.zeros((B, H, W), bool)
    for o in (range(B) if views is None else views):
        m0 = (o // aB) * aB

        def proj(k, raw=False):
            src = Pws[k][m0:m0 + aB]                          # [aB,4,HW]
            q = np.einsum("ij,vjn->vin", fromWorld[o], src)[:, :3].transpose(1, 0, 2).reshape(3, -1)
            return _bin(q, g, raw)
        row, col, d = proj(0)
        ell = np.log2(d + 1) / 6 * np.float64(smod)
        valid = (col > -1) & (col < W) & (row > -1) & (row < g["big"]) & ex
        if setting == 5:
            valid &= ell > thr
        inten = x[m0:m0 + aB, 1].reshape(-1)
        acc = _accumulate(row, col, ell, inten, valid, g)
        code, I, cm = _resolve(*acc, smod, allowance, controlled=True)
        dep, inn, cmask = _crop_flip(code, I, cm, isneg[o], g)
        new[o, 0] = dep.astype(np.float32)
        new[o, 1] = inn
        maskimg[o] = np.logical_and(exist[0], cmask)
        if flags:
            cf = flag_cells(lambda k: proj(k, True), smod, allowance, True, thr if setting == 5 else None, ex, g)
            flagged[o] = _flag_pixels(cf, isneg[o], g)
    out = _apply(x, new, maskimg, sky, refmask, too_high, cc)
    return (new, out, flagged) if flags else (new, out)


def allforone_origins(mods) -> np.ndarray:
    """models/__init__.py:224-231 evaluated in float32: 10*sign(m) up to rounding."""
    m = np.asarray(mods, np.int64)
    # each transcendental in float64 then rounded: the correctly rounded float32 result
    l2 = np.log2((np.abs(m) + 1).astype(np.float64)).astype(np.float32)
    o = (l2 / F32(6)) * F32(1)
    o = np.exp2((o * F32(6)).astype(np.float32).astype(np.float64)).astype(np.float32) - F32(1)
    den = (m.astype(np.float32) + F32(1e-8)).astype(np.float32)
    return ((o / den).astype(np.float32) * F32(10)).astype(np.float32)


def allforone_merge(x, refmask, sky, exist, mods, aB, sigma, setting=7, cc=0.01, views=None, absmax=None,
                    flags=False):
    """One merge of the origin-offset sampler (models/__init__.py:263-579).  absmax, flags: as kitti_merge."""
    B, _, H, W = x.shape
    g = merge_geometry(H, W)
    smod = sigma_mod_of(sigma)
    x0 = x[:, 0]
    isneg = x0 < 0
    m = F32(np.abs(x0).max()) if absmax is None else F32(absmax)
    too_high = bool(F32(m * F32(6)) / F32(smod) > 50)
    rd32 = real_distance(x0, smod)
    rds = [rd32.astype(np.float64)] + (list(_rd_perturbed(rd32)) if flags else [])
    org = allforone_origins(mods).astype(np.float64)[:aB]       # [aB,3]
    caz, saz = np.cos(g["az"])[None, None, :], np.sin(g["az"])[None, None, :]
    cel, sel = np.cos(g["el"])[None, :, None], np.sin(g["el"])[None, :, None]
    thr = np.float64(min_depth_threshold(smod))
    ex = exist[:aB].reshape(-1)
    allowance = 5 if setting >= 8 else 10
    new = np.zeros_like(x)
    maskimg = np.zeros((B, H, W), bool)
    flagged = np.zeros((B, H, W), bool)
    for o in (range(B) if views is None else views):
        m0 = (o // aB) * aB
        oo = org[o - m0]

        def proj(k, raw=False):
            r = rds[k][m0:m0 + aB]
            px = (r * caz * cel + org[:, 0, None, None]).reshape(-1)
            py = (r * saz * cel + org[:, 1, None, None]).reshape(-1)
            pz = (r * sel + org[:, 2, None, None]).reshape(-1)
            return _bin(np.stack([px - oo[0], py - oo[1], pz - oo[2]]), g, raw)
        row, col, d = proj(0)
        ell = np.log2(d + 1) / 6 * np.float64(smod)
        valid = (col > -1) & (col < W) & (row > -1) & (row < g["big"])
        geo_free = sky[m0:m0 + aB].reshape(-1) & ex
        valid &= geo_free & (ell > thr)
        inten = x[m0:m0 + aB, 1].reshape(-1)
        acc = _accumulate(row, col, ell, inten, valid, g)
        code, I, cm = _resolve(*acc, smod, allowance, controlled=setting >= 7)
        dep, inn, cmask = _crop_flip(code, I, cm, isneg[o], g)
        new[o, 0] = dep.astype(np.float32)
        new[o, 1] = inn
        maskimg[o] = np.logical_and(exist[0], cmask)
        if flags:
            cf = flag_cells(lambda k: proj(k, True), smod, allowance, setting >= 7, thr, geo_free, g)
            flagged[o] = _flag_pixels(cf, isneg[o], g)
    out = _apply(x, new, maskimg, sky, refmask, too_high, cc)
    return (new, out, flagged) if flags else (new, out)


# ----------------------------------------------------------------------------- Langevin
def nan_to_num(g):
    """torch.nan_to_num defaults (KITTISampling.py:138): nan->0, +-inf -> +-float32 max."""
    return np.nan_to_num(g, nan=0.0, posinf=np.finfo(np.float32).max, neginf=np.finfo(np.float32).min).astype(F32)


def step_size_of(step_lr, sigma, sigma_last):
    """KITTISampling.py:135: step_lr * (sigma / sigmas[-1]) ** 2 in numpy float32."""
    return F32(step_lr) * (F32(sigma) / F32(sigma_last)) ** 2


def langevin_update(x, g, ref, mask, noise, step_size, grad_ref):
    """x + s*g + r*(-mask*(x-ref)) + noise*sqrt(2s), float32, reference evaluation order."""
    s = F32(step_size)
    lik = (-mask).astype(F32) * (x - ref)
    return (((x + s * g) + F32(grad_ref) * lik) + noise * F32(np.sqrt(F32(s * F32(2))))).astype(F32), lik


# ----------------------------------------------------------------------------- samplers
def sampler_baseline(x, ref, mask, score, sigmas, n_steps_each, step_lr, noise_fn, denoise=True, grad_ref=1.0):
    """anneal_Langevin_dynamics_inpainting (models/__init__.py:1385-1442); returns images list."""
    images = []
    lik = None
    for c, sigma in enumerate(sigmas):
        s = step_size_of(step_lr, sigma, sigmas[-1])
        for _ in range(n_steps_each):
            gr = score(x, np.full(x.shape[0], c, np.int64))
            x, lik = langevin_update(x, gr, ref, mask, noise_fn(x.shape), s, grad_ref)
            images.append(x.copy())
    if denoise:
        gr = score(x, np.full(x.shape[0], len(sigmas) - 1, np.int64))
        x = ((x + F32(sigmas[-1]) ** 2 * gr) + F32(grad_ref) * lik).astype(F32)
        images.append(x.copy())
    lik = (-mask).astype(F32) * (x - ref)
    x = (x + F32(grad_ref) * lik).astype(F32)
    images.append(x.copy())
    return images


def sampler_kitti(x, ref, mask, sky, min_step, setting, allowance, score, sigmas, fromWorld, toWorld, aB,
                  n_steps_each, step_lr, exist, noise_fn, denoise=True, grad_ref=1.0, cc=0.01):
    """anneal_Langevin_dynamics_inpainting_simultaneous_basic_kitti (KITTISampling.py:6-513)."""
    images, shared = [], []
    lik = None
    for c, sigma in enumerate(sigmas):
        if setting == 6:
            cc = 1 / (len(sigmas) / (c + 1))
        if setting == 7:
            cc = 0.5 / (len(sigmas) / (c + 1))
        s = step_size_of(step_lr, sigma, sigmas[-1])
        for _ in range(n_steps_each):
            gr = nan_to_num(score(x, np.full(x.shape[0], c, np.int64)))
            x, lik = langevin_update(x, gr, ref, mask, noise_fn(x.shape), s, grad_ref)
            if c >= min_step:
                new, x = kitti_merge(x, mask, sky, exist, toWorld, fromWorld, aB, sigma, setting, allowance, cc)
                if c in (0, 20, 110):
                    shared.append(new)
                if c == len(sigmas) - 1:
                    images.append(new)
    if denoise:
        gr = score(x, np.full(x.shape[0], len(sigmas) - 1, np.int64))
        x = ((x + F32(sigmas[-1]) ** 2 * gr) + F32(grad_ref) * lik).astype(F32)
    lik = (-mask).astype(F32) * (x - ref)
    x = (x + F32(grad_ref) * lik).astype(F32)
    images.append(x)
    return images, [], shared


def sampler_allforone(x, ref, mask, sky, min_step, setting, score, sigmas, mods, aB, n_steps_each, step_lr, exist,
                      noise_fn, denoise=True, grad_ref=1.0, cc=0.01):
    """anneal_Langevin_dynamics_inpainting_simultaneous_basic (models/__init__.py:112-602): the cc
    ramp of settings 5/6 (L209-212), per step score + nan_to_num + update (L236-259), from level
    minStepToShare on the origin-offset merge (L263-519; its newImages kept at levels 0/20/110 and
    the last, L505-508), denoise with the stale likelihood and the final data consistency (L580-599)."""
    images, shared = [], []
    lik = None
    L = len(sigmas)
    for c, sigma in enumerate(sigmas):
        if setting == 5:
            cc = 1 / (L / (c + 1))
        if setting == 6:
            cc = 0.5 / (L / (c + 1))
        s = step_size_of(step_lr, sigma, sigmas[-1])
        for _ in range(n_steps_each):
            gr = nan_to_num(score(x, np.full(x.shape[0], c, np.int64)))
            x, lik = langevin_update(x, gr, ref, mask, noise_fn(x.shape), s, grad_ref)
            if c >= min_step:
                new, x = allforone_merge(x, mask, sky, exist, mods, aB, sigma, setting, cc)
                if c in (0, 20, 110):
                    shared.append(new)
                if c == L - 1:
                    images.append(new)
    if denoise:
        gr = score(x, np.full(x.shape[0], L - 1, np.int64))
        x = ((x + F32(sigmas[-1]) ** 2 * gr) + F32(grad_ref) * lik).astype(F32)
    lik = (-mask).astype(F32) * (x - ref)
    x = (x + F32(grad_ref) * lik).astype(F32)
    images.append(x)
    return images, [], shared
