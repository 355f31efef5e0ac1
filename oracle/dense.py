"""ORACLE (test infrastructure only) - dense float64 restatement of the
diff-gaussian-rasterization-w-pose forward, differentiated by torch autograd.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker.  The
product path (``wildgs-slam-blackwell_amd/``) never imports it.

Source status: the CUDA rasteriser the reference uses
(``thirdparty/diff-gaussian-rasterization-w-pose``, .gitmodules:7-9) is an
empty submodule in the reference snapshot, so this restates the public
upstream algorithm and is pinned by
* the reference helpers it mirrors, checked against the reference itself by
  ``tests/golden/make_fixtures.py``: SH basis and constants
  (thirdparty/gaussian_splatting/utils/sh_utils.py:24-119), quaternion ->
  rotation (general_utils.py:113-136), ``SE3_exp``
  (src/utils/pose_utils.py:66-78), projection / view matrices
  (graphics_utils.py:33-93, camera_utils.py:137-151);
* the caller's contract (gaussian_renderer/__init__.py:24-153): output
  5-tuple, NDC units of the means2D gradient (gaussian_model.py:745-749),
  pose delta semantics new_w2c = SE3_exp([rho, theta]) @ w2c
  (pose_utils.py:81-98, camera_utils.py:69-74).
Parity with the CUDA binary itself is therefore *unpinned* (no golden vectors
exist in the reference: SURVEY.md 4); see DESIGN.md "Oracle".

Deliberate deviations from plain autograd, each matching upstream behaviour
(SURVEY.md Appendix A, V-items):
  V2  the gradient of the ``opacity`` output image is not propagated;
  V3  ``campos`` is a constant (no SH-direction pose term);
  V4  alpha = min(0.99, o G) is differentiated as if unclamped;
  V5  parity fixtures use a centred principal point;
  V8  (clamped frustum Jacobian) when |t.x/t.z| > 1.3 tanfovx the clamped
      t.x is a constant (upstream's x_grad_mul), same for y;
  V9  dL/dscales is the gradient w.r.t. scale_modifier * scales (upstream's
      computeCov3D backward omits the modifier's chain factor).
"""
from __future__ import annotations

import math

import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005,
         -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658,
         0.3731763325901154, -0.4570457994644658, 1.445305721320277,
         -0.5900435899266435]

BLOCK = 16  # tile edge (A.1)
NEAR_F32 = 0.20000000298023224  # float32(0.2): the near-plane cull constant


def eval_sh(deg: int, sh: torch.Tensor, dirs: torch.Tensor) -> torch.Tensor:
    """sh [P,K,3] (coefficient-major like the rasteriser), dirs [P,3] -> [P,3].

    Same polynomial as sh_utils.py:54-119 (which takes [...,3,K])."""
    res = SH_C0 * sh[:, 0]
    if deg > 0:
        x, y, z = dirs[:, 0:1], dirs[:, 1:2], dirs[:, 2:3]
        res = res - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
        if deg > 1:
            xx, yy, zz = x * x, y * y, z * z
            xy, yz, xz = x * y, y * z, x * z
            res = (res + SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5]
                   + SH_C2[2] * (2.0 * zz - xx - yy) * sh[:, 6]
                   + SH_C2[3] * xz * sh[:, 7] + SH_C2[4] * (xx - yy) * sh[:, 8])
            if deg > 2:
                res = (res + SH_C3[0] * y * (3 * xx - yy) * sh[:, 9]
                       + SH_C3[1] * xy * z * sh[:, 10]
                       + SH_C3[2] * y * (4 * zz - xx - yy) * sh[:, 11]
                       + SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12]
                       + SH_C3[4] * x * (4 * zz - xx - yy) * sh[:, 13]
                       + SH_C3[5] * z * (xx - yy) * sh[:, 14]
                       + SH_C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return res


def quat_to_rot(q: torch.Tensor) -> torch.Tensor:
    """general_utils.py:127-135 without the re-normalisation (A.2 step 3:
    the rasteriser does not normalise; the caller already did)."""
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
        2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
        2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y),
    ], dim=1).reshape(-1, 3, 3)
    return R


def skew(v: torch.Tensor) -> torch.Tensor:
    z = torch.zeros((), dtype=v.dtype)
    return torch.stack([
        torch.stack([z, -v[2], v[1]]),
        torch.stack([v[2], z, -v[0]]),
        torch.stack([-v[1], v[0], z]),
    ])


def se3_exp(tau: torch.Tensor) -> torch.Tensor:
    """pose_utils.py:30-78, differentiable at tau = 0 (small-angle branch)."""
    rho, theta = tau[:3], tau[3:]
    W = skew(theta)
    W2 = W @ W
    I = torch.eye(3, dtype=tau.dtype)
    angle = torch.norm(theta.detach())
    if angle < 1e-5:
        R = I + W + 0.5 * W2
        V = I + 0.5 * W + (1.0 / 6.0) * W2
    else:
        a = torch.norm(theta)
        R = I + (torch.sin(a) / a) * W + ((1 - torch.cos(a)) / a**2) * W2
        V = I + W * ((1 - torch.cos(a)) / a**2) + W2 * ((a - torch.sin(a)) / a**3)
    top = torch.cat([R, (V @ rho)[:, None]], dim=1)
    bottom = torch.tensor([[0.0, 0.0, 0.0, 1.0]], dtype=tau.dtype)
    return torch.cat([top, bottom], dim=0)


def rasterize_dense(means3D, means2D, opacities, shs, colors_precomp, scales, rotations,
                    cov3D_precomp, tau, *, H, W, tanfovx, tanfovy, bg, scale_modifier,
                    viewmatrix, projmatrix, projmatrix_raw, sh_degree, campos, touch_threshold=0.5):
    """Dense forward.  All tensor arguments float64 (leaf tensors may require
    grad).  ``tau`` = [rho(3), theta(3)] (pose delta, zero in every caller).

    Returns dict(color[3,H,W], depth[1,H,W], opacity[1,H,W], radii[P] int,
    n_touched[P] int, num_rendered int).
    """
    dt = torch.float64
    P = means3D.shape[0]
    view_rm = viewmatrix.to(dt)       # row-vector storage of W2C (V^T)
    proj_rm = projmatrix.to(dt)       # row-vector storage of (P W2C)
    Praw = projmatrix_raw.to(dt).T    # column-vector P
    W2C = view_rm.T
    dT = se3_exp(tau) - torch.eye(4, dtype=dt)  # zero-valued, carries d/dtau
    # p_view = (SE3_exp(tau) W2C) x ; p_hom = P (SE3_exp(tau) W2C) x
    # with tau = 0 these equal the given matrices bit for bit (V-matrix values
    # are taken from the f32 inputs, only the derivative comes from tau).
    Vfull = W2C + dT @ W2C
    Pfull = proj_rm.T + Praw @ dT @ W2C
    xh = torch.cat([means3D, torch.ones(P, 1, dtype=dt)], dim=1)
    p_view = xh @ Vfull.T  # [P,4]
    p_hom = xh @ Pfull.T
    p_w = 1.0 / (p_hom[:, 3:4] + 1e-7)
    p_proj = p_hom[:, :3] * p_w

    # ---- covariance (A.2 steps 3-5)
    if cov3D_precomp is not None and cov3D_precomp.numel() > 0:
        c6 = cov3D_precomp
        Sigma = torch.stack([c6[:, 0], c6[:, 1], c6[:, 2], c6[:, 1], c6[:, 3], c6[:, 4],
                             c6[:, 2], c6[:, 4], c6[:, 5]], dim=1).reshape(-1, 3, 3)
    else:
        R = quat_to_rot(rotations)
        # V9: upstream returns dL/d(scale_modifier * scales) as dL/dscales
        s = scale_modifier * scales.detach() + (scales - scales.detach())
        Sigma = R @ torch.diag_embed(s * s) @ R.transpose(1, 2)
    fx = W / (2.0 * tanfovx)
    fy = H / (2.0 * tanfovy)
    limx = 1.3 * tanfovx
    limy = 1.3 * tanfovy
    # V8: the EWA Jacobian sees the frustum-clamped mean t_c; its pose
    # derivative is rho + theta x t_c (upstream: -skew(t) of the clamped t).
    t0 = (xh @ W2C.T)[:, :3]
    with torch.no_grad():
        txtz = t0[:, 0] / t0[:, 2]
        tytz = t0[:, 1] / t0[:, 2]
        clx = (txtz < -limx) | (txtz > limx)
        cly = (tytz < -limy) | (tytz > limy)
        tc_val = torch.stack([txtz.clamp(-limx, limx) * t0[:, 2],
                              tytz.clamp(-limy, limy) * t0[:, 2], t0[:, 2]], dim=1)
        tc_val = torch.where(torch.stack([clx, cly, torch.zeros_like(clx)], 1), tc_val, t0)
    t = t0 + (torch.cat([tc_val, torch.ones(P, 1, dtype=dt)], 1) @ dT.T)[:, :3]
    tz = t[:, 2]
    tx = torch.where(clx, (txtz.clamp(-limx, limx) * tz).detach(), t[:, 0])
    ty = torch.where(cly, (tytz.clamp(-limy, limy) * tz).detach(), t[:, 1])
    zero = torch.zeros_like(tz)
    J = torch.stack([fx / tz, zero, -fx * tx / (tz * tz),
                     zero, fy / tz, -fy * ty / (tz * tz)], dim=1).reshape(-1, 2, 3)
    Wrot = Vfull[:3, :3]
    Tm = J @ Wrot
    cov2 = Tm @ Sigma @ Tm.transpose(1, 2)
    a = cov2[:, 0, 0] + 0.3
    b = cov2[:, 0, 1]
    c = cov2[:, 1, 1] + 0.3
    det = a * c - b * b
    conic = torch.stack([c / det, -b / det, a / det], dim=1)

    # ---- screen position in NDC + means2D (whose gradient is dL/d ndc)
    ndc = p_proj[:, :2] + means2D[:, :2]
    xy = torch.stack([((ndc[:, 0] + 1.0) * W - 1.0) * 0.5,
                      ((ndc[:, 1] + 1.0) * H - 1.0) * 0.5], dim=1)

    # ---- integer decisions (no grad)
    with torch.no_grad():
        visible = p_view[:, 2] > NEAR_F32  # upstream compares in float: z <= 0.2f
        visible &= det != 0
        mid = 0.5 * (a + c)
        disc = torch.clamp(mid * mid - det, min=0.1).sqrt()
        lam = torch.maximum(mid + disc, mid - disc)
        radius = torch.ceil(3.0 * torch.sqrt(lam))
        gx, gy = (W + BLOCK - 1) // BLOCK, (H + BLOCK - 1) // BLOCK
        r_int = torch.where(torch.isfinite(radius), radius, torch.zeros_like(radius)).to(torch.int64)
        xyd = xy.detach()

        def trunc(v):
            return torch.trunc(v).to(torch.int64)
        rminx = trunc((xyd[:, 0] - r_int) / BLOCK).clamp(0, gx)
        rminy = trunc((xyd[:, 1] - r_int) / BLOCK).clamp(0, gy)
        rmaxx = trunc((xyd[:, 0] + r_int + BLOCK - 1) / BLOCK).clamp(0, gx)
        rmaxy = trunc((xyd[:, 1] + r_int + BLOCK - 1) / BLOCK).clamp(0, gy)
        area = (rmaxx - rminx) * (rmaxy - rminy)
        visible &= area > 0
        radii = torch.where(visible, r_int, torch.zeros_like(r_int))
        tiles = torch.where(visible, area, torch.zeros_like(area))

    # ---- colour
    if colors_precomp is not None and colors_precomp.numel() > 0:
        rgb = colors_precomp
    else:
        K = (sh_degree + 1) ** 2
        dirs = means3D - campos.to(dt).detach()[None, :]
        dirs = dirs / dirs.norm(dim=1, keepdim=True)
        rgb = torch.clamp_min(eval_sh(sh_degree, shs[:, :K], dirs) + 0.5, 0.0)
    depth = p_view[:, 2]
    opac = opacities.reshape(-1)

    # ---- per-tile compositing (A.3), depth order stable by index
    gx, gy = (W + BLOCK - 1) // BLOCK, (H + BLOCK - 1) // BLOCK
    key = depth.detach().to(torch.float32)
    order = torch.from_numpy(
        __import__("numpy").lexsort((torch.arange(P).numpy(), key.numpy())))
    order = order[visible[order]]
    out_c = [[None] * gx for _ in range(gy)]
    out_d = [[None] * gx for _ in range(gy)]
    out_t = [[None] * gx for _ in range(gy)]
    n_touched = torch.zeros(P, dtype=torch.int64)
    bgd = bg.to(dt)
    o_minx, o_maxx = rminx[order], rmaxx[order]
    o_miny, o_maxy = rminy[order], rmaxy[order]
    for ty_ in range(gy):
        for tx_ in range(gx):
            x0, y0 = tx_ * BLOCK, ty_ * BLOCK
            x1, y1 = min(x0 + BLOCK, W), min(y0 + BLOCK, H)
            npx = (x1 - x0) * (y1 - y0)
            sel = (o_minx <= tx_) & (tx_ < o_maxx) & (o_miny <= ty_) & (ty_ < o_maxy)
            L = order[sel]
            if L.numel() == 0:
                out_c[ty_][tx_] = bgd[:, None].expand(3, npx)
                out_d[ty_][tx_] = torch.zeros(1, npx, dtype=dt)
                out_t[ty_][tx_] = torch.ones(1, npx, dtype=dt)
                continue
            py, px = torch.meshgrid(torch.arange(y0, y1, dtype=dt),
                                    torch.arange(x0, x1, dtype=dt), indexing="ij")
            px, py = px.reshape(-1, 1), py.reshape(-1, 1)
            dx = xy[L, 0][None, :] - px
            dy = xy[L, 1][None, :] - py
            con = conic[L]
            power = -0.5 * (con[:, 0][None] * dx * dx + con[:, 2][None] * dy * dy) \
                - con[:, 1][None] * dx * dy
            G = torch.exp(power)
            araw = opac[L][None] * G
            alpha = araw - torch.relu(araw - 0.99).detach()           # V4
            with torch.no_grad():
                valid = (power <= 0) & (alpha >= 1.0 / 255.0)
            alpha_v = torch.where(valid, alpha, torch.zeros_like(alpha))
            one_m = 1.0 - alpha_v
            Tinc = torch.cumprod(one_m, dim=1)
            Tbef = torch.cat([torch.ones(npx, 1, dtype=dt), Tinc[:, :-1]], dim=1)
            with torch.no_grad():
                stop = valid & (Tinc < 1e-4)
                keep = torch.cumsum(stop.to(torch.int64), dim=1) == 0
            w = alpha_v * Tbef * keep
            Cc = w @ rgb[L]                       # [npx,3]
            Dd = w @ depth[L][:, None]            # [npx,1]
            Tf = torch.prod(torch.where(keep, one_m, torch.ones_like(one_m)), dim=1, keepdim=True)
            with torch.no_grad():
                touched = keep & valid & (Tinc > touch_threshold)
                n_touched.index_add_(0, L, touched.sum(0))
            out_c[ty_][tx_] = (Cc + Tf * bgd[None, :]).T
            out_d[ty_][tx_] = Dd.T
            out_t[ty_][tx_] = Tf.T

    def assemble(parts, ch):
        rows = []
        for ty_ in range(gy):
            y0, y1 = ty_ * BLOCK, min(ty_ * BLOCK + BLOCK, H)
            cols = [parts[ty_][tx_].reshape(ch, y1 - y0, -1) for tx_ in range(gx)]
            rows.append(torch.cat(cols, dim=2))
        return torch.cat(rows, dim=1)

    color = assemble(out_c, 3)
    depth_img = assemble(out_d, 1)
    T_img = assemble(out_t, 1)
    return dict(color=color, depth=depth_img, opacity=1.0 - T_img,
                radii=radii.to(torch.int32), n_touched=n_touched.to(torch.int32),
                num_rendered=int(tiles.sum()), tiles_touched=tiles,
                # per-Gaussian geometry (detached; tests cross-check it against
                # the reference-held shader text, tests/test_shader_crosscheck.py)
                cov2d=torch.stack([a, b, c], dim=1).detach(), conic=conic.detach(), xy=xy.detach(),
                rgb=rgb.detach(), visible=visible)


def dense_forward_backward(scene: dict, settings: dict, grad_color, grad_depth):
    """Run the dense forward, backprop (dL/dcolor, dL/ddepth) and return
    forward outputs + gradients in the layout of
    ``_C.rasterize_gaussians_backward``."""
    dt = torch.float64

    def leaf(x):
        if x is None or x.numel() == 0:
            return None
        return x.detach().to(dt).clone().requires_grad_(True)

    means3D = leaf(scene["means3D"])
    P = means3D.shape[0]
    means2D = torch.zeros(P, 3, dtype=dt, requires_grad=True)
    opac = leaf(scene["opacities"])
    shs = leaf(scene.get("shs"))
    colors = leaf(scene.get("colors_precomp"))
    scales = leaf(scene.get("scales"))
    rots = leaf(scene.get("rotations"))
    cov = leaf(scene.get("cov3D_precomp"))
    tau = torch.zeros(6, dtype=dt, requires_grad=True)
    out = rasterize_dense(means3D, means2D, opac, shs, colors, scales, rots, cov, tau,
                          **settings)
    loss = (out["color"] * grad_color.to(dt)).sum() + (out["depth"] * grad_depth.to(dt)).sum()
    if loss.requires_grad:  # nothing visible -> every gradient is zero
        loss.backward()

    def g(x, shape):
        if x is None:
            return torch.zeros(shape, dtype=dt)
        return x.grad if x.grad is not None else torch.zeros(shape, dtype=dt)

    res = {k: v.detach() if torch.is_tensor(v) else v for k, v in out.items()}
    res.update(
        dL_dmeans3D=g(means3D, (P, 3)), dL_dmeans2D=g(means2D, (P, 3)),
        dL_dopacity=g(opac, (P, 1)), dL_dsh=g(shs, (P, 1, 3)) if shs is not None else None,
        dL_dcolors=g(colors, (P, 3)) if colors is not None else None,
        dL_dscales=g(scales, (P, 3)) if scales is not None else None,
        dL_drotations=g(rots, (P, 4)) if rots is not None else None,
        dL_dcov3D=g(cov, (P, 6)) if cov is not None else None,
        dL_dtau=tau.grad.detach().clone() if tau.grad is not None else torch.zeros(6, dtype=dt),
    )
    return res
