"""The CPU oracle against golden vectors produced by the reference's own Python
(tests/golden/make_golden.py) - this is what pins the oracle."""
import os

import numpy as np
import torch
import torch.nn.functional as F

from fill import det_state_dict
from oracle import corr as oc
from oracle import update_module as um


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def test_corr_pyramid_matches_reference(golden_dir):
    g = _load(golden_dir, "corr_pyramid.npz")
    pyr = oc.corr_pyramid(g["fmap1"].astype(np.float64), g["fmap2"].astype(np.float64))
    for i in range(4):
        ref = g["level%d" % i]
        assert pyr[i].shape == ref.shape
        np.testing.assert_allclose(pyr[i], ref, atol=5e-6, rtol=1e-5)


def test_alt_pyramid_matches_reference(golden_dir):
    g = _load(golden_dir, "alt_pyramid.npz")
    pyr = oc.alt_pyramid(g["fmaps"].astype(np.float64))
    for i in range(4):
        np.testing.assert_allclose(pyr[i], g["level%d" % i], atol=1e-6)


def test_volume_level_equals_feature_pyramid_dot(golden_dir):
    """level i of the volume == <f1/4, avgpool^i(f2/4)> (volume and alt paths agree)."""
    g = _load(golden_dir, "corr_pyramid.npz")
    f1 = g["fmap1"].astype(np.float64)
    f2 = g["fmap2"].astype(np.float64)
    pyr = oc.corr_pyramid(f1, f2)
    B, N, C, H, W = f1.shape
    alt2 = oc.alt_pyramid(f2)
    a1 = oc.alt_pyramid(f1)[0].reshape(B * N, H * W, C)
    for i in range(4):
        f2i = alt2[i].reshape(B * N, -1, C)
        vol = np.einsum("npc,nqc->npq", a1, f2i).reshape(pyr[i].shape)
        np.testing.assert_allclose(vol, pyr[i], atol=1e-9)


def test_update_module_matches_reference(golden_dir):
    u = _load(golden_dir, "update_module.npz")
    p = {k: torch.from_numpy(v) for k, v in det_state_dict(um.PARAM_SHAPES).items()}
    t = lambda k: torch.from_numpy(u[k])
    out = um.update_module(p, t("net"), t("inp"), t("corr"), t("flow"), t("ii"), t("jj"))
    for name, o in zip(["net_out", "delta", "weight", "eta", "upmask"], out):
        np.testing.assert_allclose(o.numpy(), u[name], atol=1e-5, rtol=1e-5)


def test_convgru_and_upsample_match_reference(golden_dir):
    c = _load(golden_dir, "convgru.npz")
    shapes = {}
    for n in ("convz", "convr", "convq"):
        shapes[n + ".weight"] = (16, 40, 3, 3)
        shapes[n + ".bias"] = (16,)
    for n in ("w", "convz_glo", "convr_glo", "convq_glo"):
        shapes[n + ".weight"] = (16, 16, 1, 1)
        shapes[n + ".bias"] = (16,)
    p = {k: torch.from_numpy(v) for k, v in det_state_dict(shapes).items()}
    o = um.conv_gru(p, "", torch.from_numpy(c["h"]), torch.from_numpy(c["x1"]), torch.from_numpy(c["x2"]))
    np.testing.assert_allclose(o.numpy(), c["out"], atol=1e-6)
    cu = _load(golden_dir, "cvx_upsample.npz")
    up = um.cvx_upsample(torch.from_numpy(cu["data"]), torch.from_numpy(cu["mask"]))
    np.testing.assert_allclose(up.numpy(), cu["up"], atol=1e-6)


def _grid_sample_lookup(vol, coords, r):
    B, H, W, H2, W2 = vol.shape
    vt = torch.from_numpy(vol.astype(np.float64)).reshape(B * H * W, 1, H2, W2)
    out = np.zeros((B, 2 * r + 1, 2 * r + 1, H, W))
    for i in range(2 * r + 1):
        for j in range(2 * r + 1):
            gx = torch.from_numpy((coords[:, 0] - r + i).astype(np.float64)).reshape(-1, 1, 1)
            gy = torch.from_numpy((coords[:, 1] - r + j).astype(np.float64)).reshape(-1, 1, 1)
            grid = torch.stack([2 * gx / (W2 - 1) - 1, 2 * gy / (H2 - 1) - 1], -1)
            s = F.grid_sample(vt, grid, align_corners=True, padding_mode="zeros")
            out[:, i, j] = s.reshape(B, H, W).numpy()
    return out


def test_lookup_equals_grid_sample(golden_dir):
    """corr_index_forward semantics == bilinear grid_sample(align_corners, zeros)
    sampled at (x0 - r + i, y0 - r + j), i the x offset."""
    g = _load(golden_dir, "corr_pyramid.npz")
    vol = g["level0"].astype(np.float32)
    B, H, W, H2, W2 = vol.shape
    rng = np.random.default_rng(0)
    base = np.stack(np.meshgrid(np.arange(W), np.arange(H)), 0)[None].astype(np.float32)
    coords = (base + rng.normal(0, 4, (B, 2, H, W))).astype(np.float32)
    out = oc.corr_index_forward(vol, coords, 3)
    ref = _grid_sample_lookup(vol, coords, 3)
    np.testing.assert_allclose(out, ref, atol=2e-5)


def test_fp16_lookup_is_half_rounded_fp32_lookup(golden_dir):
    g = _load(golden_dir, "corr_pyramid.npz")
    vol = g["level1"].astype(np.float32)
    B, H, W, H2, W2 = vol.shape
    rng = np.random.default_rng(1)
    coords = (rng.uniform(-3, max(H2, W2) + 3, (B, 2, H, W))).astype(np.float32)
    o16 = oc.corr_index_forward(vol.astype(np.float16), coords, 3)
    o32 = oc.corr_index_forward(vol.astype(np.float16).astype(np.float32), coords, 3)
    assert o16.dtype == np.float16
    np.testing.assert_allclose(o16.astype(np.float32), o32, atol=4e-3 * np.abs(o32).max())


def test_lookup_edge_cases():
    """far out-of-bounds coords give exact zeros; integer coords sample the taps."""
    rng = np.random.default_rng(2)
    vol = rng.normal(size=(1, 2, 3, 6, 7)).astype(np.float32)
    coords = np.full((1, 2, 2, 3), -100.0, dtype=np.float32)
    assert np.all(oc.corr_index_forward(vol, coords, 3) == 0)
    coords = np.zeros((1, 2, 2, 3), dtype=np.float32)
    coords[:, 0] = 3.0
    coords[:, 1] = 2.0
    out = oc.corr_index_forward(vol, coords, 1)
    for i in range(3):
        for j in range(3):
            np.testing.assert_allclose(out[0, i, j], vol[0, :, :, 2 - 1 + j, 3 - 1 + i], atol=1e-6)


# --- geom/projective_ops.py (reference, with a lietorch SE3 stand-in) -------
def _pops(golden_dir):
    return np.load(os.path.join(golden_dir, "projective_ops.npz"))


def test_oracle_projective_transform_matches_reference(golden_dir):
    """oracle/geometry.py (the reprojection the fused HIP kernel is checked
    against) vs projective_ops.projective_transform (:96-125): per-frame
    intrinsics, a stereo edge (the :105 override), the Z clamp and valid mask."""
    from oracle import geometry as og
    g = _pops(golden_dir)
    coords, valid = og.projective_transform(g["poses"], g["disps"], g["intrinsics"], g["ii"], g["jj"])
    np.testing.assert_array_equal(valid, g["valid"])
    np.testing.assert_allclose(coords, g["coords"], rtol=1e-5, atol=1e-4)


def test_oracle_ba_jacobians_match_reference(golden_dir):
    """The BA linearisation's per-pixel Jacobians (oracle/ba.py jacobians,
    restating droid_kernels.cu:281-330 incl. adjSE3) equal the reference's
    autograd-free Jacobian chain of projective_ops (jacobian=True: Jj = Jp Ja,
    Ji = -Gij.adjT(Jj), Jz = Jp (Gij * [0,0,0,1])) wherever both count the point
    (Z > 0.25, the kernel's MIN_DEPTH; the reference's own valid mask)."""
    from oracle import ba as oba
    g = _pops(golden_dir)
    E, H, W = g["Jj_shared"].shape[:3]
    J = oba.jacobians(g["poses"].astype(np.float64), g["disps"].astype(np.float64),
                      g["intrinsics"][0].astype(np.float64), g["ii"], g["jj"])
    use = (~J["bad"]).reshape(E, H, W) & (g["valid_shared"][..., 0] > 0)
    assert use.sum() > 0.7 * use.size
    ref_jj, ref_ji, ref_jz = g["Jj_shared"][use], g["Ji_shared"][use], g["Jz_shared"][use]   # (n,2,6), (n,2,1)
    ours_jj = np.stack([J["Jj_u"], J["Jj_v"]], -2).reshape(E, H, W, 2, 6)[use]
    ours_ji = np.stack([J["Ji_u"], J["Ji_v"]], -2).reshape(E, H, W, 2, 6)[use]
    ours_jz = np.stack([J["Jz_u"], J["Jz_v"]], -1).reshape(E, H, W, 2)[use]
    scale = max(1.0, np.abs(ref_jj).max())
    np.testing.assert_allclose(ours_jj, ref_jj, atol=1e-5 * scale)
    np.testing.assert_allclose(ours_ji, ref_ji, atol=1e-5 * scale)
    np.testing.assert_allclose(ours_jz, ref_jz[..., 0], atol=1e-5 * scale)
    np.testing.assert_allclose(J["coords"].reshape(E, H, W, 2)[use], g["coords_shared"][use], rtol=1e-5, atol=1e-4)


def test_torch_cpu_lookup_equals_kernel_restatement():
    """The CPU baseline's torch formulation (matmul / avg_pool2d / grid_sample)
    equals the loop restatement of CorrBlock + correlation_kernels.cu."""
    import torch
    from oracle import corr as oc
    rng = np.random.default_rng(12)
    f1 = rng.normal(size=(1, 2, 128, 16, 24)).astype(np.float32)
    f2 = rng.normal(size=(1, 2, 128, 16, 24)).astype(np.float32)
    coords = (np.stack(np.meshgrid(np.arange(24), np.arange(16)), -1)[None, None]
              + rng.normal(0, 3, (1, 2, 16, 24, 2))).astype(np.float32)
    ref = oc.lookup_pyramid(oc.corr_pyramid(f1, f2), coords, 3)[0]
    pyr = oc.corr_pyramid_torch(torch.from_numpy(f1), torch.from_numpy(f2))
    got = oc.lookup_pyramid_torch(pyr, torch.from_numpy(coords[0])).numpy()
    np.testing.assert_allclose(got, ref, atol=2e-5 * np.abs(ref).max())


def _proximity_case(z, c):
    g = lambda k: z["c%d_%s" % (c, k)]
    ei, ej, k1, k2 = g("ei"), g("ej"), int(g("k1")), int(g("k2"))
    args = dict(d=g("d"), t0=int(g("t0")), t1=int(g("t1")), t=int(g("t")), rad=int(g("rad")), nms=int(g("nms")),
                thresh=float(g("thresh")), ii_all=np.concatenate([ei[:k1], ei[k1:k2], ei[k2:]]),
                jj_all=np.concatenate([ej[:k1], ej[k1:k2], ej[k2:]]), stereo=bool(g("stereo")),
                max_factors=int(g("max_factors")))
    return args, np.stack([g("es_ii"), g("es_jj")], 1)


def test_oracle_proximity_edges_match_reference(golden_dir):
    """oracle.factor_graph.proximity_edges vs the reference's own
    add_proximity_factors (tests/golden/proximity.npz): the identical edge list
    for t0 > t1 (negative-index wrap), stereo, the max_factors cap, -1, NaN."""
    from oracle.factor_graph import proximity_edges
    z = np.load(os.path.join(golden_dir, "proximity.npz"))
    for c in range(int(z["ncases"])):
        args, ref = _proximity_case(z, c)
        np.testing.assert_array_equal(proximity_edges(**args), ref, err_msg="case %d" % c)


def _dense_ba_problem(golden_dir):
    """dense_ba.npz (geom/ba.py's undamped BA step, made by make_golden.py) as
    droid_backends.ba / oracle.ba arguments: t0 = fixedp = 1, one iteration,
    lm = ep = 0 (schur_solve damps H before the Schur complement, ba_cuda
    damps A - S after it: undamped they are the same step), geom's C + eta +
    1e-7 as eta + 1e-7, no sensor depth."""
    d = np.load(os.path.join(golden_dir, "dense_ba.npz"))
    prob = dict(poses=d["poses"][0], disps=d["disps"][0], intrinsics=d["intrinsics"][0][0],
                disps_sens=np.zeros_like(d["disps"][0]), targets=d["target"][0].transpose(0, 3, 1, 2),
                weights=d["weight"][0].transpose(0, 3, 1, 2), eta=d["eta"][0] + 1e-7, ii=d["ii"], jj=d["jj"],
                t0=1, t1=d["poses"].shape[1])
    return prob, d["ba_poses"][0], d["ba_disps"][0]


def test_oracle_ba_step_matches_reference_geom_ba(golden_dir):
    """The oracle's ba_cuda restatement (linearisation, block assembly, Schur
    complement, LLT, back-substitution, retraction) equals the reference's own
    geom/ba.py step to 1e-9 when the back-substitution keeps pose t0's rows.
    ba_cuda drops them (EvT6x1's idx <= 0 skip, droid_kernels.cu:1095-1115), so
    with that skip only the depth frames none of whose rows touch pose t0 (here
    4 and 5) still agree; frames 0-3 move by ~1e-2 (documented)."""
    from oracle import ba as oba
    prob, ref_poses, ref_disps = _dense_ba_problem(golden_dir)
    kw = dict(iterations=1, lm=0.0, ep=0.0, motion_only=False)
    full = oba.ba(**prob, **kw, skip_t0_backsub=False)
    np.testing.assert_allclose(full["poses"], ref_poses, atol=1e-9, rtol=0)
    np.testing.assert_allclose(full["disps"], ref_disps, atol=1e-9, rtol=0)
    cuda = oba.ba(**prob, **kw, skip_t0_backsub=True)
    np.testing.assert_allclose(cuda["poses"], ref_poses, atol=1e-9, rtol=0)
    np.testing.assert_allclose(cuda["disps"][4:], ref_disps[4:], atol=1e-9, rtol=0)
    assert np.abs(cuda["disps"][:4] - ref_disps[:4]).max() > 1e-3


def test_ate_matches_reference_evaluator(golden_dir):
    """oracle/ate.py vs the reference's ATEEvaluator (evaluator_base.py:33-55)
    on its own fixture pair: the known answers 0.8344983411575012 (scale,
    s = 1.0782526734172067) and 1.204507439280004 (no scale)."""
    from oracle import ate
    d = np.load(os.path.join(golden_dir, "tartanair_poses.npz"))
    e, s = ate.ate(d["pose_gt"], d["pose_est"], True)
    np.testing.assert_allclose(e, d["ate_scale"], rtol=1e-12)
    np.testing.assert_allclose(s, d["s_scale"], rtol=1e-12)
    np.testing.assert_allclose(e, 0.8344983411575012, rtol=1e-12)
    np.testing.assert_allclose(s, 1.0782526734172067, rtol=1e-12)
    e, s = ate.ate(d["pose_gt"], d["pose_est"], False)
    np.testing.assert_allclose(e, d["ate_noscale"], rtol=1e-12)
    np.testing.assert_allclose(e, 1.204507439280004, rtol=1e-12)
    assert s == 1.0
    # identical trajectories (any rigid motion + scale of the estimate) have zero ATE
    gt = d["pose_gt"][:50]
    R = np.array([[0.0, -1.0, 0.0], [1.0, 0.0, 0.0], [0.0, 0.0, 1.0]])
    est = gt.copy()
    est[:, :3] = (gt[:, :3] @ R.T + [1.0, 2.0, 3.0]) / 2.5
    assert ate.ate(gt, est, True)[0] < 1e-9
