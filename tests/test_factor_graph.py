"""Device-resident FactorGraph mirror (mast3r_slam_amd/factor_graph.py,
SURVEY §8f #3): CPU checks of the two-way edge store and the reference's edge
filter (global_opt.py:56-100), GPU check of solve_GN_* against the drop-in
entry point on the reference's prep_two_way_edges tensors, and against the
CPU oracle fed the reference's concatenated two-way edge order (all i->j,
then all j->i; global_opt.py:104-110)."""
import numpy as np
import pytest
import torch

from mast3r_slam_amd import factor_graph as fgm
from mast3r_slam_amd import synthetic


def _halves(g):
    E = g.n_edges // 2
    s = slice(0, E)
    r = slice(E, 2 * E)
    return (g.ii[s], g.jj[s], g.idx_ii2jj[s], g.idx_ii2jj[r], g.valid_match[s], g.valid_match[r],
            g.Q[s], g.Q[r])


def test_edge_store_two_way_layout_and_growth():
    g = synthetic.make_graph(6, 8, 8, seed=3)
    ii, jj, i2j, j2i, vj, vi, Qj, Qi = _halves(g)
    st = fgm.EdgeStore(64, "cpu", capacity=2)
    st.append(ii[:3], jj[:3], i2j[:3], j2i[:3], vj[:3], vi[:3], Qj[:3], Qi[:3])
    st.append(ii[3:], jj[3:], i2j[3:], j2i[3:], vj[3:], vi[3:], Qj[3:], Qi[3:])
    dii, djj, didx, dv, dQ = st.directed()
    E = ii.numel()
    assert st.capacity >= E and dii.numel() == 2 * E
    assert torch.equal(dii[0::2], ii) and torch.equal(dii[1::2], jj)
    assert torch.equal(djj[0::2], jj) and torch.equal(djj[1::2], ii)
    assert didx.dtype == torch.int32  # the store's int32 match indices (m3s_gn_args.idx_i32)
    assert torch.equal(didx[0::2].long(), i2j) and torch.equal(didx[1::2].long(), j2i)
    assert torch.equal(dv[1::2], vi) and torch.equal(dQ[0::2], Qj)
    assert didx.is_contiguous() and dv.is_contiguous() and dQ.is_contiguous()


def test_add_factors_filter():
    """global_opt.py:56-78: an edge needs both directions above min_match_frac,
    consecutive edges are always kept; is_reloc rejects any invalid edge."""
    HW = 16
    kf = fgm.KeyframeStore(4, 4, "cpu", capacity=8)
    fg = fgm.FactorGraph(kf)
    ii, jj = [0, 0, 2], [1, 2, 3]
    idx = torch.zeros(3, HW, dtype=torch.int64)
    good = torch.ones(3, HW, 1, dtype=torch.bool)
    bad = good.clone()
    bad[1] = False  # edge (0, 2): no valid matches, not consecutive -> dropped
    bad[0] = False  # edge (0, 1): consecutive -> kept anyway
    Q = torch.full((3, HW, 1), 2.0)
    assert fg.add_factors(ii, jj, idx, idx, good, bad, Q, Q, 0.1)
    assert fg.ii_u.tolist() == [0, 2] and fg.jj_u.tolist() == [1, 3]
    assert fg.edges.n == 2
    assert not fg.add_factors(ii, jj, idx, idx, good, bad, Q, Q, 0.1, is_reloc=True)
    assert fg.edges.n == 2
    assert fg.get_unique_kf_idx().tolist() == [0, 1, 2, 3]


def test_keyframe_store_keeps_gn_inputs_current():
    """Cn = C / N and Xr = constrain_points_to_ray(X) are kept on every write
    (append, set_pointmap after a fusion), and a solve over contiguous
    keyframes gets views of them: no per-solve copy."""
    from oracle.tracker_oracle import constrain_points_to_ray

    H, W = 6, 8
    g = synthetic.make_graph(5, H, W, seed=3)
    kf = fgm.KeyframeStore(H, W, "cpu", capacity=8, K=g.K)
    for k in range(5):
        kf.append(g.Xs[k], g.Cs[k] * 3.0, g.T_init.data[k], N=3)
    kf.set_pointmap(2, g.Xs[2] * 1.5, g.Cs[2] * 4.0, 4)
    for k in range(5):
        scale = 1.5 if k == 2 else 1.0
        np.testing.assert_allclose(kf.Cn[k].numpy(), g.Cs[k].numpy(), rtol=1e-6)
        ref = constrain_points_to_ray((H, W), (g.Xs[k] * scale).numpy(), g.K.numpy())
        np.testing.assert_allclose(kf.Xr[k].numpy(), ref, rtol=1e-6, atol=1e-7)
    fg = fgm.FactorGraph(kf, K=g.K)
    uk = torch.arange(1, 4)
    for calib in (False, True):
        Xs, Cs, T, contiguous = fg._poses_points(uk, calib)
        assert contiguous
        assert Xs.data_ptr() == (kf.Xr if calib else kf.X)[1].data_ptr() and Cs.data_ptr() == kf.Cn[1].data_ptr()
        assert T.data_ptr() == kf.T_WC[1].data_ptr()


@pytest.mark.gpu
@pytest.mark.parametrize("calib", [False, True])
def test_solve_matches_dropin_on_reference_layout(calib):
    import mast3r_slam_backends as be

    dev = torch.device("cuda:0")
    N, H, W = 7, 24, 32
    g = synthetic.make_graph(N, H, W, seed=11, device=dev)
    kf = fgm.KeyframeStore(H, W, dev, capacity=16, K=g.K)
    for k in range(N):
        kf.append(g.Xs[k], g.Cs[k], g.T_init.data[k])
    fg = fgm.FactorGraph(kf, K=g.K)
    assert fg.add_factors(*_halves(g), min_match_frac=0.0)
    (fg.solve_GN_calib if calib else fg.solve_GN_rays)()
    # the reference's own call on its prep_two_way_edges / get_poses_points tensors
    c = fgm.LOCAL_OPT_CFG
    T = g.T_init.data.clone().contiguous()
    if calib:
        Xs = fgm.ray_constrained(g.Xs, g.K, H, W)
        be.gauss_newton_calib(T, Xs, g.Cs, g.K, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q, H, W,
                              c["pixel_border"], c["depth_eps"], c["sigma_pixel"], c["sigma_depth"],
                              c["C_conf"], c["Q_conf"], c["max_iters"], c["delta_norm"])
    else:
        be.gauss_newton_rays(T, g.Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q,
                             c["sigma_ray"], c["sigma_dist"], c["C_conf"], c["Q_conf"], c["max_iters"],
                             c["delta_norm"])
    torch.cuda.synchronize()
    np.testing.assert_allclose(kf.T_WC[:N].cpu().numpy(), T.cpu().numpy(), atol=1e-5)
    assert torch.equal(kf.T_WC[0], g.T_init.data[0])  # pinned


@pytest.mark.gpu
@pytest.mark.parametrize("calib", [False, True])
def test_solve_matches_oracle_on_reference_edge_order(calib):
    """The mirror (interleaved edge rows, int32 idx, keyframe views) against
    oracle/gn_oracle.c on the reference's own two-way layout (forward half then
    backward half, int64 idx): 10 GN iterations of LOCAL_OPT_CFG, poses within
    the backend's 10-iteration tolerance (1e-4 absolute)."""
    from oracle import oracle as orc
    from oracle.tracker_oracle import constrain_points_to_ray

    dev = torch.device("cuda:0")
    N, H, W = 7, 24, 32
    g = synthetic.make_graph(N, H, W, seed=13)
    kf = fgm.KeyframeStore(H, W, dev, capacity=16, K=g.K.to(dev))
    for k in range(N):
        kf.append(g.Xs[k].to(dev), g.Cs[k].to(dev), g.T_init.data[k].to(dev))
    fg = fgm.FactorGraph(kf, K=g.K.to(dev))
    assert fg.add_factors(*(t.to(dev) for t in _halves(g)), min_match_frac=0.0)
    (fg.solve_GN_calib if calib else fg.solve_GN_rays)()
    torch.cuda.synchronize()
    c = fgm.LOCAL_OPT_CFG
    if calib:
        p = orc.make_params(orc.MODE_CALIB, c["sigma_pixel"], c["sigma_depth"], c["C_conf"], c["Q_conf"],
                            K=g.K.numpy(), height=H, width=W, pixel_border=c["pixel_border"],
                            z_eps=c["depth_eps"])
        Xs = np.stack([constrain_points_to_ray((H, W), x, g.K.numpy()) for x in g.Xs.numpy()])
    else:
        p = orc.make_params(orc.MODE_RAYS, c["sigma_ray"], c["sigma_dist"], c["C_conf"], c["Q_conf"])
        Xs = g.Xs.numpy()
    T_ref, dx_ref, it, failed = orc.gn(p, g.T_init.data.numpy(), Xs, g.Cs.numpy(), g.ii.numpy(), g.jj.numpy(),
                                       g.idx_ii2jj.numpy(), g.valid_match.numpy(), g.Q.numpy(), c["max_iters"],
                                       c["delta_norm"])
    assert failed == 0
    np.testing.assert_allclose(kf.T_WC[:N].cpu().numpy(), T_ref, atol=1e-4)
