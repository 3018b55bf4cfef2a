"""ATE (evo_ape -as restatement, mast3r_slam_amd/evaluate.py) on CPU.

evo is not installed and the reference holds no ATE fixtures, so the
restatement is checked by its defining properties: an exactly Sim(3)-related
trajectory has zero error and the transform is recovered; the alignment is a
least-squares optimum; reflections are excluded; the oracle GN lowers the ATE
of a perturbed synthetic graph."""
import numpy as np
import pytest
import torch

from mast3r_slam_amd import evaluate


def _rot(axis, ang):
    a = np.asarray(axis, np.float64)
    a = a / np.linalg.norm(a)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K


def _traj(P):
    T = np.zeros((P.shape[0], 8))
    T[:, :3] = P
    T[:, 6] = 1.0
    T[:, 7] = 1.0
    return T


def test_exact_sim3_is_recovered():
    rng = np.random.default_rng(0)
    P = rng.normal(size=(40, 3))
    R = _rot([0.3, -1.0, 0.5], 0.7)
    s, t = 2.5, np.array([0.1, -3.0, 0.4])
    Q = (s * (R @ P.T)).T + t
    s2, R2, t2 = evaluate.umeyama_sim3(P, Q)
    assert abs(s2 - s) < 1e-12
    np.testing.assert_allclose(R2, R, atol=1e-12)
    np.testing.assert_allclose(t2, t, atol=1e-12)
    assert evaluate.ate_rmse(_traj(P), _traj(Q)) < 1e-12
    # without scale correction a scaled copy keeps an error
    assert evaluate.ate_rmse(_traj(P), _traj(Q), correct_scale=False) > 0.1


def test_alignment_is_least_squares_optimum():
    rng = np.random.default_rng(1)
    P = rng.normal(size=(25, 3))
    Q = (1.3 * (_rot([1, 2, 3], 0.4) @ P.T)).T + 0.5 + 0.05 * rng.normal(size=(25, 3))
    s, R, t = evaluate.umeyama_sim3(P, Q)

    def cost(s_, R_, t_):
        return ((Q - ((s_ * (R_ @ P.T)).T + t_)) ** 2).sum()

    c0 = cost(s, R, t)
    assert np.sqrt(c0 / len(P)) == pytest.approx(evaluate.ate_rmse(_traj(P), _traj(Q)), rel=1e-12)
    for k in range(20):
        d = rng.normal(size=7) * 1e-3
        assert cost(s * np.exp(d[6]), _rot(d[3:6], np.linalg.norm(d[3:6])) @ R, t + d[:3]) >= c0


def test_reflection_is_excluded():
    rng = np.random.default_rng(2)
    P = rng.normal(size=(30, 3))
    Q = P * np.array([1.0, 1.0, -1.0])  # a mirror image is not a Sim(3)
    _, R, _ = evaluate.umeyama_sim3(P, Q)
    assert np.linalg.det(R) == pytest.approx(1.0, abs=1e-12)


def test_input_checks():
    with pytest.raises(ValueError):
        evaluate.umeyama_sim3(np.zeros((2, 3)), np.zeros((2, 3)))
    with pytest.raises(ValueError):
        evaluate.umeyama_sim3(np.zeros((5, 3)), np.zeros((4, 3)))


def test_oracle_gn_lowers_ate():
    """The restated backend (oracle) on a perturbed synthetic graph moves the
    keyframes towards the ground-truth trajectory."""
    from mast3r_slam_amd import synthetic
    from oracle import oracle as orc

    g = synthetic.make_graph(12, 96, 128, seed=41)  # smaller images leave the graph ill-posed
    p = orc.make_params(orc.MODE_RAYS, 0.003, 10.0, 0.0, 1.5)
    T, _, it, failed = orc.gn(p, g.T_init.data.numpy(), g.Xs.numpy(), g.Cs.numpy(), g.ii.numpy(),
                              g.jj.numpy(), g.idx_ii2jj.numpy(), g.valid_match.numpy(), g.Q.numpy(),
                              10, 0.0)
    assert failed == 0 and it == 10
    a0 = evaluate.ate_rmse(g.T_init.data, g.T_gt.data)
    a1 = evaluate.ate_rmse(torch.from_numpy(T), g.T_gt.data)
    assert a1 < 0.5 * a0
