"""CPU check of the host symbolic plan of the block-sparse LLT (the part of the
solver that replaces Eigen's SimplicialLLT analysis, gn_kernels.cu:132-153).

The plan is executed in numpy the way sparse_llt_kernel runs it (assembly
lists -> the 16 waves' list-scheduled DIAG(k) / OFF(i,k) / PART items, each waiting
for the blocks it reads -> back substitution in reverse level order); a
schedule that could deadlock fails the test on random SPD edge blocks, and the solution is compared with
a dense fp64 solve of the same assembled system.
"""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def be():
    import mast3r_slam_backends as be

    return be


def dense_system(N, ri, rj, Hjj, gj):
    n = 7 * (N - 1)
    H = np.zeros((n, n))
    g = np.zeros(n)
    for e, (a, b) in enumerate(zip(ri - 1, rj - 1)):
        if a == b:
            continue
        for x, y, s in ((a, a, 1), (b, b, 1), (a, b, -1), (b, a, -1)):
            if x >= 0 and y >= 0:
                H[7 * x:7 * x + 7, 7 * y:7 * y + 7] += s * Hjj[e]
        if a >= 0:
            g[7 * a:7 * a + 7] -= gj[e]
        if b >= 0:
            g[7 * b:7 * b + 7] += gj[e]
    return H, g


def run_plan(p, Hjj, gj):
    m, S = p["m"], p["S"]
    L = np.zeros((S, 7, 7))
    for s in range(S):
        for t in range(p["asm_ptr"][s], p["asm_ptr"][s + 1]):
            L[s] += Hjj[p["asm_edge"][t]] * (1 if s < m else -1)
    y = np.zeros((m, 7))
    for v in range(m):
        for t in range(p["g_ptr"][v], p["g_ptr"][v + 1]):
            ent = p["g_edge"][t]
            y[v] += gj[ent >> 1] * (1 if ent & 1 else -1)
    W = np.zeros((m, 7, 7))
    # the kernel's dataflow: 16 waves take items from the dispatch list
    # witems[0:wave_ptr[1]] in order (a shared counter) and wait on the blocks
    # an item reads. Simulated by stepping the waves round-robin; a full round
    # without progress would be a deadlock.
    sdone = np.zeros(S, bool)
    n_disp = p["wave_ptr"][1]
    held = [-1] * 16  # dispatch index a wave is working on
    nxt = 0

    T = len(p["task_dst"])
    NP = p["n_parts"]
    split = len(p["dpart_ptr"]) > 0
    pdone = np.zeros(NP, bool)
    parts = np.zeros((NP, 7, 7))
    pb = np.zeros((NP, 7))

    def dparts(k):
        return range(p["dpart_ptr"][k], p["dpart_ptr"][k + 1]) if split else range(0)

    def oparts(t):
        return range(p["opart_ptr"][t], p["opart_ptr"][t + 1]) if split else range(0)

    def tail(ps, q0):  # the updates a final item still applies itself
        return p["part_q1"][ps[-1]] if len(ps) else q0

    def ready(item):
        if item >= T:  # PART
            pi = item - T
            q = range(p["part_q0"][pi], p["part_q1"][pi])
            if p["part_tgt"][pi] < 0:
                return all(sdone[p["dtr_slot"][j]] for j in q)
            return all(sdone[p["tr_a"][j]] and sdone[p["tr_b"][j]] for j in q)
        if item < 0:
            k = -1 - item
            ps = dparts(k)
            return all(pdone[i] for i in ps) and all(
                sdone[p["dtr_slot"][q]] for q in range(tail(ps, p["dtr_ptr"][k]), p["dtr_ptr"][k + 1]))
        k = p["task_col"][item]
        ps = oparts(item)
        return sdone[k] and all(pdone[i] for i in ps) and all(
            sdone[p["tr_a"][q]] and sdone[p["tr_b"][q]]
            for q in range(tail(ps, p["task_tr_ptr"][item]), p["task_tr_ptr"][item + 1]))

    def run(item):
        if item >= T:
            pi = item - T
            for j in range(p["part_q0"][pi], p["part_q1"][pi]):
                if p["part_tgt"][pi] < 0:
                    A = L[p["dtr_slot"][j]]
                    parts[pi] -= A @ A.T
                    pb[pi] -= A @ y[p["dtr_p"][j]]
                else:
                    parts[pi] -= L[p["tr_a"][j]] @ L[p["tr_b"][j]].T
            pdone[pi] = True
        elif item < 0:
            k = -1 - item
            ps = dparts(k)
            D = L[k] + sum((parts[i] for i in ps), np.zeros((7, 7)))
            b = y[k] + sum((pb[i] for i in ps), np.zeros(7))
            for q in range(tail(ps, p["dtr_ptr"][k]), p["dtr_ptr"][k + 1]):
                A = L[p["dtr_slot"][q]]
                D -= A @ A.T
                b -= A @ y[p["dtr_p"][q]]
            Lk = np.linalg.cholesky(D)
            L[k] = Lk
            W[k] = np.linalg.inv(Lk)
            y[k] = W[k] @ b
            sdone[k] = True
        else:
            dst, k = p["task_dst"][item], p["task_col"][item]
            ps = oparts(item)
            A = L[dst] + sum((parts[i] for i in ps), np.zeros((7, 7)))
            for q in range(tail(ps, p["task_tr_ptr"][item]), p["task_tr_ptr"][item + 1]):
                A -= L[p["tr_a"][q]] @ L[p["tr_b"][q]].T
            L[dst] = A @ W[k].T
            sdone[dst] = True

    while nxt < n_disp or any(h >= 0 for h in held):
        progressed = False
        for w in range(16):
            if held[w] < 0 and nxt < n_disp:
                held[w], nxt = nxt, nxt + 1
                progressed = True
            if held[w] >= 0 and ready(p["witems"][held[w]]):
                run(p["witems"][held[w]])
                held[w] = -1
                progressed = True
        assert progressed, "wave schedule deadlocks"
    assert sorted(p["witems"].tolist()) == sorted(p["items"].tolist())
    nc = p["nc"]
    c0 = m - nc
    assert pdone.all()
    assert all(sdone[k] for k in range(c0))  # every non-tail block is final
    done = np.zeros(m, bool)
    if nc:
        # the kernel's dense tail (sparse_llt_kernel 1b), right-looking
        clq = p["clq"]
        ct0, bend = clq[2:2 + nc], clq[2 + nc:].reshape(nc, nc)

        def slot(i, j):  # block (c0 + i, c0 + j), i >= j
            return c0 + i if i == j else p["task_dst"][ct0[j] + i - j - 1]

        for ci in range(nc):  # B0: border updates (columns < c0)
            k = c0 + ci
            for q in range(p["dtr_ptr"][k], bend[ci, ci]):
                assert p["dtr_p"][q] < c0
                A = L[p["dtr_slot"][q]]
                L[k] -= A @ A.T
                y[k] -= A @ y[p["dtr_p"][q]]
            assert bend[ci, ci] == p["dtr_ptr"][k + 1] or p["dtr_p"][bend[ci, ci]] >= c0
            for ri in range(ci + 1, nc):
                t = ct0[ci] + ri - ci - 1
                assert p["task_col"][t] == k and p["task_dst"][t] == slot(ri, ci)
                for q in range(p["task_tr_ptr"][t], bend[ci, ri]):
                    L[slot(ri, ci)] -= L[p["tr_a"][q]] @ L[p["tr_b"][q]].T
        for ci in range(nc):  # B1
            k = c0 + ci
            Lk = np.linalg.cholesky(L[k])
            L[k], W[k] = Lk, np.linalg.inv(Lk)
            y[k] = W[k] @ y[k]
            for ri in range(ci + 1, nc):
                L[slot(ri, ci)] = L[slot(ri, ci)] @ W[k].T
                y[c0 + ri] -= L[slot(ri, ci)] @ y[k]
            for cc in range(ci + 1, nc):
                for rr in range(cc, nc):
                    L[slot(rr, cc)] -= L[slot(rr, ci)] @ L[slot(cc, ci)].T
        for ci in range(nc - 1, -1, -1):  # B2
            k = c0 + ci
            y[k] = W[k].T @ y[k]
            for cj in range(ci):
                y[c0 + cj] -= L[slot(ci, cj)].T @ y[k]
        done[c0:] = True
    for t in range(m - 1, -1, -1):
        k = p["lev_col"][t]
        if k >= c0:
            continue
        r = y[k].copy()
        for q in range(p["col_ptr"][k], p["col_ptr"][k + 1]):
            assert done[p["col_row"][q]]
            r -= L[p["col_slot"][q]].T @ y[p["col_row"][q]]
        y[k] = W[k].T @ r
        done[k] = True
    x = np.zeros((m, 7))
    for vn in range(m):
        x[p["perm"][vn]] = y[vn]
    return x.reshape(-1)


@pytest.mark.parametrize("N,seed,split,tail", [(2, 0, 0, 8), (5, 1, 0, 8), (32, 2, 0, 8), (70, 3, 0, 8),
                                               (32, 4, 2, 8), (70, 5, 3, 8), (128, 6, 8, 8), (70, 3, 0, 0),
                                               (128, 6, 8, 0), (40, 7, 0, 3), (90, 8, 4, 4)])
def test_plan_executes_to_dense_solution(be, N, seed, split, tail, knobs):
    knobs("dense_tail_min", str(tail))
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(N, 2, 2, seed=seed, edge_range=(0, 0), kf_ids=np.arange(N) * 3 + 5)
    import mast3r_slam_backends  # noqa: F401

    ii, jj = g.ii.numpy(), g.jj.numpy()
    u = np.unique(np.concatenate([ii, jj]))
    ri, rj = np.searchsorted(u, ii), np.searchsorted(u, jj)
    rng = np.random.default_rng(seed)
    E = len(ii)
    Hjj = np.zeros((E, 7, 7))
    for e in range(E):
        A = rng.standard_normal((7, 7))
        Hjj[e] = A @ A.T + 7 * np.eye(7)
    gj = rng.standard_normal((E, 7))
    p = be.sparse_plan(N, ri, rj, split, 4096 if split else 0)
    if split:
        assert p["n_parts"] > 0  # the split path is exercised
    assert p["m"] == N - 1
    assert sorted(p["perm"].tolist()) == list(range(N - 1))
    assert p["lev_ptr"][-1] == N - 1
    H, gv = dense_system(N, ri, rj, Hjj, gj)
    x = run_plan(p, Hjj, gj)
    np.testing.assert_allclose(x, np.linalg.solve(H, gv), rtol=1e-9, atol=1e-9)
    if tail and N >= 70:
        assert p["nc"] >= tail  # the dense tail is exercised


def test_plan_fill_is_sparse_on_loop_graph(be):
    """min-degree keeps fill far below dense on the C3 graph shape."""
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(32, 2, 2, seed=1003, edge_range=(0, 0))
    p = be.sparse_plan(32, g.ii.numpy(), g.jj.numpy())
    dense_slots = 31 * 32 // 2
    assert p["S"] < 0.4 * dense_slots
    assert p["levels"] < 31
