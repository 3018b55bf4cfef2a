"""GPU check of the edge-sharded GN (mast3r_slam_amd/distributed.py,
ShardedGN over HipOps, the stepwise C ABI) with REAL processes and a real
collective: two ranks spawned on the one GPU of the box, torch.distributed
over gloo (which all-gathers device tensors; RCCL refuses two ranks on one
device). This is the product path bench.py --gpus N runs, with the RCCL
all-gather replaced by gloo's. Both ranks must end with bitwise-identical
poses (nothing is broadcast in the real run), equal to those of the
in-process sharded run of tests/test_gpu_sharded.py (same slices, same
kernels, so bitwise as well), and close to the single-call drop-in.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _graph():
    from mast3r_slam_amd import synthetic

    return synthetic.make_graph(7, 48, 64, seed=41)


SIG = dict(sigma_a=0.003, sigma_b=10.0, C_thresh=0.0, Q_thresh=1.5)
ITERS = 5


def _rank_main(rank, world, port, out_dir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mast3r_slam_amd.distributed import ShardedGN, edge_shard

    dev = torch.device("cuda:0")
    g = _graph()
    E = g.n_edges
    ids, _ = edge_shard(E, rank, world)  # both halves of this rank's undirected edges
    Twc = g.T_init.data.clone().to(dev).contiguous()
    gn = ShardedGN(1, Twc, g.Xs.to(dev).contiguous(), g.Cs.to(dev).contiguous(), g.ii.to(dev), g.jj.to(dev),
                   g.idx_ii2jj[ids].to(dev).contiguous(), g.valid_match[ids].to(dev).contiguous(),
                   g.Q[ids].to(dev).contiguous(), E, **SIG)
    gn.solve(ITERS, 0.0)
    torch.cuda.synchronize()
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), Twc.cpu().numpy())
    np.save(os.path.join(out_dir, f"info{rank}.npy"), gn.info.cpu().numpy())
    gn.ops.close()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_processes_gloo_collective_match_in_process_and_single_call(tmp_path):
    import torch.multiprocessing as mp

    import mast3r_slam_backends as be

    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    poses = [np.load(tmp_path / f"rank{r}.npy") for r in range(world)]
    infos = [np.load(tmp_path / f"info{r}.npy") for r in range(world)]
    np.testing.assert_array_equal(poses[1], poses[0])
    for inf in infos:
        assert int(inf[be.INFO_ITERS]) == ITERS
        assert int(inf[be.INFO_SOLVE_FAIL]) == 0

    # the in-process sharded run (torch.cat in place of the collective)
    from test_gpu_sharded import sharded_solve

    g = _graph()
    dev = torch.device("cuda:0")
    ref, _ = sharded_solve(be, be.MODE_RAYS, g, g.Xs.to(dev).contiguous(), world, ITERS, 0.0, SIG)
    np.testing.assert_array_equal(poses[0], ref[0])

    # the single-call drop-in (fused per-edge finalize: different fp32 grouping)
    Twc = g.T_init.data.clone().to(dev).contiguous()
    info = torch.zeros(8, dtype=torch.int32, device=dev)
    args = [t.to(dev).contiguous() for t in (g.Cs, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q)]
    be.gauss_newton_rays(Twc, g.Xs.to(dev).contiguous(), *args, 0.003, 10.0, 0.0, 1.5, ITERS, 0.0, info=info)
    torch.cuda.synchronize()
    np.testing.assert_allclose(poses[0], Twc.cpu().numpy(), rtol=0, atol=1e-4)


def _rccl_main(rank, world, port, out_dir):
    """One rank over RCCL (backend "nccl"): the product's collective calls on
    device tensors (bench.py's --gpus N path: init with device_id, the
    all-gather of per-edge sums, the barrier and the max-over-ranks timing
    all-reduce). A one-GPU box cannot hold two RCCL ranks; one rank still runs
    RCCL's own init and kernels."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    from mast3r_slam_amd.distributed import ShardedGN

    g = _graph()
    E = g.n_edges
    Twc = g.T_init.data.clone().to(dev).contiguous()
    gn = ShardedGN(1, Twc, g.Xs.to(dev).contiguous(), g.Cs.to(dev).contiguous(), g.ii.to(dev), g.jj.to(dev),
                   g.idx_ii2jj.to(dev).contiguous(), g.valid_match.to(dev).contiguous(), g.Q.to(dev).contiguous(),
                   E, **SIG)
    gn.ops.prepare(0.0)
    gn.ops.linearize(0, E, gn.es_loc)
    es_all = torch.empty_like(gn.es_loc)
    dist.all_gather_into_tensor(es_all, gn.es_loc)
    dist.barrier()
    t = torch.tensor([1.5], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    torch.cuda.synchronize()
    np.save(os.path.join(out_dir, "rccl_es.npy"), gn.es_loc.cpu().numpy())
    np.save(os.path.join(out_dir, "rccl_es_all.npy"), es_all.cpu().numpy())
    np.save(os.path.join(out_dir, "rccl_meta.npy"), np.array([float(t.item()), dist.get_backend() == "nccl"]))
    gn.ops.close()
    dist.destroy_process_group()


def test_rccl_backend_collectives_on_device_tensors(tmp_path):
    import torch.multiprocessing as mp

    mp.start_processes(_rccl_main, args=(1, _free_port(), str(tmp_path)), nprocs=1, join=True,
                       start_method="spawn")
    es = np.load(tmp_path / "rccl_es.npy")
    es_all = np.load(tmp_path / "rccl_es_all.npy")
    meta = np.load(tmp_path / "rccl_meta.npy")
    assert meta[1] == 1.0 and meta[0] == 1.5
    assert np.isfinite(es).all() and np.abs(es).max() > 0
    np.testing.assert_array_equal(es_all, es)
