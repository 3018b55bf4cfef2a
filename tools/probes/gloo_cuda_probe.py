import os, sys
import torch, torch.distributed as dist
import torch.multiprocessing as mp
def run(rank, world):
    os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = "29533"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x = torch.full((4, 3), float(rank), dtype=torch.float64, device="cuda:0")
    out = torch.empty(4 * world, 3, dtype=torch.float64, device="cuda:0")
    try:
        dist.all_gather_into_tensor(out, x)
        print(rank, "all_gather_into_tensor cuda ok", out[:, 0].tolist(), flush=True)
    except Exception as e:
        print(rank, "all_gather_into_tensor failed:", type(e).__name__, str(e)[:200], flush=True)
    dist.destroy_process_group()
if __name__ == "__main__":
    mp.spawn(run, args=(2,), nprocs=2)
