"""One independent learner per GPU (the reference's ``--runs`` pool, ``sac_eo/train.py:118-152``).

The SAC update does not shard: replicas exchange nothing on the data path.  The
process group (RCCL on GPUs, gloo on CPU) is used only for the start/stop barrier
and the max-over-ranks wall time of a timed region.  Launch one process per GPU
with ``torch.distributed.run`` (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1).
"""
import os
from dataclasses import dataclass

from .seeding import derive_seeds


@dataclass
class Replica:
    rank: int
    world_size: int
    local_rank: int
    backend: str
    dist: object = None          # torch.distributed when world_size > 1
    device: object = None        # torch.device of this replica

    # ------------------------------------------------------------------ seeds
    def seeds(self, seed: int = 0) -> dict:
        """This replica's seeds: run index = rank, derived like the reference's runs."""
        all_runs = derive_seeds(seed, runs=self.world_size)
        return {k: int(v[self.rank]) for k, v in all_runs.items()}

    # ------------------------------------------------------------------ sync
    def _sync_device(self):
        if self.device is not None and self.device.type == "cuda":
            import torch
            torch.cuda.synchronize(self.device)

    def barrier(self):
        """Device drained on every rank, then a process barrier (then drained again)."""
        self._sync_device()
        if self.dist is not None:
            self.dist.barrier()
            self._sync_device()

    def max_over_ranks(self, x: float) -> float:
        if self.dist is None:
            return float(x)
        import torch
        dev = self.device if (self.device is not None and self.backend == "nccl") else "cpu"
        t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(self, x: float) -> float:
        if self.dist is None:
            return float(x)
        import torch
        dev = self.device if (self.device is not None and self.backend == "nccl") else "cpu"
        t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def broadcast_bytes(self, payload: bytes = None) -> bytes:
        """Rank 0's payload on every rank (e.g. the RCCL unique id of the data-parallel mode)."""
        if self.dist is None:
            return payload
        obj = [payload if self.rank == 0 else None]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()
            self.dist = None


def env_ranks():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_replica(backend: str = None, use_cuda: bool = True) -> Replica:
    """Reads the torch.distributed.run environment; joins the group when WORLD_SIZE > 1.
    backend defaults to "nccl" (RCCL) on GPUs and "gloo" otherwise."""
    import torch
    rank, ws, local = env_ranks()
    device = None
    # diagnostics on a one-GPU box: SACX_SHARE_DEVICE=1 folds ranks onto the visible
    # devices, SACX_REPLICA_BACKEND=gloo replaces RCCL (which refuses a shared device)
    share = os.environ.get("SACX_SHARE_DEVICE") == "1"
    if use_cuda:
        idx = local % max(1, torch.cuda.device_count()) if share else local
        device = torch.device("cuda", idx)
        torch.cuda.set_device(device)
    be = backend or os.environ.get("SACX_REPLICA_BACKEND") or ("nccl" if use_cuda else "gloo")
    rep = Replica(rank=rank, world_size=ws, local_rank=local, backend=be, device=device)
    if ws > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": device} if (be == "nccl" and device is not None) else {}
        dist.init_process_group(be, rank=rank, world_size=ws, **kw)
        rep.dist = dist
    return rep
