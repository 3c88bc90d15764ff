"""Seed-node data parallelism (new component: the reference is single-GPU,
``tbatch*.sh`` request ``--gres=gpu:1``).

One process per GPU.  Every rank holds a full replica of the graph CSR and
the feature table (products: ~0.5 GB + ~1 GB, << 288 GB HBM), draws the same
seed permutation per epoch and trains on its slice (``rank::world``), so the
data path has no collective.  The only exchange is the gradient all-reduce
after ``backward``: one flat fp32 bucket (products 2-layer h256: 75,567
params = 302 KB) averaged with a single RCCL ``all_reduce`` over xGMI —
latency-bound at this size, so one bucket, no overlap machinery.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def env_world():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init(backend: str | None = None):
    """Initialise the default process group from torchrun's env (no-op at world 1)."""
    rank, world, local = env_world()
    if world > 1 and not dist.is_initialized():
        if backend is None:  # NGNN_DIST_BACKEND=gloo: rehearse N ranks on fewer GPUs
            backend = os.environ.get("NGNN_DIST_BACKEND") or (
                "nccl" if torch.cuda.is_available() else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(minutes=10), **kw)
    return rank, world, local


def shard_seeds(nodes: torch.Tensor, rank: int, world: int, epoch: int, seed: int,
                shuffle: bool = True) -> torch.Tensor:
    """Same permutation on every rank (shared seed), strided slice per rank."""
    if shuffle:
        g = torch.Generator(device=nodes.device).manual_seed(seed + 1000 + epoch)
        nodes = nodes[torch.randperm(nodes.numel(), device=nodes.device, generator=g)]
    return nodes[rank::world]


class GradAllReduce:
    """Average gradients across ranks with ONE flat bucket all-reduce.

    The bucket is allocated once; ``__call__`` packs every parameter's grad,
    runs ``all_reduce(SUM)`` and unpacks ``bucket / world``.
    """

    def __init__(self, params, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.bucket = torch.empty(n, dtype=torch.float32, device=dev)

    def active(self) -> bool:
        return dist.is_initialized() and dist.get_world_size(self.group) > 1

    def pack(self):
        """grads -> bucket (stream-ordered copies; capturable in a HIP graph)."""
        off = 0
        for p in self.params:
            n = p.numel()
            if p.grad is None:
                self.bucket[off:off + n].zero_()
            else:
                self.bucket[off:off + n].copy_(p.grad.reshape(-1))
            off += n

    def allreduce(self):
        """The one collective: SUM over ranks (RCCL over xGMI with nccl)."""
        dist.all_reduce(self.bucket, op=dist.ReduceOp.SUM, group=self.group)

    def unpack(self):
        """bucket / world -> grads (capturable)."""
        world = dist.get_world_size(self.group)
        self.bucket.div_(world)
        off = 0
        for p in self.params:
            n = p.numel()
            if p.grad is None:
                p.grad = torch.empty_like(p)
            p.grad.copy_(self.bucket[off:off + n].view_as(p))
            off += n

    def __call__(self):
        if not self.active():
            return
        self.pack()
        self.allreduce()
        self.unpack()
