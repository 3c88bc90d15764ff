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


_DTYPE_CODE = {torch.float32: 0, torch.bfloat16: 1}  # include/ngnn.h NGNN_F32 / NGNN_BF16


def cast_tensors(src, dst, divisor: float = 1.0) -> None:
    """dst[k] = cast(src[k]) / divisor for fp32 / bf16 tensors, 16 per
    ngnn_cast_tensors_ex launch (the bucket's copies and div_ in one
    kernel).  Tensors of other dtypes or layouts take the ATen path."""
    import ctypes

    from . import _lib, fused
    ok = [i for i, (a, b) in enumerate(zip(src, dst))
          if a.dtype in _DTYPE_CODE and b.dtype in _DTYPE_CODE and a.is_contiguous()
          and b.is_contiguous() and a.numel() == b.numel() and a.is_cuda and b.is_cuda]
    rest = [i for i in range(len(src)) if i not in set(ok)]
    for i in rest:  # (not on any path ngnn's models take)
        dst[i].copy_(src[i] / divisor if divisor != 1.0 else src[i])
    lib = _lib.load() if ok else None
    for j in range(0, len(ok), 16):
        idx = ok[j:j + 16]
        k = len(idx)
        S = (ctypes.c_void_p * k)(*[src[i].data_ptr() for i in idx])
        D = (ctypes.c_void_p * k)(*[dst[i].data_ptr() for i in idx])
        N = (ctypes.c_int64 * k)(*[src[i].numel() for i in idx])
        SD = (ctypes.c_int32 * k)(*[_DTYPE_CODE[src[i].dtype] for i in idx])
        DD = (ctypes.c_int32 * k)(*[_DTYPE_CODE[dst[i].dtype] for i in idx])
        _lib.check(lib.ngnn_cast_tensors_ex(k, S, D, N, SD, DD, float(divisor),
                                            _lib.stream_handle(src[idx[0]].device)),
                   "ngnn_cast_tensors_ex")


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


def shard_len(n: int, world: int) -> int:
    """Seeds per rank: ceil(n / world) on EVERY rank (see shard_seeds)."""
    return -(-int(n) // max(int(world), 1))


def shard_seeds(nodes: torch.Tensor, rank: int, world: int, epoch: int, seed: int,
                shuffle: bool = True) -> torch.Tensor:
    """Same permutation on every rank (shared seed), strided slice per rank.

    Every rank gets exactly ``shard_len(n, world)`` seeds: when ``world`` does
    not divide ``n`` the permutation is padded cyclically with its own head
    (as torch's DistributedSampler does), so all ranks run the same number of
    batches -- and therefore the same number of gradient all-reduces -- per
    epoch.  Unequal shards would leave the ranks with more batches waiting in
    a collective the others never join."""
    if shuffle:
        g = torch.Generator(device=nodes.device).manual_seed(seed + 1000 + epoch)
        nodes = nodes[torch.randperm(nodes.numel(), device=nodes.device, generator=g)]
    n = nodes.numel()
    pad = shard_len(n, world) * world - n
    if pad and n:
        reps = -(-pad // n)
        nodes = torch.cat([nodes] + [nodes] * reps)[:n + pad]
    return nodes[rank::world]


class GradAllReduce:
    """Average gradients across ranks with ONE flat bucket all-reduce.

    The bucket is allocated once and every fp32 parameter gets a view of it
    (``p._ngnn_grad_out``).  The fused SAGE backward writes its weight
    gradients straight into those views whenever ``p.grad`` is None at
    backward time (``optimizer.zero_grad(set_to_none=True)``, as the graph
    step does), and autograd adopts the view as ``p.grad``: the bucket then
    IS the gradients and ``pack`` / ``unpack`` copy nothing -- one
    ``all_reduce(SUM)`` and one scale by 1/world per step.  Gradients that
    live elsewhere (other modules, accumulation into existing ``.grad``) are
    copied in and out as before.
    """

    def __init__(self, params, group=None):
        from . import fused
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.bucket = torch.zeros(n, dtype=torch.float32, device=dev)
        self.views = []
        off = 0
        for p in self.params:
            v = self.bucket[off:off + p.numel()].view(p.shape)
            self.views.append(v)
            if p.dtype == torch.float32:
                p._ngnn_grad_out = v
                fused.note_grad_views()
            off += p.numel()

    def active(self) -> bool:
        return dist.is_initialized() and dist.get_world_size(self.group) > 1

    @staticmethod
    def _aliased(p, v) -> bool:
        return p.grad is not None and p.grad.data_ptr() == v.data_ptr()

    def pack(self):
        """grads -> bucket (stream-ordered, none for gradients that are
        already bucket views; capturable in a HIP graph).  Gradients that are
        not views -- a bf16 model's (autograd narrows the fused backward's
        fp32 gradients to the parameters' dtype), or accumulated ones -- move
        in ONE library launch (ngnn_cast_tensors_ex: bf16 widened exactly)."""
        dst, src = [], []
        for p, v in zip(self.params, self.views):
            if p.grad is None:
                v.zero_()
            elif not self._aliased(p, v):
                dst.append(v)
                src.append(p.grad)
        if dst:
            cast_tensors(src, dst)

    def allreduce(self):
        """The one collective: SUM over ranks (RCCL over xGMI with nccl)."""
        dist.all_reduce(self.bucket, op=dist.ReduceOp.SUM, group=self.group)

    def unpack(self):
        """bucket / world -> grads in ONE library launch (capturable): in
        place for the gradients that are bucket views, rounded to bf16 into
        a bf16 parameter's gradient (ngnn_cast_tensors_ex; the division is
        Tensor.div_'s quotient)."""
        world = dist.get_world_size(self.group)
        dst, src = [], []
        for p, v in zip(self.params, self.views):
            if p.grad is None:
                p.grad = v if p.dtype == v.dtype else torch.empty(p.shape, dtype=p.dtype, device=p.device)
            dst.append(p.grad)
            src.append(v)
        cast_tensors(src, dst, divisor=float(world))

    def __call__(self):
        if not self.active():
            return
        self.pack()
        self.allreduce()
        self.unpack()
