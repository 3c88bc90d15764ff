"""Drop-in conv layers: ``SAGEConv`` and ``GCNConv(normalize=False)``.

Same constructor signatures, forward(x, edge_index), reset_parameters(),
sub-module names and state-dict keys as PyG 2.5.1's classes the reference
imports (``sage.py:4``, ``convolution.py:4``):

* SAGEConv: ``lin_l.weight [out,in]``, ``lin_l.bias [out]``, ``lin_r.weight [out,in]``
  out = lin_l(aggr_{j->i} x_j) + lin_r(x_i)          (sage.py:16-19, :34)
* GCNConv(normalize=False): ``lin.weight [out,in]`` (glorot), ``bias [out]`` (zeros)
  out = sum_{j->i} (x W^T)_j + bias                  (convolution.py:19-23, :31)

``forward`` also accepts a prebuilt :class:`ngnn.block.Block` in place of
``edge_index`` (the model wrappers build one per mini-batch).  On the GPU
(float32 / bfloat16) each conv is ONE autograd node over the hand-written
kernels (ngnn.fused: a one-layer fused stack), so a reference wrapper that
imports these classes instead of PyG's trains without library GEMMs.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .block import get_block
from .ops import segment_aggregate


class Linear(nn.Module):
    """PyG ``Linear`` init contract [ext]: kaiming_uniform(fan=in, a=sqrt(5))
    weight (or glorot), bias U(+-1/sqrt(in)).  Forward is F.linear."""

    def __init__(self, in_channels: int, out_channels: int, bias: bool = True,
                 weight_initializer: str | None = None):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.weight_initializer = weight_initializer
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels))
        if bias:
            self.bias = nn.Parameter(torch.empty(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        if self.weight_initializer == "glorot":
            a = math.sqrt(6.0 / (self.weight.size(-2) + self.weight.size(-1)))
            self.weight.data.uniform_(-a, a)
        else:
            bound = math.sqrt(6.0 / ((1 + 5.0) * self.in_channels))
            self.weight.data.uniform_(-bound, bound)
        if self.bias is not None:
            bound = 1.0 / math.sqrt(self.in_channels)
            self.bias.data.uniform_(-bound, bound)

    def forward(self, x):
        return F.linear(x, self.weight, self.bias)

    def extra_repr(self):
        return f"{self.in_channels}, {self.out_channels}, bias={self.bias is not None}"


class SAGEConv(nn.Module):
    def __init__(self, in_channels: int, out_channels: int, aggr: str = "mean",
                 normalize: bool = False, root_weight: bool = True, project: bool = False,
                 bias: bool = True):
        super().__init__()
        if normalize or project or not root_weight or not bias:
            raise NotImplementedError(
                "the reference only uses SAGEConv(in, out) defaults (sage.py:16-19)")
        if aggr not in ("mean", "max", "sum", "add"):
            raise ValueError(f"unsupported aggr {aggr!r}")
        self.in_channels, self.out_channels, self.aggr = in_channels, out_channels, aggr
        self.lin_l = Linear(in_channels, out_channels, bias=True)
        self.lin_r = Linear(in_channels, out_channels, bias=False)

    def reset_parameters(self):
        self.lin_l.reset_parameters()
        self.lin_r.reset_parameters()

    def forward(self, x: torch.Tensor, edge_index) -> torch.Tensor:
        block = get_block(edge_index, x.size(0))
        from . import fused
        needs_grad = torch.is_grad_enabled() and (
            x.requires_grad or any(p.requires_grad for p in self.parameters()))
        if (not needs_grad and x.is_cuda and x.dtype == torch.float32 and x.dim() == 2
                and self.lin_l.weight.dtype == torch.float32):
            # inference (e.g. SAGE.inference, sage.py:52): one fused launch
            aggr = "sum" if self.aggr == "add" else self.aggr
            xc = x if x.stride(1) == 1 else x.contiguous()
            return fused.sage_layer_fwd(xc, block, aggr, self.lin_l.weight, self.lin_l.bias,
                                        self.lin_r.weight, relu=False, p_drop=0.0, seed=0)
        if fused.conv_supported(self, x):
            # the per-conv drop-in (INTEGRATION.md option A: the reference's own
            # wrapper, sage.py:33-39, with this class in place of PyG's): one
            # autograd node on the hand-written kernels -- fused gather +
            # split-bf16 MFMA forward, MFMA weight gradient, narrow-space input
            # gradient -- no library GEMM; relu / dropout stay the wrapper's
            return fused.sage_conv(self, x, block)
        out = self.lin_l(segment_aggregate(x, block, self.aggr))
        return out + self.lin_r(x)

    def __repr__(self):
        return (f"{self.__class__.__name__}({self.in_channels}, {self.out_channels}, "
                f"aggr={self.aggr})")


class GCNConv(nn.Module):
    def __init__(self, in_channels: int, out_channels: int, normalize: bool = False,
                 add_self_loops: bool | None = None, bias: bool = True, **kwargs):
        super().__init__()
        if normalize or add_self_loops or not bias:
            raise NotImplementedError(
                "the reference only uses GCNConv(in, out, normalize=False) (convolution.py:19-23)")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.lin = Linear(in_channels, out_channels, bias=False, weight_initializer="glorot")
        self.bias = nn.Parameter(torch.zeros(out_channels))

    def reset_parameters(self):
        self.lin.reset_parameters()
        self.bias.data.zero_()

    def forward(self, x: torch.Tensor, edge_index) -> torch.Tensor:
        block = get_block(edge_index, x.size(0))
        from . import fused
        if fused.conv_supported(self, x):
            # per-conv drop-in (convolution.py:29-35 with this class in place of
            # PyG's): one autograd node on the hand-written kernels
            return fused.gcn_conv(self, x, block)
        h = self.lin(x)
        return segment_aggregate(h, block, "sum") + self.bias

    def __repr__(self):
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels})"
