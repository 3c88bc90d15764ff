"""torch-CPU restatement of the reference's CPU path for SAGE / SimpleGCN — ORACLE.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  The product never imports it.

The reference (hhilsber/noise-GNN @ 2024_10_08) calls PyTorch Geometric 2.5.1
(``docs/requirements.txt:11``) for the arithmetic; PyG is an un-vendored
third-party dependency that is not installed and not downloadable here.  This
module restates, op for op, what PyG 2.5.1 issues on CPU for a ``Tensor``
``edge_index`` (flow ``source_to_target``):

* ``MessagePassing.propagate``       -> ``x_j = x.index_select(0, edge_index[0])``,
                                         ``index = edge_index[1]``, ``dim_size = x.size(0)``
* ``torch_geometric.utils.scatter``  -> sum:  ``zeros.scatter_add_``
                                        mean: sum / ``count.clamp(min=1)``
                                        max:  ``zeros.scatter_reduce_(.., 'amax', include_self=False)``
* ``SAGEConv.forward`` (aggr='mean', root_weight, bias, no project/normalize)
                                     -> ``lin_l(propagate(x)) + lin_r(x)``
* ``GCNConv.forward`` (normalize=False) -> ``propagate(lin(x)) (sum) + bias``

The wrappers ``SAGE`` and ``SimpleGCN`` restate the reference's own classes
(``src/models/layers/sage.py:6-79`` and ``src/models/layers/convolution.py:7-53``);
the golden fixtures in ``tests/golden`` were produced by executing those
reference files with this module standing in for ``torch_geometric.nn``.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


# --------------------------------------------------------------------------
# PyG 2.5.1 torch_geometric/utils/_scatter.py::scatter  [ext], Tensor path
# --------------------------------------------------------------------------
def _broadcast(index: torch.Tensor, src: torch.Tensor, dim: int) -> torch.Tensor:
    size = [1] * src.dim()
    size[dim] = -1
    return index.view(size).expand_as(src)


def scatter(src: torch.Tensor, index: torch.Tensor, dim: int, dim_size: int,
            reduce: str = "sum") -> torch.Tensor:
    size = list(src.size())
    size[dim] = dim_size
    if reduce in ("sum", "add"):
        return src.new_zeros(size).scatter_add_(dim, _broadcast(index, src, dim), src)
    if reduce == "mean":
        count = src.new_zeros(dim_size)
        count.scatter_add_(0, index, src.new_ones(src.size(dim)))
        count = count.clamp(min=1)
        out = src.new_zeros(size).scatter_add_(dim, _broadcast(index, src, dim), src)
        return out / _broadcast(count, out, dim)
    if reduce in ("max", "amax"):
        # CPU path of PyG 2.5.1 (and CUDA without grad): torch.scatter_reduce_.
        return src.new_zeros(size).scatter_reduce_(
            dim, _broadcast(index, src, dim), src, reduce="amax", include_self=False)
    raise ValueError(f"unsupported reduce {reduce!r}")


def propagate(x: torch.Tensor, edge_index: torch.Tensor, reduce: str) -> torch.Tensor:
    """MessagePassing.propagate for a Tensor edge_index, message = x_j."""
    x_j = x.index_select(0, edge_index[0])
    return scatter(x_j, edge_index[1], 0, x.size(0), reduce)


# --------------------------------------------------------------------------
# PyG Linear [ext]: kaiming_uniform(fan=in, a=sqrt(5)) weight, uniform(1/sqrt(in)) bias
# --------------------------------------------------------------------------
class Linear(nn.Module):
    def __init__(self, in_channels: int, out_channels: int, bias: bool = True,
                 weight_initializer: str | None = None):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.weight_initializer = weight_initializer
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
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


class SAGEConv(nn.Module):
    """PyG 2.5.1 nn/conv/sage_conv.py::SAGEConv [ext], defaults of sage.py:16-19."""

    def __init__(self, in_channels: int, out_channels: int, aggr: str = "mean"):
        super().__init__()
        self.in_channels, self.out_channels, self.aggr = in_channels, out_channels, aggr
        self.lin_l = Linear(in_channels, out_channels, bias=True)
        self.lin_r = Linear(in_channels, out_channels, bias=False)

    def reset_parameters(self):
        self.lin_l.reset_parameters()
        self.lin_r.reset_parameters()

    def forward(self, x, edge_index):
        out = propagate(x, edge_index, self.aggr)
        out = self.lin_l(out)
        return out + self.lin_r(x)


class GCNConv(nn.Module):
    """PyG 2.5.1 nn/conv/gcn_conv.py::GCNConv [ext] with normalize=False (convolution.py:19-23)."""

    def __init__(self, in_channels: int, out_channels: int, normalize: bool = False):
        super().__init__()
        if normalize:
            raise NotImplementedError("the reference only uses normalize=False")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.lin = Linear(in_channels, out_channels, bias=False, weight_initializer="glorot")
        self.bias = nn.Parameter(torch.zeros(out_channels))

    def reset_parameters(self):
        self.lin.reset_parameters()
        self.bias.data.zero_()

    def forward(self, x, edge_index):
        x = self.lin(x)
        out = propagate(x, edge_index, "sum")
        return out + self.bias


# --------------------------------------------------------------------------
# Wrappers: restatement of the reference's own classes
# --------------------------------------------------------------------------
class SAGE(nn.Module):
    """src/models/layers/sage.py:6-79 (forward :30-40, inference :42-58)."""

    def __init__(self, in_size, hidden_size, out_size, num_layers, dropout=0.5,
                 use_bn=False, aggr="mean"):
        super().__init__()
        self.num_layers, self.dropout = num_layers, dropout
        self.convs = nn.ModuleList([SAGEConv(in_size, hidden_size, aggr)])
        for _ in range(num_layers - 2):
            self.convs.append(SAGEConv(hidden_size, hidden_size, aggr))
        self.convs.append(SAGEConv(hidden_size, out_size, aggr))
        self.use_bn = use_bn
        if use_bn:
            self.bn1 = nn.BatchNorm1d(in_size)
            self.bn2 = nn.BatchNorm1d(hidden_size)

    def reset_parameters(self):
        for conv in self.convs:
            conv.reset_parameters()

    def forward(self, x, edge_index):
        if self.use_bn:
            x = self.bn1(x)
        for i, conv in enumerate(self.convs):
            x = conv(x, edge_index)
            if i != self.num_layers - 1:
                x = x.relu()
                if self.use_bn:
                    x = self.bn2(x)
                x = F.dropout(x, p=self.dropout, training=self.training)
        return x

    def inference(self, x_all, subgraph_loader, device="cpu"):
        for i in range(self.num_layers):
            xs = []
            for batch in subgraph_loader:
                x = x_all[batch.n_id].to(device)
                x = self.convs[i](x, batch.edge_index.to(device))[:batch.batch_size]
                if i != self.num_layers - 1:
                    x = x.relu()
                xs.append(x.cpu())
            x_all = torch.cat(xs, dim=0)
        return x_all


class SimpleGCN(nn.Module):
    """src/models/layers/convolution.py:7-53."""

    def __init__(self, in_size, hidden_size, out_size, num_layers, dropout=0.5, use_bn=False):
        super().__init__()
        self.num_layers, self.dropout = num_layers, dropout
        self.convs = nn.ModuleList([GCNConv(in_size, hidden_size, normalize=False)])
        for _ in range(num_layers - 2):
            self.convs.append(GCNConv(hidden_size, hidden_size, normalize=False))
        self.convs.append(GCNConv(hidden_size, out_size, normalize=False))

    def reset_parameters(self):
        for conv in self.convs:
            conv.reset_parameters()

    def forward(self, x, edge_index):
        for i, conv in enumerate(self.convs):
            x = conv(x, edge_index)
            if i != self.num_layers - 1:
                x = x.relu()
                x = F.dropout(x, p=self.dropout, training=self.training)
        return x

    inference = SAGE.inference


def train_step(model: nn.Module, optimizer, x, edge_index, y, batch_size: int):
    """One reference training step: pipeline.py:152-169 (baseline branch)."""
    out = model(x, edge_index)[:batch_size]
    loss = F.cross_entropy(out, y[:batch_size])
    optimizer.zero_grad()
    loss.backward()
    optimizer.step()
    return loss
