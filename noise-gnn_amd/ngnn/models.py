"""Drop-in model wrappers: ``SAGE``, ``SimpleGCN`` and the ``NGNN`` factory.

Mirror the reference classes one to one:

* ``SAGE``      src/models/layers/sage.py:6-79
* ``SimpleGCN`` src/models/layers/convolution.py:7-53
* ``NGNN``      src/models/model.py:10-69 (module string -> network, Adam optimiser)

Differences are internal only: ``forward`` builds the validated CSR
:class:`~ngnn.block.Block` once per call and hands it to every layer (the
reference's PyG convs re-scan ``edge_index`` per layer), and ``inference``
keeps each layer's activations on the device (see its docstring).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import fused
from .block import get_block
from .loader import IndexedRows
from .nn import GCNConv, SAGEConv


def _refuse_sync_free(edge_index):
    """A NeighborLoader(sync_free=True) batch holds capacity-sized buffers
    whose real extent only the device knows (ABI 19): refused before anything
    reads them (ngnn.block.get_block checks again for direct conv calls)."""
    if getattr(edge_index, "_ngnn_counts", None) is not None:
        raise ValueError("a sync_free NeighborLoader batch feeds GraphedTrainStep only; "
                         "use NeighborLoader(sync_free=False) for eager training")


def _dropout_seed(model, x, block):
    """(host seed, device seed word) of a fused stack's hash dropout."""
    seed, seed_dev = 0, None
    if model.training and model.dropout > 0:
        if torch.cuda.is_current_stream_capturing():
            # HIP-graph capture: a device seed, fresh at every replay -- the
            # slot's (advanced by each slot load), else drawn by torch's
            # graph-safe generator inside the graph.  The host part is the
            # model's graph salt (0 unless set: two models captured over one
            # slot -- GraphedCoTeachingStep -- draw independent masks)
            seed = int(getattr(model, "_ngnn_graph_salt", 0))
            seed_dev = block.seed_dev
            if seed_dev is None:
                seed_dev = torch.randint(0, 2**62, (1,), device=x.device)
        else:
            seed = int(torch.randint(0, 2**62, (1,)).item())  # torch's (CPU) RNG stream
    return seed, seed_dev


class SAGE(nn.Module):
    def __init__(self, in_size, hidden_size, out_size, num_layers, dropout=0.5, use_bn=False,
                 aggr: str = "mean"):
        super().__init__()
        self.num_layers = num_layers
        self.dropout = dropout
        self.convs = nn.ModuleList()
        self.convs.append(SAGEConv(in_size, hidden_size, aggr=aggr))
        for _ in range(num_layers - 2):
            self.convs.append(SAGEConv(hidden_size, hidden_size, aggr=aggr))
        self.convs.append(SAGEConv(hidden_size, out_size, aggr=aggr))
        self.use_bn = use_bn
        if self.use_bn:
            self.bn1 = nn.BatchNorm1d(in_size)
            self.bn2 = nn.BatchNorm1d(hidden_size)

    def reset_parameters(self):
        for conv in self.convs:
            conv.reset_parameters()

    def forward(self, x, edge_index):
        _refuse_sync_free(edge_index)
        if isinstance(x, IndexedRows):  # eager: gather the rows (graph replays fuse it)
            x = x.materialize()
        block = get_block(edge_index, x.size(0))
        if fused.sage_stack_supported(self, x):
            # one autograd node for the stack: fused layer kernels forward,
            # receptive-field-bounded backward (ngnn/fused.py)
            return fused.sage_stack(self, x, block, *_dropout_seed(self, x, block))
        if self.use_bn:
            x = self.bn1(x)
        for i, conv in enumerate(self.convs):
            x = conv(x, block)
            if i != self.num_layers - 1:
                x = x.relu()
                if self.use_bn:
                    x = self.bn2(x)
                x = F.dropout(x, p=self.dropout, training=self.training)
        return x

    @torch.no_grad()
    def inference(self, x_all, subgraph_loader, device):
        """Layer-wise inference, sage.py:42-58 semantics.

        Per layer i and per loader batch: ``convs[i](x_all[n_id], edge_index)[:batch_size]``,
        relu except after the last layer, rows concatenated in loader order.
        ``x_all`` may live on the host (as in the reference) or on the device;
        the result is returned where ``x_all`` was given.  Between layers the
        activations stay on the device (the reference round-trips every batch
        through the host, sage.py:50,56).
        """
        return _layerwise_inference(self.convs, self.num_layers, x_all, subgraph_loader, device)


class SimpleGCN(nn.Module):
    def __init__(self, in_size, hidden_size, out_size, num_layers, dropout=0.5, use_bn=False):
        super().__init__()
        self.num_layers = num_layers
        self.dropout = dropout
        self.convs = nn.ModuleList()
        self.convs.append(GCNConv(in_size, hidden_size, normalize=False))
        for _ in range(num_layers - 2):
            self.convs.append(GCNConv(hidden_size, hidden_size, normalize=False))
        self.convs.append(GCNConv(hidden_size, out_size, normalize=False))

    def reset_parameters(self):
        for conv in self.convs:
            conv.reset_parameters()

    def forward(self, x, edge_index):
        _refuse_sync_free(edge_index)
        if isinstance(x, IndexedRows):  # eager: gather the rows (graph replays fuse it)
            x = x.materialize()
        block = get_block(edge_index, x.size(0))
        if fused.gcn_stack_supported(self, x):
            # one autograd node for the stack (ngnn/fused.py: SAGE layers with
            # W_r = 0, sum aggregation); dropout seed as SAGE.forward
            return fused.gcn_stack(self, x, block, *_dropout_seed(self, x, block))
        for i, conv in enumerate(self.convs):
            x = conv(x, block)
            if i != self.num_layers - 1:
                x = x.relu()
                x = F.dropout(x, p=self.dropout, training=self.training)
        return x

    @torch.no_grad()
    def inference(self, x_all, subgraph_loader, device):
        """convolution.py:37-53 semantics (same loop as SAGE.inference)."""
        return _layerwise_inference(self.convs, self.num_layers, x_all, subgraph_loader, device)


def _layerwise_inference(convs, num_layers, x_all, subgraph_loader, device):
    out_device = x_all.device
    x_cur = x_all.to(device)
    for i in range(num_layers):
        xs = []
        for batch in subgraph_loader:
            n_id = batch.n_id.to(device)
            edge_index = batch.edge_index.to(device)
            x = convs[i](x_cur.index_select(0, n_id), edge_index)
            x = x[:batch.batch_size]
            if i != num_layers - 1:
                x = x.relu()
            xs.append(x)
        x_cur = torch.cat(xs, dim=0)
    return x_cur.to(out_device)


class NGNN(object):
    """src/models/model.py:10-69: builds ``self.network`` from ``module`` and an
    Adam optimiser (weight decay commented out in the reference, model.py:68-69)."""

    def __init__(self, in_size=100, hidden_size=128, out_size=47, num_layers=2, dropout=0.5,
                 lr=0.001, optimizer='adam', module='sage', nbr_nodes=1, use_bn=False, wd=0.0005,
                 aggr='mean'):
        self.criterion = None
        self.score_func = None
        self.metric_name = None
        self.in_size, self.hidden_size, self.out_size = in_size, hidden_size, out_size
        self.num_layers, self.dropout, self.nbr_nodes = num_layers, dropout, nbr_nodes
        self.lr, self.wd = lr, wd
        self.optimizer = optimizer
        self.module = module
        self.use_bn = use_bn
        self.aggr = aggr
        self.init_network()
        self.init_optimizer()

    def init_network(self):
        if self.module == 'gcn':
            self.network = SimpleGCN(in_size=self.in_size, hidden_size=self.hidden_size,
                                     out_size=self.out_size, num_layers=self.num_layers,
                                     dropout=self.dropout)
        elif self.module == 'sage':
            self.network = SAGE(in_size=self.in_size, hidden_size=self.hidden_size,
                                out_size=self.out_size, num_layers=self.num_layers,
                                dropout=self.dropout, use_bn=self.use_bn, aggr=self.aggr)
        else:
            raise ValueError(f"module {self.module!r} is outside this path "
                             "(supported: 'sage', 'gcn'; see DESIGN.md scope)")

    def init_optimizer(self):
        if self.optimizer == 'adam':
            self.optimizer = torch.optim.Adam(self.network.parameters(), lr=self.lr)
        else:
            raise ValueError(f"optimizer {self.optimizer!r}: only 'adam' is reachable in the "
                             "reference (model.py:67-69; the other branches reference "
                             "undefined attributes)")
