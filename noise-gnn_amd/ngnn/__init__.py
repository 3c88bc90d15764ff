"""ngnn — MI355X-native GraphSAGE / GCN sampled-subgraph aggregation path.

Drop-in for the reference's ``SAGE`` / ``SimpleGCN`` (hhilsber/noise-GNN
``src/models/layers/sage.py``, ``convolution.py``) and the PyG ``SAGEConv`` /
``GCNConv`` they call, backed by hand-written HIP kernels for gfx950 behind the
C ABI in ``include/ngnn.h``.  GPU only: there is no CPU fallback.
"""
from . import _lib
from .block import Block, get_block
from .models import NGNN, SAGE, SimpleGCN
from .nn import GCNConv, Linear, SAGEConv
from .ops import segment_aggregate

__all__ = ["Block", "get_block", "NGNN", "SAGE", "SimpleGCN", "GCNConv", "Linear", "SAGEConv",
           "segment_aggregate", "_lib"]
