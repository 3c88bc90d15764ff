"""CPU oracle for the SAGE / SimpleGCN aggregation path — TEST INFRASTRUCTURE ONLY.

Nothing in the product (``noise-gnn_amd/ngnn``) imports this package.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may use it, and only as the checker / the timed CPU baseline.

Contents
--------
``pyg_ref``   torch-CPU restatement of the exact ATen op sequence PyTorch
              Geometric 2.5.1 issues for ``SAGEConv`` / ``GCNConv(normalize=False)``
              with a ``Tensor`` edge_index (PyG is pinned at
              ``docs/requirements.txt:11`` of the reference and is not vendored,
              not installed and not downloadable here), plus the reference's own
              ``SAGE`` / ``SimpleGCN`` wrapper composition
              (``src/models/layers/sage.py:6-79``, ``convolution.py:7-53``).
``seg_agg.c`` plain-C restatement of the per-destination aggregation (sum /
              mean / max, forward and backward) in edge order, built into
              ``oracle/build/liboracle_agg.so`` and wrapped by ``c_agg``.

Parity status: the wrapper composition is pinned by executing the reference's
own ``sage.py`` / ``convolution.py`` (see ``tests/golden/make_golden.py``); the
conv arithmetic itself follows PyG 2.5.1's documented op sequence [ext] and is
pinned only by hand-computed known-answer tests — the reference holds no
numeric fixture for it ("conv arithmetic: parity unpinned by reference data").
"""
