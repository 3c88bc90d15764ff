"""Training steps of the reference's SAGE wrapper structure (sage.py:6-40)
with ngnn.SAGEConv swapped in (INTEGRATION.md option A), for a rocprofv3
kernel trace: every kernel the step issues should be an ngnn kernel or a
torch elementwise one -- no rocBLAS / hipBLASLt GEMM.

    rocprofv3 --kernel-trace --stats -d OUT -o run --output-format csv -- \\
        python3 tools/perconv_step.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "noise-gnn_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import ngnn  # noqa: E402
from ngnn.loader import sample_block, synthetic_graph  # noqa: E402


class RefSAGE(torch.nn.Module):
    def __init__(self, in_size, hidden, out, num_layers, dropout=0.5):
        super().__init__()
        self.num_layers, self.dropout = num_layers, dropout
        dims = [in_size] + [hidden] * (num_layers - 1) + [out]
        self.convs = torch.nn.ModuleList(ngnn.SAGEConv(dims[i], dims[i + 1])
                                         for i in range(num_layers))

    def forward(self, x, edge_index):
        for i, conv in enumerate(self.convs):
            x = conv(x, edge_index)
            if i != self.num_layers - 1:
                x = F.relu(x)
                x = F.dropout(x, p=self.dropout, training=self.training)
        return x


def main():
    dev = torch.device("cuda:0")
    g = synthetic_graph("ogbn-products", dev, seed=0, scale=0.2)
    torch.manual_seed(0)
    model = RefSAGE(100, 256, 47, 2).to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    for s in range(5):
        b = sample_block(g, g.train_idx[s * 1024:(s + 1) * 1024], [15, 10], seed=s)
        out = model(b.x, b.edge_index)[:b.batch_size]
        loss = F.cross_entropy(out, b.y[:b.batch_size])
        opt.zero_grad()
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    print("loss", float(loss))


if __name__ == "__main__":
    main()
