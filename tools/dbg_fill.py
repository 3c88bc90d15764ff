import sys, traceback
sys.path.insert(0, "noise-gnn_amd"); sys.path.insert(0, ".")
import torch
import ngnn
from ngnn.graphs import GraphedTrainStep, slot_size
from ngnn.loader import NeighborLoader, synthetic_graph
from ngnn.optim import Adam
dev = torch.device("cuda:0")
g = synthetic_graph("ogbn-products", dev, seed=0, scale=0.05)
lo = NeighborLoader(g, g.train_idx, [15, 10], 1024, shuffle=True, seed=3)
bs = [b for _, b in zip(range(3), lo)]
m = ngnn.SAGE(100, 256, 47, 2).to(dev).train()
opt = Adam(m.parameters(), lr=1e-3)
n_cap, e_cap = slot_size(1024, [15, 10])
st = GraphedTrainStep(m, opt, 1024, n_cap, e_cap, 100, dev)
orig_full = torch.full
def full(*a, **k):
    if torch.cuda.is_current_stream_capturing():
        print("torch.full during capture:", a, k); traceback.print_stack(limit=6)
    return orig_full(*a, **k)
torch.full = full
orig_zeros = torch.zeros
def zeros(*a, **k):
    if torch.cuda.is_current_stream_capturing():
        print("torch.zeros during capture:", a, k); traceback.print_stack(limit=6)
    return orig_zeros(*a, **k)
torch.zeros = zeros
st.capture(bs[0].x, bs[0].edge_index, bs[0].y)
print("captured")
