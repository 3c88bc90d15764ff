import sys
import torch
a, b = torch.load(sys.argv[1]), torch.load(sys.argv[2])
for k in a:
    for name, x, y in zip(("h", "out", "agg"), a[k], b[k]):
        d = (x - y).abs()
        bad = (d > 1e-5 * (1 + y.abs())).nonzero()
        print(k, name, tuple(x.shape), "maxdiff", float(d.max()), "nbad", bad.size(0), "first", bad[:5].tolist())
