"""ngnn.losses.seed_cross_entropy == F.cross_entropy(out[:B], y[:B]) (the
reference loop's loss, pipeline.py:158): value, input gradient, ignored
labels, and the SAGE backward fed by it (row-bound hint) against the same
backward fed by torch's loss."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.mark.parametrize("C,B", [(47, 256), (10, 256), (130, 256), (47, 5000)])
def test_value_and_grad(C, B):
    from ngnn.losses import seed_cross_entropy
    g = torch.Generator().manual_seed(C)
    N = B + 444
    x = (torch.randn(N, C, generator=g) * 3).to(DEV).requires_grad_(True)
    y = torch.randint(0, C, (N,), generator=g).to(DEV)
    y[5] = -100  # ignored label
    x2 = x.detach().clone().requires_grad_(True)
    got = seed_cross_entropy(x, y, B)
    ref = F.cross_entropy(x2[:B], y[:B])
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
    got.backward()
    ref.backward()
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-5, atol=1e-7)
    assert torch.count_nonzero(x.grad[B:]) == 0


def test_sage_step_same_grads_as_torch_loss():
    import ngnn
    from ngnn.losses import seed_cross_entropy
    from ngnn.loader import NeighborLoader, synthetic_graph
    gr = synthetic_graph("ogbn-arxiv", DEV, seed=0, scale=0.05)
    b = next(iter(NeighborLoader(gr, gr.train_idx, [10, 5], 256, shuffle=True, seed=3)))
    torch.manual_seed(4)
    m1 = ngnn.SAGE(gr.x.size(1), 64, gr.num_classes, 2, dropout=0.0).to(DEV)
    m2 = ngnn.SAGE(gr.x.size(1), 64, gr.num_classes, 2, dropout=0.0).to(DEV)
    m2.load_state_dict(m1.state_dict())
    seed_cross_entropy(m1(b.x, b.edge_index), b.y, b.batch_size).backward()
    F.cross_entropy(m2(b.x, b.edge_index)[:b.batch_size], b.y[:b.batch_size]).backward()
    for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        torch.testing.assert_close(p1.grad, p2.grad, rtol=1e-4, atol=1e-6, msg=n)


def test_cpu_raises():
    from ngnn.losses import seed_cross_entropy
    with pytest.raises(RuntimeError):
        seed_cross_entropy(torch.zeros(4, 3), torch.zeros(4, dtype=torch.long), 2)
