"""ngnn.optim.Adam == torch.optim.Adam (the reference optimiser,
model.py:66-69) step for step, with and without weight decay; capturable
in a HIP graph."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.mark.parametrize("wd", [0.0, 5e-4])
def test_matches_torch_adam(wd):
    from ngnn.optim import Adam
    g = torch.Generator().manual_seed(3)
    shapes = [(256, 100), (256,), (47, 256), (47,), (5, 3, 2)]
    ps = [torch.randn(s, generator=g).to(DEV) for s in shapes]
    p1 = [p.clone().requires_grad_(True) for p in ps]
    p2 = [p.clone().requires_grad_(True) for p in ps]
    o1 = Adam(p1, lr=1e-3, weight_decay=wd)
    o2 = torch.optim.Adam(p2, lr=1e-3, weight_decay=wd)
    for it in range(6):
        for a, b in zip(p1, p2):
            gr = torch.randn(a.shape, generator=g).to(DEV) * (it + 1)
            a.grad = gr.clone()
            b.grad = gr.clone()
        o1.step()
        o2.step()
    for a, b in zip(p1, p2):
        torch.testing.assert_close(a, b, rtol=2e-6, atol=2e-7)
    st = o1.state[p1[0]]
    assert float(st["step"]) == 6.0


def test_graph_capturable():
    from ngnn.optim import Adam
    p = torch.randn(1000, device=DEV, requires_grad=True)
    ref = p.detach().clone().requires_grad_(True)
    o, oref = Adam([p], lr=1e-2), torch.optim.Adam([ref], lr=1e-2)
    p.grad = torch.ones_like(p)
    ref.grad = torch.ones_like(ref)
    o.step()  # state created eagerly
    oref.step()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        o.step()
    for _ in range(3):
        gr.replay()
        oref.step()
    torch.cuda.synchronize()
    torch.testing.assert_close(p, ref, rtol=2e-6, atol=2e-7)


def test_bf16_params_match_rounded_fp32_adam():
    """bf16 parameters (BASELINE config #3): the update runs in fp32 against
    fp32 moments and is rounded to bf16 on store -- equal to torch's fp32 Adam
    whose parameters are rounded to bf16 after every step (within one bf16
    ulp)."""
    from ngnn.optim import Adam
    g = torch.Generator().manual_seed(5)
    shapes = [(256, 100), (256,), (47, 256)]
    base = [torch.randn(s, generator=g).to(DEV).to(torch.bfloat16) for s in shapes]
    pb = [b.clone().requires_grad_(True) for b in base]
    pf = [b.float().clone().requires_grad_(True) for b in base]
    ob, of = Adam(pb, lr=1e-2), torch.optim.Adam(pf, lr=1e-2)
    for it in range(4):
        for a, c in zip(pb, pf):
            gr = torch.randn(a.shape, generator=g).to(DEV).to(torch.bfloat16)
            a.grad = gr.clone()
            c.grad = gr.float()
        ob.step()
        of.step()
        with torch.no_grad():
            for c in pf:
                c.copy_(c.to(torch.bfloat16).float())
    for a, c in zip(pb, pf):
        assert a.dtype == torch.bfloat16
        torch.testing.assert_close(a.float(), c, rtol=8e-3, atol=1e-6)
    assert ob.state[pb[0]]["exp_avg"].dtype == torch.float32


@pytest.mark.parametrize("shapes", [
    [(512, 767), (512, 767), (10, 512), (10,), (512,)],  # Amazon-Computers: the 2-CU cap, 16 full groups
    [(300, 1000), (7,), (33, 5)],                        # ~300 workgroups: a ragged last group
])
def test_two_level_ticket_many_workgroups(shapes):
    """ABI 17: the update's workgroups count on a two-level ticket (groups of
    32, then the top word).  Three steps against torch's Adam, the device step
    count advanced once per call, every ticket word zero again after each."""
    from ngnn.optim import Adam
    g = torch.Generator().manual_seed(11)
    ps = [torch.randn(s, generator=g).to(DEV) for s in shapes]
    p1 = [p.clone().requires_grad_(True) for p in ps]
    p2 = [p.clone().requires_grad_(True) for p in ps]
    o1, o2 = Adam(p1, lr=1e-3), torch.optim.Adam(p2, lr=1e-3)
    for it in range(3):
        for a, b in zip(p1, p2):
            gr = torch.randn(a.shape, generator=g).to(DEV)
            a.grad, b.grad = gr.clone(), gr.clone()
        o1.step()
        o2.step()
        torch.cuda.synchronize()
        step = o1.state[p1[0]]["step"]
        assert float(step) == it + 1
        ticket = o1._tickets[step.data_ptr()]
        assert int(ticket.count_nonzero()) == 0
        for a, b in zip(p1, p2):
            torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-6, atol=1e-7)
