"""CPU checks of the round-4 step fusions' host side (no kernel launches):

* ngnn_xent_head / ngnn_adam_fold / the row-bounded logits cast through the
  C ABI: workspace sizing, argument errors returned before any launch;
* fused.AdamFoldSpec.make: the Adam step folds only into a two-layer SAGE
  stack whose optimizer is ngnn.optim.Adam over exactly its six fp32
  tensors with their state made, and the struct's tensor order is the
  header's (dW_l1, db1, dW_r1, dW_l0, db0, dW_r0).
"""
import ctypes

import torch

import ngnn
from ngnn import _lib, fused
from ngnn.optim import Adam


def test_head_and_fold_argument_errors():
    lib = _lib.load()
    # the head's workspace: ticket + count + 32 group tickets, 32 group sums, B partials
    assert lib.ngnn_xent_head_workspace_bytes(0) == 0
    assert lib.ngnn_xent_head_workspace_bytes(1024) == 256 + 4 * (32 + 1024)
    # (pointer arguments: aligned placeholders -- nothing is dereferenced on
    # the host, and every call below returns before a launch)
    A, mean = 4096, _lib.REDUCE["mean"]
    args = [A, None, None, None, 0, 100, 100, 64, None, 64, None, A, A, None, mean,
            A, A, A, 100, 256, A, A, A, 256, 47, 0.0, 0, None, A, 256, 64, None, A, 100, A, 47]
    # a head with a null label pointer: E_ARG before any launch
    hd = _lib.XentHead(None, 4, -100, A, A, A, 47, None, 0, None, A, 1 << 20)
    assert lib.ngnn_sage2_fwd(*args, ctypes.byref(hd), _lib.SAGE2_ALL, A, 1 << 30, None) == _lib.E_ARG
    # B larger than the block's rows
    hd2 = _lib.XentHead(A, 65, -100, A, A, A, 47, None, 0, None, A, 1 << 20)
    assert lib.ngnn_sage2_fwd(*args, ctypes.byref(hd2), _lib.SAGE2_ALL, A, 1 << 30, None) == _lib.E_ARG
    # a workspace below ngnn_xent_head_workspace_bytes(B)
    hd3 = _lib.XentHead(A, 16, -100, A, A, A, 47, None, 0, None, A, 8)
    assert lib.ngnn_sage2_fwd(*args, ctypes.byref(hd3), _lib.SAGE2_ALL, A, 1 << 30, None) == _lib.E_WORKSPACE
    # the folded Adam step needs every tensor and the step count
    P = (ctypes.c_void_p * 6)(*([A] * 6))
    af = _lib.AdamFold(P, P, P, None, 1e-3, 0.9, 0.999, 1e-8, 0.0)
    assert lib.ngnn_sage2_bwd(A, 47, 47, A, A, 256, A, 256, 1.0, A, None, None, None, 0, 100, 100, A, 100,
                              A, A, 64, A, A, mean, A, A, A, A, A, A, None, ctypes.byref(af), A, 1 << 30,
                              None) == _lib.E_ARG
    # the row-bounded cast: negative sizes are argument errors, empty is a no-op
    assert lib.ngnn_cast_f32_bf16_rows(None, None, -1, 47, None, None) == _lib.E_ARG
    assert lib.ngnn_cast_f32_bf16_rows(None, None, 0, 47, None, None) == 0


def _with_state(model, opt):
    """The optimizer state a first step would make (CPU tensors, no launch)."""
    step = torch.zeros(())
    for p in model.parameters():
        opt.state[p] = dict(step=step, exp_avg=torch.zeros_like(p), exp_avg_sq=torch.zeros_like(p))


def test_adam_fold_eligibility_and_order():
    torch.manual_seed(0)
    m = ngnn.SAGE(100, 256, 47, 2, dropout=0.5)
    opt = Adam(m.parameters(), lr=1e-3)
    assert fused.AdamFoldSpec.make(opt, m) is None  # no state yet (before the warm-up)
    _with_state(m, opt)
    spec = fused.AdamFoldSpec.make(opt, m)
    assert spec is not None
    c0, c1 = m.convs
    want = [c1.lin_l.weight, c1.lin_l.bias, c1.lin_r.weight, c0.lin_l.weight, c0.lin_l.bias,
            c0.lin_r.weight]
    assert [spec.struct.param[k] for k in range(6)] == [q.data_ptr() for q in want]
    assert [spec.struct.exp_avg[k] for k in range(6)] == [opt.state[q]["exp_avg"].data_ptr() for q in want]
    assert abs(spec.struct.lr - 1e-3) < 1e-9 and not spec.used
    # torch's Adam, a 3-layer stack, or two parameter groups: no fold
    t_opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    assert fused.AdamFoldSpec.make(t_opt, m) is None
    m3 = ngnn.SAGE(100, 256, 47, 3, dropout=0.5)
    o3 = Adam(m3.parameters())
    _with_state(m3, o3)
    assert fused.AdamFoldSpec.make(o3, m3) is None
    ps = list(m.parameters())
    o2 = Adam([{"params": ps[:3]}, {"params": ps[3:]}])
    _with_state(m, o2)
    assert fused.AdamFoldSpec.make(o2, m) is None
    # a parameter outside the stack in the group: no fold
    extra = torch.nn.Parameter(torch.zeros(3))
    o4 = Adam(list(m.parameters()) + [extra])
    _with_state(m, o4)
    o4.state[extra] = dict(step=torch.zeros(()), exp_avg=torch.zeros(3), exp_avg_sq=torch.zeros(3))
    assert fused.AdamFoldSpec.make(o4, m) is None
