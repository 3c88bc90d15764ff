"""The fp32 weight-gradient bar, shared by every GPU test
that compares a gradient against the oracle or a float64 restatement:

    max |g - g_ref|  <=  WGRAD_REL * max |g_ref|       (WGRAD_REL = 1e-5)

i.e. the north star's 1e-5 fp32 bar scaled to each tensor.  (An absolute
atol of 1e-4, the round-4 bar, exceeded the median entry of the products
model's dW_l0 -- it could not tell a right gradient from a 60 %-wrong one.)
Elementwise, every entry with |g_ref| >= 0.1 max|g_ref| is then within
1e-4 of itself relative, which the bar implies.

With NGNN_GRAD_LOG=<path> every comparison appends one JSON line (test,
tensor, max|err|, max|ref|, ratio) -- the committed evidence of what the
kernels deliver (profiles/r05_grad_errors.jsonl).
"""
import json
import os

import torch

WGRAD_REL = 1e-5


def _log(name, err, ref, bar):
    path = os.environ.get("NGNN_GRAD_LOG")
    if not path:
        return
    test = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    with open(path, "a") as f:
        f.write(json.dumps(dict(test=test, tensor=str(name), max_err=err, max_ref=ref,
                                ratio=(err / ref if ref > 0 else 0.0), bar=bar)) + "\n")


def grad_ratio(got, want):
    """max|got - want| / max|want| (float64), and its parts."""
    got = got.detach().double().cpu()
    want = want.detach().double().cpu()
    assert got.shape == want.shape, (got.shape, want.shape)
    ref = float(want.abs().max()) if want.numel() else 0.0
    err = float((got - want).abs().max()) if want.numel() else 0.0
    return err, ref


def assert_wgrad(got, want, msg="", rel=WGRAD_REL):
    """Assert max|got - want| <= rel * max|want| (a zero reference must be
    matched by a zero gradient up to 1e-30)."""
    err, ref = grad_ratio(got, want)
    _log(msg, err, ref, rel)
    assert torch.isfinite(got.detach().double()).all(), f"{msg}: non-finite gradient"
    assert err <= rel * ref + 1e-30, (
        f"{msg}: max|err| {err:.3e} > {rel:g} * max|ref| {ref:.3e} (ratio {err / max(ref, 1e-300):.3e})")
