"""CPU checks of the drop-in boundary: the C-ABI library loads, exports every
symbol include/ngnn.h declares, rejects bad arguments before launching, and
the Python layer refuses to run anywhere but the GPU (no silent fallback)."""
import ctypes
import os
import re

import pytest
import torch

import ngnn
from ngnn import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ngnn.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ngnn_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 8
    for s in syms:
        assert hasattr(lib, s), s
    # the ctypes signature table covers exactly the header
    assert sorted(_lib.SIGNATURES) == syms


def test_abi_version_and_strerror():
    lib = _lib.load()
    assert lib.ngnn_abi_version() == _lib.ABI_VERSION
    m = re.search(r"#define NGNN_ABI_VERSION (\d+)", open(HEADER).read())
    assert int(m.group(1)) == _lib.ABI_VERSION
    assert b"invalid argument" in lib.ngnn_strerror(-1)
    assert b"dtype" in lib.ngnn_strerror(-2)
    assert b"unknown" in lib.ngnn_strerror(-99)


def test_docs_cite_the_current_abi():
    """INTEGRATION.md's ctypes stub reads the header's version (no stale
    literal), DESIGN.md states the current one, and every profiles/ file the
    docs cite exists (the stub asserted 11 against ABI 12)."""
    import glob
    root = os.path.dirname(HEADER.rstrip("/")).rsplit("/include", 1)[0]
    integ = open(os.path.join(root, "INTEGRATION.md")).read()
    design = open(os.path.join(root, "DESIGN.md")).read()
    assert not re.search(r"ngnn_abi_version\(\)\s*==\s*\d", integ)
    assert "NGNN_ABI_VERSION" in integ
    for v in re.findall(r"ABI v(\d+)", design):
        assert int(v) == _lib.ABI_VERSION
    # the stub's version probe, run as written against the built library
    cwd = os.getcwd()
    try:
        os.chdir(root)
        m = re.search(r'NGNN_ABI_VERSION = int\(re\.search\((.*?)\)\.group\(1\)\)', integ, re.S)
        assert m, "the stub derives its version from the header"
        ver = int(eval("re.search(" + m.group(1) + ").group(1)", {"re": re}))
        assert ver == _lib.load().ngnn_abi_version()
        for cite in set(re.findall(r"profiles/[A-Za-z0-9_.*\-]+", integ + design)):
            if cite.endswith((".txt", ".csv", ".log", ".json")) or "*" in cite:
                assert glob.glob(cite.rstrip(".,)")), f"cited but absent: {cite}"
    finally:
        os.chdir(cwd)


def test_argument_errors_return_before_launch():
    lib = _lib.load()
    # bad reduce enum, bad dtype, ld < F, null pointers: no kernel is launched
    assert lib.ngnn_seg_agg_fwd(None, 4, 4, None, None, 10, 7, 0, None, 4, None) == -1
    assert lib.ngnn_seg_agg_fwd(None, 4, 4, None, None, 10, 1, 5, None, 4, None) == -2
    assert lib.ngnn_seg_agg_fwd(1, 2, 4, 1, 1, 10, 1, 0, 1, 4, None) == -3
    assert lib.ngnn_seg_agg_fwd(None, 4, 4, 1, None, 10, 1, 0, None, 4, None) == -1
    assert lib.ngnn_edge_probe(None, 10, 5, 5, None, None) == -1
    assert lib.ngnn_edge_probe(1, 2**31, 5, 5, 1, None) == -5
    assert lib.ngnn_csr_build(None, None, -1, 3, 1, None, None, None, None, 0, None) == -1
    assert lib.ngnn_sample_hop(1, 1, 1, 4, 65, 0, 1, 1, None) == -3
    assert lib.ngnn_seg_agg_bwd_workspace_bytes(10, 4, 1) == 0
    assert lib.ngnn_seg_agg_bwd_workspace_bytes(10, 4, 2) == 160
    # whole-block sampler: workspace sizing and argument checks (no launch)
    import ctypes
    fan = (ctypes.c_int32 * 2)(15, 10)
    ws = lib.ngnn_sample_block_workspace_bytes(1024, fan, 2)
    assert ws >= 4 * (1024 * 166 + 2 * 1024 * 165)  # n_id + both edge rows, int32
    bad = (ctypes.c_int32 * 2)(15, 65)
    assert lib.ngnn_sample_block_workspace_bytes(1024, bad, 2) == 0
    assert lib.ngnn_sample_block(1, 1, 100, 1, 1024, bad, 2, 0, 1, 1, 1 << 30, 1, None) == -3
    assert lib.ngnn_sample_block(1, 1, 100, 1, 1024, fan, 2, 0, 1, 1, ws - 1, 1, None) == -6
    assert lib.ngnn_sample_block(1, 1, 100, 1, 1024, fan, 2, 0, None, 1, ws, 1, None) == -1
    assert lib.ngnn_sample_block_finish(fan, 2, 1024, 1023, 0, 1, 100, 1, ws, 1, 1, None, None,
                                        None, 0, 0, None, 0, 0, None, None, None, None) == -3
    # ABI 18: the CSR outputs come as a pair (col may be absent only without edges)
    assert lib.ngnn_sample_block_finish(fan, 2, 1024, 1024, 5, 1, 100, 1, ws, 1, 1, None, None,
                                        None, 0, 0, None, 0, 0, 16, None, None, None) == -1
    # two-layer backward: operands past the 32-bit buffer range are refused
    # before any launch: n_rows x ldh x 4 B > 3.75 GiB
    big = 1 << 22
    assert lib.ngnn_sage2_bwd(16, 47, 47, 16, 16, 256, 16, 1024, 1.0, 16, None, None, None, 0, 100, 100,
                              16, 100, 16, 16, big, 16, 16, 0, 16, 16, 16, 16, 16, 16, None, None,
                              256, 1 << 40, None) == -5
    # ABI 18: a root-free stack passes BOTH dW_r0 and dW_r1 as NULL (x may be
    # NULL then); one of them alone is an argument error, as is an indexed x
    # without a root term -- refused before any launch
    assert lib.ngnn_sage2_bwd(16, 47, 47, 16, 16, 256, 16, 256, 1.0, None, None, None, None, 0, 100, 100,
                              16, 100, 16, 16, 1024, 16, 16, 0, 16, 16, None, 16, 16, 16, None, None,
                              256, 1 << 40, None) == -1
    assert lib.ngnn_sage2_bwd(16, 47, 47, 16, 16, 256, 16, 256, 1.0, None, None, None, 16, 1, 100, 100,
                              16, 100, 16, 16, 1024, 16, 16, 0, 16, 16, None, 16, 16, None, None, None,
                              256, 1 << 40, None) == -1
    # ABI 18: the mixed-dtype cast refuses a bad dtype / an in-place width change
    import ctypes as ct
    one = (ct.c_void_p * 1)(16)
    n1 = (ct.c_int64 * 1)(4)
    f32, bf16, bad = (ct.c_int32 * 1)(0), (ct.c_int32 * 1)(1), (ct.c_int32 * 1)(7)
    assert lib.ngnn_cast_tensors_ex(1, one, one, n1, f32, bad, 1.0, None) == -2
    assert lib.ngnn_cast_tensors_ex(1, one, one, n1, f32, bf16, 1.0, None) == -1
    assert lib.ngnn_cast_tensors_ex(1, one, one, n1, f32, f32, 0.0, None) == -1
    assert lib.ngnn_cast_tensors_ex(0, None, None, None, None, None, 2.0, None) == 0
    # zero-size work is a no-op success
    assert lib.ngnn_seg_agg_fwd(None, 4, 4, 1, None, 0, 1, 0, None, 4, None) == 0


def test_check_raises_with_message():
    with pytest.raises(_lib.NGNNError, match="invalid argument"):
        _lib.check(-1, "x")


def test_cpu_tensors_fail_loudly():
    conv = ngnn.SAGEConv(8, 4)
    x = torch.randn(5, 8)
    ei = torch.tensor([[0, 1], [1, 2]])
    with pytest.raises(RuntimeError, match="GPU only"):
        conv(x, ei)
    model = ngnn.SAGE(8, 16, 3, 2)
    with pytest.raises(RuntimeError, match="GPU only"):
        model(x, ei)
    with pytest.raises(RuntimeError, match="GPU only"):
        ngnn.SimpleGCN(8, 16, 3, 2)(x, ei)


def test_state_dict_contract_matches_reference_keys():
    m = ngnn.SAGE(100, 256, 47, 3)
    keys = list(m.state_dict())
    want = []
    for i in range(3):
        want += [f"convs.{i}.lin_l.weight", f"convs.{i}.lin_l.bias", f"convs.{i}.lin_r.weight"]
    assert keys == want
    assert m.convs[0].lin_l.weight.shape == (256, 100)
    g = ngnn.SimpleGCN(20, 32, 6, 2)
    assert list(g.state_dict()) == ["convs.0.bias", "convs.0.lin.weight", "convs.1.bias",
                                    "convs.1.lin.weight"]


def test_param_counts_match_survey():
    # products 2-layer h256 75,567; 3-layer 206,895; arxiv 86,312
    n = lambda m: sum(p.numel() for p in m.parameters())
    assert n(ngnn.SAGE(100, 256, 47, 2)) == 75_567
    assert n(ngnn.SAGE(100, 256, 47, 3)) == 206_895
    assert n(ngnn.SAGE(128, 256, 40, 2)) == 86_312


def test_ngnn_factory():
    m = ngnn.NGNN(100, 64, 47, 2, 0.5, 0.01, "adam", "sage")
    assert isinstance(m.network, ngnn.SAGE)
    assert isinstance(m.optimizer, torch.optim.Adam)
    assert m.optimizer.param_groups[0]["lr"] == 0.01
    g = ngnn.NGNN(100, 64, 47, 2, 0.5, 0.01, "adam", "gcn")
    assert isinstance(g.network, ngnn.SimpleGCN)
    with pytest.raises(ValueError):
        ngnn.NGNN(module="sageFC")


def test_pyg_compatible_init_matches_oracle_rng_order():
    from oracle import pyg_ref
    torch.manual_seed(3)
    a = ngnn.SAGE(10, 12, 4, 3)
    torch.manual_seed(3)
    b = pyg_ref.SAGE(10, 12, 4, 3)
    for (k, p), (k2, q) in zip(a.state_dict().items(), b.state_dict().items()):
        assert k == k2 and torch.equal(p, q)
    torch.manual_seed(4)
    a = ngnn.SimpleGCN(10, 12, 4, 2)
    torch.manual_seed(4)
    b = pyg_ref.SimpleGCN(10, 12, 4, 2)
    for (k, p), (k2, q) in zip(a.state_dict().items(), b.state_dict().items()):
        assert k == k2 and torch.equal(p, q)


def test_eager_extension_loads_and_binds():
    """The eager stack's C++ node (ngnn/lib/eager/ngnn_eager.so, built by
    __graft_entry__.build()) imports and takes the library's entry points
    (no compute call: no GPU here)."""
    from ngnn import _eager
    if not os.path.exists(_eager.SO_PATH):
        pytest.skip("ngnn_eager.so not built")
    mod = _eager.load()
    assert mod is not None and callable(mod.sage2) and callable(mod.init)
