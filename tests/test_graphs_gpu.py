"""HIP-graph replay of the training step (ngnn/graphs.py) against eager
training on the same batches: same parameters after several steps (dropout
off), fresh dropout masks per replay (dropout on), padded slot rows inert."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _setup(dropout, seed=5):
    import ngnn
    from ngnn.loader import NeighborLoader, synthetic_graph
    g = synthetic_graph("ogbn-arxiv", DEV, seed=0, scale=0.05)
    loader = NeighborLoader(g, g.train_idx, [10, 5], 256, shuffle=True, seed=seed)
    batches = [b for _, b in zip(range(4), loader)]
    torch.manual_seed(11)
    model = ngnn.SAGE(g.x.size(1), 64, g.num_classes, 2, dropout=dropout).to(DEV)
    return model, batches


def _eager_train(model, batches, lr=1e-2):
    opt = torch.optim.Adam(model.parameters(), lr=lr, fused=True, capturable=True)
    losses = []
    for b in batches:
        out = model(b.x, b.edge_index)[:b.batch_size]
        loss = F.cross_entropy(out, b.y[:b.batch_size])
        opt.zero_grad(set_to_none=False)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    return losses


def test_graph_training_matches_eager():
    from ngnn.graphs import GraphedTrainStep, slot_size
    m_e, batches = _setup(0.0)
    m_g, _ = _setup(0.0)
    m_g.load_state_dict(m_e.state_dict())
    le = _eager_train(m_e, batches)
    opt = torch.optim.Adam(m_g.parameters(), lr=1e-2, fused=True, capturable=True)
    n_cap, e_cap = slot_size(256, [10, 5])
    step = GraphedTrainStep(m_g, opt, 256, n_cap, e_cap, batches[0].x.size(1), DEV)
    step.capture(batches[0].x, batches[0].edge_index, batches[0].y)  # restores the state
    lg = []
    for b in batches:
        lg.append(float(step(b.x, b.edge_index, b.y)))
    torch.cuda.synchronize()
    for a, b in zip(le, lg):
        assert abs(a - b) < 1e-4 * max(1.0, abs(a)), (le, lg)
    for (n, pe), pg in zip(m_e.named_parameters(), m_g.parameters()):
        torch.testing.assert_close(pg, pe, rtol=1e-4, atol=1e-5, msg=n)


def test_graph_dropout_fresh_mask_per_replay():
    from ngnn.graphs import GraphedTrainStep, slot_size
    m, batches = _setup(0.5)
    opt = torch.optim.Adam(m.parameters(), lr=0.0, fused=True, capturable=True)  # lr 0: only masks vary
    n_cap, e_cap = slot_size(256, [10, 5])
    step = GraphedTrainStep(m, opt, 256, n_cap, e_cap, batches[0].x.size(1), DEV)
    b = batches[0]
    step.capture(b.x, b.edge_index, b.y)
    losses = [float(step(b.x, b.edge_index, b.y)) for _ in range(4)]
    assert all(torch.isfinite(torch.tensor(losses)))
    assert len(set(losses)) == 4, losses  # a new dropout mask every replay


def test_slot_padding_rows_inert():
    """A batch loaded into a bigger slot gives the same seed-row outputs as
    the bare batch (padding self-loops never reach a real row)."""
    from ngnn.graphs import GraphedTrainStep, slot_size
    m, batches = _setup(0.0)
    m.eval()
    b = batches[1]
    n_cap, e_cap = slot_size(256, [10, 5])
    opt = torch.optim.Adam(m.parameters(), lr=0.0, fused=True, capturable=True)
    step = GraphedTrainStep(m, opt, 256, n_cap, e_cap, b.x.size(1), DEV)
    step.load(b.x, b.edge_index, b.y)
    from ngnn.block import hint_edge_index
    hint_edge_index(step.ei, dst_sorted=True, src_sorted=False, n_rows_dev=step.n_valid)
    with torch.no_grad():
        full = m(step.x, step.ei)[:b.num_nodes]
        ref = m(b.x, b.edge_index)
    torch.testing.assert_close(full, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("tight", [False, True])
def test_slot_csr_and_seed(tight):
    """The CSR the slot load writes equals the one the Block builder makes
    from the slot's padded edges (with and without padding edges), and the
    dropout seed state moves on every load."""
    from ngnn.block import build_csr
    from ngnn.graphs import GraphedTrainStep, slot_size
    m, batches = _setup(0.0)
    b = batches[2]
    N, E = b.x.size(0), b.edge_index.size(1)
    n_cap, e_cap = (N + 1, E) if tight else slot_size(256, [10, 5])
    opt = torch.optim.Adam(m.parameters(), lr=0.0, fused=True, capturable=True)
    step = GraphedTrainStep(m, opt, 256, n_cap, e_cap, b.x.size(1), DEV)
    seeds = []
    for _ in range(2):
        step.load(b.x, b.edge_index, b.y)
        seeds.append(int(step.seed_state.item()))
    ref = build_csr(step.ei[1], step.ei[0], n_cap, True)
    assert torch.equal(step.rowptr, ref.rowptr)
    assert torch.equal(step.col, ref.col)
    assert seeds[0] != seeds[1]


def test_graph_short_last_batch_matches_eager():
    """an epoch's last batch (drop_last off) has fewer seeds than
    the captured B.  Its replay must equal the reference loop on that batch,
    F.cross_entropy(out[:bs], y[:bs]) (pipeline.py:155-158): rows [bs, B)
    carry no loss."""
    import ngnn
    from ngnn.graphs import GraphedTrainStep, slot_size
    from ngnn.loader import NeighborLoader, synthetic_graph
    g = synthetic_graph("ogbn-arxiv", DEV, seed=0, scale=0.05)
    seeds = g.train_idx[:256 * 2 + 37]
    loader = NeighborLoader(g, seeds, [10, 5], 256, shuffle=False)
    batches = list(loader)
    assert [b.batch_size for b in batches] == [256, 256, 37]
    torch.manual_seed(11)
    m_e = ngnn.SAGE(g.x.size(1), 64, g.num_classes, 2, dropout=0.0).to(DEV)
    torch.manual_seed(11)
    m_g = ngnn.SAGE(g.x.size(1), 64, g.num_classes, 2, dropout=0.0).to(DEV)
    le = _eager_train(m_e, batches)
    opt = torch.optim.Adam(m_g.parameters(), lr=1e-2, fused=True, capturable=True)
    n_cap, e_cap = slot_size(256, [10, 5])
    step = GraphedTrainStep(m_g, opt, 256, n_cap, e_cap, g.x.size(1), DEV)
    step.capture(batches[0].x, batches[0].edge_index, batches[0].y)
    lg = [float(step(b.x, b.edge_index, b.y, b.batch_size)) for b in batches]
    torch.cuda.synchronize()
    for a, c in zip(le, lg):
        assert abs(a - c) < 1e-4 * max(1.0, abs(a)), (le, lg)
    for (n, pe), pg in zip(m_e.named_parameters(), m_g.parameters()):
        torch.testing.assert_close(pg, pe, rtol=1e-4, atol=1e-5, msg=n)


def test_bucket_view_gradients_adopted():
    """GradAllReduce registers bucket views; the fused backward writes the
    weight gradients into them and autograd adopts them as .grad (no pack /
    unpack copies), in eager and in graph replay, with the same values as
    without the bucket."""
    import ngnn
    from ngnn.distributed import GradAllReduce
    m, batches = _setup(0.0)
    ref = {k: None for k, _ in m.named_parameters()}
    b = batches[0]
    F.cross_entropy(m(b.x, b.edge_index)[:b.batch_size], b.y[:b.batch_size]).backward()
    ref = {k: p.grad.clone() for k, p in m.named_parameters()}
    red = GradAllReduce(m.parameters())
    m.zero_grad(set_to_none=True)
    F.cross_entropy(m(b.x, b.edge_index)[:b.batch_size], b.y[:b.batch_size]).backward()
    for (k, p), v in zip(m.named_parameters(), red.views):
        assert p.grad.data_ptr() == v.data_ptr(), k
        # (the input-gradient scatter uses float atomics: order-dependent bits)
        torch.testing.assert_close(p.grad, ref[k], rtol=1e-5, atol=1e-6, msg=k)


@pytest.mark.parametrize("mode", ["two_forwards", "retain_graph", "accumulate"])
def test_bucket_views_not_aliased(mode):
    """Bucket views registered, the gradients must equal the ones computed
    without the bucket when the views could alias: two forwards (sharing the
    parameters) before one backward (pipeline_contrast.py:146-154 runs the
    model on several batches per step), one graph back-propagated twice
    (retain_graph), and accumulation over two steps without zero_grad."""
    from ngnn.distributed import GradAllReduce
    m, batches = _setup(0.0)
    b0, b1 = batches[0], batches[1]

    def loss_of(b):
        return F.cross_entropy(m(b.x, b.edge_index)[:b.batch_size], b.y[:b.batch_size])

    def run():
        m.zero_grad(set_to_none=True)
        if mode == "two_forwards":
            (loss_of(b0) + loss_of(b1)).backward()
        elif mode == "retain_graph":
            l0 = loss_of(b0)
            l0.backward(retain_graph=True)
            l0.backward()
        else:
            loss_of(b0).backward()
            loss_of(b1).backward()
        torch.cuda.synchronize()
        return {k: p.grad.clone() for k, p in m.named_parameters()}

    ref = run()
    red = GradAllReduce(m.parameters())
    got = run()
    for k in ref:
        # (the input-gradient scatter uses float atomics: order-dependent bits)
        torch.testing.assert_close(got[k], ref[k], rtol=1e-5, atol=1e-6, msg=k)
    # the bucket still works for the next plain step
    got2 = run()
    for k in ref:
        torch.testing.assert_close(got2[k], ref[k], rtol=1e-5, atol=1e-6, msg=k)
    del red


@pytest.mark.parametrize("arch", ["sage", "gcn"])
def test_graph_fused_row_gather_matches_eager(arch):
    """NeighborLoader(gather_features=False) batches carry x = graph.x[n_id]
    unmaterialized; the captured step hands table + n_id to the layer-0
    kernels (forward gather and weight gradient read table rows n_id[r]).
    Same losses and parameters as eager training on the materialized rows,
    and a plain batch loaded into the same graph (index word 0) still works."""
    import ngnn
    from ngnn.graphs import GraphedTrainStep, slot_size
    from ngnn.loader import IndexedRows, NeighborLoader, synthetic_graph
    g = synthetic_graph("ogbn-arxiv", DEV, seed=0, scale=0.05)
    lo = NeighborLoader(g, g.train_idx, [10, 5], 256, shuffle=True, seed=3, gather_features=False)
    batches = [b for _, b in zip(range(4), lo)]
    assert isinstance(batches[0].x, IndexedRows)
    torch.testing.assert_close(batches[0].x.materialize(), g.x[batches[0].n_id], rtol=0, atol=0)

    def make():
        torch.manual_seed(11)
        if arch == "sage":
            return ngnn.SAGE(g.x.size(1), 64, g.num_classes, 2, dropout=0.0).to(DEV)
        return ngnn.SimpleGCN(g.x.size(1), 160, g.num_classes, 2, dropout=0.0).to(DEV)

    m_e, m_g = make(), make()
    plain = [type(b)(b.x.materialize(), b.y, b.edge_index, b.n_id, b.batch_size) for b in batches]
    le = _eager_train(m_e, plain)
    opt = torch.optim.Adam(m_g.parameters(), lr=1e-2, fused=True, capturable=True)
    n_cap, e_cap = slot_size(256, [10, 5])
    step = GraphedTrainStep(m_g, opt, 256, n_cap, e_cap, g.x.size(1), DEV)
    step.capture(batches[0].x, batches[0].edge_index, batches[0].y)
    assert step.zero_copy and step.x_rows == g.num_nodes
    lg = [float(step(b.x, b.edge_index, b.y)) for b in batches[:3]]
    lg.append(float(step(plain[3].x, plain[3].edge_index, plain[3].y)))  # word 0: plain rows
    torch.cuda.synchronize()
    for a, c in zip(le, lg):
        assert abs(a - c) < 1e-4 * max(1.0, abs(a)), (le, lg)
    for (n, pe), pg in zip(m_e.named_parameters(), m_g.parameters()):
        torch.testing.assert_close(pg, pe, rtol=1e-4, atol=1e-5, msg=n)


def test_graph_bf16_features_slot_matches_eager():
    """bf16 features: the slot is bf16 and the captured layer 0 reads the
    batch's bf16 rows in place (NGNN_X_BF16 + zero-copy); same losses and
    parameters as eager training on the same bf16 batches.  Deterministic
    mode (gather-based input gradient): with the atomic scatter, Adam's
    division by sqrt(v) turns ordering noise on ~0 gradient entries into
    update differences of order lr."""
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        _graph_bf16_features_slot_matches_eager()
    finally:
        torch.use_deterministic_algorithms(False)


def _graph_bf16_features_slot_matches_eager():
    from ngnn.graphs import GraphedTrainStep, slot_size
    m_e, batches = _setup(0.0)
    m_g, _ = _setup(0.0)
    m_g.load_state_dict(m_e.state_dict())
    bb = [type(b)(b.x.to(torch.bfloat16), b.y, b.edge_index, b.n_id, b.batch_size) for b in batches]
    # eager reference with the step's own loss (fp32 softmax over the bf16
    # logits; F.cross_entropy on bf16 logits would round the loss to bf16)
    from ngnn.losses import seed_cross_entropy
    o_e = torch.optim.Adam(m_e.parameters(), lr=1e-2, fused=True, capturable=True)
    le = []
    for b in bb:
        loss = seed_cross_entropy(m_e(b.x, b.edge_index), b.y, b.batch_size)
        o_e.zero_grad(set_to_none=False)
        loss.backward()
        o_e.step()
        le.append(float(loss))
    opt = torch.optim.Adam(m_g.parameters(), lr=1e-2, fused=True, capturable=True)
    n_cap, e_cap = slot_size(256, [10, 5])
    step = GraphedTrainStep(m_g, opt, 256, n_cap, e_cap, bb[0].x.size(1), DEV)
    step.capture(bb[0].x, bb[0].edge_index, bb[0].y)
    assert step.x.dtype == torch.bfloat16 and step.zero_copy
    lg = [float(step(b.x, b.edge_index, b.y)) for b in bb]
    torch.cuda.synchronize()
    for a, c in zip(le, lg):
        assert abs(a - c) < 1e-4 * max(1.0, abs(a)), (le, lg)
    for (n, pe), pg in zip(m_e.named_parameters(), m_g.parameters()):
        torch.testing.assert_close(pg, pe, rtol=1e-4, atol=1e-5, msg=lambda m, n=n: f"{n}: {m}")


@pytest.mark.parametrize("case", ["block", "gaps", "empty", "full"])
def test_slot_load_csr_equals_lower_bound(case):
    """ngnn_slot_load's target-grouped CSR of the padded edges: rowptr[r] =
    the lower bound of r over the padded targets (real edges, then padding
    self-loops spread over rows N .. n_cap), rowptr[n_cap] = e_cap, col the
    sources -- for a NeighborLoader-like block, targets with gaps (rows with
    no in-edges among the targets, first target > 0), no edges, and a full
    slot (E = e_cap)."""
    from ngnn import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(3)
    N, n_cap, e_cap, F = 500, 700, 3000, 4
    if case == "empty":
        dst = torch.zeros(0, dtype=torch.int64)
    elif case == "gaps":
        dst = torch.sort(5 + 2 * torch.randint(0, 120, (2000,), generator=g)).values
    elif case == "full":
        N = n_cap = 500
        dst = torch.sort(torch.randint(0, N, (e_cap,), generator=g)).values
    else:
        dst = torch.sort(torch.randint(0, 300, (2500,), generator=g)).values
    E = dst.numel()
    src = torch.randint(0, N, (E,), generator=g)
    ei = torch.stack([src, dst]).to(DEV).contiguous()
    x = torch.randn(N, F, generator=g).to(DEV)
    y = torch.zeros(8, dtype=torch.int64, device=DEV)
    sx = torch.zeros(n_cap, F, device=DEV)
    sei = torch.full((2 * e_cap,), -1, dtype=torch.int64, device=DEV)
    sy = torch.zeros(8, dtype=torch.int64, device=DEV)
    nv = torch.zeros(1, dtype=torch.int32, device=DEV)
    rowptr = torch.full((n_cap + 1,), -7, dtype=torch.int32, device=DEV)
    col = torch.full((e_cap,), -7, dtype=torch.int32, device=DEV)
    _lib.check(lib.ngnn_slot_load(
        _lib.ptr(x), x.stride(0), N, F, _lib.ptr(ei) if E else None, max(E, 0), E, _lib.ptr(y), 8,
        _lib.ptr(sx), sx.stride(0), n_cap, _lib.ptr(sei), e_cap, _lib.ptr(sy), _lib.ptr(nv),
        _lib.ptr(rowptr), _lib.ptr(col), None, None, None, 0, None, None, None, None,
        None, 0, 0, 0, None, None, None, None, _lib.stream_handle(DEV)), "ngnn_slot_load")
    torch.cuda.synchronize()
    n_pad, span = e_cap - E, n_cap - N
    pad = N + (torch.arange(n_pad) * span) // max(n_pad, 1) if n_pad else torch.zeros(0, dtype=torch.int64)
    dst_p = torch.cat([dst, pad])
    want = torch.searchsorted(dst_p, torch.arange(n_cap + 1), right=False).to(torch.int32)
    want[n_cap] = e_cap
    assert torch.equal(rowptr.cpu(), want)
    assert torch.equal(col.cpu(), torch.cat([src, pad]).to(torch.int32))
    assert torch.equal(sei.cpu()[e_cap:], dst_p)


def test_slot_rejects_unsorted_targets():
    """The slot load writes the CSR for non-decreasing targets only: the slot
    kernel checks every batch itself (ABI 16, no host read-back), and an
    unsorted one is reported -- by check_inputs() after a sync, and by the
    next load() without one."""
    from ngnn.graphs import GraphedTrainStep, slot_size
    m, batches = _setup(0.0)
    b = batches[0]
    opt = torch.optim.Adam(m.parameters(), lr=1e-2, fused=True, capturable=True)
    n_cap, e_cap = slot_size(256, [10, 5])
    step = GraphedTrainStep(m, opt, 256, n_cap, e_cap, b.x.size(1), DEV)
    step.load(b.x, b.edge_index, b.y)            # sampler output (hinted): accepted
    step.load(b.x, b.edge_index.clone(), b.y)    # unhinted but sorted: accepted
    step.check_inputs()
    perm = torch.randperm(b.edge_index.size(1), device=DEV)
    step.load(b.x, b.edge_index[:, perm], b.y)
    with pytest.raises(ValueError, match="not sorted"):
        step.check_inputs()
    step.load(b.x, b.edge_index[:, perm], b.y)
    torch.cuda.synchronize()
    with pytest.raises(ValueError, match="not sorted"):
        step.load(b.x, b.edge_index, b.y)  # (the previous batch's word, no sync in load)
    step.load(b.x, b.edge_index, b.y)
    step.check_inputs()


@pytest.mark.parametrize("fo,k", [(256, 100), (47, 256), (5, 3), (600, 64)])
def test_slot_pack_job_equals_pack_weight(fo, k):
    """ngnn_slot_load's pack job writes exactly ngnn_pack_weight's fragment
    layout (zero padding included) of the weight's current values."""
    from ngnn import _lib
    from ngnn.fused import pack_weight
    lib = _lib.load()
    g = torch.Generator().manual_seed(fo + k)
    w = torch.randn(fo, k + 3, generator=g).to(DEV)[:, :k]  # row stride k + 3
    dst = torch.full((lib.ngnn_pack_weight_bytes(fo, k) // 4,), 7.0, device=DEV)
    N, F, n_cap = 4, 4, 8
    x = torch.zeros(N, F, device=DEV)
    y = torch.zeros(1, dtype=torch.int64, device=DEV)
    sx = torch.zeros(n_cap, F, device=DEV)
    sy = torch.zeros(1, dtype=torch.int64, device=DEV)
    sei = torch.zeros(2, 2, dtype=torch.int64, device=DEV)
    ei = torch.tensor([[0, 1], [0, 1]], device=DEV)
    nv = torch.zeros(1, dtype=torch.int32, device=DEV)
    _lib.check(lib.ngnn_slot_load(
        _lib.ptr(x), F, N, F, _lib.ptr(ei), 2, 2, _lib.ptr(y), 1, _lib.ptr(sx), F, n_cap,
        _lib.ptr(sei), 2, _lib.ptr(sy), _lib.ptr(nv), None, None, None, None, None, 0, None,
        None, None, None, _lib.ptr(w), w.stride(0), fo, k, _lib.ptr(dst), None, None, None,
        _lib.stream_handle(DEV)), "ngnn_slot_load")
    want = pack_weight(w)
    torch.cuda.synchronize()
    assert torch.equal(dst, want)


def test_slot_prepacked_wl_never_stale():
    """the slot's packed layer-0 W_l is valid for the one forward
    after each load() only.  An eager forward over the slot after a replay
    (whose Adam changed W_l, no new load) must pack W_l itself: it equals a
    forward of the same model on an unhinted copy of the batch."""
    import ngnn
    from ngnn.graphs import GraphedTrainStep, slot_size
    from ngnn.loader import sample_block, synthetic_graph
    from ngnn.optim import Adam
    g = synthetic_graph("ogbn-products", DEV, seed=1, scale=0.02)
    b = sample_block(g, g.train_idx[:256], [15, 10, 5], seed=3)
    torch.manual_seed(5)
    model = ngnn.SAGE(100, 256, 47, 3, dropout=0.0).to(DEV)  # per-layer path: layer 0 streams W_l
    opt = Adam(model.parameters(), lr=1e-2)
    n_cap, e_cap = slot_size(256, [15, 10, 5])
    step = GraphedTrainStep(model, opt, 256, n_cap, e_cap, 100, DEV)
    step.capture(b.x, b.edge_index, b.y)
    step(b.x, b.edge_index, b.y)  # load (packs W_l), replay (Adam moves W_l)
    with torch.no_grad():
        got = model(step.x, step.ei)[:b.num_nodes]
        want = model(b.x.clone(), b.edge_index.clone())
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-5)


def test_slot_contract_error_word():
    """ABI 16: the slot kernel checks the block's contract itself (targets
    non-decreasing, ids in [0, N)) and ORs NGNN_SLOT_* into a pinned word --
    no host read-back of the targets per load; check_inputs() syncs and
    raises, and a good batch afterwards trains normally."""
    import ngnn
    from ngnn.graphs import GraphedTrainStep, slot_size
    from ngnn.loader import sample_block, synthetic_graph
    from ngnn.optim import Adam
    graph = synthetic_graph("ogbn-products", DEV, seed=3, scale=0.005)
    b = sample_block(graph, graph.train_idx[:64], [5, 3], seed=1)
    torch.manual_seed(0)
    model = ngnn.SAGE(100, 64, 47, 2).to(DEV)
    n_cap, e_cap = slot_size(64, [5, 3])
    step = GraphedTrainStep(model, Adam(model.parameters(), lr=1e-3), 64, n_cap, e_cap, 100, DEV)
    step.capture(b.x, b.edge_index, b.y)
    step(b.x, b.edge_index, b.y)
    step.check_inputs()  # a NeighborLoader block: clean
    bad = b.edge_index.flip(1).contiguous()  # targets descending
    before = [p.detach().clone() for p in model.parameters()]
    n_step = float(step.opt.state[next(model.parameters())]["step"])
    step(b.x, bad, b.y)
    with pytest.raises(ValueError, match="not sorted"):
        step.check_inputs()
    # ABI 20: the contract gate -- the replay of a bad block updated nothing
    for p, q in zip(model.parameters(), before):
        assert torch.equal(p, q)
    assert float(step.opt.state[next(model.parameters())]["step"]) == n_step
    oob = b.edge_index.clone()
    oob[0, 0] = b.num_nodes + 5
    step(b.x, oob, b.y)
    with pytest.raises(ValueError, match="outside"):
        step.check_inputs()
    step(b.x, b.edge_index, b.y)
    step.check_inputs()
    assert torch.isfinite(step.loss).all()
    # sources far outside the slot (past n_cap, negative) are
    # flagged AND stored as row 0 -- no replayed gather or scatter leaves
    # its buffer; the CSR columns stay in [0, N)
    E = b.edge_index.shape[1]
    for v in (n_cap + 10**6, -7):
        far = b.edge_index.clone()
        far[0, :: max(1, E // 17)] = v
        step(b.x, far, b.y)
        with pytest.raises(ValueError, match="outside"):
            step.check_inputs()
        col = step.col[:E].cpu()
        assert int(col.min()) >= 0 and int(col.max()) < b.num_nodes
        assert 0 < (int(step.r_next.item()) & 0xFFFFFFFF) <= b.num_nodes
    step(b.x, b.edge_index, b.y)
    step.check_inputs()
    torch.cuda.synchronize()
    assert torch.isfinite(step.loss).all()
    assert all(torch.isfinite(p).all() for p in model.parameters())


def test_replay_survives_workspace_growth():
    """a captured step holds the raw addresses of the fused
    kernels' cached workspaces; an eager call on a larger block grows them --
    the superseded buffers must stay alive (fused._ws_retired), so the next
    replay reads and writes valid memory and gives the same gradients."""
    import ngnn
    from ngnn import fused
    from ngnn.graphs import GraphedTrainStep, slot_size
    from ngnn.loader import sample_block, synthetic_graph
    from ngnn.losses import seed_cross_entropy
    from ngnn.optim import Adam
    from gradbar import assert_wgrad
    # (a fresh workspace cache, sized by this test's small slot; the older
    # buffers retired, as a growth would)
    fused._ws_retired.extend(fused._ws.values())
    fused._ws.clear()
    graph = synthetic_graph("ogbn-products", DEV, seed=4, scale=0.02)
    small = sample_block(graph, graph.train_idx[:128], [15, 10], seed=2)
    big = sample_block(graph, graph.train_idx[:2048], [15, 10], seed=3)
    assert big.num_nodes > 2 * small.num_nodes
    torch.manual_seed(0)
    model = ngnn.SAGE(100, 256, 47, 2, dropout=0.0).to(DEV).train()
    opt = Adam(model.parameters(), lr=0.0)  # parameters fixed: replays comparable
    n_cap, e_cap = slot_size(128, [15, 10])
    step = GraphedTrainStep(model, opt, 128, n_cap, e_cap, 100, DEV)
    step.capture(small.x, small.edge_index, small.y)
    step(small.x, small.edge_index, small.y)
    torch.cuda.synchronize()
    g1 = {k: p.grad.detach().clone() for k, p in model.named_parameters()}
    before = {k: v.data_ptr() for k, v in fused._ws.items()}
    # an eager step on a block with many more rows: the workspaces grow
    other = ngnn.SAGE(100, 256, 47, 2, dropout=0.0).to(DEV).train()
    out = other(big.x, big.edge_index)
    seed_cross_entropy(out, big.y, big.batch_size).backward()
    torch.cuda.synchronize()
    grown = [k for k, v in fused._ws.items() if k in before and v.data_ptr() != before[k]]
    assert grown, "the larger block did not grow any workspace"
    torch.empty(1 << 28, dtype=torch.uint8, device=DEV).fill_(0xFF)  # reuse freed memory, if any
    step(small.x, small.edge_index, small.y)
    torch.cuda.synchronize()
    for k, p in model.named_parameters():
        assert_wgrad(p.grad, g1[k], msg=k)


@pytest.mark.parametrize("gather", [True, False])
def test_graph_training_over_sync_free_loader(gather):
    """GraphedTrainStep over NeighborLoader(sync_free=True) (ABI 19: the slot
    load reads the block's counts on the device, no host read-back per
    batch) trains exactly as over the synchronous loader's batches: same
    losses and parameters after a pass of 8 batches (headline architecture:
    the two-layer kernels, loss head and Adam fold in the replay)."""
    import ngnn
    from ngnn.graphs import GraphedTrainStep, slot_size
    from ngnn.loader import NeighborLoader, synthetic_graph
    from ngnn.optim import Adam
    g = synthetic_graph("ogbn-products", DEV, seed=0, scale=0.05)
    torch.manual_seed(2)
    init = ngnn.SAGE(100, 256, 47, 2, dropout=0.0).to(DEV).state_dict()
    res = []
    for sf in (False, True):
        m = ngnn.SAGE(100, 256, 47, 2, dropout=0.0).to(DEV)
        m.load_state_dict(init)
        opt = Adam(m.parameters(), lr=1e-3)
        n_cap, e_cap = slot_size(512, [15, 10])
        kw = dict(batch_size=512, shuffle=True, seed=4, gather_features=gather)
        cap = next(iter(NeighborLoader(g, g.train_idx, [15, 10], **kw)))
        step = GraphedTrainStep(m, opt, 512, n_cap, e_cap, 100, DEV)
        step.capture(cap.x, cap.edge_index, cap.y)
        losses = []
        for i, b in enumerate(NeighborLoader(g, g.train_idx, [15, 10], sync_free=sf, **kw)):
            if i == 8:
                break
            losses.append(step(b.x, b.edge_index, b.y).clone())
        step.check_inputs()
        res.append((torch.stack(losses).cpu(), [p.detach().clone() for p in m.parameters()]))
    # (the loss head's multi-edge scatter uses float atomics: its summation
    # order is not fixed, so the two runs agree to rounding, not bitwise)
    torch.testing.assert_close(res[1][0], res[0][0], rtol=1e-5, atol=1e-6)
    for a, b in zip(res[1][1], res[0][1]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


def test_graph_epoch_over_sync_free_loader_with_short_last_batch():
    """A whole epoch whose last block is short (train seeds not a multiple of
    the batch size) through GraphedTrainStep, sync-free loader against the
    synchronous one: the same losses and parameters (the short block's
    batch_size reaches the slot's ignore_index rows)."""
    import ngnn
    from ngnn.graphs import GraphedTrainStep, slot_size
    from ngnn.loader import NeighborLoader, synthetic_graph
    from ngnn.optim import Adam
    g = synthetic_graph("ogbn-products", DEV, seed=3, scale=0.01)
    assert g.train_idx.numel() % 512 != 0
    torch.manual_seed(5)
    init = ngnn.SAGE(100, 256, 47, 2, dropout=0.0).to(DEV).state_dict()
    res = []
    for sf in (False, True):
        m = ngnn.SAGE(100, 256, 47, 2, dropout=0.0).to(DEV)
        m.load_state_dict(init)
        opt = Adam(m.parameters(), lr=1e-3)
        n_cap, e_cap = slot_size(512, [15, 10])
        kw = dict(batch_size=512, shuffle=True, seed=9)
        cap = next(iter(NeighborLoader(g, g.train_idx, [15, 10], **kw)))
        step = GraphedTrainStep(m, opt, 512, n_cap, e_cap, 100, DEV)
        step.capture(cap.x, cap.edge_index, cap.y)
        losses = [step(b.x, b.edge_index, b.y, b.batch_size).clone()
                  for b in NeighborLoader(g, g.train_idx, [15, 10], sync_free=sf, **kw)]
        step.check_inputs()
        res.append((torch.stack(losses).cpu(), [p.detach().clone() for p in m.parameters()]))
    assert res[0][0].numel() == -(-g.train_idx.numel() // 512)
    torch.testing.assert_close(res[1][0], res[0][0], rtol=1e-5, atol=1e-6)
    for a, b in zip(res[1][1], res[0][1]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


def test_contract_gate_on_the_folded_step():
    """ABI 20 on the headline step (two-layer kernels, Adam folded into the
    backward's reduction): a block that breaks the slot's contract is
    replayed but changes no parameter, moment or step count; the next good
    block trains."""
    import ngnn
    from ngnn.graphs import GraphedTrainStep, slot_size
    from ngnn.loader import sample_block, synthetic_graph
    from ngnn.optim import Adam
    graph = synthetic_graph("ogbn-products", DEV, seed=3, scale=0.02)
    b = sample_block(graph, graph.train_idx[:256], [15, 10], seed=1)
    torch.manual_seed(0)
    model = ngnn.SAGE(100, 256, 47, 2).to(DEV)
    opt = Adam(model.parameters(), lr=1e-3)
    n_cap, e_cap = slot_size(256, [15, 10])
    step = GraphedTrainStep(model, opt, 256, n_cap, e_cap, 100, DEV)
    step.capture(b.x, b.edge_index, b.y)
    assert step.folded
    step(b.x, b.edge_index, b.y)
    step.check_inputs()

    def snap():
        p0 = next(model.parameters())
        st = opt.state[p0]
        return ([p.detach().clone() for p in model.parameters()], st["exp_avg"].clone(), float(st["step"]))

    before = snap()
    oob = b.edge_index.clone()
    oob[0, 3] = b.num_nodes + 7
    step(b.x, oob, b.y)
    with pytest.raises(ValueError, match="outside"):
        step.check_inputs()
    after = snap()
    assert all(torch.equal(p, q) for p, q in zip(after[0], before[0]))
    assert torch.equal(after[1], before[1]) and after[2] == before[2]
    step(b.x, b.edge_index, b.y)
    step.check_inputs()
    good = snap()
    assert good[2] == before[2] + 1
    assert not all(torch.equal(p, q) for p, q in zip(good[0], before[0]))
