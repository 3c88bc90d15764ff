"""Reference restatement of NeighborLoader's block construction for the
sampler parity tests (test infrastructure, never imported by the product).

The hops use the product's own per-hop sampler (``ngnn.loader.sample_hop``,
checked on its own in test_loader_gpu.py); the relabelling, first-appearance
ordering and edge layout are restated with plain torch ops, the way PyG's
NeighborLoader / pyg-lib neighbor_sample [ext] assigns local ids
(pipeline.py:75-83: seeds first, then every newly reached node in sampling
order)."""
import torch

from ngnn.loader import Batch, sample_hop


def sample_block_ref(graph, seeds, fanouts, seed):
    dev = seeds.device
    n_id = seeds.to(torch.int64)
    frontier = n_id
    frontier_local = torch.arange(n_id.numel(), device=dev)
    srcs, dsts = [], []
    n_active = n_id.numel()
    for hop, k in enumerate(fanouts):
        nbr, _ = sample_hop(graph, frontier, int(k), seed * 1_000_003 + hop)
        mask = nbr >= 0
        dst_local = frontier_local.unsqueeze(1).expand(-1, int(k))[mask]
        cand = nbr[mask]
        n_old = n_id.numel()
        n_active = n_old
        all_ids = torch.cat([n_id, cand])
        uniq, inv = torch.unique(all_ids, return_inverse=True)
        pos = torch.arange(all_ids.numel(), device=dev)
        first = torch.full((uniq.numel(),), all_ids.numel(), dtype=torch.int64, device=dev)
        first.scatter_reduce_(0, inv, pos, reduce="amin")
        order = torch.argsort(first)
        rank = torch.empty_like(order)
        rank[order] = torch.arange(order.numel(), device=dev)
        local_all = rank[inv]
        srcs.append(local_all[n_old:])
        dsts.append(dst_local)
        new_nodes = uniq[order[n_old:]]
        frontier_local = torch.arange(n_old, n_old + new_nodes.numel(), device=dev)
        n_id = torch.cat([n_id, new_nodes])
        frontier = new_nodes
    edge_index = torch.stack([torch.cat(srcs), torch.cat(dsts)]) if srcs else \
        torch.empty(2, 0, dtype=torch.int64, device=dev)
    x = graph.x.index_select(0, n_id)
    y = graph.y.index_select(0, n_id)
    return Batch(x, y, edge_index, n_id, int(seeds.numel())), n_active
