"""Layer sharding of a model's Linear weights across the GPUs of one node.

The reference quantizes layer after layer on whichever GPU accelerate placed them
(utils.py:43 device_map="balanced", quant_wrapper.py:52-82) — one GPU busy at a time.  Here
every Linear weight is an independent unit of work, so the set is bin-packed by bytes over the
ranks (one process per GPU) and each rank quantizes its shard with ONE batched launch; there is no
exchange in the data path.  Optionally the fp16 weights start on rank 0 and are scattered to the
ranks that own them (`scatter_from_rank0`: one point-to-point send per destination, all in flight
together, so rank 0's xGMI links to the other GPUs run in parallel), and the packed results (int
codes + fp16 scales/zeros, ~1/4 of the fp16 bytes) are gathered back to rank 0 by the mirror
image: one point-to-point send per rank, all receives posted together on rank 0 (RCCL over xGMI on
MI355X, gloo in the CPU tests).
"""
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

# Linear shapes [out_features, in_features] per decoder layer (HF naming)
LLAMA_LAYERS = {
    "llama2-7b": (32, [("self_attn.q_proj", 4096, 4096), ("self_attn.k_proj", 4096, 4096),
                       ("self_attn.v_proj", 4096, 4096), ("self_attn.o_proj", 4096, 4096),
                       ("mlp.gate_proj", 11008, 4096), ("mlp.up_proj", 11008, 4096),
                       ("mlp.down_proj", 4096, 11008)]),
    "llama2-70b": (80, [("self_attn.q_proj", 8192, 8192), ("self_attn.k_proj", 1024, 8192),
                        ("self_attn.v_proj", 1024, 8192), ("self_attn.o_proj", 8192, 8192),
                        ("mlp.gate_proj", 28672, 8192), ("mlp.up_proj", 28672, 8192),
                        ("mlp.down_proj", 8192, 28672)]),
    "opt-125m": (12, [("self_attn.q_proj", 768, 768), ("self_attn.k_proj", 768, 768),
                      ("self_attn.v_proj", 768, 768), ("self_attn.out_proj", 768, 768),
                      ("fc1", 3072, 768), ("fc2", 768, 3072)]),
}


def model_linear_shapes(model: str) -> List[Tuple[str, Tuple[int, int]]]:
    """All quantized Linear weights of a model (lm_head excluded, quant_wrapper.py:53)."""
    n_layers, per = LLAMA_LAYERS[model]
    prefix = "model.decoder.layers" if model.startswith("opt") else "model.layers"
    return [(f"{prefix}.{i}.{n}", (r, c)) for i in range(n_layers) for n, r, c in per]


def plan_shards(shapes: Sequence[Tuple[str, Tuple[int, int]]], world: int) -> List[List[int]]:
    """Greedy longest-processing-time bin packing by element count; deterministic (ties by index).

    Returns, per rank, the indices into `shapes` it owns (in ascending index order)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    order = sorted(range(len(shapes)), key=lambda i: (-shapes[i][1][0] * shapes[i][1][1], i))
    loads = [0] * world
    bins: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: (loads[k], k))
        bins[r].append(i)
        loads[r] += shapes[i][1][0] * shapes[i][1][1]
    return [sorted(b) for b in bins]


def shard_imbalance(shapes, bins) -> float:
    loads = [sum(shapes[i][1][0] * shapes[i][1][1] for i in b) for b in bins]
    return max(loads) / (sum(loads) / len(loads))


@dataclass
class ShardResult:
    names: List[str]
    codes: List[torch.Tensor]     # packed codes per owned tensor (uint8)
    scales: List[torch.Tensor]
    zeros: List[Optional[torch.Tensor]]


def quantize_shard(named: Dict[str, torch.Tensor], n_bits: int, group: int, symmetric: bool,
                   quantize_fn: Optional[Callable] = None) -> ShardResult:
    """Quantize this rank's weights IN PLACE (dequantized values overwrite them, QuantLinear
    semantics) and keep packed codes + scales/zeros.  `quantize_fn(list_of_weights) -> (codes,
    scales, zeros)` may be injected by tests; the default is one batched gfx950 launch."""
    names = sorted(named)
    ws = [named[n] for n in names]
    if quantize_fn is None:
        from . import kernels
        plan = kernels.BatchPlan(ws, n_bits, group, symmetric, outs=ws, want_codes=True)
        plan.run()
        codes, scales, zeros = plan.codes, plan.scales, plan.zeros
    else:
        codes, scales, zeros = quantize_fn(ws)
    return ShardResult(names, list(codes), list(scales), list(zeros))


def _flatten(res: ShardResult) -> torch.Tensor:
    """One rank's packed results back to back in name order (the order gather_to_rank0 unpacks)."""
    parts = []
    order = sorted(range(len(res.names)), key=lambda i: res.names[i])
    for i in order:
        c, s, z = res.codes[i], res.scales[i], res.zeros[i]
        parts.append(c.reshape(-1).view(torch.uint8))
        parts.append(s.reshape(-1).view(torch.uint8))
        if z is not None:
            parts.append(z.reshape(-1).view(torch.uint8))
    if not parts:
        return torch.zeros(0, dtype=torch.uint8)
    return torch.cat([p.to(parts[0].device) for p in parts])


def n_groups(rows: int, cols: int, group: int) -> int:
    """Parameter count G of one [rows, cols] weight (quant_dim 0, the sharded path's layout):
    group > 0 -> rows*cols/group, -1 (per-tensor) -> 1, -2 (per-channel) -> rows
    (quant_linear.py:896-906; kernels.group_geometry without the torch dependency)."""
    if group > 0:
        if cols % group:
            raise ValueError(f"group {group} does not divide {cols} columns")
        return rows * cols // group
    if group == -1:
        return 1
    if group == -2:
        return rows
    raise ValueError("Invalid w_group_size")


def packed_nbytes(shape: Tuple[int, int], n_bits: int, group: int, symmetric: bool, esz: int = 2) -> int:
    """Bytes of one weight's packed result in the gather layout: codes, scales[, zeros]."""
    rows, cols = shape
    ncode = rows * (cols // 2) if n_bits <= 4 else rows * cols
    G = n_groups(rows, cols, group)
    return ncode + G * esz * (1 if symmetric else 2)


def gather_to_rank0(res: ShardResult, shapes: Dict[str, Tuple[int, int]], all_bins_names: List[List[str]],
                    n_bits: int, group: int, symmetric: bool, dtype=torch.float16, pg=None, stats=None):
    """Rooted gather of every rank's packed results to rank 0: each rank r > 0 sends its flat
    buffer once, rank 0 posts one receive per rank, all in flight together (batch_isend_irecv; on an
    xGMI node the 7 links into rank 0 run in parallel).  Every bin's size follows from the shard
    plan, so there is no size exchange, and each byte crosses the fabric exactly once (an all_gather
    would deliver every shard to every rank: N x the bytes).

    `stats` (a dict, optional) receives the bytes this rank sent / received.
    Returns {name: (codes, scales, zeros)} on rank 0, None elsewhere."""
    import torch.distributed as dist
    rank = dist.get_rank(pg)
    world = dist.get_world_size(pg)
    esz = torch.tensor([], dtype=dtype).element_size()
    sizes = [sum(packed_nbytes(shapes[n], n_bits, group, symmetric, esz) for n in all_bins_names[r])
             for r in range(world)]
    flat = _flatten(res)
    if flat.numel() != sizes[rank]:
        raise ValueError(f"gather_to_rank0: rank {rank} holds {flat.numel()} packed bytes, the plan says {sizes[rank]}")
    # gloo (CPU tests / 1-GPU rehearsal) has no device-memory point-to-point: stage through the host
    staged = dist.get_backend(pg) == "gloo" and flat.is_cuda
    if staged:
        flat = flat.cpu()
    dev = flat.device
    # point-to-point peers are GLOBAL ranks, also inside a sub-group
    peer = (lambda r: r) if pg is None else (lambda r: dist.get_global_rank(pg, r))
    if any(sz == 0 for sz in sizes[1:]):
        # a rank with an empty bin posts no operation; batch_isend_irecv must not be the group's
        # first collective then (RCCL/NCCL: every rank joins the first one)
        dist.barrier(group=pg)
    outs = [None] * world
    if rank == 0:
        outs[0] = flat
        ops = []
        for r in range(1, world):
            outs[r] = torch.empty(sizes[r], dtype=torch.uint8, device=dev)
            if sizes[r]:
                ops.append(dist.P2POp(dist.irecv, outs[r], peer(r), group=pg))
    else:
        ops = [dist.P2POp(dist.isend, flat, peer(0), group=pg)] if sizes[rank] else []
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if stats is not None:
        stats["sent_bytes"] = 0 if rank == 0 else sizes[rank]
        stats["recv_bytes"] = sum(sizes[1:]) if rank == 0 else 0
    if rank != 0:
        return None
    result = {}
    for r in range(world):
        off = 0
        data = outs[r]
        for name in sorted(all_bins_names[r]):
            rows, cols = shapes[name]
            ncode = rows * (cols // 2) if n_bits <= 4 else rows * cols
            G = n_groups(rows, cols, group)
            codes = data[off: off + ncode].clone()
            off += ncode
            scales = data[off: off + G * esz].clone().view(dtype)
            off += G * esz
            zeros = None
            if not symmetric:
                zeros = data[off: off + G * esz].clone().view(dtype)
                off += G * esz
            result[name] = (codes, scales, zeros)
    return result


def bin_layout(shapes: Sequence[Tuple[str, Tuple[int, int]]], bin_: List[int]):
    """Flat layout of one rank's weights: [(name, element offset, (rows, cols))], total elements.
    Tensors are placed back to back in name order, each start rounded to 8 elements (16 B)."""
    items, off = [], 0
    for i in sorted(bin_, key=lambda i: shapes[i][0]):
        name, (r, c) = shapes[i]
        items.append((name, off, (r, c)))
        off += (r * c + 7) // 8 * 8
    return items, off


def views_of(flat: torch.Tensor, layout) -> Dict[str, torch.Tensor]:
    """{name: [rows, cols] view} into a rank's flat weight buffer (no copies)."""
    return {name: flat[off: off + r * c].view(r, c) for name, off, (r, c) in layout}


def scatter_from_rank0(send_flats: Optional[List[torch.Tensor]], recv_flat: Optional[torch.Tensor], pg=None):
    """Rank 0 holds every rank's flat weight buffer (send_flats[r]); every other rank receives its
    own into recv_flat.  One isend per destination, issued together (batch_isend_irecv), so on an
    xGMI node rank 0 drives its links to the 7 other GPUs concurrently.  Returns this rank's flat
    buffer (rank 0: send_flats[0], no copy)."""
    import torch.distributed as dist
    rank = dist.get_rank(pg)
    world = dist.get_world_size(pg)
    # gloo (CPU tests / 1-GPU rehearsal) has no device-memory point-to-point: stage through the host
    staged = dist.get_backend(pg) == "gloo" and any(
        t is not None and t.is_cuda for t in ([recv_flat] + list(send_flats or [])))
    host = (lambda t: t.cpu()) if staged else (lambda t: t)
    peer = (lambda r: r) if pg is None else (lambda r: dist.get_global_rank(pg, r))  # global ranks
    if rank == 0:
        ops = [dist.P2POp(dist.isend, host(send_flats[r]), peer(r), group=pg) for r in range(1, world)]
        rbuf = None
    else:
        rbuf = torch.empty(recv_flat.shape, dtype=recv_flat.dtype) if staged else recv_flat
        ops = [dist.P2POp(dist.irecv, rbuf, peer(0), group=pg)]
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if rank != 0 and staged:
        recv_flat.copy_(rbuf)
    return send_flats[0] if rank == 0 else recv_flat
