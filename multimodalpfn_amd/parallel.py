"""Ensemble-member sharding across the GPUs of one node.

Members are independent forwards (``inference.py:294-349``); the only cross-member
step is the softmax mean (``classifier.py:555-561``).  Each rank (one process per
GPU, ``torch.distributed`` with the ``nccl`` backend = RCCL over xGMI) runs the
members assigned to it by greedy longest-processing-time on the forward's flop model
(``member_cost``; units of equal-geometry members kept together) and contributes its fixed-size logit block to ONE all-gather.
There is no other collective on the data path.
"""

from __future__ import annotations

import heapq

import torch


def lpt_assign(costs: list[float], world: int, keys: list | None = None, unit: int = 1) -> list[list[int]]:
    """Greedy LPT: member indices per rank, heaviest first, to the least-loaded rank.

    With ``keys`` (one geometry key per member) and ``unit > 1`` the members of one key are first cut
    into units of ``unit`` (the engine's batched forward stacks exactly such members), and whole units
    are assigned, so the per-rank batching the single-GPU scheduler relies on survives the split."""
    if keys is None or unit <= 1:
        groups = [[i] for i in range(len(costs))]
    else:
        by_key: dict = {}
        for i, k in enumerate(keys):
            by_key.setdefault(k, []).append(i)
        groups = [ids[j : j + unit] for ids in by_key.values() for j in range(0, len(ids), unit)]
    gcost = [sum(costs[i] for i in g) for g in groups]
    heap = [(0.0, r) for r in range(world)]
    heapq.heapify(heap)
    out: list[list[int]] = [[] for _ in range(world)]
    for gi in sorted(range(len(groups)), key=lambda g: (-gcost[g], groups[g][0])):
        load, r = heapq.heappop(heap)
        out[r].extend(groups[gi])
        heapq.heappush(heap, (load + gcost[gi], r))
    return [sorted(x) for x in out]


def member_cost(n_tokens: int, S: int, N: int, E: int = 192, FF: int = 768) -> float:
    """Forward flops of one member per layer, up to a constant: per token the feature
    and item QKV / out projections (16 E^2), the MLP (4 E FF), the feature attention over the row's
    T tokens (4 T E) and the item attention against the N train rows (4 N E)."""
    T = float(n_tokens)
    return T * S * E * (16.0 * E + 4.0 * FF + 4.0 * N + 4.0 * T)


def allgather_logits(local: torch.Tensor, assignment: list[list[int]], rank: int, group=None,
                     force_collective: bool = False) -> torch.Tensor:
    """Gather every rank's ``[m_r, Q, n_out]`` logits into ``[n_members, Q, n_out]`` in member order.

    ``assignment`` (identical on every rank, from :func:`lpt_assign`) fixes the block
    sizes, so this is exactly one fixed-size ``all_gather`` of ``max_r m_r`` padded
    blocks; with one process it is a reorder.  ``force_collective`` (tests) takes the
    collective branch even for a world of one, so a single-GPU box executes the RCCL
    all-gather path.
    """
    import torch.distributed as dist

    n_members = sum(len(a) for a in assignment)
    tail = tuple(local.shape[1:])
    out = torch.empty((n_members,) + tail, device=local.device, dtype=local.dtype)
    distributed = dist.is_available() and dist.is_initialized()
    if not distributed or (dist.get_world_size(group) == 1 and not force_collective):
        if list(assignment[rank]) == list(range(n_members)):
            return local  # one process running every member in order: nothing to move
        out[_index(assignment[rank], local.device)] = local
        return out
    world = dist.get_world_size(group)
    assert len(assignment) == world and local.shape[0] == len(assignment[rank])
    m_max = max(len(a) for a in assignment)
    # RCCL gathers device tensors in place; a host-only backend (gloo) gathers host copies
    cdev = local.device if (local.device.type == "cpu" or dist.get_backend(group) != "gloo") else torch.device("cpu")
    pad = torch.zeros((m_max,) + tail, device=cdev, dtype=local.dtype)
    pad[: local.shape[0]] = local
    gathered = torch.empty((world * m_max,) + tail, device=cdev, dtype=local.dtype)
    dist.all_gather_into_tensor(gathered, pad, group=group)
    gathered = gathered.to(local.device)
    for r, ids in enumerate(assignment):
        if ids:
            out[_index(ids, local.device)] = gathered[r * m_max : r * m_max + len(ids)]
    return out


def _index(ids, device) -> torch.Tensor:
    """Member indices on the device without a host wait (pinned, non-blocking: a pageable copy would
    block the host until the stream drains)."""
    t = torch.as_tensor(list(ids), dtype=torch.long)
    if device.type == "cuda":
        return t.pin_memory().to(device, non_blocking=True)
    return t.to(device)


def member_shard(n_members: int, costs: list[float], group=None, keys: list | None = None, unit: int = 1):
    """This rank's members and a gather function for the classifier's member loop.

    Returns ``(mine, gather)``: ``mine`` lists the member indices this rank runs;
    ``gather(outs, device, Q, n_out)`` takes ``{member: logits [Q, n_out]}`` of this
    rank and returns every member's logits in member order, on every rank (one
    all-gather when ``torch.distributed`` runs more than one rank, else a reorder).
    """
    import torch.distributed as dist

    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    world = dist.get_world_size(group) if multi else 1
    rank = dist.get_rank(group) if multi else 0
    assignment = lpt_assign(costs, world, keys, unit) if multi else [list(range(n_members))]
    mine = assignment[rank]

    def gather(outs: dict[int, torch.Tensor], device, Q: int, n_out: int) -> list[torch.Tensor]:
        if not multi:
            return [outs[i] for i in range(n_members)]
        local = (torch.stack([outs[i] for i in mine]) if mine
                 else torch.zeros((0, Q, n_out), device=device, dtype=torch.float32))
        full = allgather_logits(local, assignment, rank, group)
        return [full[i] for i in range(n_members)]

    return mine, gather
