"""Ensemble sharding: LPT assignment and the logit all-gather (gloo, world_size 2, CPU)."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from multimodalpfn_amd.parallel import allgather_logits, lpt_assign, member_cost


def test_lpt_balances_ragged_members():
    costs = [member_cost(t, 2298, 1838) for t in (36, 36, 26, 26, 11, 11, 51)]
    a = lpt_assign(costs, 3)
    assert sorted(i for r in a for i in r) == list(range(7))
    loads = [sum(costs[i] for i in r) for r in a]
    assert max(loads) / min(loads) < 1.6


def test_lpt_more_ranks_than_members():
    a = lpt_assign([1.0, 2.0], 4)
    assert sorted(len(r) for r in a) == [0, 0, 1, 1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_members, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    assignment = lpt_assign([1.0 + (i % 3) for i in range(n_members)], world)
    mine = assignment[rank]
    local = torch.stack([torch.full((5, 10), float(m)) for m in mine]) if mine else torch.zeros(0, 5, 10)
    out = allgather_logits(local, assignment, rank)
    ok = all(torch.all(out[m] == float(m)).item() for m in range(n_members))
    q.put((rank, ok))
    dist.destroy_process_group()


@pytest.mark.parametrize("n_members", [4, 5, 1])
def test_allgather_logits_gloo_world2(n_members):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_members, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res


def test_allgather_single_process_reorders():
    a = [[2, 0, 1]]
    local = torch.stack([torch.full((2, 3), float(m)) for m in a[0]])
    out = allgather_logits(local, a, 0)
    assert [out[i, 0, 0].item() for i in range(3)] == [0.0, 1.0, 2.0]


def _shard_worker(rank, world, port, n_members, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from multimodalpfn_amd.parallel import member_shard

    mine, gather = member_shard(n_members, [float(1 + i % 3) for i in range(n_members)])
    outs = {i: torch.full((4, 10), float(i)) for i in mine}
    full = gather(outs, torch.device("cpu"), 4, 10)
    ok = len(full) == n_members and all(torch.all(full[i] == float(i)).item() for i in range(n_members))
    q.put((rank, ok, mine))
    dist.destroy_process_group()


@pytest.mark.parametrize("n_members", [5, 1])
def test_member_shard_gloo_world2(n_members):
    """The classifier's member loop split over 2 ranks returns every member on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, n_members, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    assert sorted(i for _, _, mine in res for i in mine) == list(range(n_members))
