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


# ---- world 8: 32 ragged members (config D's member count), real per-member logits from the oracle
D_MEMBERS, D_WORLD, D_S, D_N = 32, 8, 40, 30
D_WIDTHS = (5, 9, 13)  # ragged preprocessed widths -> three member geometries


def _d_members():
    """Per-member inputs of a small image+text ensemble: feature-shuffled / column-subset tables of
    three widths, permuted labels (the reference's member loop, inference.py:294-349)."""
    import numpy as np

    from synth import synth_image, synth_labels, synth_table

    x = synth_table(D_S, max(D_WIDTHS), 3, n_cat=4)
    y = synth_labels(D_S, 3, 3)[:D_N]
    rng = np.random.default_rng(7)
    out = []
    for m in range(D_MEMBERS):
        F = D_WIDTHS[m % len(D_WIDTHS)]
        cols = rng.permutation(max(D_WIDTHS))[:F]
        perm = rng.permutation(3)
        out.append((np.ascontiguousarray(x[:, cols]), perm[y.astype(np.int64)].astype(np.float32), perm))
    return out, synth_image(D_S, 2, 3)


def _d_logits(ids):
    import torch

    from helpers import oracle_spec, torch_sd
    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec
    from oracle.forward import oracle_forward, oracle_mixer
    from synth import synth_state_dict

    torch.set_num_threads(1)
    cfg = ModelConfig(nlayers=1, mgm_heads=4, cap_heads=4)
    spec = oracle_spec(cfg)
    w = torch_sd(synth_state_dict(state_dict_spec(cfg), 3))
    members, image = _d_members()
    tok = oracle_mixer(spec, w, torch.from_numpy(image))  # shared by every member (computed once per rank)
    out = {}
    for i in ids:
        x, y, _ = members[i]
        out[i] = oracle_forward(spec, w, torch.from_numpy(x), None, torch.from_numpy(y), mixer_tokens=tok)
    return out


def _d_proba(logits_by_member, n_cls=3, temperature=0.9):
    """classifier.py:541-561: logits[:, :n_cls] / T, undo the class permutation, softmax, member mean."""
    import torch

    members, _ = _d_members()
    probs = []
    for i in range(D_MEMBERS):
        lg = logits_by_member[i][:, :n_cls] / temperature
        probs.append(torch.softmax(lg[:, torch.as_tensor(members[i][2])], dim=-1))
    p = torch.stack(probs).mean(0)
    return p / p.sum(-1, keepdim=True)


def _d_costs_keys():
    from multimodalpfn_amd.parallel import member_cost

    members, _ = _d_members()
    costs = [member_cost((x.shape[1] + 1) // 2 + 4 + 1, D_S, D_N) for x, _, _ in members]
    keys = [(x.shape[1], D_N) for x, _, _ in members]
    return costs, keys


def _d_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=__import__("datetime").timedelta(seconds=120))
    except Exception as e:  # noqa: BLE001 - reported to the parent, which retries on a fresh port
        q.put((rank, None, None, None, f"init: {type(e).__name__}: {e}"))
        return
    try:
        from multimodalpfn_amd.parallel import member_shard

        costs, keys = _d_costs_keys()
        mine, gather = member_shard(D_MEMBERS, costs, keys=keys, unit=2)
        outs = _d_logits(mine)
        full = gather(outs, torch.device("cpu"), D_S - D_N, 10)
        q.put((rank, list(mine), torch.stack(full), _d_proba(full), None))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        q.put((rank, None, None, None, f"{type(e).__name__}: {e}"))
    finally:
        dist.destroy_process_group()


def _run_world8():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_d_worker, args=(r, D_WORLD, port, q)) for r in range(D_WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    return res


def test_member_shard_world8_ragged_members_bitwise():
    """32 ragged members over 8 gloo ranks: the grouped LPT split is disjoint and complete, keeps
    equal-geometry pairs on one rank, and every rank's gathered logits and ensemble probabilities
    equal the single-process member loop bitwise (member order restored by the all-gather)."""
    costs, keys = _d_costs_keys()
    ref_logits = _d_logits(range(D_MEMBERS))
    ref_proba = _d_proba(ref_logits)
    res = _run_world8()
    if any(err for *_, err in res):  # a rendezvous on a port taken between probe and bind: one retry
        res = _run_world8()
    shares = {}
    for rank, mine, logits, proba, err in res:
        assert err is None, [(r[0], r[-1]) for r in res]
        shares[rank] = mine
        assert torch.equal(logits, torch.stack([ref_logits[i] for i in range(D_MEMBERS)])), rank
        assert torch.equal(proba, ref_proba), rank
    allm = sorted(i for m in shares.values() for i in m)
    assert allm == list(range(D_MEMBERS))
    assert max(len(m) for m in shares.values()) <= 5
    by_key = {}
    for i, k in enumerate(keys):
        by_key.setdefault(k, []).append(i)
    units = [ids[j : j + 2] for ids in by_key.values() for j in range(0, len(ids), 2)]
    assert sum(len(u) == 2 for u in units) == 15  # widths 11 / 11 / 10 members -> 15 pairs + 2 singles
    for u in units:  # equal-geometry pairs stay on one rank (batched there into one forward)
        assert sum(set(u) <= set(m) for m in shares.values()) == 1, (u, shares)


def test_lpt_grouped_units_and_cost_model():
    from multimodalpfn_amd.parallel import lpt_assign, member_cost

    # the flop model counts projections and MLP, so a wide member is not T x a narrow one's attention
    c36, c11 = member_cost(36, 2298, 1838), member_cost(11, 2298, 1838)
    assert 36 / 11 * 0.99 < c36 / c11 < 36 / 11 * 1.01  # linear in T at fixed S, N (T^2 term small)
    keys = ["a"] * 5 + ["b"] * 3
    a = lpt_assign([1.0] * 8, 3, keys, unit=2)
    assert sorted(i for r in a for i in r) == list(range(8))
    units = [[0, 1], [2, 3], [4], [5, 6], [7]]
    for r in a:  # every rank holds whole units
        assert all(set(u) <= set(r) or not set(u) & set(r) for u in units), a
