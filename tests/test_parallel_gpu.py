"""Ensemble sharding with the real engine: MMPFNClassifier.predict_proba under torch.distributed
(world size 2, gloo, both ranks on cuda:0 of the one-GPU box) returns, on every rank, exactly the
single-process probabilities -- each rank forwards its LPT share of the members and the all-gather
reassembles them in member order (inference.py:294-349, classifier.py:541-576; parallel.py)."""

from __future__ import annotations

import os
import socket
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from test_api_host import _case, case_data, make_classifier, write_ckpt

pytestmark = pytest.mark.gpu

CASE = "variants"  # 5 members of ragged widths: an uneven LPT split over the 2 ranks


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _probas(ckdir: Path):
    case = _case(CASE)
    d = case_data(case)
    out = {}
    for prec, kw in (("f32", {"inference_precision": torch.float32}), ("auto16", {})):
        (ckdir / prec).mkdir(parents=True, exist_ok=True)
        clf = make_classifier(case, write_ckpt(case, ckdir / prec), **kw)
        clf.fit(d["X_train"], d["image_train"], d["y_train"])
        out[prec] = clf.predict_proba(d["X_test"], d["image_test"])
    return out


def _worker(rank, world, port, ckdir, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import multimodalpfn_amd.parallel as par

        shares, orig = [], par.member_shard

        def recording(n, costs, group=None, **kw):  # the members this rank actually forwards
            mine, gather = orig(n, costs, group, **kw)
            shares.append((n, list(mine)))
            return mine, gather

        par.member_shard = recording
        torch.cuda.set_device(0)
        res = _probas(Path(ckdir) / f"rank{rank}")
        res["shares"] = shares
        q.put((rank, res, None))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        q.put((rank, None, f"{type(e).__name__}: {e}"))
    finally:
        dist.destroy_process_group()


def test_sharded_predict_proba_equals_single_process(tmp_path):
    single = _probas(tmp_path / "single")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, got, err in res:
        assert err is None, (rank, err)
        for prec in ("f32", "auto16"):
            np.testing.assert_array_equal(got[prec], single[prec], err_msg=f"rank {rank} {prec}")
    # every predict split its members over the two ranks (disjoint, complete, both non-empty)
    by_rank = {rank: got["shares"] for rank, got, _ in res}
    assert len(by_rank[0]) == len(by_rank[1]) >= 2
    for (n0, m0), (n1, m1) in zip(by_rank[0], by_rank[1]):
        assert n0 == n1 and m0 and m1 and sorted(m0 + m1) == list(range(n0)), (m0, m1)


def _nccl_world1(port, q):
    """A fresh process: RCCL process group of one rank, then the all-gather's collective branch."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    try:
        dist.init_process_group("nccl", rank=0, world_size=1)
        torch.cuda.set_device(0)
        from multimodalpfn_amd.parallel import allgather_logits

        g = torch.Generator().manual_seed(7)
        local = torch.randn((5, 460, 10), generator=g).cuda()
        assignment = [[3, 0, 4, 1, 2]]  # a non-identity member order: the reorder is exercised too
        coll = allgather_logits(local, assignment, 0, force_collective=True)
        ref = allgather_logits(local, assignment, 0)
        torch.cuda.synchronize()
        q.put((dist.get_backend(), coll.device.type, bool(torch.equal(coll, ref)),
               bool(torch.equal(ref[torch.tensor(assignment[0])], local)), None))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        q.put((None, None, False, False, f"{type(e).__name__}: {e}"))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_rccl_allgather_branch_world1():
    """the device-tensor ``all_gather_into_tensor`` of ``allgather_logits`` runs on RCCL
    (backend ``nccl``) with one rank, forced past the world-size-1 short-circuit, and equals the reorder path
    bitwise (parallel.py; the reference's member mean, classifier.py:555-561, has no collective)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_world1, args=(_free_port(), q))
    p.start()
    backend, dev, equal, reordered, err = q.get(timeout=180)
    p.join(timeout=60)
    assert err is None, err
    assert backend == "nccl" and dev == "cuda"
    assert equal and reordered
