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
    for prec, kw in (("f32", {"inference_precision": torch.float32}), ("bf16", {})):
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
        for prec in ("f32", "bf16"):
            np.testing.assert_array_equal(got[prec], single[prec], err_msg=f"rank {rank} {prec}")
    # every predict split its members over the two ranks (disjoint, complete, both non-empty)
    by_rank = {rank: got["shares"] for rank, got, _ in res}
    assert len(by_rank[0]) == len(by_rank[1]) >= 2
    for (n0, m0), (n1, m1) in zip(by_rank[0], by_rank[1]):
        assert n0 == n1 and m0 and m1 and sorted(m0 + m1) == list(range(n0)), (m0, m1)
