"""Key-sharded runs on the device: W ranks (gloo transport,
all on this box's GPU), each with a replica of the Bloom preload and the HLL
keys it owns, process only the swipes routed to them; the cross-shard union
PFCOUNT, per-lecture rollup and per-key PFCOUNT equal the one-shard answers
computed by the oracle.  RCCL replaces gloo on a multi-GPU node; the device
path (K1, K3 into torch tensors, K2) is the same."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world,backend", [(2, "gloo"), (4, "gloo"), (1, "nccl")])
def test_sharded_queries_equal_one_shard(orc, tmp_path, world, backend):
    """backend nccl: RCCL, one rank on the box's one GPU with the collectives
    forced on (reduce_scatter_tensor / all_reduce / all_gather on their RCCL
    code path; a second RCCL rank on the same GPU is refused: "Duplicate GPU")."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from sharded_worker import workload
    out = str(tmp_path / "res.npz")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", WORKER_BACKEND=backend,
               WORKER_FORCE_COLLECTIVES="1" if backend == "nccl" else "0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        f"--nproc-per-node={world}", "--master-addr", "127.0.0.1",
                        "--master-port", str(29600 + world + (10 if backend == "nccl" else 0)),
                        os.path.join(ROOT, "tests", "sharded_worker.py"),
                        out], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = np.load(out)
    members, ids, keys, groups = workload()
    chain = orc.Chain(20000, 0.01)
    for m in members:
        chain.add(str(int(m)).encode())
    hlls = {}
    for i, k in zip(ids, keys):
        b = str(int(i)).encode()
        if chain.exists(b):
            hlls.setdefault(k, orc.HLL()).add(b)
    all_keys = sorted(set(keys))
    u = orc.HLL()
    for h in hlls.values():
        u.merge(h)
    assert int(res["union"][0]) == u.count()
    want_roll = []
    for g in groups:
        gu = orc.HLL()
        for k in g:
            if k in hlls:
                gu.merge(hlls[k])
        want_roll.append(gu.count())
    assert res["rollup"].tolist() == want_roll
    assert res["each"].tolist() == [hlls[k].count() if k in hlls else 0 for k in all_keys]
