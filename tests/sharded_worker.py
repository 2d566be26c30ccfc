"""Worker of tests/test_sharded_gpu.py: one rank of a key-sharded run on the
device.  Launched by torch.distributed.run with the gloo
backend so that several ranks can share one GPU in the test; the device side
(BF.MADD replica, K1 over the owned swipes, K3 group merges into torch
tensors, K2 counts) is the real libsketch path, only the collective transport
differs from RCCL.

usage: python -m torch.distributed.run --nproc-per-node W tests/sharded_worker.py OUT.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def workload():
    rng = np.random.default_rng(31)
    members = rng.choice(np.arange(10**6, 10**7), 20000, replace=False)
    ids = np.where(rng.random(60000) < 0.9, rng.choice(members, 60000),
                   rng.integers(10**6, 10**7, 60000))
    lectures, days = 12, 9
    keys = [f"hll:unique:L{int(l):02d}:2025-03-{int(d) + 1:02d}"
            for l, d in zip(rng.integers(0, lectures, 60000), rng.integers(0, days, 60000))]
    groups = [[f"hll:unique:L{l:02d}:2025-03-{d + 1:02d}" for d in range(days)] for l in range(lectures)]
    return members, ids, keys, groups


def main():
    import torch
    import torch.distributed as dist
    out = sys.argv[1]
    pkg = ge.load_package()
    from rtsas_amd.distributed import ShardedSketch, route
    torch.cuda.set_device(0)
    # WORKER_BACKEND=nccl: RCCL with every rank on this box's one GPU (the
    # device collectives of a multi-GPU node, rehearsed); default gloo
    if os.environ.get("WORKER_BACKEND", "gloo") == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    members, ids, keys, groups = workload()
    client = pkg.SketchClient(decode_responses=True, device=0)
    client.execute_command("BF.RESERVE", "bf:students", 0.01, 20000)
    client.bf_madd_packed("bf:students", *pkg.pack_ints(members))  # replicated preload
    mine = np.nonzero(route(keys, world) == rank)[0]
    buf, offs = pkg.pack_ints(ids[mine])
    client.swipes("bf:students", [keys[i] for i in mine], packed=(buf, offs))
    sk = ShardedSketch(client, rank, world)
    if os.environ.get("WORKER_FORCE_COLLECTIVES") == "1":
        sk.solo = False  # world 1: the collectives are still called
    all_keys = sorted(set(keys))
    union = sk.pfcount_union(all_keys)
    roll = sk.rollup(groups)
    each = sk.pfcount_each(all_keys)
    if rank == 0:
        np.savez(out, union=np.array([union], np.uint64), rollup=roll, each=each)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
