"""One rank of test_exchange_gpu.py (run under torch.distributed.run, gloo,
every rank on this box's GPU): a slice of a C2-shaped stream over GLOBAL key
indices of a named key universe (distributed.KeyMap), routed to the key
owners by distributed.SwipeExchange, K1 on the device per rank, then queried
by name through distributed.ShardedSketch over a client that KeyMap.bind
named.  Saves the answers (input order), this rank's registers, the
cluster-wide query answers and its stream for the parent's oracle check."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NK, N = 37, 400_000


def workload():
    from rtsas_amd import synthetic
    w = synthetic.WORKLOADS["c2"]
    return synthetic.Workload(**{**w.__dict__, "n_keys": NK})


def names():
    from rtsas_amd import synthetic
    w = workload()
    return [synthetic.key_name(w, k) for k in range(NK)]


def groups(nm):
    return [nm[i::5] for i in range(5)] + [nm, []]


def main(out_dir, mode="exact"):
    import torch
    import torch.distributed as dist
    import __graft_entry__ as ge
    ge.load_package()
    pkg = ge.load_package()
    from rtsas_amd.distributed import KeyMap, ShardedSketch, SwipeExchange, engine_k1
    from rtsas_amd.engine import SketchEngine
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    # WORKER_BACKEND=nccl: RCCL with every rank on this box's one GPU (the
    # device collectives of a multi-GPU node, rehearsed); default gloo
    if os.environ.get("WORKER_BACKEND", "gloo") == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo")
    w = workload()
    eng = SketchEngine(0)
    eng.reserve(0, w.bf_error, w.bf_capacity)
    p = eng.gen_params(w)
    eng.preload(0, p, w.n_members)
    nm = names()
    km = KeyMap(nm, world)
    client = pkg.SketchClient(context=eng.ctx)
    km.bind(client, rank)
    nlocal = km.slots_end(rank)
    sinks = [km.slots_end(r) for r in range(world)]  # one spare slot past the universe per rank
    eng.hll_reserve(nlocal + 1)
    n = N - 1000 * rank                      # uneven slices
    b = eng.swipe_batch(p, rank * N, n)
    buf, offs, slot = b.to_host()
    width = int(offs[1] - offs[0])
    assert (np.diff(offs.astype(np.int64)) == width).all()
    ids = torch.from_numpy(buf[:n * width].reshape(n, width).copy()).cuda()
    slots = torch.from_numpy(slot.astype(np.int64)).cuda()
    k1 = engine_k1(eng)
    # async*: the pipelined form (routing of batch j+1 beside K1 of batch j,
    # two parities of rows) unless "serial" (one stream)
    ex = SwipeExchange(rank, world, k1, km, engine=eng, sink_slots=sinks,
                       slack=-0.6 if mode == "async_overflow" else world - 1.0, overlap="serial" not in mode)
    force = os.environ.get("WORKER_FORCE_COLLECTIVES") == "1"  # world 1: collectives still called
    if force:
        ex.solo = False
    if mode == "exact":
        ans = ex.swipes(ids, slots)
    else:
        # async_many: 5 batches (each parity of rows reused), of uneven sizes
        nb = 5 if "many" in mode else 2
        h = -(-N // nb)  # n_max: no rank's slice of a batch is longer
        parts = [ex.swipes_async(ids[j * h:(j + 1) * h], slots[j * h:(j + 1) * h], n_max=h) for j in range(nb)]
        redone = ex.settle()
        assert (redone == nb) == (mode == "async_overflow"), (mode, redone, ex.stats)
        ans = torch.cat(parts)
    torch.cuda.synchronize()
    eng.sync()
    sk = ShardedSketch(client, rank, world)
    if force:
        sk.solo = False
    union = sk.pfcount_union(nm)
    each = sk.pfcount_each(nm)
    roll = sk.rollup(groups(nm))
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), ans=ans.cpu().numpy(), regs=eng.registers_all(nlocal),
             buf=buf, offs=offs, slot=slot, union=np.array([union], np.uint64), each=each, roll=roll,
             mine=km.keys_of(rank))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "exact")
