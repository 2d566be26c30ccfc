"""bench.py's launcher (`--gpus N` runs N ranks) and its per-rank stream
shares, on CPU.  The reference scales by N Shared-subscription consumers
(attendance_processor.py:30-34); bench.py --gpus N must therefore be N ranks
whether or not an external torch.distributed.run started it."""
import importlib.util
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_self_launch_when_no_world_size():
    b = _bench()
    argv = ["--gpus", "4", "--steps", "3", "--warmup", "1"]
    cmd = b.launch_plan(b.parse(argv), argv, {})
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd
    port = [c for c in cmd if c.startswith("--master-port=")]
    assert len(port) == 1 and 0 < int(port[0].split("=")[1]) < 65536
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == argv  # the ranks get the same arguments


@pytest.mark.parametrize("argv", [[], ["--gpus", "1"]])
def test_one_rank_in_process(argv):
    b = _bench()
    assert b.launch_plan(b.parse(argv), argv, {}) is None


def test_under_external_launcher():
    b = _bench()
    argv = ["--gpus", "8"]
    assert b.launch_plan(b.parse(argv), argv, {"WORLD_SIZE": "8"}) is None
    assert b.launch_plan(b.parse([]), [], {"WORLD_SIZE": "8"}) is None  # --gpus omitted
    with pytest.raises(SystemExit):
        b.launch_plan(b.parse(["--gpus", "2"]), ["--gpus", "2"], {"WORLD_SIZE": "8"})


def test_parent_does_not_touch_the_gpu():
    """The self-launching parent runs the ranks as a child and exits with its
    status without importing torch (so no HIP call happens in the parent, and
    no exec replaces a process that initialised the GPU).  subprocess.run is
    replaced by a stand-in child that exits 3: the parent must pass that
    status on, having started exactly one launcher."""
    code = ("import sys; sys.argv = ['bench.py', '--gpus', '2', '--config', 'nope']\n"
            "import bench, subprocess\n"
            "calls = []\n"
            "def fake(cmd, *a, **k):\n"
            "    calls.append(cmd)\n"
            "    assert 'torch' not in sys.modules, 'parent imported torch'\n"
            "    class R: returncode = 3\n"
            "    return R()\n"
            "subprocess.run = fake\n"
            "try:\n"
            "    bench.main()\n"
            "except SystemExit as e:\n"
            "    assert e.code == 3, e.code\n"
            "    assert len(calls) == 1 and '--nproc-per-node=2' in calls[0]\n"
            "    print('OK')\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "OK" in r.stdout, r.stderr


def test_mass_shares_c3():
    """C3 at N = 8 (mass mode): the ranks' batches add up to 8 x 16M swipes
    per step and follow the Zipf mass of the keys each owns."""
    b = _bench()
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge
    ge.load_package()
    from rtsas_amd import synthetic
    from rtsas_amd.distributed import KeyMap
    w = synthetic.WORKLOADS["c3"]
    names = synthetic.key_names(w)
    probs = synthetic.key_probs(w)
    world = 8
    km = KeyMap(names, world)
    mass = [float(probs[km.keys_of(r)].sum()) for r in range(world)]
    assert abs(sum(mass) - 1.0) < 1e-9
    n = [b.rank_swipes(w.step_swipes, m, world, "mass") for m in mass]
    assert abs(sum(n) - world * w.step_swipes) <= world
    assert max(n) / (sum(n) / world) < 1.2  # hashing the 100k day keys spreads the hot lectures
    assert [b.rank_swipes(w.step_swipes, m, world, "equal") for m in mass] == [w.step_swipes] * world
    assert b.rank_swipes(w.step_swipes, 1.0, 1, "mass") == w.step_swipes  # N = 1: the config's step
    assert np.isclose(sum(m for m in mass), 1.0)
