"""Pass A's group layout (option "rec_groups"; sketch_part.hip k_part_a3<11,
1024, true> -> k_part_b<2, 4, true, true>): a slice unit's probe records of 8
consecutive tiles are written adjacently in a (group, unit) region so pass B
reads them as one span; a run that does not fit its region goes to the tile's
overflow row (bit 31 of its run word).  Same answers and registers as the
per-tile layout and the oracle (oracle/sketch_oracle.c, the restatement of
RedisBloom SBChain_Check + Redis hllAdd that attendance_processor.py:109-113 /
:127-129 reach), including:

- ragged batches whose last group of 8 tiles is partial and whose last tile
  is partial, over several sub-batches;
- every run of some units overflowing (one id repeated: its 11 probes put
  thousands of records per group into the same few units) next to units
  that fit, and a batch of one repeated id only.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _c3(engine, n_members, n_keys, invalid=0.5):
    from rtsas_amd import synthetic
    w = synthetic.WORKLOADS["c3"]
    w = synthetic.Workload(**{**w.__dict__, "n_members": n_members, "n_keys": n_keys,
                              "zipf_lectures": 0, "zipf_days": 0, "invalid_frac": invalid})
    engine.reserve(0, w.bf_error, w.bf_capacity)   # the 19.8 MB C3 geometry: 152 slice pairs
    p = engine.gen_params(w, seed=5151)
    engine.preload(0, p, w.n_members)
    engine.hll_reserve(w.n_keys)
    assert engine.variant(0) == 3
    return w, p


def _oracle_chain(engine, orc, w, p):
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    mb = engine.members_batch(p, 0, w.n_members).to_host()
    chain.madd_packed(mb[0], mb[1])
    return chain


def _with_hot(engine, b, frac, rng):
    """b with a fraction `frac` of its swipes replaced by its first id (one
    key for them all)"""
    from rtsas_amd.engine import DeviceBatch
    buf, offs, slot = b.to_host()
    assert np.all(np.diff(offs.astype(np.int64)) == 8)
    ids = buf[:offs[-1]].reshape(-1, 8).copy()
    hot = rng.random(b.n) < frac
    ids[hot] = ids[0]
    slot = slot.astype(np.uint32).copy()
    slot[hot] = 3
    buf2 = np.concatenate([ids.reshape(-1), np.zeros(16, np.uint8)])
    return DeviceBatch.from_host(engine.ctx, buf2, offs, slot), (buf2, offs, slot)


@pytest.mark.parametrize("sub", [0, 3 * 8 * 1024 + 5 * 1024])
def test_group_layout_ragged_vs_oracle(engine, orc, sub):
    """Ragged batches in the group layout (partial last group and tile;
    sub-batches of 29 tiles: groups cut by the sub-batch edge) == the oracle,
    answers and registers over the batches in order."""
    from rtsas_amd.engine import DeviceBuffer
    w, p = _c3(engine, 300_000, 97)
    engine.set_option("part_sub", sub)
    engine.set_option("rec_groups", 1)
    chain = _oracle_chain(engine, orc, w, p)
    regs = np.zeros((w.n_keys, 16384), np.uint8)
    start = 0
    for n in [1, 1000, 8 * 1024 * 3 + 777, 700_000 + 333]:
        b = engine.swipe_batch(p, start, n)
        start += n
        out = DeviceBuffer(engine.ctx, b.n)
        engine.swipes(0, b, out)
        buf, offs, slot = b.to_host()
        v, _, _ = orc.process_swipes(chain, regs, slot.astype(np.uint32), buf, offs)
        assert np.array_equal(out.to_host(np.uint8, b.n), v)
    assert np.array_equal(engine.registers_all(w.n_keys), regs)


@pytest.mark.parametrize("frac", [0.05, 0.3, 1.0])
def test_group_layout_overflow_rows_vs_oracle(engine, orc, frac):
    """A fraction of the swipes repeat one id, so the few units its 11 probes
    land in get 8192 * frac extra records per group of 8 tiles against a
    region of ~864 (593 expected): at 5 % their runs overflow in a group's
    later tiles only, at 30 % from the second tile, at 100 % in every tile
    (and every other unit is empty); answers and registers == the oracle."""
    from rtsas_amd.engine import DeviceBuffer
    w, p = _c3(engine, 200_000, 64)
    rng = np.random.default_rng(int(frac * 1000) + 7)
    b0 = engine.swipe_batch(p, 0, 600_000 + 123)
    d, (buf, offs, slot) = _with_hot(engine, b0, frac, rng)
    engine.set_option("rec_groups", 1)
    out = DeviceBuffer(engine.ctx, d.n)
    engine.swipes(0, d, out)
    chain = _oracle_chain(engine, orc, w, p)
    regs = np.zeros((w.n_keys, 16384), np.uint8)
    v, _, _ = orc.process_swipes(chain, regs, slot, buf, offs)
    assert np.array_equal(out.to_host(np.uint8, d.n), v)
    assert np.array_equal(engine.registers_all(w.n_keys), regs)


def test_group_layout_option_values(engine):
    from rtsas_amd._lib import SketchLibError
    for v in (-1, 0, 1):
        engine.set_option("rec_groups", v)
    with pytest.raises(SketchLibError):
        engine.set_option("rec_groups", 2)
    engine.set_option("rec_groups", -1)
