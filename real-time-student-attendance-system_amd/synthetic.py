"""Synthetic swipe streams for configs C1..C5 (BASELINE.json).

There is no dataset: the reference's generator draws 1000 valid ids with
``faker.unique.random_int(10000, 99999)`` (data_generator.py:53-54), 50
invalid ids from [100000, 999999] (:80-81) and mixes ~7 % invalid swipes
(:140, :162).  The device generator (``ske_gen_swipes``) scales that shape up
with a counter-based definition so any slice of a 1B-event stream can be made
on any GPU independently:

  member(i) = lo + (mul*i + add) mod R,  i < N        (R = hi - lo)
  swipe i   : invalid if hi32(mix(seed,i,0)) < P_inv*2^32
              valid   -> member(mix(seed,i,1) mod N)
              invalid -> near-collision of a member (C4) or a uniform
                         non-member (rejection over mix(seed,i,4+t))
              key     -> slot_base + (mix(seed,i,200) mod n_keys | CDF)
  ids are decimal ASCII of fixed width (redis-py's int encoding).

``tests/golden/gen_ref.py`` restates it in numpy for the parity tests.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field

import numpy as np

from ._lib import GenParams

SEED = 20251003


@dataclass
class Workload:
    name: str
    bf_error: float
    bf_capacity: int
    id_lo: int
    id_hi: int
    n_members: int
    n_swipes: int
    n_keys: int
    invalid_frac: float
    near_frac: float = 0.0           # share of invalids that are near-collisions
    zipf_lectures: int = 0           # >0: keys = lectures x days, lecture ~ Zipf(s)
    zipf_days: int = 0
    zipf_s: float = 1.1
    gpus: int = 1
    step_swipes: int = 1_000_000     # swipes per benchmark step (one K1 launch)
    seed: int = SEED
    notes: str = ""
    extra: dict = field(default_factory=dict)


WORKLOADS = {
    # C1: README default on CPU (bf:students 1e5 / 0.01, 10k swipes, one key)
    "c1": Workload("c1-readme-default", 0.01, 100_000, 10_000, 100_000, 1_000, 10_000, 1, 0.071,
                   notes="valid ids 5 digits as data_generator.py:53; invalids drawn from the "
                         "same width (the reference's 6-digit invalids are a host-side case)"),
    # C2: 1M swipes, 100k students, 50 lecture-day keys, 10% invalid, 1 GPU
    "c2": Workload("c2-1M-100k-50keys", 0.01, 100_000, 1_000_000, 10_000_000, 100_000,
                   1_000_000, 50, 0.10),
    # C3: 1B swipes, 10M students (0.001), 100k lecture-day keys (Zipf lectures)
    "c3": Workload("c3-1B-10M-100kkeys", 0.001, 10_000_000, 10_000_000, 100_000_000, 10_000_000,
                   1_000_000_000, 100_000, 0.10, zipf_lectures=1000, zipf_days=100, gpus=8,
                   step_swipes=16_000_000),
    # C4: adversarial, 50% invalid of which half near-collisions
    "c4": Workload("c4-adversarial", 0.01, 100_000, 1_000_000, 10_000_000, 100_000, 1_000_000, 50,
                   0.50, near_frac=0.5),
    # C5: campus-year rollup 365 days x 5000 lectures
    "c5": Workload("c5-campus-year", 0.001, 10_000_000, 10_000_000, 100_000_000, 10_000_000,
                   1_000_000_000, 365 * 5000, 0.10, zipf_lectures=5000, zipf_days=365, gpus=8,
                   step_swipes=16_000_000),
}


def shard(w: Workload, world: int) -> Workload:
    """This rank's share of a multi-GPU workload: the key space split over
    `world` owners (keys are routed to their owner at ingest), swipes per step
    unchanged (weak scaling).  Zipf lectures are split the same way."""
    if world <= 1:
        return w
    d = dict(w.__dict__)
    if w.zipf_lectures:
        d["zipf_lectures"] = max(1, w.zipf_lectures // world)
        d["n_keys"] = d["zipf_lectures"] * w.zipf_days
    else:
        d["n_keys"] = max(1, -(-w.n_keys // world))
    return Workload(**d)


def _coprime_mul(R: int, seed: int) -> int:
    m = (0x9E3779B97F4A7C15 ^ seed) % R
    m |= 1
    while math.gcd(m, R) != 1:
        m += 2
    return m % R


def key_probs(w: Workload) -> np.ndarray | None:
    """Probability of every key = lecture*days + day (None: uniform)."""
    if not w.zipf_lectures:
        return None
    L, D = w.zipf_lectures, w.zipf_days
    assert L * D == w.n_keys
    p_lect = 1.0 / np.arange(1, L + 1, dtype=np.float64) ** w.zipf_s
    p_lect /= p_lect.sum()
    return np.repeat(p_lect / D, D)


def cdf_from_probs(p: np.ndarray) -> np.ndarray:
    """u32 CDF (scaled by 2^32) of a key distribution (renormalised)."""
    cdf = np.cumsum(p / p.sum()) * 2.0 ** 32
    return np.minimum(np.round(cdf), 2 ** 32 - 1).astype(np.uint32)


def key_cdf(w: Workload) -> np.ndarray | None:
    """u32 CDF (scaled by 2^32) over keys = lecture*days + day."""
    p = key_probs(w)
    return None if p is None else cdf_from_probs(p)


def key_names(w: Workload) -> list[str]:
    """key_name() of every key of the workload (the job's key universe)."""
    import datetime as _dt
    days = w.zipf_days or max(1, w.n_keys)
    dates = []
    for day in range(days):
        y, d = divmod(day, 365)
        dt = _dt.date(2025, 1, 1) + _dt.timedelta(days=int(d))
        dates.append(f"{dt.year + y:04d}-{dt.month:02d}-{dt.day:02d}")
    if not w.zipf_lectures:
        return [f"hll:unique:LECT{k:05d}:{dates[0]}" for k in range(w.n_keys)]
    return [f"hll:unique:LECT{k // days:05d}:{dates[k % days]}" for k in range(w.n_keys)]


def gen_params(w: Workload, seed: int | None = None, slot_base: int = 0,
               key_cdf_dev: int | None = None) -> GenParams:
    R = w.id_hi - w.id_lo
    s = w.seed if seed is None else seed
    mul = _coprime_mul(R, s)
    p = GenParams()
    p.seed = s & (2 ** 64 - 1)
    p.id_lo, p.id_hi = w.id_lo, w.id_hi
    p.n_members = w.n_members
    p.perm_mul = mul
    p.perm_add = (s * 0x2545F4914F6CDD1D) % R
    p.perm_mul_inv = pow(mul, -1, R)
    p.invalid_thresh = min(int(round(w.invalid_frac * 2 ** 32)), 2 ** 32 - 1)
    p.near_thresh = min(int(round(w.near_frac * 2 ** 32)), 2 ** 32 - 1)
    p.n_keys = w.n_keys
    p.slot_base = slot_base
    p.key_cdf = key_cdf_dev
    return p


def id_width(w: Workload) -> int:
    return len(str(w.id_hi - 1))


def key_name(w: Workload, k: int) -> str:
    """README key form hll:unique:<lecture_id>:<YYYY-MM-DD> for key index k."""
    days = w.zipf_days or max(1, w.n_keys)
    lecture, day = (k // days, k % days) if w.zipf_lectures else (k, 0)
    y, d = divmod(day, 365)
    import datetime as _dt
    date = _dt.date(2025, 1, 1) + _dt.timedelta(days=int(d))
    return f"hll:unique:LECT{lecture:05d}:{date.year + y:04d}-{date.month:02d}-{date.day:02d}"
