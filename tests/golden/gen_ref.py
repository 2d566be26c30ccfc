"""numpy restatement of the device synthetic generator (ske_gen_swipes /
ske_gen_members; sketch_common.h mix/gen_member/gen_is_member and
sketch_kernels.hip gen_swipe_id).  Test infrastructure: used to check the
device generator's bytes / offsets / slots exactly."""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15


def _fin(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def mix(seed: int, i, j: int):
    i = np.asarray(i, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = np.uint64(seed) + np.uint64(GOLDEN) * (i * np.uint64(256) + np.uint64(j + 1))
    return _fin(x)


class Gen:
    def __init__(self, p):
        self.seed = int(p.seed)
        self.lo = int(p.id_lo)
        self.R = int(p.id_hi - p.id_lo)
        self.N = int(p.n_members)
        self.mul = int(p.perm_mul) % self.R
        self.add = int(p.perm_add) % self.R
        self.inv = int(p.perm_mul_inv) % self.R
        self.inv_thr = int(p.invalid_thresh)
        self.near_thr = int(p.near_thresh)
        self.n_keys = int(p.n_keys)
        self.slot_base = int(p.slot_base)
        self.width = len(str(int(p.id_hi) - 1))

    def member(self, i):
        i = np.asarray(i, dtype=np.uint64)
        return np.uint64(self.lo) + (np.uint64(self.mul) * i + np.uint64(self.add)) % np.uint64(self.R)

    def is_member(self, x):
        x = np.asarray(x, dtype=np.uint64)
        inr = (x >= self.lo) & (x < self.lo + self.R)
        xs = np.where(inr, x, np.uint64(self.lo))
        r = (xs - np.uint64(self.lo) + np.uint64(self.R) - np.uint64(self.add % self.R)) % np.uint64(self.R)
        return inr & ((r * np.uint64(self.inv)) % np.uint64(self.R) < np.uint64(self.N))

    def swipe_ids(self, start: int, n: int) -> np.ndarray:
        i = np.arange(start, start + n, dtype=np.uint64)
        u0 = mix(self.seed, i, 0)
        invalid = (u0 >> np.uint64(32)) < np.uint64(self.inv_thr)
        out = self.member(mix(self.seed, i, 1) % np.uint64(self.N))
        todo = invalid.copy()
        if self.near_thr:
            near = todo & ((mix(self.seed, i, 1) >> np.uint64(32)) < np.uint64(self.near_thr))
            base = self.member(mix(self.seed, i, 2) % np.uint64(self.N)).astype(np.int64)
            u = mix(self.seed, i, 3)
            kind0 = (u & np.uint64(1)) == 0
            plus = ((u >> np.uint64(1)) & np.uint64(1)) == 1
            cand_pm = np.where(plus, base + 1, base - 1)
            pos = ((u >> np.uint64(8)) % np.uint64(self.width)).astype(np.int64)
            p10 = (10 ** pos).astype(np.int64)
            dold = (base // p10) % 10
            dnew = (dold + 1 + ((u >> np.uint64(16)) % np.uint64(9)).astype(np.int64)) % 10
            cand_dg = base + (dnew - dold) * p10
            cand = np.where(kind0, cand_pm, cand_dg)
            ok = near & (cand >= self.lo) & (cand < self.lo + self.R)
            ok &= ~self.is_member(np.where(ok, cand, self.lo).astype(np.uint64))
            out = np.where(ok, cand.astype(np.uint64), out)
            todo &= ~ok
        x = np.zeros(n, np.uint64)
        done = ~todo
        for t in range(64):
            if done.all():
                break
            cand = np.uint64(self.lo) + mix(self.seed, i, 4 + t) % np.uint64(self.R)
            take = ~done
            x = np.where(take, cand, x)
            done |= take & ~self.is_member(cand)
        out = np.where(todo, x, out)
        return out.astype(np.uint64)

    def swipe_slots(self, start: int, n: int, cdf: np.ndarray | None) -> np.ndarray:
        i = np.arange(start, start + n, dtype=np.uint64)
        u = mix(self.seed, i, 200)
        if cdf is None:
            s = (u % np.uint64(self.n_keys)).astype(np.int64)
        else:
            u32 = (u >> np.uint64(32)).astype(np.uint32)
            s = np.searchsorted(cdf[:-1], u32, side="right")
        return (s + self.slot_base).astype(np.uint32)

    def encode(self, ids: np.ndarray):
        w = self.width
        n = ids.shape[0]
        digits = np.zeros((n, w), np.uint8)
        x = ids.astype(np.uint64).copy()
        for d in range(w - 1, -1, -1):
            digits[:, d] = (x % np.uint64(10)).astype(np.uint8) + 48
            x //= np.uint64(10)
        offs = (np.arange(n + 1, dtype=np.uint64) * w).astype(np.uint32)
        return digits.reshape(-1), offs
