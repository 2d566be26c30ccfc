"""Batched counterpart of the reference's processor and analytics callers.

``AttendanceProcessor`` mirrors attendance_processor.py:26-165 with the
transport (Pulsar) and persistence (Cassandra) removed: messages arrive as an
iterable of JSON payloads, and the per-event loop at :100-137 (decode ->
``BF.EXISTS`` -> valid-gated ``PFADD``) runs as one fused device call per
batch.  The rows it returns are what the reference inserts into Cassandra
(:116-124), including invalid events.

``lecture_rankings`` is attendance_analysis.py:87-97 in the PFCOUNT form the
README describes (README.md:179: "rank by unique daily counts (from HLL)").
"""
from __future__ import annotations

import json
import logging
from datetime import datetime, timezone
from typing import Iterable, Sequence

import numpy as np

from .client import SketchClient
from .config import AttendanceConfig
from .encoding import encode
from .exceptions import ResponseError

logger = logging.getLogger(__name__)


class AttendanceProcessor:
    def __init__(self, client: SketchClient | None = None, config: AttendanceConfig | None = None):
        self.config = config or AttendanceConfig()
        # attendance_processor.py:37-41
        self.redis_client = client or SketchClient(decode_responses=True, device=self.config.device)
        self.acked = 0
        self.nacked = 0

    # attendance_processor.py:74-92
    def _setup_bloom_filter(self):
        cfg = self.config
        try:
            self.redis_client.execute_command("BF.EXISTS", cfg.bloom_filter_key, "test")
            logger.info("Bloom Filter already exists")
            if cfg.faithful_setup:
                return
            if self.redis_client.exists(cfg.bloom_filter_key):
                return
            raise ResponseError("ERR not found")
        except ResponseError:
            try:
                self.redis_client.execute_command("BF.RESERVE", cfg.bloom_filter_key,
                                                  cfg.bloom_filter_error_rate,
                                                  cfg.bloom_filter_capacity)
                logger.info("Created new Bloom Filter")
            except ResponseError as e:
                if "already exists" not in str(e):
                    raise

    def hll_key(self, lecture_id: str, timestamp: datetime) -> str:
        """attendance_processor.py:128 (code form) or README.md:105-106 form."""
        if self.config.hll_key_form == "code":
            return f"{self.config.hll_key_prefix}{lecture_id}"
        if timestamp.tzinfo is not None:
            timestamp = timestamp.astimezone(timezone.utc)
        return f"{self.config.hll_key_prefix}{lecture_id}:{timestamp.date().isoformat()}"

    def process_batch(self, messages: Sequence) -> list[dict]:
        """One batch of the loop at attendance_processor.py:100-137.

        Returns one row per acknowledged message: student_id, lecture_id,
        timestamp, is_valid (what :121-124 inserts).  A message is negatively
        acknowledged (:134-136), produces no row and no PFADD when any step of
        the reference's loop would raise for it, in the loop's order:
          - json.loads / a missing field / datetime.fromisoformat (:103-106);
          - BF.EXISTS: redis-py refuses to encode the id (bool, None, list,
            dict: DataError, :109-113);
          - the Cassandra INSERT (:116-124, before PFADD): the table's
            ``student_id int`` / ``lecture_id text`` columns refuse an id that
            is not an int in the 32-bit range or a lecture_id that is not a
            string (``config.cassandra_row_types``; off: any id redis-py can
            encode is counted).
        The surviving messages go through one fused device call."""
        cfg = self.config
        ids, keys, rows = [], [], []
        for m in messages:
            try:
                data = json.loads(m.decode() if isinstance(m, (bytes, bytearray)) else m) \
                    if not isinstance(m, dict) else m
                student_id = data["student_id"]
                lecture_id = data["lecture_id"]
                ts = datetime.fromisoformat(data["timestamp"])
                sid = encode(student_id)  # redis-py's Encoder: DataError as BF.EXISTS raises it
                if cfg.cassandra_row_types:
                    if type(student_id) is not int or not -2**31 <= student_id < 2**31:
                        raise TypeError(f"Received an argument of invalid type for column "
                                        f"\"student_id\": {student_id!r}")
                    if not isinstance(lecture_id, str):
                        raise TypeError(f"Received an argument of invalid type for column "
                                        f"\"lecture_id\": {lecture_id!r}")
                key = self.hll_key(lecture_id, ts)
            except Exception as e:  # :134-136
                logger.error(f"Error processing message: {e}")
                self.nacked += 1
                continue
            ids.append(sid)
            keys.append(key)
            rows.append({"student_id": student_id, "lecture_id": lecture_id, "timestamp": ts})
        if rows:
            valid = self.redis_client.swipes(cfg.bloom_filter_key, keys, ids)
            for r, v in zip(rows, valid):
                r["is_valid"] = bool(v)
            self.acked += len(rows)
        return rows

    def process_attendance(self, source: Iterable, batch_size: int | None = None):
        """attendance_processor.py:94-141 over an in-memory message source;
        yields the rows of each processed batch."""
        logger.info("Starting attendance processing...")
        self._setup_bloom_filter()
        bs = batch_size or self.config.batch_size
        batch = []
        for m in source:
            batch.append(m)
            if len(batch) >= bs:
                yield self.process_batch(batch)
                batch = []
        if batch:
            yield self.process_batch(batch)

    # attendance_processor.py:149-165 (the Cassandra half is out of scope)
    def get_attendance_stats(self, lecture_id: str, day: str | None = None) -> dict:
        """PFCOUNT of the lecture's key (:151-152).  In the README key form a
        lecture is counted per day: with a day, that day's key; without one
        (the reference's signature), the union of every day key
        prefix+lecture:YYYY-MM-DD in the store -- PFCOUNT k1 k2 ...  The day
        keys come from the key table's stem index (KeySpace.day_keys, kept
        by every key creation / DEL, so a fresh processor on the same store
        answers the same without scanning every key; a lecture id that is a
        prefix of another, e.g. 'A' and 'A:B', keeps its own keys)."""
        prefix = self.config.hll_key_prefix
        if self.config.hll_key_form == "code":
            key = f"{prefix}{lecture_id}" + (f":{day}" if day else "")
            return {"unique_attendees": self.redis_client.pfcount(key)}
        if day is not None:
            return {"unique_attendees": self.redis_client.pfcount(f"{prefix}{lecture_id}:{day}")}
        stem = f"{prefix}{lecture_id}"
        index = getattr(self.redis_client, "day_keys", None)
        if callable(index):  # SketchClient: the key table's stem index
            keys = index(stem)
        else:  # any redis-py-like client: SCAN for exactly <stem>:YYYY-MM-DD
            pat = glob_escape(stem)
            keys = list(self.redis_client.scan_iter(match=pat + ":" + "[0-9]" * 4 + "-" + "[0-9]" * 2 + "-" +
                                                     "[0-9]" * 2, _type="string"))
        return {"unique_attendees": self.redis_client.pfcount(*keys) if keys else 0}


def glob_escape(text: str) -> str:
    """`text` as a Redis MATCH pattern that matches exactly it: every glob
    special byte backslash-escaped (redis src/util.c stringmatchlen reads
    ``\\x`` as a literal x outside a class; a bracket class would not do:
    ``[^]`` is an empty negated class, ``[]]`` and ``[\\]`` misparse)."""
    return "".join("\\" + ch if ch in "*?[]\\^" else ch for ch in text)


def rank_top_bottom(counts: np.ndarray, keys: Sequence[str], k: int) -> tuple[list, list]:
    """Indices of the first k and the last k keys of the order (count
    descending, key ascending), without sorting every key: only the keys tied
    with or beyond the k-th count (np.partition) are ordered (np.lexsort).
    Returns (head, tail), tail in that order as ``.tail(k)`` lists it."""
    n = len(keys)
    k = min(max(int(k), 0), n)
    if k == 0:
        return [], []
    # counts compare as unsigned: PFCOUNT replies are u64, and a saturated
    # key's (2^63, Redis' llroundl(inf)) is the largest even when the caller
    # holds it in an int64 array
    c = np.ascontiguousarray(np.asarray(counts).astype(np.int64)).view(np.uint64)
    karr = np.asarray(keys)

    def ordered(idx):
        return idx[np.lexsort((karr[idx], ~c[idx]))]

    hi = np.partition(c, n - k)[n - k]      # k-th largest count
    head = ordered(np.nonzero(c >= hi)[0])[:k]
    lo = np.partition(c, k - 1)[k - 1]      # k-th smallest count
    tail = ordered(np.nonzero(c <= lo)[0])[-k:]
    return head.tolist(), tail.tolist()


def rank_top_bottom_dev(counts, k: int, key_rank=None) -> tuple[list, list]:
    """rank_top_bottom over a torch tensor of PFCOUNTs (int64 holding the u64
    replies; device or CPU) without moving the counts: the k-th largest and
    k-th smallest counts come from ``torch.topk`` on the tensor, and only the
    keys tied with or beyond them (normally k each) are copied to the host
    and ordered there.  Order: count descending, then key ascending, where a
    key's place in the key order is ``key_rank[i]`` (a tensor, or None when
    the keys are already in ascending order by index, as C5's
    ``LECT%05d`` / day-key universes are).  Counts compare as unsigned, so a
    saturated key's PFCOUNT (2^63, Redis' llroundl(inf)) stays the largest.
    Returns (head, tail) as rank_top_bottom does."""
    import torch
    n = int(counts.numel())
    k = min(max(int(k), 0), n)
    if k == 0:
        return [], []
    u = counts.view(torch.int64) ^ torch.iinfo(torch.int64).min  # unsigned order as signed order
    hi = torch.topk(u, k, largest=True, sorted=True).values[-1]
    lo = torch.topk(u, k, largest=False, sorted=True).values[-1]

    def ordered(mask):
        idx = torch.nonzero(mask).flatten()
        c = counts.view(torch.int64)[idx].cpu().numpy().view(np.uint64)
        key = (key_rank[idx] if key_rank is not None else idx).cpu().numpy()
        return idx.cpu().numpy()[np.lexsort((key, ~c))]  # ~c: descending unsigned counts

    head = ordered(u >= hi)[:k]
    tail = ordered(u <= lo)[-k:]
    return head.tolist(), tail.tolist()


def lecture_rankings(client: SketchClient, keys: Sequence[str], k: int = 3) -> dict:
    """Most / least attended lecture-day keys by PFCOUNT (one K2 launch).

    Order: count descending, then key ascending (the reference's pandas
    ``sort_values(ascending=False)`` leaves ties in quicksort order; a total
    order is used here so results are reproducible).  ``least_attended`` is
    the tail of the same order, as ``.tail(3)`` (attendance_analysis.py:95).
    At C5 scale (1.8M lecture-day keys) only the tie sets at the two ends are
    ordered (``rank_top_bottom``)."""
    keys = list(keys)
    counts = client.pfcount_each(keys).astype(np.int64)
    head, tail = rank_top_bottom(counts, keys, k)
    return {"most_attended": {keys[i]: int(counts[i]) for i in head},
            "least_attended": {keys[i]: int(counts[i]) for i in tail}}


def campus_rollup(client: SketchClient, groups: dict, dest: str | None = None) -> dict:
    """Per-lecture unions over their day keys (PFCOUNT k1..kn per lecture, one
    launch) and, when ``dest`` is given, a campus-wide PFMERGE of every key."""
    names = list(groups)
    counts = client.pfcount_groups([groups[n] for n in names])
    out = {"per_lecture": {n: int(c) for n, c in zip(names, counts)}}
    if dest is not None:
        client.pfmerge(dest, *[k for n in names for k in groups[n]])
        out["campus_unique"] = client.pfcount(dest)
    return out
