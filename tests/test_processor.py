"""Processor counterpart (attendance_processor.py:26-165) and rankings
(attendance_analysis.py:87-97): host logic on CPU with an oracle-backed
client double; the real device client in the gpu-marked test."""
import json
from datetime import datetime, timedelta

import numpy as np
import pytest


def reference_messages(seed=0, n_students=200, days=3):
    """Messages with the reference generator's schema and mix
    (data_generator.py:84-185): entry + exit per student-day, ~15 % invalid
    attempts from a 6-digit pool, plus 20 standalone invalids."""
    rng = np.random.default_rng(seed)
    valid = [int(x) for x in rng.choice(np.arange(10000, 100000), n_students, replace=False)]
    invalid = [int(x) for x in rng.choice(np.arange(100000, 1000000), 50, replace=False)]
    base = datetime(2025, 3, 17)
    msgs = []
    for sid in valid:
        for d in rng.choice(days, int(rng.integers(1, days + 1)), replace=False):
            day = base + timedelta(days=int(d))
            entry = day.replace(hour=int(rng.integers(8, 12)), minute=int(rng.integers(0, 60)))
            exit_ = entry + timedelta(hours=int(rng.integers(3, 5)))
            for ts, et in ((entry, "entry"), (exit_, "exit")):
                msgs.append({"student_id": sid, "timestamp": ts.isoformat(),
                             "lecture_id": f"LECTURE_{ts.strftime('%Y%m%d')}", "is_valid": True,
                             "event_type": et})
            if rng.random() < 0.15:
                msgs.append({"student_id": int(rng.choice(invalid)), "timestamp": entry.isoformat(),
                             "lecture_id": f"LECTURE_{entry.strftime('%Y%m%d')}",
                             "is_valid": False, "event_type": "entry"})
    for _ in range(20):
        day = base + timedelta(days=int(rng.integers(0, days)))
        msgs.append({"student_id": int(rng.choice(invalid)), "timestamp": day.isoformat(),
                     "lecture_id": f"LECTURE_{day.strftime('%Y%m%d')}", "is_valid": False,
                     "event_type": "entry"})
    return valid, [json.dumps(m).encode() for m in msgs]


class OracleClient:
    """Test double with the SketchClient methods the processor uses."""

    def __init__(self, orc):
        self.orc = orc
        self.chains, self.hlls, self.calls = {}, {}, []

    def execute_command(self, *a):
        self.calls.append(a[0])
        if a[0] == "BF.EXISTS":
            c = self.chains.get(a[1])
            return c.exists(str(a[2]).encode()) if c else 0
        if a[0] == "BF.RESERVE":
            self.chains[a[1]] = self.orc.Chain(int(a[3]), float(a[2]))
            return "OK"
        if a[0] == "BF.ADD":
            c = self.chains.setdefault(a[1], self.orc.Chain(100, 0.01))
            return c.add(str(a[2]).encode())
        raise NotImplementedError(a[0])

    def exists(self, k):
        return int(k in self.chains or k in self.hlls)

    def swipes(self, bf_key, keys, ids):
        c = self.chains.get(bf_key)
        out = []
        for k, i in zip(keys, ids):
            b = i if isinstance(i, bytes) else str(i).encode()
            v = bool(c.exists(b)) if c else False
            if v:
                self.hlls.setdefault(k, self.orc.HLL()).add(b)
            out.append(v)
        return np.array(out)

    def pfcount(self, *keys):
        u = self.orc.HLL()
        for k in keys:
            if k in self.hlls:
                u.merge(self.hlls[k])
        return u.count()

    def scan_iter(self, match=None, count=None, _type=None):
        import fnmatch
        for k in sorted(self.hlls):
            if fnmatch.fnmatchcase(k, match or "*") and _type in (None, "string"):
                yield k


def test_setup_quirk_and_batches(pkg, orc):
    """BF.EXISTS on the missing key answers 0, so the reference's BF.RESERVE
    branch never runs (attendance_processor.py:76-92) -- reproduced."""
    cl = OracleClient(orc)
    p = pkg.AttendanceProcessor(client=cl, config=pkg.AttendanceConfig(batch_size=100))
    valid, msgs = reference_messages()
    for sid in valid:  # data_generator.py:57-63: BF.ADD per id (auto-create)
        cl.execute_command("BF.ADD", "bf:students", sid)
    rows = [r for batch in p.process_attendance(msgs + [b"{not json", b'{"student_id": 1}'])
            for r in batch]
    assert "BF.RESERVE" not in cl.calls
    assert len(rows) == len(msgs) and p.nacked == 2 and p.acked == len(msgs)
    truth = [json.loads(m)["is_valid"] for m in msgs]
    assert sum(r["is_valid"] for r in rows) >= sum(truth)      # Bloom: no false negatives
    assert all(r["is_valid"] for r, t in zip(rows, truth) if t)
    key = "hll:unique:LECTURE_20250317:2025-03-17"
    assert key in cl.hlls
    assert p.get_attendance_stats("LECTURE_20250317", "2025-03-17")["unique_attendees"] == \
        cl.hlls[key].count()


def _per_event_reference(orc, chain, msgs, row_types=True):
    """attendance_processor.py:100-137 one message at a time: json.loads,
    fields, fromisoformat, BF.EXISTS (redis-py encoding), the Cassandra INSERT's
    column types, then PFADD if valid.  Returns (acked, nacked, answers, hlls)."""
    from rtsas_amd.encoding import encode
    from rtsas_amd.exceptions import DataError
    acked = nacked = 0
    answers, hlls = [], {}
    for m in msgs:
        try:
            data = json.loads(m)
            sid, lecture = data["student_id"], data["lecture_id"]
            ts = datetime.fromisoformat(data["timestamp"])
            b = encode(sid)
            v = bool(chain.exists(b))
            if row_types and (type(sid) is not int or not -2**31 <= sid < 2**31
                              or not isinstance(lecture, str)):
                raise TypeError("INSERT")
            if v:
                hlls.setdefault(f"hll:unique:{lecture}:{ts.date().isoformat()}", orc.HLL()).add(b)
            answers.append(v)
            acked += 1
        except (ValueError, KeyError, TypeError, DataError):
            nacked += 1
    return acked, nacked, answers, hlls


ODD_IDS = [True, None, {"a": 1}, [1, 2], 12.5, "12345", 2**31, -2**31 - 1, -5, 0, 2**31 - 1]


def _odd_messages(valid):
    """Messages whose student_id redis-py refuses (bool, None, dict, list), or
    the Cassandra int column refuses (float, str, out of int32), mixed with
    ordinary ones, plus a non-string lecture_id."""
    msgs = []
    for j, sid in enumerate(ODD_IDS + valid[:40]):
        msgs.append(json.dumps({"student_id": sid, "timestamp": "2025-03-19T09:00:00",
                                "lecture_id": "LECTURE_20250319", "is_valid": True,
                                "event_type": "entry"}).encode())
    msgs.append(json.dumps({"student_id": valid[0], "timestamp": "2025-03-19T09:00:00",
                            "lecture_id": 20250319}).encode())
    return msgs


@pytest.mark.parametrize("row_types", [True, False])
def test_process_batch_nacks_per_message(pkg, orc, row_types):
    """One refused id does not fail the batch: every message gets the per-event
    loop's ack / nack, answers and registers (attendance_processor.py:134-136)."""
    cl = OracleClient(orc)
    valid, _ = reference_messages(n_students=60)
    for sid in valid:
        cl.execute_command("BF.ADD", "bf:students", sid)
    msgs = _odd_messages(valid)
    p = pkg.AttendanceProcessor(client=cl, config=pkg.AttendanceConfig(cassandra_row_types=row_types))
    rows = p.process_batch(msgs)
    acked, nacked, answers, hlls = _per_event_reference(orc, cl.chains["bf:students"], msgs, row_types)
    assert (p.acked, p.nacked) == (acked, nacked) == (len(rows), len(msgs) - len(rows))
    assert [r["is_valid"] for r in rows] == answers
    assert set(cl.hlls) == set(hlls)
    for k, h in hlls.items():
        assert np.array_equal(cl.hlls[k].regs, h.regs)
    if row_types:
        assert nacked == 4 + 4 + 1  # 4 unencodable, 4 non-int32 ids, 1 int lecture_id


def test_stats_without_day_unions_the_lecture_days(pkg, orc):
    """README key form: get_attendance_stats(lecture_id) -- the reference's
    signature -- is the PFCOUNT union of the lecture's day keys."""
    cl = OracleClient(orc)
    valid, msgs = reference_messages(n_students=150, days=3)
    for sid in valid:
        cl.execute_command("BF.ADD", "bf:students", sid)
    same = [json.loads(m) for m in msgs]
    for m in same:
        m["lecture_id"] = "CS101-L1"
    p = pkg.AttendanceProcessor(client=cl)
    p.process_batch([json.dumps(m).encode() for m in same])
    days = sorted(k for k in cl.hlls if k.startswith("hll:unique:CS101-L1:"))
    assert len(days) == 3
    assert p.get_attendance_stats("CS101-L1")["unique_attendees"] == cl.pfcount(*days)
    assert p.get_attendance_stats("CS999")["unique_attendees"] == 0
    # the day keys come from the store: a fresh processor (another process, a
    # restart) on the same store answers the same
    q = pkg.AttendanceProcessor(client=cl)
    assert q.get_attendance_stats("CS101-L1")["unique_attendees"] == cl.pfcount(*days)
    # a lecture id that is a prefix of another is not mixed in
    cl.hlls["hll:unique:CS101-L10:2025-03-17"] = cl.hlls[days[0]]
    assert q.get_attendance_stats("CS101-L1")["unique_attendees"] == cl.pfcount(*days)


def test_non_faithful_setup_reserves(pkg, orc):
    cl = OracleClient(orc)
    cfg = pkg.AttendanceConfig(faithful_setup=False)
    pkg.AttendanceProcessor(client=cl, config=cfg)._setup_bloom_filter()
    assert "BF.RESERVE" in cl.calls
    assert cl.chains["bf:students"].link_info(0)["entries"] == 100000


def test_key_forms(pkg, orc):
    p = pkg.AttendanceProcessor(client=OracleClient(orc))
    ts = datetime.fromisoformat("2025-03-19T23:30:00-02:00")
    assert p.hll_key("CS101-L1", ts) == "hll:unique:CS101-L1:2025-03-20"   # UTC day
    p.config.hll_key_form = "code"
    assert p.hll_key("LECTURE_20250319", ts) == "hll:unique:LECTURE_20250319"


@pytest.mark.gpu
def test_processor_end_to_end_on_device(pkg, orc):
    client = pkg.SketchClient(decode_responses=True)
    p = pkg.AttendanceProcessor(client=client, config=pkg.AttendanceConfig(batch_size=257))
    ref = OracleClient(orc)
    pref = pkg.AttendanceProcessor(client=ref)
    valid, msgs = reference_messages(seed=3, n_students=1000, days=7)
    for sid in valid:
        client.execute_command("BF.ADD", "bf:students", sid)
        ref.execute_command("BF.ADD", "bf:students", sid)
    rows = [r for b in p.process_attendance(msgs) for r in b]
    want = [r for b in pref.process_attendance(msgs) for r in b]
    assert [r["is_valid"] for r in rows] == [r["is_valid"] for r in want]
    keys = sorted(ref.hlls)
    for k in keys:
        assert np.array_equal(client.hll_registers(k), ref.hlls[k].regs)
    got = pkg.lecture_rankings(client, keys, k=3)
    counts = {k: ref.hlls[k].count() for k in keys}
    order = sorted(keys, key=lambda k: (-counts[k], k))
    assert list(got["most_attended"]) == order[:3]
    assert list(got["least_attended"]) == order[-3:]
    roll = pkg.campus_rollup(client, {"all": keys}, dest="hll:campus")
    u = orc.HLL()
    for k in keys:
        u.merge(ref.hlls[k])
    assert roll["per_lecture"]["all"] == u.count() == roll["campus_unique"]


def test_rank_top_bottom_matches_full_sort(pkg):
    """rank_top_bottom == the first / last k of sorted(keys, (-count, key)),
    with heavy ties (few distinct counts), k larger than n, and k = 0."""
    from rtsas_amd.processor import rank_top_bottom
    rng = np.random.default_rng(4)
    for n, distinct, k in [(1, 1, 3), (5, 2, 3), (200, 3, 3), (5000, 40, 7), (50, 50, 60), (9, 4, 0)]:
        keys = [f"hll:unique:L{int(x):05d}:2025-{int(y):02d}-01" for x, y in
                zip(rng.integers(0, 10 * n, n), rng.integers(1, 13, n))]
        keys = list(dict.fromkeys(keys))
        counts = rng.integers(0, distinct, len(keys))
        order = sorted(range(len(keys)), key=lambda i: (-counts[i], keys[i]))
        head, tail = rank_top_bottom(counts, keys, k)
        kk = min(k, len(keys))
        assert head == order[:kk]
        assert tail == (order[-kk:] if kk else [])


def test_rank_top_bottom_dev_matches_host(pkg):
    """rank_top_bottom_dev (torch.topk on the counts, only the tie sets moved
    to the host) == rank_top_bottom, keys in index order or ranked by a key
    order tensor; the saturated PFCOUNT 2^63 (held as int64: negative) sorts
    as the largest in both."""
    import torch
    from rtsas_amd.processor import rank_top_bottom, rank_top_bottom_dev
    rng = np.random.default_rng(5)
    for n, distinct, k in [(1, 1, 3), (7, 2, 3), (300, 3, 3), (20000, 50, 3), (64, 64, 70), (9, 4, 0)]:
        counts = rng.integers(0, distinct, n).astype(np.int64)
        if n > 5:
            counts[[1, 4]] = np.uint64(1 << 63).astype(np.int64)  # two saturated keys
        names = [f"LECT{i:05d}" for i in range(n)]
        assert rank_top_bottom_dev(torch.from_numpy(counts), k) == rank_top_bottom(counts, names, k)
        perm = rng.permutation(n)  # key i is the perm[i]-th name in ascending order
        pnames = [f"K{int(p):06d}" for p in perm]
        got = rank_top_bottom_dev(torch.from_numpy(counts), k, key_rank=torch.from_numpy(perm))
        assert got == rank_top_bottom(counts, pnames, k)
        if n > 5 and k:
            assert got[0][:2] == sorted([1, 4], key=lambda i: pnames[i])


@pytest.mark.gpu
@pytest.mark.parametrize("row_types", [True, False])
def test_process_batch_nacks_per_message_on_device(pkg, orc, row_types):
    """The same odd ids through the real client: acks, nacks, answers and
    registers equal the per-event loop; the refused ids fail no other
    message of the batch."""
    client = pkg.SketchClient(decode_responses=True)
    valid, _ = reference_messages(n_students=60)
    ref = OracleClient(orc)
    for sid in valid:
        client.execute_command("BF.ADD", "bf:students", sid)
        ref.execute_command("BF.ADD", "bf:students", sid)
    msgs = _odd_messages(valid)
    p = pkg.AttendanceProcessor(client=client,
                                config=pkg.AttendanceConfig(cassandra_row_types=row_types))
    rows = p.process_batch(msgs)
    acked, nacked, answers, hlls = _per_event_reference(orc, ref.chains["bf:students"], msgs,
                                                        row_types)
    assert (p.acked, p.nacked) == (acked, nacked)
    assert [r["is_valid"] for r in rows] == answers
    for k, h in hlls.items():
        assert np.array_equal(client.hll_registers(k), h.regs)
        assert client.pfcount(k) == h.count()
    client.flushall()


@pytest.mark.gpu
def test_c1_readme_default_exact(pkg, orc):
    """C1 exactly as BASELINE.json configs[0] states it: bf:students RESERVE
    0.01 / 100000, 1000 unique 5-digit ids preloaded one BF.ADD each
    (data_generator.py:53-63), 10k swipes of lecture CS101-L1 on one day with
    the reference's invalid mix (~7 %, 50 six-digit ids, :80-81), through the
    processor: every answer, the register array and PFCOUNT == the per-event
    loop over the oracle."""
    rng = np.random.default_rng(20251003)
    client = pkg.SketchClient(decode_responses=True)
    p = pkg.AttendanceProcessor(client=client, config=pkg.AttendanceConfig(batch_size=4096,
                                                                           faithful_setup=False))
    p._setup_bloom_filter()   # BF.RESERVE bf:students 0.01 100000
    ref = OracleClient(orc)
    ref.execute_command("BF.RESERVE", "bf:students", 0.01, 100000)
    members = [int(x) for x in rng.choice(np.arange(10000, 100000), 1000, replace=False)]
    invalid = [int(x) for x in rng.choice(np.arange(100000, 1000000), 50, replace=False)]
    adds = [client.execute_command("BF.ADD", "bf:students", sid) for sid in members]
    assert adds == [ref.execute_command("BF.ADD", "bf:students", sid) for sid in members]
    info = client.bf_links("bf:students")
    assert len(info) == 1 and info[0]["bytes"] == 137848 and info[0]["hashes"] == 8
    bad = rng.random(10_000) < 0.071
    ids = np.where(bad, rng.choice(invalid, 10_000), rng.choice(members, 10_000))
    msgs = [json.dumps({"student_id": int(s), "timestamp": f"2025-03-19T{9 + i % 3:02d}:00:00",
                        "lecture_id": "CS101-L1", "is_valid": not bool(b),
                        "event_type": "entry"}).encode() for i, (s, b) in enumerate(zip(ids, bad))]
    rows = [r for batch in p.process_attendance(msgs) for r in batch]
    acked, nacked, answers, hlls = _per_event_reference(orc, ref.chains["bf:students"], msgs)
    assert (p.acked, p.nacked) == (acked, nacked) == (10_000, 0)
    assert [r["is_valid"] for r in rows] == answers
    key = "hll:unique:CS101-L1:2025-03-19"
    assert list(hlls) == [key]
    assert np.array_equal(client.hll_registers(key), hlls[key].regs)
    assert p.get_attendance_stats("CS101-L1", "2025-03-19")["unique_attendees"] == hlls[key].count()
    assert p.get_attendance_stats("CS101-L1")["unique_attendees"] == hlls[key].count()
    client.flushall()


@pytest.mark.gpu
def test_sketch_client_day_key_index(pkg):
    """get_attendance_stats(lecture) without a day reads the key table's day
    index (KeySpace.day_keys), not a scan of every key: only README day keys
    <prefix><lecture>:YYYY-MM-DD count, a lecture id that prefixes another
    ('A' vs 'A:B') keeps its own keys, and DEL / FLUSHALL keep the index
    (ADVICE r3)."""
    c = pkg.SketchClient(decode_responses=True)
    for k, v in [("hll:unique:A:2025-03-01", 1), ("hll:unique:A:2025-03-02", 2),
                 ("hll:unique:A:B:2025-03-01", 3), ("hll:unique:A:notes", 4), ("hll:unique:AB:2025-03-01", 5)]:
        c.pfadd(k, v)
    assert c.day_keys("hll:unique:A") == ["hll:unique:A:2025-03-01", "hll:unique:A:2025-03-02"]
    assert c.day_keys("hll:unique:A:B") == ["hll:unique:A:B:2025-03-01"]
    p = pkg.AttendanceProcessor(client=c)
    assert p.get_attendance_stats("A")["unique_attendees"] == c.pfcount("hll:unique:A:2025-03-01",
                                                                        "hll:unique:A:2025-03-02") == 2
    c.delete("hll:unique:A:2025-03-01")
    assert c.day_keys("hll:unique:A") == ["hll:unique:A:2025-03-02"]
    assert p.get_attendance_stats("A")["unique_attendees"] == 1
    c.flushall()
    assert c.day_keys("hll:unique:A") == [] and p.get_attendance_stats("A")["unique_attendees"] == 0
