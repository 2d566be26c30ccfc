"""Ingest: batched JSON decode + key-slot resolution on
the device, checked against the reference's per-event loop
(attendance_processor.py:100-137) run in Python over the CPU oracle on the
same payloads -- BF.EXISTS answers, nacks and every HLL register array."""
import json
from datetime import datetime, timezone

import numpy as np
import pytest

from test_processor import reference_messages

pytestmark = pytest.mark.gpu

PREFIX = "hll:unique:"


def oracle_loop(orc, chain, messages, key_form="readme"):
    """attendance_processor.py:100-137 with redis-py's argument encoding."""
    from rtsas_amd.encoding import encode
    hlls, valid, nack = {}, [], []
    for m in messages:
        try:
            data = json.loads(bytes(m).decode())
            sid = encode(data["student_id"])
            lecture_id = data["lecture_id"]
            ts = datetime.fromisoformat(data["timestamp"])
            if key_form == "code":
                key = f"{PREFIX}{lecture_id}"
            else:
                if ts.tzinfo is not None:
                    ts = ts.astimezone(timezone.utc)
                key = f"{PREFIX}{lecture_id}:{ts.date().isoformat()}"
        except Exception:
            valid.append(False)
            nack.append(True)
            continue
        v = bool(chain.exists(sid))
        if v:
            hlls.setdefault(key.encode(), orc.HLL()).add(sid)
        valid.append(v)
        nack.append(False)
    return np.array(valid), np.array(nack), hlls


def check_against_oracle(client, orc, chain, msgs, key_form="readme"):
    valid, status = client.ingest("bf:students", msgs, key_form=key_form)
    want_valid, want_nack, hlls = oracle_loop(orc, chain, msgs, key_form)
    assert np.array_equal(valid, want_valid)
    assert np.array_equal(status == -1, want_nack)
    for k, h in hlls.items():
        assert np.array_equal(client.hll_registers(k), h.regs), k
    hll_keys = {k for k, kind in client.keys.kind.items() if kind == "hll"}
    assert hll_keys == set(hlls)
    return status


def preload(client, orc, ids):
    client.execute_command("BF.RESERVE", "bf:students", 0.01, 100000)
    client.execute_command("BF.MADD", "bf:students", *ids)
    chain = orc.Chain(100000, 0.01)
    for i in ids:
        chain.add(str(i).encode())
    return chain


@pytest.mark.parametrize("key_form", ["readme", "code"])
def test_ingest_reference_stream(client, orc, key_form):
    """The reference generator's message stream (data_generator.py:84-185):
    every message decoded on the device, answers and registers exact."""
    valid_ids, msgs = reference_messages(seed=5, n_students=800, days=5)
    chain = preload(client, orc, valid_ids)
    status = check_against_oracle(client, orc, chain, msgs, key_form)
    assert (status == 0).all()


def adversarial_messages(rng, valid_ids):
    good = lambda sid, lec="CS101-L1", ts="2025-03-19T09:15:00": json.dumps(  # noqa: E731
        {"student_id": sid, "timestamp": ts, "lecture_id": lec, "is_valid": True})
    v = lambda: int(rng.choice(valid_ids))  # noqa: E731
    msgs = [
        good(v()), good(v(), ts="2025-03-19"), good(v(), ts="2025-03-19 09:15:00"),
        good(v(), ts="2025-03-19x09:15:00.123"), good(v(), ts="2025-03-19T09:15:00.123456"),
        good(v(), ts="2025-03-19T23:30:00-05:00"), good(v(), ts="2025-03-20T01:30:00+05:30"),
        good(v(), ts="2024-02-29T23:59:59-23:59"), good(v(), ts="2025-01-01T00:00:00+00:00"),
        good(v(), ts="2025-03-19T09:15:00+05:30:00"),      # host (offset seconds)
        good(v(), ts="2025-03-19T09:15"),                   # host (no seconds)
        good(v(), ts="2025-03-19T09:15:00.1234"),           # rejected by fromisoformat: nack
        good(v(), ts="2025-02-29"), good(v(), ts="2025-13-01"), good(v(), ts="2025-03-19T24:00:00"),
        good(v(), ts="2025-03-19T09:15:00Z"), good(v(), ts="0001-01-01T00:10:00+05:30"),
        good(v(), ts="9999-12-31T23:00:00-05:00"),
        good(str(v())), good(v(), lec=7), good(v(), lec="Ünïcode"), good(v(), lec='a"b'),
        good(v(), lec="tab\there"), good(v(), lec=""), good(v(), lec="L:2025"),
        good(float(v())), good(True), good(None), good(-0), good(-5), good([1, 2]),
        good({"x": 1}), good(12345678901234567890), good(v(), lec=["x"]),
        '{"student_id": -0, "lecture_id": "L", "timestamp": "2025-03-19"}',
        '{"student_id": %d, "lecture_id": "L", "timestamp": "2025-03-19T09:15:00", "x": {"y": 1}}' % v(),
        '{"student_id": 1e5, "lecture_id": "L", "timestamp": "2025-03-19"}',
        '{"student_id": NaN, "lecture_id": "L", "timestamp": "2025-03-19"}',
        '{"student_id": %d, "student_id": %d, "lecture_id": "L", "timestamp": "2025-03-19"}' % (999999, v()),
        '  {"student_id" :%d ,"lecture_id":"L","timestamp":"2025-03-19T09:15:00"}\n\t ' % v(),
        '{"student_id": 0123, "lecture_id": "L", "timestamp": "2025-03-19"}',
        '{"student_id": %d, "lecture_id": "L", "timestamp": "2025-03-19",}' % v(),
        '{"lecture_id": "L", "timestamp": "2025-03-19"}',
        '{"student_id": %d, "timestamp": "2025-03-19"}' % v(),
        '{"student_id": %d, "lecture_id": "L"}' % v(),
        '{"student_id": %d, "lecture_id": "L", "timestamp": 20250319}' % v(),
        '[1, 2, 3]', '{}', '', 'not json', '{"student_id": 1', '{"student_id": 1} extra',
        '{"student_id": %d, "lecture_id": "L", "timestamp": "2025-03-19", "ok": true, "no": null,'
        ' "f": false, "n": -12}' % v(),
    ]
    return [m.encode() if isinstance(m, str) else m for m in msgs] + [b"\xff\xfe{}"]


def test_ingest_adversarial_json(client, orc):
    """Escapes, unicode, nested values, floats / bools / null / huge ints as
    ids, duplicate keys, whitespace, missing fields, malformed JSON and every
    timestamp form: decoded on the device when its fast path applies, by
    Python otherwise -- the same answers, nacks and registers either way."""
    rng = np.random.default_rng(6)
    valid_ids = [int(x) for x in rng.choice(np.arange(10000, 100000), 500, replace=False)]
    chain = preload(client, orc, valid_ids)
    msgs = adversarial_messages(rng, valid_ids)
    status = check_against_oracle(client, orc, chain, msgs * 3)
    assert (status == 0).any() and (status == 1).any() and (status == -1).any()


def test_ingest_key_table_lifecycle(client, orc):
    """Keys resolved through the device key table across batches; a key
    deleted between batches is recreated empty (the table is rebuilt)."""
    valid_ids, msgs = reference_messages(seed=7, n_students=300, days=3)
    chain = preload(client, orc, valid_ids)
    half = len(msgs) // 2
    client.ingest("bf:students", msgs[:half])
    client.ingest("bf:students", msgs[half:])
    _, _, hlls = oracle_loop(orc, chain, msgs)
    for k, h in hlls.items():
        assert np.array_equal(client.hll_registers(k), h.regs)
    gone = sorted(hlls)[0]
    client.delete(gone)
    client.ingest("bf:students", msgs[:half])
    _, _, again = oracle_loop(orc, chain, msgs[:half])
    if gone in again:
        assert np.array_equal(client.hll_registers(gone), again[gone].regs)
    for k in set(hlls) - {gone}:
        assert np.array_equal(client.hll_registers(k), hlls[k].regs)


def test_ingest_invalid_only_key_not_created(client, orc):
    """A lecture-day key whose every swipe is invalid is not created (the
    reference only PFADDs valid events)."""
    chain = preload(client, orc, [11111, 22222])
    msgs = [json.dumps({"student_id": 99999, "lecture_id": "EMPTY", "timestamp": "2025-03-19"}).encode(),
            json.dumps({"student_id": 11111, "lecture_id": "FULL", "timestamp": "2025-03-19"}).encode()]
    valid, status = client.ingest("bf:students", msgs)
    assert valid.tolist() == [False, True] and status.tolist() == [0, 0]
    assert client.exists(f"{PREFIX}EMPTY:2025-03-19") == 0
    assert client.exists(f"{PREFIX}FULL:2025-03-19") == 1
