"""Configuration of the attendance sketch path.

The reference imports these names from a ``config/config.py`` that is not in
the repository (attendance_processor.py:13-17, data_generator.py:13-16); the
README gives the values (README.md:104-106, :236-239).  One dataclass keeps
both spellings' meaning; defaults are the README's.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass
class AttendanceConfig:
    # BLOOM_FILTER_KEY / BLOOM_KEY (README.md:104, :236)
    bloom_filter_key: str = "bf:students"
    # BLOOM_FILTER_ERROR_RATE / BLOOM_ERROR_RATE (README.md:104, :238)
    bloom_filter_error_rate: float = 0.01
    # BLOOM_FILTER_CAPACITY / BLOOM_CAPACITY (README.md:104, :239)
    bloom_filter_capacity: int = 100_000
    # HLL_KEY_PREFIX (attendance_processor.py:128); README key form
    # hll:unique:<lecture_id>:<YYYY-MM-DD> (README.md:105-106)
    hll_key_prefix: str = "hll:unique:"
    # "code": f"{prefix}{lecture_id}" exactly as attendance_processor.py:128;
    # "readme": f"{prefix}{lecture_id}:{YYYY-MM-DD}" (UTC day of the event)
    hll_key_form: str = "readme"
    # reproduce _setup_bloom_filter's behaviour (attendance_processor.py:74-92):
    # BF.EXISTS on a missing key answers 0, so BF.RESERVE is never reached.
    faithful_setup: bool = True
    # the Cassandra INSERT (attendance_processor.py:116-124) runs before PFADD;
    # its `student_id int` / `lecture_id text` columns refuse other types, so
    # such a message is nacked and never counted.  False: count any id that
    # redis-py can encode (the bare redis-py semantics of SketchClient.ingest)
    cassandra_row_types: bool = True
    device: int = 0
    batch_size: int = 1 << 16
