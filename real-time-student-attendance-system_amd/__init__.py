"""MI355X sketch engine for the attendance validate-and-count hot path.

Drop-in for the reference's redis-py Bloom + HyperLogLog calls
(attendance_processor.py:109-129, data_generator.py:57-63,
attendance_processor.py:152), executed by hand-written gfx950 HIP kernels in
``csrc/libsketch.so`` through the C-ABI of ``include/sketch.h``.
"""
from . import exceptions
from ._lib import Context, SketchLibError, load as load_library, LIB_PATH
from .client import BloomCommands, Pipeline, Redis, SketchClient
from .config import AttendanceConfig
from .encoding import encode, pack, pack_ints
from .exceptions import DataError, RedisError, ResponseError
from .processor import AttendanceProcessor, campus_rollup, lecture_rankings

__all__ = [
    "AttendanceConfig", "AttendanceProcessor", "BloomCommands", "Context", "DataError",
    "LIB_PATH", "Pipeline", "Redis", "RedisError", "ResponseError", "SketchClient",
    "SketchLibError", "campus_rollup", "encode", "exceptions", "lecture_rankings",
    "load_library", "pack", "pack_ints",
]
