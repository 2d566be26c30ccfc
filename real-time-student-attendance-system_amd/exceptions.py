"""Exception classes with redis-py's names (``redis.exceptions``).

The reference catches ``redis.exceptions.ResponseError`` around its Bloom
calls (attendance_processor.py:80, :90; data_generator.py:65), so the facade
raises the same class names with the same Redis / RedisBloom error texts.
"""


class RedisError(Exception):
    pass


class ResponseError(RedisError):
    """An error reply (``-ERR ...`` / ``-WRONGTYPE ...``)."""


class DataError(RedisError):
    """Argument that redis-py refuses to encode (e.g. a ``bool``)."""


WRONGTYPE = "WRONGTYPE Operation against a key holding the wrong kind of value"
