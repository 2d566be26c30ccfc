"""The C-ABI library loads and exports every symbol include/sketch.h declares
(no compute calls: this runs on CPU-only machines too)."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sketch.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ske_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_surface():
    syms = header_symbols()
    for s in ["ske_open", "ske_swipes", "ske_bf_madd", "ske_bf_mexists", "ske_hll_pfadd",
              "ske_hll_pfcount", "ske_hll_pfmerge", "ske_bf_reserve"]:
        assert s in syms


def test_library_exports_every_header_symbol(pkg):
    lib = pkg.load_library()
    path = pkg.LIB_PATH
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (ske_[a-z0-9_]+)", out))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing
    for s in header_symbols():
        assert getattr(lib, s) is not None


def test_ctypes_signatures_cover_header(pkg):
    from rtsas_amd import _lib
    assert sorted(_lib.SIGNATURES) == header_symbols()


def test_library_is_gfx950(pkg):
    """The fat binary carries gfx950 code objects only."""
    data = open(pkg.LIB_PATH, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in data


def test_strerror_texts(pkg):
    from rtsas_amd import _lib
    assert _lib.strerror(-5) == "ERR item exists"
    assert _lib.strerror(-6) == "ERR non scaling filter is full"
    assert _lib.strerror(-8) == "ERR (0 < error rate range < 1)"
    assert _lib.strerror(-9) == "ERR (capacity should be larger than 0)"


def test_open_without_gpu_fails_loudly(pkg):
    """No CPU fallback: without a usable GPU ske_open returns an error and
    the Python context raises."""
    lib = pkg.load_library()
    p = C.c_void_p()
    rc = lib.ske_open(0, C.byref(p))
    if rc == 0:  # a GPU is present (run on the GPU box): close and stop here
        lib.ske_close(p)
        pytest.skip("GPU present")
    assert rc < 0
    with pytest.raises(pkg.SketchLibError):
        pkg.Context(0)


def test_null_context_is_rejected(pkg):
    lib = pkg.load_library()
    assert lib.ske_close(None) == -1
    assert lib.ske_sync(None) == -1
    assert lib.ske_swipes(None, 0, None, None, None, 0, None, 0) == -1


def test_swipe_batch_struct_layout(tmp_path):
    """ctypes' SweBatch mirrors ske_swipe_batch (include/sketch.h) field by field."""
    from rtsas_amd.engine import SweBatch
    src = tmp_path / "layout.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "sketch.h"\n'
                   "int main(void) { printf(\"%zu %zu %zu %zu %zu %zu %zu\\n\", "
                   "sizeof(ske_swipe_batch), offsetof(ske_swipe_batch, slot), "
                   "offsetof(ske_swipe_batch, bytes), offsetof(ske_swipe_batch, offs), "
                   "offsetof(ske_swipe_batch, width), offsetof(ske_swipe_batch, n), "
                   "offsetof(ske_swipe_batch, out_valid)); return 0; }\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)],
                   check=True)
    got = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    want = [C.sizeof(SweBatch)] + [getattr(SweBatch, f).offset
                                   for f in ("slot", "bytes", "offs", "width", "n", "out_valid")]
    assert got == want


def test_swipes_many_rejects_bad_arguments(pkg):
    lib = pkg.load_library()
    # a null context is rejected before any device work
    assert lib.ske_swipes_many_async(None, 0, None, 0, 0) < 0
