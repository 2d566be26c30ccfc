"""bench.py's algorithmic-bytes model (DESIGN.md §3 "Roofline per K1 variant"),
on CPU: the per-pass byte counts the roofline divides by a kernel's live
duration, restated by hand for C3's one-GPU step and C2's LDS K1."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_partitioned_pass_bytes_c3():
    b = _bench()
    n = 16_000_000
    nvalid, probes = int(0.9 * n), int(10.1 * n)
    bits, k = 158_202_880, 11                     # RESERVE 0.001 / 1e7
    alg = b.pass_bytes(n, nvalid, probes, 8, False, [(bits, k)])
    nslices, ntiles = 302, 15_625                  # ceil(bits / 2^19), ceil(n / 1024)
    rec = 4 * k * n
    # (the fail-list chain: no fail bytes -- overflow flags in the HLL word)
    assert alg["k_part_a"] == n * (8 + 4) + rec + 4 * (nslices + 1) * ntiles + 4 * n
    assert alg["k_part_b"] == rec + 8 * nslices * ntiles + bits // 8
    assert alg["k_part_c"] == n * (4 + 4 + 1) + 128 * nvalid   # 128 B per valid swipe
    # a two-link chain keeps one fail byte per swipe and link
    alg2 = b.pass_bytes(n, nvalid, probes, 8, False, [(bits, 8), (2 * bits, 9)])
    assert alg2["k_part_c"] == n * (2 + 4 + 4 + 1) + 128 * nvalid
    assert alg["k1_stage"] == 0


def test_lds_k1_bytes_c2_slab_on_chip():
    b = _bench()
    n, nvalid, probes = 1_000_000, 900_000, 7_200_000
    bits, k = 1_102_784, 8                         # RESERVE 0.01 / 1e5
    alg = b.pass_bytes(n, nvalid, probes, 7, False, [(bits, k)], lds_k1=True,
                       slab_bytes=(50 + 64) * 16384, cus=256)
    assert alg["k1"] == n * (7 + 4 + 4 + 1)       # probes in LDS, registers on chip
    assert alg["k1_stage"] == (bits // 8) * 256    # the filter staged into every block
    big = b.pass_bytes(n, nvalid, probes, 7, False, [(bits, k)], lds_k1=True,
                       slab_bytes=1 << 30, cus=256)
    assert big["k1"] == n * 16 + 128 * nvalid      # a slab off chip: one line read + written


def test_sector_model_generic_k1():
    b = _bench()
    alg = b.pass_bytes(1000, 900, 7200, 7, True, [(1_102_784, 8)])
    assert alg["k1"] == 1000 * (7 + 0 + 4 + 1) + 64 * 7200 + 128 * 900


def test_checked_reports_a_raising_check():
    """A check that raises (an unsupported collective, a shape mismatch) is
    reported in the bench line as ok false with the error, not by losing the
    line; a passing check's dict comes through unchanged."""
    b = _bench()

    def boom(x):
        raise RuntimeError("alltoall unsupported %d" % x)

    r = b.checked(boom, 3)
    assert r["ok"] is False and r["error"] == "RuntimeError: alltoall unsupported 3"
    assert b.checked(lambda **k: {"ok": True, **k}, a=1) == {"ok": True, "a": 1}
