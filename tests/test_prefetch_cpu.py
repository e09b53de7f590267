"""Native host prefetcher (csrc/host/prefetch.cpp): ring protocol and gathered contents on CPU."""
import pytest
import torch


def _lib():
    from masters_thesis_amd.ops import _lib

    C = _lib.lib(required=False)
    if C is None or not hasattr(C, "HostPrefetcher"):
        pytest.skip("native extension not built")
    return C


@pytest.mark.parametrize("B,R,threads", [(1, 4, 2), (3, 2, 1), (4, 3, 3)])
def test_host_prefetcher_ring_gathers_permuted_rows(B, R, threads):
    C = _lib()
    g = torch.Generator().manual_seed(0)
    X = torch.randn(50, 7, 3, generator=g)
    F = torch.randn(50, 2, generator=g)
    staging = [torch.empty((R * B, 7, 3)), torch.empty((R * B, 2))]
    pf = C.HostPrefetcher([X, F], staging, B, R, threads)
    idx = torch.randperm(50, generator=g)
    nb = 50 // B
    pf.start(idx, nb)
    for b in range(nb):
        slot = pf.wait(b, 5000)
        assert slot == b % R
        rows = idx[b * B:(b + 1) * B]
        assert torch.equal(staging[0][slot * B:(slot + 1) * B], X[rows])
        assert torch.equal(staging[1][slot * B:(slot + 1) * B], F[rows])
        # the slot after the ring cannot be filled until b is released
        if b + R < nb:
            assert not pf.ready(b + R)
        pf.release(b)
    # restart for a second epoch on the same object
    pf.start(idx.flip(0).contiguous(), 2)
    assert pf.wait(1, 5000) == 1 % R
    pf.close()


def test_host_prefetcher_rejects_out_of_range_indices():
    C = _lib()
    X = torch.randn(5, 3)
    pf = C.HostPrefetcher([X], [torch.empty(2, 3)], 1, 2, 1)
    with pytest.raises(RuntimeError):
        pf.start(torch.tensor([0, 9]), 2)
    pf.close()


def test_streaming_loader_cpu_fallback_matches_base():
    from masters_thesis_amd.data.datamodule import TensorBatchLoader
    from masters_thesis_amd.data.prefetch import StreamingLoader

    X = torch.arange(40.0).view(10, 4)
    base = TensorBatchLoader([X], 3, shuffle=True, seed=1)
    ld = StreamingLoader(base, "cpu")
    assert not ld.supports_static()
    got = torch.cat([b[0] for b in ld])
    ref = torch.cat([b[0] for b in base])
    assert torch.equal(got, ref) and len(ld) == 4


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_prefetcher_under_sanitizers(kind):
    """SURVEY §5 race / memory-error detection for the native host runtime: the prefetcher's ring protocol
    stress driver (csrc/host/tests/prefetch_stress.cpp) built with AddressSanitizer+UBSan and with
    ThreadSanitizer (host code only; no GPU sanitizers on this pool) must run clean."""
    import shutil
    import subprocess

    from masters_thesis_amd.ops.build import build_host_sanitized

    if shutil.which("g++") is None and shutil.which("clang++") is None:
        pytest.skip("no host C++ compiler")
    (exe,) = build_host_sanitized((kind,))
    env = {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1", "UBSAN_OPTIONS": "halt_on_error=1",
           "TSAN_OPTIONS": "halt_on_error=1"}
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "prefetch_stress: OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
