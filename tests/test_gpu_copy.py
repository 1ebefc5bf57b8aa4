"""qgcm_stream_copy, the in-repo copy kernel bench.py quotes the roofline against (`copy_achievable`):
every byte arrives and nothing past the buffer is written, for sizes around the 4-KiB tile of one
workgroup; a size that is not a multiple of 16 is refused (include/qgcm.h) and writes nothing."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nbytes", [16, 4096, 4096 + 16, 4096 * 3 - 16, (1 << 20) + 48, (1 << 20) + 55])
def test_stream_copy_exact(ctx, nbytes):
    import torch

    from quantum_amd import _lib

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    src = torch.randint(0, 256, (nbytes + 64,), dtype=torch.uint8, device="cuda")
    dst = torch.full((nbytes + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    rc = _lib.lib().qgcm_stream_copy(ctx.handle, dst.data_ptr(), src.data_ptr(), nbytes, s.cuda_stream)
    torch.cuda.synchronize()
    if nbytes % 16:
        assert rc == _lib.QGCM_E_ARG and bool((dst == 0xA5).all())
        return
    assert rc == 0
    assert torch.equal(dst[:nbytes], src[:nbytes])
    assert bool((dst[nbytes:] == 0xA5).all())
