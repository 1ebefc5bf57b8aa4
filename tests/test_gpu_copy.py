"""qgcm_stream_copy, the in-repo copy kernel bench.py quotes the roofline against (`copy_achievable`):
every whole 16-B piece of the buffer arrives, nothing past it is written, for sizes around the 4-KiB
tile of one workgroup."""
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
    _lib.check(_lib.lib().qgcm_stream_copy(ctx.handle, dst.data_ptr(), src.data_ptr(), nbytes, s.cuda_stream),
               "qgcm_stream_copy")
    torch.cuda.synchronize()
    whole = nbytes // 16 * 16
    assert torch.equal(dst[:whole], src[:whole])
    assert bool((dst[whole:] == 0xA5).all())
