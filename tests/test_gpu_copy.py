"""hj_dev_stream_copy (the bench's copy floor): both shapes copy every byte,
tails past the last whole tile included, and bad arguments are refused."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mlir-hashjoin_amd"))

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", ["persistent", "flat"])
@pytest.mark.parametrize("rows", [1, 4095, 4096, 256 * 4096 + 17, 3 * (1 << 20) + 5])
def test_stream_copy_bytes(shape, rows):
    import hashjoin
    g = torch.Generator(device="cuda").manual_seed(rows)
    a = torch.randint(-(1 << 62), 1 << 62, (2 * rows,), dtype=torch.int64, device="cuda", generator=g)
    b = torch.full_like(a, -1)
    hashjoin.stream_copy(a, b, shape)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_stream_copy_refuses_bad_args():
    import hashjoin
    a = torch.zeros(8, dtype=torch.int64, device="cuda")
    with pytest.raises(ValueError):
        hashjoin.stream_copy(a, torch.zeros(6, dtype=torch.int64, device="cuda"))
    lib = hashjoin.lib
    assert lib.hj_dev_stream_copy(a.data_ptr(), a.data_ptr(), 4, 7, None) == -1     # bad shape
    assert lib.hj_dev_stream_copy(a.data_ptr() + 8, a.data_ptr(), 2, 0, None) == -1  # misaligned
    assert lib.hj_dev_stream_copy(None, None, 0, 1, None) == 0                      # nothing to copy
