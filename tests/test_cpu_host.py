"""Host-side helpers that run without a GPU: the chunked weight-gradient reduction used by the
HIP-path Linear / head backward must equal the plain g^T x."""
import torch

from regnn_hip import ops


def test_batched_wgrad_matches_mm():
    torch.manual_seed(0)
    for rows in (5, 4096, 3 * 4096 + 17):
        g = torch.randn(rows, 7, dtype=torch.float64)
        x = torch.randn(rows, 5, dtype=torch.float64)
        got = ops.batched_wgrad(g, x, chunk=1024)
        assert torch.allclose(got, g.t() @ x, rtol=1e-12, atol=1e-10)
