"""regnn_gemm_x6 against torch.mm (hipBLASLt fp32) on the wide NS model's shapes: ms per call
and TFLOP/s (fp32-equivalent 2 M N K), HIP events, median of 20."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "re-gnn_amd"))
from regnn_hip import ops  # noqa: E402


def t_ms(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = "cuda"
    for (M, N, K, ta, tb, name) in [(13312, 512, 512, False, False, "S @ Wc (fwd)"),
                                     (13312, 512, 512, False, True, "dS = dA Wc^T"),
                                     (512, 512, 13312, True, False, "dWc = S^T dA"),
                                     (512, 512, 512, False, False, "512^3"),
                                     (512, 349, 512, False, True, "out_lin"),
                                     (5606, 512, 512, False, False, "n1=5606 fwd"),
                                     (512, 512, 349, False, False, "out_lin gx"),
                                     (349, 512, 512, True, False, "out_lin gw"),
                                     (13312, 512, 4, False, False, "w @ b_c"),
                                     (13312, 4, 512, False, True, "g b_c^T"),
                                     (4, 512, 13312, True, False, "w^T g"),
                                     (4, 512, 512, False, False, "b_cat @ W")]:
        a = torch.randn(*((K, M) if ta else (M, K)), device=dev)
        b = torch.randn(*((N, K) if tb else (K, N)), device=dev)
        if not (ops.gemm_x6_ok(a) and ops.gemm_x6_ok(b)):
            print(f"{name}: skipped (alignment)")
            continue
        A = a.t() if ta else a
        B = b.t() if tb else b
        tt = t_ms(lambda: torch.mm(A, B))
        tx = t_ms(lambda: ops.gemm_x6(a, b, trans_a=ta, trans_b=tb))
        fl = 2.0 * M * N * K
        print(f"{name:16s} M={M:6d} N={N:4d} K={K:6d}: torch {tt * 1e3:8.1f} us "
              f"({fl / tt / 1e9:6.1f} TF/s)  x6 {tx * 1e3:8.1f} us ({fl / tx / 1e9:6.1f} TF/s) "
              f"splits {ops._gemm_splits(M, N, K)}")


if __name__ == "__main__":
    main()
