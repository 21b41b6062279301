"""FiLM weight-gradient GEMM at the bs128 shapes: ``dy^T @ x`` with fp32
output over every pixel of a level (K up to 1M).  Compares hipBLASLt's
single mixed-precision GEMM (``torch.mm(out_dtype=fp32)``, what the step runs)
with an explicit split-K as a batched GEMM + fp32 sum of the partials."""
import sys
import time

import torch


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def main():
    dev = torch.device("cuda", 0)
    # (rows, S, K): level 0..3 of the bs128 step (256 images of 64^2 .. 8^2)
    shapes = [(1048576, 2048, 1024), (262144, 4608, 1024), (65536, 4608, 1024), (16384, 9216, 1024)]
    if len(sys.argv) > 1 and sys.argv[1] == "bs32":   # the 4-GPU per-GPU share
        shapes = [(262144, 2048, 1024), (65536, 4608, 1024), (16384, 4608, 1024), (4096, 9216, 1024)]
    for rows, S, K in shapes:
        dy = torch.randn(rows, S, device=dev, dtype=torch.bfloat16)
        x = torch.randn(rows, K, device=dev, dtype=torch.bfloat16)
        ref = torch.mm(dy.t(), x, out_dtype=torch.float32)
        flop = 2.0 * rows * S * K
        t = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
        print(f"rows={rows} S={S} K={K} mm_f32 {1e3 * t:.3f} ms {flop / t / 1e12:.0f} TF/s", flush=True)
        for sp in (2, 4, 8, 16):
            if rows % sp:
                continue
            a = dy.view(sp, rows // sp, S).transpose(1, 2)
            b = x.view(sp, rows // sp, K)

            def f():
                return torch.bmm(a, b, out_dtype=torch.float32).sum(0)
            try:
                out = f()
            except (RuntimeError, TypeError) as e:
                print(f"  split{sp}: unsupported ({e})", flush=True)
                break
            err = float((out - ref).norm() / ref.norm())
            t = timeit(f)
            print(f"  split{sp} bmm_f32+sum {1e3 * t:.3f} ms {flop / t / 1e12:.0f} TF/s rel_err {err:.2e}",
                  flush=True)
        del dy, x, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    sys.exit(main())
