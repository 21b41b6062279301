"""Print tools/kbench_gemm.py JSON lines as a table."""
import json
import sys

for line in sys.stdin:
    try:
        d = json.loads(line)
    except ValueError:
        continue
    vs = sorted(k[:-7] for k in d if k.endswith("_tflops") and k != "blas_tflops")
    cells = "  ".join(f"{v} {d[v + '_tflops']:7.1f} (err {d[v + '_err']})" for v in vs)
    print(f"{d['shape'][:30]:30s} blas {d['blas_tflops']:7.1f}  {cells}")
