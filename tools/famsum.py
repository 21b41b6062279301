"""Kernel-family summary of an rpstats --stats table (tools/rpstats.py):
ms/step and launches per family, the weight-gradient family total."""
import re
import sys

FAM = ["wgrad_halo", "wgrad_grp", "wgrad_tn", "conv_wgrad", "wgrad_reduce", "reduce9", "reduce2", "chansum", "gn_bwd_reduce",
       "gn_bwd_apply", "gn_apply", "gn_stats", "silu_k", "at::native", "halo", "conv_w8_k", "conv_bufl",
       "conv_s64", "attn", "gemm_fw", "adam", "mlp", "sgemm", "border", "ray", "cond_prep", "diff", "pack", "period_sum"]
WG = ("wgrad_halo", "wgrad_grp", "wgrad_tn", "conv_wgrad", "wgrad_reduce", "reduce9", "reduce2")


def main(path):
    lines = open(path).read().splitlines()
    fam = {}
    for l in lines[1:]:
        m = re.match(r'\s*([\d.]+) ms\s+[\d.]+%\s+([\d.]+) calls\s+[\d.]+ us\s+(.*)', l)
        if not m:
            continue
        ms, c, name = float(m.group(1)), float(m.group(2)), m.group(3)
        key = next((k for k in FAM if k in name), "other")
        v = fam.setdefault(key, [0.0, 0.0])
        v[0] += ms
        v[1] += c
    print(path, lines[0])
    wg = sum(v[0] for k, v in fam.items() if k in WG)
    wgc = sum(v[1] for k, v in fam.items() if k in WG)
    print(f"  weight-gradient family {wg:.2f} ms/step in {wgc:.0f} launches")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1][0]):
        print(f"  {k:15s} {v[0]:7.2f} ms {v[1]:7.1f} launches")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
