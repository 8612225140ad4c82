"""Merge the f32-headline and bf16-variant PMC traffic passes (tools/pmc_traffic.sh with
MX_PMC_PRECISION=f32 / bf16) into one file for bench.py's roofline.traffic: kernels present in both
runs (BN, RoIAlign, NMS ...) keep the f32 figures; the bf16-only conv kernels (conv_igemm_buf_kernel,
conv_wgrad_buf_kernel) come from the bf16 pass.

    python tools/merge_traffic.py f32.json bf16.json > profiles/r03_traffic.json
"""
import json
import sys

a, b = (json.load(open(f)) for f in sys.argv[1:3])
k = dict(b["kernels"])
k.update(a["kernels"])
print(json.dumps({"method": a["method"], "passes": {"f32": sorted(a["kernels"]), "bf16": sorted(b["kernels"])},
                  "kernels": k}, indent=1))
