"""Bitwise check of the persistent overlap builds against pingpong8c on one
MI355X (developer tool): repeated launches on shapes with 1 to 4 tiles per
workgroup; prints the count of differing elements per run and, for the first
bad run, the count per accumulator row (16-row group of a wave's 128 rows) -
the fingerprint that located the asm-MFMA hazard in profiles/r3_w4o/.

    python tools/experiments/overlap_bitwise_check.py [--variants pingpong8o,pingpong8od] [--repeats 5]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from nvidia_terraform_modules_amd import ops  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="pingpong8o,pingpong8od")
    ap.add_argument("--shapes", default="256x256x256,2048x2048x1024,8192x8192x512")
    ap.add_argument("--repeats", type=int, default=5)
    args = ap.parse_args()
    torch.manual_seed(0)
    total = 0
    for sh in args.shapes.split(","):
        m, n, k = (int(x) for x in sh.split("x"))
        a = (torch.rand(m, k, device="cuda") * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(n, k, device="cuda") * 2 - 1).to(torch.bfloat16)
        ref = ops.gemm_bf16(a, b, variant="pingpong8c")
        for v in args.variants.split(","):
            bads = []
            for rep in range(args.repeats):
                c = torch.full((m, n), float("nan"), dtype=torch.bfloat16, device="cuda")
                ops.gemm_bf16(a, b, c, variant=v)
                torch.cuda.synchronize()
                bad = c != ref
                bads.append(int(bad.sum()))
                if bads[-1] and sum(bads) == bads[-1]:
                    rows = bad.view(m // 16, 16, n).sum(dim=(1, 2)).view(-1, 8).sum(0).tolist()
                    print(f"  {v} bad per accumulator row {rows}", flush=True)
            total += sum(bads)
            print((m, n, k), v, "bad", bads, flush=True)
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
