"""Which hipBLASLt kernel torch.matmul picks for given bf16 K1 shapes, beside
our default plan - run under rocprofv3 --kernel-trace and read the trace.

    rocprofv3 --kernel-trace --stats -d gpurun_out/bl -o run -- \\
        python3 tools/experiments/blaslt_kernels.py 3904x2584x12760 7288x1344x5768

Each shape runs hipBLASLt then our default dispatch, `--iters` times each, in
that order, so the trace's dispatch order maps back to the shapes (printed as
one JSON line per shape with the dispatch index range)."""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from nvidia_terraform_modules_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shapes", nargs="+", help="MxNxK")
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    for s in args.shapes:
        m, n, k = (int(x) for x in s.lower().split("x"))
        a = ops.fill_uniform_(torch.empty(m, k, dtype=torch.bfloat16, device="cuda"), seed=1)
        b = ops.fill_uniform_(torch.empty(n, k, dtype=torch.bfloat16, device="cuda"), seed=2)
        c = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
        torch.cuda.synchronize()
        for _ in range(args.iters):
            torch.matmul(a, b.T, out=c)
        torch.cuda.synchronize()
        for _ in range(args.iters):
            ops.gemm_bf16(a, b, out=c)
        torch.cuda.synchronize()
        print(json.dumps({"shape": [m, n, k], "plan": list(ops.k1_splitk_plan(m, n, k))}),
              flush=True)


if __name__ == "__main__":
    main()
