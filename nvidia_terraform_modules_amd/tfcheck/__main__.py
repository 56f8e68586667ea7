"""CLI: ``python -m nvidia_terraform_modules_amd.tfcheck [DIR ...]``

Recursively finds Terraform modules under each DIR (default: repo root,
skipping the ``.terraform`` caches), parses every file, runs the static
checks, and (``--contract FIXTURE``) diffs the call surface against the
reference. Exit status 1 on any error finding.

This is the offline stand-in for ``terraform fmt -check && terraform
validate`` (``--fmt-write`` is ``terraform fmt -recursive``: tfcheck/fmt.py) (CONTRIBUTING.md in the reference asks for both, manually); it
does NOT validate provider schemas, which needs the network.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

from .analysis import analyze, errors
from .config import find_modules, load_module
from .contract import compare, load_expected
from .lexer import HCLSyntaxError


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="tfcheck", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("dirs", nargs="*", default=["."])
    ap.add_argument("--no-vendor-lint", action="store_true")
    ap.add_argument("--no-fmt", action="store_true")
    ap.add_argument("--fmt-write", action="store_true",
                    help="rewrite every .tf / .tfvars under DIR in canonical layout "
                         "(terraform fmt without -check) and exit")
    ap.add_argument("--warnings-as-errors", action="store_true")
    ap.add_argument("--contract", help="reference surface fixture (JSON) to diff against")
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--docs", action="store_true",
                    help="regenerate the terraform-docs tables in every module README")
    ap.add_argument("--docs-check", action="store_true",
                    help="exit 1 if any module README's generated tables are stale")
    ap.add_argument("--plan", action="store_true",
                    help="offline plan of the FIRST dir: variables + validations, count/for_each "
                         "expansion, preconditions, local child modules")
    ap.add_argument("--var-file", action="append", default=[])
    ap.add_argument("--var", action="append", default=[], help="NAME=VALUE (repeatable)")
    args = ap.parse_args(argv)

    if args.plan:
        from .plan import plan

        res = plan(args.dirs[0], args.var_file, args.var)
        if args.json:
            print(json.dumps(res.as_dict(), indent=2))
        else:
            for a in res.data_sources:
                print(f" <= {a}")
            for a in res.resources:
                print(f"  + {a}")
            for m in res.registry_modules:
                print(f"  ? {m}")
            for w in res.warnings:
                print(f"warning: {w}")
            for e in res.errors:
                print(f"error: {e}")
            print(res.summary())
        return 0 if res.ok else 1

    if args.docs or args.docs_check:
        from .docs import update

        stale = []
        for d in args.dirs:
            for mdir in find_modules(d):
                if any(part in ("charts", "fixtures") for part in mdir.parts):
                    continue
                if not update(load_module(mdir), check=args.docs_check):
                    stale.append(str(mdir))
        verb = "stale" if args.docs_check else "updated"
        for m in stale:
            print(f"{verb}: {m}")
        print(f"{len(stale)} README(s) {verb}")
        return 1 if (stale and args.docs_check) else 0

    if args.fmt_write:
        from .fmt import write_formatted

        changed = [str(f) for d in args.dirs for f in write_formatted(Path(d))]
        for f in changed:
            print(f)
        print(f"{len(changed)} file(s) reformatted")
        return 0

    results = {}
    nerr = 0
    for d in args.dirs:
        for mdir in find_modules(d):
            if any(part in ("charts", "fixtures") for part in mdir.parts):
                continue
            try:
                mod = load_module(mdir)
            except HCLSyntaxError as e:
                results[str(mdir)] = [f"error: [parse] {e}"]
                nerr += 1
                continue
            fs = analyze(mod, vendor_lint=not args.no_vendor_lint, check_fmt=not args.no_fmt)
            bad = fs if args.warnings_as_errors else errors(fs)
            nerr += len(bad)
            results[str(mdir)] = [str(f) for f in fs]
    if args.contract:
        root = Path(args.dirs[0])
        for diff in compare(load_expected(args.contract), root):
            if not diff.ok:
                nerr += 1
            results[f"contract:{diff.module}"] = [] if diff.ok else [str(diff)]
    if args.json:
        print(json.dumps(results, indent=2))
    else:
        for k, v in results.items():
            print(f"{k}: {'ok' if not v else ''}")
            for line in v:
                print(f"  {line}")
        print(f"{nerr} error(s)")
    return 1 if nerr else 0


if __name__ == "__main__":
    sys.exit(main())
